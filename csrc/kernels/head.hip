// Classifier head of the ResNet engine: global average pool + fully connected layer.
//
// The reference ends the network with avg_pool -> view -> fc (models/resnet.py forward,
// reference resnet.py ResNet.forward); run eagerly under autocast that is ~15 small PyTorch
// kernels per step (mean reduction, three bf16 weight/bias/activation casts, a library GEMM,
// and in backward two GEMMs, a bias reduction, the pooling backward broadcast and the fp32
// gradient-accumulation casts) plus the host gaps between them.  Here the head is two
// launches that live INSIDE the body's HIP graphs:
//
//   head_fwd : body [N,HW,C] bf16 -> pooled [N,C] bf16 (kept for the weight gradient) and
//              logits [N,K] bf16 = bf16(pooled) . bf16(W)^T + bf16(b), fp32 accumulation --
//              the autocast numerics of F.linear on a mean-pooled fp32 input.
//   head_bwd : blocks [0, N*cy): dpool[n,c] = bf16(sum_k dl[n,k] bf16(W[k,c])) / HW (the last
//              block's join backward reads it broadcast over HW: no [N,HW,C] gradient is
//              ever written);  blocks [N*cy, ...): W.grad[k,c] += sum_n dl[n,k] pooled[n,c],
//              one owner thread per (k,c) (deterministic, no atomics), and b.grad from
//              the first of them.
//
// K (classes) <= 32: CIFAR-10/100-sized heads.  Larger heads keep the PyTorch path.
#include "common.h"

namespace fdt {
namespace {

constexpr int kHB = 256;

__device__ __forceinline__ float bf16r(float x) { return __bfloat162float(__float2bfloat16(x)); }

template <int KT, int S>
__global__ __launch_bounds__(kHB) void head_fwd_kernel(const bf16* __restrict__ h, const float* __restrict__ W,
                                                       const float* __restrict__ b, bf16* __restrict__ pooled,
                                                       bf16* __restrict__ logits, int HW, int C, int K) {
  __shared__ float red[kHB / 64][S * KT];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const long n0 = (long)blockIdx.x * S;
  const float inv = 1.f / (float)HW;
  float acc[S][KT];
#pragma unroll
  for (int s = 0; s < S; ++s)
#pragma unroll
    for (int k = 0; k < KT; ++k) acc[s][k] = 0.f;

  for (int cg = tid; cg < C / 8; cg += kHB) {
    const int c = cg * 8;
    float p[S][8];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const bf16* src = h + (n0 + s) * (long)HW * C + c;
      float a0[8] = {0, 0, 0, 0, 0, 0, 0, 0}, a1[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      int q = 0;
      // two rows per trip, both loads issued before use
      for (; q + 1 < HW; q += 2) {
        float v0[8], v1[8];
        Vec8<bf16>::load(src + (long)q * C, v0);
        Vec8<bf16>::load(src + (long)(q + 1) * C, v1);
#pragma unroll
        for (int i = 0; i < 8; ++i) { a0[i] += v0[i]; a1[i] += v1[i]; }
      }
      if (q < HW) {
        float v0[8];
        Vec8<bf16>::load(src + (long)q * C, v0);
#pragma unroll
        for (int i = 0; i < 8; ++i) a0[i] += v0[i];
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) p[s][i] = bf16r((a0[i] + a1[i]) * inv);
      Vec8<bf16>::store(pooled + (n0 + s) * C + c, p[s]);
    }
#pragma unroll
    for (int k = 0; k < KT; ++k) {
      if (k < K) {
        float w[8];
        Vec8<float>::load(W + (long)k * C + c, w);
#pragma unroll
        for (int i = 0; i < 8; ++i) w[i] = bf16r(w[i]);
#pragma unroll
        for (int s = 0; s < S; ++s)
#pragma unroll
          for (int i = 0; i < 8; ++i) acc[s][k] = fmaf(p[s][i], w[i], acc[s][k]);
      }
    }
  }
#pragma unroll
  for (int s = 0; s < S; ++s)
#pragma unroll
    for (int k = 0; k < KT; ++k) {
      if (k < K) {
        const float v = wave_sum(acc[s][k]);
        if (lane == 0) red[wv][s * KT + k] = v;
      }
    }
  __syncthreads();
  if (tid < S * K) {
    const int s = tid / K, k = tid % K;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < kHB / 64; ++w) v += red[w][s * KT + k];
    v += bf16r(b[k]);
    logits[(n0 + s) * K + k] = __float2bfloat16(v);
  }
}

constexpr int kCPB = 32;          // weight-gradient block: 32 channels ...
constexpr int kNL = kHB / kCPB;   // ... x 8 sample lanes
constexpr int kNChunk = 256;      // samples staged per LDS round

template <int KT>
__global__ __launch_bounds__(kHB) void head_bwd_kernel(const bf16* __restrict__ dl, const float* __restrict__ W,
                                                       const bf16* __restrict__ pooled, bf16* __restrict__ dpool,
                                                       float* __restrict__ gW, float* __restrict__ gb, int N, int C,
                                                       int K, int HW, int cy) {
  const int tid = threadIdx.x;
  const int ndx = N * cy;
  if ((int)blockIdx.x < ndx) {
    // ---- pooled gradient of one sample, 8 channels per thread
    const int n = blockIdx.x / cy;
    const int cg = (blockIdx.x % cy) * kHB + tid;
    if (cg >= C / 8) return;
    const int c = cg * 8;
    float a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int k = 0; k < K; ++k) {
      const float d = __bfloat162float(dl[(long)n * K + k]);
      float w[8];
      Vec8<float>::load(W + (long)k * C + c, w);
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = fmaf(d, bf16r(w[i]), a[i]);
    }
    const float inv = 1.f / (float)HW;
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = bf16r(a[i]) * inv;
    Vec8<bf16>::store(dpool + (long)n * C + c, a);
    return;
  }
  // ---- weight / bias gradient of kCPB channels
  __shared__ float sdl[kNChunk][KT];
  __shared__ float red[kNL][kCPB][KT + 1];
  const int j = blockIdx.x - ndx;
  const int cl = tid % kCPB, nl = tid / kCPB;
  const int c = j * kCPB + cl;
  const bool bias_block = (j == 0);
  float a[KT], bs = 0.f;
#pragma unroll
  for (int k = 0; k < KT; ++k) a[k] = 0.f;
  for (int nb = 0; nb < N; nb += kNChunk) {
    const int rows = min(kNChunk, N - nb);
    __syncthreads();
    for (int i = tid; i < rows * K; i += kHB) sdl[i / K][i % K] = __bfloat162float(dl[(long)nb * K + i]);
    __syncthreads();
    if (c < C) {
      int q = nl;
      for (; q + kNL < rows; q += 2 * kNL) {
        const float p0 = __bfloat162float(pooled[(long)(nb + q) * C + c]);
        const float p1 = __bfloat162float(pooled[(long)(nb + q + kNL) * C + c]);
#pragma unroll
        for (int k = 0; k < KT; ++k) a[k] = fmaf(sdl[q + kNL][k], p1, fmaf(sdl[q][k], p0, a[k]));
      }
      if (q < rows) {
        const float p0 = __bfloat162float(pooled[(long)(nb + q) * C + c]);
#pragma unroll
        for (int k = 0; k < KT; ++k) a[k] = fmaf(sdl[q][k], p0, a[k]);
      }
    }
    if (bias_block && tid < K)
      for (int q = 0; q < rows; ++q) bs += sdl[q][tid];
  }
#pragma unroll
  for (int k = 0; k < KT; ++k) red[nl][cl][k] = a[k];
  __syncthreads();
  if (nl == 0 && c < C) {
    for (int k = 0; k < K; ++k) {
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < kNL; ++q) v += red[q][cl][k];
      gW[(long)k * C + c] += v;
    }
  }
  if (bias_block && tid < K) gb[tid] += bs;
}

}  // namespace

void head_fwd(uint64_t h, uint64_t W, uint64_t b, uint64_t pooled, uint64_t logits, int N, int HW, int C, int K,
              uint64_t stream) {
  FDT_CHECK(K >= 1 && K <= 32, "head_fwd: 1 <= classes <= 32");
  FDT_CHECK(C % 8 == 0 && N >= 1 && HW >= 1, "head_fwd: channels must be a multiple of 8");
  hipStream_t st = as_stream(stream);
  const bool wide = N >= 512;
  if (K <= 16) {
    if (wide && N % 4 == 0)
      head_fwd_kernel<16, 4><<<N / 4, kHB, 0, st>>>(P<const bf16>(h), P<const float>(W), P<const float>(b),
                                                    P<bf16>(pooled), P<bf16>(logits), HW, C, K);
    else
      head_fwd_kernel<16, 1><<<N, kHB, 0, st>>>(P<const bf16>(h), P<const float>(W), P<const float>(b),
                                                P<bf16>(pooled), P<bf16>(logits), HW, C, K);
  } else {
    if (wide && N % 2 == 0)
      head_fwd_kernel<32, 2><<<N / 2, kHB, 0, st>>>(P<const bf16>(h), P<const float>(W), P<const float>(b),
                                                    P<bf16>(pooled), P<bf16>(logits), HW, C, K);
    else
      head_fwd_kernel<32, 1><<<N, kHB, 0, st>>>(P<const bf16>(h), P<const float>(W), P<const float>(b),
                                                P<bf16>(pooled), P<bf16>(logits), HW, C, K);
  }
  FDT_LAUNCH_CHECK();
}

void head_bwd(uint64_t dl, uint64_t W, uint64_t pooled, uint64_t dpool, uint64_t gW, uint64_t gb, int N, int HW,
              int C, int K, uint64_t stream) {
  FDT_CHECK(K >= 1 && K <= 32, "head_bwd: 1 <= classes <= 32");
  FDT_CHECK(C % 8 == 0 && N >= 1 && HW >= 1, "head_bwd: channels must be a multiple of 8");
  const int cy = (C / 8 + kHB - 1) / kHB;
  const int nw = (C + kCPB - 1) / kCPB;
  const int grid = N * cy + nw;
  hipStream_t st = as_stream(stream);
  if (K <= 16)
    head_bwd_kernel<16><<<grid, kHB, 0, st>>>(P<const bf16>(dl), P<const float>(W), P<const bf16>(pooled),
                                              P<bf16>(dpool), P<float>(gW), P<float>(gb), N, C, K, HW, cy);
  else
    head_bwd_kernel<32><<<grid, kHB, 0, st>>>(P<const bf16>(dl), P<const float>(W), P<const bf16>(pooled),
                                              P<bf16>(dpool), P<float>(gW), P<float>(gb), N, C, K, HW, cy);
  FDT_LAUNCH_CHECK();
}

}  // namespace fdt
