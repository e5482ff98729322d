// Fused dropout epilogues of the transformer sublayers (reference transformer.py:159-177,
// :246-262: ``dropout(sublayer(x)) + x`` and the FFN's ``dropout(gelu(w_1 x))``).
//
// PyTorch runs each of these as 2-4 kernels per direction (dropout with a stored bool mask,
// a separate add / GELU / masked-scale / GELU-backward) over [tokens x 512 | 2048] tensors.
// Here one streaming pass per direction: the keep/drop decision is a counter-based hash of
// (seed, element index) -- no mask tensor is stored, the backward regenerates it.  The seed is
// a host-drawn per-call constant XORed with an optional device word (``seed_ptr``) so that a
// replayed HIP graph draws fresh masks each step (the runner rewrites that word per replay).
//
// Layout: 8 elements per lane (one 16-B bf16 load), one 64-bit hash per 2 elements (its two
// 32-bit halves), grid-stride loop over n / 8 lane-chunks.
#include "common.h"
#include "dropout_math.h"

#include <algorithm>

namespace fdt {
namespace {
using drop::drop_hash;
using drop::keep8;
using drop::gelu_erf;
using drop::gelu_erf_grad;
using drop::live_seed;

__device__ __forceinline__ void unpack8(const uint4 v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    f[2 * j] = __uint_as_float(w[j] << 16);
    f[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
  }
}

__device__ __forceinline__ uint32_t pack2(float a, float b) {
  // round-to-nearest-even bf16 pair
  uint32_t ua = __float_as_uint(a), ub = __float_as_uint(b);
  ua += 0x7fffu + ((ua >> 16) & 1u);
  ub += 0x7fffu + ((ub >> 16) & 1u);
  return (ua >> 16) | (ub & 0xffff0000u);
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  return make_uint4(pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7]));
}

// out = x + keep * y * scale   (y bf16, x / out fp32: the residual stream)
__global__ __launch_bounds__(256) void dropout_add_fwd_kernel(const bf16* __restrict__ y, const float* __restrict__ x,
                                                              float* __restrict__ out, long n8, uint32_t thr,
                                                              float scale, uint64_t seed, const uint64_t* seed_ptr) {
  const uint64_t s = live_seed(seed, seed_ptr);
  for (long c = blockIdx.x * 256L + threadIdx.x; c < n8; c += (long)gridDim.x * 256) {
    float f[8];
    unpack8(reinterpret_cast<const uint4*>(y)[c], f);
    const uint32_t m = keep8(c, s, thr);
    const float4 x0 = reinterpret_cast<const float4*>(x)[2 * c];
    const float4 x1 = reinterpret_cast<const float4*>(x)[2 * c + 1];
    float4 o0, o1;
    o0.x = x0.x + ((m >> 0) & 1 ? f[0] * scale : 0.f);
    o0.y = x0.y + ((m >> 1) & 1 ? f[1] * scale : 0.f);
    o0.z = x0.z + ((m >> 2) & 1 ? f[2] * scale : 0.f);
    o0.w = x0.w + ((m >> 3) & 1 ? f[3] * scale : 0.f);
    o1.x = x1.x + ((m >> 4) & 1 ? f[4] * scale : 0.f);
    o1.y = x1.y + ((m >> 5) & 1 ? f[5] * scale : 0.f);
    o1.z = x1.z + ((m >> 6) & 1 ? f[6] * scale : 0.f);
    o1.w = x1.w + ((m >> 7) & 1 ? f[7] * scale : 0.f);
    reinterpret_cast<float4*>(out)[2 * c] = o0;
    reinterpret_cast<float4*>(out)[2 * c + 1] = o1;
  }
}

// gy = keep * g * scale   (g fp32 -> gy bf16)
__global__ __launch_bounds__(256) void dropout_bwd_kernel(const float* __restrict__ g, bf16* __restrict__ gy, long n8,
                                                          uint32_t thr, float scale, uint64_t seed,
                                                          const uint64_t* seed_ptr) {
  const uint64_t s = live_seed(seed, seed_ptr);
  for (long c = blockIdx.x * 256L + threadIdx.x; c < n8; c += (long)gridDim.x * 256) {
    const uint32_t m = keep8(c, s, thr);
    const float4 g0 = reinterpret_cast<const float4*>(g)[2 * c];
    const float4 g1 = reinterpret_cast<const float4*>(g)[2 * c + 1];
    const float gf[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
    float f[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = (m >> j) & 1 ? gf[j] * scale : 0.f;
    reinterpret_cast<uint4*>(gy)[c] = pack8(f);
  }
}

// h = keep * gelu(a) * scale   (bf16 in / out)
__global__ __launch_bounds__(256) void gelu_dropout_fwd_kernel(const bf16* __restrict__ a, bf16* __restrict__ h,
                                                               long n8, uint32_t thr, float scale, uint64_t seed,
                                                               const uint64_t* seed_ptr) {
  const uint64_t s = live_seed(seed, seed_ptr);
  for (long c = blockIdx.x * 256L + threadIdx.x; c < n8; c += (long)gridDim.x * 256) {
    float f[8];
    unpack8(reinterpret_cast<const uint4*>(a)[c], f);
    const uint32_t m = thr ? keep8(c, s, thr) : 0xffu;
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = (m >> j) & 1 ? gelu_erf(f[j]) * scale : 0.f;
    reinterpret_cast<uint4*>(h)[c] = pack8(f);
  }
}

// ga = keep * g * scale * gelu'(a)   (bf16 in / out)
__global__ __launch_bounds__(256) void gelu_dropout_bwd_kernel(const bf16* __restrict__ g, const bf16* __restrict__ a,
                                                               bf16* __restrict__ ga, long n8, uint32_t thr,
                                                               float scale, uint64_t seed, const uint64_t* seed_ptr) {
  const uint64_t s = live_seed(seed, seed_ptr);
  for (long c = blockIdx.x * 256L + threadIdx.x; c < n8; c += (long)gridDim.x * 256) {
    float fa[8], fg[8];
    unpack8(reinterpret_cast<const uint4*>(a)[c], fa);
    unpack8(reinterpret_cast<const uint4*>(g)[c], fg);
    const uint32_t m = thr ? keep8(c, s, thr) : 0xffu;
#pragma unroll
    for (int j = 0; j < 8; ++j) fa[j] = (m >> j) & 1 ? fg[j] * scale * gelu_erf_grad(fa[j]) : 0.f;
    reinterpret_cast<uint4*>(ga)[c] = pack8(fa);
  }
}

// The two backward passes above with the bias gradient of the linear layer that PRODUCED the
// dropout input folded in: gb[c] += sum over rows of the stored gradient (what a separate
// colsum pass would re-read from HBM).  2-D layout: a block is 32 column groups (8 columns,
// one 16-B vector each) x 8 row lanes over a chunk of rows; element e = r*cols + c0 keeps
// the forward's hash index (chunk e/8), so the masks are the grid-stride kernels' masks.
// KIND 0: g fp32 -> gy = keep*g*scale (bf16);  KIND 1: g, a bf16 -> ga = keep*g*scale*gelu'(a).
template <int KIND>
__global__ __launch_bounds__(256) void dropout_bwd_colsum_kernel(const void* __restrict__ gin,
                                                                 const bf16* __restrict__ a, bf16* __restrict__ out,
                                                                 float* __restrict__ gb, long rows, int cols,
                                                                 int rows_per_blk, uint32_t thr, float scale,
                                                                 uint64_t seed, const uint64_t* seed_ptr) {
  __shared__ float red[256 * 8];
  const uint64_t s = live_seed(seed, seed_ptr);
  const int lanes = min(cols / 8 - (int)blockIdx.x * 32, 32);
  const int cg = threadIdx.x % 32, rl = threadIdx.x / 32;
  const long r0 = (long)blockIdx.y * rows_per_blk;
  const long r1 = min(rows, r0 + rows_per_blk);
  const int c0 = (blockIdx.x * 32 + cg) * 8;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (cg < lanes) {
    // 4 rows per trip (row lanes stride 8): all loads of a trip are issued before any use
    constexpr int U = 4;
    for (long rb = r0 + rl; rb < r1; rb += 8 * U) {
      float4 g4[U][2];
      uint4 gu[U], au[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long r = rb + 8 * u;
        if (r < r1) {
          const long c = (r * cols + c0) >> 3;
          if constexpr (KIND == 0) {
            g4[u][0] = reinterpret_cast<const float4*>(gin)[2 * c];
            g4[u][1] = reinterpret_cast<const float4*>(gin)[2 * c + 1];
          } else {
            gu[u] = reinterpret_cast<const uint4*>(gin)[c];
            au[u] = reinterpret_cast<const uint4*>(a)[c];
          }
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long r = rb + 8 * u;
        if (r >= r1) break;
        const long c = (r * cols + c0) >> 3;  // 16-B chunk index = the forward's hash index
        const uint32_t m = thr ? keep8(c, s, thr) : 0xffu;
        float f[8];
        if constexpr (KIND == 0) {
          const float gf[8] = {g4[u][0].x, g4[u][0].y, g4[u][0].z, g4[u][0].w,
                               g4[u][1].x, g4[u][1].y, g4[u][1].z, g4[u][1].w};
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = (m >> j) & 1 ? gf[j] * scale : 0.f;
        } else {
          float fa[8];
          unpack8(au[u], fa);
          unpack8(gu[u], f);
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = (m >> j) & 1 ? f[j] * scale * gelu_erf_grad(fa[j]) : 0.f;
        }
        const uint4 o = pack8(f);
        reinterpret_cast<uint4*>(out)[c] = o;
        // the bias gradient sums the STORED (bf16-rounded) values, as a colsum pass would
        float q[8];
        unpack8(o, q);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += q[j];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[(rl * 32 + cg) * 8 + j] = acc[j];
  __syncthreads();
  const int col = threadIdx.x;  // cg * 8 + j
  if (col / 8 < lanes) {
    float t = 0.f;
#pragma unroll
    for (int l = 0; l < 8; ++l) t += red[(l * 32 + col / 8) * 8 + (col % 8)];
    atomicAdd(gb + blockIdx.x * 256 + col, t);
  }
}

unsigned grid_for(long n8) { return (unsigned)std::max<long>(1, std::min<long>((n8 + 255) / 256, 4096)); }

// Row chunks per column block: few enough that same-address fp32 atomics (serialised in L2)
// stay cheap -- 256 for one or two column blocks, 512 when wider rows already give >= 4
// column blocks of parallelism (measured: 512 -> 256 chunks at 512 columns 36 -> 24 us,
// 256 -> 512 at 1024 columns 66 -> 60 us) -- and >= 32 rows (4 per row lane) per block
dim3 colsum_grid(long rows, int cols, int* rpb_out) {
  const int cblk = (cols / 8 + 31) / 32;
  const long chunks = cblk >= 4 ? 512 : 256;
  long rpb = (rows + chunks - 1) / chunks;
  if (rpb < 32) rpb = 32;
  rpb = (rpb + 7) / 8 * 8;
  *rpb_out = (int)rpb;
  return dim3((unsigned)cblk, (unsigned)((rows + rpb - 1) / rpb));
}

uint32_t threshold(float p) {
  FDT_CHECK(p >= 0.f && p < 1.f, "dropout: p in [0, 1)");
  return (uint32_t)std::min(p * 4294967296.0, 4294967295.0);
}

}  // namespace

void dropout_add_fwd(uint64_t y, uint64_t x, uint64_t out, long n, float p, uint64_t seed, uint64_t seed_ptr,
                     uint64_t stream) {
  FDT_CHECK(n % 8 == 0 && y % 16 == 0 && x % 16 == 0 && out % 16 == 0, "dropout_add: n % 8, 16-B aligned");
  if (n == 0) return;
  dropout_add_fwd_kernel<<<grid_for(n / 8), 256, 0, as_stream(stream)>>>(
      P<const bf16>(y), P<const float>(x), P<float>(out), n / 8, threshold(p), 1.f / (1.f - p), seed,
      P<const uint64_t>(seed_ptr));
  FDT_LAUNCH_CHECK();
}

void dropout_bwd(uint64_t g, uint64_t gy, long n, float p, uint64_t seed, uint64_t seed_ptr, uint64_t stream) {
  FDT_CHECK(n % 8 == 0 && g % 16 == 0 && gy % 16 == 0, "dropout_bwd: n % 8, 16-B aligned");
  if (n == 0) return;
  dropout_bwd_kernel<<<grid_for(n / 8), 256, 0, as_stream(stream)>>>(
      P<const float>(g), P<bf16>(gy), n / 8, threshold(p), 1.f / (1.f - p), seed, P<const uint64_t>(seed_ptr));
  FDT_LAUNCH_CHECK();
}

void dropout_bwd_colsum(uint64_t g, uint64_t gy, uint64_t gb, long rows, int cols, float p, uint64_t seed,
                        uint64_t seed_ptr, uint64_t stream) {
  FDT_CHECK(cols % 8 == 0 && g % 16 == 0 && gy % 16 == 0 && gb % 4 == 0 && gb != 0,
            "dropout_bwd_colsum: cols % 8, 16-B aligned rows, fp32 bias gradient");
  if (rows == 0) return;
  int rpb;
  const dim3 grid = colsum_grid(rows, cols, &rpb);
  dropout_bwd_colsum_kernel<0><<<grid, 256, 0, as_stream(stream)>>>(
      P<const void>(g), nullptr, P<bf16>(gy), P<float>(gb), rows, cols, rpb, threshold(p), 1.f / (1.f - p), seed,
      P<const uint64_t>(seed_ptr));
  FDT_LAUNCH_CHECK();
}

void gelu_dropout_bwd_colsum(uint64_t g, uint64_t a, uint64_t ga, uint64_t gb, long rows, int cols, float p,
                             uint64_t seed, uint64_t seed_ptr, uint64_t stream) {
  FDT_CHECK(cols % 8 == 0 && g % 16 == 0 && a % 16 == 0 && ga % 16 == 0 && gb % 4 == 0 && gb != 0,
            "gelu_dropout_bwd_colsum: cols % 8, 16-B aligned rows, fp32 bias gradient");
  if (rows == 0) return;
  int rpb;
  const dim3 grid = colsum_grid(rows, cols, &rpb);
  dropout_bwd_colsum_kernel<1><<<grid, 256, 0, as_stream(stream)>>>(
      P<const void>(g), P<const bf16>(a), P<bf16>(ga), P<float>(gb), rows, cols, rpb, threshold(p), 1.f / (1.f - p),
      seed, P<const uint64_t>(seed_ptr));
  FDT_LAUNCH_CHECK();
}

void gelu_dropout_fwd(uint64_t a, uint64_t h, long n, float p, uint64_t seed, uint64_t seed_ptr, uint64_t stream) {
  FDT_CHECK(n % 8 == 0 && a % 16 == 0 && h % 16 == 0, "gelu_dropout: n % 8, 16-B aligned");
  if (n == 0) return;
  gelu_dropout_fwd_kernel<<<grid_for(n / 8), 256, 0, as_stream(stream)>>>(
      P<const bf16>(a), P<bf16>(h), n / 8, threshold(p), 1.f / (1.f - p), seed, P<const uint64_t>(seed_ptr));
  FDT_LAUNCH_CHECK();
}

void gelu_dropout_bwd(uint64_t g, uint64_t a, uint64_t ga, long n, float p, uint64_t seed, uint64_t seed_ptr,
                      uint64_t stream) {
  FDT_CHECK(n % 8 == 0 && g % 16 == 0 && a % 16 == 0 && ga % 16 == 0, "gelu_dropout_bwd: n % 8, 16-B aligned");
  if (n == 0) return;
  gelu_dropout_bwd_kernel<<<grid_for(n / 8), 256, 0, as_stream(stream)>>>(
      P<const bf16>(g), P<const bf16>(a), P<bf16>(ga), n / 8, threshold(p), 1.f / (1.f - p), seed,
      P<const uint64_t>(seed_ptr));
  FDT_LAUNCH_CHECK();
}

}  // namespace fdt
