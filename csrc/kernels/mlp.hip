// FusedMLP elementwise stages (reference MLPScratch, transformer.py:292-338).
//  bias_relu_fwd : pre += b (in place, kept for the mask); act = relu(pre)      one pass
//  relu_bwd_colsum: gpre = gact * (pre > 0);  gb[c] += sum_rows gpre           one pass
// The reference does the ReLU backward with a per-element Python loop and a host sync
// per element (survey Q6); this is the whole of it in one launch.
#include "common.h"

#include <algorithm>

namespace fdt {

template <typename T>
__global__ __launch_bounds__(256) void bias_relu_fwd_kernel(T* __restrict__ pre, const float* __restrict__ b,
                                                            T* __restrict__ act, long n, int cols) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float v = to_f(pre[i]);
    if (b) {
      v += b[i % cols];
      pre[i] = from_f<T>(v);
    }
    act[i] = from_f<T>(fmaxf(v, 0.f));
  }
}

template <typename T>
__global__ __launch_bounds__(256) void relu_bwd_colsum_kernel(const T* __restrict__ gact, const T* __restrict__ pre,
                                                              T* __restrict__ gpre, float* __restrict__ gb, long rows,
                                                              int cols, int rows_per_blk) {
  const long r0 = (long)blockIdx.y * rows_per_blk;
  long r1 = r0 + rows_per_blk;
  if (r1 > rows) r1 = rows;
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < cols; c += gridDim.x * blockDim.x) {
    float acc = 0.f;
    for (long r = r0; r < r1; ++r) {
      long i = r * cols + c;
      float g = to_f(pre[i]) > 0.f ? to_f(gact[i]) : 0.f;
      gpre[i] = from_f<T>(g);
      acc += g;
    }
    if (gb) atomicAdd(gb + c, acc);
  }
}

// out[c] += sum_r x[r][c] for bf16 x [rows][cols] (cols % 8 == 0), fp32 out zeroed by the
// caller: the bias gradient of a linear layer.  Lane = 8 adjacent columns (one 16-B load);
// a 256-thread block covers (256 / lanes_per_row) rows x cols_blk columns of a row chunk,
// folds its rows in registers + LDS, one atomic per column per block.
__global__ __launch_bounds__(256) void colsum_bf16_kernel(const bf16* __restrict__ x, float* __restrict__ out,
                                                          long rows, int cols, long ld, int rows_per_blk) {
  __shared__ float red[256 * 8];
  const int lanes = min(cols / 8 - blockIdx.x * 32, 32);  // column groups of this block
  const int cg = threadIdx.x % 32, rl = threadIdx.x / 32;  // 32 column groups x 8 row lanes
  const long r0 = (long)blockIdx.y * rows_per_blk;
  const long r1 = min(rows, r0 + rows_per_blk);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int c0 = (blockIdx.x * 32 + cg) * 8;
  if (cg < lanes) {
    for (long r = r0 + rl; r < r1; r += 8) {
      const uint4 v = *reinterpret_cast<const uint4*>(x + r * ld + c0);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[2 * j] += __uint_as_float(w[j] << 16);
        acc[2 * j + 1] += __uint_as_float(w[j] & 0xffff0000u);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[(rl * 32 + cg) * 8 + j] = acc[j];
  __syncthreads();
  // 256 threads fold the 8 row lanes of 32 x 8 columns
  const int col = threadIdx.x;  // 0..255 = cg * 8 + j
  if (col / 8 < lanes) {
    float s = 0.f;
#pragma unroll
    for (int l = 0; l < 8; ++l) s += red[(l * 32 + col / 8) * 8 + (col % 8)];
    atomicAdd(out + blockIdx.x * 256 + col, s);
  }
}

void colsum_bf16(uint64_t x, uint64_t out, long rows, int cols, long ld, uint64_t stream) {
  if (ld == 0) ld = cols;
  FDT_CHECK(cols % 8 == 0 && ld % 8 == 0 && ld >= cols && x % 16 == 0, "colsum_bf16: cols, ld % 8 == 0, 16-B aligned rows");
  if (rows == 0 || cols == 0) return;
  const int cblk = (cols / 8 + 31) / 32;
  // ~512 workgroups in total, >= 64 rows per block
  long rpb = rows * cblk / 512;
  if (rpb < 64) rpb = 64;
  rpb = (rpb + 7) / 8 * 8;
  dim3 grid((unsigned)cblk, (unsigned)((rows + rpb - 1) / rpb));
  colsum_bf16_kernel<<<grid, 256, 0, as_stream(stream)>>>(P<const bf16>(x), P<float>(out), rows, cols, ld, (int)rpb);
  FDT_LAUNCH_CHECK();
}

// dst[i] += sum_j src[j * ld + i] for j < s (fp32): the split-K weight-gradient slabs (or
// per-block LayerNorm partials) folded straight into the fp32 master gradient -- one pass
// instead of a reduction kernel + a separate accumulate kernel.  Block = 64 float4 columns x
// 4 slab lanes; grid.y splits the slab axis when the columns alone give too few workgroups
// (LayerNorm: 512 slabs x 128 float4) -- those blocks combine with atomics.
__global__ __launch_bounds__(256) void slab_sum_acc_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                                           int s, long ld4, long n4, int s_per_blk) {
  __shared__ float4 red[4][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const long i = blockIdx.x * 64L + cl;
  const int j0 = blockIdx.y * s_per_blk, j1 = min(s, j0 + s_per_blk);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < n4)
    for (int j = j0 + rl; j < j1; j += 4) {
      const float4 v = reinterpret_cast<const float4*>(src)[(long)j * ld4 + i];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  red[rl][cl] = acc;
  __syncthreads();
  if (rl == 0 && i < n4) {
#pragma unroll
    for (int r = 1; r < 4; ++r) {
      acc.x += red[r][cl].x; acc.y += red[r][cl].y; acc.z += red[r][cl].z; acc.w += red[r][cl].w;
    }
    float4* d = reinterpret_cast<float4*>(dst) + i;
    if (gridDim.y == 1) {
      float4 o = *d;
      o.x += acc.x; o.y += acc.y; o.z += acc.z; o.w += acc.w;
      *d = o;
    } else {
      float* df = reinterpret_cast<float*>(d);
      atomicAdd(df + 0, acc.x); atomicAdd(df + 1, acc.y); atomicAdd(df + 2, acc.z); atomicAdd(df + 3, acc.w);
    }
  }
}

void slab_sum_acc(uint64_t src, uint64_t dst, int s, long ld, long n, uint64_t stream) {
  FDT_CHECK(n % 4 == 0 && ld % 4 == 0 && src % 16 == 0 && dst % 16 == 0 && s >= 1,
            "slab_sum_acc: n, ld multiples of 4, 16-B aligned");
  if (n == 0) return;
  const long n4 = n / 4;
  const long nbx = (n4 + 63) / 64;
  int spb = s;
  if (nbx < 512) {  // split the slab axis: ~512 workgroups, >= 16 slabs each
    spb = (int)std::max<long>(16, ((long)s * nbx + 511) / 512);
    spb = (spb + 3) / 4 * 4;
    if (spb > s) spb = s;
  }
  dim3 grid((unsigned)nbx, (unsigned)((s + spb - 1) / spb));
  slab_sum_acc_kernel<<<grid, 256, 0, as_stream(stream)>>>(P<const float>(src), P<float>(dst), s, ld / 4, n4, spb);
  FDT_LAUNCH_CHECK();
}

#define DISPATCH_T(dt, ...)                                     \
  switch (dt) {                                                 \
    case kF32: { using T = float; __VA_ARGS__; break; }         \
    case kBF16: { using T = bf16; __VA_ARGS__; break; }         \
    case kF16: { using T = f16; __VA_ARGS__; break; }           \
    default: throw std::runtime_error("bad dtype code");        \
  }

void bias_relu_fwd(uint64_t pre, uint64_t b, uint64_t act, long rows, int cols, int dt, uint64_t stream) {
  long n = rows * cols;
  if (n == 0) return;
  int g = (int)((n + 255) / 256);
  if (g > 2048) g = 2048;
  DISPATCH_T(dt, {
    bias_relu_fwd_kernel<T><<<g, 256, 0, as_stream(stream)>>>(P<T>(pre), P<const float>(b), P<T>(act), n, cols);
  });
  FDT_LAUNCH_CHECK();
}

void relu_bwd_colsum(uint64_t gact, uint64_t pre, uint64_t gpre, uint64_t gb, long rows, int cols, int dt,
                     uint64_t stream) {
  if (rows == 0) return;
  const int rpb = 32;
  dim3 grid((unsigned)((cols + 255) / 256), (unsigned)((rows + rpb - 1) / rpb));
  DISPATCH_T(dt, {
    relu_bwd_colsum_kernel<T><<<grid, 256, 0, as_stream(stream)>>>(P<const T>(gact), P<const T>(pre), P<T>(gpre),
                                                                  P<float>(gb), rows, cols, rpb);
  });
  FDT_LAUNCH_CHECK();
}

}  // namespace fdt
