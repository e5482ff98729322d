// LayerNorm with the reference's numerics (transformer.py:230-242):
//     y = a * (x - mean) / (std_unbiased + eps) + b
// One row per wave64; each lane owns E = d/64 elements held in registers, so x is read
// once (forward) / x and dy once (backward).  Statistics in fp32, two-pass in registers.
// Backward (r = 1/(std+eps), ga = a*dy, S1 = sum ga, S2 = sum ga*(x-mean)):
//     dx = r*(ga - S1/d) - r^2 * S2 * (x-mean) / ((d-1)*std)
// plus per-block partials of dgamma = sum dy*z and dbeta = sum dy (no atomics).
#include "common.h"

namespace fdt {

constexpr int kLnWaves = 4;
constexpr int kMaxE = 32;  // d <= 2048

template <int E, typename T>
__device__ __forceinline__ void ln_load(const T* row, int d, int lane, float* v) {
  if constexpr (E % 8 == 0) {
    for (int k = 0; k < E / 8; ++k) Vec8<T>::load(row + k * 512 + lane * 8, v + k * 8);
  } else {
    _Pragma("unroll") for (int k = 0; k < E; ++k) v[k] = to_f(row[k * 64 + lane]);
  }
}
template <int E, typename T>
__device__ __forceinline__ void ln_store(T* row, int d, int lane, const float* v) {
  if constexpr (E % 8 == 0) {
    for (int k = 0; k < E / 8; ++k) Vec8<T>::store(row + k * 512 + lane * 8, v + k * 8);
  } else {
    _Pragma("unroll") for (int k = 0; k < E; ++k) row[k * 64 + lane] = from_f<T>(v[k]);
  }
}
// column index of the lane's k-th element (matches ln_load's layout)
template <int E>
__device__ __forceinline__ int ln_col(int d, int lane, int k) {
  return (E % 8 == 0) ? (k / 8) * 512 + lane * 8 + (k % 8) : k * 64 + lane;
}

template <int E, typename TX, typename TY, typename TW>
__global__ __launch_bounds__(64 * kLnWaves) void layernorm_fwd_kernel(const TX* __restrict__ x, const TW* __restrict__ a,
                                                                      const TW* __restrict__ b, TY* __restrict__ y,
                                                                      float* __restrict__ mean_out,
                                                                      float* __restrict__ rstd_out, long rows, int d,
                                                                      float eps) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * kLnWaves + (threadIdx.x >> 6);
  if (row >= rows) return;
  float v[E];
  ln_load<E>(x + row * d, d, lane, v);
  float s = 0.f;
  _Pragma("unroll") for (int k = 0; k < E; ++k) s += v[k];
  const float mean = wave_sum(s) / (float)d;
  float q = 0.f;
  _Pragma("unroll") for (int k = 0; k < E; ++k) { float c = v[k] - mean; q = fmaf(c, c, q); }
  const float var = wave_sum(q) / (float)(d - 1);
  const float r = 1.f / (sqrtf(var) + eps);
  _Pragma("unroll") for (int k = 0; k < E; ++k) {
    int c = ln_col<E>(d, lane, k);
    v[k] = to_f(a[c]) * (v[k] - mean) * r + to_f(b[c]);
  }
  ln_store<E>(y + row * d, d, lane, v);
  if (lane == 0) { mean_out[row] = mean; rstd_out[row] = r; }
}

template <int E, typename TG, typename TX, typename TW>
__global__ __launch_bounds__(64 * kLnWaves) void layernorm_bwd_kernel(const TG* __restrict__ gy, const TX* __restrict__ x,
                                                                      const TW* __restrict__ a,
                                                                      const float* __restrict__ mean_in,
                                                                      const float* __restrict__ rstd_in, TX* __restrict__ gx,
                                                                      const TX* __restrict__ gres,
                                                                      float* __restrict__ part, long rows, int d,
                                                                      long rows_per_blk, float eps_unused) {
  extern __shared__ float lds[];  // [kLnWaves][2][d]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float pg[E], pb[E], av[E];
  _Pragma("unroll") for (int k = 0; k < E; ++k) { pg[k] = 0.f; pb[k] = 0.f; av[k] = to_f(a[ln_col<E>(d, lane, k)]); }
  const long r0 = (long)blockIdx.x * rows_per_blk;
  long r1 = r0 + rows_per_blk;
  if (r1 > rows) r1 = rows;
  // the next row's dy / x are requested before this row's math (one row of loads in flight
  // behind the compute: the loop was latency-bound at a few rows per wave)
  float gn[E], xn[E];
  if (r0 + w < r1) {
    ln_load<E>(gy + (r0 + w) * d, d, lane, gn);
    ln_load<E>(x + (r0 + w) * d, d, lane, xn);
  }
  for (long row = r0 + w; row < r1; row += kLnWaves) {
    float gv[E], xv[E];
    _Pragma("unroll") for (int k = 0; k < E; ++k) { gv[k] = gn[k]; xv[k] = xn[k]; }
    if (row + kLnWaves < r1) {
      ln_load<E>(gy + (row + kLnWaves) * d, d, lane, gn);
      ln_load<E>(x + (row + kLnWaves) * d, d, lane, xn);
    }
    const float mean = mean_in[row], r = rstd_in[row];
    float s1 = 0.f, s2 = 0.f;
    _Pragma("unroll") for (int k = 0; k < E; ++k) {
      float xc = xv[k] - mean;
      float ga = av[k] * gv[k];
      s1 += ga;
      s2 = fmaf(ga, xc, s2);
      pg[k] = fmaf(gv[k], xc * r, pg[k]);
      pb[k] += gv[k];
      xv[k] = xc;
    }
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    // std = 1/r - eps is recovered from the forward through r; std>0 for any non-constant row
    const float inv_d = 1.f / (float)d;
    const float sd = fmaxf(1.f / r - eps_unused, 1e-30f);
    const float c2 = r * r * s2 / ((float)(d - 1) * sd);
    _Pragma("unroll") for (int k = 0; k < E; ++k) gv[k] = r * (av[k] * gv[k] - s1 * inv_d) - c2 * xv[k];
    if (gres != nullptr) {  // + the residual (skip-path) gradient of x: no separate add pass
      float rv[E];
      ln_load<E>(gres + row * d, d, lane, rv);
      _Pragma("unroll") for (int k = 0; k < E; ++k) gv[k] += rv[k];
    }
    ln_store<E>(gx + row * d, d, lane, gv);
  }
  _Pragma("unroll") for (int k = 0; k < E; ++k) {
    int c = ln_col<E>(d, lane, k);
    lds[(w * 2 + 0) * d + c] = pg[k];
    lds[(w * 2 + 1) * d + c] = pb[k];
  }
  __syncthreads();
  for (int j = threadIdx.x; j < 2 * d; j += blockDim.x) {
    int q = j / d, c = j % d;
    float acc = 0.f;
    for (int ww = 0; ww < kLnWaves; ++ww) acc += lds[(ww * 2 + q) * d + c];
    part[((long)blockIdx.x * 2 + q) * d + c] = acc;  // [block][gamma | beta][d]
  }
}

#define DISPATCH_T(dt, ...)                                     \
  switch (dt) {                                                 \
    case kF32: { using T = float; __VA_ARGS__; break; }         \
    case kBF16: { using T = bf16; __VA_ARGS__; break; }         \
    case kF16: { using T = f16; __VA_ARGS__; break; }           \
    default: throw std::runtime_error("bad dtype code");        \
  }

#define DISPATCH_E(ev, ...)                                        \
  switch (ev) {                                                    \
    case 1: { constexpr int E = 1; __VA_ARGS__; break; }           \
    case 2: { constexpr int E = 2; __VA_ARGS__; break; }           \
    case 4: { constexpr int E = 4; __VA_ARGS__; break; }           \
    case 8: { constexpr int E = 8; __VA_ARGS__; break; }           \
    case 16: { constexpr int E = 16; __VA_ARGS__; break; }         \
    case 32: { constexpr int E = 32; __VA_ARGS__; break; }         \
    default: throw std::runtime_error("layernorm: d must be 64*{1,2,4,8,16,32}"); \
  }

void layernorm_fwd(uint64_t x, uint64_t a, uint64_t b, uint64_t y, uint64_t mean, uint64_t rstd, long rows, int d,
                   float eps, int dt_x, int dt_y, int dt_w, uint64_t stream) {
  FDT_CHECK(d % 64 == 0 && d / 64 <= kMaxE, "layernorm: unsupported d");
  FDT_CHECK(dt_w == kF32, "layernorm weights must be fp32");
  dim3 grid((unsigned)((rows + kLnWaves - 1) / kLnWaves));
  if (rows == 0) return;
  DISPATCH_T(dt_x, {
    using TX = T;
    DISPATCH_T(dt_y, {
      DISPATCH_E(d / 64, {
        layernorm_fwd_kernel<E, TX, T, float><<<grid, 64 * kLnWaves, 0, as_stream(stream)>>>(
            P<const TX>(x), P<const float>(a), P<const float>(b), P<T>(y), P<float>(mean), P<float>(rstd), rows, d, eps);
      });
    });
  });
  FDT_LAUNCH_CHECK();
}

// part: [2][nblk][d] fp32 (dgamma partials, dbeta partials); caller sums over nblk.
void layernorm_bwd(uint64_t gy, uint64_t x, uint64_t a, uint64_t mean, uint64_t rstd, uint64_t gx, uint64_t gres,
                   uint64_t part, long rows, int d, int nblk, int dt_g, int dt_x, int dt_w, float eps, uint64_t stream) {
  FDT_CHECK(d % 64 == 0 && d / 64 <= kMaxE, "layernorm: unsupported d");
  FDT_CHECK(dt_w == kF32, "layernorm weights must be fp32");
  if (rows == 0) return;
  long rpb = (rows + nblk - 1) / nblk;
  size_t lds = (size_t)kLnWaves * 2 * d * sizeof(float);
  DISPATCH_T(dt_g, {
    using TG = T;
    DISPATCH_T(dt_x, {
      DISPATCH_E(d / 64, {
        layernorm_bwd_kernel<E, TG, T, float><<<nblk, 64 * kLnWaves, lds, as_stream(stream)>>>(
            P<const TG>(gy), P<const T>(x), P<const float>(a), P<const float>(mean), P<const float>(rstd), P<T>(gx),
            P<const T>(gres), P<float>(part), rows, d, rpb, eps);
      });
    });
  });
  FDT_LAUNCH_CHECK();
}

}  // namespace fdt
