// Online natural-gradient (NGD) preconditioner update -- the rank x rank "small math" of one
// update step, fused (optim/ngd.py NGState._step; reference ngd_optimizer.py:205-324).
//
// Written with PyTorch ops this is ~70 launches per (shape group, axis) on [G,R] / [G,R,R]
// tensors (R <= 80): thousands of tiny kernels per NGD update step whose launch latency,
// not arithmetic, bounds the step.  Here it is two launches per (group, axis), one
// workgroup per preconditioner g:
//
//   ngd_pre_eigh : (K = J J^T, L, d, rho)           -> Z (symmetric, to the eigensolver),
//                                                      ise = e^-1/2, drho = d + rho, zs, sum d
//   ngd_post_eigh: (eigenpairs of Z ascending, ...)  -> A = U^T diag(lp) diag(ise) (R x R),
//                                                      wc, and d, rho updated in place
// followed on the host side by W <- A (J + wc W) (one batched GEMM).  fp32 throughout,
// same expressions as the PyTorch formulation (GPU test compares the two).
#include "common.h"

namespace fdt {

constexpr int kNgdMaxR = 128;
constexpr float kNgdEpsilon = 1.0e-10f;
constexpr float kNgdDelta = 5.0e-4f;

__device__ __forceinline__ float block_sum256(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

__device__ __forceinline__ float block_max256(float v, float* red) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

__global__ __launch_bounds__(256) void ngd_pre_eigh_kernel(const float* __restrict__ K, const float* __restrict__ L,
                                                           const float* __restrict__ d, const float* __restrict__ rho,
                                                           float* __restrict__ Z, float* __restrict__ ise_o,
                                                           float* __restrict__ drho_o, float* __restrict__ zs_o,
                                                           float* __restrict__ dsum_o, int R, float alpha, float eta,
                                                           float N, float D) {
  __shared__ float s_ise[kNgdMaxR], s_drho[kNgdMaxR], red[4];
  const int g = blockIdx.x, tid = threadIdx.x;
  const float* Kg = K + (long)g * R * R;
  const float* Lg = L + (long)g * R * R;
  const float* dg = d + (long)g * R;
  const float rh = rho[g];
  float ds = 0.f, tr = 0.f;
  for (int i = tid; i < R; i += 256) { ds += dg[i]; tr += Kg[i * R + i]; }
  const float dsum = block_sum256(ds, red);
  const float trK = block_sum256(tr, red);
  const float beta = rh * (1.f + alpha) + alpha * dsum / D;
  const float zs = fmaxf(trK, 1.f);
  for (int i = tid; i < R; i += 256) {
    const float e = 1.f / (beta / dg[i] + 1.f);
    const float is = rsqrtf(e);
    s_ise[i] = is;
    s_drho[i] = dg[i] + rh;
    ise_o[(long)g * R + i] = is;
    drho_o[(long)g * R + i] = dg[i] + rh;
  }
  if (tid == 0) { zs_o[g] = zs; dsum_o[g] = dsum; }
  __syncthreads();
  const float en = eta / N;
  const float c1 = en * en / zs, c2 = en * (1.f - eta) / zs, c3 = (1.f - eta) * (1.f - eta) / zs;
  float* Zg = Z + (long)g * R * R;
  for (int e = tid; e < R * R; e += 256) {
    const int i = e / R, j = e - i * R;
    const float oo = s_ise[i] * s_ise[j];
    // o1 + o1^T = ise_i ise_j (drho_j + drho_i)
    float z = Kg[e] * (c1 * oo) + Lg[e] * (c2 * (s_ise[i] * (s_ise[j] * s_drho[j]) + s_ise[j] * (s_ise[i] * s_drho[i])));
    if (i == j) z += c3 * s_drho[i] * s_drho[i];
    Zg[e] = z;
  }
}

// c: eigenvalues ascending [G][R]; U: eigenvectors as columns, ascending [G][R][R].
__global__ __launch_bounds__(256) void ngd_post_eigh_kernel(const float* __restrict__ c, const float* __restrict__ U,
                                                            const float* __restrict__ ise, const float* __restrict__ drho,
                                                            const float* __restrict__ zs_in, const float* __restrict__ dsum_in,
                                                            const float* __restrict__ trXX, float* __restrict__ d,
                                                            float* __restrict__ rho, float* __restrict__ A,
                                                            float* __restrict__ wc, int R, float alpha, float eta, float N,
                                                            float D) {
  __shared__ float s_sqc[kNgdMaxR], s_lp[kNgdMaxR], s_ise[kNgdMaxR], red[4];
  const int g = blockIdx.x, tid = threadIdx.x;
  const float rh = rho[g], zs = zs_in[g], dsum = dsum_in[g];
  const float en = eta / N;
  const float cfl = (rh * (1.f - eta)) * (rh * (1.f - eta)) / zs;
  float part = 0.f, mx = 0.f;
  for (int k = tid; k < R; k += 256) {
    const float ck = fmaxf(c[(long)g * R + (R - 1 - k)], cfl);  // descending order
    const float sq = sqrtf(ck) * sqrtf(zs);
    s_sqc[k] = sq;
    part += sq;
    mx = fmaxf(mx, sq);
    s_ise[k] = ise[(long)g * R + k];
  }
  const float sum_sqc = block_sum256(part, red);
  const float max_sqc = block_max256(mx, red);
  float rho1 = (en * trXX[g] + (1.f - eta) * (D * rh + dsum) - sum_sqc) / (D - (float)R);
  const float floor = fmaxf(kNgdDelta * max_sqc, kNgdEpsilon);
  float pd = 0.f;
  for (int k = tid; k < R; k += 256) {
    const float d1 = fmaxf(s_sqc[k] - rho1, floor);
    d[(long)g * R + k] = d1;
    pd += d1;
  }
  const float sum_d1 = block_sum256(pd, red);  // (its barriers also order the d writes)
  rho1 = fmaxf(rho1, floor);
  const float beta1 = rho1 * (1.f + alpha) + alpha * sum_d1 / D;
  for (int k = tid; k < R; k += 256) {
    const float d1 = d[(long)g * R + k];
    const float e1 = 1.f / (beta1 / d1 + 1.f);
    s_lp[k] = en * sqrtf(e1) / s_sqc[k];
    wc[(long)g * R + k] = ((1.f - eta) / en) * drho[(long)g * R + k];
  }
  __syncthreads();
  if (tid == 0) rho[g] = rho1;
  // A[k][j] = U_desc[j][k] * lp[k] * ise[j],  U_desc[:, k] = U[:, R-1-k]
  const float* Ug = U + (long)g * R * R;
  float* Ag = A + (long)g * R * R;
  for (int e = tid; e < R * R; e += 256) {
    const int k = e / R, j = e - k * R;
    Ag[e] = Ug[j * R + (R - 1 - k)] * s_lp[k] * s_ise[j];
  }
}

// ---------------------------------------------------------------- norm-preserving rescale
// The preconditioned direction keeps the Frobenius norm of the input per matrix g
// (reference ngd_optimizer.py:151-168):  Y <- isnan(|Y|^2) ? X : Y * sqrt(|X|^2 / |Y|^2).
// ngd_sumsq: out[g] += sum of squares of the g-th slab (float4 loads, block reduce, one
// atomic per block; out zeroed by the caller) -- one launch instead of square + reduce.
__global__ __launch_bounds__(256) void ngd_sumsq_kernel(const float* __restrict__ X, long per, int chunks,
                                                        float* __restrict__ out) {
  __shared__ float red[4];
  const int g = blockIdx.x / chunks, ch = blockIdx.x - g * chunks;
  const float* x = X + (long)g * per;
  const long n4 = per / 4;
  const long b0 = n4 * ch / chunks, b1 = n4 * (ch + 1) / chunks;
  float acc = 0.f;
  for (long i = b0 + threadIdx.x; i < b1; i += 256) {
    const float4 v = reinterpret_cast<const float4*>(x)[i];
    acc = fmaf(v.x, v.x, fmaf(v.y, v.y, fmaf(v.z, v.z, fmaf(v.w, v.w, acc))));
  }
  if (ch == chunks - 1)
    for (long i = n4 * 4 + threadIdx.x; i < per; i += 256) acc = fmaf(x[i], x[i], acc);
  acc = block_sum256(acc, red);
  if (threadIdx.x == 0) atomicAdd(out + g, acc);
}

__global__ __launch_bounds__(256) void ngd_rescale_kernel(const float* __restrict__ X, float* __restrict__ Y, long per,
                                                          int chunks, const float* __restrict__ ip,
                                                          const float* __restrict__ fp) {
  // X is read only by the (block-uniform) NaN branch; float4 body + scalar tail
  const int g = blockIdx.x / chunks, ch = blockIdx.x - g * chunks;
  const float f = fp[g];
  const bool bad = isnan(f);
  const float sc = sqrtf(ip[g] / (f + 1e-30f));
  const float* x = X + (long)g * per;
  float* y = Y + (long)g * per;
  const long n4 = per / 4;
  const long b0 = n4 * ch / chunks, b1 = n4 * (ch + 1) / chunks;
  float4* y4 = reinterpret_cast<float4*>(y);
  if (bad) {
    const float4* x4 = reinterpret_cast<const float4*>(x);
    for (long i = b0 + threadIdx.x; i < b1; i += 256) y4[i] = x4[i];
    if (ch == chunks - 1)
      for (long i = n4 * 4 + threadIdx.x; i < per; i += 256) y[i] = x[i];
    return;
  }
  for (long i = b0 + threadIdx.x; i < b1; i += 256) {
    float4 v = y4[i];
    v.x *= sc; v.y *= sc; v.z *= sc; v.w *= sc;
    y4[i] = v;
  }
  if (ch == chunks - 1)
    for (long i = n4 * 4 + threadIdx.x; i < per; i += 256) y[i] *= sc;
}

// ---------------------------------------------------------------- tiny-dim axes (D <= 8)
// The kh / kw axes of the 3x3 convs (D = 3, R = 2, N up to 2.4M rows per matrix) as batched
// GEMMs are the worst shapes there are: H = X W^T has K = 3, and J = H^T X is a 2 x 3 output
// with a 786K-long reduction that the library tiles as a handful of 16x16 workgroups (~250 us
// each, measured).  It is one streaming pass: each thread owns rows, keeps W (R x D) in
// registers, and produces in one read of X
//   Xh = X - (X W^T) W  (written in X's own layout, so no transpose copies),
//   |X|^2, |Xh|^2, and (update steps) J = H^T X, H^T H  -- block-reduced into per-workgroup
//   partial slots, summed in workgroup order by ngd_small_sums_kernel (bitwise repeatable).
// X is addressed in the parameter's canonical layout: element (g, a, d, b) of a
// [G][A][D][B] tensor, row n = a * B + b (the transpose the GEMM path copies into).
template <int D, int R>
__global__ __launch_bounds__(256) void ngd_small_proj_kernel(const float* __restrict__ X, float* __restrict__ Y,
                                                             const float* __restrict__ W, int A, int B, int chunks,
                                                             float* __restrict__ part, bool upd) {
  constexpr int NV = 2 + R * D + R * R;
  __shared__ float red[4][NV];
  const int g = blockIdx.x / chunks, ch = blockIdx.x - g * chunks;
  const int per = A * D * B, rows = A * B;
  const float* x = X + (long)g * per;
  float* y = Y + (long)g * per;
  float w[R][D];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int d = 0; d < D; ++d) w[r][d] = W[((long)g * R + r) * D + d];
  float v[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = 0.f;
  const int r0 = (int)((long)rows * ch / chunks), r1 = (int)((long)rows * (ch + 1) / chunks);
  for (int n = r0 + threadIdx.x; n < r1; n += 256) {
    const int a = n / B, b = n - a * B;
    const int base = a * D * B + b;
    float xv[D], h[R];
#pragma unroll
    for (int d = 0; d < D; ++d) xv[d] = x[base + d * B];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < D; ++d) s = fmaf(w[r][d], xv[d], s);
      h[r] = s;
    }
#pragma unroll
    for (int d = 0; d < D; ++d) {
      float o = xv[d];
#pragma unroll
      for (int r = 0; r < R; ++r) o = fmaf(-h[r], w[r][d], o);
      y[base + d * B] = o;
      v[0] = fmaf(xv[d], xv[d], v[0]);
      v[1] = fmaf(o, o, v[1]);
    }
    if (upd) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
#pragma unroll
        for (int d = 0; d < D; ++d) v[2 + r * D + d] = fmaf(h[r], xv[d], v[2 + r * D + d]);
#pragma unroll
        for (int s = 0; s < R; ++s) v[2 + R * D + r * R + s] = fmaf(h[r], h[s], v[2 + R * D + r * R + s]);
      }
    }
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nv = upd ? NV : 2;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    if (i < nv) {
      const float s = wave_sum(v[i]);
      if (lane == 0) red[wv][i] = s;
    }
  }
  __syncthreads();
  // per-workgroup partials, summed in a fixed order by ngd_small_sums_kernel (no atomics)
  float* out = part + ((long)g * chunks + ch) * NV;
  for (int i = threadIdx.x; i < nv; i += 256) out[i] = red[0][i] + red[1][i] + red[2][i] + red[3][i];
}

// sums[0][g] = |X|^2, sums[1][g] = |Y|^2, J[g], HH[g] from the partials of the g-th matrix's
// workgroups, in workgroup order
__global__ __launch_bounds__(256) void ngd_small_sums_kernel(const float* __restrict__ part, int chunks, int nv, int NV,
                                                             int RD, float* __restrict__ sums, float* __restrict__ J,
                                                             float* __restrict__ HH) {
  const int g = blockIdx.x, G = gridDim.x;
  for (int i = threadIdx.x; i < nv; i += 256) {
    float s = 0.f;
    for (int c = 0; c < chunks; ++c) s += part[((long)g * chunks + c) * NV + i];
    if (i < 2) sums[(long)i * G + g] = s;
    else if (i < 2 + RD) J[(long)g * RD + (i - 2)] = s;
    else HH[(long)g * (NV - 2 - RD) + (i - 2 - RD)] = s;
  }
}

bool ngd_small_supported(int D, int R) {
  return (D == 2 && R == 1) || (D == 3 && R == 2) || (D == 4 && R == 2) || (D == 5 && R == 3) ||
         (D == 6 && R == 3) || (D == 7 && R == 4) || (D == 8 && R == 4);
}

static long small_chunks(long rows) {
  long ch = rows / (256 * 16);  // ~16 rows per thread
  if (ch < 1) ch = 1;
  if (ch > 1024) ch = 1024;
  return ch;
}

long ngd_small_part_numel(int G, int A, int D, int B, int R) {
  return (long)G * small_chunks((long)A * B) * (2 + R * D + R * R);
}

void ngd_small_proj(uint64_t X, uint64_t Y, uint64_t W, int G, int A, int D, int B, int R, uint64_t sums, uint64_t J,
                    uint64_t HH, uint64_t part, uint64_t stream) {
  FDT_CHECK(ngd_small_supported(D, R), "ngd_small_proj: unsupported (dim, rank)");
  FDT_CHECK((long)A * D * B < (1L << 31), "ngd_small_proj: matrix too large");
  FDT_CHECK((J == 0) == (HH == 0), "ngd_small_proj: J and HH together");
  FDT_CHECK(part != 0, "ngd_small_proj: partial-sum buffer required");
  if (G == 0 || A == 0 || B == 0) return;
  const long ch = small_chunks((long)A * B);
  const dim3 grid((unsigned)(G * ch));
  const bool upd = J != 0;
  hipStream_t s = as_stream(stream);
#define FDT_NGD_SMALL(DD, RR)                                                                                      \
  if (D == DD && R == RR)                                                                                         \
    ngd_small_proj_kernel<DD, RR><<<grid, 256, 0, s>>>(P<const float>(X), P<float>(Y), P<const float>(W), A, B, \
                                                       (int)ch, P<float>(part), upd);
  FDT_NGD_SMALL(2, 1) FDT_NGD_SMALL(3, 2) FDT_NGD_SMALL(4, 2) FDT_NGD_SMALL(5, 3) FDT_NGD_SMALL(6, 3)
  FDT_NGD_SMALL(7, 4) FDT_NGD_SMALL(8, 4)
#undef FDT_NGD_SMALL
  FDT_LAUNCH_CHECK();
  const int NV = 2 + R * D + R * R;
  ngd_small_sums_kernel<<<G, 256, 0, s>>>(P<const float>(part), (int)ch, upd ? NV : 2, NV, R * D, P<float>(sums),
                                          P<float>(J), P<float>(HH));
  FDT_LAUNCH_CHECK();
}

// ---------------------------------------------------------------- general axes (D >= 9)
// One axis of a stacked parameter in its OWN layout [G][A][D][B] (row n = a B + b, the D
// elements of a row strided by B): what the PyTorch formulation does as transpose copy ->
// H = X W^T (batched GEMM) -> Xh = X - H W (batched GEMM) -> |X|^2, |Xh|^2 reductions, and
// on update steps J = H^T X and H^T H (two more batched GEMMs) -- six or more launches with
// a full read or write of X each, the GEMMs at [N x D] x [D x R<=80] shapes that the library
// tiles poorly (profiles/ngd_step_bench.txt) -- is one kernel here.  A workgroup owns 64 rows
// of one matrix g:
//   phase 1  H[64][R] = X_tile W^T over 32-wide d chunks staged in LDS (fp32 FMA, each
//            thread a 4-row x 5-rank register block, float4 LDS reads), |X|^2 on the way;
//            H^T H of the tile (update steps, when the caller needs it) -> atomics;
//   phase 2  per d chunk again (second read of X: L2): Y = X - H W (4 rows x 2 d per
//            thread, W staged transposed so both operands are float4 reads), J += H^T X
//            (update steps) -> atomics, Y staged through LDS so the store is coalesced in
//            the tensor's own layout, |Y|^2 on the way.
// The norm-preserving rescale of Y (and its NaN guard) stays ngd_rescale: it needs |Y|^2 of
// the whole matrix.  fp32 throughout (the NGD golden tests compare against fp64).
constexpr int kPN = 64;      // rows per workgroup
constexpr int kPD = 32;      // d per staged chunk
constexpr int kPR = 80;      // max rank
constexpr int kXs = kPD + 4;  // [row][d] stride (float4-aligned)
constexpr int kWr = kPD + 4;  // W as [r][d] (phase 1)
constexpr int kWd = kPR + 4;  // W as [d][r] (phase 2); also the H stride

// X chunk [kPN rows][kPD d] of one row tile: global -> 8 registers per thread (issued a chunk
// ahead, so the loads are in flight during the previous chunk's FMAs), then -> LDS.
//   VEC (B = 1, D % 4 == 0): rows contiguous in d, float4 loads: thread -> row (q >> 3),
//                            d 4 (q & 7) for q = tid + 256 i, i < 2
//   B > 1: thread -> row tid & 63 (consecutive b: coalesced), d (tid >> 6) + 4 i
//   B = 1: thread -> d tid & 31, rows (tid >> 5) + 8 i
template <bool VEC>
__device__ __forceinline__ void proj_load_x(float (&v)[8], const float* x, long n0, long N, int dend, int D, int B,
                                            int d0, int tid) {
  if (VEC) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = tid + 256 * i;
      const long n = n0 + (q >> 3);
      const int d = d0 + 4 * (q & 7);
      const float4 t = (n < N && d < dend) ? *reinterpret_cast<const float4*>(x + n * D + d)
                                           : make_float4(0.f, 0.f, 0.f, 0.f);
      v[4 * i] = t.x; v[4 * i + 1] = t.y; v[4 * i + 2] = t.z; v[4 * i + 3] = t.w;
    }
  } else if (B > 1) {
    const long n = n0 + (tid & 63);
    const bool rv = n < N;
    const long a = rv ? n / B : 0, b = rv ? n - a * B : 0;
    const float* xr = x + a * (long)D * B + b;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int d = d0 + (tid >> 6) + 4 * i;
      v[i] = (rv && d < dend) ? xr[(long)d * B] : 0.f;
    }
  } else {
    const int d = d0 + (tid & 31);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const long n = n0 + (tid >> 5) + 8 * i;
      v[i] = (n < N && d < dend) ? x[n * D + d] : 0.f;
    }
  }
}

template <bool VEC>
__device__ __forceinline__ void proj_put_x(float* Xs, const float (&v)[8], int B, int tid, float* sq) {
  if (VEC) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = tid + 256 * i;
      *reinterpret_cast<float4*>(Xs + (q >> 3) * kXs + 4 * (q & 7)) =
          make_float4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = B > 1 ? (tid & 63) : (tid >> 5) + 8 * i;
      const int dd = B > 1 ? (tid >> 6) + 4 * i : (tid & 31);
      Xs[row * kXs + dd] = v[i];
    }
  }
  if (sq) {
#pragma unroll
    for (int i = 0; i < 8; ++i) *sq = fmaf(v[i], v[i], *sq);
  }
}

// W chunk [80 r][kPD d]: VEC -> float4 (r = q >> 3, d 4 (q & 7), q = tid + 256 i < 640);
// else thread -> d tid & 31, r (tid >> 5) + 8 i
template <bool VEC>
__device__ __forceinline__ void proj_load_w(float (&v)[12], const float* w, int R, int D, int dend, int d0, int tid) {
  if (VEC) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int q = tid + 256 * i;
      const int r = q >> 3, d = d0 + 4 * (q & 7);
      const float4 t = (q < kPR * 8 && r < R && d < dend) ? *reinterpret_cast<const float4*>(w + (long)r * D + d)
                                                          : make_float4(0.f, 0.f, 0.f, 0.f);
      v[4 * i] = t.x; v[4 * i + 1] = t.y; v[4 * i + 2] = t.z; v[4 * i + 3] = t.w;
    }
  } else {
    const int d = d0 + (tid & 31);
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      const int r = (tid >> 5) + 8 * i;
      v[i] = (r < R && d < dend) ? w[(long)r * D + d] : 0.f;
    }
  }
}

// W chunk into LDS as [r][d] (stride kWr) or [d][r] (stride kWd)
template <bool VEC, bool RD>
__device__ __forceinline__ void proj_put_w(float* Ws, const float (&v)[12], int tid) {
  if (VEC) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int q = tid + 256 * i;
      if (q >= kPR * 8) continue;
      const int r = q >> 3, c = 4 * (q & 7);
      if (RD) {
        *reinterpret_cast<float4*>(Ws + r * kWr + c) = make_float4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) Ws[(c + j) * kWd + r] = v[4 * i + j];
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      const int r = (tid >> 5) + 8 * i, dd = tid & 31;
      if (RD) Ws[r * kWr + dd] = v[i];
      else Ws[dd * kWd + r] = v[i];
    }
  }
}

__device__ __forceinline__ void proj_store_y(const float* Ys, float* y, long n0, long N, int dend, int D, int B,
                                             int d0, int tid, float* sq) {
  if (B > 1) {
    const long n = n0 + (tid & 63);
    const int row = tid & 63;
    if (n >= N) return;
    const long a = n / B, b = n - a * B;
    float* yr = y + a * (long)D * B + b;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int dd = (tid >> 6) + 4 * i, d = d0 + dd;
      if (d < dend) {
        const float v = Ys[row * kXs + dd];
        yr[(long)d * B] = v;
        *sq = fmaf(v, v, *sq);
      }
    }
  } else {
    const int dd = tid & 31, d = d0 + dd;
    if (d >= dend) return;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = (tid >> 5) + 8 * i;
      const long n = n0 + row;
      if (n < N) {
        const float v = Ys[row * kXs + dd];
        y[n * D + d] = v;
        *sq = fmaf(v, v, *sq);
      }
    }
  }
}

// Split over d as well as rows: a [N x D] matrix with few rows and a long D (ResNet's
// [2048, 512] axis 0: 8 row tiles; the transformer embedding's 30522-long axis) would
// otherwise run as a handful of workgroups walking D serially.  Kernel 1 accumulates
// partial H of one (row tile, d range) into Hbuf [G][N][R] (atomics when D is split);
// kernel 2 reloads the tile's H and produces Y, J and |Y|^2 over its own d range.
// Every reduction across workgroups goes through per-workgroup partial slots summed in a
// fixed order afterwards (ngd_proj_sums_kernel / ngd_slab_sum_kernel): no atomics, so the
// projection is bitwise repeatable (NGD's early near-degenerate eigenproblems turn atomic-
// order noise into O(1) run-to-run differences).
struct ProjArgs {
  const float* X;
  float* Y;
  const float* W;
  float* H;    // [G][N][R] (+ ds slabs of partial H when d is split)
  float* ipp;  // [G][tiles * ds] partial |X|^2 (nullptr: not wanted)
  float* fpp;  // [G][tiles * ds] partial |Y|^2
  float* Jp;   // [tiles][G][R][D] partial J (nullptr: not an update step)
  float* HHp;  // [tiles][G][R][R] partial H^T H (nullptr: not wanted)
  int A, D, B, R;
  int tiles, ds, dlen;  // row tiles, d splits, d per split (multiple of kPD)
};

// MF: the chunk products run on the matrix cores (v_mfma_f32_16x16x4_f32: exact fp32, one
// rounding per product, k-ordered -- the same fmaf chain in the same d / r / n order as the
// VALU loops, so both forms give identical bits).  Operand map of 16x16x4: lane l supplies
// A[l & 15][k = l >> 4] and B[k = l >> 4][l & 15]; C[4 (l >> 4) + v][l & 15] in register v.
typedef float ngd_f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ ngd_f32x4 mfma4(float a, float b, ngd_f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// 1 = the matrix-core forms (default), 0 = the VALU loops (FDT_NGD_MFMA=0, A/B; ngd_mfma())
static int g_ngd_mfma = -1;
static bool ngd_mfma_on() {
  if (g_ngd_mfma < 0) {
    const char* e = getenv("FDT_NGD_MFMA");
    g_ngd_mfma = (e && e[0] == '0') ? 0 : 1;
  }
  return g_ngd_mfma != 0;
}

template <bool VEC, bool MF>
__global__ __launch_bounds__(256) void ngd_proj_h_kernel(ProjArgs p) {
  __shared__ __attribute__((aligned(16))) float Xs[kPN * kXs];
  __shared__ __attribute__((aligned(16))) float Ws[kPR * kWr];
  __shared__ float red[4];
  const int tid = threadIdx.x;
  const int per_g = p.tiles * p.ds;
  const int g = blockIdx.x / per_g, rem = blockIdx.x - g * per_g;
  const int tile = rem / p.ds, sp = rem - tile * p.ds;
  const int D = p.D, R = p.R;
  const long N = (long)p.A * p.B;
  const long n0 = (long)tile * kPN;
  const float* x = p.X + g * N * D;
  const float* w = p.W + (long)g * R * D;
  const int dbeg = sp * p.dlen, dend = min(D, dbeg + p.dlen);
  const int tr = tid >> 4, tc = tid & 15;
  float sx = 0.f;
  float acc[4][5];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 5; ++j) acc[i][j] = 0.f;
  ngd_f32x4 hm[5];
#pragma unroll
  for (int t = 0; t < 5; ++t) hm[t] = ngd_f32x4{0.f, 0.f, 0.f, 0.f};
  float xv8[8], wv12[12];
  if (dbeg < dend) {
    proj_load_x<VEC>(xv8, x, n0, N, dend, D, p.B, dbeg, tid);
    proj_load_w<VEC>(wv12, w, R, D, dend, dbeg, tid);
  }
  for (int d0 = dbeg; d0 < dend; d0 += kPD) {
    proj_put_x<VEC>(Xs, xv8, p.B, tid, p.ipp ? &sx : nullptr);
    proj_put_w<VEC, true>(Ws, wv12, tid);  // W chunk as [r][d]
    __syncthreads();
    if (d0 + kPD < dend) {  // next chunk's loads in flight during this chunk's FMAs
      proj_load_x<VEC>(xv8, x, n0, N, dend, D, p.B, d0 + kPD, tid);
      proj_load_w<VEC>(wv12, w, R, D, dend, d0 + kPD, tid);
    }
    __syncthreads();
    if constexpr (MF) {
      // wave w: rows 16w..16w+15 x the 5 rank tiles (5 independent accumulators)
      const int lr = tid & 15, lk = (tid >> 4) & 3, w = tid >> 6;
#pragma unroll
      for (int kk = 0; kk < kPD / 4; ++kk) {
        const float a = Xs[(16 * w + lr) * kXs + 4 * kk + lk];
#pragma unroll
        for (int t = 0; t < 5; ++t) hm[t] = mfma4(a, Ws[(16 * t + lr) * kWr + 4 * kk + lk], hm[t]);
      }
    } else {
#pragma unroll 2
    for (int dq = 0; dq < kPD; dq += 4) {
      float4 xv[4], wv[5];
#pragma unroll
      for (int i = 0; i < 4; ++i) xv[i] = *reinterpret_cast<const float4*>(Xs + (4 * tr + i) * kXs + dq);
#pragma unroll
      for (int j = 0; j < 5; ++j) wv[j] = *reinterpret_cast<const float4*>(Ws + (tc + 16 * j) * kWr + dq);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 5; ++j) {
          acc[i][j] = fmaf(xv[i].x, wv[j].x, acc[i][j]);
          acc[i][j] = fmaf(xv[i].y, wv[j].y, acc[i][j]);
          acc[i][j] = fmaf(xv[i].z, wv[j].z, acc[i][j]);
          acc[i][j] = fmaf(xv[i].w, wv[j].w, acc[i][j]);
        }
    }
    }
    __syncthreads();
  }
  float* h = p.H + g * N * R;
  if constexpr (MF) {
    const int lr = tid & 15, lk = (tid >> 4) & 3, w = tid >> 6;
#pragma unroll
    for (int t = 0; t < 5; ++t) {
      const int r = 16 * t + lr;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const long n = n0 + 16 * w + 4 * lk + v;
        if (n >= N || r >= R) continue;
        if (p.ds == 1) h[n * R + r] = hm[t][v];
        else p.H[((long)sp * (gridDim.x / per_g) + g) * N * R + n * R + r] = hm[t][v];
      }
    }
  } else {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const long n = n0 + 4 * tr + i;
    if (n >= N) continue;
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const int r = tc + 16 * j;
      if (r >= R) continue;
      if (p.ds == 1) h[n * R + r] = acc[i][j];
      else p.H[((long)sp * (gridDim.x / per_g) + g) * N * R + n * R + r] = acc[i][j];  // slab sp
    }
  }
  }
  if (p.ipp != nullptr) {
    sx = block_sum256(sx, red);
    if (tid == 0) p.ipp[(long)g * per_g + rem] = sx;
  }
}

// STR (strided axis, B > 1): a thread owns one row and 8 consecutive d (lanes = rows =
// consecutive b), so Y goes out as coalesced stores straight from registers and each H
// float4 feeds 32 FMAs (W reads are wave-uniform broadcasts); the [4 rows x 2 d] mapping
// needed an LDS round trip and two extra barriers per chunk for the strided store and sat
// at ~0.63 of its wave cycles waiting (profiles/pmc/ngd_proj_counters.md).
template <bool VEC, bool STR, bool MF>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void ngd_proj_y_kernel(ProjArgs p) {
  __shared__ __attribute__((aligned(16))) float Xs[kPN * kXs];
  __shared__ __attribute__((aligned(16))) float Ws[kPD * kWd];
  __shared__ __attribute__((aligned(16))) float Hs[kPN * kWd];
  __shared__ float red[4];
  const int tid = threadIdx.x;
  const int per_g = p.tiles * p.ds;
  const int g = blockIdx.x / per_g, rem = blockIdx.x - g * per_g;
  const int tile = rem / p.ds, sp = rem - tile * p.ds;
  const int D = p.D, R = p.R;
  const long N = (long)p.A * p.B;
  const long n0 = (long)tile * kPN;
  const float* x = p.X + g * N * D;
  float* y = p.Y + g * N * D;
  const float* w = p.W + (long)g * R * D;
  const float* h = p.H + g * N * R;
  const int dbeg = sp * p.dlen, dend = min(D, dbeg + p.dlen);
  const int tr = tid >> 4, tc = tid & 15;
  if ((R & 3) == 0) {  // the tile's H rows are one contiguous [rows][R] block: float4 loads
    const long nrows = N - n0 < kPN ? N - n0 : kPN;
    const int q4 = R >> 2;
    for (int e = tid; e < kPN * (kPR / 4); e += 256) {
      const int row = e / (kPR / 4), c = 4 * (e - row * (kPR / 4));
      float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
      if (row < nrows && c < R) t = reinterpret_cast<const float4*>(h + (n0 + row) * R)[c >> 2];
      *reinterpret_cast<float4*>(Hs + row * kWd + c) = t;
    }
    (void)q4;
  } else {
    for (int e = tid; e < kPN * kPR; e += 256) {  // H rows of the tile, zero past N / R
      const int row = e / kPR, r = e - row * kPR;
      const long n = n0 + row;
      Hs[row * kWd + r] = (n < N && r < R) ? h[n * R + r] : 0.f;
    }
  }
  __syncthreads();
  if (p.HHp != nullptr && sp == 0) {
    const int G = gridDim.x / per_g;
    for (int e = tid; e < R * R; e += 256) {
      const int r = e / R, q = e - r * R;
      float s = 0.f;
#pragma unroll 8
      for (int n = 0; n < kPN; ++n) s = fmaf(Hs[n * kWd + r], Hs[n * kWd + q], s);
      p.HHp[((long)tile * G + g) * R * R + e] = s;
    }
  }
  float sy = 0.f;
  float xv8[8], wv12[12];
  if (dbeg < dend) {
    proj_load_x<VEC>(xv8, x, n0, N, dend, D, p.B, dbeg, tid);
    proj_load_w<VEC>(wv12, w, R, D, dend, dbeg, tid);
  }
  for (int d0 = dbeg; d0 < dend; d0 += kPD) {
    proj_put_x<VEC>(Xs, xv8, p.B, tid, nullptr);
    proj_put_w<VEC, false>(Ws, wv12, tid);  // W chunk as [d][r]
    __syncthreads();
    if (d0 + kPD < dend) {
      proj_load_x<VEC>(xv8, x, n0, N, dend, D, p.B, d0 + kPD, tid);
      proj_load_w<VEC>(wv12, w, R, D, dend, d0 + kPD, tid);
    }
    float yv[4][2];
    float ys[8];
    ngd_f32x4 ym[2];
    const int lr = tid & 15, lk = (tid >> 4) & 3, wv_ = tid >> 6;
    const int nk4 = (R + 3) >> 2;  // (H / W columns past R are zero)
    if constexpr (MF) {
      if constexpr (STR) {
        // Y^T [d][n] = X^T - W^T H^T: C columns = rows n (lanes -> consecutive b: coalesced
        // strided stores); wave w: n tile w, d tiles 0 and 1
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int v = 0; v < 4; ++v) ym[j][v] = Xs[(16 * wv_ + lr) * kXs + 16 * j + 4 * lk + v];
        for (int kk = 0; kk < nk4; ++kk) {
          const float hb = -Hs[(16 * wv_ + lr) * kWd + 4 * kk + lk];
#pragma unroll
          for (int j = 0; j < 2; ++j) ym[j] = mfma4(Ws[(16 * j + lr) * kWd + 4 * kk + lk], hb, ym[j]);
        }
      } else {
        // Y [n][d] = X - H W: C columns = d; wave w: rows 16w.., d tiles 0 and 1
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int v = 0; v < 4; ++v) ym[j][v] = Xs[(16 * wv_ + 4 * lk + v) * kXs + 16 * j + lr];
        for (int kk = 0; kk < nk4; ++kk) {
          const float ha = -Hs[(16 * wv_ + lr) * kWd + 4 * kk + lk];
#pragma unroll
          for (int j = 0; j < 2; ++j) ym[j] = mfma4(ha, Ws[(16 * j + lr) * kWd + 4 * kk + lk], ym[j]);
        }
      }
    } else if (STR) {
      const int row = tid & 63, dq = tid >> 6;
      const float4 a0 = *reinterpret_cast<const float4*>(Xs + row * kXs + 8 * dq);
      const float4 a1 = *reinterpret_cast<const float4*>(Xs + row * kXs + 8 * dq + 4);
      ys[0] = a0.x; ys[1] = a0.y; ys[2] = a0.z; ys[3] = a0.w;
      ys[4] = a1.x; ys[5] = a1.y; ys[6] = a1.z; ys[7] = a1.w;
#pragma unroll 2
      for (int r0 = 0; r0 < R; r0 += 4) {
        const float4 hv = *reinterpret_cast<const float4*>(Hs + row * kWd + r0);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float4 wk = *reinterpret_cast<const float4*>(Ws + (8 * dq + k) * kWd + r0);
          float v = ys[k];
          v = fmaf(-hv.x, wk.x, v);
          v = fmaf(-hv.y, wk.y, v);
          v = fmaf(-hv.z, wk.z, v);
          v = fmaf(-hv.w, wk.w, v);
          ys[k] = v;
        }
      }
    } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int k = 0; k < 2; ++k) yv[i][k] = Xs[(4 * tr + i) * kXs + tc + 16 * k];
#pragma unroll 2
    for (int r0 = 0; r0 < R; r0 += 4) {  // H / W columns past R are zero
      float4 hv[4], wv[2];
#pragma unroll
      for (int i = 0; i < 4; ++i) hv[i] = *reinterpret_cast<const float4*>(Hs + (4 * tr + i) * kWd + r0);
#pragma unroll
      for (int k = 0; k < 2; ++k) wv[k] = *reinterpret_cast<const float4*>(Ws + (tc + 16 * k) * kWd + r0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          float v = yv[i][k];
          v = fmaf(-hv[i].x, wv[k].x, v);
          v = fmaf(-hv[i].y, wv[k].y, v);
          v = fmaf(-hv[i].z, wv[k].z, v);
          v = fmaf(-hv[i].w, wv[k].w, v);
          yv[i][k] = v;
        }
    }
    }
    if (MF && p.Jp != nullptr) {
      // J[r][d] = sum_n H[n][r] X[n][d] over the tile's 64 rows: A = H^T (k = n), B = X;
      // wave w: d tile w & 1, rank tiles (w >> 1) + 2 i (5 tiles over 2 wave pairs)
      const int jd = wv_ & 1, t0 = wv_ >> 1;
      ngd_f32x4 jm[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) jm[i] = ngd_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
      for (int kk = 0; kk < kPN / 4; ++kk) {
        const int n = 4 * kk + lk;
        const float xb = Xs[n * kXs + 16 * jd + lr];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const int t = t0 + 2 * i;
          if (t < 5) jm[i] = mfma4(Hs[n * kWd + 16 * t + lr], xb, jm[i]);
        }
      }
      const int d = d0 + 16 * jd + lr;
      if (d < dend) {
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const int t = t0 + 2 * i;
          if (t >= 5) continue;
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const int r = 16 * t + 4 * lk + v;
            if (r < R) p.Jp[(((long)tile * (gridDim.x / per_g) + g) * R + r) * D + d] = jm[i][v];
          }
        }
      }
    } else if (p.Jp != nullptr) {  // J[r][d] += sum_n H[n][r] X[n][d]: thread d = tid & 31, r = (tid >> 5) + 8 j
      const int dd = tid & 31, d = d0 + dd;
      float ja[10];
#pragma unroll
      for (int j = 0; j < 10; ++j) ja[j] = 0.f;
#pragma unroll 4
      for (int n = 0; n < kPN; ++n) {
        const float xv = Xs[n * kXs + dd];
#pragma unroll
        for (int j = 0; j < 10; ++j) ja[j] = fmaf(Hs[n * kWd + (tid >> 5) + 8 * j], xv, ja[j]);
      }
      if (d < dend) {
#pragma unroll
        for (int j = 0; j < 10; ++j) {
          const int r = (tid >> 5) + 8 * j;
          if (r < R) p.Jp[(((long)tile * (gridDim.x / per_g) + g) * R + r) * D + d] = ja[j];
        }
      }
    }
    if (MF && STR) {  // C columns = rows n: lanes -> consecutive b
      const long n = n0 + 16 * wv_ + lr;
      if (n < N) {
        const long a = n / p.B, b = n - a * p.B;
        float* yr = y + a * (long)D * p.B + b;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const int d = d0 + 16 * j + 4 * lk + v;
            if (d < dend) {
              yr[(long)d * p.B] = ym[j][v];
              sy = fmaf(ym[j][v], ym[j][v], sy);
            }
          }
      }
      __syncthreads();  // Xs / Ws reads done before the next chunk is staged
    } else if (MF && VEC) {  // rows contiguous in d: 16 lanes = 64 contiguous bytes
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const long n = n0 + 16 * wv_ + 4 * lk + v;
          const int d = d0 + 16 * j + lr;
          if (n < N && d < dend) {
            y[n * D + d] = ym[j][v];
            sy = fmaf(ym[j][v], ym[j][v], sy);
          }
        }
      __syncthreads();
    } else if (MF) {  // B = 1, unaligned: stage Y through Xs for the coalesced store
      __syncthreads();
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int v = 0; v < 4; ++v) Xs[(16 * wv_ + 4 * lk + v) * kXs + 16 * j + lr] = ym[j][v];
      __syncthreads();
      proj_store_y(Xs, y, n0, N, dend, D, p.B, d0, tid, &sy);
      __syncthreads();
    } else if (STR) {  // lanes = consecutive rows (b): one coalesced store per d
      const int row = tid & 63, dq = tid >> 6;
      const long n = n0 + row;
      if (n < N) {
        const long a = n / p.B, b = n - a * p.B;
        float* yr = y + a * (long)D * p.B + b;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int d = d0 + 8 * dq + k;
          if (d < dend) {
            yr[(long)d * p.B] = ys[k];
            sy = fmaf(ys[k], ys[k], sy);
          }
        }
      }
      __syncthreads();  // Xs / Ws reads done before the next chunk is staged
    } else if (VEC) {  // rows contiguous in d: store Y from registers (16 lanes = 64 contiguous bytes)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const long n = n0 + 4 * tr + i;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int d = d0 + tc + 16 * k;
          if (n < N && d < dend) {
            y[n * D + d] = yv[i][k];
            sy = fmaf(yv[i][k], yv[i][k], sy);
          }
        }
      }
      __syncthreads();  // Xs / Ws reads done before the next chunk is staged
    } else {
      __syncthreads();  // every read of Xs done: stage Y through it (coalesced strided store)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int k = 0; k < 2; ++k) Xs[(4 * tr + i) * kXs + tc + 16 * k] = yv[i][k];
      __syncthreads();
      proj_store_y(Xs, y, n0, N, dend, D, p.B, d0, tid, &sy);
      __syncthreads();
    }
  }
  sy = block_sum256(sy, red);
  if (tid == 0) p.fpp[(long)g * per_g + rem] = sy;
}

// fixed-order sums of the per-workgroup partials, one block per (g, quantity): block b < G
// sums |Y|^2 of matrix b, block G + b (when ipp is given) |X|^2
__global__ __launch_bounds__(256) void ngd_proj_sums_kernel(const float* __restrict__ fpp, float* __restrict__ fp,
                                                            const float* __restrict__ ipp, float* __restrict__ ip,
                                                            int G, int nk) {
  __shared__ float red[4];
  const bool second = (int)blockIdx.x >= G;
  const int g = second ? blockIdx.x - G : blockIdx.x;
  const float* part = second ? ipp : fpp;
  float s = 0.f;
  for (int k = threadIdx.x; k < nk; k += 256) s += part[(long)g * nk + k];
  s = block_sum256(s, red);
  if (threadIdx.x == 0) (second ? ip : fp)[g] = s;
}

// dst[e] = sum_{k < ns} src[k n + e], k in order; a second (src2, dst2, n2) slab set in the
// same launch (J and H^T H of an update step) follows the first in the index space
// Block = 64 columns x 4 slab lanes: lane r sums slabs r, r+4, ... and the four partials are
// added in a fixed order (deterministic).  The embedding's J / H slabs (~240-480 slabs of
// 40960 floats) left one thread per column on ~160 workgroups latency-bound (135 us).
__global__ __launch_bounds__(256) void ngd_slab_sum_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                                           long n, int ns, const float* __restrict__ src2,
                                                           float* __restrict__ dst2, long n2) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  for (long e0 = (long)blockIdx.x * 64; e0 < n + n2; e0 += (long)gridDim.x * 64) {
    const long e = e0 + cl;
    const bool ok = e < n + n2;
    const bool two = e >= n;
    const float* s_ = two ? src2 : src;
    const long m = two ? n2 : n, i = two ? e - n : e;
    float s = 0.f;
    if (ok) {
      int k = rl;
      for (; k + 12 < ns; k += 16) {  // four independent loads in flight per lane
        const float a = s_[(long)k * m + i], b = s_[(long)(k + 4) * m + i];
        const float c = s_[(long)(k + 8) * m + i], d = s_[(long)(k + 12) * m + i];
        s += a; s += b; s += c; s += d;
      }
      for (; k < ns; k += 4) s += s_[(long)k * m + i];
    }
    red[rl][cl] = s;
    __syncthreads();
    if (rl == 0 && ok) (two ? dst2 : dst)[i] = (red[0][cl] + red[1][cl]) + (red[2][cl] + red[3][cl]);
    __syncthreads();
  }
}

bool ngd_proj_supported(int D, int R) { return D >= 9 && R >= 1 && R <= kPR; }

int ngd_mfma(int on) {
  const int prev = ngd_mfma_on() ? 1 : 0;
  if (on >= 0) g_ngd_mfma = on ? 1 : 0;
  return prev;
}

static void proj_split(int G, long N, int D, int& tiles, int& ds, int& dlen) {
  tiles = (int)((N + kPN - 1) / kPN);
  const int chunks = (D + kPD - 1) / kPD;
  // enough workgroups to cover the chip ~4 deep; at least 2 d chunks per workgroup
  long want = (2048 + (long)G * tiles - 1) / ((long)G * tiles);
  long cap = (chunks + 1) / 2;
  ds = (int)(want < 1 ? 1 : (want > cap ? (cap < 1 ? 1 : cap) : want));
  const int cps = (chunks + ds - 1) / ds;
  dlen = cps * kPD;
  ds = (D + dlen - 1) / dlen;
}

// scratch layout of one ngd_proj call (floats): final H [G][N][R], then (d split) ds slabs
// of partial H, the partial |X|^2 and |Y|^2 slots [G][tiles * ds], and on update steps the
// partial J [tiles][G][R][D] and H^T H [tiles][G][R][R] slabs.  Every slot is written
// exactly once per call, so the buffer needs no zero fill.
struct ProjLayout {
  long h, hslab, ipp, fpp, jp, hhp, total;
};

static ProjLayout proj_layout(int G, long N, int D, int R, int tiles, int ds, bool need_ip, bool need_j,
                              bool need_hh) {
  ProjLayout L{};
  const long hn = (long)G * N * R, nwg = (long)G * tiles * ds;
  long o = 0;
  L.h = o; o += hn;
  L.hslab = o; o += ds > 1 ? ds * hn : 0;
  L.ipp = o; o += need_ip ? nwg : 0;
  L.fpp = o; o += nwg;
  L.jp = o; o += need_j ? (long)tiles * G * R * D : 0;
  L.hhp = o; o += need_hh ? (long)tiles * G * R * R : 0;
  L.total = o;
  return L;
}

long ngd_proj_hbuf_numel(int G, int A, int D, int B, int R, bool need_ip, bool need_j, bool need_hh) {
  int tiles, ds, dlen;
  proj_split(G, (long)A * B, D, tiles, ds, dlen);
  return proj_layout(G, (long)A * B, D, R, tiles, ds, need_ip, need_j, need_hh).total;
}

static int slab_blocks(long n) {
  long nb = (n + 63) / 64;  // (ngd_slab_sum_kernel: 64 columns per workgroup)
  return (int)(nb > 4096 ? 4096 : (nb < 1 ? 1 : nb));
}

void ngd_proj(uint64_t X, uint64_t Y, uint64_t W, uint64_t Hbuf, int G, int A, int D, int B, int R, uint64_t ip,
              uint64_t fp, uint64_t J, uint64_t HH, uint64_t stream) {
  FDT_CHECK(ngd_proj_supported(D, R), "ngd_proj: needs D >= 9 and rank <= 80");
  FDT_CHECK(fp != 0 && Hbuf != 0, "ngd_proj: |Y|^2 output and the scratch buffer are required");
  FDT_CHECK(HH == 0 || J != 0, "ngd_proj: H^T H only on update steps (with J)");
  if (G == 0 || A == 0 || B == 0) return;
  const long N = (long)A * B;
  ProjArgs p{};
  p.X = P<const float>(X);
  p.Y = P<float>(Y);
  p.W = P<const float>(W);
  p.A = A; p.D = D; p.B = B; p.R = R;
  proj_split(G, N, D, p.tiles, p.ds, p.dlen);
  const ProjLayout L = proj_layout(G, N, D, R, p.tiles, p.ds, ip != 0, J != 0, HH != 0);
  float* sc = P<float>(Hbuf);
  // kernel 1 writes partial H into the slabs when d is split (summed into sc + L.h below)
  p.H = p.ds > 1 ? sc + L.hslab : sc + L.h;
  p.ipp = ip ? sc + L.ipp : nullptr;
  p.fpp = sc + L.fpp;
  p.Jp = J ? sc + L.jp : nullptr;
  p.HHp = HH ? sc + L.hhp : nullptr;
  const long grid = (long)G * p.tiles * p.ds;
  FDT_CHECK(grid < (1L << 31), "ngd_proj: grid too large");
  hipStream_t st = as_stream(stream);
  const long hn = (long)G * N * R;
  // float4 path: rows contiguous in d (the last axis) and 16-B aligned rows / matrices
  const bool vec = B == 1 && D % 4 == 0 && X % 16 == 0 && Y % 16 == 0 && W % 16 == 0;
  const bool mf = ngd_mfma_on();
  if (vec) {
    if (mf) ngd_proj_h_kernel<true, true><<<(unsigned)grid, 256, 0, st>>>(p);
    else ngd_proj_h_kernel<true, false><<<(unsigned)grid, 256, 0, st>>>(p);
  } else {
    if (mf) ngd_proj_h_kernel<false, true><<<(unsigned)grid, 256, 0, st>>>(p);
    else ngd_proj_h_kernel<false, false><<<(unsigned)grid, 256, 0, st>>>(p);
  }
  FDT_LAUNCH_CHECK();
  if (p.ds > 1) {
    ngd_slab_sum_kernel<<<slab_blocks(hn), 256, 0, st>>>(sc + L.hslab, sc + L.h, hn, p.ds, nullptr, nullptr, 0);
    FDT_LAUNCH_CHECK();
    p.H = sc + L.h;
  }
#define FDT_PROJ_Y(V_, S_)                                                   \
  if (mf) ngd_proj_y_kernel<V_, S_, true><<<(unsigned)grid, 256, 0, st>>>(p); \
  else ngd_proj_y_kernel<V_, S_, false><<<(unsigned)grid, 256, 0, st>>>(p);
  if (vec) {
    FDT_PROJ_Y(true, false)
  } else if (B > 1) {
    FDT_PROJ_Y(false, true)
  } else {
    FDT_PROJ_Y(false, false)
  }
#undef FDT_PROJ_Y
  FDT_LAUNCH_CHECK();
  const int nwg = p.tiles * p.ds;
  ngd_proj_sums_kernel<<<ip ? 2 * G : G, 256, 0, st>>>(p.fpp, P<float>(fp), p.ipp, P<float>(ip), G, nwg);
  FDT_LAUNCH_CHECK();
  if (J) {  // J (and H^T H) slab sums in one launch
    const long jn = (long)G * R * D, hhn = HH ? (long)G * R * R : 0;
    ngd_slab_sum_kernel<<<slab_blocks(jn + hhn), 256, 0, st>>>(p.Jp, P<float>(J), jn, p.tiles, p.HHp, P<float>(HH),
                                                               hhn);
    FDT_LAUNCH_CHECK();
  }
}

static int ngd_chunks(long per) {
  // ~8 float4 per thread, enough workgroups per matrix to fill the chip (the first version
  // ran 64 scalar elements per thread on a few hundred workgroups: ~10% of HBM bandwidth)
  long c = per / (256 * 4 * 8);
  if (c < 1) c = 1;
  if (c > 4096) c = 4096;
  return (int)c;
}

void ngd_sumsq(uint64_t X, long per, int G, uint64_t out, uint64_t stream) {
  if (G == 0 || per == 0) return;
  FDT_CHECK(X % 16 == 0 && per % 4 == 0, "ngd_sumsq: 16-B aligned slabs");
  const int ch = ngd_chunks(per);
  ngd_sumsq_kernel<<<G * ch, 256, 0, as_stream(stream)>>>(P<const float>(X), per, ch, P<float>(out));
  FDT_LAUNCH_CHECK();
}

void ngd_rescale(uint64_t X, uint64_t Y, long per, int G, uint64_t ip, uint64_t fp, uint64_t stream) {
  if (G == 0 || per == 0) return;
  FDT_CHECK(X % 16 == 0 && Y % 16 == 0 && per % 4 == 0, "ngd_rescale: 16-B aligned slabs");
  const int ch = ngd_chunks(per);
  ngd_rescale_kernel<<<G * ch, 256, 0, as_stream(stream)>>>(P<const float>(X), P<float>(Y), per, ch, P<const float>(ip),
                                                           P<const float>(fp));
  FDT_LAUNCH_CHECK();
}

void ngd_pre_eigh(uint64_t K, uint64_t L, uint64_t d, uint64_t rho, uint64_t Z, uint64_t ise, uint64_t drho, uint64_t zs,
                  uint64_t dsum, int G, int R, float alpha, float eta, float N, float D, uint64_t stream) {
  FDT_CHECK(R >= 1 && R <= kNgdMaxR, "ngd: rank out of range");
  if (G == 0) return;
  ngd_pre_eigh_kernel<<<G, 256, 0, as_stream(stream)>>>(P<const float>(K), P<const float>(L), P<const float>(d),
                                                       P<const float>(rho), P<float>(Z), P<float>(ise), P<float>(drho),
                                                       P<float>(zs), P<float>(dsum), R, alpha, eta, N, D);
  FDT_LAUNCH_CHECK();
}

void ngd_post_eigh(uint64_t c, uint64_t U, uint64_t ise, uint64_t drho, uint64_t zs, uint64_t dsum, uint64_t trXX,
                   uint64_t d, uint64_t rho, uint64_t A, uint64_t wc, int G, int R, float alpha, float eta, float N,
                   float D, uint64_t stream) {
  FDT_CHECK(R >= 1 && R <= kNgdMaxR, "ngd: rank out of range");
  if (G == 0) return;
  ngd_post_eigh_kernel<<<G, 256, 0, as_stream(stream)>>>(P<const float>(c), P<const float>(U), P<const float>(ise),
                                                        P<const float>(drho), P<const float>(zs), P<const float>(dsum),
                                                        P<const float>(trXX), P<float>(d), P<float>(rho), P<float>(A),
                                                        P<float>(wc), R, alpha, eta, N, D);
  FDT_LAUNCH_CHECK();
}

// ---------------------------------------------------------------- rank x rank products
// The R x R products of an update step (reference ngd_optimizer.py:215-218 / :319), which the
// library GEMMs ran as [G,R,D] x [G,D,R] batched launches with 80x256 macro tiles (mostly
// padding at R <= 80):
//   ngd_gram : K = J J^T (upper tiles only, mirrored) and, in the same launch, L = J W^T --
//              32 x 32 output tiles, each over a contiguous d range (split so that the grid
//              fills the chip), partial tiles to a slab summed in split order (no atomics:
//              an NGD step stays bitwise repeatable)
//   ngd_wupdate: W <- A (J + wc W) in place, one workgroup per (g, 64-column block): A and
//              the block of J + wc W in LDS, 20 outputs per thread
constexpr int kGT = 32;

constexpr int kGK = 64;  // d per LDS chunk

template <bool VEC>
__global__ __launch_bounds__(256) void ngd_gram_partial_kernel(const float* __restrict__ J, const float* __restrict__ W,
                                                               float* __restrict__ slab, int R, int D, int nt,
                                                               int tiles_per_g, int S, int dlen) {
  __shared__ float a[kGT][kGK + 1], b[kGT][kGK + 1];
  const int s = blockIdx.x % S;
  const int t = (blockIdx.x / S) % tiles_per_g;
  const int g = blockIdx.x / (S * tiles_per_g);
  // tile t: first the upper-triangle tiles of K (ti <= tj), then the nt x nt tiles of L
  const int nsym = nt * (nt + 1) / 2;
  int ti, tj;
  const float* Bsrc;
  if (t < nsym) {
    int r = t, i = 0;
    while (r >= nt - i) { r -= nt - i; ++i; }
    ti = i; tj = i + r;
    Bsrc = J;
  } else {
    ti = (t - nsym) / nt; tj = (t - nsym) % nt;
    Bsrc = W;
  }
  const long base = (long)g * R * D;
  const int i0 = ti * kGT, j0 = tj * kGT;
  const int d0 = s * dlen, d1 = min(D, d0 + dlen);
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  float acc[2][2] = {{0.f, 0.f}, {0.f, 0.f}};
  // register-staged loads of the NEXT chunk are in flight while the current one is computed
  // (the loop is latency-bound: 256 FMAs per thread per chunk against one global round trip)
  constexpr int NL = kGT * kGK / 256;  // floats per thread per operand (8)
  float ra[NL], rb[NL];
  auto load = [&](int dc) {
    if constexpr (VEC) {
#pragma unroll
      for (int q = 0; q < NL / 4; ++q) {
        const int e = threadIdx.x + q * 256;
        const int r = e / (kGK / 4), c = (e % (kGK / 4)) * 4, d = dc + c;
        float4 va = make_float4(0.f, 0.f, 0.f, 0.f), vb = va;
        if (d < d1) {  // (d1 and D are multiples of 4 here: a float4 never straddles the end)
          if (i0 + r < R) va = *reinterpret_cast<const float4*>(J + base + (long)(i0 + r) * D + d);
          if (j0 + r < R) vb = *reinterpret_cast<const float4*>(Bsrc + base + (long)(j0 + r) * D + d);
        }
        ra[4 * q] = va.x; ra[4 * q + 1] = va.y; ra[4 * q + 2] = va.z; ra[4 * q + 3] = va.w;
        rb[4 * q] = vb.x; rb[4 * q + 1] = vb.y; rb[4 * q + 2] = vb.z; rb[4 * q + 3] = vb.w;
      }
    } else {
#pragma unroll
      for (int q = 0; q < NL; ++q) {
        const int e = threadIdx.x + q * 256;
        const int r = e / kGK, c = e % kGK, d = dc + c;
        ra[q] = (i0 + r < R && d < d1) ? J[base + (long)(i0 + r) * D + d] : 0.f;
        rb[q] = (j0 + r < R && d < d1) ? Bsrc[base + (long)(j0 + r) * D + d] : 0.f;
      }
    }
  };
  auto store = [&]() {
    if constexpr (VEC) {
#pragma unroll
      for (int q = 0; q < NL / 4; ++q) {
        const int e = threadIdx.x + q * 256;
        const int r = e / (kGK / 4), c = (e % (kGK / 4)) * 4;
#pragma unroll
        for (int k = 0; k < 4; ++k) { a[r][c + k] = ra[4 * q + k]; b[r][c + k] = rb[4 * q + k]; }
      }
    } else {
#pragma unroll
      for (int q = 0; q < NL; ++q) {
        const int e = threadIdx.x + q * 256;
        a[e / kGK][e % kGK] = ra[q];
        b[e / kGK][e % kGK] = rb[q];
      }
    }
  };
  if (d0 < d1) load(d0);
  for (int dc = d0; dc < d1; dc += kGK) {
    store();
    __syncthreads();
    if (dc + kGK < d1) load(dc + kGK);
#pragma unroll 16
    for (int c = 0; c < kGK; ++c) {
      const float a0 = a[ty * 2][c], a1 = a[ty * 2 + 1][c], b0 = b[tx * 2][c], b1 = b[tx * 2 + 1][c];
      acc[0][0] = fmaf(a0, b0, acc[0][0]);
      acc[0][1] = fmaf(a0, b1, acc[0][1]);
      acc[1][0] = fmaf(a1, b0, acc[1][0]);
      acc[1][1] = fmaf(a1, b1, acc[1][1]);
    }
    __syncthreads();
  }
  float* o = slab + ((long)(g * tiles_per_g + t) * S + s) * (kGT * kGT);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) o[(ty * 2 + i) * kGT + tx * 2 + j] = acc[i][j];
}

__global__ __launch_bounds__(256) void ngd_gram_sum_kernel(const float* __restrict__ slab, float* __restrict__ K,
                                                           float* __restrict__ L, int R, int nt, int tiles_per_g,
                                                           int S, long total) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= total) return;
  const int w = (int)(e % (kGT * kGT));
  const long gt = e / (kGT * kGT);
  const int t = (int)(gt % tiles_per_g), g = (int)(gt / tiles_per_g);
  const int nsym = nt * (nt + 1) / 2;
  int ti, tj;
  bool sym = t < nsym;
  if (sym) {
    int r = t, i = 0;
    while (r >= nt - i) { r -= nt - i; ++i; }
    ti = i; tj = i + r;
  } else {
    ti = (t - nsym) / nt; tj = (t - nsym) % nt;
  }
  const int i = ti * kGT + w / kGT, j = tj * kGT + w % kGT;
  if (i >= R || j >= R) return;
  const float* src = slab + gt * S * (kGT * kGT) + w;
  float v = 0.f;
  for (int s = 0; s < S; ++s) v += src[(long)s * (kGT * kGT)];  // split order: deterministic
  if (sym) {
    if (ti == tj && j < i) return;  // diagonal tile: the lower half comes from the mirror below
    K[((long)g * R + i) * R + j] = v;
    K[((long)g * R + j) * R + i] = v;
  } else {
    L[((long)g * R + i) * R + j] = v;
  }
}

static void gram_split(int G, int tiles_per_g, int D, int& S, int& dlen) {
  // ~2048 workgroups in all, each reducing >= 128 of d (a multiple of the 64-wide chunk)
  const long wgs = (long)G * tiles_per_g;
  long s = (2048 + wgs - 1) / wgs;
  long smax = (D + 127) / 128;
  if (s > smax) s = smax;
  if (s < 1) s = 1;
  dlen = (int)(((D + s - 1) / s + kGK - 1) / kGK * kGK);
  S = (D + dlen - 1) / dlen;
}

long ngd_gram_slab_numel(int G, int R, int D, bool with_l) {
  const int nt = (R + kGT - 1) / kGT;
  const int tpg = nt * (nt + 1) / 2 + (with_l ? nt * nt : 0);
  int S, dlen;
  gram_split(G, tpg, D, S, dlen);
  return (long)G * tpg * S * kGT * kGT;
}

void ngd_gram(uint64_t J, uint64_t W, uint64_t K, uint64_t L, uint64_t slab, int G, int R, int D, uint64_t stream) {
  FDT_CHECK(R >= 1 && R <= kNgdMaxR && D >= 1, "ngd_gram: shape");
  if (G == 0) return;
  const bool with_l = L != 0;
  FDT_CHECK(!with_l || W != 0, "ngd_gram: L needs W");
  const int nt = (R + kGT - 1) / kGT;
  const int tpg = nt * (nt + 1) / 2 + (with_l ? nt * nt : 0);
  int S, dlen;
  gram_split(G, tpg, D, S, dlen);
  hipStream_t st = as_stream(stream);
  const bool vec = D % 4 == 0 && J % 16 == 0 && (W == 0 || W % 16 == 0);
  (vec ? ngd_gram_partial_kernel<true> : ngd_gram_partial_kernel<false>)<<<G * tpg * S, 256, 0, st>>>(
      P<const float>(J), P<const float>(W), P<float>(slab), R, D, nt, tpg, S, dlen);
  FDT_LAUNCH_CHECK();
  const long total = (long)G * tpg * kGT * kGT;
  ngd_gram_sum_kernel<<<(int)((total + 255) / 256), 256, 0, st>>>(P<const float>(slab), P<float>(K), P<float>(L), R,
                                                                  nt, tpg, S, total);
  FDT_LAUNCH_CHECK();
}

constexpr int kWuCols = 64;

__global__ __launch_bounds__(256) void ngd_wupdate_kernel(const float* __restrict__ A, const float* __restrict__ J,
                                                          const float* __restrict__ wc, float* __restrict__ W, int R,
                                                          int D, int nblk) {
  extern __shared__ float lds[];
  constexpr int LB = kWuCols + 4;         // B row stride (16-B aligned rows)
  float* As = lds;                        // [R][R + 1]
  float* Bs = lds + R * (R + 1);          // [R][LB]  (R*(R+1) is even; Bs 8-B aligned, see the 16-B fix below)
  Bs = reinterpret_cast<float*>((reinterpret_cast<uintptr_t>(Bs) + 15) & ~(uintptr_t)15);
  const int g = blockIdx.x / nblk, blk = blockIdx.x % nblk;
  const int c0 = blk * kWuCols;
  const float* Ag = A + (long)g * R * R;
  const long base = (long)g * R * D;
  // operand staging with several loads in flight per thread (a load-then-store loop waits out
  // one global round trip per element: ~27 us per launch at R = 80, ~20x the arithmetic)
  constexpr int IF = 4;
  if ((R & 3) == 0) {
    const float4* A4 = reinterpret_cast<const float4*>(Ag);
    const int n4 = R * R / 4;
    for (int e0 = threadIdx.x; e0 < n4; e0 += 256 * IF) {
      float4 v[IF];
#pragma unroll
      for (int q = 0; q < IF; ++q) {
        const int i = e0 + q * 256;
        v[q] = i < n4 ? A4[i] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int q = 0; q < IF; ++q) {
        const int i = e0 + q * 256;
        if (i < n4) {
          const float vv[4] = {v[q].x, v[q].y, v[q].z, v[q].w};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int e = 4 * i + k;
            As[(e / R) * (R + 1) + e % R] = vv[k];
          }
        }
      }
    }
  } else {
    for (int e = threadIdx.x; e < R * R; e += 256) As[(e / R) * (R + 1) + e % R] = Ag[e];
  }
  const bool vec = (D & 3) == 0 && c0 + kWuCols <= D;
  if (vec) {
    constexpr int C4 = kWuCols / 4;
    const int n4 = R * C4;
    for (int e0 = threadIdx.x; e0 < n4; e0 += 256 * IF) {
      float4 vw[IF], vj[IF];
      float sc[IF];
#pragma unroll
      for (int q = 0; q < IF; ++q) {
        const int i = e0 + q * 256;
        const int r = i / C4, c = (i % C4) * 4;
        if (i < n4) {
          vw[q] = *reinterpret_cast<const float4*>(W + base + (long)r * D + c0 + c);
          vj[q] = *reinterpret_cast<const float4*>(J + base + (long)r * D + c0 + c);
          sc[q] = wc[(long)g * R + r];
        }
      }
#pragma unroll
      for (int q = 0; q < IF; ++q) {
        const int i = e0 + q * 256;
        if (i < n4) {
          const int r = i / C4, c = (i % C4) * 4;
          float4 o;
          o.x = fmaf(sc[q], vw[q].x, vj[q].x);
          o.y = fmaf(sc[q], vw[q].y, vj[q].y);
          o.z = fmaf(sc[q], vw[q].z, vj[q].z);
          o.w = fmaf(sc[q], vw[q].w, vj[q].w);
          *reinterpret_cast<float4*>(Bs + r * LB + c) = o;
        }
      }
    }
  } else {
    for (int e = threadIdx.x; e < R * kWuCols; e += 256) {
      const int r = e / kWuCols, c = e % kWuCols, d = c0 + c;
      float v = 0.f;
      if (d < D) v = fmaf(wc[(long)g * R + r], W[base + (long)r * D + d], J[base + (long)r * D + d]);
      Bs[r * LB + c] = v;
    }
  }
  __syncthreads();  // (every W value of this block is in LDS before any is overwritten)
  // thread: 4 consecutive columns x rows rg, rg + 16, ... (A reads broadcast over the 16
  // column groups of a row group, one 16-B B read per k)
  const int cg = threadIdx.x & 15, rg = threadIdx.x >> 4;
  constexpr int MR = (kNgdMaxR + 15) / 16;
  float acc[MR][4];
#pragma unroll
  for (int q = 0; q < MR; ++q)
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[q][k] = 0.f;
  for (int k = 0; k < R; ++k) {
    const float4 bk = *reinterpret_cast<const float4*>(Bs + k * LB + cg * 4);
#pragma unroll
    for (int q = 0; q < MR; ++q) {
      const int r = rg + 16 * q;
      if (r < R) {
        const float av = As[r * (R + 1) + k];
        acc[q][0] = fmaf(av, bk.x, acc[q][0]);
        acc[q][1] = fmaf(av, bk.y, acc[q][1]);
        acc[q][2] = fmaf(av, bk.z, acc[q][2]);
        acc[q][3] = fmaf(av, bk.w, acc[q][3]);
      }
    }
  }
#pragma unroll
  for (int q = 0; q < MR; ++q) {
    const int r = rg + 16 * q;
    if (r < R) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int d = c0 + cg * 4 + k;
        if (d < D) W[base + (long)r * D + d] = acc[q][k];
      }
    }
  }
}

void ngd_wupdate(uint64_t A, uint64_t J, uint64_t wc, uint64_t W, int G, int R, int D, uint64_t stream) {
  FDT_CHECK(R >= 1 && R <= kNgdMaxR && D >= 1, "ngd_wupdate: shape");
  if (G == 0) return;
  const int nblk = (D + kWuCols - 1) / kWuCols;
  const size_t lds = ((size_t)R * (R + 1) + (size_t)R * (kWuCols + 4) + 4) * sizeof(float);
  ngd_wupdate_kernel<<<G * nblk, 256, lds, as_stream(stream)>>>(P<const float>(A), P<const float>(J), P<const float>(wc),
                                                              P<float>(W), R, D, nblk);
  FDT_LAUNCH_CHECK();
}

}  // namespace fdt
