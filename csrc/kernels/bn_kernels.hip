// Per-channel normalisation kernels for the NHWC ResNet engine (ops/resnet_engine.py).
//
// A conv output y[M][C] (M = N*H*W, NHWC, bf16) is never normalised in place: the
// engine keeps it raw and carries a per-channel affine (s[c], t[c]) that the CONSUMER
// applies while loading (a = act(y*s + t)).  These kernels provide
//   * batch statistics: per-block partial (sum, sumsq) slabs + an fp64 finalize that
//     produces (s, t) for FusedConvBN numerics (unbiased var, 1/(sqrt(var)+eps);
//     reference resnet.py:75-100) or BatchNorm2d numerics (biased var, affine, running
//     stats update with the unbiased var);
//   * the backward of that map: the consumer's act backward + per-channel reductions
//     (sum g_pre*x, sum g_pre), the producer's coefficient kernel turning (g_s, g_t)
//     into an affine correction g_y += alpha + beta*y, and its apply pass;
//   * the residual join  out = act(y_a*s_a + t_a + [y_b*s_b + t_b | x])  fwd/bwd.
// Partial slabs (not float atomics) keep the reductions deterministic and avoid
// contention on the C channel addresses (MI355X_MICROARCH: one-row contention is 14x
// slower).  All kernels stream 16 B per lane.
#include "common.h"
#include "bn_math.h"

namespace fdt {

constexpr int kBlk = 256;
inline int wt_flag() { return conv_write_through() ? 1 : 0; }  // write-through streaming outputs (common.h st8)

// Channel-group geometry for [M][C] with 8 channels per thread.
struct ChanGeom {
  int G;    // channel groups (C / 8)
  int TPR;  // threads per row
  int RPP;  // rows per pass (kBlk / TPR)
  int gy;   // grid.y (channel-group tiles)
};
inline ChanGeom chan_geom(int C) {
  FDT_CHECK(C % 8 == 0, "channel count must be a multiple of 8");
  ChanGeom g;
  g.G = C / 8;
  g.TPR = g.G < kBlk ? g.G : kBlk;
  FDT_CHECK((g.G <= kBlk && kBlk % g.G == 0) || (g.G % kBlk == 0),
            "C/8 must divide 256 or be a multiple of 256");
  g.RPP = kBlk / g.TPR;
  g.gy = g.G / g.TPR;
  return g;
}

// 8 consecutive per-channel fp32 parameters (c multiple of 8 -> two 16-B loads)
__device__ __forceinline__ void load8f(const float* __restrict__ p, int c, float* v) {
  float4 a = *reinterpret_cast<const float4*>(p + c), b = *reinterpret_cast<const float4*>(p + c + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// ------------------------------------------------------------------ act(x*s+t)
template <typename T, typename TO>
__global__ __launch_bounds__(kBlk) void act_affine_fwd_kernel(const T* __restrict__ x, const float* __restrict__ s,
                                                              const float* __restrict__ t, TO* __restrict__ out,
                                                              long nvec, int C, int act, float alpha, int wt) {
  long stride = (long)gridDim.x * blockDim.x;
  for (long v = (long)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    long e = v * 8;
    int c = (int)(e % C);
    float a[8];
    Vec8<T>::load(x + e, a);
    if (s != nullptr) {
      float4 s0 = *reinterpret_cast<const float4*>(s + c), s1 = *reinterpret_cast<const float4*>(s + c + 4);
      float4 t0 = *reinterpret_cast<const float4*>(t + c), t1 = *reinterpret_cast<const float4*>(t + c + 4);
      float sv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
      float tv[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = fmaf(a[i], sv[i], tv[i]);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = act_fwd(a[i], act, alpha);
    st8(out, e, a, wt);
  }
}

// Streaming form of the BN-backward fold (kEwU vectors per thread per trip, every load of the
// trip issued before the first store; the grid stride is a multiple of the channel-vector count
// G -- host: ew_grid_u -- so a thread's channels and per-channel parameters are fixed, loaded
// once): 5.0 -> 5.3-5.4 TB/s on the 268-537 MB batch-1024 tensors (scripts/ew_probe.py,
// profiles/r5/ew_probe_bs1024.txt).  The same form of the join and normalise passes measured
// 3-8 % SLOWER than their grid-stride loops, which already run at the device-copy rate of
// those tensors (4.7-5.0 TB/s): those keep the one/two-vector loops.
constexpr int kEwU = 4;
inline int& ew_unroll_flag() {
  static int f = 1;
  return f;
}

// ------------------------------------------------------------------ stats partials
// part[blk][q][C], q = 0: sum y, q = 1: sum y^2
template <typename T>
__global__ __launch_bounds__(kBlk) void channel_stats_partial_kernel(const T* __restrict__ y, float* __restrict__ part,
                                                                     long M, int C, int TPR, int RPP, long rows_per_blk) {
  __shared__ float sm[kBlk * 16];
  const int tid = threadIdx.x;
  const int gi = tid % TPR, rr = tid / TPR;
  const int c0 = (blockIdx.y * TPR + gi) * 8;
  const long r_begin = (long)blockIdx.x * rows_per_blk;
  long r_end = r_begin + rows_per_blk;
  if (r_end > M) r_end = M;
  float s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (long r = r_begin + rr; r < r_end; r += RPP) {
    float v[8];
    Vec8<T>::load(y + r * C + c0, v);
#pragma unroll
    for (int i = 0; i < 8; ++i) { s1[i] += v[i]; s2[i] = fmaf(v[i], v[i], s2[i]); }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) { sm[tid * 16 + i] = s1[i]; sm[tid * 16 + 8 + i] = s2[i]; }
  __syncthreads();
  // reduce over rr for each (gi, i): thread j handles j < TPR*16
  for (int j = tid; j < TPR * 16; j += kBlk) {
    int g = j / 16, i = j % 16;
    float acc = 0.f;
    for (int q = 0; q < RPP; ++q) acc += sm[(q * TPR + g) * 16 + i];
    int c = (blockIdx.y * TPR + g) * 8 + (i & 7);
    part[((long)blockIdx.x * 2 + (i >> 3)) * C + c] = acc;
  }
}

// Sum nq partial rows over nb blocks in fp64: acc[q] = sum_{b = w, w+nw, ...} part[b][q][c]
// (4-way unrolled so the independent loads are in flight together)
template <int NQ>
__device__ __forceinline__ void zero_partials(float* part, int nb, int C, int c, int w, int nw) {
  for (int b = w; b < nb; b += nw) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) part[((long)b * NQ + q) * C + c] = 0.f;
  }
}

template <int NQ>
__device__ __forceinline__ void sum_partials_f64(const float* __restrict__ part, int nb, int C, int c, double* acc,
                                                 int w, int nw) {
  // 4 rows per trip (4*NQ independent loads in flight): large-M producers spread their
  // workgroups over hundreds of slot rows, and this loop is latency-bound
  double a0[NQ], a1[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) { a0[q] = 0.0; a1[q] = 0.0; }
  int b = w;
  for (; b + 3 * nw < nb; b += 4 * nw) {
    float v[4][NQ];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int q = 0; q < NQ; ++q) v[u][q] = part[((long)(b + u * nw) * NQ + q) * C + c];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      a0[q] += (double)v[0][q] + (double)v[2][q];
      a1[q] += (double)v[1][q] + (double)v[3][q];
    }
  }
  for (; b < nb; b += nw) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) a0[q] += (double)part[((long)b * NQ + q) * C + c];
  }
#pragma unroll
  for (int q = 0; q < NQ; ++q) acc[q] = a0[q] + a1[q];
}

constexpr int kRedWaves = 16;  // finalize / reduce kernels: 1024 threads per 64-channel tile

// Modes and outputs: bn_math.h.  zero_after: re-zero the (slot) rows after reading them, so
// the next producer can accumulate into the same workspace without a memset launch.
__global__ __launch_bounds__(64 * kRedWaves) void stats_finalize_kernel(float* __restrict__ part, int nb, int C,
                                                                        int zero_after, FinArgs f) {
  __shared__ double sm[kRedWaves][64][2];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  double acc[2] = {0.0, 0.0};
  if (c < C && f.mode != 2) sum_partials_f64<2>(part, nb, C, c, acc, w, kRedWaves);
  if (c < C && zero_after) zero_partials<2>(part, nb, C, c, w, kRedWaves);
  sm[w][lane][0] = acc[0];
  sm[w][lane][1] = acc[1];
  __syncthreads();
  if (w != 0 || c >= C) return;
  double S = 0.0, Q = 0.0;
#pragma unroll
  for (int k = 0; k < kRedWaves; ++k) { S += sm[k][lane][0]; Q += sm[k][lane][1]; }
  bn_finalize_channel(f, c, S, Q);
}

// ------------------------------------------------------------------ consumer backward
// Input transform a = act(x*s + t).  Given g = dL/da:
//   g_pre = g * act'(x*s+t);  gx = g_pre * s;  part = [sum g_pre*x, sum g_pre]
template <typename T>
__global__ __launch_bounds__(kBlk) void act_bwd_reduce_kernel(const T* __restrict__ g, const T* __restrict__ x,
                                                              const float* __restrict__ s, const float* __restrict__ t,
                                                              T* __restrict__ gx, float* __restrict__ part,
                                                              unsigned slot_mask, long M, int C, int TPR, int RPP,
                                                              long rows_per_blk, int act, float alpha, int wt) {
  __shared__ float sm[kBlk * 16];
  const int tid = threadIdx.x;
  const int gi = tid % TPR, rr = tid / TPR;
  const int c0 = (blockIdx.y * TPR + gi) * 8;
  float sv[8], tv[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { sv[i] = s[c0 + i]; tv[i] = t[c0 + i]; }
  const long r_begin = (long)blockIdx.x * rows_per_blk;
  long r_end = r_begin + rows_per_blk;
  if (r_end > M) r_end = M;
  float a1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, a0[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (long r = r_begin + rr; r < r_end; r += RPP) {
    float gv[8], xv[8], o[8];
    Vec8<T>::load(g + r * C + c0, gv);
    Vec8<T>::load(x + r * C + c0, xv);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float z = fmaf(xv[i], sv[i], tv[i]);
      float gp = gv[i] * act_grad(z, act, alpha);
      o[i] = gp * sv[i];
      a1[i] = fmaf(gp, xv[i], a1[i]);
      a0[i] += gp;
    }
    st8(gx, r * C + c0, o, wt);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) { sm[tid * 16 + i] = a1[i]; sm[tid * 16 + 8 + i] = a0[i]; }
  __syncthreads();
  for (int j = tid; j < TPR * 16; j += kBlk) {
    int gg = j / 16, i = j % 16;
    float acc = 0.f;
    for (int q = 0; q < RPP; ++q) acc += sm[(q * TPR + gg) * 16 + i];
    int c = (blockIdx.y * TPR + gg) * 8 + (i & 7);
    atomicAdd(&part[((long)(blockIdx.x & slot_mask) * 2 + (i >> 3)) * C + c], acc);
  }
}

// generic fp64 reduction of partial slabs: out[q][c] = sum_b part[b][q][c]
template <int NQ>
__global__ __launch_bounds__(64 * kRedWaves) void reduce_partials_kernel(float* __restrict__ part, int nb, int C,
                                                                         float* __restrict__ out, int zero_after) {
  __shared__ double sm[kRedWaves][64][NQ];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  double acc[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) acc[q] = 0.0;
  if (c < C) sum_partials_f64<NQ>(part, nb, C, c, acc, w, kRedWaves);
  if (c < C && zero_after) zero_partials<NQ>(part, nb, C, c, w, kRedWaves);
#pragma unroll
  for (int q = 0; q < NQ; ++q) sm[w][lane][q] = acc[q];
  __syncthreads();
  if (w != 0 || c >= C) return;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    double t = 0.0;
#pragma unroll
    for (int k = 0; k < kRedWaves; ++k) t += sm[k][lane][q];
    out[(long)q * C + c] = (float)t;
  }
}

// ------------------------------------------------------------------ slab compaction
// part [nb][W] -> out [ceil(nb/R)][W]: out[k][w] = sum_{r in chunk k} part[r][w] (fp32,
// fixed order).  The conv epilogues emit one slab row per workgroup (thousands of rows
// at batch 1024); compacting with a wide grid first keeps the fp64 finalize short and
// the whole reduction at HBM speed instead of a handful of workgroups.
__global__ __launch_bounds__(256) void partials_compact_kernel(const float* __restrict__ part, int nb, int W,
                                                               int R, float* __restrict__ out) {
  const int w = blockIdx.x * 256 + threadIdx.x;
  const int k = blockIdx.y;
  if (w >= W) return;
  const int r0 = k * R;
  int r1 = r0 + R;
  if (r1 > nb) r1 = nb;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int r = r0;
  for (; r + 3 < r1; r += 4) {
    a0 += part[(long)r * W + w];
    a1 += part[(long)(r + 1) * W + w];
    a2 += part[(long)(r + 2) * W + w];
    a3 += part[(long)(r + 3) * W + w];
  }
  for (; r < r1; ++r) a0 += part[(long)r * W + w];
  out[(long)k * W + w] = (a0 + a1) + (a2 + a3);
}

// ------------------------------------------------------------------ producer backward
// (g_s, g_t) -> affine correction of dL/dy:  g_y += alpha + beta * y
// mode 0 (FusedConvBN): s = 1/(sd+eps), t = -mean*s
//    beta = -(g_s - mean g_t) s^2 / ((N-1) sd),   alpha = -beta*mean - g_t s / N
// mode 1 (BatchNorm2d): s = gamma*inv, t = b - mean*s, inv = (var_b+eps)^-1/2
//    beta = -(g_s - mean g_t) gamma inv^3 / N,    alpha = -beta*mean - g_t s / N
//    g_gamma = (g_s - mean g_t) inv,  g_beta = g_t
// mode 2 (BatchNorm2d eval, running stats): beta = alpha = 0, g_gamma/g_beta as above
__global__ void stats_bwd_coef_kernel(const float* __restrict__ gs, const float* __restrict__ gt, int C, CoefArgs a) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  bwd_coef_one(a, c, gs ? gs[c] : 0.0, gt ? gt[c] : 0.0);
}

// Slots [kStatSlots][NQ][C] -> fp64 sums -> BN-backward coefficients, in one launch:
// unit A from (q0 = g_s, q1 = g_t); with NQ = 3 also unit B (the block's shortcut branch,
// sharing g_t) from (q2, q1).  Re-zeroes the slots.
template <int NQ>
__global__ __launch_bounds__(64 * kRedWaves) void stats_bwd_finalize_kernel(float* __restrict__ part, int nb, int C,
                                                                            CoefArgs A, CoefArgs B) {
  __shared__ double sm[kRedWaves][64][NQ];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  double acc[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) acc[q] = 0.0;
  if (c < C) {
    sum_partials_f64<NQ>(part, nb, C, c, acc, w, kRedWaves);
    zero_partials<NQ>(part, nb, C, c, w, kRedWaves);
  }
#pragma unroll
  for (int q = 0; q < NQ; ++q) sm[w][lane][q] = acc[q];
  __syncthreads();
  if (w != 0 || c >= C) return;
  double t[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    t[q] = 0.0;
#pragma unroll
    for (int k = 0; k < kRedWaves; ++k) t[q] += sm[k][lane][q];
  }
  bwd_coef_one(A, c, t[0], t[1]);
  if constexpr (NQ == 3) {
    if (B.alpha) bwd_coef_one(B, c, t[2], t[1]);
  }
}

// out = g_y + alpha[c] + beta[c] * y   (g_y may alias out)
template <typename T>
__global__ __launch_bounds__(kBlk) void affine_fold_kernel(const T* __restrict__ gy, const T* __restrict__ y,
                                                           const float* __restrict__ alpha, const float* __restrict__ beta,
                                                           const float* __restrict__ gs, T* __restrict__ out, long nvec,
                                                           int G, int wt) {
  // out = gy*gs + alpha + beta*y  (gs nullptr: 1; gy nullptr: 0)
  long stride = (long)gridDim.x * blockDim.x;
  for (long v = (long)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    long e = v * 8;
    int c = (int)((unsigned long)v % (unsigned)G) * 8;
    float gv[8], yv[8];
    if (gy) Vec8<T>::load(gy + e, gv);
    else {
#pragma unroll
      for (int i = 0; i < 8; ++i) gv[i] = 0.f;
    }
    Vec8<T>::load(y + e, yv);
    float av[8], bv[8], sv[8];
    load8f(alpha, c, av);
    load8f(beta, c, bv);
    if (gs) load8f(gs, c, sv);
    else {
#pragma unroll
      for (int i = 0; i < 8; ++i) sv[i] = 1.f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) gv[i] = fmaf(gv[i], sv[i], fmaf(bv[i], yv[i], av[i]));
    st8(out, e, gv, wt);
  }
}

template <typename T>
__global__ __launch_bounds__(kBlk) void affine_fold_u_kernel(const T* __restrict__ gy, const T* __restrict__ y,
                                                             const float* __restrict__ alpha,
                                                             const float* __restrict__ beta,
                                                             const float* __restrict__ gs, T* __restrict__ out,
                                                             long nvec, int G, int wt) {
  const long stride = (long)gridDim.x * blockDim.x;
  long v = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int c = (int)((unsigned long)v % (unsigned)G) * 8;
  float av[8], bv[8], sv[8];
  load8f(alpha, c, av);
  load8f(beta, c, bv);
  if (gs) load8f(gs, c, sv);
  else {
#pragma unroll
    for (int i = 0; i < 8; ++i) sv[i] = 1.f;
  }
  for (; v + (kEwU - 1) * stride < nvec; v += kEwU * stride) {
    float gv[kEwU][8], yv[kEwU][8];
#pragma unroll
    for (int u = 0; u < kEwU; ++u) {
      const long e = (v + u * stride) * 8;
      if (gy) Vec8<T>::load(gy + e, gv[u]);
      Vec8<T>::load(y + e, yv[u]);
    }
#pragma unroll
    for (int u = 0; u < kEwU; ++u) {
#pragma unroll
      for (int i = 0; i < 8; ++i) gv[u][i] = fmaf(gy ? gv[u][i] : 0.f, sv[i], fmaf(bv[i], yv[u][i], av[i]));
      st8(out, (v + u * stride) * 8, gv[u], wt);
    }
  }
  for (; v < nvec; v += stride) {
    const long e = v * 8;
    float gv[8], yv[8];
    if (gy) Vec8<T>::load(gy + e, gv);
    Vec8<T>::load(y + e, yv);
#pragma unroll
    for (int i = 0; i < 8; ++i) gv[i] = fmaf(gy ? gv[i] : 0.f, sv[i], fmaf(bv[i], yv[i], av[i]));
    st8(out, e, gv, wt);
  }
}

// ------------------------------------------------------------------ residual join
// out = act(ya*sa + ta + (yb ? yb*sb + tb : xid)).  mask (optional, ReLU joins): one byte per
// 8-element vector, bit i = out[8v+i] > 0 -- the backward reads 1/16 of the bytes of `out`.
// Two vectors per thread per iteration (more loads in flight); channel offset by 32-bit
// modulo on the vector index (no 64-bit division).
template <typename T>
__device__ __forceinline__ void residual_fwd_vec(const T* __restrict__ ya, const float* __restrict__ sa,
                                                 const float* __restrict__ ta, const T* __restrict__ yb,
                                                 const float* __restrict__ sb, const float* __restrict__ tb,
                                                 const T* __restrict__ xid, T* __restrict__ out,
                                                 uint8_t* __restrict__ mask, long v, int G, int act, float alpha,
                                                 int wt) {
  const long e = v * 8;
  const int c = (int)((unsigned long)v % (unsigned)G) * 8;
  float a[8], b[8], s8[8], t8[8];
  Vec8<T>::load(ya + e, a);
  if (yb) {
    Vec8<T>::load(yb + e, b);
    load8f(sb, c, s8);
    load8f(tb, c, t8);
#pragma unroll
    for (int i = 0; i < 8; ++i) b[i] = fmaf(b[i], s8[i], t8[i]);
  } else {
    Vec8<T>::load(xid + e, b);
  }
  load8f(sa, c, s8);
  load8f(ta, c, t8);
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = act_fwd(fmaf(a[i], s8[i], t8[i]) + b[i], act, alpha);
    m |= (a[i] > 0.f ? 1u : 0u) << i;
  }
  st8(out, e, a, wt);
  if (mask) mask[v] = (uint8_t)m;
}

// one 8-channel vector with the branch affines already in registers
template <typename T>
__device__ __forceinline__ void residual_fwd_vec_p(const T* __restrict__ ya, const float (&s8)[8], const float (&t8)[8],
                                                   const T* __restrict__ yb, const float (&sb8)[8],
                                                   const float (&tb8)[8], const T* __restrict__ xid,
                                                   T* __restrict__ out, uint8_t* __restrict__ mask, long v, int act,
                                                   float alpha, int wt) {
  const long e = v * 8;
  float a[8], b[8];
  Vec8<T>::load(ya + e, a);
  if (yb) {
    Vec8<T>::load(yb + e, b);
#pragma unroll
    for (int i = 0; i < 8; ++i) b[i] = fmaf(b[i], sb8[i], tb8[i]);
  } else {
    Vec8<T>::load(xid + e, b);
  }
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = act_fwd(fmaf(a[i], s8[i], t8[i]) + b[i], act, alpha);
    m |= (a[i] > 0.f ? 1u : 0u) << i;
  }
  st8(out, e, a, wt);
  if (mask) mask[v] = (uint8_t)m;
}

// HOIST: the grid stride is a multiple of the channel-vector count G, so every vector a
// thread visits has the same channels -- the four affine vectors are loaded once instead of
// per vector (8 float4 cache loads per 16-B data vector otherwise)
template <typename T, bool HOIST>
__global__ __launch_bounds__(kBlk) void residual_act_fwd_kernel(const T* __restrict__ ya, const float* __restrict__ sa,
                                                                const float* __restrict__ ta, const T* __restrict__ yb,
                                                                const float* __restrict__ sb, const float* __restrict__ tb,
                                                                const T* __restrict__ xid, T* __restrict__ out,
                                                                uint8_t* __restrict__ mask, long nvec, int G, int act,
                                                                float alpha, int wt) {
  const long stride = (long)gridDim.x * blockDim.x;
  long v = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (HOIST) {
    const int c = (int)((unsigned long)v % (unsigned)G) * 8;
    float s8[8], t8[8], sb8[8], tb8[8];
    load8f(sa, c, s8);
    load8f(ta, c, t8);
    if (yb) {
      load8f(sb, c, sb8);
      load8f(tb, c, tb8);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) { sb8[i] = 1.f; tb8[i] = 0.f; }
    }
    for (; v + stride < nvec; v += 2 * stride) {
      residual_fwd_vec_p(ya, s8, t8, yb, sb8, tb8, xid, out, mask, v, act, alpha, wt);
      residual_fwd_vec_p(ya, s8, t8, yb, sb8, tb8, xid, out, mask, v + stride, act, alpha, wt);
    }
    if (v < nvec) residual_fwd_vec_p(ya, s8, t8, yb, sb8, tb8, xid, out, mask, v, act, alpha, wt);
    return;
  }
  for (; v + stride < nvec; v += 2 * stride) {
    residual_fwd_vec(ya, sa, ta, yb, sb, tb, xid, out, mask, v, G, act, alpha, wt);
    residual_fwd_vec(ya, sa, ta, yb, sb, tb, xid, out, mask, v + stride, G, act, alpha, wt);
  }
  if (v < nvec) residual_fwd_vec(ya, sa, ta, yb, sb, tb, xid, out, mask, v, G, act, alpha, wt);
}

// act'(z) from the activation OUTPUT o (ReLU: o>0; CELU: o>0 ? 1 : o/alpha + 1)
__device__ __forceinline__ float act_grad_from_out(float o, int act, float alpha) {
  if (act == kActRelu) return o > 0.f ? 1.f : 0.f;
  if (act == kActCelu) return o > 0.f ? 1.f : o / alpha + 1.f;
  return 1.f;
}

// g_pre = g * act'(out) -- the ONE gradient both branches consume (the consumers scale it
// by their own s through the fold prologue's gs):
// part[blk][3][C] = [sum g_pre*ya, sum g_pre, sum g_pre*yb].  act' comes from the forward's
// bit mask when given (ReLU), else from `out`.
template <typename T>
__global__ __launch_bounds__(kBlk) void residual_act_bwd_kernel(const T* __restrict__ g, const T* __restrict__ out,
                                                                const uint8_t* __restrict__ mask,
                                                                const T* __restrict__ ya, const T* __restrict__ yb,
                                                                T* __restrict__ gpre, float* __restrict__ part,
                                                                unsigned slot_mask, long M, int C, int TPR, int RPP,
                                                                long rows_per_blk, int act, float alpha, int ghw,
                                                                int wt, const float* __restrict__ zsa,
                                                                const float* __restrict__ zta,
                                                                const float* __restrict__ zsb,
                                                                const float* __restrict__ ztb,
                                                                const T* __restrict__ xid) {
  __shared__ float sm[kBlk * 24];
  const int tid = threadIdx.x;
  const int gi = tid % TPR, rr = tid / TPR;
  const int c0 = (blockIdx.y * TPR + gi) * 8;
  // z mode (zsa set; CELU joins): act'(z) = exp(z/alpha) from the fp32 pre-activation, recomputed
  // exactly as the forward join formed it, z = ya*sa + ta + (yb ? yb*sb + tb : xid).  The CELU
  // output o is no substitute below z ~ -0.3: 1 + o/alpha from a bf16 o carries an absolute error
  // of ~2^-11/alpha ~ 6.5e-3 against a true derivative of < 0.02, and o(z -> -inf) rounds to
  // -0.07520 < -alpha, a sign-flipped derivative for every deeply negative z.
  const bool zm = zsa != nullptr && !mask;
  float sa8[8], ta8[8], sb8[8], tb8[8];
  if (zm) {
    load8f(zsa, c0, sa8);
    load8f(zta, c0, ta8);
    if (yb) {
      load8f(zsb, c0, sb8);
      load8f(ztb, c0, tb8);
    }
  }
  const T* osrc = zm ? (yb ? nullptr : xid) : out;  // the 4th streamed operand: out | xid | none
  const long r_begin = (long)blockIdx.x * rows_per_blk;
  long r_end = r_begin + rows_per_blk;
  if (r_end > M) r_end = M;
  float p0[8] = {0, 0, 0, 0, 0, 0, 0, 0}, p1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, p2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  // Two rows per iteration: every load of both rows is issued before the first use, so each
  // thread keeps 6-8 16-B loads in flight (one row per trip left the kernel at ~3 TB/s on the
  // small per-GPU batches where each thread only walks ~16 rows).
  auto row = [&](long e, const float* gv, const float* av, const float* bv, const float* ov, uint32_t m) {
    float gp8[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float gp;
      if (mask) {
        gp = (m >> i) & 1u ? gv[i] : 0.f;
      } else if (zm) {
        const float z = fmaf(av[i], sa8[i], ta8[i]) + (yb ? fmaf(bv[i], sb8[i], tb8[i]) : ov[i]);
        gp = gv[i] * act_grad(z, act, alpha);
      } else {
        gp = gv[i] * act_grad_from_out(ov[i], act, alpha);
      }
      gp8[i] = gp;
      p0[i] = fmaf(gp, av[i], p0[i]);
      p1[i] += gp;
      if (yb) p2[i] = fmaf(gp, bv[i], p2[i]);
    }
    st8(gpre, e, gp8, wt);
  };
  // ghw > 0: g is [M/ghw, C] and broadcast over each group of ghw rows (the classifier
  // head's pooled gradient, already divided by ghw: see head.hip)
  auto gofs = [&](long rw, long e) { return ghw > 0 ? (rw / ghw) * C + c0 : e; };
  long r = r_begin + rr;
  for (; r + RPP < r_end; r += 2 * RPP) {
    const long e0 = r * C + c0, e1 = e0 + (long)RPP * C;
    float g0[8], a0[8], b0[8], o0[8], g1[8], a1[8], b1[8], o1[8];
    uint32_t m0 = 0, m1 = 0;
    Vec8<T>::load(g + gofs(r, e0), g0);
    Vec8<T>::load(g + gofs(r + RPP, e1), g1);
    Vec8<T>::load(ya + e0, a0);
    Vec8<T>::load(ya + e1, a1);
    if (yb) { Vec8<T>::load(yb + e0, b0); Vec8<T>::load(yb + e1, b1); }
    if (mask) { m0 = mask[e0 >> 3]; m1 = mask[e1 >> 3]; }
    else if (osrc) { Vec8<T>::load(osrc + e0, o0); Vec8<T>::load(osrc + e1, o1); }
    row(e0, g0, a0, b0, o0, m0);
    row(e1, g1, a1, b1, o1, m1);
  }
  if (r < r_end) {
    const long e = r * C + c0;
    float gv[8], av[8], bv[8], ov[8];
    uint32_t m = 0;
    Vec8<T>::load(g + gofs(r, e), gv);
    Vec8<T>::load(ya + e, av);
    if (yb) Vec8<T>::load(yb + e, bv);
    if (mask) m = mask[e >> 3];
    else if (osrc) Vec8<T>::load(osrc + e, ov);
    row(e, gv, av, bv, ov, m);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) { sm[tid * 24 + i] = p0[i]; sm[tid * 24 + 8 + i] = p1[i]; sm[tid * 24 + 16 + i] = p2[i]; }
  __syncthreads();
  for (int j = tid; j < TPR * 24; j += kBlk) {
    int gg = j / 24, i = j % 24;
    float acc = 0.f;
    for (int q = 0; q < RPP; ++q) acc += sm[(q * TPR + gg) * 24 + i];
    int c = (blockIdx.y * TPR + gg) * 8 + (i & 7);
    atomicAdd(&part[((long)(blockIdx.x & slot_mask) * 3 + (i >> 3)) * C + c], acc);
  }
}

// ------------------------------------------------------------------ lazy-statistics consumers
// The finalize of the producer's batch statistics moves INTO its elementwise consumer: every
// workgroup finalises all C channels from the slot rows into LDS (workgroup 0 also writes the
// unit's s / t / saved mean / sd, bn_math.h LazyStats), then streams.  One launch instead of
// finalize + pass.  The first two vectors of each thread are loaded BEFORE the slot reduction
// (independent of it) so their latency overlaps it; the grid is sized so the per-workgroup slot
// reads stay a small fraction of the streamed bytes (host: lazy_grid).
template <typename T>
__global__ __launch_bounds__(kBlk) void act_affine_lazy_kernel(const T* __restrict__ x, const LazyStats L,
                                                              T* __restrict__ out, long nvec, int C, int act, float alpha) {
  extern __shared__ float sst[];  // [2][C]
  const long stride = (long)gridDim.x * blockDim.x;
  long v = (long)blockIdx.x * blockDim.x + threadIdx.x;
  float a0[8], a1[8];
  const bool h0 = v < nvec, h1 = v + stride < nvec;
  if (h0) Vec8<T>::load(x + v * 8, a0);
  if (h1) Vec8<T>::load(x + (v + stride) * 8, a1);
  lazy_fill<kBlk>(L, C, sst, sst + C, threadIdx.x, blockIdx.x == 0);
  __syncthreads();
  const unsigned G = (unsigned)(C / 8);
  auto fin = [&](long w, float* a) {
    const int c = (int)((unsigned long)w % G) * 8;
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = act_fwd(fmaf(a[i], sst[c + i], sst[C + c + i]), act, alpha);
    Vec8<T>::store(out + w * 8, a);
  };
  if (h0) fin(v, a0);
  if (h1) fin(v + stride, a1);
  for (v += 2 * stride; v < nvec; v += stride) {
    float a[8];
    Vec8<T>::load(x + v * 8, a);
    fin(v, a);
  }
}

// out = act(ya*sa + ta + (yb ? yb*sb + tb : xid)); (sa, ta) from La; (sb, tb) from Lb when lazy,
// else the finalised vectors sb / tb
template <typename T>
__global__ __launch_bounds__(kBlk) void residual_act_lazy_kernel(const T* __restrict__ ya, const LazyStats La,
                                                                const T* __restrict__ yb, const LazyStats Lb,
                                                                const float* __restrict__ sb,
                                                                const float* __restrict__ tb,
                                                                const T* __restrict__ xid, T* __restrict__ out,
                                                                uint8_t* __restrict__ mask, long nvec, int C, int act,
                                                                float alpha) {
  extern __shared__ float sst[];  // [4][C]: sa ta sb tb
  const long stride = (long)gridDim.x * blockDim.x;
  long v = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const T* src2 = yb ? yb : xid;
  float a0[8], b0[8];
  const bool h0 = v < nvec;
  if (h0) {
    Vec8<T>::load(ya + v * 8, a0);
    Vec8<T>::load(src2 + v * 8, b0);
  }
  const bool w0 = blockIdx.x == 0;
  lazy_fill<kBlk>(La, C, sst, sst + C, threadIdx.x, w0);
  if (yb) {
    if (Lb.base) {
      lazy_fill<kBlk>(Lb, C, sst + 2 * C, sst + 3 * C, threadIdx.x, w0);
    } else {
      for (int c = threadIdx.x; c < C; c += kBlk) {
        sst[2 * C + c] = sb[c];
        sst[3 * C + c] = tb[c];
      }
    }
  }
  __syncthreads();
  const unsigned G = (unsigned)(C / 8);
  auto fin = [&](long w, float* a, float* b) {
    const int c = (int)((unsigned long)w % G) * 8;
    if (yb) {
#pragma unroll
      for (int i = 0; i < 8; ++i) b[i] = fmaf(b[i], sst[2 * C + c + i], sst[3 * C + c + i]);
    }
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      a[i] = act_fwd(fmaf(a[i], sst[c + i], sst[C + c + i]) + b[i], act, alpha);
      m |= (a[i] > 0.f ? 1u : 0u) << i;
    }
    Vec8<T>::store(out + w * 8, a);
    if (mask) mask[w] = (uint8_t)m;
  };
  if (h0) fin(v, a0, b0);
  for (v += stride; v < nvec; v += stride) {
    float a[8], b[8];
    Vec8<T>::load(ya + v * 8, a);
    Vec8<T>::load(src2 + v * 8, b);
    fin(v, a, b);
  }
}

// ------------------------------------------------------------------ launchers
inline int ew_grid(long nvec) {
  long g = (nvec + kBlk - 1) / kBlk;
  if (g > 2048) g = 2048;  // grid-stride beyond ~8 blocks/CU
  if (g < 1) g = 1;
  return (int)g;
}

// grid of a streaming (_u) pass: <= 2048 blocks, kEwU vectors per thread per trip, and the
// stride (blocks * kBlk) a multiple of G (channels fixed per thread); 0 = not applicable
inline int ew_grid_u(long nvec, int G) {
  if (!ew_unroll_flag()) return 0;
  long g = (nvec + (long)kBlk * kEwU - 1) / ((long)kBlk * kEwU);
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  // round up to a multiple of G / gcd(G, kBlk) blocks (G a power of two here)
  if ((G & (G - 1)) != 0) return 0;
  const long q = G > kBlk ? G / kBlk : 1;
  g = (g + q - 1) / q * q;
  return (int)g;
}

// rows per block so that the grid holds ~1024-4096 blocks of >= RPP rows
inline long rows_per_block(long M, const ChanGeom& g) {
  // ~512 partial rows per channel: enough blocks to fill 256 CUs (x gy channel tiles)
  // while keeping the fp64 finalize short
  long target_blocks = 512 / (g.gy > 0 ? g.gy : 1);
  if (target_blocks < 128) target_blocks = 128;
  long r = (M + target_blocks - 1) / target_blocks;
  if (r < g.RPP) r = g.RPP;
  r = (r + g.RPP - 1) / g.RPP * g.RPP;
  return r;
}

void set_ew_unroll(bool on) { ew_unroll_flag() = on ? 1 : 0; }

int stats_num_blocks(long M, int C) {
  ChanGeom g = chan_geom(C);
  long r = rows_per_block(M, g);
  return (int)((M + r - 1) / r);
}

#define DISPATCH_T(dt, ...)                                     \
  switch (dt) {                                                 \
    case kF32: { using T = float; __VA_ARGS__; break; }         \
    case kBF16: { using T = bf16; __VA_ARGS__; break; }         \
    case kF16: { using T = f16; __VA_ARGS__; break; }           \
    default: throw std::runtime_error("bad dtype code");        \
  }

void act_affine_fwd(uint64_t x, uint64_t s, uint64_t t, uint64_t out, long M, int C, int act, float alpha, int dt_in,
                    int dt_out, uint64_t stream) {
  FDT_CHECK(C % 8 == 0, "C % 8");
  long nvec = M * (long)C / 8;
  if (nvec == 0) return;
  DISPATCH_T(dt_in, {
    using TI = T;
    DISPATCH_T(dt_out, {
      act_affine_fwd_kernel<TI, T><<<ew_grid(nvec), kBlk, 0, as_stream(stream)>>>(
          P<const TI>(x), P<const float>(s), P<const float>(t), P<T>(out), nvec, C, act, alpha, wt_flag());
    });
  });
  FDT_LAUNCH_CHECK();
}

void channel_stats_partial(uint64_t y, uint64_t part, long M, int C, int dt, uint64_t stream) {
  ChanGeom g = chan_geom(C);
  long r = rows_per_block(M, g);
  dim3 grid((unsigned)((M + r - 1) / r), g.gy);
  DISPATCH_T(dt, {
    channel_stats_partial_kernel<T><<<grid, kBlk, 0, as_stream(stream)>>>(P<const T>(y), P<float>(part), M, C, g.TPR,
                                                                         g.RPP, r);
  });
  FDT_LAUNCH_CHECK();
}

void stats_finalize(uint64_t part, int nb, int C, double count, int mode, float eps, float momentum, uint64_t gamma,
                    uint64_t beta, uint64_t run_mean, uint64_t run_var, uint64_t nbt, uint64_t out_s, uint64_t out_t,
                    uint64_t save_mean, uint64_t save_aux, int zero_after, uint64_t stream) {
  FinArgs f{mode, eps, momentum, count, P<const float>(gamma), P<const float>(beta), P<float>(run_mean),
            P<float>(run_var), P<long long>(nbt), P<float>(out_s), P<float>(out_t), P<float>(save_mean),
            P<float>(save_aux)};
  stats_finalize_kernel<<<(C + 63) / 64, 64 * kRedWaves, 0, as_stream(stream)>>>(P<float>(part), part ? nb : 0, C,
                                                                                 zero_after, f);
  FDT_LAUNCH_CHECK();
}

void set_deterministic_mode(bool on) { set_deterministic(on); }
bool deterministic_mode() { return deterministic(); }

// deterministic mode: at most `rows` blocks along the slot axis (one slot row per block)
static long cap_rows_per_block(long M, long r, const ChanGeom& g, int rows) {
  if (!deterministic() || (M + r - 1) / r <= rows) return r;
  r = (M + rows - 1) / rows;
  return (r + g.RPP - 1) / g.RPP * g.RPP;
}

void act_bwd_reduce(uint64_t g, uint64_t x, uint64_t s, uint64_t t, uint64_t gx, uint64_t part, int part_rows, long M,
                    int C, int act, float alpha, int dt, uint64_t stream) {
  ChanGeom gg = chan_geom(C);
  long r = cap_rows_per_block(M, rows_per_block(M, gg), gg, part_rows);
  dim3 grid((unsigned)((M + r - 1) / r), gg.gy);
  const unsigned mask = stat_slot_mask(part_rows, grid.x);
  DISPATCH_T(dt, {
    act_bwd_reduce_kernel<T><<<grid, kBlk, 0, as_stream(stream)>>>(P<const T>(g), P<const T>(x), P<const float>(s),
                                                                  P<const float>(t), P<T>(gx), P<float>(part), mask, M,
                                                                  C, gg.TPR, gg.RPP, r, act, alpha, wt_flag());
  });
  FDT_LAUNCH_CHECK();
}

int partials_compact(uint64_t part, int nb, int W, int R, uint64_t out, uint64_t stream) {
  const int nk = (nb + R - 1) / R;
  if (nb == 0 || W == 0) return 0;
  partials_compact_kernel<<<dim3((W + 255) / 256, nk), 256, 0, as_stream(stream)>>>(P<const float>(part), nb, W, R,
                                                                                     P<float>(out));
  FDT_LAUNCH_CHECK();
  return nk;
}

void reduce_partials(uint64_t part, int nb, int nq, int C, uint64_t out, int zero_after, uint64_t stream) {
  const dim3 grid((C + 63) / 64);
  switch (nq) {
    case 1: reduce_partials_kernel<1><<<grid, 64 * kRedWaves, 0, as_stream(stream)>>>(P<float>(part), nb, C, P<float>(out), zero_after); break;
    case 2: reduce_partials_kernel<2><<<grid, 64 * kRedWaves, 0, as_stream(stream)>>>(P<float>(part), nb, C, P<float>(out), zero_after); break;
    case 3: reduce_partials_kernel<3><<<grid, 64 * kRedWaves, 0, as_stream(stream)>>>(P<float>(part), nb, C, P<float>(out), zero_after); break;
    default: throw std::runtime_error("reduce_partials: nq in [1,3]");
  }
  FDT_LAUNCH_CHECK();
}

static CoefArgs coef_args(int mode, float eps, double count, uint64_t save_mean, uint64_t save_aux, uint64_t gamma,
                          uint64_t alpha, uint64_t beta, uint64_t ggamma, uint64_t gbeta) {
  CoefArgs a;
  a.mode = mode;
  a.eps = eps;
  a.count = count;
  a.save_mean = P<const float>(save_mean);
  a.save_aux = P<const float>(save_aux);
  a.gamma = P<const float>(gamma);
  a.alpha = P<float>(alpha);
  a.beta = P<float>(beta);
  a.ggamma = P<float>(ggamma);
  a.gbeta = P<float>(gbeta);
  return a;
}

void stats_bwd_coef(uint64_t gs, uint64_t gt, int C, double count, int mode, float eps, uint64_t save_mean,
                    uint64_t save_aux, uint64_t gamma, uint64_t alpha, uint64_t beta, uint64_t ggamma, uint64_t gbeta,
                    uint64_t stream) {
  stats_bwd_coef_kernel<<<(C + 255) / 256, 256, 0, as_stream(stream)>>>(
      P<const float>(gs), P<const float>(gt), C,
      coef_args(mode, eps, count, save_mean, save_aux, gamma, alpha, beta, ggamma, gbeta));
  FDT_LAUNCH_CHECK();
}

void stats_bwd_finalize(uint64_t part, int nb, int nq, int C, int a_mode, float a_eps, double a_count, uint64_t a_sm,
                        uint64_t a_sa, uint64_t a_gamma, uint64_t a_alpha, uint64_t a_beta, uint64_t a_gg,
                        uint64_t a_gb, int b_mode, float b_eps, double b_count, uint64_t b_sm, uint64_t b_sa,
                        uint64_t b_gamma, uint64_t b_alpha, uint64_t b_beta, uint64_t b_gg, uint64_t b_gb,
                        uint64_t stream) {
  const CoefArgs A = coef_args(a_mode, a_eps, a_count, a_sm, a_sa, a_gamma, a_alpha, a_beta, a_gg, a_gb);
  const CoefArgs B = coef_args(b_mode, b_eps, b_count, b_sm, b_sa, b_gamma, b_alpha, b_beta, b_gg, b_gb);
  const dim3 grid((C + 63) / 64);
  if (nq == 2) {
    stats_bwd_finalize_kernel<2><<<grid, 64 * kRedWaves, 0, as_stream(stream)>>>(P<float>(part), nb, C, A, B);
  } else if (nq == 3) {
    stats_bwd_finalize_kernel<3><<<grid, 64 * kRedWaves, 0, as_stream(stream)>>>(P<float>(part), nb, C, A, B);
  } else {
    throw std::runtime_error("stats_bwd_finalize: nq in {2,3}");
  }
  FDT_LAUNCH_CHECK();
}

void affine_fold(uint64_t gy, uint64_t y, uint64_t alpha, uint64_t beta, uint64_t gs, uint64_t out, long M, int C,
                 int dt, uint64_t stream) {
  FDT_CHECK(C % 8 == 0, "C % 8");
  long nvec = M * (long)C / 8;
  if (nvec == 0) return;
  const int gu = ew_grid_u(nvec, C / 8);
  DISPATCH_T(dt, {
    if (gu)
      affine_fold_u_kernel<T><<<gu, kBlk, 0, as_stream(stream)>>>(
          P<const T>(gy), P<const T>(y), P<const float>(alpha), P<const float>(beta), P<const float>(gs), P<T>(out),
          nvec, C / 8, wt_flag());
    else
      affine_fold_kernel<T><<<ew_grid(nvec), kBlk, 0, as_stream(stream)>>>(
          P<const T>(gy), P<const T>(y), P<const float>(alpha), P<const float>(beta), P<const float>(gs), P<T>(out),
          nvec, C / 8, wt_flag());
  });
  FDT_LAUNCH_CHECK();
}

void residual_act_fwd(uint64_t ya, uint64_t sa, uint64_t ta, uint64_t yb, uint64_t sb, uint64_t tb, uint64_t xid,
                      uint64_t out, uint64_t mask, long M, int C, int act, float alpha, int dt, uint64_t stream) {
  FDT_CHECK(C % 8 == 0, "C % 8");
  long nvec = M * (long)C / 8;
  if (nvec == 0) return;
  FDT_CHECK(yb != 0 || xid != 0, "residual needs a second branch");
  FDT_CHECK(mask == 0 || act == kActRelu, "the activation bit mask is for ReLU joins");
  long g = (nvec + 2 * kBlk - 1) / (2 * kBlk);  // two vectors per thread
  if (g > 4096) g = 4096;
  const bool hoist = ((g * kBlk) % (C / 8)) == 0;
  DISPATCH_T(dt, {
    auto kern = hoist ? residual_act_fwd_kernel<T, true> : residual_act_fwd_kernel<T, false>;
    kern<<<(int)g, kBlk, 0, as_stream(stream)>>>(
        P<const T>(ya), P<const float>(sa), P<const float>(ta), P<const T>(yb), P<const float>(sb), P<const float>(tb),
        P<const T>(xid), P<T>(out), P<uint8_t>(mask), nvec, C / 8, act, alpha, wt_flag());
  });
  FDT_LAUNCH_CHECK();
}

// grid of a lazy-statistics consumer: per-workgroup slot reads (rows x nq x C fp32) at most
// ~1/4 of the bytes the pass streams, at least 32 workgroups, at most the plain pass's grid
static int lazy_grid(long nvec, long stream_bytes, long stats_bytes) {
  long g = stream_bytes / (4 * (stats_bytes > 0 ? stats_bytes : 1));
  const long cap = ew_grid(nvec);
  if (g > cap) g = cap;
  if (g < 32) g = 32;
  if (g > (nvec + kBlk - 1) / kBlk) g = (nvec + kBlk - 1) / kBlk;
  return (int)(g < 1 ? 1 : g);
}

void act_affine_lazy(uint64_t x, const std::vector<uint64_t>& lz_ptr, const std::vector<double>& lz_val, uint64_t out,
                     long M, int C, int act, float alpha, int dt, uint64_t stream) {
  FDT_CHECK(C % 8 == 0 && C <= 8192, "act_affine_lazy: C % 8 == 0, C <= 8192");
  const LazyStats L = make_lazy(lz_ptr, lz_val);
  FDT_CHECK(L.base != nullptr, "act_affine_lazy: lazy statistics required");
  const long nvec = M * (long)C / 8;
  if (nvec == 0) return;
  const int T = dt == kF32 ? 4 : 2;
  const int g = lazy_grid(nvec, 2 * M * (long)C * T, (long)L.rows * 2 * C * 4);
  const size_t lds = (size_t)2 * C * sizeof(float);
  DISPATCH_T(dt, {
    act_affine_lazy_kernel<T><<<g, kBlk, lds, as_stream(stream)>>>(P<const T>(x), L, P<T>(out), nvec, C, act, alpha);
  });
  FDT_LAUNCH_CHECK();
}

void residual_act_lazy(uint64_t ya, const std::vector<uint64_t>& la_ptr, const std::vector<double>& la_val,
                       uint64_t yb, const std::vector<uint64_t>& lb_ptr, const std::vector<double>& lb_val,
                       uint64_t sb, uint64_t tb, uint64_t xid, uint64_t out, uint64_t mask, long M, int C, int act,
                       float alpha, int dt, uint64_t stream) {
  FDT_CHECK(C % 8 == 0 && C <= 4096, "residual_act_lazy: C % 8 == 0, C <= 4096");
  FDT_CHECK((yb != 0) != (xid != 0), "residual_act_lazy: a projection shortcut yb or an identity xid");
  FDT_CHECK(mask == 0 || act == kActRelu, "the activation bit mask is for ReLU joins");
  const LazyStats La = make_lazy(la_ptr, la_val);
  const LazyStats Lb = make_lazy(lb_ptr, lb_val);
  FDT_CHECK(La.base != nullptr, "residual_act_lazy: the residual branch's statistics must be lazy");
  FDT_CHECK(yb == 0 || Lb.base != nullptr || (sb != 0 && tb != 0), "residual_act_lazy: shortcut statistics");
  const long nvec = M * (long)C / 8;
  if (nvec == 0) return;
  const int T = dt == kF32 ? 4 : 2;
  const long sbytes = ((long)La.rows + (Lb.base ? Lb.rows : 0)) * 2 * C * 4;
  const int g = lazy_grid(nvec, 3 * M * (long)C * T, sbytes);
  const size_t lds = (size_t)4 * C * sizeof(float);
  DISPATCH_T(dt, {
    residual_act_lazy_kernel<T><<<g, kBlk, lds, as_stream(stream)>>>(
        P<const T>(ya), La, P<const T>(yb), Lb, P<const float>(sb), P<const float>(tb), P<const T>(xid), P<T>(out),
        P<uint8_t>(mask), nvec, C, act, alpha);
  });
  FDT_LAUNCH_CHECK();
}

void residual_act_bwd(uint64_t g, uint64_t out, uint64_t mask, uint64_t ya, uint64_t yb, uint64_t gpre, uint64_t part,
                      int part_rows, long M, int C, int act, float alpha, int dt, uint64_t stream, int ghw,
                      const std::vector<uint64_t>& jz) {
  // jz = {} or {sa, ta, sb, tb, xid}: act' from the recomputed pre-activation (z mode, see the kernel)
  FDT_CHECK(jz.empty() || jz.size() == 5, "residual_act_bwd: jz = [] | [sa, ta, sb, tb, xid]");
  const bool zm = jz.size() == 5;
  FDT_CHECK(!zm || (jz[0] && jz[1] && (yb ? (jz[2] && jz[3]) : jz[4] != 0)),
            "residual_act_bwd z mode: sa, ta and the shortcut's sb, tb (BN'd) or xid (identity)");
  FDT_CHECK(out != 0 || mask != 0 || zm, "residual_act_bwd needs the output, its mask or the z operands");
  FDT_CHECK(ghw >= 0 && (ghw == 0 || M % ghw == 0), "residual_act_bwd: broadcast rows must divide M");
  ChanGeom gg = chan_geom(C);
  // ~1024 blocks: more waves in flight for this 4-5 stream kernel than the stats default
  constexpr long kBlocks = 1024;
  long target = kBlocks / (gg.gy > 0 ? gg.gy : 1);
  long r = (M + target - 1) / target;
  if (r < gg.RPP) r = gg.RPP;
  r = (r + gg.RPP - 1) / gg.RPP * gg.RPP;
  r = cap_rows_per_block(M, r, gg, part_rows);
  dim3 grid((unsigned)((M + r - 1) / r), gg.gy);
  const unsigned smask = stat_slot_mask(part_rows, grid.x);
  DISPATCH_T(dt, {
    residual_act_bwd_kernel<T><<<grid, kBlk, 0, as_stream(stream)>>>(
        P<const T>(g), P<const T>(out), P<const uint8_t>(mask), P<const T>(ya), P<const T>(yb), P<T>(gpre), P<float>(part),
        smask, M, C, gg.TPR, gg.RPP, r, act, alpha, ghw, wt_flag(), zm ? P<const float>(jz[0]) : nullptr,
        zm ? P<const float>(jz[1]) : nullptr, zm ? P<const float>(jz[2]) : nullptr,
        zm ? P<const float>(jz[3]) : nullptr, zm ? P<const T>(jz[4]) : nullptr);
  });
  FDT_LAUNCH_CHECK();
}

}  // namespace fdt
