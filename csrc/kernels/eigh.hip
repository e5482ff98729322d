// Batched symmetric eigendecomposition for the NGD preconditioner (gfx950 / CDNA4).
//
// NGD (reference ngd_optimizer.py:265) needs eigh of many small symmetric R x R matrices
// (R <= 80 by default); the reference calls LAPACK/cuSOLVER
// once per (parameter, axis) with a host round-trip each.  Here one 1024-thread workgroup
// owns one matrix: A ([n][n+1] fp32, odd stride against bank conflicts, upper triangle only)
// and the TRANSPOSED eigenvector accumulator Vt ([n][n+4], 16-B rows: a column rotation of V
// is a float4 rotation of two Vt rows) live in LDS (~52 KB at R = 80), and cyclic two-sided
// Jacobi runs with the round-robin (tournament) ordering -- every round rotates n/2 disjoint
// (p,q) pairs at once.  1024 threads measured fastest (1024 / 512 / 256: 0.92 / 1.16 / 2.00
// ms on the transformer's 147 80x80 matrices, profiles/r4/eigh_threads_*.txt): a round is
// LDS / VALU throughput bound, not latency bound.
//
// Round structure (two barriers):
//   1. one lane per pair computes (c, s) and the closed-form new diagonal entries;
//   2. A <- J^T A J as independent 2x2 blocks: the pairs partition the indices, so every
//      element belongs to exactly one (pair k1, pair k2) block and each block's update
//      needs only its own four entries.  Only upper blocks (k1 <= k2) are computed, and only
//      the upper-triangle entries are stored.  The
//      diagonal block of a rotated pair is written in closed form (a_pq <- 0 exactly, a_pp
//      and a_qq from t) -- without exact annihilation, fp32 rounding residue in a_pq stalls
//      convergence at ~1e-4 relative.  V <- V J runs in the same phase.
// Pairs with |a_pq| <= 1e-9 sqrt|a_pp a_qq| are zeroed without rotating.  Sweeps stop once
// the off-diagonal Frobenius mass is below tol^2 * ||A||_F^2 (one LDS reduction per sweep;
// typically 5-8 sweeps at R <= 128) or after max_sweeps.  Eigenvalues are returned
// ascending with matching eigenvector columns (rank sort), the torch.linalg.eigh
// convention.  No host synchronisation; graph-capturable.
//
// Ragged batches: an optional int table [batch][3] = (n, offset of the matrix in A/V,
// offset of its eigenvalues in w) lets one launch cover every NGD shape group (different
// ranks) -- the optimizer issues one eigh launch per axis level instead of one per group.
#include "common.h"

namespace fdt {

constexpr int kEighThreadsMax = 1024;
constexpr int kEighMaxN = 128;
constexpr int kEighMaxPairs = kEighMaxN / 2;
// upper 2x2 blocks per thread: 64*65/2 = 2080 blocks / 1024 threads
template <int NT>
constexpr int eigh_blk_per_thread() { return (kEighMaxPairs * (kEighMaxPairs + 1) / 2 + NT - 1) / NT; }
// V tasks (pair, 4-row chunk) per thread: 64 x 32 / 1024
template <int NT>
constexpr int eigh_vt_per_thread() { return (kEighMaxPairs * (kEighMaxN / 4) + NT - 1) / NT; }
// Vt row stride: float4 rows, +4 floats so consecutive rows start on other banks
__host__ __device__ constexpr int eigh_ldv(int n) { return ((n + 3) & ~3) + 4; }

template <int kEighThreads>
__global__ __launch_bounds__(kEighThreads) void jacobi_eigh_kernel(const float* __restrict__ Ain,
                                                                   float* __restrict__ wout, float* __restrict__ Vout,
                                                                   const int* __restrict__ table, int n_uniform,
                                                                   int max_sweeps, float tol) {
  constexpr int kEighBlkPerThread = eigh_blk_per_thread<kEighThreads>();
  constexpr int kEighVtPerThread = eigh_vt_per_thread<kEighThreads>();
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const long mat = blockIdx.x;
  int n = n_uniform;
  long offA = mat * (long)n * n, offw = mat * n;
  if (table) {
    n = table[3 * mat];
    offA = table[3 * mat + 1];
    offw = table[3 * mat + 2];
  }
  const int ld = n + 1;
  float4* prm = reinterpret_cast<float4*>(sm);                     // [64] (c, s, new a_pp, new a_qq)
  int2* pidx = reinterpret_cast<int2*>(prm + kEighMaxPairs);        // [64] (p, q); q = -1 for the dummy
  float* red = reinterpret_cast<float*>(pidx + kEighMaxPairs);      // [32]
  int* rank = reinterpret_cast<int*>(red + 32);                     // [128]
  float* A = reinterpret_cast<float*>(rank + kEighMaxN);            // [n][ld]
  // the eigenvector accumulator TRANSPOSED: Vt[j][i] = V[i][j], so V <- V J (a rotation of
  // columns p, q of V) is a rotation of two contiguous rows -- float4 LDS reads / writes, one
  // (pair, 4-row chunk) task per thread instead of four scalar (row, pair) elements
  const int ldv = eigh_ldv(n);
  float* Vt = A + ((n * ld + 3) & ~3);                              // [n][ldv], 16-B rows
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const float* src = Ain + offA;

  for (int e = tid; e < n * n; e += kEighThreads) {
    const int i = e / n, j = e - (e / n) * n;
    // symmetrise from the upper triangle (torch UPLO='U' convention)
    const float v = i <= j ? src[(long)i * n + j] : src[(long)j * n + i];
    A[i * ld + j] = v;
  }
  for (int e = tid; e < n * ldv; e += kEighThreads) {
    const int j = e / ldv, i = e - j * ldv;
    Vt[e] = (i == j) ? 1.f : 0.f;  // (padding columns i >= n stay finite: never output)
  }

  const int m = (n + 1) & ~1;  // players (a dummy when n is odd)
  const int npairs = m / 2;
  const int nblk = npairs * (npairs + 1) / 2;

  // this thread's upper blocks (k1 <= k2), decoded once
  int bk1[kEighBlkPerThread], bk2[kEighBlkPerThread];
#pragma unroll
  for (int u = 0; u < kEighBlkPerThread; ++u) {
    const int b = tid + u * kEighThreads;
    int k2 = (int)((sqrtf(8.f * b + 1.f) - 1.f) * 0.5f);
    while (k2 * (k2 + 1) / 2 > b) --k2;
    while ((k2 + 1) * (k2 + 2) / 2 <= b) ++k2;
    bk2[u] = b < nblk ? k2 : -1;
    bk1[u] = b - k2 * (k2 + 1) / 2;
  }
  // this thread's V tasks (pair slot k, 4-element chunk c of the two Vt rows), decoded once:
  // no integer division inside the round loop
  const int nch = (n + 3) >> 2, ntask = npairs * nch;
  int vk[kEighVtPerThread], vc[kEighVtPerThread];
#pragma unroll
  for (int u = 0; u < kEighVtPerThread; ++u) {
    const int t = tid + u * kEighThreads;
    const int k = t / nch;
    vk[u] = t < ntask ? k : -1;
    vc[u] = (t - k * nch) * 4;
  }
  // A is kept in its UPPER triangle only (a 2x2 block update writes 4 entries, not 8)
  auto at = [ld](int a, int b) { return a < b ? a * ld + b : b * ld + a; };
  __syncthreads();

  for (int sweep = 0; sweep < max_sweeps; ++sweep) {
    float o = 0.f, t = 0.f;
    for (int e = tid; e < n * n; e += kEighThreads) {
      const int i = e / n, j = e - (e / n) * n;
      if (i > j) continue;
      const float v = A[i * ld + j];
      const float v2 = i == j ? v * v : 2.f * v * v;
      t += v2;
      if (i != j) o += v2;
    }
    o = wave_sum(o);
    t = wave_sum(t);
    if (lane == 0) { red[wid] = o; red[16 + wid] = t; }
    __syncthreads();
    float off = 0.f, tot = 0.f;
#pragma unroll
    for (int w = 0; w < kEighThreads / 64; ++w) { off += red[w]; tot += red[16 + w]; }
    __syncthreads();
    if (off <= tol * tol * tot) break;

    for (int r = 0; r < m - 1; ++r) {
      // ---- 1. rotation per pair (tournament pairing: slot 0 fixed, slots 1..m-1 rotate)
      if (tid < npairs) {
        const int i = tid;
        // (i - 1 + r, m - 2 - i + r < 2 (m - 1): the modulo is one conditional subtract)
        int ta = i - 1 + r, tb = m - 2 - i + r;
        ta = ta >= m - 1 ? ta - (m - 1) : ta;
        tb = tb >= m - 1 ? tb - (m - 1) : tb;
        const int a = i == 0 ? 0 : 1 + ta;
        const int b = 1 + tb;
        int p = a < b ? a : b, q = a < b ? b : a;
        float c = 1.f, s = 0.f, dp = 0.f, dq = 0.f;
        if (q < n) {
          const float apq = A[p * ld + q];
          const float app = A[p * ld + p], aqq = A[q * ld + q];
          dp = app;
          dq = aqq;
          if (fabsf(apq) > 1e-9f * sqrtf(fabsf(app * aqq)) && fabsf(apq) > 1e-30f) {
            const float theta = (aqq - app) / (2.f * apq);
            // t = sign(theta) / (|theta| + sqrt(theta^2 + 1)); 1/(2 theta) once theta^2 overflows
            const float at = fabsf(theta);
            const float tt = at < 1e18f ? copysignf(1.f, theta) / (at + sqrtf(theta * theta + 1.f)) : 0.5f / theta;
            c = rsqrtf(tt * tt + 1.f);
            s = tt * c;
            dp = app - tt * apq;
            dq = aqq + tt * apq;
          }
        } else {
          q = -1;  // paired with the dummy: index p is not rotated this round
        }
        prm[i] = make_float4(c, s, dp, dq);
        pidx[i] = make_int2(p, q);
      }
      __syncthreads();
      // ---- 2. A <- J^T A J by 2x2 blocks (upper blocks, mirrored), V <- V J
#pragma unroll
      for (int u = 0; u < kEighBlkPerThread; ++u) {
        const int k1 = bk1[u], k2 = bk2[u];
        if (k2 < 0) continue;
        const int2 i1 = pidx[k1], i2 = pidx[k2];
        if (k1 == k2) {
          if (i1.y >= 0) {  // rotated pair: closed form, exact zero off the diagonal
            const float4 r1 = prm[k1];
            A[i1.x * ld + i1.x] = r1.z;
            A[i1.y * ld + i1.y] = r1.w;
            A[i1.x * ld + i1.y] = 0.f;  // (p < q: the upper entry)
          }
          continue;
        }
        const float4 r1 = prm[k1], r2 = prm[k2];
        const bool h1 = i1.y >= 0, h2 = i2.y >= 0;
        const int o00 = at(i1.x, i2.x);
        const int o01 = h2 ? at(i1.x, i2.y) : 0, o10 = h1 ? at(i1.y, i2.x) : 0;
        const int o11 = (h1 && h2) ? at(i1.y, i2.y) : 0;
        const float a00 = A[o00];
        const float a01 = h2 ? A[o01] : 0.f;
        const float a10 = h1 ? A[o10] : 0.f;
        const float a11 = (h1 && h2) ? A[o11] : 0.f;
        // rows (pair k1): row_p <- c row_p - s row_q, row_q <- s row_p + c row_q
        const float b00 = r1.x * a00 - r1.y * a10, b01 = r1.x * a01 - r1.y * a11;
        const float b10 = r1.y * a00 + r1.x * a10, b11 = r1.y * a01 + r1.x * a11;
        // columns (pair k2)
        const float n00 = r2.x * b00 - r2.y * b01, n01 = r2.y * b00 + r2.x * b01;
        const float n10 = r2.x * b10 - r2.y * b11, n11 = r2.y * b10 + r2.x * b11;
        A[o00] = n00;
        if (h2) A[o01] = n01;
        if (h1) A[o10] = n10;
        if (h1 && h2) A[o11] = n11;
      }
#pragma unroll
      for (int u = 0; u < kEighVtPerThread; ++u) {
        const int k = vk[u];
        if (k < 0) continue;
        const int2 pq = pidx[k];
        if (pq.y < 0) continue;
        const float4 rr = prm[k];
        float4* vp = reinterpret_cast<float4*>(Vt + pq.x * ldv + vc[u]);
        float4* vq = reinterpret_cast<float4*>(Vt + pq.y * ldv + vc[u]);
        const float4 a = *vp, b = *vq;
        *vp = make_float4(rr.x * a.x - rr.y * b.x, rr.x * a.y - rr.y * b.y, rr.x * a.z - rr.y * b.z,
                          rr.x * a.w - rr.y * b.w);
        *vq = make_float4(rr.y * a.x + rr.x * b.x, rr.y * a.y + rr.x * b.y, rr.y * a.z + rr.x * b.z,
                          rr.y * a.w + rr.x * b.w);
      }
      __syncthreads();
    }
  }

  // ascending order: eigenvalue j goes to slot rank(j) (ties broken by index)
  float* wo = wout + offw;
  float* vo = Vout + offA;
  for (int j = tid; j < n; j += kEighThreads) {
    const float d = A[j * ld + j];
    int rk = 0;
    for (int k = 0; k < n; ++k) {
      const float dk = A[k * ld + k];
      rk += (dk < d) || (dk == d && k < j);
    }
    rank[j] = rk;
    wo[rk] = d;
  }
  __syncthreads();
  for (int e = tid; e < n * n; e += kEighThreads) {
    const int i = e / n, j = e - (e / n) * n;
    vo[(long)i * n + rank[j]] = Vt[j * ldv + i];
  }
}

void jacobi_eigh(uint64_t A, uint64_t w, uint64_t V, uint64_t table, int batch, int n, int max_sweeps, float tol,
                 uint64_t stream) {
  // n: the uniform size, or (with a table) the largest n in the table (sizes the LDS)
  FDT_CHECK(n >= 1 && n <= kEighMaxN, "jacobi_eigh: n must be in [1, 128]");
  if (batch == 0) return;
  const size_t lds = (size_t)((n * (n + 1) + 3) & ~3) * 4 + (size_t)n * eigh_ldv(n) * 4 + kEighMaxPairs * (16 + 8) +
                     32 * 4 + kEighMaxN * 4;
  // workgroup size: 1024 threads (16 waves) by default; FDT_EIGH_THREADS = 512 / 256 (A/B)
  static const int nt = [] {
    const char* e = getenv("FDT_EIGH_THREADS");
    const int v = e ? atoi(e) : 1024;
    return (v == 256 || v == 512) ? v : 1024;
  }();
  auto go = [&](auto kern, int threads) {
    static size_t set[3] = {64 * 1024, 64 * 1024, 64 * 1024};
    size_t& s_ = set[threads == 1024 ? 0 : (threads == 512 ? 1 : 2)];
    if (lds > s_) {
      FDT_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                        (int)lds));
      s_ = lds;
    }
    hipLaunchKernelGGL(kern, dim3(batch), dim3(threads), lds, as_stream(stream), P<const float>(A), P<float>(w),
                       P<float>(V), P<const int>(table), n, max_sweeps, tol);
  };
  if (nt == 256) go(jacobi_eigh_kernel<256>, 256);
  else if (nt == 512) go(jacobi_eigh_kernel<512>, 512);
  else go(jacobi_eigh_kernel<1024>, 1024);
  FDT_LAUNCH_CHECK();
}

}  // namespace fdt
