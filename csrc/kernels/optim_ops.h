// Per-element update rules of the flat optimizers, shared by the flat kernels (optim.hip) and
// the fused update-and-pack kernel (optim_pack.hip), so both apply bitwise the same math.
// Each op is built on the device at kernel start (device scalars: clip coefficient, skipped-step
// count, scheduled lr) and applied per element: reads p / g / state, writes p / state /
// (optional) bf16 shadow / zeroed g, returns the new parameter.
#pragma once
#include "common.h"

namespace fdt {
namespace opt {

__device__ __forceinline__ bool skip_step(const int* found_inf) { return found_inf && *found_inf != 0; }

// A skipped (non-finite / fp16-overflow) step still clears the gradient when the optimizer
// owns zero_grad: otherwise the bad values would accumulate into every following step.
__device__ __forceinline__ void skip_zero(float* __restrict__ g, long n, int zero_grad) {
  if (!zero_grad) return;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) g[i] = 0.f;
}
__device__ __forceinline__ float gscale(const float* p) { return p ? *p : 1.f; }

// Step counters of MADGRAD / MirrorMADGRAD / Adam count APPLIED steps only (torch's
// GradScaler skips optimizer.step() on an overflow, so the reference never advances them on
// a skipped step).  The host passes the number of step() calls k; the device counter
// kskip holds the number of skipped ones: a skipped step bumps it (one thread; no other
// block reads it in a skipped step), an applied step uses k - kskip.
__device__ __forceinline__ void count_skip(int* kskip) {
  if (kskip && blockIdx.x == 0 && threadIdx.x == 0) *kskip += 1;
}
__device__ __forceinline__ long applied_k(long k, const int* kskip) { return kskip ? k - (long)*kskip : k; }

// ---------------------------------------------------------------- MADGRAD (dual averaging)
// k = step index (0-based).  lamb = (lr+eps)*sqrt(k+1).  momentum==0 -> x0 recomputed
// from (p, s, old rms) like the reference package; else x0 is a stored state buffer.
struct MadArgs {
  float *p, *g, *gss, *s, *x0;
  bf16* shadow;
  float lr, momentum, wd, eps;
  int decouple;
  long k;
  int* kskip;
  const float* gsc;
  const int* found_inf;
  int zero_grad;
  int count_skips = 1;  // 0: a second launch of the same step (the first one counts a skipped step)
};

struct MadOp {
  MadArgs a;
  float c, lr_e, lamb, ck;
  __device__ explicit MadOp(const MadArgs& args) : a(args) {
    c = gscale(a.gsc);
    lr_e = a.lr + a.eps;
    lamb = lr_e * sqrtf((float)(applied_k(a.k, a.kskip) + 1));
    ck = 1.f - a.momentum;
  }
  __device__ __forceinline__ static bool skipped(const MadArgs& a) { return skip_step(a.found_inf); }
  __device__ __forceinline__ static void on_skip(const MadArgs& a, long n) {
    if (a.count_skips) count_skip(a.kskip);
    skip_zero(a.g, n, a.zero_grad);
  }
  // the rule on loaded values: q = grad_sum_sq, sv = s (updated in place); returns the new p
  // (no FMA contraction here: every caller -- wherever it inlines this -- rounds identically)
  __device__ __forceinline__ float rule(float pv, float gv, float& q, float& sv, float x0v) const {
#pragma clang fp contract(off)
    gv *= c;
    if (a.wd != 0.f && !a.decouple) gv += a.wd * pv;
    if (a.momentum == 0.f) x0v = pv + sv / (cbrtf(q) + a.eps);
    q = fmaf(lamb * gv, gv, q);
    float rms = cbrtf(q) + a.eps;
    if (a.wd != 0.f && a.decouple) pv -= lr_e * a.wd * pv;
    sv = fmaf(lamb, gv, sv);
    float z = x0v - sv / rms;
    return a.momentum == 0.f ? z : (1.f - ck) * pv + ck * z;
  }
  __device__ __forceinline__ void store(long i, float pv, float q, float sv) const {
    a.p[i] = pv;
    a.gss[i] = q;
    a.s[i] = sv;
    if (a.shadow) a.shadow[i] = __float2bfloat16(pv);
    if (a.zero_grad) a.g[i] = 0.f;
  }
  __device__ __forceinline__ float operator()(long i) const {
    float q = a.gss[i], sv = a.s[i];
    const float pv = rule(a.p[i], a.g[i], q, sv, a.momentum == 0.f ? 0.f : a.x0[i]);
    store(i, pv, q, sv);
    return pv;
  }
  // U elements at once: every load issued before any math / store (latency-bound callers)
  template <int U>
  __device__ __forceinline__ void apply(const long (&i)[U], const bool (&ok)[U], float (&out)[U]) const {
    float pv[U], gv[U], q[U], sv[U], x0v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (ok[u]) {
        pv[u] = a.p[i[u]];
        gv[u] = a.g[i[u]];
        q[u] = a.gss[i[u]];
        sv[u] = a.s[i[u]];
        x0v[u] = a.momentum == 0.f ? 0.f : a.x0[i[u]];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (ok[u]) {
        out[u] = rule(pv[u], gv[u], q[u], sv[u], x0v[u]);
        store(i[u], out[u], q[u], sv[u]);
      } else {
        out[u] = 0.f;
      }
    }
  }
};

// ---------------------------------------------------------------- SGD (+momentum, NGD tail)
// One rule for optim.hip sgd_kernel (float4 lanes) and the fused update-and-pack kernel.
struct SgdArgs {
  float *p, *g, *buf;
  bf16* shadow;
  float lr, momentum, dampening, wd;
  int nesterov, first;
  const float* gsc;
  const int* found_inf;
  int zero_grad;
  const float* lr_dev;
};

struct SgdOp {
  SgdArgs a;
  float c, lr, momentum;
  __device__ explicit SgdOp(const SgdArgs& args) : a(args) {
    c = gscale(a.gsc);
    lr = a.lr_dev ? a.lr_dev[0] : a.lr;
    momentum = a.lr_dev ? a.lr_dev[1] : a.momentum;
  }
  __device__ __forceinline__ static bool skipped(const SgdArgs& a) { return skip_step(a.found_inf); }
  __device__ __forceinline__ static void on_skip(const SgdArgs& a, long n) { skip_zero(a.g, n, a.zero_grad); }
  // the rule on loaded values: bv = momentum buffer (updated in place); returns the new p
  __device__ __forceinline__ float rule(float pv, float gv, float& bv) const {
#pragma clang fp contract(off)
    float d = gv * c + a.wd * pv;
    if (momentum != 0.f) {
      if (a.first) bv = d;
      else bv = momentum * bv + (1.f - a.dampening) * d;
      if (a.nesterov) d += momentum * bv;
      else d = bv;
    }
    return pv - lr * d;
  }
  __device__ __forceinline__ void store(long i, float pv, float bv) const {
    if (momentum != 0.f) a.buf[i] = bv;
    a.p[i] = pv;
    if (a.shadow) a.shadow[i] = __float2bfloat16(pv);
    if (a.zero_grad) a.g[i] = 0.f;
  }
  __device__ __forceinline__ float operator()(long i) const {
    float bv = (momentum != 0.f && !a.first) ? a.buf[i] : 0.f;
    const float pv = rule(a.p[i], a.g[i], bv);
    store(i, pv, bv);
    return pv;
  }
  template <int U>
  __device__ __forceinline__ void apply(const long (&i)[U], const bool (&ok)[U], float (&out)[U]) const {
    float pv[U], gv[U], bv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (ok[u]) {
        pv[u] = a.p[i[u]];
        gv[u] = a.g[i[u]];
        bv[u] = (momentum != 0.f && !a.first) ? a.buf[i[u]] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (ok[u]) {
        out[u] = rule(pv[u], gv[u], bv[u]);
        store(i[u], out[u], bv[u]);
      } else {
        out[u] = 0.f;
      }
    }
  }
};

}  // namespace opt
}  // namespace fdt
