// Fused optimizer kernels over FLAT parameter / gradient / state buffers.
//
// The engine keeps all parameters of a model in one fp32 buffer and all gradients in
// another (utils/flat.py), so each optimizer step is ONE launch over ~23.5M (ResNet-50)
// or ~29.3M (Transformer) elements instead of 69/105 per-tensor launches x several ops.
// Every step kernel fuses:  grad * clip_coef (device scalar, no host sync)
//   -> [skip if found_inf (device flag), GradScaler semantics]
//   -> weight decay -> update rule -> optional bf16 shadow-weight write (the compute copy
//   used by the HIP conv/GEMM kernels) -> optional grad zeroing.
// Reference update rules: SGD/NGD momentum ngd_optimizer.py:478-506; MADGRAD and
// MirrorMADGRAD from the external madgrad package used at resnet50_test.py:493 and
// transformer_test.py:220 (package not vendored; rules re-derived, see optim/madgrad.py).
#include "common.h"
#include "optim_ops.h"

namespace fdt {

constexpr int kOB = 256;

inline int opt_grid(long n4) {
  long g = (n4 + kOB - 1) / kOB;
  if (g > 4096) g = 4096;
  return g < 1 ? 1 : (int)g;
}

using opt::applied_k;
using opt::count_skip;
using opt::gscale;
using opt::skip_step;
using opt::skip_zero;

__device__ __forceinline__ void store_shadow(bf16* sh, long i, float4 v) {
  uint2 u;
  u.x = pack_bf16x2(v.x, v.y);
  u.y = pack_bf16x2(v.z, v.w);
  *reinterpret_cast<uint2*>(sh + i) = u;
}

// --------------------------------------------------------------- grad norm / unscale
// part[blk] = sum (g*inv_scale)^2 ; writes g *= inv_scale when unscale; found_inf |= !finite
__global__ __launch_bounds__(kOB) void grad_sumsq_kernel(float* __restrict__ g, long n4, const float* __restrict__ inv_scale,
                                                         int unscale, float* __restrict__ part, int* __restrict__ found_inf) {
  __shared__ float sm[kOB / 64];
  float sc = inv_scale ? *inv_scale : 1.f;
  float acc = 0.f;
  bool bad = false;
  float4* g4 = reinterpret_cast<float4*>(g);
  for (long i = (long)blockIdx.x * kOB + threadIdx.x; i < n4; i += (long)gridDim.x * kOB) {
    float4 v = g4[i];
    v.x *= sc; v.y *= sc; v.z *= sc; v.w *= sc;
    if (unscale) g4[i] = v;
    bad |= !(isfinite(v.x) && isfinite(v.y) && isfinite(v.z) && isfinite(v.w));
    acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = acc;
  if (found_inf && __any(bad) && (threadIdx.x & 63) == 0) atomicOr(found_inf, 1);
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < kOB / 64; ++w) t += sm[w];
    part[blockIdx.x] = t;
  }
}

// norm = sqrt(sum part); coef = min(1, max_norm/(norm+1e-6)) (torch clip_grad_norm_);
// max_norm <= 0 -> coef = 1.  out[0] = norm, out[1] = coef
// phase 0: parts -> [norm, coef];  phase 1: parts -> fp64 total (a sharded gradient all-reduces
// it);  phase 2: fp64 total -> [norm, coef].  Phases 1+2 give bitwise the phase-0 result on
// one rank (same summation tree, same fp64 finalize), so sharded and unsharded runs agree.
__global__ void grad_norm_finalize_kernel(const float* __restrict__ part, int nb, float max_norm, float* __restrict__ out,
                                          double* __restrict__ total, int phase) {
  __shared__ double sm[256];
  if (phase != 2) {
    double a = 0.0;
    for (int i = threadIdx.x; i < nb; i += blockDim.x) a += part[i];
    sm[threadIdx.x] = a;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
      if (threadIdx.x < o) sm[threadIdx.x] += sm[threadIdx.x + o];
      __syncthreads();
    }
  }
  if (threadIdx.x == 0) {
    if (phase == 1) {
      total[0] = sm[0];
      return;
    }
    const double sq = phase == 2 ? total[0] : sm[0];
    double norm = sqrt(sq);
    out[0] = (float)norm;
    double c = max_norm > 0.f ? (double)max_norm / (norm + 1e-6) : 1.0;
    out[1] = (float)(c < 1.0 ? c : 1.0);
  }
}

// --------------------------------------------------------------- SGD (+momentum, NGD tail)
__global__ __launch_bounds__(kOB) void sgd_kernel(const opt::SgdArgs args, long n4) {
  if (opt::SgdOp::skipped(args)) { opt::SgdOp::on_skip(args, n4 * 4); return; }
  // (device [lr, momentum] in args.lr_dev: a captured HIP graph follows the schedules)
  const opt::SgdOp op(args);
  const bool mom = op.momentum != 0.f;
  float4* p4 = reinterpret_cast<float4*>(args.p);
  float4* g4 = reinterpret_cast<float4*>(args.g);
  float4* b4 = reinterpret_cast<float4*>(args.buf);
  for (long i = (long)blockIdx.x * kOB + threadIdx.x; i < n4; i += (long)gridDim.x * kOB) {
    float4 pv = p4[i];
    const float4 gv = g4[i];
    float4 bv = (mom && !args.first) ? b4[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    pv.x = op.rule(pv.x, gv.x, bv.x);
    pv.y = op.rule(pv.y, gv.y, bv.y);
    pv.z = op.rule(pv.z, gv.z, bv.z);
    pv.w = op.rule(pv.w, gv.w, bv.w);
    if (mom) b4[i] = bv;
    p4[i] = pv;
    if (args.shadow) store_shadow(args.shadow, i * 4, pv);
    if (args.zero_grad) g4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// --------------------------------------------------------------- MADGRAD (optim_ops.h MadOp)
__global__ __launch_bounds__(kOB) void madgrad_kernel(const opt::MadArgs args, long n) {
  if (opt::MadOp::skipped(args)) { opt::MadOp::on_skip(args, n); return; }
  const opt::MadOp op(args);
  for (long i = (long)blockIdx.x * kOB + threadIdx.x; i < n; i += (long)gridDim.x * kOB) op(i);
}

// --------------------------------------------------------------- MirrorMADGRAD
// z <- z - lamb * g / rms_{k+1};  p <- (1-ck) p + ck z   (rms == 0 -> step skipped)
__global__ __launch_bounds__(kOB) void mirror_madgrad_kernel(float* __restrict__ p, float* __restrict__ g,
                                                             float* __restrict__ gss, float* __restrict__ z,
                                                             bf16* __restrict__ shadow, long n, float lr, float momentum,
                                                             float wd, float eps, int decouple, long k,
                                                             int* __restrict__ kskip, const float* __restrict__ gsc,
                                                             const int* __restrict__ found_inf, int zero_grad) {
  if (skip_step(found_inf)) { count_skip(kskip); skip_zero(g, n, zero_grad); return; }
  const float c = gscale(gsc);
  const float lr_e = lr + eps;
  const float lamb = lr_e * sqrtf((float)(applied_k(k, kskip) + 1));
  const float ck = 1.f - momentum;
  for (long i = (long)blockIdx.x * kOB + threadIdx.x; i < n; i += (long)gridDim.x * kOB) {
    float pv = p[i], gv = g[i] * c;
    if (wd != 0.f && !decouple) gv += wd * pv;
    float q = fmaf(lamb * gv, gv, gss[i]);
    float rms = cbrtf(q) + eps;
    float zv = z[i];
    if (rms > 0.f) zv -= lamb * gv / rms;
    if (wd != 0.f && decouple) zv -= lr_e * wd * zv;
    pv = (1.f - ck) * pv + ck * zv;
    p[i] = pv;
    gss[i] = q;
    z[i] = zv;
    if (shadow) shadow[i] = __float2bfloat16(pv);
    if (zero_grad) g[i] = 0.f;
  }
}

// --------------------------------------------------------------- Adam / AdamW (extra)
__global__ __launch_bounds__(kOB) void adam_kernel(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                                                   float* __restrict__ v, bf16* __restrict__ shadow, long n, float lr,
                                                   float b1, float b2, float eps, float wd, int adamw, long step,
                                                   int* __restrict__ kskip, const float* __restrict__ gsc,
                                                   const int* __restrict__ found_inf, int zero_grad) {
  if (skip_step(found_inf)) { count_skip(kskip); skip_zero(g, n, zero_grad); return; }
  const float c = gscale(gsc);
  const float st = (float)applied_k(step, kskip);
  const float bc1 = 1.f - powf(b1, st), bc2 = 1.f - powf(b2, st);
  for (long i = (long)blockIdx.x * kOB + threadIdx.x; i < n; i += (long)gridDim.x * kOB) {
    float pv = p[i], gv = g[i] * c;
    if (wd != 0.f) {
      if (adamw) pv -= lr * wd * pv;
      else gv += wd * pv;
    }
    float mv = b1 * m[i] + (1.f - b1) * gv;
    float vv = b2 * v[i] + (1.f - b2) * gv * gv;
    m[i] = mv;
    v[i] = vv;
    pv -= lr * (mv / bc1) / (sqrtf(vv / bc2) + eps);
    p[i] = pv;
    if (shadow) shadow[i] = __float2bfloat16(pv);
    if (zero_grad) g[i] = 0.f;
  }
}

// --------------------------------------------------------------- f32 -> bf16 cast
__global__ __launch_bounds__(kOB) void cast_bf16_kernel(const float* __restrict__ x, bf16* __restrict__ y, long n4) {
  const float4* x4 = reinterpret_cast<const float4*>(x);
  for (long i = (long)blockIdx.x * kOB + threadIdx.x; i < n4; i += (long)gridDim.x * kOB) store_shadow(y, i * 4, x4[i]);
}

// --------------------------------------------------------------- launchers
void grad_sumsq(uint64_t g, long n, uint64_t inv_scale, int unscale, uint64_t part, int nb, uint64_t found_inf,
                uint64_t stream) {
  FDT_CHECK(n % 4 == 0, "flat buffer must be padded to a multiple of 4");
  grad_sumsq_kernel<<<nb, kOB, 0, as_stream(stream)>>>(P<float>(g), n / 4, P<const float>(inv_scale), unscale,
                                                        P<float>(part), P<int>(found_inf));
  FDT_LAUNCH_CHECK();
}

void grad_norm_finalize(uint64_t part, int nb, float max_norm, uint64_t out, uint64_t total, int phase,
                        uint64_t stream) {
  FDT_CHECK(phase >= 0 && phase <= 2 && (phase == 0 || total != 0), "grad_norm_finalize: phase / total");
  grad_norm_finalize_kernel<<<1, 256, 0, as_stream(stream)>>>(P<const float>(part), nb, max_norm, P<float>(out),
                                                             P<double>(total), phase);
  FDT_LAUNCH_CHECK();
}

void sgd_step(uint64_t p, uint64_t g, uint64_t buf, uint64_t shadow, long n, float lr, float momentum, float dampening,
              float wd, int nesterov, int first, uint64_t gsc, uint64_t found_inf, int zero_grad, uint64_t lr_dev,
              uint64_t stream) {
  FDT_CHECK(n % 4 == 0, "flat buffer must be padded to a multiple of 4");
  FDT_CHECK(momentum == 0.f || buf != 0, "momentum buffer required");
  const opt::SgdArgs a{P<float>(p), P<float>(g), P<float>(buf), P<bf16>(shadow), lr, momentum, dampening, wd,
                       nesterov, first, P<const float>(gsc), P<const int>(found_inf), zero_grad,
                       P<const float>(lr_dev)};
  sgd_kernel<<<opt_grid(n / 4), kOB, 0, as_stream(stream)>>>(a, n / 4);
  FDT_LAUNCH_CHECK();
}

void madgrad_step(uint64_t p, uint64_t g, uint64_t gss, uint64_t s, uint64_t x0, uint64_t shadow, long n, float lr,
                  float momentum, float wd, float eps, int decouple, long k, uint64_t kskip, uint64_t gsc,
                  uint64_t found_inf, int zero_grad, uint64_t stream) {
  FDT_CHECK(n % 4 == 0, "flat buffer must be padded to a multiple of 4");
  FDT_CHECK(momentum == 0.f || x0 != 0, "x0 buffer required with momentum");
  const opt::MadArgs a{P<float>(p), P<float>(g), P<float>(gss), P<float>(s), P<float>(x0), P<bf16>(shadow),
                       lr, momentum, wd, eps, decouple, k, P<int>(kskip), P<const float>(gsc),
                       P<const int>(found_inf), zero_grad};
  madgrad_kernel<<<opt_grid(n / 4), kOB, 0, as_stream(stream)>>>(a, n);
  FDT_LAUNCH_CHECK();
}

void mirror_madgrad_step(uint64_t p, uint64_t g, uint64_t gss, uint64_t z, uint64_t shadow, long n, float lr,
                         float momentum, float wd, float eps, int decouple, long k, uint64_t kskip, uint64_t gsc,
                         uint64_t found_inf, int zero_grad, uint64_t stream) {
  mirror_madgrad_kernel<<<opt_grid(n), kOB, 0, as_stream(stream)>>>(P<float>(p), P<float>(g), P<float>(gss), P<float>(z),
                                                                     P<bf16>(shadow), n, lr, momentum, wd, eps, decouple,
                                                                     k, P<int>(kskip), P<const float>(gsc),
                                                                     P<const int>(found_inf), zero_grad);
  FDT_LAUNCH_CHECK();
}

void adam_step(uint64_t p, uint64_t g, uint64_t m, uint64_t v, uint64_t shadow, long n, float lr, float b1, float b2,
               float eps, float wd, int adamw, long step, uint64_t kskip, uint64_t gsc, uint64_t found_inf,
               int zero_grad, uint64_t stream) {
  adam_kernel<<<opt_grid(n), kOB, 0, as_stream(stream)>>>(P<float>(p), P<float>(g), P<float>(m), P<float>(v),
                                                           P<bf16>(shadow), n, lr, b1, b2, eps, wd, adamw, step,
                                                           P<int>(kskip), P<const float>(gsc), P<const int>(found_inf), zero_grad);
  FDT_LAUNCH_CHECK();
}

void cast_bf16(uint64_t x, uint64_t y, long n, uint64_t stream) {
  FDT_CHECK(n % 4 == 0, "n % 4");
  cast_bf16_kernel<<<opt_grid(n / 4), kOB, 0, as_stream(stream)>>>(P<const float>(x), P<bf16>(y), n / 4);
  FDT_LAUNCH_CHECK();
}

}  // namespace fdt
