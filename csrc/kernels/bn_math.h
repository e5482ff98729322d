// Per-channel batch-norm finalisation math shared by the standalone finalize kernel
// (bn_kernels.hip) and any kernel that finalises statistics in its own epilogue,
// so both produce bit-identical (s, t) for the same fp64 sums.
//
// mode 0: FusedConvBN (unbiased var, s = 1/(sqrt(var)+eps), no affine)   resnet.py:75-100
// mode 1: BatchNorm2d train (biased var + eps, affine, running stats with momentum and the
//         unbiased var)
// mode 2: BatchNorm2d eval  (running stats, affine)
// save_mean[c], save_aux[c]: mode 0 -> sd ; modes 1/2 -> invstd
#pragma once
#include "common.h"

namespace fdt {

struct FinArgs {
  int mode;
  float eps;
  float momentum;
  double count;
  const float* gamma;
  const float* beta;
  float* run_mean;
  float* run_var;
  long long* nbt;
  float* out_s;
  float* out_t;
  float* save_mean;
  float* save_aux;
};

__device__ __forceinline__ void bn_finalize_channel(const FinArgs& f, int c, double S, double Q) {
  if (f.mode == 0) {
    const double mean = S / f.count;
    double var = (Q - S * mean) / (f.count - 1.0);
    if (var < 0.0) var = 0.0;
    const double sd = sqrt(var);
    const double sc = 1.0 / (sd + (double)f.eps);
    f.out_s[c] = (float)sc;
    f.out_t[c] = (float)(-mean * sc);
    f.save_mean[c] = (float)mean;
    f.save_aux[c] = (float)sd;
  } else if (f.mode == 1) {
    const double mean = S / f.count;
    double m2 = Q - S * mean;
    if (m2 < 0.0) m2 = 0.0;
    const double var_b = m2 / f.count;
    const double var_u = f.count > 1.0 ? m2 / (f.count - 1.0) : var_b;
    const double inv = 1.0 / sqrt(var_b + (double)f.eps);
    const double g = f.gamma ? (double)f.gamma[c] : 1.0, b = f.beta ? (double)f.beta[c] : 0.0;
    f.out_s[c] = (float)(g * inv);
    f.out_t[c] = (float)(b - mean * g * inv);
    f.save_mean[c] = (float)mean;
    f.save_aux[c] = (float)inv;
    if (f.run_mean) {
      f.run_mean[c] = (float)((1.0 - f.momentum) * f.run_mean[c] + f.momentum * mean);
      f.run_var[c] = (float)((1.0 - f.momentum) * f.run_var[c] + f.momentum * var_u);
    }
    if (f.nbt && c == 0) f.nbt[0] += 1;
  } else {
    const double mean = f.run_mean[c];
    const double inv = 1.0 / sqrt((double)f.run_var[c] + (double)f.eps);
    const double g = f.gamma ? (double)f.gamma[c] : 1.0, b = f.beta ? (double)f.beta[c] : 0.0;
    f.out_s[c] = (float)(g * inv);
    f.out_t[c] = (float)(b - mean * g * inv);
    f.save_mean[c] = (float)mean;
    f.save_aux[c] = (float)inv;
  }
}

// BN-backward coefficients from the per-channel reductions (g_s, g_t) of dL/dy; see the mode
// table above stats_bwd_coef_kernel (bn_kernels.hip).
struct CoefArgs {
  int mode;
  float eps;
  double count;
  const float* save_mean;
  const float* save_aux;
  const float* gamma;
  float* alpha;
  float* beta;
  float* ggamma;
  float* gbeta;
};

__device__ __forceinline__ void bwd_coef_one(const CoefArgs& a, int c, double g_s, double g_t) {
  const double mean = a.save_mean[c], aux = a.save_aux[c];
  const double count = a.count;
  if (a.mode == 0) {
    const double sd = aux;
    const double s = 1.0 / (sd + (double)a.eps);
    const double b = sd > 0.0 ? -(g_s - mean * g_t) * s * s / ((count - 1.0) * sd) : 0.0;
    a.beta[c] = (float)b;
    a.alpha[c] = (float)(-b * mean - g_t * s / count);
  } else {
    const double inv = aux;
    const double g = a.gamma ? (double)a.gamma[c] : 1.0;
    const double s = g * inv;
    if (a.mode == 1) {
      const double b = -(g_s - mean * g_t) * g * inv * inv * inv / count;
      a.beta[c] = (float)b;
      a.alpha[c] = (float)(-b * mean - g_t * s / count);
    } else {
      a.beta[c] = 0.f;
      a.alpha[c] = 0.f;
    }
    // accumulate (+=) into the parameter gradients (flat gradient views)
    if (a.ggamma) a.ggamma[c] += (float)((g_s - mean * g_t) * inv);
    if (a.gbeta) a.gbeta[c] += (float)g_t;
  }
}

}  // namespace fdt
