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
#include <vector>

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

// (s, t) of channel c from its fp64 sums; ``write``: also the unit's outputs (out_s / out_t,
// saved mean / aux, running statistics, num_batches_tracked) -- exactly one thread per channel
// may write them
__device__ __forceinline__ void bn_finalize_st(const FinArgs& f, int c, double S, double Q, float& s_out,
                                               float& t_out, bool write) {
  double sc, tt, mean, aux;
  if (f.mode == 0) {
    mean = S / f.count;
    double var = (Q - S * mean) / (f.count - 1.0);
    if (var < 0.0) var = 0.0;
    aux = sqrt(var);
    sc = 1.0 / (aux + (double)f.eps);
    tt = -mean * sc;
  } else if (f.mode == 1) {
    mean = S / f.count;
    double m2 = Q - S * mean;
    if (m2 < 0.0) m2 = 0.0;
    const double var_b = m2 / f.count;
    const double var_u = f.count > 1.0 ? m2 / (f.count - 1.0) : var_b;
    aux = 1.0 / sqrt(var_b + (double)f.eps);
    const double g = f.gamma ? (double)f.gamma[c] : 1.0, b = f.beta ? (double)f.beta[c] : 0.0;
    sc = g * aux;
    tt = b - mean * g * aux;
    if (write && f.run_mean) {
      f.run_mean[c] = (float)((1.0 - f.momentum) * f.run_mean[c] + f.momentum * mean);
      f.run_var[c] = (float)((1.0 - f.momentum) * f.run_var[c] + f.momentum * var_u);
    }
    if (write && f.nbt && c == 0) f.nbt[0] += 1;
  } else {
    mean = f.run_mean[c];
    aux = 1.0 / sqrt((double)f.run_var[c] + (double)f.eps);
    const double g = f.gamma ? (double)f.gamma[c] : 1.0, b = f.beta ? (double)f.beta[c] : 0.0;
    sc = g * aux;
    tt = b - mean * g * aux;
  }
  s_out = (float)sc;
  t_out = (float)tt;
  if (write) {
    f.out_s[c] = s_out;
    f.out_t[c] = t_out;
    f.save_mean[c] = (float)mean;
    f.save_aux[c] = (float)aux;
  }
}

__device__ __forceinline__ void bn_finalize_channel(const FinArgs& f, int c, double S, double Q) {
  float s, t;
  bn_finalize_st(f, c, S, Q, s, t, true);
}

// Lazy batch statistics (FusedConvBN units, mode 0): the producer's slot rows and the unit's
// outputs live in ONE region  [rows][2][C] slots | s[C] | t[C] | save_mean[C] | save_aux[C]
// (C = the unit's channels); the slots are finalised by the unit's CONSUMER while staging its
// own inputs (the channels it needs; rows summed in fp64 in a fixed order) instead of by a
// standalone finalize launch between the two, and the consumer's workgroup 0 also writes the
// four output vectors (the backward reads them).  base == nullptr: not lazy (the consumer reads
// the finalised s / t).  Compact on purpose: it travels in the conv kernels' arguments (SGPRs).
struct LazyStats {
  float* base;
  int rows;
  float eps;
  float count;  // rows of the producer's output (N*H*W), exact in fp32 up to 2^24
};

// (s, t) of channel c; ``write``: also the four output vectors (one writer per channel)
__device__ __forceinline__ void lazy_finish(const LazyStats& L, int C, int c, double S, double Q, float& s, float& t,
                                            bool write) {
  const double n = (double)L.count;
  const double mean = S / n;
  double var = (Q - S * mean) / (n - 1.0);
  if (var < 0.0) var = 0.0;
  const float sd = (float)sqrt(var);
  s = 1.f / (sd + L.eps);  // unbiased sd + eps (resnet.py:75-100), fp32 reciprocal
  t = (float)(-mean) * s;
  if (write) {
    float* o = L.base + (long)L.rows * 2 * C;
    o[c] = s;
    o[C + c] = t;
    o[2 * C + c] = (float)mean;
    o[3 * C + c] = sd;
  }
}

__device__ __forceinline__ void lazy_st(const LazyStats& L, int C, int c, float& s, float& t, bool write) {
  double S = 0.0, Q = 0.0;
  const float* p = L.base;
  for (int r = 0; r < L.rows; ++r) {
    S += (double)p[(long)(2 * r) * C + c];
    Q += (double)p[(long)(2 * r + 1) * C + c];
  }
  lazy_finish(L, C, c, S, Q, s, t, write);
}

// every channel of L into s_out[C] / t_out[C] (LDS) by NT threads: four channels per thread and
// pass, every slot-row load of a pass issued before the sums
template <int NT>
__device__ __forceinline__ void lazy_fill(const LazyStats& L, int C, float* s_out, float* t_out, int tid, bool w0) {
  for (int c0 = tid; c0 < C; c0 += 4 * NT) {
    double S[4] = {0.0, 0.0, 0.0, 0.0}, Q[4] = {0.0, 0.0, 0.0, 0.0};
    for (int r = 0; r < L.rows; ++r) {
      const float* p = L.base + (long)(2 * r) * C;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int c = c0 + NT * k;
        if (c < C) {
          S[k] += (double)p[c];
          Q[k] += (double)p[C + c];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = c0 + NT * k;
      if (c < C) {
        float sv, tv;
        lazy_finish(L, C, c, S[k], Q[k], sv, tv, w0);
        s_out[c] = sv;
        t_out[c] = tv;
      }
    }
  }
}

// host: LazyStats from the Python launch lists -- ptr = [region base], val = [rows, eps, count];
// empty lists = not lazy
inline LazyStats make_lazy(const std::vector<uint64_t>& ptr, const std::vector<double>& val) {
  LazyStats L{};
  if (ptr.empty()) return L;
  FDT_CHECK(ptr.size() == 1 && val.size() == 3, "lazy statistics: [base] + [rows, eps, count]");
  L.base = P<float>(ptr[0]);
  L.rows = (int)val[0];
  L.eps = (float)val[1];
  L.count = (float)val[2];
  FDT_CHECK(L.base != nullptr && L.rows >= 1 && L.count > 1.f && val[2] < 16777216.0, "lazy statistics: values");
  return L;
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
