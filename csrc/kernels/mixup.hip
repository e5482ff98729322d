// Mixup kernels (reference resnet50_test.py:355-457, transformer.py:71-80).
//  * mixup_fwd:  out[i] = lam[i]*x[i] + (1-lam[i])*x[perm[i]]   (permuted gather + lerp)
//  * mixup_bwd:  gx[i] = lam[i]*g[i] + (1-lam[inv[i]])*g[inv[i]]  (inverse-permutation
//                gather: no atomics, deterministic); optional per-sample
//                dlam[i] = sum_j g[i,j]*(x[i,j]-x[perm[i],j]) for the learnable meta-mixup.
//  * mixup_ce_fwd: fused log-softmax cross entropy against two targets with per-sample
//                lambda: loss, dlogits and dloss/dlam in one single-block kernel (the
//                logits are tiny: B x 10 / B x 4), no host sync.
#include "common.h"

namespace fdt {

template <typename T>
__global__ __launch_bounds__(256) void mixup_fwd_kernel(const T* __restrict__ x, const int* __restrict__ perm,
                                                        const float* __restrict__ lam, T* __restrict__ out, long inner) {
  const int i = blockIdx.y;
  const int j = perm[i];
  const float l = lam[i];
  const T* xi = x + (long)i * inner;
  const T* xj = x + (long)j * inner;
  T* o = out + (long)i * inner;
  if (inner % 8 == 0) {
    for (long v = (long)blockIdx.x * blockDim.x + threadIdx.x; v < inner / 8; v += (long)gridDim.x * blockDim.x) {
      float a[8], b[8];
      Vec8<T>::load(xi + v * 8, a);
      Vec8<T>::load(xj + v * 8, b);
#pragma unroll
      for (int k = 0; k < 8; ++k) a[k] = l * a[k] + (1.f - l) * b[k];
      Vec8<T>::store(o + v * 8, a);
    }
  } else {
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < inner; e += (long)gridDim.x * blockDim.x)
      o[e] = from_f<T>(l * to_f(xi[e]) + (1.f - l) * to_f(xj[e]));
  }
}

template <typename T>
__global__ __launch_bounds__(256) void mixup_bwd_kernel(const T* __restrict__ g, const T* __restrict__ x,
                                                        const int* __restrict__ perm, const int* __restrict__ inv,
                                                        const float* __restrict__ lam, T* __restrict__ gx,
                                                        float* __restrict__ dlam, long inner) {
  __shared__ float sm[4];
  const int i = blockIdx.x;
  const int ii = inv[i], pj = perm[i];
  const float li = lam[i], lk = 1.f - lam[ii];
  const T* gi = g + (long)i * inner;
  const T* gk = g + (long)ii * inner;
  const T* xi = x + (long)i * inner;
  const T* xp = x + (long)pj * inner;
  T* o = gx + (long)i * inner;
  float acc = 0.f;
  for (long e = threadIdx.x; e < inner; e += blockDim.x) {
    float gv = to_f(gi[e]);
    o[e] = from_f<T>(li * gv + lk * to_f(gk[e]));
    if (dlam) acc += gv * (to_f(xi[e]) - to_f(xp[e]));
  }
  if (dlam) {
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) dlam[i] = sm[0] + sm[1] + sm[2] + sm[3];
  }
}

// One row per THREAD when C <= 64 (CIFAR: 10 classes -- a wave per row would idle 54 of
// its 64 lanes and serialise B/16 rows per wave), one row per WAVE otherwise.
template <typename T, typename L, bool ROW_PER_THREAD>
__global__ __launch_bounds__(1024) void mixup_ce_kernel(const T* __restrict__ logits, const L* __restrict__ ya,
                                                        const L* __restrict__ yb, const float* __restrict__ lam,
                                                        float lam_s, float* __restrict__ loss, T* __restrict__ glog,
                                                        float* __restrict__ dlam, float* __restrict__ meter, int B,
                                                        int C) {
  // meter (optional): training accumulators [loss sum, lambda-weighted correct, samples]
  // updated in place (one block: plain read-modify-write) -- the reference's per-batch
  // accuracy bookkeeping (resnet50_test.py:550-558) without a dozen separate launches.
  __shared__ float sm[16], smc[16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  float tot = 0.f, corr = 0.f;
  const float invB = 1.f / (float)B;
  if constexpr (ROW_PER_THREAD) {
    for (int r = threadIdx.x; r < B; r += blockDim.x) {
      const T* row = logits + (long)r * C;
      // (the row is re-read from L1 per pass: a runtime-indexed register array would spill)
      float mx = -INFINITY;
      int am = 0;
      for (int c = 0; c < C; ++c) {
        const float x = to_f(row[c]);
        if (x > mx) { mx = x; am = c; }  // strict >: first occurrence (torch.argmax)
      }
      float se = 0.f;
      for (int c = 0; c < C; ++c) se += __expf(to_f(row[c]) - mx);
      const float lse = mx + __logf(se);
      const int a = (int)ya[r], b = (int)yb[r];
      const float l = lam ? lam[r] : lam_s;
      const float cea = lse - to_f(row[a]), ceb = lse - to_f(row[b]);
      for (int c = 0; c < C; ++c) {
        const float p = __expf(to_f(row[c]) - lse);
        const float t = (c == a ? l : 0.f) + (c == b ? 1.f - l : 0.f);
        glog[(long)r * C + c] = from_f<T>((p - t) * invB);
      }
      tot += l * cea + (1.f - l) * ceb;
      if (dlam) dlam[r] = (cea - ceb) * invB;
      corr += (am == a ? l : 0.f) + (am == b ? 1.f - l : 0.f);
    }
    tot = wave_sum(tot);
    corr = wave_sum(corr);
  } else {
    for (int r = w; r < B; r += nw) {
      const T* row = logits + (long)r * C;
      float mx = -INFINITY;
      for (int c = lane; c < C; c += 64) mx = fmaxf(mx, to_f(row[c]));
      mx = wave_max(mx);
      float se = 0.f;
      for (int c = lane; c < C; c += 64) se += __expf(to_f(row[c]) - mx);
      se = wave_sum(se);
      const float lse = mx + __logf(se);
      const int a = (int)ya[r], b = (int)yb[r];
      int am = C;  // argmax, first occurrence (torch.argmax)
      if (meter) {
        for (int c = lane; c < C; c += 64)
          if (to_f(row[c]) == mx) { am = c; break; }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) am = min(am, __shfl_xor(am, o, 64));
      }
      const float l = lam ? lam[r] : lam_s;
      const float cea = lse - to_f(row[a]), ceb = lse - to_f(row[b]);
      for (int c = lane; c < C; c += 64) {
        float p = __expf(to_f(row[c]) - lse);
        float t = (c == a ? l : 0.f) + (c == b ? 1.f - l : 0.f);
        glog[(long)r * C + c] = from_f<T>((p - t) * invB);
      }
      if (lane == 0) {
        tot += l * cea + (1.f - l) * ceb;
        if (dlam) dlam[r] = (cea - ceb) * invB;
        corr += (am == a ? l : 0.f) + (am == b ? 1.f - l : 0.f);
      }
    }
  }
  if (lane == 0) { sm[w] = tot; smc[w] = corr; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f, cc = 0.f;
    for (int k = 0; k < nw; ++k) { t += sm[k]; cc += smc[k]; }
    *loss = t * invB;
    if (meter) {
      meter[0] += t * invB;
      meter[1] += cc;
      meter[2] += (float)B;
    }
  }
}

#define DISPATCH_T(dt, ...)                                     \
  switch (dt) {                                                 \
    case kF32: { using T = float; __VA_ARGS__; break; }         \
    case kBF16: { using T = bf16; __VA_ARGS__; break; }         \
    case kF16: { using T = f16; __VA_ARGS__; break; }           \
    default: throw std::runtime_error("bad dtype code");        \
  }

void mixup_fwd(uint64_t x, uint64_t perm, uint64_t lam, uint64_t out, int b, long inner, int dt, uint64_t stream) {
  long work = inner % 8 == 0 ? inner / 8 : inner;
  int gx = (int)((work + 255) / 256);
  if (gx > 64) gx = 64;
  dim3 grid(gx, b);
  DISPATCH_T(dt, {
    mixup_fwd_kernel<T><<<grid, 256, 0, as_stream(stream)>>>(P<const T>(x), P<const int>(perm), P<const float>(lam),
                                                            P<T>(out), inner);
  });
  FDT_LAUNCH_CHECK();
}

void mixup_bwd(uint64_t g, uint64_t x, uint64_t perm, uint64_t inv, uint64_t lam, uint64_t gx, uint64_t dlam, int b,
               long inner, int dt, uint64_t stream) {
  DISPATCH_T(dt, {
    mixup_bwd_kernel<T><<<b, 256, 0, as_stream(stream)>>>(P<const T>(g), P<const T>(x), P<const int>(perm),
                                                         P<const int>(inv), P<const float>(lam), P<T>(gx),
                                                         P<float>(dlam), inner);
  });
  FDT_LAUNCH_CHECK();
}

void mixup_ce_fwd(uint64_t logits, uint64_t ya, uint64_t yb, uint64_t lam, float lam_s, uint64_t loss, uint64_t glog,
                  uint64_t dlam, uint64_t meter, int B, int C, int dt, int labels64, uint64_t stream) {
  auto go = [&](auto tag_t, auto tag_l) {
    using T = decltype(tag_t);
    using L = decltype(tag_l);
    if (C <= 64)
      mixup_ce_kernel<T, L, true><<<1, 1024, 0, as_stream(stream)>>>(P<const T>(logits), P<const L>(ya), P<const L>(yb),
                                                                     P<const float>(lam), lam_s, P<float>(loss), P<T>(glog),
                                                                     P<float>(dlam), P<float>(meter), B, C);
    else
      mixup_ce_kernel<T, L, false><<<1, 1024, 0, as_stream(stream)>>>(P<const T>(logits), P<const L>(ya), P<const L>(yb),
                                                                      P<const float>(lam), lam_s, P<float>(loss), P<T>(glog),
                                                                      P<float>(dlam), P<float>(meter), B, C);
  };
  DISPATCH_T(dt, {
    if (labels64) go(T{}, int64_t{});
    else go(T{}, int{});
  });
  FDT_LAUNCH_CHECK();
}

// One workgroup: a uniformly random permutation of b <= 1024 samples (bitonic sort in LDS of
// 64-bit counter-hash keys -- distinct, the hash is a bijection), the permuted labels and the
// per-sample lambda vector: replaces randperm's sort passes, the int32 cast, the label gather
// and the lambda fill of an input-mixup step (reference resnet50_test.py:355-376).
__global__ __launch_bounds__(1024) void mixup_prep_kernel(const int64_t* __restrict__ y, int b, float lam,
                                                          uint64_t seed, int* __restrict__ perm,
                                                          int64_t* __restrict__ yb, float* __restrict__ lam_vec) {
  __shared__ uint64_t key[1024];
  __shared__ int idx[1024];
  int n = 1;
  while (n < b) n <<= 1;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    key[i] = i < b ? mix64(seed + (uint64_t)i * 0xD1B54A32D192ED03ull) : ~0ull;
    idx[i] = i;
  }
  __syncthreads();
  for (int k = 2; k <= n; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int p = i ^ j;
        if (p > i) {
          const bool up = (i & k) == 0;
          const uint64_t a = key[i], c = key[p];
          if ((a > c) == up) {
            key[i] = c;
            key[p] = a;
            const int t = idx[i];
            idx[i] = idx[p];
            idx[p] = t;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int i = threadIdx.x; i < b; i += blockDim.x) {
    const int j = idx[i];
    perm[i] = j;
    yb[i] = y[j];
    lam_vec[i] = lam;
  }
}

void mixup_prep(uint64_t y, int b, float lam, uint64_t seed, uint64_t perm, uint64_t yb, uint64_t lam_vec,
                uint64_t stream) {
  FDT_CHECK(b >= 1 && b <= 1024, "mixup_prep: 1 <= batch <= 1024");
  mixup_prep_kernel<<<1, 1024, 0, as_stream(stream)>>>(P<const int64_t>(y), b, lam, seed, P<int>(perm),
                                                       P<int64_t>(yb), P<float>(lam_vec));
  FDT_LAUNCH_CHECK();
}

}  // namespace fdt
