// GPU batch augmentation for CIFAR-style uint8 images (replaces the reference's
// per-sample TorchScript transforms in CPU workers, resnet50_test.py:301-318, K17).
//
// The whole uint8 dataset stays resident in HBM (CIFAR-10 train = 153 MB of 288 GB);
// a batch is a list of sample indices.  One pass per batch does: gather by index ->
// /255 -> random crop with zero padding -> random horizontal flip -> per-channel
// normalise -> bf16/f32 store in NHWC (optionally zero-padded channels for the conv
// kernels) or NCHW.  Per-sample random parameters come from a counter-based hash of
// (seed, counter, sample) read from device memory, so the kernel is graph-replayable
// and needs no host RNG.
//
// Transform order (the reference permutes crop / flip / normalise once per run,
// resnet50_test.py:304-309): flip commutes with both other transforms in distribution
// (a mirrored uniform crop offset is again uniform), so the only observable difference is
// whether normalisation runs before the zero-padded crop: then padding is 0 in normalised
// space (pad_norm = 1) instead of raw 0 -> -mean/std (pad_norm = 0, torchvision's
// crop -> flip -> normalise order).
#include "common.h"

namespace fdt {

template <typename TO>
__global__ __launch_bounds__(256) void augment_kernel(const uint8_t* __restrict__ src, const int* __restrict__ idx,
                                                      const int* __restrict__ labels_src, int* __restrict__ labels_out,
                                                      TO* __restrict__ out, int B, int H, int W, int C, int Cout,
                                                      int pad, int do_flip, const long long* __restrict__ rng,
                                                      float m0, float m1, float m2, float is0, float is1, float is2,
                                                      int nchw, int pad_norm) {
  const long total = (long)B * H * W;
  const uint64_t seed = rng ? (uint64_t)rng[0] : 0ull, ctr = rng ? (uint64_t)rng[1] : 0ull;
  for (long p = (long)blockIdx.x * blockDim.x + threadIdx.x; p < total; p += (long)gridDim.x * blockDim.x) {
    const int b = (int)(p / (H * W));
    const int rem = (int)(p % (H * W));
    const int y = rem / W, x = rem % W;
    const uint64_t h = mix64(seed ^ mix64(ctr * 0x100000001B3ull + (uint64_t)b));
    const int span = 2 * pad + 1;
    const int dy = pad > 0 ? (int)(h % span) : pad;
    const int dx = pad > 0 ? (int)((h >> 16) % span) : pad;
    const bool flip = do_flip && ((h >> 40) & 1ull);
    const int xs0 = flip ? (W - 1 - x) : x;
    const int sy = y + dy - pad, sx = xs0 + dx - pad;
    const int n = idx ? idx[b] : b;
    if (labels_out && rem == 0) labels_out[b] = labels_src[n];
    const bool inside = sy >= 0 && sy < H && sx >= 0 && sx < W;
    const uint8_t* px = src + (((long)n * H + (inside ? sy : 0)) * W + (inside ? sx : 0)) * C;
    const float mean[3] = {m0, m1, m2}, istd[3] = {is0, is1, is2};
    for (int c = 0; c < Cout; ++c) {
      float v = 0.f;
      if (c < C) {
        const float raw = inside ? (float)px[c] * (1.f / 255.f) : 0.f;
        v = (inside || !pad_norm) ? (raw - mean[c < 3 ? c : 2]) * istd[c < 3 ? c : 2] : 0.f;
      }
      long o = nchw ? (((long)b * Cout + c) * H + y) * W + x : p * Cout + c;
      out[o] = from_f<TO>(v);
    }
  }
}

void augment(uint64_t src, uint64_t idx, uint64_t labels_src, uint64_t labels_out, uint64_t out, int B, int H, int W,
             int C, int Cout, int pad, int do_flip, uint64_t rng, float m0, float m1, float m2, float s0, float s1,
             float s2, int nchw, int pad_norm, int dt_out, uint64_t stream) {
  FDT_CHECK(C <= 3 && Cout >= C, "augment: C <= 3 and Cout >= C");
  long total = (long)B * H * W;
  if (total == 0) return;
  int g = (int)((total + 255) / 256);
  if (g > 4096) g = 4096;
  if (dt_out == kBF16) {
    augment_kernel<bf16><<<g, 256, 0, as_stream(stream)>>>(P<const uint8_t>(src), P<const int>(idx),
                                                          P<const int>(labels_src), P<int>(labels_out), P<bf16>(out), B,
                                                          H, W, C, Cout, pad, do_flip, P<const long long>(rng), m0, m1,
                                                          m2, 1.f / s0, 1.f / s1, 1.f / s2, nchw, pad_norm);
  } else if (dt_out == kF32) {
    augment_kernel<float><<<g, 256, 0, as_stream(stream)>>>(P<const uint8_t>(src), P<const int>(idx),
                                                           P<const int>(labels_src), P<int>(labels_out), P<float>(out),
                                                           B, H, W, C, Cout, pad, do_flip, P<const long long>(rng), m0,
                                                           m1, m2, 1.f / s0, 1.f / s1, 1.f / s2, nchw, pad_norm);
  } else {
    throw std::runtime_error("augment: output dtype must be f32 or bf16");
  }
  FDT_LAUNCH_CHECK();
}

// rng[1] += 1 (advance the per-step counter on the device; graph-replay safe)
__global__ void rng_advance_kernel(long long* rng) { rng[1] += 1; }
void rng_advance(uint64_t rng, uint64_t stream) {
  rng_advance_kernel<<<1, 1, 0, as_stream(stream)>>>(P<long long>(rng));
  FDT_LAUNCH_CHECK();
}

}  // namespace fdt
