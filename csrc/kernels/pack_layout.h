// Packed bf16 weight layouts of the implicit-GEMM convolutions, written from a bf16 LDS image of
// one 32 (co) x 64 (ci) x T block (img[(co * T + t) * kPackLd + ci]):
//   forward  wf[co][t][ci]  (Cxp-padded rows; the conv B operand, K = (t, ci) contiguous)
//   dgrad    wd[ci][t][co]  (the data-gradient B operand, K = (t, co) contiguous)
// Shared by the standalone repack (conv_wgrad.hip pack_weights_kernel, which fills the image from
// the fp32 OIHW master weights) and the optimizer's fused update-and-pack (optim_pack.hip, which
// fills it with the freshly updated weights).  16-B stores of 8 consecutive bf16 per lane
// (2-byte stores left the repack at ~1.6 TB/s); row stride 66 elements so the co-strided reads
// of the dgrad pass hit distinct banks.
#pragma once
#include "common.h"

namespace fdt {
namespace pack {

constexpr int kCo = 32;
constexpr int kT = 64;  // ci per block
constexpr int kLd = kT + 2;
constexpr int kMaxTaps = 9;

__device__ __forceinline__ uint32_t bf16_bits(bf16 v) { return (uint32_t)(*reinterpret_cast<uint16_t*>(&v)); }

// block b of a (Cout, Cxp) weight: first co / ci and the valid extents
struct Block {
  int co0, ci0, nco, nci_v, nci_s;
};

__device__ __forceinline__ Block block_of(int b, int Cout, int Cin, int Cxp) {
  const int nci = (Cxp + kT - 1) / kT;
  Block k;
  k.co0 = (b / nci) * kCo;
  k.ci0 = (b % nci) * kT;
  k.nco = min(kCo, Cout - k.co0);
  k.nci_v = min(kT, Cxp - k.ci0);              // columns of the (padded) forward layout
  k.nci_s = max(0, min(kT, Cin - k.ci0));      // columns present in the OIHW source
  return k;
}

inline long blocks_of(int Cout, int Cxp) { return (long)((Cout + kCo - 1) / kCo) * ((Cxp + kT - 1) / kT); }

template <int T>
__device__ __forceinline__ void store_layouts(const bf16* img, const Block& k, bf16* wf, bf16* wd, int Cout,
                                              int Cxp) {
  const int tid = threadIdx.x;
  if (wf != nullptr) {
    for (int e = tid; e < k.nco * T * (kT / 8); e += blockDim.x) {
      const int c8 = (e % (kT / 8)) * 8, r = e / (kT / 8);  // r = col * T + t
      if (c8 < k.nci_v) {
        const int col = r / T, t = r - col * T;
        const uint32_t* src = reinterpret_cast<const uint32_t*>(img + r * kLd + c8);  // 4-B aligned
        const uint4 u = make_uint4(src[0], src[1], src[2], src[3]);
        *reinterpret_cast<uint4*>(wf + ((long)(k.co0 + col) * T + t) * Cxp + k.ci0 + c8) = u;
      }
    }
  }
  if (wd != nullptr) {
    for (int e = tid; e < k.nci_s * T * (kCo / 8); e += blockDim.x) {
      const int c8 = (e % (kCo / 8)) * 8, r = e / (kCo / 8);  // r = cl * T + t
      if (c8 < k.nco) {
        const int cl = r / T, t = r - cl * T;
        uint32_t w[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          w[q] = bf16_bits(img[((c8 + 2 * q) * T + t) * kLd + cl]) |
                 (bf16_bits(img[((c8 + 2 * q + 1) * T + t) * kLd + cl]) << 16);
        *reinterpret_cast<uint4*>(wd + ((long)(k.ci0 + cl) * T + t) * Cout + k.co0 + c8) =
            make_uint4(w[0], w[1], w[2], w[3]);
      }
    }
  }
}

}  // namespace pack
}  // namespace fdt
