// Stride-1 3x3 convolutions (forward and the data gradient) with the input staged ONCE per
// K chunk as a halo tile in LDS (gfx950 / CDNA4).
//
// The generic implicit-GEMM kernel (conv_igemm_impl.h) forms the im2col operand by re-loading
// the input for every one of the 9 taps: a workgroup's 128 output pixels x K = 9*Cin reads
// 9 x 128 x Cin input elements through the texture path -- plus the 9 x BN x Cin weights --
// which holds the 3x3 layers at ~25-30 % of MFMA peak at batch 1024.  Here a workgroup owns
// 128 output pixels that are whole image rows (W = 32: 4 rows; 16: 8 rows; 8 / 4: 2 / 8 whole
// images) and, per chunk of 16 input channels, stages the (rows + 2) x (W + 2) halo of those
// rows (zero padding from out-of-range buffer loads) plus the 9 taps' weights in LDS; the
// 9 tap GEMMs then read shifted pixel rows of the same halo (halo pixel = output pixel +
// dh * (W + 2) + dw).  Input bytes per workgroup drop from 9 x 128 to ~1.6 x 128 rows per
// channel (x2.2 fewer bytes in total at BN = 64).
//
// Operand roles, MFMA (32x32x16 bf16), wave grid (2 x 2) and accumulator layout are the
// generic kernel's, so the fused epilogue is shared (igemm_epilogue): EPI_STATS (forward:
// per-channel sums for the lazy batch norm) and EPI_ACTBWD (data gradient through the
// producer's act(x*s+t), with its BN-backward reductions).  The tap table (dh, dw, wt) is the
// caller's: forward taps, or the mirrored taps of a stride-1 data gradient (wd layout).
//
// Pipeline: one register stage + two LDS buffers, one barrier per K chunk -- the next chunk's
// loads are in flight during the current chunk's 9 x TM x TN MFMAs.
//
// Reference semantics: resnet.py:72-113 (FusedConvBN) / :193-227 (the 3x3 convolutions of
// the residual blocks).
#include "conv_igemm_impl.h"

namespace fdt {
namespace conv {

constexpr int kHaloBM = 128;  // output pixels per workgroup
constexpr int kHaloBK = 16;   // input channels per K chunk (one MFMA K step)

// LDS rows of 16 channels are 32 B: rows r and r + 8 share banks, so the two 16-B halves of
// every 8-row group swap places (a ds_read_b128 of 16 consecutive rows is conflict-free)
__device__ __forceinline__ int hswz(int row) { return (row >> 3) & 1; }

template <int BN, int EPI, int ACT>
__global__ __launch_bounds__(256, (BN == 64 ? 3 : 2)) void conv3x3_halo_kernel(const ConvArgs a, int rows_t,
                                                                             int imgs_t, int halo_px) {
  constexpr int BM = kHaloBM, BK = kHaloBK;
  constexpr int CPR = BK / 8;  // 16-B chunks per row (2)
  constexpr int TM = BM / 64, TN = BN / 64;
  constexpr int NQ = EPI == kEpiJoinBwd ? 3 : 2;
  constexpr int NWC = 9 * BN * CPR;                     // weight chunks per K chunk
  constexpr int NW = (NWC + 255) / 256;                 // ... per thread (the last round partial)
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wn = wid & 1, wm = wid >> 1;
  const int H = a.Hi, W = a.Wi, HWc = W + 2;
  const int HR = rows_t + 2;               // halo rows per image
  const int img_px = rows_t * W;           // output pixels of one image in this tile
  const int rid = xcd_remap(blockIdx.x, a.nbm * a.nbn);
  const int bn = rid % a.nbn, bm = rid / a.nbn;
  const long m0 = (long)bm * BM;
  const int n0 = bn * BN;
  const int img0 = (int)(m0 / ((long)H * W));
  const int h0 = (int)((m0 % ((long)H * W)) / W);
  const float inv_alpha = ACT == kActCelu ? 1.f / a.epi_alpha : 1.f;

  // LDS: [statistics scratch of the epilogue | 2 x (halo [halo_px][BK] | weights [9][BN][BK])]
  float* red = reinterpret_cast<float*>(smem);
  const int hdr = ((4 * NQ * BN) * 4 + 15) & ~15;
  bf16* bufs = reinterpret_cast<bf16*>(smem + hdr);
  const int halo_elems = ((halo_px * BK) + 63) & ~63;
  const int buf_elems = halo_elems + 9 * BN * BK;

  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0,
                                                                      (int)a.Nb_HiWi_Cx_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, (short)0, (int)a.w_bytes,
                                                                      0x00020000);

  // ---- this thread's halo chunks (fixed over K): pixel offset in the input, or invalid
  const int nhc = halo_px * CPR;
  constexpr int NHMAX = 3;  // <= 288 halo pixels x 2 chunks / 256 threads
  // hoff: input element of the chunk (-1: padding -> zeros); hls: its LDS element (-1: none)
  int hoff[NHMAX], hls[NHMAX];
#pragma unroll
  for (int u = 0; u < NHMAX; ++u) {
    const int q = tid + u * 256;
    const int hp = q / CPR, cc = q % CPR;
    const int img = hp / (HR * HWc), rem = hp - img * (HR * HWc);
    const int r = rem / HWc, c = rem - r * HWc;
    const int h = h0 - 1 + r, w = c - 1;
    const bool ok = q < nhc && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
    hoff[u] = ok ? ((((img0 + img) * H + h) * W + w) << a.log2Cx) + cc * 8 : -1;
    hls[u] = q < nhc ? hp * BK + 8 * (cc ^ hswz(hp)) : -1;
  }
  // weight chunks: row (tap t, local channel co), chunk cc
  int woff[NW], wls[NW];
#pragma unroll
  for (int u = 0; u < NW; ++u) {
    const int q = tid + u * 256;
    const int row = q / CPR, cc = q % CPR;
    const int t = row / BN, co = row - t * BN;
    const bool ok = q < NWC;
    woff[u] = ok ? (n0 + co) * a.ldw + a.wt[t < 9 ? t : 0] * a.Cx + cc * 8 : -1;
    wls[u] = ok ? halo_elems + row * BK + 8 * (cc ^ hswz(row)) : -1;
  }

  struct Stage {
    uint4 h[NHMAX];
    uint4 w[NW];
  };
  auto load = [&](Stage& S, int kc, bool live) {
    const int ci = kc * BK;
#pragma unroll
    for (int u = 0; u < NHMAX; ++u) {
      S.h[u] = ld_buf16(rx, (live && hoff[u] >= 0) ? (uint32_t)(hoff[u] + ci) * 2u : kOOB);
    }
#pragma unroll
    for (int u = 0; u < NW; ++u) S.w[u] = ld_buf16(rw, (live && woff[u] >= 0) ? (uint32_t)(woff[u] + ci) * 2u : kOOB);
  };
  auto store = [&](const Stage& S, int buf) {
    bf16* B = bufs + buf * buf_elems;
#pragma unroll
    for (int u = 0; u < NHMAX; ++u)
      if (hls[u] >= 0) *reinterpret_cast<uint4*>(B + hls[u]) = S.h[u];
#pragma unroll
    for (int u = 0; u < NW; ++u)
      if (wls[u] >= 0) *reinterpret_cast<uint4*>(B + wls[u]) = S.w[u];
  };

  // ---- fragment rows: halo pixel of each 32-pixel block's lane (tap (0,0)), weight rows
  int hp0[TM];
#pragma unroll
  for (int j = 0; j < TM; ++j) {
    const int p = wm * (BM / 2) + j * 32 + (lane & 31);
    const int img = p / img_px, rem = p - img * img_px;
    const int r = rem / W, c = rem - r * W;
    hp0[j] = img * HR * HWc + (r + 1) * HWc + (c + 1);
  }
  int tap_off[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) tap_off[t] = a.dh[t] * HWc + a.dw[t];

  f32x16 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto compute = [&](int buf) {
    const bf16* B = bufs + buf * buf_elems;
    const bf16* Wl = B + halo_elems;
    const int ch = lane >> 5;  // this lane's 16-B chunk of the K=16 step
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      bf16x8_t wf[TN], xf[TM];
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        const int row = t * BN + wn * (BN / 2) + i * 32 + (lane & 31);
        wf[i] = *reinterpret_cast<const bf16x8_t*>(Wl + row * BK + 8 * (ch ^ hswz(row)));
      }
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const int hp = hp0[j] + tap_off[t];
        xf[j] = *reinterpret_cast<const bf16x8_t*>(B + hp * BK + 8 * (ch ^ hswz(hp)));
      }
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[i], xf[j], acc[i][j], 0, 0, 0);
    }
  };

  const int nk = a.Cx / BK;
  {
    Stage S;
    load(S, 0, true);
    store(S, 0);
    load(S, 1, nk > 1);
    __syncthreads();
    for (int k = 0; k < nk; ++k) {
      compute(k & 1);
      if (k + 1 >= nk) break;
      store(S, (k + 1) & 1);
      __syncthreads();
      load(S, k + 2, k + 2 < nk);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  igemm_epilogue<BM, BN, EPI, ACT, TN, TM>(a, acc, smem, hdr, red, m0, n0, bm, 0, inv_alpha);
}

template <int BN, int EPI, int ACT>
static void launch_halo(const ConvArgs& a, int rows_t, int imgs_t, int halo_px, hipStream_t st) {
  constexpr int NQ = EPI == kEpiJoinBwd ? 3 : 2;
  const size_t hdr = ((4 * NQ * BN) * 4 + 15) & ~(size_t)15;
  const size_t halo_elems = (((size_t)halo_px * kHaloBK) + 63) & ~(size_t)63;
  const size_t bufs = 2 * (halo_elems + 9 * (size_t)BN * kHaloBK) * 2;
  const size_t stage = (size_t)64 * (BN + 4) * 4;
  const size_t lds = hdr + (bufs > stage ? bufs : stage);
  auto kern = conv3x3_halo_kernel<BN, EPI, ACT>;
  static size_t attr_set = 64 * 1024;
  if (lds > attr_set) {
    FDT_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)lds));
    attr_set = lds;
  }
  hipLaunchKernelGGL(kern, dim3(a.nbm * a.nbn), dim3(256), lds, st, a, rows_t, imgs_t, halo_px);
  FDT_LAUNCH_CHECK();
}

}  // namespace conv

// Geometry of a halo tile for an H x W image, or false when the shape is not supported
// (128 output pixels must be whole rows of one image or whole images).
static bool halo_geometry(int H, int W, int* rows_t, int* imgs_t, int* halo_px) {
  if (W <= 0 || H <= 0 || W > conv::kHaloBM) return false;
  if (H * W >= conv::kHaloBM) {
    if (conv::kHaloBM % W) return false;
    *rows_t = conv::kHaloBM / W;
    if (H % *rows_t) return false;
    *imgs_t = 1;
  } else {
    if (conv::kHaloBM % (H * W)) return false;
    *rows_t = H;
    *imgs_t = conv::kHaloBM / (H * W);
  }
  *halo_px = *imgs_t * (*rows_t + 2) * (W + 2);
  return *halo_px * conv::kHaloBK / 8 <= 3 * 256;  // NHMAX chunks per thread
}

bool conv3x3_halo_supported(long Nb, int H, int W, int Cx, int Cout, int BN) {
  int r, i, hp;
  if (!halo_geometry(H, W, &r, &i, &hp)) return false;
  if (BN != 64 && BN != 128) return false;
  return Cx >= conv::kHaloBM / 8 && Cx % conv::kHaloBK == 0 && (Cx & (Cx - 1)) == 0 && Cout % BN == 0 &&
         (Nb * (long)H * W) % conv::kHaloBM == 0;
}

// Stride-1 3x3 convolution on the halo kernel: epi 0 (EPI_STATS: forward, y + statistics
// slots) or 1 (EPI_ACTBWD: data gradient through act(ex*es + et) + its reductions); taps =
// 9 (dh, dw, wt) triples with dh, dw in {-1, 0, 1} (forward or mirrored dgrad taps).
void conv3x3_halo(uint64_t x, uint64_t w, uint64_t out, uint64_t part, int part_rows, uint64_t ex, uint64_t es,
                  uint64_t et, long Nb, int H, int W, int Cx, int Cout, int ldw, const std::vector<int>& dh,
                  const std::vector<int>& dw, const std::vector<int>& wt, int epi, int act, float alpha, int BN,
                  uint64_t stream) {
  using namespace conv;
  FDT_CHECK(conv3x3_halo_supported(Nb, H, W, Cx, Cout, BN), "conv3x3_halo: unsupported shape");
  FDT_CHECK(dh.size() == 9 && dw.size() == 9 && wt.size() == 9, "conv3x3_halo: 9 taps");
  for (int t = 0; t < 9; ++t)
    FDT_CHECK(dh[t] >= -1 && dh[t] <= 1 && dw[t] >= -1 && dw[t] <= 1 && wt[t] >= 0 && wt[t] < 9,
              "conv3x3_halo: taps in {-1,0,1}^2");
  FDT_CHECK(epi == kEpiStats || epi == kEpiActBwd, "conv3x3_halo: EPI_STATS or EPI_ACTBWD");
  FDT_CHECK(epi != kEpiActBwd || (ex && es && et), "conv3x3_halo: ACTBWD needs ex, es, et");
  FDT_CHECK(part != 0, "conv3x3_halo: statistics slots");
  FDT_CHECK(ldw % 8 == 0 && ldw >= 9 * Cx, "conv3x3_halo: packed weight row stride");
  int rows_t, imgs_t, halo_px;
  halo_geometry(H, W, &rows_t, &imgs_t, &halo_px);
  ConvArgs a{};
  a.x = P<const bf16>(x);
  a.w = P<const bf16>(w);
  a.out = P<bf16>(out);
  a.part = P<float>(part);
  a.ex = P<const bf16>(ex);
  a.es = P<const float>(es);
  a.et = P<const float>(et);
  a.M = Nb * (long)H * W;
  a.Hi = a.Ho = a.Hout = H;
  a.Wi = a.Wo = a.Wout = W;
  a.Cx = Cx;
  a.log2Cx = 31 - __builtin_clz((unsigned)Cx);
  a.S = a.OS = 1;
  a.ntaps = 9;
  a.K = 9 * Cx;
  a.Cout = Cout;
  a.ldw = ldw;
  a.epi_act = act;
  a.epi_alpha = alpha;
  for (int t = 0; t < 9; ++t) {
    a.dh[t] = (int8_t)dh[t];
    a.dw[t] = (int8_t)dw[t];
    a.wt[t] = (int8_t)wt[t];
  }
  a.Nb_HiWi_Cx_bytes = a.M * Cx * 2;
  a.w_bytes = (long)Cout * ldw * 2;
  FDT_CHECK(a.Nb_HiWi_Cx_bytes < 0x7FFFFFF0L && a.w_bytes < 0x7FFFFFF0L && a.M * (long)Cout < 0x7FFFFFFFL,
            "conv3x3_halo: operand exceeds the 2 GiB buffer-descriptor range");
  a.nbm = (int)(a.M / kHaloBM);
  a.nbn = Cout / BN;
  a.nsplit = 1;
  a.det = deterministic() ? 1 : 0;
  a.slot_mask = stat_slot_mask(part_rows, a.nbm);
  hipStream_t st = as_stream(stream);
  if (a.M == 0) return;
#define FDT_H(BN_, E_, A_)                                                            \
  if (BN == BN_ && epi == E_ && act == A_) {                                          \
    launch_halo<BN_, E_, A_>(a, rows_t, imgs_t, halo_px, st);                         \
    return;                                                                           \
  }
  FDT_H(64, kEpiStats, kActNone) FDT_H(128, kEpiStats, kActNone)
  FDT_H(64, kEpiActBwd, kActRelu) FDT_H(128, kEpiActBwd, kActRelu)
  FDT_H(64, kEpiActBwd, kActCelu) FDT_H(128, kEpiActBwd, kActCelu)
  FDT_H(64, kEpiActBwd, kActNone) FDT_H(128, kEpiActBwd, kActNone)
#undef FDT_H
  FDT_CHECK(false, "conv3x3_halo: unsupported (epilogue, activation)");
}

}  // namespace fdt
