// Implicit-GEMM convolution for the NHWC ResNet engine on MI355X (gfx950 / CDNA4).
//
// One kernel template covers every forward convolution and every data-gradient
// (dgrad) convolution of the network:
//
//   C^T[ch][px] = sum_k  W[ch][k] * X[px][k],   k = (tap, ci),  px = output pixel
//
// The weight tile is the MFMA "A" operand (rows = output channels) and the activation
// tile the "B" operand (columns = pixels), so an accumulator lane holds 4-channel runs
// of ONE pixel: after a permlane32 swap every lane owns 8 consecutive channels of one
// NHWC row and the epilogue reads/writes 16 B per lane (T21).  mfma_f32_32x32x16_bf16,
// 4 waves (2 x 2) per 256-thread workgroup, BK = 64-element K tiles double-buffered in
// LDS with register-staged prefetch (loads for tile k+1 are issued before the MFMAs of
// tile k, the prologue math and LDS write happen after them, one barrier per tile),
// XOR-swizzled LDS rows (conflict-free ds_read_b128 for the fragment reads), XCD-aware
// workgroup remap so tiles sharing activation rows sit on one L2.  The epilogue transposes
// the accumulators through LDS so every global access is a full row segment.
//
// Fusion (the reason this is not a library call):
//  * prologue on the activation operand, applied while staging to LDS:
//      PRO_AFFINE_ACT  x -> act(x*s[c] + t[c])   (the producer's lazy batch-norm)
//      PRO_FOLD        g -> g*gs[c] + alpha[c] + beta[c]*y  (batch-norm backward correction;
//                      gs lets the residual join store one un-scaled gradient for both branches)
//      PRO_JOIN        (y, r) -> relu(y*s[c] + t[c] + r*s2[c] + t2[c])  -- the previous residual
//                      block's join (its BN'd residual branch + BN'd / identity shortcut), computed
//                      while staging the first 1x1 conv of the next block; the workgroups of the
//                      first output-channel tile also store the joined rows (the block output the
//                      identity shortcut and the backward need) and their ReLU bit mask, so the
//                      standalone join pass (read y, r; write out) and this conv's re-read of
//                      `out` become one pass
//    zero padding is applied AFTER the transform (the conv pads the normalised input);
//  * epilogue:
//      EPI_STATS   y (bf16) + per-block per-channel (sum y, sum y^2) slabs -> BN stats
//      EPI_ACTBWD  dgrad through the producer's lazy act(x*s+t): gx = g*act'(z)*s and
//                  per-channel (sum g_pre*x, sum g_pre) slabs
//      EPI_STORE / EPI_ADD  plain bf16 store / accumulate into an existing gradient.
//      EPI_GELU_FWD  the transformer FFN's first linear as a GEMM (x [tokens][d_model] the
//                  "pixels", W_1 the weights): a = acc + bias stored (bf16, the backward's
//                  GELU input) AND h = dropout(gelu(a)) stored -- the separate GELU-dropout
//                  pass (read a, write h) disappears (reference transformer.py:175-176)
//      EPI_GELU_BWD  the data gradient of the FFN's second linear (g_y W_2 -> dL/dh) finished
//                  through the GELU-dropout backward: ga = keep*scale*gelu'(a)*acc stored, and
//                  the column sums of ga = W_1's bias gradient accumulated (fp32 atomics)
//      EPI_JOINBWD  accumulate into the existing gradient of a residual-block output AND
//                  run that block's join backward on it: g_pre = g*act'(out) (ReLU bit
//                  mask or the stored CELU output), stored in place, plus the per-channel
//                  (sum g_pre*y_res, sum g_pre, sum g_pre*y_shortcut) slot reductions that
//                  the block's BN backward needs.  This is the dgrad that completes the
//                  gradient (the first 1x1 of the next block), so the standalone join pass
//                  (a full read of g + write of g_pre) disappears.
//
// Split-K (small-M layers: the 8x8 / 4x4 stages at the per-GPU batch of an 8-GPU run
// have only 32-512 output tiles but K up to 4608): nsplit workgroups share one output tile,
// each reducing a contiguous range of K tiles; all but the last to finish write their fp32
// accumulators to a slab (in register order: [tile][split][reg/4][thread] float4, so the
// reducer's thread t reads exactly its own registers' counterparts, coalesced) with
// write-through (sc1) stores, drain them and take a ticket; the last arriver adds the other
// slabs with sc1 loads (no L2 write-back / invalidate fences) and runs the normal fused
// epilogue.  Counters are reset by the last arriver.
//
// K groups (KG = 2, small-M layers): the workgroup is 8 waves = two 4-wave groups, each with its
// own double-buffered LDS tiles, taking alternate K tiles of the same output tile; group 1
// hands its accumulators to group 0 through LDS and group 0 runs the epilogue.  At the
// per-GPU batch of an 8-GPU run the 8x8 / 4x4 stages launch ~256 workgroups -- one 4-wave
// workgroup per CU leaves each SIMD a single wave that serialises load waits, prologue VALU,
// LDS reads and MFMAs (measured 44 % of wave time waiting, 23 % VALU, 10 % MFMA); two waves
// per SIMD overlap them with no extra global traffic (unlike split-K's fp32 slabs).
//
// Strided convolutions: forward uses the input stride S; the dgrad of a stride-2
// convolution is split by output parity into 4 dense classes (each its own tap table and
// output row map: hi = ho*OS + oy), so no MFMA work is spent on structural zeros.
//
// Reference semantics being accelerated: resnet.py:72-113 (FusedConvBN forward and its
// hand-derived backward), resnet.py:201-227 (strided conv + BatchNorm2d blocks).
#pragma once
#include "common.h"
#include "bn_math.h"
#include "dropout_math.h"
#include <vector>

#ifndef FDT_CONV_FRAG_PIPE
#define FDT_CONV_FRAG_PIPE 0  // 1: +16 VGPRs -- spills 19-125 VGPRs under the occupancy floors (measured, -Rpass-analysis)
#endif

namespace fdt {
namespace conv {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

enum Pro : int { kProNone = 0, kProAffineAct = 1, kProFold = 2, kProJoin = 3 };
enum Epi : int { kEpiStats = 0, kEpiActBwd = 1, kEpiStore = 2, kEpiAdd = 3, kEpiJoinBwd = 4, kEpiGeluFwd = 5,
                 kEpiGeluBwd = 6 };

struct ConvArgs {
  const bf16* x;     // activation operand [Nb][Hi][Wi][Cx]   (PRO_FOLD: the gradient G)
  const bf16* x2;    // PRO_FOLD: the producer output Y (same shape as x); PRO_JOIN: the shortcut operand r
  const float* ps;   // prologue per-channel scale: s (AFFINE_ACT) or alpha (FOLD)   [Cx]
  const float* pt;   // prologue per-channel shift: t (AFFINE_ACT) or beta  (FOLD)   [Cx]
  const float* pg;   // FOLD: per-channel scale of g (nullptr = 1): g*pg + alpha + beta*y    [Cx]
                     // JOIN: shortcut scale s2 (nullptr: identity shortcut, r used as is)
  const float* pt2;  // JOIN: shortcut shift t2 [Cx]
  bf16* pout;        // JOIN: the joined block output [M][Cx] (stored by the n0 == 0 workgroups)
  uint8_t* pmask;    // JOIN: its ReLU bit mask (bit i of byte e/8 = out[e] > 0), or nullptr
  const bf16* w;     // packed weights [Cout][ldw], k-index = wt[tap]*Cx + ci
  bf16* out;         // [Nb][Hout][Wout][Cout]
  float* part;       // statistics slots [rows][NQ][Cout], fp32 atomics (zeroed by the consumer)
  unsigned slot_mask;  // slot = row block & slot_mask (deterministic mode: no wrap, one writer per slot)
  int det;             // deterministic mode: the split-K reducer sums every split in split order
  const bf16* ex;    // ACTBWD: producer raw output x (shape of out); JOINBWD: residual-branch y
  const float* es;   // ACTBWD: producer scale s [Cout]
  const float* et;   // ACTBWD: producer shift t [Cout]
  const uint8_t* jmask;  // JOINBWD: ReLU join bit mask (bit i of byte e/8 = out[e] > 0), or nullptr
  const bf16* jyb;       // JOINBWD: shortcut-branch y (nullptr: identity shortcut)
  const bf16* jout;      // JOINBWD: join output (CELU joins, legacy o-mode; read when jmask and es are nullptr)
  // JOINBWD z mode (es / et = the residual branch's BN affine (s, t) set; CELU joins): act'(z) =
  // exp(z/alpha) from the recomputed fp32 pre-activation z = ya*s + t + (jyb ? jyb*jsb + jtb : jx),
  // exactly as the forward join formed it.  (From the bf16 output o, 1 + o/alpha is off by up to
  // ~2^-11/alpha = 6.5e-3 -- against a true derivative below 0.02 for z < -0.3 -- and o(z -> -inf)
  // rounds to -0.07520 < -alpha: a sign-flipped derivative for every deeply negative z.)
  const float* jsb;      // shortcut BN scale / shift (jyb set)
  const float* jtb;
  const bf16* jx;        // identity shortcut operand (the block input; jyb nullptr)
  const float* fbias;    // GELU_FWD: per-column bias [Cout]
  bf16* out2;            // GELU_FWD: h = dropout(gelu(a)) [M][Cout]   (GELU_BWD: a is `ex`)
  float* gb;             // GELU_BWD: bias-gradient accumulator [Cout] (fp32 atomics)
  uint32_t drop_thr;     // GELU_*: dropout keep threshold on the 32-bit hash (0: no dropout)
  float drop_scale;      // 1 / (1 - p)
  uint64_t drop_seed;    // host seed, XORed with *drop_seed_ptr when set (per-replay word)
  const uint64_t* drop_seed_ptr;
  long M;            // Nb*Ho*Wo GEMM rows
  int Hi, Wi, Cx, log2Cx;
  int Ho, Wo, S;
  int ntaps, K, Cout, ldw;
  int Hout, Wout, OS, oy, ox;
  int pro_act;
  float pro_alpha;
  int epi_act;
  float epi_alpha;
  int nbm, nbn;
  int nsplit, kps;   // split-K: workgroups per output tile, K tiles per split
  float* slab;       // split-K partials [tiles][nsplit][TN*TM*4][256] float4
  int* cnt;          // split-K tickets [tiles], zero between launches
  int8_t dh[12], dw[12], wt[12];
  // lazy batch statistics (bn_math.h): AFFINE_ACT / JOIN take (s, t) -- JOIN's shortcut (s2,
  // t2) from ls2 -- by finalising the producer's slot rows in the prologue (ps / pt unused)
  LazyStats ls1, ls2;
  int wthru;              // epilogue output stores write-through (sc1): see st_out
  int dbg;                // cost probes (scripts/conv_probe2.py): bit 0 = skip the statistics atomics
  long Nb_HiWi_Cx_bytes;  // bytes of the activation operand(s)
  long w_bytes;           // bytes of the packed weights
};

__device__ __forceinline__ uint32_t pk_bf16(float lo, float hi) { return pack_bf16x2(lo, hi); }

template <int CPR>
__device__ __forceinline__ int swz(int row) {
  // conflict-free ds_read_b128 of one 16-B chunk from 32 consecutive rows (see file header);
  // CPR = 16 (BK = 128): a row is exactly the 64 banks, 16 consecutive rows -> 16 distinct chunks
  if constexpr (CPR == 16) return row & 15;
  else if constexpr (CPR == 8) return (row >> 1) & 7;
  else return (row >> 2) & 3;
}

__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
  const int q = nblk >> 3, r = nblk & 7, xcd = bid & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

__device__ __forceinline__ void swap32(float& a, float& b) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  a = __uint_as_float(r[0]);
  b = __uint_as_float(r[1]);
}

// Activation helpers specialised at compile time (ACT: 0 none, 1 ReLU, 2 CELU(alpha)).
template <int ACT>
__device__ __forceinline__ float actf(float z, float alpha, float inv_alpha) {
  if constexpr (ACT == kActRelu) return fmaxf(z, 0.f);
  else if constexpr (ACT == kActCelu) return z > 0.f ? z : alpha * (__expf(z * inv_alpha) - 1.f);
  else return z;
}
template <int ACT>
__device__ __forceinline__ float actg(float z, float inv_alpha) {
  if constexpr (ACT == kActRelu) return z > 0.f ? 1.f : 0.f;
  else if constexpr (ACT == kActCelu) return z > 0.f ? 1.f : __expf(z * inv_alpha);
  else return 1.f;
}
// act'(z) from the activation OUTPUT o = act(z) (CELU: exp(z/alpha) = o/alpha + 1 for z <= 0)
template <int ACT>
__device__ __forceinline__ float actg_out(float o, float inv_alpha) {
  if constexpr (ACT == kActRelu) return o > 0.f ? 1.f : 0.f;
  else if constexpr (ACT == kActCelu) return o > 0.f ? 1.f : fmaf(o, inv_alpha, 1.f);
  else return 1.f;
}

__device__ __forceinline__ uint4 ld_buf16(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  auto v = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0);
  return *reinterpret_cast<uint4*>(&v);
}

// split-K slabs cross workgroups (and XCDs) inside one launch: written WRITE-THROUGH (sc1,
// cache-policy aux bit 16) and read back with sc1 loads, so the hand-off needs no agent-scope
// release / acquire fence (an L2 write-back / invalidate per workgroup) -- only every writing
// wave's vmcnt drain before the ticket add.
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_buf16_sc1(__amdgpu_buffer_rsrc_t r, uint32_t byte_off, float4 v) {
  u32x4_t u = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
  __builtin_amdgcn_raw_buffer_store_b128(u, r, byte_off, 0, 16);
}
__device__ __forceinline__ float4 ld_buf16_sc1(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  auto v = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 16);
  return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
}

constexpr uint32_t kOOB = 0xFFFFFFF0u;  // byte offset past any buffer: the load returns zeros

// Epilogue output store.  wt: write-through (sc1) -- the bytes leave the XCD's L2 as they are
// written instead of in the end-of-kernel write-back that the next (dependent) launch waits for
// (MI355X_MICROARCH: a boundary costs + dirty bytes / 6 TB/s); plain stores otherwise.
__device__ __forceinline__ void st_out(__amdgpu_buffer_rsrc_t r, uint32_t byte_off, bf16* p, const float* v, int wt) {
  if (wt) {
    u32x4_t u = {pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7])};
    __builtin_amdgcn_raw_buffer_store_b128(u, r, byte_off, 0, 16);
  } else {
    Vec8<bf16>::store(p, v);
  }
}

// Occupancy floor per instantiation: the 128x128x32 tiles whose prologue / epilogue fit in
// 128 registers without spilling (no fold prologue, no epilogue loads beyond one tensor:
// measured with -Rpass-analysis=kernel-resource-usage) are held to 4 waves per SIMD instead
// of the compiler's 2 (136 VGPRs + 64 AGPRs) -- these are the memory-bound 1x1 / plain-dgrad
// layers, where twice the workgroups in flight hide load and store latency.  The other 128x128
// tiles (fold prologue at BK = 32, any prologue but the fold at BK = 64) are held to 3 waves
// (168 registers: spill-free except <= 8-34 VGPRs on a few non-PURE variants, measured the
// same way); the fold-prologue BK = 64 tiles would spill 120+ and keep the compiler's 2.
template <int BM, int BN, int BK, int PRO, bool PURE>
constexpr int kMinWavesPerEU =
    (BM == 128 && BN == 128 && BK == 32 && (PRO == kProNone || (PRO == kProAffineAct && PURE))) ? 4
    : (BM == 128 && BN == 128 && (BK == 32 || (PRO != 2 && PRO != 3))) ? 3 : 1;

// ------------------------------------------------------------------ epilogue
// The accumulators are transposed through LDS before touching memory: a lane's MFMA
// result is 8 channels of ONE pixel, so a direct store / load covers 32 pixels x 32 B per
// wave instruction (32 partial cache lines).  Staged as fp32 rows [WM x 32 pixels][BN] (one
// pass per 32-pixel block j of every M-wave), each thread then owns 8 channels of whole rows and
// every wave instruction moves full contiguous 128-256 B row segments; per-channel statistics
// reduce over a thread's rows, then across the lanes sharing its channels (shuffles),
// then across the waves in LDS.  Rows padded by 4 floats: conflict-free ds_write_b128
// of the accumulator layout and ds_read_b128 of the row layout.
// Wave layout WM x WN (wave w: wm = w / WN along the pixels, wn = w % WN along the channels),
// NT threads; stg: >= WM*32*(BN+4) floats of LDS; red: [NT/64][NQ][BN] floats of LDS.
// ew: this thread owns the epilogue (K group 1 of a KG = 2 launch only meets the barriers).
// pix(wm, j, n): the tile-local output pixel of MFMA column n of block j of M-wave wm (the
// implicit-GEMM kernel: wm*BM/WM + 32 j + n; the halo kernel permutes columns, conv_h3.hip).
struct PixLinear {
  int wstride;
  __device__ __forceinline__ int operator()(int wm, int j, int n) const { return wm * wstride + j * 32 + n; }
};
template <int BM, int BN, int EPI, int ACT, int NT, int WM, int WN, class PixF = PixLinear>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& a, f32x16 (&acc)[BN / WN / 32][BM / WM / 32], long m0,
                                              int n0, int bm, int tid, float* stg, float* red, bool ew,
                                              float inv_alpha, PixF pix = PixLinear{BM / WM}) {
  constexpr int TN = BN / WN / 32, TM = BM / WM / 32;
  constexpr int NQ = EPI == kEpiJoinBwd ? 3 : 2;
  constexpr int SW = BN + 4;     // staged row stride (floats)
  constexpr int CG = BN / 8;     // 8-channel groups per row
  constexpr int RPS = NT / CG;       // rows per sweep
  constexpr int NSW = WM * 32 / RPS;  // sweeps per (WM x 32)-row pass
  static_assert(NSW >= 1 && NSW * RPS == WM * 32, "epilogue sweep geometry");
  constexpr int NW = NT / 64;
  const int lane = tid & 63, wid = tid >> 6, wn = wid % WN, wm = wid / WN;
  constexpr bool STATS = EPI == kEpiStats || EPI == kEpiActBwd || EPI == kEpiJoinBwd;
  const int h = lane >> 5;
  const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.out, (short)0, (int)0xFFFFFFFF, 0x00020000);
  const int cg = tid % CG, rs = tid / CG;
  const int c = n0 + cg * 8;  // this thread's 8 output channels
  const bool dense = a.OS == 1 && a.oy == 0 && a.ox == 0 && a.Hout == a.Ho && a.Wout == a.Wo;
  float sv[8], tv[8];
  constexpr bool GELU = EPI == kEpiGeluFwd || EPI == kEpiGeluBwd;
  uint64_t dseed = 0;
  if constexpr (GELU) dseed = drop::live_seed(a.drop_seed, a.drop_seed_ptr);
  if constexpr (EPI == kEpiGeluFwd) {
    const float4* bp = reinterpret_cast<const float4*>(a.fbias + c);
    const float4 b0 = bp[0], b1 = bp[1];
    sv[0] = b0.x; sv[1] = b0.y; sv[2] = b0.z; sv[3] = b0.w; sv[4] = b1.x; sv[5] = b1.y; sv[6] = b1.z; sv[7] = b1.w;
  }
  float sbv[8], tbv[8];
  const bool zm = EPI == kEpiJoinBwd && ACT == kActCelu && a.es != nullptr;
  if (EPI == kEpiActBwd || zm) {
    const float4* sp = reinterpret_cast<const float4*>(a.es + c);
    const float4* tp = reinterpret_cast<const float4*>(a.et + c);
    const float4 s0 = sp[0], s1 = sp[1], t0 = tp[0], t1 = tp[1];
    sv[0] = s0.x; sv[1] = s0.y; sv[2] = s0.z; sv[3] = s0.w; sv[4] = s1.x; sv[5] = s1.y; sv[6] = s1.z; sv[7] = s1.w;
    tv[0] = t0.x; tv[1] = t0.y; tv[2] = t0.z; tv[3] = t0.w; tv[4] = t1.x; tv[5] = t1.y; tv[6] = t1.z; tv[7] = t1.w;
  }
  if (zm && a.jyb != nullptr) {
#pragma unroll
    for (int k = 0; k < 8; ++k) { sbv[k] = a.jsb[c + k]; tbv[k] = a.jtb[c + k]; }
  }
  float q0[8], q1[8], q2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { q0[k] = 0.f; q1[k] = 0.f; q2[k] = 0.f; }
  __syncthreads();  // every wave is done with the K tiles (and the split-K flag)
#pragma unroll
  for (int j = 0; j < TM; ++j) {
    // ---- stage accumulator block j: local row = wm*32 + pixel, 8 channels per (i, p)
#pragma unroll
    for (int i = 0; i < TN; ++i) {
      if (!ew) break;
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int g = 2 * p;
        float v[8];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float lo = acc[i][j][4 * g + q], hi = acc[i][j][4 * g + 4 + q];
          swap32(lo, hi);
          v[q] = lo;
          v[4 + q] = hi;
        }
        float* dst = stg + (wm * 32 + (lane & 31)) * SW + wn * (BN / WN) + i * 32 + 16 * p + 8 * h;
        *reinterpret_cast<float4*>(dst) = make_float4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<float4*>(dst + 4) = make_float4(v[4], v[5], v[6], v[7]);
      }
    }
    __syncthreads();
    // ---- rows of this pass: 8 channels x NSW rows per thread
#pragma unroll
    for (int sw = 0; sw < NSW; ++sw) {
      const int lr = rs + sw * RPS;
      const long m = m0 + pix(lr >> 5, j, lr & 31);
      if (ew && m < a.M) {
        uint32_t orow;
        if (dense) {
          orow = (uint32_t)m;
        } else {
          const int mi = (int)m, hw = a.Ho * a.Wo;
          const int n = mi / hw, rem = mi - n * hw;
          const int oh = rem / a.Wo, ow = rem - oh * a.Wo;
          orow = (uint32_t)((n * a.Hout + oh * a.OS + a.oy) * a.Wout + ow * a.OS + a.ox);
        }
        const uint32_t e = orow * (uint32_t)a.Cout + c;
        const float4 va = *reinterpret_cast<const float4*>(stg + lr * SW + cg * 8);
        const float4 vb = *reinterpret_cast<const float4*>(stg + lr * SW + cg * 8 + 4);
        float v[8] = {va.x, va.y, va.z, va.w, vb.x, vb.y, vb.z, vb.w};
        if constexpr (EPI == kEpiStats) {
#pragma unroll
          for (int k = 0; k < 8; ++k) { q0[k] += v[k]; q1[k] = fmaf(v[k], v[k], q1[k]); }
          st_out(ro, e * 2u, a.out + e, v, a.wthru);
        } else if constexpr (EPI == kEpiActBwd) {
          float x8[8];
          Vec8<bf16>::load(a.ex + e, x8);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const float gp = v[k] * actg<ACT>(fmaf(x8[k], sv[k], tv[k]), inv_alpha);
            v[k] = gp * sv[k];
            q0[k] = fmaf(gp, x8[k], q0[k]);
            q1[k] += gp;
          }
          st_out(ro, e * 2u, a.out + e, v, a.wthru);
        } else if constexpr (EPI == kEpiJoinBwd) {
          float e8[8], ya[8], yb[8], o8[8];
          Vec8<bf16>::load(a.out + e, e8);
          Vec8<bf16>::load(a.ex + e, ya);
          const bool hb = a.jyb != nullptr;
          if (hb) Vec8<bf16>::load(a.jyb + e, yb);
          uint32_t mk = 0;
          if constexpr (ACT == kActRelu) mk = a.jmask[e >> 3];
          else if (!zm) Vec8<bf16>::load(a.jout + e, o8);
          else if (!hb) Vec8<bf16>::load(a.jx + e, o8);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const float gv = v[k] + e8[k];
            float gp;
            if constexpr (ACT == kActRelu) {
              gp = ((mk >> k) & 1u) ? gv : 0.f;
            } else if (zm) {
              const float z = fmaf(ya[k], sv[k], tv[k]) + (hb ? fmaf(yb[k], sbv[k], tbv[k]) : o8[k]);
              gp = gv * actg<ACT>(z, inv_alpha);
            } else {
              gp = gv * actg_out<ACT>(o8[k], inv_alpha);
            }
            v[k] = gp;
            q0[k] = fmaf(gp, ya[k], q0[k]);
            q1[k] += gp;
            if (hb) q2[k] = fmaf(gp, yb[k], q2[k]);
          }
          st_out(ro, e * 2u, a.out + e, v, a.wthru);
        } else if constexpr (EPI == kEpiAdd) {
          float e8[8];
          Vec8<bf16>::load(a.out + e, e8);
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] += e8[k];
          st_out(ro, e * 2u, a.out + e, v, a.wthru);
        } else if constexpr (EPI == kEpiGeluFwd) {
          // a = acc + bias, rounded to bf16 as stored (the backward reads the stored a);
          // h from the rounded a, exactly as the standalone GELU-dropout pass computes it
          uint32_t pa[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) pa[q] = pk_bf16(v[2 * q] + sv[2 * q], v[2 * q + 1] + sv[2 * q + 1]);
          *reinterpret_cast<uint4*>(a.out + e) = make_uint4(pa[0], pa[1], pa[2], pa[3]);
          const uint32_t mk = a.drop_thr ? drop::keep8((long)(e >> 3), dseed, a.drop_thr) : 0xffu;
          float h[8];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            h[2 * q] = bf16_lo(pa[q]);
            h[2 * q + 1] = bf16_hi(pa[q]);
          }
#pragma unroll
          for (int k = 0; k < 8; ++k) h[k] = ((mk >> k) & 1u) ? drop::gelu_erf(h[k]) * a.drop_scale : 0.f;
          Vec8<bf16>::store(a.out2 + e, h);
        } else if constexpr (EPI == kEpiGeluBwd) {
          // ga = keep * scale * gelu'(a) * dL/dh; the bias gradient sums the stored ga
          float a8[8];
          Vec8<bf16>::load(a.ex + e, a8);
          const uint32_t mk = a.drop_thr ? drop::keep8((long)(e >> 3), dseed, a.drop_thr) : 0xffu;
          uint32_t pg[4];
#pragma unroll
          for (int k = 0; k < 8; ++k)
            v[k] = ((mk >> k) & 1u) ? v[k] * a.drop_scale * drop::gelu_erf_grad(a8[k]) : 0.f;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            pg[q] = pk_bf16(v[2 * q], v[2 * q + 1]);
            q0[2 * q] += bf16_lo(pg[q]);
            q0[2 * q + 1] += bf16_hi(pg[q]);
          }
          *reinterpret_cast<uint4*>(a.out + e) = make_uint4(pg[0], pg[1], pg[2], pg[3]);
        } else {
          st_out(ro, e * 2u, a.out + e, v, a.wthru);
        }
      }
    }
    if (j + 1 < TM) __syncthreads();  // the next pass overwrites the staging rows
  }
  if constexpr (EPI == kEpiGeluBwd) {
    // column sums of ga: rows of a thread -> lanes sharing its columns -> 4 waves -> one
    // fp32 atomic per column per workgroup into the bias gradient
#pragma unroll
    for (int o = CG; o < 64; o <<= 1) {
      if (!ew) break;
#pragma unroll
      for (int k = 0; k < 8; ++k) q0[k] += __shfl_xor(q0[k], o, 64);
    }
    if (ew && lane < CG) {
#pragma unroll
      for (int k = 0; k < 8; ++k) red[wid * BN + cg * 8 + k] = q0[k];
    }
    __syncthreads();
    for (int e = tid; ew && e < BN; e += NT) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) t += red[w * BN + e];
      atomicAdd(&a.gb[n0 + e], t);
    }
  }
  if constexpr (STATS) {
    // lanes l, l + CG, l + 2CG, ... of a wave hold the same channels
#pragma unroll
    for (int o = CG; o < 64; o <<= 1) {
      if (!ew) break;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        q0[k] += __shfl_xor(q0[k], o, 64);
        q1[k] += __shfl_xor(q1[k], o, 64);
        if constexpr (NQ == 3) q2[k] += __shfl_xor(q2[k], o, 64);
      }
    }
    if (ew && lane < CG) {
      float* rw = red + wid * NQ * BN + cg * 8;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        rw[k] = q0[k];
        rw[BN + k] = q1[k];
        if constexpr (NQ == 3) rw[2 * BN + k] = q2[k];
      }
    }
    __syncthreads();
    for (int e = tid; ew && e < NQ * BN; e += NT) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) t += red[w * NQ * BN + e];
      const int q = e / BN, cc2 = e - q * BN;
      if (!(a.dbg & 1)) atomicAdd(&a.part[((long)(bm & a.slot_mask) * NQ + q) * a.Cout + n0 + cc2], t);
    }
  }
}

// KG: 1 = one 4-wave K group, register-staged (legacy K loop, see the main loop); 4 = the same with
// the rotated K loop (a true 2-deep register prefetch); 2 = two K groups (see above);
// 3 = one group whose operand tiles move global -> LDS by LDS-DMA (buffer_load ... lds) into a
// 3-buffer ring, two tiles in flight ACROSS the per-tile barrier (counted vmcnt + raw
// s_barrier: __syncthreads() would drain every in-flight DMA) -- prologue-free convolutions
// only (the DMA cannot transform), no staging registers and no ds_write pass.
template <int BM, int BN, int BK, int PRO, int EPI, bool PURE, int ACT, int KG>
__global__ __launch_bounds__(256 * (KG == 2 ? 2 : 1),
                             ((KG == 1 || KG == 4) ? kMinWavesPerEU<BM, BN, BK, PRO, PURE> : 1)) void
igemm_kernel(const ConvArgs a) {
  constexpr bool GL = KG == 3;
  static_assert(!GL || PRO == kProNone, "LDS-DMA staging moves bytes untransformed: prologue-free convolutions only");
  constexpr int CPR = BK / 8;        // 16-B chunks per LDS row
  constexpr int RPR = 256 / CPR;     // rows covered by one load round
  constexpr int NXL = BM / RPR;      // activation chunks per thread per tile
  constexpr int NWL = BN / RPR;      // weight chunks per thread per tile
  constexpr int TM = BM / 64, TN = BN / 64;
  constexpr int XT = BM * BK, WT = BN * BK;
  static_assert(NXL >= 1 && NWL >= 1, "tile too small for 256 threads");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nkt = (a.K + BK - 1) / BK;
  constexpr bool HASPRO = PRO == kProAffineAct || PRO == kProFold || PRO == kProJoin;
  constexpr bool TWOX = PRO == kProFold || PRO == kProJoin;  // two activation operands
  constexpr int NPRM = PRO == kProJoin ? 4 : (PRO == kProFold ? 3 : (HASPRO ? 2 : 0));
  static_assert(PRO != kProJoin || PURE, "the join prologue is for 1x1 stride-1 convolutions");
  constexpr int NQ = EPI == kEpiJoinBwd ? 3 : 2;                       // statistics rows
  // LDS: [prologue params | per-wave statistics | tap tables | K tiles, reused as the
  // epilogue's staging area] (the header size must match lds_bytes() on the host)
  float* pst = reinterpret_cast<float*>(smem);                         // [2|3][Cx] (PRO != none)
  float* red = pst + NPRM * a.Cx;                                      // [4 waves][NQ][BN]
  int* tapt = reinterpret_cast<int*>(red + 4 * NQ * BN);               // [12]: tap pixel offset
  int* tapw = tapt + 12;                                               // [12]: dh | dw<<8 | wt<<16
  const int hdr = ((NPRM * a.Cx + 4 * NQ * BN + 24) * 4 + 15) & ~15;
  bf16* tiles = reinterpret_cast<bf16*>(smem + hdr);                   // [nbuf][WT + XT]

  // tid / lane / wid are local to the K group (every load / fragment / epilogue mapping below
  // is written for 256 threads); grp selects the group's K tiles and LDS buffers
  const int tid = threadIdx.x & 255, lane = tid & 63, wid = tid >> 6;
  const int grp = KG == 2 ? (int)(threadIdx.x >> 8) : 0;
  static_assert(KG == 1 || KG == 2 || KG == 3 || KG == 4, "one or two K groups, the LDS-DMA ring, or rotated");
  const int wn = wid & 1, wm = wid >> 1;
  // a tile's splits are consecutive ids -> the same XCD after the remap
  const int rid = xcd_remap(blockIdx.x, a.nbm * a.nbn * a.nsplit);
  const int id = rid / a.nsplit, split = rid - id * a.nsplit;
  const int bn = id % a.nbn, bm = id / a.nbn;
  const long m0 = (long)bm * BM;
  const int n0 = bn * BN;
  const float inv_alpha = ACT == kActCelu ? 1.f / (PRO == kProAffineAct ? a.pro_alpha : a.epi_alpha) : 1.f;
  static_assert(!(PRO == kProAffineAct && EPI == kEpiJoinBwd), "one activation per instantiation");

  // buffer descriptors (wave-uniform, built from kernel arguments): 32-bit offsets and
  // hardware bounds checking -> zero padding / K tails need no branches
  const __amdgpu_buffer_rsrc_t rx_d = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.x, (short)0, (int)(a.Nb_HiWi_Cx_bytes), 0x00020000);
  const __amdgpu_buffer_rsrc_t ry_d = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(TWOX ? a.x2 : a.x), (short)0, (int)(a.Nb_HiWi_Cx_bytes), 0x00020000);
  const __amdgpu_buffer_rsrc_t rw_d = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.w, (short)0, (int)(a.w_bytes), 0x00020000);

  // ---- per-thread activation rows (fixed across K tiles): pixel index of tap (0,0)
  const int cc = tid % CPR;  // this thread's 16-B chunk column inside a K tile
  int pixb[NXL], ohs[NXL], ows[NXL];
  bool rv[NXL];
#pragma unroll
  for (int j = 0; j < NXL; ++j) {
    const long m = m0 + tid / CPR + j * RPR;
    rv[j] = m < a.M;
    if constexpr (PURE) {
      pixb[j] = (int)m;
      ohs[j] = ows[j] = 0;
    } else {
      const int hw = a.Ho * a.Wo;
      const int mi = rv[j] ? (int)m : 0;
      const int n = mi / hw;
      const int rem = mi - n * hw;
      const int oh = rem / a.Wo, ow = rem - (rem / a.Wo) * a.Wo;
      ohs[j] = oh * a.S;
      ows[j] = ow * a.S;
      pixb[j] = (n * a.Hi + ohs[j]) * a.Wi + ows[j];
    }
  }

  // one register stage = the global loads of one K tile (staged to LDS after the MFMAs
  // of the previous tile).  Two stages alternate so that the loads of tile k+2 are in
  // flight during the MFMAs of tiles k and k+1.
  struct Stage {
    uint4 rx[NXL], rx2[TWOX ? NXL : 1], rw[NWL];
    bool xv[NXL];
    int kci;
  };

  // Loads are issued unconditionally (a K tile past this split's range, or past K, reads
  // the OOB offset and returns zeros): no branch around a load, so hipcc's waitcnt pass
  // can count the two in-flight stages exactly (vmcnt(N), not vmcnt(0)) -- a branch-guarded
  // prefetch degenerates to a full-latency wait every K tile.
  auto load_tile = [&](Stage& S, int kt, bool live) {
    const int k = kt * BK + cc * 8;
    const int tap = k >> a.log2Cx;
    const int ci = k & (a.Cx - 1);
    S.kci = ci;
    const bool tok = live && tap < a.ntaps;
    int dh = 0, dw = 0, wt = 0, toff = 0;
    if constexpr (!PURE) {
      const int tq = tap < 12 ? tap : 11;  // branch-free LDS lookup (masked by tok below)
      const int e = tapw[tq];
      dh = (int)(int8_t)(e & 0xff);
      dw = (int)(int8_t)((e >> 8) & 0xff);
      wt = (e >> 16) & 0xff;
      toff = tapt[tq];
    }
#pragma unroll
    for (int j = 0; j < NXL; ++j) {
      bool v = rv[j] & tok;  // bitwise: no short-circuit branch around the load
      if constexpr (!PURE)
        v = v & ((unsigned)(ohs[j] + dh) < (unsigned)a.Hi) & ((unsigned)(ows[j] + dw) < (unsigned)a.Wi);
      S.xv[j] = v;
      const uint32_t off = v ? (((uint32_t)(pixb[j] + toff) << a.log2Cx) + ci) * 2u : kOOB;
      S.rx[j] = ld_buf16(rx_d, off);
      if constexpr (TWOX) S.rx2[j] = ld_buf16(ry_d, off);
    }
    const uint32_t wk = (uint32_t)((PURE ? 0 : wt) * a.Cx + ci);
#pragma unroll
    for (int j = 0; j < NWL; ++j) {
      const int row = tid / CPR + j * RPR;
      S.rw[j] = ld_buf16(rw_d, tok ? ((uint32_t)(n0 + row) * (uint32_t)a.ldw + wk) * 2u : kOOB);
    }
  };

  bf16* const gtiles = tiles + grp * 2 * (WT + XT);  // this K group's two LDS buffers
  auto store_tile = [&](const Stage& S, int buf) {
    bf16* Wl = gtiles + buf * (WT + XT);
    bf16* Xl = Wl + WT;
#pragma unroll
    for (int j = 0; j < NWL; ++j) {
      const int row = tid / CPR + j * RPR;
      *reinterpret_cast<uint4*>(Wl + row * BK + 8 * (cc ^ swz<CPR>(row))) = S.rw[j];
    }
    float sv[8], tv[8], gv[8];
    if constexpr (PRO == kProFold) {
      const float4* gp = reinterpret_cast<const float4*>(pst + 2 * a.Cx + S.kci);
      float4 g0 = gp[0], g1 = gp[1];
      gv[0] = g0.x; gv[1] = g0.y; gv[2] = g0.z; gv[3] = g0.w; gv[4] = g1.x; gv[5] = g1.y; gv[6] = g1.z; gv[7] = g1.w;
    }
    if constexpr (HASPRO) {
      const float4* sp = reinterpret_cast<const float4*>(pst + S.kci);
      const float4* tp = reinterpret_cast<const float4*>(pst + a.Cx + S.kci);
      float4 s0 = sp[0], s1 = sp[1], t0 = tp[0], t1 = tp[1];
      sv[0] = s0.x; sv[1] = s0.y; sv[2] = s0.z; sv[3] = s0.w; sv[4] = s1.x; sv[5] = s1.y; sv[6] = s1.z; sv[7] = s1.w;
      tv[0] = t0.x; tv[1] = t0.y; tv[2] = t0.z; tv[3] = t0.w; tv[4] = t1.x; tv[5] = t1.y; tv[6] = t1.z; tv[7] = t1.w;
    }
#pragma unroll
    for (int j = 0; j < NXL; ++j) {
      const int row = tid / CPR + j * RPR;
      uint4 o = S.rx[j];
      if constexpr (PRO == kProAffineAct) {
        // act(x*s+t), then zero where the conv pads (select, no branch)
        float v[8];
        const uint32_t u[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) { v[2 * q] = bf16_lo(u[q]); v[2 * q + 1] = bf16_hi(u[q]); }
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = actf<ACT>(fmaf(v[q], sv[q], tv[q]), a.pro_alpha, inv_alpha);
        o = make_uint4(pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3]), pk_bf16(v[4], v[5]), pk_bf16(v[6], v[7]));
        if (!S.xv[j]) o = make_uint4(0, 0, 0, 0);
      } else if constexpr (PRO == kProJoin) {
        // relu(y*s + t + r*s2 + t2): the previous block's output, rounded to bf16 exactly as
        // the standalone join stores it; the first column tile also materialises it
        float v[8], r[8];
        const uint32_t u[4] = {o.x, o.y, o.z, o.w};
        const uint32_t ur[4] = {S.rx2[j].x, S.rx2[j].y, S.rx2[j].z, S.rx2[j].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          v[2 * q] = bf16_lo(u[q]); v[2 * q + 1] = bf16_hi(u[q]);
          r[2 * q] = bf16_lo(ur[q]); r[2 * q + 1] = bf16_hi(ur[q]);
        }
        const float4* s2p = reinterpret_cast<const float4*>(pst + 2 * a.Cx + S.kci);
        const float4* t2p = reinterpret_cast<const float4*>(pst + 3 * a.Cx + S.kci);
        const float4 a0 = s2p[0], a1 = s2p[1], b0 = t2p[0], b1 = t2p[1];
        const float s2v[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
        const float t2v[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
        uint32_t mk = 0;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          v[q] = actf<ACT>(fmaf(v[q], sv[q], tv[q]) + fmaf(r[q], s2v[q], t2v[q]), a.pro_alpha, inv_alpha);
          mk |= (v[q] > 0.f ? 1u : 0u) << q;
        }
        o = make_uint4(pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3]), pk_bf16(v[4], v[5]), pk_bf16(v[6], v[7]));
        if (!S.xv[j]) o = make_uint4(0, 0, 0, 0);
        if (n0 == 0 && S.xv[j]) {
          const long e = ((long)pixb[j] << a.log2Cx) + S.kci;
          *reinterpret_cast<uint4*>(a.pout + e) = o;
          if (a.pmask) a.pmask[e >> 3] = (uint8_t)mk;
        }
      } else if constexpr (PRO == kProFold) {
        // g + alpha + beta*y (padding: g = y = 0 from the bounds-checked load -> masked)
        float g[8], y[8];
        const uint32_t u[4] = {o.x, o.y, o.z, o.w};
        const uint32_t uy[4] = {S.rx2[j].x, S.rx2[j].y, S.rx2[j].z, S.rx2[j].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          g[2 * q] = bf16_lo(u[q]); g[2 * q + 1] = bf16_hi(u[q]);
          y[2 * q] = bf16_lo(uy[q]); y[2 * q + 1] = bf16_hi(uy[q]);
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) g[q] = fmaf(g[q], gv[q], fmaf(tv[q], y[q], sv[q]));
        o = make_uint4(pk_bf16(g[0], g[1]), pk_bf16(g[2], g[3]), pk_bf16(g[4], g[5]), pk_bf16(g[6], g[7]));
        if (!S.xv[j]) o = make_uint4(0, 0, 0, 0);
      }
      *reinterpret_cast<uint4*>(Xl + row * BK + 8 * (cc ^ swz<CPR>(row))) = o;
    }
  };

  f32x16 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // Fragments double-buffered in registers across the tile's 16-deep K steps: step ks+1's LDS
  // reads issue before step ks's MFMAs (pinned by sched_barrier), so their latency hides behind
  // MFMAs (FDT_CONV_FRAG_PIPE, off by default: the extra fragment set spills under the occupancy floors).
  auto compute = [&](int buf) {
    const bf16* Wl = gtiles + buf * (WT + XT);
    const bf16* Xl = Wl + WT;
#if FDT_CONV_FRAG_PIPE
    bf16x8_t wf[2][TN], xf[2][TM];
    auto fetch = [&](int ks, int sl) {
      const int ch = ks * 2 + (lane >> 5);
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        const int row = wn * (BN / 2) + i * 32 + (lane & 31);
        wf[sl][i] = *reinterpret_cast<const bf16x8_t*>(Wl + row * BK + 8 * (ch ^ swz<CPR>(row)));
      }
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const int row = wm * (BM / 2) + j * 32 + (lane & 31);
        xf[sl][j] = *reinterpret_cast<const bf16x8_t*>(Xl + row * BK + 8 * (ch ^ swz<CPR>(row)));
      }
    };
    fetch(0, 0);
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      const int sl = ks & 1;
      if (ks + 1 < BK / 16) fetch(ks + 1, sl ^ 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[sl][i], xf[sl][j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
#else
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      const int ch = ks * 2 + (lane >> 5);
      bf16x8_t wf[TN], xf[TM];
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        const int row = wn * (BN / 2) + i * 32 + (lane & 31);
        wf[i] = *reinterpret_cast<const bf16x8_t*>(Wl + row * BK + 8 * (ch ^ swz<CPR>(row)));
      }
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const int row = wm * (BM / 2) + j * 32 + (lane & 31);
        xf[j] = *reinterpret_cast<const bf16x8_t*>(Xl + row * BK + 8 * (ch ^ swz<CPR>(row)));
      }
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[i], xf[j], acc[i][j], 0, 0, 0);
    }
#endif
  };

  // this split's K tiles [kb, kb + nk); K group g takes tiles kb + i*KG + g, i < nkk (the
  // same trip count in both groups -- a group's tile past nk loads zeros -- so both groups
  // meet every barrier)
  const int kb = split * a.kps;
  const int nk = min(nkt - kb, a.kps);
  constexpr int KGN = KG == 2 ? 2 : 1;
  const int nkk = (nk + KGN - 1) / KGN;
  auto ld = [&](Stage& S, int i) { load_tile(S, kb + i * KGN + grp, i < nkk && i * KGN + grp < nk); };

  if constexpr (GL) {
    // ---- LDS-DMA ring: tile t lands in buffer t % 3.  Lane l of a wave instruction writes
    // LDS base + 16 l, so a wave's 64 lanes fill 64 consecutive 16-B slots; the slot of
    // (row, chunk) is row*CPR + chunk (= tid + 256 j for this thread's j-th chunk), and the XOR
    // swizzle the fragment reads expect is applied on the SOURCE address (the lane filling
    // physical chunk cc fetches logical chunk cc ^ swz(row)).  Out-of-range offsets (padding,
    // K tail, past this split) read zeros.
    constexpr int G = NXL + NWL;  // DMA instructions per tile per thread
    if (tid < 12) {
      const int dh = a.dh[tid], dw = a.dw[tid];
      tapt[tid] = dh * a.Wi + dw;
      tapw[tid] = (int)(uint8_t)a.dh[tid] | ((int)(uint8_t)a.dw[tid] << 8) | ((int)(uint8_t)a.wt[tid] << 16);
    }
    __syncthreads();              // LDS header (tap table) ready
    // (readfirstlane: the DMA's LDS base goes to M0 -- a base the compiler cannot prove
    // wave-uniform is issued as a waterfall loop of exec-masked DMAs)
    const int wave_slot = __builtin_amdgcn_readfirstlane(wid) * 64;
    auto issue = [&](int i) {
      const int kt = kb + i;
      const bool live = i < nk;
      bf16* Wl = tiles + (i % 3) * (WT + XT);
      bf16* Xl = Wl + WT;
#pragma unroll
      for (int j = 0; j < NXL; ++j) {
        const int row = tid / CPR + j * RPR;
        const int lc = cc ^ swz<CPR>(row);
        const int k = kt * BK + lc * 8;
        const int tap = k >> a.log2Cx;
        const int ci = k & (a.Cx - 1);
        bool v = rv[j] & live & (tap < a.ntaps);
        int toff = 0;
        if constexpr (!PURE) {
          const int tq = tap < 12 ? tap : 11;
          const int e = tapw[tq];
          const int dh = (int)(int8_t)(e & 0xff), dw = (int)(int8_t)((e >> 8) & 0xff);
          toff = tapt[tq];
          v = v & ((unsigned)(ohs[j] + dh) < (unsigned)a.Hi) & ((unsigned)(ows[j] + dw) < (unsigned)a.Wi);
        }
        const uint32_t off = v ? (((uint32_t)(pixb[j] + toff) << a.log2Cx) + ci) * 2u : kOOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rx_d, (__attribute__((address_space(3))) void*)(Xl + (wave_slot + j * 256) * 8), 16, off, 0, 0, 0);
      }
#pragma unroll
      for (int j = 0; j < NWL; ++j) {
        const int row = tid / CPR + j * RPR;
        const int lc = cc ^ swz<CPR>(row);
        const int k = kt * BK + lc * 8;
        const int tap = k >> a.log2Cx;
        const int ci = k & (a.Cx - 1);
        const bool tok = live & (tap < a.ntaps);
        int wt = 0;
        if constexpr (!PURE) wt = (tapw[tap < 12 ? tap : 11] >> 16) & 0xff;
        const uint32_t off = tok ? ((uint32_t)(n0 + row) * (uint32_t)a.ldw + (uint32_t)(wt * a.Cx + ci)) * 2u : kOOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rw_d, (__attribute__((address_space(3))) void*)(Wl + (wave_slot + j * 256) * 8), 16, off, 0, 0, 0);
      }
    };
    if (nk > 0) {
      issue(0);
      issue(1);  // (a tile past nk loads zeros: the count below stays exact)
    }
    for (int t = 0; t < nk; ++t) {
      // tile t landed (this wave's DMAs: all but the G of tile t+1), then everyone's
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G) : "memory");
      __builtin_amdgcn_s_barrier();
      // buffer (t+2) % 3 held tile t-1: every wave finished its MFMAs before this barrier
      issue(t + 2);
      compute(t % 3);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the zero-tiles past nk)
  } else {
  // prologue: tile 0 -> LDS buf 0; tile 1 pending in B; tile 2 in flight in A.
  // 1x1 convolutions address their operands without the LDS tap table, so their first two
  // K tiles are requested BEFORE the LDS setup (prologue parameters, tap table) and its
  // barrier: the workgroup pays one memory latency at start-up instead of two (these
  // memory-bound layers run many short workgroups).
  Stage SA, SB;
  if constexpr (PURE) {
    if (nkk > 0) {
      ld(SA, 0);
      __builtin_amdgcn_sched_barrier(0);  // issue order SA, SB, SA' pinned (exact vmcnt counting)
      ld(SB, 1);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (grp == 0) {
    if constexpr (HASPRO) {
      const bool w0 = blockIdx.x == 0;  // the one workgroup that writes a lazy unit's outputs
      if (PRO != kProFold && a.ls1.base) {
        lazy_fill<256>(a.ls1, a.Cx, pst, pst + a.Cx, tid, w0);
      } else {
        for (int i = tid; i < a.Cx; i += 256) {
          pst[i] = a.ps[i];
          pst[a.Cx + i] = a.pt[i];
        }
      }
      if constexpr (PRO == kProFold) {
        for (int i = tid; i < a.Cx; i += 256) pst[2 * a.Cx + i] = a.pg ? a.pg[i] : 1.f;
      }
      if constexpr (PRO == kProJoin) {
        if (a.ls2.base) {
          lazy_fill<256>(a.ls2, a.Cx, pst + 2 * a.Cx, pst + 3 * a.Cx, tid, w0);
        } else {
          for (int i = tid; i < a.Cx; i += 256) {
            pst[2 * a.Cx + i] = a.pg ? a.pg[i] : 1.f;
            pst[3 * a.Cx + i] = a.pg ? a.pt2[i] : 0.f;
          }
        }
      }
    }
    if (tid < 12) {
      const int dh = a.dh[tid], dw = a.dw[tid];
      tapt[tid] = dh * a.Wi + dw;
      tapw[tid] = (int)(uint8_t)a.dh[tid] | ((int)(uint8_t)a.dw[tid] << 8) | ((int)(uint8_t)a.wt[tid] << 16);
    }
  }

  __syncthreads();
  if constexpr (!PURE) {
    if (nkk > 0) {
      ld(SA, 0);
      __builtin_amdgcn_sched_barrier(0);
      ld(SB, 1);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if constexpr (KG == 4) {
  // Main loop, two K tiles per trip, rotated so that every trip begins exactly as the loop
  // is entered: tiles kt (SA) and kt+1 (SB) in flight, the older one stored first.  (hipcc's
  // waitcnt pass merges the loop-entry and back-edge states; with the entry store peeled ahead
  // of the loop and exits inside the trip -- the legacy form below -- it waits for EVERY
  // outstanding load, vmcnt(0), at the first LDS store of each trip, draining the tile k+2
  // prefetch: a 1-deep pipeline.  Which form is faster depends on the layer -- the deeper
  // pipeline holds the loads' registers longer -- so the tuned table picks per layer: "loop".)
  int kt = 0;
  for (; kt + 1 < nkk; kt += 2) {
    store_tile(SA, 0);                  // tile kt -> buf 0 (SB: kt+1 still in flight)
    __syncthreads();
    ld(SA, kt + 2);
    __builtin_amdgcn_sched_barrier(0);  // keep the prefetch issued ahead of the MFMAs
    compute(0);
    store_tile(SB, 1);                  // tile kt+1 -> buf 1 (SA: kt+2 in flight)
    __syncthreads();
    ld(SB, kt + 3);
    __builtin_amdgcn_sched_barrier(0);
    compute(1);
  }
  if (kt < nkk) {  // odd tile count: the last tile
    store_tile(SA, 0);
    __syncthreads();
    compute(0);
  }
  } else {
  // legacy form: tile 0 stored ahead of the loop, exits inside the trip
  if (nkk > 0) {
    store_tile(SA, 0);
    ld(SA, 2);
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
  }
  for (int kt = 0; kt < nkk; kt += 2) {
    compute(0);
    if (kt + 1 >= nkk) break;
    store_tile(SB, 1);
    __syncthreads();
    ld(SB, kt + 3);
    __builtin_amdgcn_sched_barrier(0);
    compute(1);
    if (kt + 2 >= nkk) break;
    store_tile(SA, 0);
    __syncthreads();
    ld(SA, kt + 4);
    __builtin_amdgcn_sched_barrier(0);
  }
  }
  }

  if constexpr (KG == 2) {
    // group 1's partial sums -> LDS -> group 0 (register order [reg][thread]: conflict-free)
    float* xs = reinterpret_cast<float*>(tiles);
    __syncthreads();  // every wave is done reading its K tiles
    if (grp == 1) {
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) xs[((i * TM + j) * 16 + r) * 256 + tid] = acc[i][j][r];
    }
    __syncthreads();
    if (grp == 0) {
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][j][r] += xs[((i * TM + j) * 16 + r) * 256 + tid];
    }
    // (the epilogue's first barrier orders these reads before its staging writes)
  }

  // ------------------------------------------------------------------ split-K combine
  // (KG == 2 launches never split K over workgroups: the host refuses nsplit > 1 there)
  if (KG != 2 && a.nsplit > 1) {
    constexpr int NR4 = TN * TM * 4;  // float4 registers per thread
    // this tile's slabs [nsplit][NR4][256] float4 behind one buffer descriptor
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(reinterpret_cast<float4*>(a.slab) + (long)id * a.nsplit * NR4 * 256), (short)0,
        (int)(a.nsplit * NR4 * 256 * 16), 0x00020000);
    {
      const uint32_t mine = (uint32_t)((split * NR4 * 256 + tid) * 16);
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            st_buf16_sc1(rs, mine + (uint32_t)(((i * TM + j) * 4 + q) * 256 * 16),
                         make_float4(acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every writing wave drains its sc1 stores
    __syncthreads();
    int* flag = reinterpret_cast<int*>(red);
    if (tid == 0) {
      const int t = __hip_atomic_fetch_add(&a.cnt[id], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = t == a.nsplit - 1;
      if (last) __hip_atomic_store(&a.cnt[id], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      flag[0] = last;
    }
    __syncthreads();
    const int last = flag[0];
    __syncthreads();  // red is reused by the epilogue
    if (!last) return;
    if (a.det) {
      // fixed summation order whichever split arrived last (its own slab was written too)
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    }
    for (int sp = 0; sp < a.nsplit; ++sp) {
      if (sp == split && !a.det) continue;
      const uint32_t other = (uint32_t)((sp * NR4 * 256 + tid) * 16);
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float4 v = ld_buf16_sc1(rs, other + (uint32_t)(((i * TM + j) * 4 + q) * 256 * 16));
            acc[i][j][4 * q] += v.x;
            acc[i][j][4 * q + 1] += v.y;
            acc[i][j][4 * q + 2] += v.z;
            acc[i][j][4 * q + 3] += v.w;
          }
    }
  }

  conv_epilogue<BM, BN, EPI, ACT, 256, 2, 2>(a, acc, m0, n0, bm, tid, reinterpret_cast<float*>(smem + hdr), red,
                                           grp == 0, inv_alpha);
}

// ---------------------------------------------------------------------- host side
struct Cfg {
  int BM, BN;
};

template <int BM, int BN, int BK, int PRO, int EPI, bool PURE, int ACT, int KG>
static void launch_one(const ConvArgs& a, size_t lds, hipStream_t st) {
  auto kern = igemm_kernel<BM, BN, BK, PRO, EPI, PURE, ACT, KG>;
  static size_t attr_set = 64 * 1024;  // default dynamic-LDS limit; raise only when needed
  if (lds > attr_set) {
    FDT_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)lds));
    attr_set = lds;
  }
  hipLaunchKernelGGL(kern, dim3(a.nbm * a.nbn * a.nsplit), dim3(KG == 2 ? 512 : 256), lds, st, a);
  FDT_LAUNCH_CHECK();
}

template <int BM, int BN, int BK, int PRO, int EPI, int ACT, int KG>
static void launch_pure(const ConvArgs& a, bool pure, size_t lds, hipStream_t st) {
  if constexpr (PRO == kProJoin) {
    FDT_CHECK(pure, "the join prologue needs a 1x1 stride-1 convolution");
    launch_one<BM, BN, BK, PRO, EPI, true, ACT, KG>(a, lds, st);
  } else {
    if (pure) launch_one<BM, BN, BK, PRO, EPI, true, ACT, KG>(a, lds, st);
    else launch_one<BM, BN, BK, PRO, EPI, false, ACT, KG>(a, lds, st);
  }
}

template <int PRO, int EPI, int ACT>
static void launch_tile(const ConvArgs& a, int BM, int BN, int BK, int kg, bool pure, hipStream_t st) {
  const int nkt = (a.K + BK - 1) / BK;
  const size_t nbuf = kg == 3 ? 3 : (nkt > 1 ? 2 : 1);
  FDT_CHECK(kg == 1 || kg == 3 || kg == 4 || (kg == 2 && a.nsplit == 1 && nkt >= 2),
            "K groups: kg 1 | 2 (2: no split-K, >= 2 K tiles) | 3 (LDS-DMA ring) | 4 (rotated K loop)");
  FDT_CHECK(kg != 3 || PRO == kProNone, "the LDS-DMA ring is for prologue-free convolutions");
  // header (must match the kernel's hdr) + max(K tiles of every K group, epilogue staging
  // [64][BN + 4] fp32, K-group hand-off [BM*BN] fp32)
  const int nprm = PRO == kProJoin ? 4 : (PRO == kProFold ? 3 : ((PRO == kProAffineAct) ? 2 : 0));
  const size_t hdr = (((size_t)nprm * a.Cx + 4 * (EPI == kEpiJoinBwd ? 3 : 2) * BN + 24) * 4 + 15) & ~(size_t)15;
  const size_t tiles = (kg == 2 ? 2 * 2 : nbuf) * (BM + BN) * BK * 2, stage = (size_t)64 * (BN + 4) * 4;
  const size_t hand = kg == 2 ? (size_t)BM * BN * 4 : 0;
  size_t body = tiles > stage ? tiles : stage;
  if (hand > body) body = hand;
  size_t lds = hdr + body;
#define FDT_T(BM_, BN_, BK_)                                                              \
  if (BM == BM_ && BN == BN_ && BK == BK_) {                                              \
    if constexpr (PRO == kProNone) {                                                      \
      if (kg == 3) { launch_pure<BM_, BN_, BK_, PRO, EPI, ACT, 3>(a, pure, lds, st); return; } \
    }                                                                                     \
    if (kg == 4) launch_pure<BM_, BN_, BK_, PRO, EPI, ACT, 4>(a, pure, lds, st);          \
    else launch_pure<BM_, BN_, BK_, PRO, EPI, ACT, 1>(a, pure, lds, st);                  \
    return;                                                                               \
  }
  // two K groups: the tiles the small-M (latency-bound, ~256-workgroup) layers use
#define FDT_T2(BM_, BN_, BK_)                                                                   \
  if (BM == BM_ && BN == BN_ && BK == BK_) {                                                   \
    if constexpr (PRO == kProNone) {                                                           \
      if (kg == 3) { launch_pure<BM_, BN_, BK_, PRO, EPI, ACT, 3>(a, pure, lds, st); return; }  \
    }                                                                                          \
    if (kg == 2) launch_pure<BM_, BN_, BK_, PRO, EPI, ACT, 2>(a, pure, lds, st);              \
    else if (kg == 4) launch_pure<BM_, BN_, BK_, PRO, EPI, ACT, 4>(a, pure, lds, st);         \
    else launch_pure<BM_, BN_, BK_, PRO, EPI, ACT, 1>(a, pure, lds, st);                      \
    return;                                                                                    \
  }
  // (K groups at 128x64x128 / 64x128x128 spill with the two-operand prologues under the
  // 256-VGPR budget of 8-wave workgroups: those tiles stay single-group)
  FDT_CHECK(kg != 2 || BK == 64 || (BM == 64 && BN == 64), "K groups: unsupported tile");
  FDT_T2(128, 128, 64) FDT_T2(128, 64, 64) FDT_T2(64, 128, 64) FDT_T2(64, 64, 64) FDT_T(256, 64, 64)
  FDT_T(128, 128, 32) FDT_T(128, 64, 32) FDT_T(64, 128, 32) FDT_T(64, 64, 32) FDT_T(256, 128, 32)
  // BK = 128: half the K-loop trips for the latency-bound small-M layers (8x8 / 4x4 stages at
  // the 8-GPU per-GPU batch), twice the bytes in flight per prefetch stage
  FDT_T2(64, 64, 128) FDT_T(128, 64, 128) FDT_T(64, 128, 128)
  // one 256-wide output-channel tile for the join prologue: each joined row is computed and
  // stored once (with two column tiles every tile re-reads both join operands)
  if constexpr (PRO == kProJoin) {
    FDT_T(64, 256, 64) FDT_T(128, 256, 32) FDT_T(128, 256, 64)
  }
#undef FDT_T
#undef FDT_T2
  FDT_CHECK(false, "unsupported conv tile");
}


// (PRO, EPI, ACT) case groups, each instantiated in its own translation unit so the
// kernel matrix compiles in parallel (conv_igemm_inst_*.hip)
bool launch_cases_fwd(int pro, int epi, int act, const ConvArgs& a, int BM, int BN, int BK, int kg, bool pure,
                      hipStream_t st);
bool launch_cases_fold(int pro, int epi, int act, const ConvArgs& a, int BM, int BN, int BK, int kg, bool pure,
                       hipStream_t st);
bool launch_cases_join(int pro, int epi, int act, const ConvArgs& a, int BM, int BN, int BK, int kg, bool pure,
                       hipStream_t st);
bool launch_cases_plain(int pro, int epi, int act, const ConvArgs& a, int BM, int BN, int BK, int kg, bool pure,
                        hipStream_t st);
bool launch_cases_ffn(int pro, int epi, int act, const ConvArgs& a, int BM, int BN, int BK, int kg, bool pure,
                      hipStream_t st);
// halo-staged 3x3 stride-1 main loop (conv_h3.hip): kg 5 register-staged, kg 6 LDS-DMA (two
// stages), kg 7 LDS-DMA single stage (two workgroups per CU), kg 8 LDS-DMA two stages, 16 waves
bool h3_supported(const ConvArgs& a, int BM);
bool launch_h3(int pro, int epi, int act, const ConvArgs& a, int BM, int BN, int kg, hipStream_t st);

}  // namespace conv
}  // namespace fdt
