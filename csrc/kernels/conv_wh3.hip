// Weight gradient of the 3x3 stride-1 convolutions with a halo-staged input operand
// (MI355X / gfx950).
//
//   dW[co][t][ci] = sum_p  g[p][co] * x[p + off(t)][ci],   off(t) = (kh - 1, kw - 1)
//
// The implicit-GEMM weight gradient (conv_wgrad.hip) treats K = (tap, ci) as the GEMM's N
// dimension: every 32-pixel tile re-gathers the input once per tap (9x from L2), and the 3x3
// layers sat at 22-27 % of their bound at batch 1024 (profiles/pmc/r5_bs1024_roofline.md).
// Here a workgroup owns BMC output channels x BNC input channels x ALL NINE taps and walks its
// pixel range in 128-pixel chunks (whole image rows, or whole small images -- the halo loop's
// geometry, conv_h3.hip).  Per chunk it stages
//   * the gradient rows [128 px][BMC co] (16-B chunks XOR-swizzled by pixel row), and
//   * the zero-padded halo of those pixels' inputs [halo rows][BNC ci] ONCE for all nine taps:
//     tap t of pixel p is halo row q(p) + off(t), a constant shift,
// register-staged one chunk ahead into a double-buffered LDS ring.  Each of the 4 waves owns
// one 32 x 32 (co, ci) block and its nine tap accumulators: per 16 pixels it reads one gradient
// fragment and nine shifted input fragments with the gfx950 transposing LDS read
// (ds_read_b64_tr_b16: the reduction runs over pixels, which are LDS rows) and issues nine
// independent mfma_f32_32x32x16_bf16.  The input bytes moved per FLOP drop ~9x against the
// im2col staging; the gradient tile is read once per (co, ci) block pair as before.
//
// Pixels are split over workgroups (split-K); each split writes its fp32 [Cout][9*Cx] slab
// (slab column t*Cx + ci, the layout of conv_wgrad.hip) and wgrad_reduce sums the splits in a
// fixed order into the OIHW gradient: deterministic.  The grid is XCD-mapped so the (co, ci)
// tiles of one pixel split run on one XCD and share its L2 copy of the chunk.
//
// Operands are the engine's materialised 3x3 operands: the folded output gradient and the
// normalised + activated input (no prologue arithmetic in this loop).
//
// Reference semantics: the conv2d weight gradient of resnet.py:21-34 (FusedConvBN backward).
#include "conv_igemm_impl.h"

namespace fdt {
namespace conv {

typedef short bf16x4w_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4w_t lds_bf16x4w;

constexpr int kWh3Px = 128;                 // pixels per chunk
constexpr int kWh3HaloMax = kWh3Px / 16 * 36;  // 8 images of 4x4 -> 8 blocks of 6x6 halo rows
// halo row stride (bf16 elements): 64-B rows as they are (4 consecutive rows = 4 distinct bank
// sixteens), 128-B rows padded to 144 B (4 consecutive rows -> bank offsets 0 / 36 / 8 / 44): a
// tap then stays a constant byte shift of every fragment address
template <int BNC>
constexpr int wh3_xs() { return BNC == 64 ? 72 : BNC; }

struct Wh3Args {
  const bf16* g;   // [M][Cout]
  const bf16* x;   // [N][H][W][Cx]
  float* slab;     // [nsplit][Cout][9 * Cx]
  int H, W, Cx, Cout;
  int lw, lrb, Rb, bhr, HR;  // geometry (W, Rb * W powers of two)
  int nbco, nbci, nsplit, nchunks, cps;  // tiles, splits, chunks, chunks per split
  long g_bytes, x_bytes;
};

// 16-B chunk swizzle of a gradient-tile row of RB bytes (conflict-free transposing reads of 4
// consecutive rows): 256-B rows by row & 3, 128-B rows by row bit 1
template <int RB>
__device__ __forceinline__ int wh3_swz(int row) {
  if constexpr (RB == 256) return 4 * (row & 3);
  else if constexpr (RB == 128) return 4 * ((row >> 1) & 1);
  else return 0;
}

// CPW: 32-row output-channel blocks per wave (each fragment read then feeds more MFMAs; CPW = 2
// needs 288 accumulator registers and spilled ~350 VGPRs: only CPW = 1 is instantiated); PIPE:
// register double-buffered fragments across 16-pixel steps (measured at the final register
// allocation: slower on every tile, profiles/r6/wh3_ts*_p*_*.txt -- opt-in)
// TS: waves per (co, ci) block, each holding ceil(9 / TS) of the nine tap accumulators (TS = 2:
// eight waves, two per SIMD -- one wave's LDS reads under the other's MFMAs -- at <= 256
// registers each)
template <int BMC, int BNC, int CPW, bool PIPE, int TS = 1>
__global__ __launch_bounds__(256 * TS, 1) void wh3_kernel(const Wh3Args a) {
  static_assert((BMC / 32 / CPW) * (BNC / 32) == 4, "four (co, ci) block groups of CPW x 1 32 x 32 blocks");
  static_assert(TS == 1 || CPW == 1, "tap split: one co block per wave");
  constexpr int NTH = 256 * TS;             // threads
  constexpr int TPW = (9 + TS - 1) / TS;    // tap accumulators per wave
  constexpr int GT = kWh3Px * BMC;         // gradient tile, bf16 elements
  constexpr int XS = wh3_xs<BNC>();
  constexpr int XT = kWh3HaloMax * XS;     // halo tile
  constexpr int GCH = BMC / 8, XCH = BNC / 8;      // 16-B chunks per row
  constexpr int NGP = kWh3Px * GCH / NTH;          // gradient pieces per thread
  constexpr int NXP = (kWh3HaloMax * XCH + NTH - 1) / NTH;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* tiles = reinterpret_cast<bf16*>(smem);  // [2][GT + XT]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ntile = a.nbco * a.nbci;
  const int rid = xcd_remap(blockIdx.x, ntile * a.nsplit);
  const int split = rid / ntile, tile = rid - split * ntile;
  const int bco = tile / a.nbci, bci = tile - bco * a.nbci;
  const int co0 = bco * BMC, ci0 = bci * BNC;
  constexpr int NCP = BMC / 32 / CPW;
  const int blk = wid & 3, t0 = (wid >> 2) * TPW;  // (co, ci) block group; first tap of this wave
  const int cb = (blk % NCP) * CPW, nb = blk / NCP;  // this wave's first co block, its ci block
  const int ntw = 9 - t0 < TPW ? 9 - t0 : TPW;       // taps of this wave (wave-uniform)
  const int c_begin = split * a.cps;
  int c_end = c_begin + a.cps;
  if (c_end > a.nchunks) c_end = a.nchunks;

  const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc((void*)a.g, (short)0, (int)a.g_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, (int)a.x_bytes, 0x00020000);

  const int W = a.W, H = a.H, W2 = W + 2, HW = H * W, Rb = a.Rb, bhr = a.bhr;
  auto halo_row = [&](int p) {
    return (p >> a.lrb) * bhr + (((p >> a.lw) & (Rb - 1)) + 1) * W2 + (p & (W - 1)) + 1;
  };

  // per-thread staging pieces: fixed tile-local coordinates, the chunk moves the base
  uint32_t goffl[NGP];
  int gdst[NGP];
#pragma unroll
  for (int j = 0; j < NGP; ++j) {
    const int i = tid + j * NTH, row = i / GCH, cc = i - row * GCH;
    goffl[j] = ((uint32_t)row * (uint32_t)a.Cout + (uint32_t)(co0 + 8 * cc)) * 2u;
    gdst[j] = row * BMC + 8 * (cc ^ wh3_swz<BMC * 2>(row));
  }
  // halo piece j: packed (block b, halo row hr, halo column hc, chunk cc) of the tile, -1 past it
  int xpk[NXP], xdst[NXP];
#pragma unroll
  for (int j = 0; j < NXP; ++j) {
    const int i = tid + j * NTH, q = i / XCH, cc = i - q * XCH;
    const bool v = q < a.HR;
    const int b = q / bhr, r2 = q - b * bhr, hr = r2 / W2, hc = r2 - hr * W2;
    xpk[j] = v ? (b | (hr << 4) | (hc << 10) | (cc << 17)) : -1;
    xdst[j] = v ? q * XS + 8 * cc : -1;
  }

  uint4 rgv[NGP], rxv[NXP];
  auto gload = [&](int c) {
    const uint32_t pb = (uint32_t)c * (uint32_t)kWh3Px * (uint32_t)a.Cout * 2u;
#pragma unroll
    for (int j = 0; j < NGP; ++j) rgv[j] = ld_buf16(rg, pb + goffl[j]);
    const int P0 = c * kWh3Px;
    const int img0 = P0 / HW, h0 = (P0 >> a.lw) & (H - 1);
#pragma unroll
    for (int j = 0; j < NXP; ++j) {
      uint32_t off = kOOB;
      const int pk = xpk[j];
      if (pk >= 0) {
        const int b = pk & 15, hr = (pk >> 4) & 63, hc = (pk >> 10) & 127, cc = pk >> 17;
        const int hh = h0 + hr - 1, ww = hc - 1;
        if ((unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W)
          off = ((uint32_t)((img0 + b) * HW + hh * W + ww) * (uint32_t)a.Cx + (uint32_t)(ci0 + 8 * cc)) * 2u;
      }
      rxv[j] = ld_buf16(rx, off);
    }
  };
  auto lstore = [&](int buf) {
    bf16* Gl = tiles + buf * (GT + XT);
    bf16* Xl = Gl + GT;
#pragma unroll
    for (int j = 0; j < NGP; ++j) *reinterpret_cast<uint4*>(Gl + gdst[j]) = rgv[j];
#pragma unroll
    for (int j = 0; j < NXP; ++j)
      if (xdst[j] >= 0) *reinterpret_cast<uint4*>(Xl + xdst[j]) = rxv[j];
  };

  f32x16 acc[CPW][TPW];
#pragma unroll
  for (int i = 0; i < CPW; ++i)
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][t][r] = 0.f;

  // transposed fragment reads (conv_wgrad.hip): lane (gq, gp) of a 16-lane group supplies row
  // gq's 4 columns 4gp..4gp+3; lane l receives column l & 31, rows 8h..8h+7 of the 16-row step
  const int gq = (lane & 15) >> 2, gp = lane & 3, h = lane >> 5;
  const int colg = ((lane >> 4) & 1) * 16;
  const int gcol = cb * 32 + colg + 4 * gp, xcol = nb * 32 + colg + 4 * gp;
  int toff[TPW];  // a tap = a constant element shift of the halo fragment addresses
#pragma unroll
  for (int tt = 0; tt < TPW; ++tt) {
    const int t = t0 + tt;
    toff[tt] = ((t / 3 - 1) * W2 + (t % 3 - 1)) * XS;
  }
  // halo fragment addresses of this lane's pixels (tap (1, 1)), per 16-pixel step: rows r0, r0 + 4
  int hq[kWh3Px / 16][2];
#pragma unroll
  for (int ks = 0; ks < kWh3Px / 16; ++ks) {
    const int r0 = ks * 16 + 8 * h + gq;
    hq[ks][0] = halo_row(r0) * XS + xcol;
    hq[ks][1] = halo_row(r0 + 4) * XS + xcol;
  }

  // Fragments double-buffered in registers across the 16-pixel steps: step ks+1's ten reads are
  // issued before step ks's nine MFMAs (sched_barrier pins the order), so their LDS latency hides
  // behind the MFMAs of the one wave per SIMD (the default schedule issued each read just before
  // its MFMA and waited on it).
  auto compute = [&](int buf) {
    const bf16* Gl = tiles + buf * (GT + XT);
    const bf16* Xl = Gl + GT;
    constexpr int NSL = PIPE ? 2 : 1;
    bf16x8_t af[NSL][CPW], bfv[NSL][TPW];
    auto fetch = [&](int ks, int sl) {
      const int r0 = ks * 16 + 8 * h + gq, r1 = r0 + 4;
#pragma unroll
      for (int i = 0; i < CPW; ++i) {
        const int col = gcol + 32 * i;
        const bf16* p0 = Gl + r0 * BMC + 8 * ((col >> 3) ^ wh3_swz<BMC * 2>(r0)) + (col & 7);
        const bf16* p1 = Gl + r1 * BMC + 8 * ((col >> 3) ^ wh3_swz<BMC * 2>(r1)) + (col & 7);
        const bf16x4w_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4w*)(p0));
        const bf16x4w_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4w*)(p1));
        af[sl][i] = bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const bf16* p0 = Xl + hq[ks][0] + toff[t];
        const bf16* p1 = Xl + hq[ks][1] + toff[t];
        const bf16x4w_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4w*)(p0));
        const bf16x4w_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4w*)(p1));
        bfv[sl][t] = bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
    };
    auto mma = [&](int sl) {
#pragma unroll
      for (int t = 0; t < TPW; ++t)
#pragma unroll
        for (int i = 0; i < CPW; ++i)
          if (TS == 1 || t < ntw)  // (the last wave of a tap split holds fewer taps)
            acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[sl][i], bfv[sl][t], acc[i][t], 0, 0, 0);
    };
    if constexpr (PIPE) {
      // step ks+1's reads issued before step ks's MFMAs (sched_barrier pins the order): their
      // LDS latency hides behind the MFMAs of the one wave per SIMD
      fetch(0, 0);
#pragma unroll
      for (int ks = 0; ks < kWh3Px / 16; ++ks) {
        const int sl = ks & 1;
        if (ks + 1 < kWh3Px / 16) fetch(ks + 1, sl ^ 1);
        __builtin_amdgcn_sched_barrier(0);
        mma(sl);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < kWh3Px / 16; ++ks) {
        fetch(ks, 0);
        mma(0);
      }
    }
  };

  if (c_begin < c_end) {
    gload(c_begin);
    lstore(0);
    if (c_begin + 1 < c_end) gload(c_begin + 1);
    __syncthreads();
    for (int c = c_begin; c < c_end; ++c) {
      const int buf = (c - c_begin) & 1;
      compute(buf);
      if (c + 1 < c_end) {
        lstore(buf ^ 1);  // buffer buf^1 was last read in chunk c-1, before the previous barrier
        if (c + 2 < c_end) gload(c + 2);
      }
      __syncthreads();
    }
  }

  // epilogue: this split's slab, column t*Cx + ci; accumulator row co = (r&3) + 8(r>>2) + 4h,
  // column ci = lane & 31
  float* dst = a.slab + (long)split * a.Cout * 9 * a.Cx;
  const int ci = ci0 + nb * 32 + (lane & 31);
#pragma unroll
  for (int i = 0; i < CPW; ++i)
#pragma unroll
    for (int t = 0; t < TPW; ++t)
      if (TS == 1 || t < ntw) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int co = co0 + (cb + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          dst[((long)co * 9 + t0 + t) * a.Cx + ci] = acc[i][t][r];
        }
      }
}

}  // namespace conv

// Host: shapes checked here (the kernel trusts them).  Returns the number of pixel splits used
// (the slab holds nsplit x Cout x 9*Cx floats).
void conv_wgrad_h3(uint64_t g, uint64_t x, uint64_t slab, int N, int H, int W, int Cx, int Cout, int BMC, int BNC,
                   int nsplit, int pipe, uint64_t stream) {
  using namespace conv;
  auto ispow2 = [](int v) { return v > 0 && (v & (v - 1)) == 0; };
  FDT_CHECK(ispow2(W) && ispow2(H) && W >= 4 && H >= 4, "wgrad_h3: power-of-two image >= 4x4");
  FDT_CHECK((BMC == 128 && BNC == 32) || (BMC == 64 && BNC == 64), "wgrad_h3: tile (128, 32) or (64, 64)");
  FDT_CHECK(Cout % BMC == 0 && Cx % BNC == 0, "wgrad_h3: channels a multiple of the tile");
  const long M = (long)N * H * W;
  FDT_CHECK(M % kWh3Px == 0, "wgrad_h3: pixel count a multiple of 128");
  Wh3Args a{};
  a.g = P<const bf16>(g);
  a.x = P<const bf16>(x);
  a.slab = P<float>(slab);
  a.H = H; a.W = W; a.Cx = Cx; a.Cout = Cout;
  a.lw = 31 - __builtin_clz((unsigned)W);
  a.Rb = H < kWh3Px / W ? H : kWh3Px / W;
  a.lrb = 31 - __builtin_clz((unsigned)(a.Rb * W));
  a.bhr = (a.Rb + 2) * (W + 2);
  a.HR = (kWh3Px / (a.Rb * W)) * a.bhr;
  FDT_CHECK(a.HR <= kWh3HaloMax, "wgrad_h3: halo exceeds the LDS tile");
  FDT_CHECK(a.Rb == H || (H % a.Rb == 0), "wgrad_h3: whole row blocks");
  a.nbco = Cout / BMC;
  a.nbci = Cx / BNC;
  a.nchunks = (int)(M / kWh3Px);
  FDT_CHECK(nsplit >= 1 && nsplit <= a.nchunks, "wgrad_h3: 1 <= nsplit <= chunks");
  a.cps = (a.nchunks + nsplit - 1) / nsplit;
  a.nsplit = (a.nchunks + a.cps - 1) / a.cps;
  FDT_CHECK(a.nsplit == nsplit, "wgrad_h3: nsplit must divide the chunks evenly enough (host computes it)");
  a.g_bytes = M * Cout * 2;
  a.x_bytes = M * Cx * 2;
  FDT_CHECK(a.g_bytes < 0x7FFFFFF0L && a.x_bytes < 0x7FFFFFF0L, "wgrad_h3: operand exceeds the descriptor range");
  const size_t lds = (size_t)2 * (kWh3Px * BMC + kWh3HaloMax * (BNC == 64 ? 72 : BNC)) * 2;
  const int grid = a.nbco * a.nbci * a.nsplit;
  hipStream_t st = as_stream(stream);
#define FDT_WH3(BMC_, BNC_, CPW_, PIPE_, TS_)                                                             \
  if (BMC == BMC_ && BNC == BNC_ && (pipe & 1) == PIPE_ && ts == TS_) {                                  \
    auto k = wh3_kernel<BMC_, BNC_, CPW_, PIPE_, TS_>;                                                   \
    static bool attr = false;                                                                            \
    if (!attr) {                                                                                         \
      FDT_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(k),                                \
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));          \
      attr = true;                                                                                       \
    }                                                                                                    \
    hipLaunchKernelGGL(k, dim3(grid), dim3(256 * TS_), lds, st, a);                                      \
    FDT_LAUNCH_CHECK();                                                                                  \
    return;                                                                                              \
  }
  const int ts = (pipe & 4) ? 2 : 1;
  // (the tap split with pipelined fragments computed wrong results: not instantiated)
  FDT_CHECK(ts == 1 || (pipe & 1) == 0, "wgrad_h3: the tap split runs without the fragment pipeline");
  FDT_WH3(128, 32, 1, false, 1)
  FDT_WH3(128, 32, 1, true, 1)
  FDT_WH3(64, 64, 1, false, 1)
  FDT_WH3(64, 64, 1, true, 1)
  FDT_WH3(128, 32, 1, false, 2)
  FDT_WH3(64, 64, 1, false, 2)
#undef FDT_WH3
}

}  // namespace fdt
