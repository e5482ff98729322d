// Weight gradient of the NHWC implicit-GEMM convolutions (gfx950 / CDNA4), plus the
// per-step weight packing kernel.
//
//   dW[co][k] = sum_px  G~[px][co] * A[px][k],   k = (tap, ci)
//   G~ = g*gs[co] + alpha[co] + beta[co]*y   (batch-norm backward correction, PRO_FOLD;
//        gs = nullptr means 1)
//   A  = act(x*s + t) at the tap's input pixel (zero outside the image)
//
// Both operands are pixel-major in HBM with channels contiguous, and the reduction runs
// over pixels, so each 32-pixel K tile is staged [px][ch] (16-B channel chunks, an XOR
// swizzle on the chunk index keyed by the pixel row) and the MFMA fragments are read
// with the gfx950 transposing LDS read ds_read_b64_tr_b16 (two per fragment: pixels
// 8h..8h+3 and 8h+4..8h+7 of one channel column), conflict-free per 32-lane half.
// mfma_f32_32x32x16_bf16, 256 threads (2 x 2 waves), double-buffered LDS with
// register-staged prefetch, one barrier per K tile.  The pixel range is split over
// blockIdx.z; each split writes an fp32 slab that `wgrad_reduce` sums (fixed order ->
// deterministic) into the fp32 OIHW gradient of the flat gradient buffer.
//
// Reference semantics: the conv2d(X^T, g^T) weight gradient of resnet.py:21-34 and the
// autograd of nn.Conv2d for the strided convolutions.
#include "common.h"
#include "pack_layout.h"
#include <vector>
#include <algorithm>

namespace fdt {
namespace wg {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef short bf16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) bf16x4_t lds_bf16x4;

struct WgArgs {
  const bf16* g;     // [M][Cout]  gradient wrt conv output (pre-correction)
  const bf16* y;     // [M][Cout]  conv output (for the correction)
  const float* al;   // alpha [Cout]  (nullptr: no correction)
  const float* be;   // beta  [Cout]
  const float* gs;   // gradient scale [Cout] (nullptr: 1)
  const bf16* x;     // [Nb][Hi][Wi][Cx]  conv input (raw)
  const float* xs;   // s [Cx] (nullptr: identity input transform)
  const float* xt;   // t [Cx]
  float* slab;       // [nsplit][Cout][ldw]; direct: the fp32 OIHW gradient itself
  float* slab_out;   // fused_reduce: the fp32 OIHW gradient
  int direct;        // 1x1, Cx == Cin: every split atomically adds into the gradient (no reduce)
  long M;            // Nb*Ho*Wo
  int Hi, Wi, Cx, log2Cx, Ho, Wo, S, log2Ho, log2Wo;
  int ntaps, Cout, ldw, act;
  float act_alpha;
  int nbm, nbn, nsplit;
  long px_per_split;  // multiple of BK
  int8_t dh[12], dw[12];
  long g_bytes, x_bytes;  // buffer-descriptor ranges
  // split-K combined in-kernel (few splits, slab-reduced layers): the partial tiles go to the
  // slab in register order with write-through stores, the last of a tile's splits to arrive
  // (ticket in cnt[tile]) sums them and writes the OIHW gradient -- no wgrad_reduce launch
  int* cnt;          // tickets [tiles], zero between launches (reset by each last arriver)
  int fused_reduce, accumulate, det, Cin;
};

__device__ __forceinline__ void wst16_sc1(__amdgpu_buffer_rsrc_t r, uint32_t byte_off, float4 v) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  u32x4 u = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
  __builtin_amdgcn_raw_buffer_store_b128(u, r, byte_off, 0, 16);
}
__device__ __forceinline__ float4 wld16_sc1(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  auto v = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 16);
  return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
}

__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
  const int q = nblk >> 3, r = nblk & 7, xcd = bid & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// chunk swizzle for a [32 px][RB bytes] tile: conflict-free ds_read_b64_tr_b16
template <int RB>
__device__ __forceinline__ int tswz(int px) {
  if constexpr (RB == 256) return 4 * (px & 3);
  else return 4 * ((px >> 1) & 1);
}

template <int ACT>
__device__ __forceinline__ float wactf(float z, float alpha, float inv_alpha) {
  if constexpr (ACT == kActRelu) return fmaxf(z, 0.f);
  else if constexpr (ACT == kActCelu) return z > 0.f ? z : alpha * (__expf(z * inv_alpha) - 1.f);
  else return z;
}

__device__ __forceinline__ uint4 wld16(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  auto v = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0);
  return *reinterpret_cast<uint4*>(&v);
}
constexpr uint32_t kWOOB = 0xFFFFFFF0u;

// ADDR: 0 = 1x1 stride-1 (input pixel == output pixel), 1 = power-of-two Ho/Wo (shifts),
//       2 = general (integer division).  ACT: input transform act(x*s+t) (XAFF only).
// NS: register-staged K tiles in flight (the prefetch distance).  2 for the big tiles; the
// small tiles of the small-batch layers (a 64 x 64 tile has 2 MFMAs per wave per 32-pixel K
// tile: latency-bound per iteration, ~1 us each at batch 128) keep 4 in flight.
template <int BM, int BN, int BK, bool FOLD, bool XAFF, int ADDR, int ACT, int NS = 2>
__global__ __launch_bounds__(256) void wgrad_kernel(const WgArgs a) {
  static_assert(NS >= 2 && NS % 2 == 0, "even number of register stages (static LDS buffer parity)");
  constexpr int GC = BM / 8, XC = BN / 8;      // 16-B chunks per LDS row
  constexpr int GR = 256 / GC, XR = 256 / XC;  // rows per load round
  constexpr int NG = BK / GR, NX = BK / XR;    // chunks per thread per tile
  constexpr int TM = BM / 64, TN = BN / 64;
  constexpr int GT = BK * BM, XT = BK * BN;
  static_assert(NG >= 1 && NX >= 1, "bad wgrad tile");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* tiles = reinterpret_cast<bf16*>(smem);  // [2][GT + XT]
  float* prm = reinterpret_cast<float*>(smem + 2 * (GT + XT) * 2);  // al|be|gs [BM] , xs|xt [Cx]
  int* tapt = reinterpret_cast<int*>(prm + 3 * BM + (XAFF ? 2 * a.Cx : 0));

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wn = wid & 1, wm = wid >> 1;
  const int nt = a.nbm * a.nbn;
  const int id = xcd_remap(blockIdx.x, nt);
  const int bn = id % a.nbn, bm = id / a.nbn;
  const int co0 = bm * BM, k0 = bn * BN;
  const int p_begin = (int)((long)blockIdx.y * a.px_per_split);
  int p_end = (int)(p_begin + a.px_per_split);
  if ((long)p_end > a.M) p_end = (int)a.M;

  const __amdgpu_buffer_rsrc_t rg_d = __builtin_amdgcn_make_buffer_rsrc((void*)a.g, (short)0, (int)a.g_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ry_d =
      __builtin_amdgcn_make_buffer_rsrc((void*)(FOLD ? a.y : a.g), (short)0, (int)a.g_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rx_d = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, (int)a.x_bytes, 0x00020000);

  if constexpr (FOLD) {
    for (int i = tid; i < BM; i += 256) {
      prm[i] = a.al[co0 + i];
      prm[BM + i] = a.be[co0 + i];
      prm[2 * BM + i] = a.gs ? a.gs[co0 + i] : 1.f;
    }
  }
  if constexpr (XAFF) {
    for (int i = tid; i < a.Cx; i += 256) { prm[3 * BM + i] = a.xs[i]; prm[3 * BM + a.Cx + i] = a.xt[i]; }
  }
  if (tid < 12) tapt[tid] = (int)(uint8_t)a.dh[tid] | ((int)(uint8_t)a.dw[tid] << 8);

  // per-thread fixed chunk columns
  const int gcc = tid % GC, xcc = tid % XC;
  // X chunk column -> (tap, ci) for this block's k columns (fixed across K tiles)
  const int kx = k0 + xcc * 8;
  const int xtap = kx >> a.log2Cx, xci = kx & (a.Cx - 1);
  const bool xtok = xtap < a.ntaps;
  __syncthreads();
  int xdh = 0, xdw = 0;
  if (xtok) {
    const int e = tapt[xtap];
    xdh = (int)(int8_t)(e & 0xff);
    xdw = (int)(int8_t)((e >> 8) & 0xff);
  }
  const int xtoff = xdh * a.Wi + xdw;
  float xsv[8], xtv[8];
  if constexpr (XAFF) {
#pragma unroll
    for (int q = 0; q < 8; ++q) { xsv[q] = prm[3 * BM + xci + q]; xtv[q] = prm[3 * BM + a.Cx + xci + q]; }
  }
  float alv[8], bev[8], gsv[8];
  if constexpr (FOLD) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      alv[q] = prm[gcc * 8 + q];
      bev[q] = prm[BM + gcc * 8 + q];
      gsv[q] = prm[2 * BM + gcc * 8 + q];
    }
  }
  const float inv_alpha = ACT == kActCelu ? 1.f / a.act_alpha : 1.f;
  const int hw = a.Ho * a.Wo;
  const int lw = a.log2Wo, lhw = a.log2Wo + a.log2Ho;

  struct Stage {
    uint4 rg[NG], ry[FOLD ? NG : 1], rx[NX];
    bool xv[NX];
  };

  // Unconditional issue (a tile past the split end reads the OOB offset -> zeros): no branch
  // around a load, so hipcc counts the two in-flight stages exactly (vmcnt(N), not 0).
  auto load_tile = [&](Stage& S, int pt) {
#pragma unroll
    for (int j = 0; j < NG; ++j) {
      const int p = pt + tid / GC + j * GR;
      const uint32_t off = p < p_end ? ((uint32_t)p * (uint32_t)a.Cout + co0 + gcc * 8) * 2u : kWOOB;
      S.rg[j] = wld16(rg_d, off);
      if constexpr (FOLD) S.ry[j] = wld16(ry_d, off);
    }
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      const int p = pt + tid / XC + j * XR;
      bool v = xtok & (p < p_end);  // bitwise: no short-circuit branch around the load
      uint32_t pix;
      if constexpr (ADDR == 0) {
        pix = (uint32_t)p;
      } else {
        int n, oh, ow;
        if constexpr (ADDR == 1) {
          n = p >> lhw;
          oh = (p >> lw) & (a.Ho - 1);
          ow = p & (a.Wo - 1);
        } else {
          n = p / hw;
          const int rem = p - n * hw;
          oh = rem / a.Wo;
          ow = rem - oh * a.Wo;
        }
        const int ih = oh * a.S + xdh, iw = ow * a.S + xdw;
        v = v & ((unsigned)ih < (unsigned)a.Hi) & ((unsigned)iw < (unsigned)a.Wi);
        pix = (uint32_t)((n * a.Hi + oh * a.S) * a.Wi + ow * a.S + xtoff);
      }
      S.xv[j] = v;
      S.rx[j] = wld16(rx_d, v ? ((pix << a.log2Cx) + xci) * 2u : kWOOB);
    }
  };

  auto store_tile = [&](const Stage& S, int buf) {
    bf16* Gl = tiles + buf * (GT + XT);
    bf16* Xl = Gl + GT;
#pragma unroll
    for (int j = 0; j < NG; ++j) {
      const int row = tid / GC + j * GR;
      uint4 o = S.rg[j];
      if constexpr (FOLD) {
        // pixels past the split end fold to alpha, but their X rows load as zero, so they
        // contribute nothing to dW
        const uint32_t u[4] = {o.x, o.y, o.z, o.w}, uy[4] = {S.ry[j].x, S.ry[j].y, S.ry[j].z, S.ry[j].w};
        float v[8];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          v[2 * q] = fmaf(bf16_lo(u[q]), gsv[2 * q], fmaf(bev[2 * q], bf16_lo(uy[q]), alv[2 * q]));
          v[2 * q + 1] = fmaf(bf16_hi(u[q]), gsv[2 * q + 1], fmaf(bev[2 * q + 1], bf16_hi(uy[q]), alv[2 * q + 1]));
        }
        o = make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]),
                       pack_bf16x2(v[6], v[7]));
      }
      *reinterpret_cast<uint4*>(Gl + row * BM + 8 * (gcc ^ tswz<BM * 2>(row))) = o;
    }
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      const int row = tid / XC + j * XR;
      uint4 o = S.rx[j];
      if constexpr (XAFF) {
        const uint32_t u[4] = {o.x, o.y, o.z, o.w};
        float v[8];
#pragma unroll
        for (int q = 0; q < 4; ++q) { v[2 * q] = bf16_lo(u[q]); v[2 * q + 1] = bf16_hi(u[q]); }
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = wactf<ACT>(fmaf(v[q], xsv[q], xtv[q]), a.act_alpha, inv_alpha);
        o = make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]),
                       pack_bf16x2(v[6], v[7]));
        if (!S.xv[j]) o = make_uint4(0, 0, 0, 0);
      }
      *reinterpret_cast<uint4*>(Xl + row * BN + 8 * (xcc ^ tswz<BN * 2>(row))) = o;
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // transposed fragment read: 16-lane group supplies rows q (lane 4q+p) and columns 4p..4p+3
  const int gq = (lane & 15) >> 2, gp = lane & 3;
  const int h = lane >> 5;
  const int colg = ((lane >> 4) & 1) * 16;  // groups 1/3 -> columns 16..31 of the 32-col subtile
  auto compute = [&](int buf) {
    const bf16* Gl = tiles + buf * (GT + XT);
    const bf16* Xl = Gl + GT;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8_t af[TM], bfv[TN];
      const int r0 = ks * 16 + 8 * h + gq, r1 = r0 + 4;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int col = wm * (BM / 2) + i * 32 + colg + 4 * gp;
        const bf16* p0 = Gl + r0 * BM + 8 * ((col >> 3) ^ tswz<BM * 2>(r0)) + (col & 7);
        const bf16* p1 = Gl + r1 * BM + 8 * ((col >> 3) ^ tswz<BM * 2>(r1)) + (col & 7);
        const bf16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(p0));
        const bf16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(p1));
        af[i] = bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn * (BN / 2) + j * 32 + colg + 4 * gp;
        const bf16* p0 = Xl + r0 * BN + 8 * ((col >> 3) ^ tswz<BN * 2>(r0)) + (col & 7);
        const bf16* p1 = Xl + r1 * BN + 8 * ((col >> 3) ^ tswz<BN * 2>(r1)) + (col & 7);
        const bf16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(p0));
        const bf16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(p1));
        bfv[j] = bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfv[j], acc[i][j], 0, 0, 0);
    }
  };

  const int nkt = p_end > p_begin ? (p_end - p_begin + BK - 1) / BK : 0;
  // register stage i holds K tile t with t % NS == i; the stage stored at iteration k (tile
  // k + 1) is reloaded at once with tile k + 1 + NS
  Stage S[NS];
  if (nkt > 0) {
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      load_tile(S[i], p_begin + i * BK);
      __builtin_amdgcn_sched_barrier(0);  // issue order pinned (exact vmcnt counting)
    }
    store_tile(S[0], 0);
    load_tile(S[0], p_begin + NS * BK);
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
  }
  for (int kt = 0; kt < nkt; kt += NS) {
#pragma unroll
    for (int u = 0; u < NS; ++u) {
      compute(u & 1);
      if (kt + u + 1 >= nkt) break;
      store_tile(S[(u + 1) % NS], (u + 1) & 1);
      __syncthreads();
      load_tile(S[(u + 1) % NS], p_begin + (kt + u + 1 + NS) * BK);
      __builtin_amdgcn_sched_barrier(0);  // keep the prefetch issued ahead of the MFMAs
    }
  }

  // epilogue: C[co][k]: lane column k = lane&31, rows co = (r&3) + 8(r>>2) + 4h
  // direct (1x1 with Cx == Cin: slab row layout == OIHW): fp32 atomics accumulate every
  // split straight into the gradient (each wave instruction = two 128-B row segments);
  // otherwise a plain store into this split's slab for wgrad_reduce.
  if (a.fused_reduce) {
    // ---- split-K combine (same protocol as the conv kernels' split-K, conv_igemm_impl.h)
    constexpr int NR4 = TM * TN * 4;
    __shared__ int last_flag;
    const int tile = bm * a.nbn + bn, split = blockIdx.y;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(reinterpret_cast<float4*>(a.slab) + (long)tile * a.nsplit * NR4 * 256), (short)0,
        (int)(a.nsplit * NR4 * 256 * 16), 0x00020000);
    {
      const uint32_t mine = (uint32_t)((split * NR4 * 256 + tid) * 16);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            wst16_sc1(rs, mine + (uint32_t)(((i * TN + j) * 4 + q) * 256 * 16),
                      make_float4(acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every writing wave drains its write-through stores
    __syncthreads();
    if (tid == 0) {
      const int t = __hip_atomic_fetch_add(&a.cnt[tile], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = t == a.nsplit - 1;
      if (last) __hip_atomic_store(&a.cnt[tile], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last_flag = last;
    }
    __syncthreads();
    if (!last_flag) return;
    if (a.det) {  // fixed summation order whichever split arrived last
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    }
    for (int sp = 0; sp < a.nsplit; ++sp) {
      if (sp == split && !a.det) continue;
      const uint32_t other = (uint32_t)((sp * NR4 * 256 + tid) * 16);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float4 v = wld16_sc1(rs, other + (uint32_t)(((i * TN + j) * 4 + q) * 256 * 16));
            acc[i][j][4 * q] += v.x;
            acc[i][j][4 * q + 1] += v.y;
            acc[i][j][4 * q + 2] += v.z;
            acc[i][j][4 * q + 3] += v.w;
          }
    }
    // OIHW: slab column kk = tap * Cx + ci -> ((co * Cin + ci) * ntaps + tap)
    float* out = a.slab_out;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int kk = k0 + wn * (BN / 2) + j * 32 + (lane & 31);
        const int t = kk >> a.log2Cx, ci = kk & (a.Cx - 1);
        if (kk < a.ldw && t < a.ntaps && ci < a.Cin) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int co = co0 + wm * (BM / 2) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            float* o = out + ((long)co * a.Cin + ci) * a.ntaps + t;
            *o = a.accumulate ? *o + acc[i][j][r] : acc[i][j][r];
          }
        }
      }
    return;
  }
  const bool direct = a.direct != 0;
  float* dst = direct ? a.slab : a.slab + (long)blockIdx.y * a.Cout * a.ldw;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int kk = k0 + wn * (BN / 2) + j * 32 + (lane & 31);
      if (kk < a.ldw) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int co = co0 + wm * (BM / 2) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          if (direct)
            atomicAdd(&dst[(long)co * a.ldw + kk], acc[i][j][r]);
          else
            dst[(long)co * a.ldw + kk] = acc[i][j][r];
        }
      }
    }
}

// slab [nsplit][Cout][ntaps*Cxp] -> fp32 OIHW grad [Cout][Cin][KH][KW] (fixed summation
// order: deterministic).  One workgroup per 64 consecutive slab columns of one output channel:
// 16 column quads (16-B loads) x 16 split lanes, each thread keeping up to 8 independent loads
// in flight (the small-batch splits are many and short: the earlier one-column-per-lane form
// walked them two loads at a time and ran latency-bound, ~1 TB/s), LDS combines the lanes.
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ slab, float* __restrict__ out,
                                                           int nsplit, int Cout, int Cin, int ntaps, int Cxp,
                                                           int accumulate) {
  __shared__ float red[16][65];
  const int ld = ntaps * Cxp;
  const int cblk = (ld + 63) / 64;
  const int co = blockIdx.x / cblk;
  const int c0 = (blockIdx.x - co * cblk) * 64;
  const int q = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const int col = c0 + q * 4;
  const long sstride = (long)Cout * ld;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  auto add = [](float4& x, const float4& y) { x.x += y.x; x.y += y.y; x.z += y.z; x.w += y.w; };
  if (col < ld) {
    const float* p = slab + (long)co * ld + col;
    auto ld4 = [&](int k) { return *reinterpret_cast<const float4*>(p + k * sstride); };
    int k = sl;
    for (; k + 7 * 16 < nsplit; k += 8 * 16) {
      float4 v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = ld4(k + i * 16);
      add(v[0], v[4]); add(v[1], v[5]); add(v[2], v[6]); add(v[3], v[7]);
      add(v[0], v[2]); add(v[1], v[3]);
      add(v[0], v[1]);
      add(a, v[0]);
    }
    for (; k < nsplit; k += 16) add(a, ld4(k));
  }
  red[sl][q * 4 + 0] = a.x;
  red[sl][q * 4 + 1] = a.y;
  red[sl][q * 4 + 2] = a.z;
  red[sl][q * 4 + 3] = a.w;
  __syncthreads();
  if (threadIdx.x < 64) {
    const int c = c0 + threadIdx.x;
    float s = 0.f;
#pragma unroll
    for (int l = 0; l < 16; ++l) s += red[l][threadIdx.x];
    if (c < ld) {
      const int t = c / Cxp, ci = c - t * Cxp;
      if (ci < Cin) {
        const long e = ((long)co * Cin + ci) * ntaps + t;
        out[e] = accumulate ? out[e] + s : s;
      }
    }
  }
}

// The few-split form (nsplit <= 8, Cin a multiple of 64, unpadded channels): one workgroup
// per (output channel, 64-input-channel block); each wave sums all splits of its taps for 64
// consecutive channels (256-B coalesced reads), and the taps x channels block is transposed
// in LDS so the OIHW write -- and the read of an accumulated gradient -- is one contiguous
// run of NT*64 floats.  (The column form above scatters its OIHW stores NT floats apart: at
// 2 splits over the 512-channel 3x3 layers it ran at ~1.5 TB/s.)
template <int NT>
__global__ __launch_bounds__(256) void wgrad_reduce_cm_kernel(const float* __restrict__ slab, float* __restrict__ out,
                                                              int nsplit, int Cout, int Cin, int accumulate) {
  __shared__ float tile[NT * 64 + 1];
  const int cblk = Cin / 64;
  const int co = blockIdx.x / cblk, ci0 = (blockIdx.x - co * cblk) * 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long ld = (long)NT * Cin;
  const long sstride = (long)Cout * ld;
  const float* p = slab + (long)co * ld + ci0 + lane;
#pragma unroll
  for (int t0 = 0; t0 < NT; t0 += 4) {
    const int t = t0 + w;
    if (t < NT) {
      float a = 0.f;
      for (int s = 0; s < nsplit; ++s) a += p[s * sstride + (long)t * Cin];
      tile[lane * NT + t] = a;
    }
  }
  __syncthreads();
  float* o = out + ((long)co * Cin + ci0) * NT;
  for (int i = threadIdx.x; i < 64 * NT; i += 256) o[i] = accumulate ? o[i] + tile[i] : tile[i];
}

// ---------------------------------------------------------------------- weight packing
struct PackEntry {
  const float* src;  // fp32 OIHW
  bf16* wf;          // [Cout][ntaps][Cxp]      (forward)
  bf16* wd;          // [Cin][ntaps][Cout]      (dgrad; nullptr to skip)
  int Cout, Cin, Cxp, ntaps;
  long blk0;          // first block of this entry
};

constexpr int kMaxPack = 64;  // keeps the kernel-argument table under 4 KB
struct PackTable {
  PackEntry e[kMaxPack];
  int n;
};

// One workgroup packs a 32 (co) x 64 (ci) x ntaps block: coalesced fp32 reads of the OIHW
// source (ci, tap contiguous per co; 16 B per lane) into a bf16 LDS image [co][tap][ci], then
// both packed layouts from the image (pack_layout.h, shared with the optimizer's fused
// update-and-pack, optim_pack.hip).
constexpr int kPackCo = pack::kCo;
constexpr int kPackT = pack::kT;
constexpr int kPackLd = pack::kLd;
constexpr int kPackMaxTaps = pack::kMaxTaps;

// T (taps per kernel: 1, 9, ...) is a compile-time constant in the body, so the per-element
// index math is multiplies and shifts instead of integer divisions.
template <int T>
__device__ __forceinline__ void pack_block(const PackEntry& E, int b, bf16* img) {
  const pack::Block k = pack::block_of(b, E.Cout, E.Cin, E.Cxp);
  const int tid = threadIdx.x;
  const int nco = k.nco, nci_s = k.nci_s;
  // load: for each co row the source run [ci0, ci0 + nci_s) x T is contiguous
  constexpr int run = kPackT * T;
  const float* rowp = E.src + ((long)k.co0 * E.Cin + k.ci0) * T;
  if (nci_s == kPackT && ((E.Cin * T) & 3) == 0) {
    // full block, 16-B aligned rows: float4 loads (4 consecutive (ci, t) elements)
    for (int e = tid; e < nco * (run / 4); e += 256) {
      const int col = e / (run / 4), q = (e - col * (run / 4)) * 4;
      const float4 v = *reinterpret_cast<const float4*>(rowp + (long)col * E.Cin * T + q);
      const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int cl = (q + j) / T, t = (q + j) - cl * T;
        img[(col * T + t) * kPackLd + cl] = __float2bfloat16(vv[j]);
      }
    }
  } else {
    for (int e = tid; e < nco * run; e += 256) {
      const int col = e / run, rem = e - col * run;
      const int cl = rem / T, t = rem - cl * T;
      float v = 0.f;
      if (cl < nci_s) v = rowp[(long)col * E.Cin * T + rem];
      img[(col * T + t) * kPackLd + cl] = __float2bfloat16(v);
    }
  }
  __syncthreads();
  pack::store_layouts<T>(img, k, E.wf, E.wd, E.Cout, E.Cxp);
}

__global__ __launch_bounds__(256) void pack_weights_kernel(const PackTable tab) {
  __shared__ bf16 img[kPackCo * kPackMaxTaps * kPackLd];
  // binary search the entry of this block
  int lo = 0, hi = tab.n - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (tab.e[mid].blk0 <= (long)blockIdx.x) lo = mid; else hi = mid - 1;
  }
  const PackEntry& E = tab.e[lo];
  const int b = (int)((long)blockIdx.x - E.blk0);
  if (E.ntaps == 1) pack_block<1>(E, b, img);
  else if (E.ntaps == 9) pack_block<9>(E, b, img);
  else if (E.ntaps == 4) pack_block<4>(E, b, img);
  else pack_block<kPackMaxTaps>(E, b, img);  // unreachable: launcher checks ntaps in {1, 4, 9}
}

}  // namespace wg

void conv_wgrad(uint64_t g, uint64_t y, uint64_t al, uint64_t be, uint64_t gs, uint64_t x, uint64_t xs, uint64_t xt,
                uint64_t slab,
                long Nb, int Hi, int Wi, int Cx, int Ho, int Wo, int S, const std::vector<int>& dh,
                const std::vector<int>& dw, int Cout, int ldw, int act, float act_alpha, int BM, int BN, int BK,
                int nsplit, int direct, int stages, uint64_t out, uint64_t cnt, int Cin, int accumulate,
                uint64_t stream) {
  using namespace wg;
  WgArgs a{};
  // out != 0: combine the splits in-kernel (last arriver) into the OIHW gradient `out`
  a.fused_reduce = out != 0 && nsplit > 1 && !direct;
  a.slab_out = P<float>(out);
  a.cnt = P<int>(cnt);
  a.Cin = Cin;
  a.accumulate = accumulate;
  a.det = deterministic() ? 1 : 0;
  FDT_CHECK(!a.fused_reduce || cnt != 0, "fused wgrad reduce needs a ticket buffer");
  a.g = P<const bf16>(g); a.y = P<const bf16>(y);
  a.al = P<const float>(al); a.be = P<const float>(be);
  a.gs = P<const float>(gs);
  a.x = P<const bf16>(x); a.xs = P<const float>(xs); a.xt = P<const float>(xt);
  a.slab = P<float>(slab);
  a.direct = direct;
  FDT_CHECK(!direct || (dh.size() == 1 && ldw == Cx), "direct wgrad needs a 1x1 conv with ldw == Cx");
  FDT_CHECK(Cx >= 8 && (Cx & (Cx - 1)) == 0, "Cx must be a power of two >= 8");
  FDT_CHECK(Cout % BM == 0, "Cout must be a multiple of BM");
  FDT_CHECK(dh.size() == dw.size() && dh.size() <= 12, "bad tap table");
  FDT_CHECK(nsplit >= 1, "nsplit >= 1");
  FDT_CHECK((al == 0) == (be == 0) && (xs == 0) == (xt == 0), "paired params");
  a.M = Nb * (long)Ho * Wo;
  a.Hi = Hi; a.Wi = Wi; a.Cx = Cx; a.log2Cx = 31 - __builtin_clz((unsigned)Cx);
  a.Ho = Ho; a.Wo = Wo; a.S = S;
  auto ispow2 = [](int v) { return v > 0 && (v & (v - 1)) == 0; };
  a.log2Ho = ispow2(Ho) ? 31 - __builtin_clz((unsigned)Ho) : 0;
  a.log2Wo = ispow2(Wo) ? 31 - __builtin_clz((unsigned)Wo) : 0;
  const int addr = (dh.size() == 1 && dh[0] == 0 && dw[0] == 0 && S == 1 && Hi == Ho && Wi == Wo)
                       ? 0 : ((ispow2(Ho) && ispow2(Wo)) ? 1 : 2);
  a.ntaps = (int)dh.size(); a.Cout = Cout; a.ldw = ldw; a.act = act; a.act_alpha = act_alpha;
  FDT_CHECK(ldw >= a.ntaps * Cx, "ldw too small");
  for (size_t i = 0; i < dh.size(); ++i) { a.dh[i] = (int8_t)dh[i]; a.dw[i] = (int8_t)dw[i]; }
  a.g_bytes = a.M * Cout * 2;
  a.x_bytes = Nb * (long)Hi * Wi * Cx * 2;
  FDT_CHECK(a.g_bytes < 0x7FFFFFF0L && a.x_bytes < 0x7FFFFFF0L, "wgrad operand exceeds the 2 GiB descriptor range");
  a.nbm = Cout / BM;
  a.nbn = (ldw + BN - 1) / BN;
  long per = (a.M + nsplit - 1) / nsplit;
  per = (per + BK - 1) / BK * BK;
  a.px_per_split = per;
  a.nsplit = nsplit;
  const bool fold = al != 0, xaff = xs != 0;
  size_t lds = (size_t)2 * BK * (BM + BN) * 2 + 3 * BM * 4 + (xaff ? 2 * Cx * 4 : 0) + 64;
  dim3 grid(a.nbm * a.nbn, nsplit);
  hipStream_t st = as_stream(stream);
  const int wact = xaff ? act : 0;
  // 4 register stages only where they are instantiated (the small tiles); 2 elsewhere
  const bool deep = stages >= 4 && BM * BN <= 64 * 128 && BK == 32;
#define FDT_WG(BM_, BN_, BK_, F_, X_, A_, ACT_)                                                           \
  if (BM == BM_ && BN == BN_ && BK == BK_ && fold == F_ && xaff == X_ && addr == A_ && wact == ACT_) {  \
    auto k = wgrad_kernel<BM_, BN_, BK_, F_, X_, A_, ACT_, 2>;                                          \
    if constexpr (BM_ * BN_ <= 64 * 128 && BK_ == 32) {                                                 \
      if (deep) k = wgrad_kernel<BM_, BN_, BK_, F_, X_, A_, ACT_, 4>;                                   \
    }                                                                                                   \
    static size_t set = 64 * 1024;                                                                      \
    if (lds > set) {                                                                                    \
      FDT_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(k),                               \
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));         \
      set = lds;                                                                                        \
    }                                                                                                   \
    hipLaunchKernelGGL(k, grid, dim3(256), lds, st, a);                                                 \
    FDT_LAUNCH_CHECK();                                                                                 \
    return;                                                                                             \
  }
#define FDT_WG_A(BM_, BN_, BK_, F_, X_, ACT_) FDT_WG(BM_, BN_, BK_, F_, X_, 0, ACT_) \
  FDT_WG(BM_, BN_, BK_, F_, X_, 1, ACT_) FDT_WG(BM_, BN_, BK_, F_, X_, 2, ACT_)
#define FDT_WG_T(BM_, BN_, BK_) FDT_WG_A(BM_, BN_, BK_, true, true, 1) FDT_WG_A(BM_, BN_, BK_, true, true, 2) \
  FDT_WG_A(BM_, BN_, BK_, true, false, 0) FDT_WG_A(BM_, BN_, BK_, false, false, 0)                          \
  FDT_WG_A(BM_, BN_, BK_, false, true, 1) FDT_WG_A(BM_, BN_, BK_, true, true, 0)
  FDT_WG_T(128, 128, 32)
  FDT_WG_T(64, 128, 32)
  FDT_WG_T(128, 64, 32)
  FDT_WG_T(64, 64, 32)
  FDT_WG_T(128, 128, 64)
  FDT_WG_T(64, 128, 64)
  FDT_WG_T(128, 64, 64)
  FDT_WG_T(64, 64, 64)
#undef FDT_WG_T
#undef FDT_WG_A
#undef FDT_WG
  FDT_CHECK(false, "unsupported wgrad tile");
}

void wgrad_reduce(uint64_t slab, uint64_t out, int nsplit, int Cout, int Cin, int ntaps, int Cxp, int accumulate,
                  uint64_t stream) {
  const int ld = ntaps * Cxp;
  if (ntaps == 9 && Cxp == Cin && Cin % 64 == 0 && nsplit <= 8) {
    hipLaunchKernelGGL(wg::wgrad_reduce_cm_kernel<9>, dim3(Cout * (Cin / 64)), dim3(256), 0, as_stream(stream),
                       P<const float>(slab), P<float>(out), nsplit, Cout, Cin, accumulate);
    FDT_LAUNCH_CHECK();
    return;
  }
  FDT_CHECK(ld % 4 == 0 && slab % 16 == 0, "wgrad_reduce: 16-B aligned slab rows");
  const int grid = Cout * ((ld + 63) / 64);
  hipLaunchKernelGGL(wg::wgrad_reduce_kernel, dim3(grid), dim3(256), 0, as_stream(stream), P<const float>(slab),
                     P<float>(out), nsplit, Cout, Cin, ntaps, Cxp, accumulate);
  FDT_LAUNCH_CHECK();
}

// entries: list of (src, wf, wd, Cout, Cin, Cxp, ntaps); one launch for all of them
void pack_weights(const std::vector<uint64_t>& src, const std::vector<uint64_t>& wf, const std::vector<uint64_t>& wd,
                  const std::vector<int>& cout, const std::vector<int>& cin, const std::vector<int>& cxp,
                  const std::vector<int>& ntaps, uint64_t stream) {
  using namespace wg;
  const size_t n = src.size();
  size_t i = 0;
  while (i < n) {
    PackTable tab{};
    long blk = 0;
    int k = 0;
    for (; i < n && k < kMaxPack; ++i, ++k) {
      PackEntry& E = tab.e[k];
      E.src = P<const float>(src[i]);
      E.wf = P<bf16>(wf[i]);
      E.wd = P<bf16>(wd[i]);
      E.Cout = cout[i]; E.Cin = cin[i]; E.Cxp = cxp[i]; E.ntaps = ntaps[i];
      E.blk0 = blk;
      FDT_CHECK(E.ntaps == 1 || E.ntaps == 4 || E.ntaps == 9, "pack_weights: 1x1, 2x2 or 3x3 kernels");
      FDT_CHECK(E.Cout % 8 == 0 && E.Cxp % 8 == 0, "pack_weights: 16-B packed rows need Cout, Cxp % 8 == 0");
      blk += (long)((E.Cout + kPackCo - 1) / kPackCo) * ((E.Cxp + kPackT - 1) / kPackT);
    }
    tab.n = k;
    if (blk == 0) continue;
    hipLaunchKernelGGL(pack_weights_kernel, dim3((unsigned)blk), dim3(256), 0, as_stream(stream), tab);
    FDT_LAUNCH_CHECK();
  }
}

}  // namespace fdt
