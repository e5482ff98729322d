// Fused multi-head attention for the Transformer classifier (gfx950 / CDNA4), head_dim 64.
//
// Reference: ScaledDotProduct (transformer.py:180-193): softmax(q k^T / sqrt(d_k), key
// padding mask) -> dropout -> @ v, with L <= 512 and B x H = 64 x 8 per GPU.  PyTorch
// materialises the B x H x L x L scores (plus the softmax and dropout masks) in HBM; here
// nothing L x L ever leaves the chip.
//
// Layout: q, k, v are (B, L, H, 64) strided views of the projection outputs (no transpose
// copies); O / dO / dQ / dK / dV are contiguous (B, L, H, 64); the log-sum-exp and
// delta = rowsum(dO * O) are (B, H, L) fp32.  Scores live in the log2 domain
// (x = s * log2(e)/sqrt(d)); exp2 everywhere.
//
// MFMA mapping (mfma_f32_32x32x16_bf16; C[row][col]: col = lane & 31, row = (r&3) + 8(r>>2)
// + 4(lane>>5)): every product is oriented so that the accumulator of the first GEMM is
// already the B operand of the next one (its k index = the accumulator's row index, in the
// permuted order row(j) = 16s + 8(j>>2) + 4h + (j&3)); the other operand is read in that
// same permuted order from the row image itself with the gfx950 transposing LDS read
// (ds_read_b64_tr_b16, two per fragment) -- no transposed copy is staged.
//   forward     S^T = K Q^T (query on the lane -> row max / sum are in-register plus one
//               lane^32 exchange), online softmax, O^T += V^T P^T.          grid (L/128, H, B)
//   bwd dK,dV   S = Q K^T, dP = dO V^T (key on the lane), dV^T += dO^T P, dK^T += Q^T dS:
//               each wave owns 32 keys, the workgroup sweeps all queries.   grid (L/128, H, B)
//   bwd dQ      S^T, dP^T as in forward, dQ^T += K^T dS^T: each wave owns 32 queries,
//               the workgroup sweeps all keys (recomputes P instead of atomics / a dS
//               round trip -- at L <= 512 the kernels are latency-, not FLOP-bound).
// Masking: keys past L are absent; key-padding-masked keys get the fill value (-inf = true
// mask; the reference's -1e-9 fill, survey Q7, is reproduced with fill = -1e-9).  Dropout:
// a counter-based hash of (seed, b, h, q, key) -- the same keep mask in all kernels, no
// mask tensor.
#include "common.h"

namespace fdt {
namespace attn {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef short bf16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kD = 64;
constexpr int kRowLd = kD + 8;  // [row][d] images: 144-B rows -> ds_read_b128 of 16 rows hits 64 distinct banks
constexpr int kBlk = 128;       // queries (fwd, dq) / keys (dkdv) per workgroup: 4 waves x 32
constexpr int kTile = 64;       // keys (fwd, dq) / queries (dkdv) staged per loop iteration

struct Args {
  const bf16* q;
  const bf16* k;
  const bf16* v;
  long qb, ql, qh, kb, kl, kh, vb, vl, vh;  // element strides (batch, position, head); d contiguous
  const bf16* o;                            // forward output [B][L][H][D]
  const bf16* dout;                         // [B][L][H][D]
  bf16* out;
  bf16* dq;
  bf16* dk;
  bf16* dv;
  long gl;  // position stride of dq/dk/dv (H*D contiguous; 3*H*D = packed [B][L][3][H][D])
  const uint8_t* mask;  // [B][L] nonzero = keep; nullptr = no mask
  float* lse;           // [B][H][L] log2-domain log-sum-exp
  float* delta;         // [B][H][L]
  int B, L, H;
  float c2;           // log2(e) / sqrt(D)
  float fill2;        // masked score in the log2 domain (-inf = true mask)
  float scale;        // 1 / sqrt(D)
  uint32_t drop_thr;  // drop iff hash < drop_thr (p * 2^32); 0 = no dropout
  float keep_scale;   // 1 / (1 - p)
  uint64_t seed;
  // optional device word XORed into the seed at kernel start: a HIP-graph replay draws new
  // dropout masks from a per-step seed written before the replay (the kernel argument is
  // frozen at capture)
  const uint64_t* seed_ptr;
};

// keep-mask hash of (bh, q, key) under the per-call seed: 32-bit murmur3 finaliser (two
// 32-bit multiplies; the 64-bit mix it replaces cost ~3x the VALU work per score element)
// (lin = (bh L + q) L + key: the callers form it with adds from per-lane / per-tile bases)
__device__ __forceinline__ bool dropped_lin(const Args& a, uint32_t lin) {
  uint32_t x = lin ^ (uint32_t)a.seed;
  x += (uint32_t)(a.seed >> 32);
  x ^= x >> 16;
  x *= 0x85ebca6bu;
  x ^= x >> 13;
  x *= 0xc2b2ae35u;
  x ^= x >> 16;
  return x < a.drop_thr;
}

// raw v_exp_f32 (exp2f adds a compare / select / ldexp per call for denormal results, which
// probabilities below 2^-126 do not need); exp2(-inf) = 0
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ bf16x8_t ld8(const bf16* p) { return *reinterpret_cast<const bf16x8_t*>(p); }

typedef __attribute__((address_space(3))) bf16x4_t lds_bf16x4;

// Transposed MFMA fragment straight from a ROW image [row][kRowLd] (gfx950 ds_read_b64_tr_b16,
// no transposed LDS copy): lane l gets column c0 + (l & 31) and the k elements = rows
// R..R+3 (lo) and R+8..R+11 (hi), R = r0 + 4h -- the permuted order of the accumulator rows.
// In each 16-lane group lane 4q+p supplies row R+q, columns 16g + 4p..4p+3 (g = (l >> 4) & 1).
__device__ __forceinline__ bf16x8_t ldtr(const bf16* img, int r0, int c0, int lane) {
  const int q = (lane & 15) >> 2, p = lane & 3, g = (lane >> 4) & 1, h = lane >> 5;
  const bf16* p0 = img + (r0 + 4 * h + q) * kRowLd + c0 + 16 * g + 4 * p;
  const bf16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(p0));
  const bf16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(p0 + 8 * kRowLd));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

__device__ __forceinline__ bf16x8_t pack8(const float* v) {
  const uint4 u = make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]),
                             pack_bf16x2(v[6], v[7]));
  return __builtin_bit_cast(bf16x8_t, u);
}

__device__ __forceinline__ f32x16 mfma(bf16x8_t a, bf16x8_t b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// rows [r0, r0 + 64) of a strided [L][64] matrix -> row image [64][kRowLd] (16-B stores;
// transposed operands are read from it with ldtr); rows past L are zero.
__device__ __forceinline__ void stage(bf16* rows, const bf16* src, long ld, int r0, int L, int tid) {
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int c = tid + it * 256;
    const int row = c >> 3, ch = c & 7;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r0 + row < L) v = *reinterpret_cast<const uint4*>(src + (long)(r0 + row) * ld + ch * 8);
    *reinterpret_cast<uint4*>(rows + row * kRowLd + ch * 8) = v;
  }
}

// key-state of key index key: 1 keep, 0 masked (fill), -1 absent (past L)
__device__ __forceinline__ int8_t key_state(const Args& a, int b, int key) {
  if (key >= a.L) return -1;
  return a.mask ? (int8_t)(a.mask[(long)b * a.L + key] != 0) : (int8_t)1;
}

// key state -> (score multiplier, addend, dS factor): the masked log2-domain score is one
// FMA, x = s * mul + add, and dS is zeroed by a multiply instead of per-element selects
__device__ __forceinline__ float4 key_coef(const Args& a, int st) {
  return st > 0 ? make_float4(a.c2, 0.f, 1.f, 0.f)
                : make_float4(0.f, st == 0 ? a.fill2 : -INFINITY, 0.f, 0.f);
}

// log-sum-exp of a fully masked row is -inf: +inf makes exp2(x - lse) = 0 without a select
__device__ __forceinline__ float lse_safe(float l) { return l == -INFINITY ? INFINITY : l; }

// ------------------------------------------------------------------------------ forward
template <bool DROP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void attn_fwd_kernel(Args a) {
  if (a.seed_ptr != nullptr) a.seed ^= *a.seed_ptr;
  __shared__ __attribute__((aligned(16))) bf16 Ks[kTile * kRowLd];
  __shared__ __attribute__((aligned(16))) bf16 Vs[kTile * kRowLd];
  __shared__ __attribute__((aligned(16))) float2 km[kTile];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int b = blockIdx.z, hd = blockIdx.y, bh = b * a.H + hd;
  const int q = blockIdx.x * kBlk + w * 32 + l32;
  const bool qv = q < a.L;
  const bf16* qp = a.q + b * a.qb + (long)(qv ? q : a.L - 1) * a.ql + hd * a.qh;
  bf16x8_t qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = ld8(qp + 16 * s + 8 * h);
  const bf16* kp = a.k + b * a.kb + hd * a.kh;
  const bf16* vp = a.v + b * a.vb + hd * a.vh;
  f32x16 oacc[2];
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) oacc[dt][r] = 0.f;
  float m = -INFINITY, l = 0.f;
  const uint32_t qlin = ((uint32_t)bh * (uint32_t)a.L + (uint32_t)q) * (uint32_t)a.L;

  for (int k0 = 0; k0 < a.L; k0 += kTile) {
    stage(Ks, kp, a.kl, k0, a.L, tid);
    stage(Vs, vp, a.vl, k0, a.L, tid);
    if (tid < kTile) {
      const float4 c = key_coef(a, key_state(a, b, k0 + tid));
      km[tid] = make_float2(c.x, c.y);
    }
    __syncthreads();
    float x[2][16];
    float mb = -INFINITY;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      f32x16 s;
#pragma unroll
      for (int r = 0; r < 16; ++r) s[r] = 0.f;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) s = mfma(ld8(Ks + (32 * t + l32) * kRowLd + 16 * ks + 8 * h), qf[ks], s);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float2 c = km[32 * t + crow(r, h)];
        x[t][r] = fmaf(s[r], c.x, c.y);
        mb = fmaxf(mb, x[t][r]);
      }
    }
    mb = fmaxf(mb, __shfl_xor(mb, 32));
    const float mn = fmaxf(m, mb);
    const float mu = mn == -INFINITY ? 0.f : mn;
    const float alpha = fexp2(m - mu);
    float ls = 0.f;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = fexp2(x[t][r] - mu);
        ls += p;
        x[t][r] = p;
      }
    ls += __shfl_xor(ls, 32);
    l = l * alpha + ls;
    m = mn;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int r = 0; r < 16; ++r) oacc[dt][r] *= alpha;
    if (DROP) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          x[t][r] = dropped_lin(a, qlin + (uint32_t)(k0 + 32 * t + crow(r, h))) ? 0.f : x[t][r] * a.keep_scale;
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int hs = 0; hs < 2; ++hs) {
        const bf16x8_t pb = pack8(&x[t][8 * hs]);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) oacc[dt] = mfma(ldtr(Vs, 32 * t + 16 * hs, 32 * dt, lane), pb, oacc[dt]);
      }
    __syncthreads();
  }

  if (qv) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    bf16* op = a.out + (((long)b * a.L + q) * a.H + hd) * kD;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const uint2 u = make_uint2(pack_bf16x2(oacc[dt][4 * g] * inv, oacc[dt][4 * g + 1] * inv),
                                   pack_bf16x2(oacc[dt][4 * g + 2] * inv, oacc[dt][4 * g + 3] * inv));
        *reinterpret_cast<uint2*>(op + 32 * dt + 8 * g + 4 * h) = u;
      }
    if (h == 0) a.lse[(long)bh * a.L + q] = l > 0.f ? m + log2f(l) : -INFINITY;
  }
}

// ------------------------------------------------------------------------------ backward
// delta[b][h][q] = sum_d dO * O   (one thread per (b, q, h) row of 64)
__global__ __launch_bounds__(256) void attn_bwd_prep_kernel(Args a) {
  const long row = (long)blockIdx.x * 256 + threadIdx.x;
  if (row >= (long)a.B * a.L * a.H) return;
  const bf16* o = a.o + row * kD;
  const bf16* g = a.dout + row * kD;
  float acc = 0.f;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const uint4 uo = *reinterpret_cast<const uint4*>(o + 8 * c);
    const uint4 ug = *reinterpret_cast<const uint4*>(g + 8 * c);
    const uint32_t po[4] = {uo.x, uo.y, uo.z, uo.w}, pg[4] = {ug.x, ug.y, ug.z, ug.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) acc += bf16_lo(po[e]) * bf16_lo(pg[e]) + bf16_hi(po[e]) * bf16_hi(pg[e]);
  }
  const int hd = (int)(row % a.H);
  const long bl = row / a.H;
  const int qpos = (int)(bl % a.L);
  const int b = (int)(bl / a.L);
  a.delta[((long)b * a.H + hd) * a.L + qpos] = acc;
}

// 2 waves / SIMD: without the floor the dropout variant is allocated 183 VGPRs + 96 AGPRs and
// runs one wave per SIMD
template <bool DROP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void attn_bwd_dkdv_kernel(Args a) {
  if (a.seed_ptr != nullptr) a.seed ^= *a.seed_ptr;
  __shared__ __attribute__((aligned(16))) bf16 Qs[kTile * kRowLd];
  __shared__ __attribute__((aligned(16))) bf16 Gs[kTile * kRowLd];  // dO rows
  __shared__ __attribute__((aligned(16))) float lse_s[kTile];
  __shared__ __attribute__((aligned(16))) float del_s[kTile];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int b = blockIdx.z, hd = blockIdx.y, bh = b * a.H + hd;
  const int key = blockIdx.x * kBlk + w * 32 + l32;
  const bool kv = key < a.L;
  const int kc = kv ? key : a.L - 1;
  bf16x8_t kf[4], vf[4];
  {
    const bf16* kp = a.k + b * a.kb + (long)kc * a.kl + hd * a.kh;
    const bf16* vp = a.v + b * a.vb + (long)kc * a.vl + hd * a.vh;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      kf[s] = ld8(kp + 16 * s + 8 * h);
      vf[s] = ld8(vp + 16 * s + 8 * h);
    }
  }
  const float4 kc4 = key_coef(a, key_state(a, b, key));
  const float smul = kc4.x, sadd = kc4.y, dsm = kc4.z;
  // dropout index (bh L + q) L + key for q = q0 + 32 qt + 4h + (r & 3) + 8 (r >> 2): per-tile
  // base + lo[r & 3] + hi[r >> 2] (adds, no per-element 32-bit multiplies)
  const uint32_t Lu = (uint32_t)a.L;
  const uint32_t lo[4] = {0u, Lu, 2u * Lu, 3u * Lu}, hi[4] = {0u, 8u * Lu, 16u * Lu, 24u * Lu};
  const bf16* qbase = a.q + b * a.qb + hd * a.qh;
  const long gl = (long)a.H * kD;  // row stride of the contiguous tensors
  const bf16* gbase = a.dout + (long)b * a.L * gl + hd * kD;
  f32x16 dk[2], dv[2];
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) { dk[dt][r] = 0.f; dv[dt][r] = 0.f; }

  for (int q0 = 0; q0 < a.L; q0 += kTile) {
    stage(Qs, qbase, a.ql, q0, a.L, tid);
    stage(Gs, gbase, gl, q0, a.L, tid);
    if (tid < kTile) {
      const int qq = q0 + tid;
      lse_s[tid] = qq < a.L ? lse_safe(a.lse[(long)bh * a.L + qq]) : INFINITY;
      del_s[tid] = qq < a.L ? a.delta[(long)bh * a.L + qq] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      f32x16 S, dP;
#pragma unroll
      for (int r = 0; r < 16; ++r) { S[r] = 0.f; dP[r] = 0.f; }
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        S = mfma(ld8(Qs + (32 * qt + l32) * kRowLd + 16 * ks + 8 * h), kf[ks], S);
        dP = mfma(ld8(Gs + (32 * qt + l32) * kRowLd + 16 * ks + 8 * h), vf[ks], dP);
      }
      float p[16], ds[16], lv[16], dv16[16];
      const uint32_t tlin = ((uint32_t)bh * Lu + (uint32_t)(q0 + 32 * qt + 4 * h)) * Lu + (uint32_t)key;
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {  // rows crow(4 g4 + j, h) = 32 qt + 8 g4 + 4h + j: one float4
        const float4 l4 = *reinterpret_cast<const float4*>(lse_s + 32 * qt + 8 * g4 + 4 * h);
        const float4 d4 = *reinterpret_cast<const float4*>(del_s + 32 * qt + 8 * g4 + 4 * h);
        lv[4 * g4] = l4.x; lv[4 * g4 + 1] = l4.y; lv[4 * g4 + 2] = l4.z; lv[4 * g4 + 3] = l4.w;
        dv16[4 * g4] = d4.x; dv16[4 * g4 + 1] = d4.y; dv16[4 * g4 + 2] = d4.z; dv16[4 * g4 + 3] = d4.w;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float pv = fexp2(fmaf(S[r], smul, sadd) - lv[r]);
        float z = 1.f;
        if (DROP) z = dropped_lin(a, tlin + lo[r & 3] + hi[r >> 2]) ? 0.f : a.keep_scale;
        p[r] = pv * z;
        ds[r] = dsm * pv * (dP[r] * z - dv16[r]);
      }
#pragma unroll
      for (int hs = 0; hs < 2; ++hs) {
        const bf16x8_t pb = pack8(&p[8 * hs]);
        const bf16x8_t sb = pack8(&ds[8 * hs]);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          dv[dt] = mfma(ldtr(Gs, 32 * qt + 16 * hs, 32 * dt, lane), pb, dv[dt]);
          dk[dt] = mfma(ldtr(Qs, 32 * qt + 16 * hs, 32 * dt, lane), sb, dk[dt]);
        }
      }
    }
    __syncthreads();
  }

  if (kv) {
    const long off = ((long)b * a.L + key) * a.gl + hd * kD;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d0 = 32 * dt + 8 * g + 4 * h;
        *reinterpret_cast<uint2*>(a.dk + off + d0) =
            make_uint2(pack_bf16x2(dk[dt][4 * g] * a.scale, dk[dt][4 * g + 1] * a.scale),
                       pack_bf16x2(dk[dt][4 * g + 2] * a.scale, dk[dt][4 * g + 3] * a.scale));
        *reinterpret_cast<uint2*>(a.dv + off + d0) =
            make_uint2(pack_bf16x2(dv[dt][4 * g], dv[dt][4 * g + 1]), pack_bf16x2(dv[dt][4 * g + 2], dv[dt][4 * g + 3]));
      }
  }
}

template <bool DROP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void attn_bwd_dq_kernel(Args a) {
  if (a.seed_ptr != nullptr) a.seed ^= *a.seed_ptr;
  __shared__ __attribute__((aligned(16))) bf16 Ks[kTile * kRowLd];
  __shared__ __attribute__((aligned(16))) bf16 Vs[kTile * kRowLd];
  __shared__ __attribute__((aligned(16))) float4 km[kTile];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int b = blockIdx.z, hd = blockIdx.y, bh = b * a.H + hd;
  const int q = blockIdx.x * kBlk + w * 32 + l32;
  const bool qv = q < a.L;
  const int qc = qv ? q : a.L - 1;
  bf16x8_t qf[4], gf[4];
  {
    const bf16* qp = a.q + b * a.qb + (long)qc * a.ql + hd * a.qh;
    const bf16* gp = a.dout + (((long)b * a.L + qc) * a.H + hd) * kD;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      qf[s] = ld8(qp + 16 * s + 8 * h);
      gf[s] = ld8(gp + 16 * s + 8 * h);
    }
  }
  const float lse2 = qv ? lse_safe(a.lse[(long)bh * a.L + q]) : INFINITY;
  const uint32_t qlin = ((uint32_t)bh * (uint32_t)a.L + (uint32_t)q) * (uint32_t)a.L;
  const float dl = qv ? a.delta[(long)bh * a.L + q] : 0.f;
  const bf16* kp = a.k + b * a.kb + hd * a.kh;
  const bf16* vp = a.v + b * a.vb + hd * a.vh;
  f32x16 dq[2];
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) dq[dt][r] = 0.f;

  for (int k0 = 0; k0 < a.L; k0 += kTile) {
    stage(Ks, kp, a.kl, k0, a.L, tid);
    stage(Vs, vp, a.vl, k0, a.L, tid);
    if (tid < kTile) km[tid] = key_coef(a, key_state(a, b, k0 + tid));
    __syncthreads();
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      f32x16 S, dP;
#pragma unroll
      for (int r = 0; r < 16; ++r) { S[r] = 0.f; dP[r] = 0.f; }
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        S = mfma(ld8(Ks + (32 * t + l32) * kRowLd + 16 * ks + 8 * h), qf[ks], S);
        dP = mfma(ld8(Vs + (32 * t + l32) * kRowLd + 16 * ks + 8 * h), gf[ks], dP);
      }
      float ds[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int kr = 32 * t + crow(r, h);
        const float4 c = km[kr];
        const float pv = fexp2(fmaf(S[r], c.x, c.y) - lse2);
        float z = 1.f;
        if (DROP) z = dropped_lin(a, qlin + (uint32_t)(k0 + kr)) ? 0.f : a.keep_scale;
        ds[r] = c.z * pv * (dP[r] * z - dl);
      }
#pragma unroll
      for (int hs = 0; hs < 2; ++hs) {
        const bf16x8_t sb = pack8(&ds[8 * hs]);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) dq[dt] = mfma(ldtr(Ks, 32 * t + 16 * hs, 32 * dt, lane), sb, dq[dt]);
      }
    }
    __syncthreads();
  }

  if (qv) {
    bf16* dp = a.dq + ((long)b * a.L + q) * a.gl + hd * kD;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<uint2*>(dp + 32 * dt + 8 * g + 4 * h) =
            make_uint2(pack_bf16x2(dq[dt][4 * g] * a.scale, dq[dt][4 * g + 1] * a.scale),
                       pack_bf16x2(dq[dt][4 * g + 2] * a.scale, dq[dt][4 * g + 3] * a.scale));
  }
}

static Args make_args(uint64_t q, uint64_t k, uint64_t v, const std::vector<long>& st, uint64_t mask, int B, int L,
                      int H, float fill, float p_drop, uint64_t seed, uint64_t seed_ptr) {
  FDT_CHECK(st.size() == 9, "attention: 9 strides (q, k, v x batch, position, head)");
  FDT_CHECK(L >= 1 && L <= 4096 && B >= 1 && H >= 1, "attention: bad shape");
  FDT_CHECK(p_drop >= 0.f && p_drop < 1.f, "attention: dropout in [0, 1)");
  Args a{};
  a.q = P<const bf16>(q);
  a.k = P<const bf16>(k);
  a.v = P<const bf16>(v);
  a.qb = st[0]; a.ql = st[1]; a.qh = st[2];
  a.kb = st[3]; a.kl = st[4]; a.kh = st[5];
  a.vb = st[6]; a.vl = st[7]; a.vh = st[8];
  a.mask = P<const uint8_t>(mask);
  a.B = B; a.L = L; a.H = H;
  const float log2e = 1.4426950408889634f;
  a.scale = 0.125f;  // 1/sqrt(64)
  a.c2 = log2e * a.scale;
  a.fill2 = fill * log2e;  // -inf stays -inf
  a.drop_thr = (uint32_t)fminf(p_drop * 4294967296.f, 4294967295.f);
  a.keep_scale = 1.f / (1.f - p_drop);
  a.seed = seed;
  a.seed_ptr = P<const uint64_t>(seed_ptr);
  return a;
}

}  // namespace attn

void attn_fwd(uint64_t q, uint64_t k, uint64_t v, const std::vector<long>& strides, uint64_t out, uint64_t lse,
              uint64_t mask, int B, int L, int H, float fill, float p_drop, uint64_t seed, uint64_t seed_ptr,
              uint64_t stream) {
  using namespace attn;
  Args a = make_args(q, k, v, strides, mask, B, L, H, fill, p_drop, seed, seed_ptr);
  a.out = P<bf16>(out);
  a.lse = P<float>(lse);
  const dim3 grid((L + kBlk - 1) / kBlk, H, B);
  if (a.drop_thr) hipLaunchKernelGGL(attn_fwd_kernel<true>, grid, dim3(256), 0, as_stream(stream), a);
  else hipLaunchKernelGGL(attn_fwd_kernel<false>, grid, dim3(256), 0, as_stream(stream), a);
  FDT_LAUNCH_CHECK();
}

void attn_bwd(uint64_t q, uint64_t k, uint64_t v, const std::vector<long>& strides, uint64_t o, uint64_t dout,
              uint64_t lse, uint64_t delta, uint64_t mask, uint64_t dq, uint64_t dk, uint64_t dv, int B, int L, int H,
              float fill, float p_drop, uint64_t seed, uint64_t seed_ptr, long grad_ld, uint64_t stream) {
  using namespace attn;
  Args a = make_args(q, k, v, strides, mask, B, L, H, fill, p_drop, seed, seed_ptr);
  FDT_CHECK(grad_ld == 0 || (grad_ld >= (long)H * kD && grad_ld % 8 == 0), "attention: bad gradient row stride");
  a.gl = grad_ld == 0 ? (long)H * kD : grad_ld;
  a.o = P<const bf16>(o);
  a.dout = P<const bf16>(dout);
  a.lse = P<float>(lse);
  a.delta = P<float>(delta);
  a.dq = P<bf16>(dq);
  a.dk = P<bf16>(dk);
  a.dv = P<bf16>(dv);
  hipStream_t st = as_stream(stream);
  const long rows = (long)B * L * H;
  hipLaunchKernelGGL(attn_bwd_prep_kernel, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, st, a);
  FDT_LAUNCH_CHECK();
  const dim3 grid((L + kBlk - 1) / kBlk, H, B);
  if (a.drop_thr) hipLaunchKernelGGL(attn_bwd_dkdv_kernel<true>, grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(attn_bwd_dkdv_kernel<false>, grid, dim3(256), 0, st, a);
  FDT_LAUNCH_CHECK();
  if (a.drop_thr) hipLaunchKernelGGL(attn_bwd_dq_kernel<true>, grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(attn_bwd_dq_kernel<false>, grid, dim3(256), 0, st, a);
  FDT_LAUNCH_CHECK();
}

}  // namespace fdt
