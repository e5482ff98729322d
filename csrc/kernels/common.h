// Common helpers for the MI355X (gfx950 / CDNA4) kernels of faster_distributed_training_amd.
//
// Conventions
//  * wave64 everywhere: block sizes are multiples of 64, lane = threadIdx.x & 63.
//  * 16-byte vector memory access for every streaming kernel (8 x bf16 / 4 x f32 per
//    lane): hipcc never auto-vectorises bf16 loads.
//  * dtype codes shared with Python (ops/*.py: DT): 0 = f32, 1 = bf16, 2 = f16.
//  * every launcher takes the raw hipStream_t of the current torch stream so kernels
//    order with PyTorch work and are captured by HIP graphs; launchers never allocate
//    or synchronise (graph-capture safe).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <cstdint>
#include <stdexcept>
#include <string>

namespace fdt {

using bf16 = __hip_bfloat16;
using f16 = __half;

enum DType : int { kF32 = 0, kBF16 = 1, kF16 = 2 };

#define FDT_HIP_CHECK(expr)                                                              \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess)                                                                \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) +      \
                               " at " + __FILE__ + ":" + std::to_string(__LINE__));      \
  } while (0)

#define FDT_CHECK(cond, msg)                                                             \
  do {                                                                                   \
    if (!(cond)) throw std::runtime_error(std::string("fdt check failed: ") + (msg));   \
  } while (0)

#define FDT_LAUNCH_CHECK() FDT_HIP_CHECK(hipGetLastError())

inline hipStream_t as_stream(uint64_t s) { return reinterpret_cast<hipStream_t>(s); }
template <typename T>
inline T* P(uint64_t p) { return reinterpret_cast<T*>(p); }

// ---------------------------------------------------------------- scalar conversion
__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(bf16 x) { return __bfloat162float(x); }
__device__ __forceinline__ float to_f(f16 x) { return __half2float(x); }

template <typename T> __device__ __forceinline__ T from_f(float x);
template <> __device__ __forceinline__ float from_f<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f<bf16>(float x) { return __float2bfloat16(x); }
template <> __device__ __forceinline__ f16 from_f<f16>(float x) { return __float2half(x); }

// bf16 bit tricks (exact): bf16 -> f32 is a 16-bit shift.
__device__ __forceinline__ float bf16_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  bf16 a = __float2bfloat16(lo), b = __float2bfloat16(hi);
  return (uint32_t)(*reinterpret_cast<uint16_t*>(&a)) | ((uint32_t)(*reinterpret_cast<uint16_t*>(&b)) << 16);
}

// ---------------------------------------------------------------- 8-wide vector I/O
// Load / store 8 consecutive elements of T as f32 (16 B for bf16/f16, 2 x 16 B for f32).
template <typename T> struct Vec8;
template <> struct Vec8<bf16> {
  __device__ static __forceinline__ void load(const bf16* p, float* v) {
    uint4 u = *reinterpret_cast<const uint4*>(p);
    v[0] = bf16_lo(u.x); v[1] = bf16_hi(u.x); v[2] = bf16_lo(u.y); v[3] = bf16_hi(u.y);
    v[4] = bf16_lo(u.z); v[5] = bf16_hi(u.z); v[6] = bf16_lo(u.w); v[7] = bf16_hi(u.w);
  }
  __device__ static __forceinline__ void store(bf16* p, const float* v) {
    uint4 u;
    u.x = pack_bf16x2(v[0], v[1]); u.y = pack_bf16x2(v[2], v[3]);
    u.z = pack_bf16x2(v[4], v[5]); u.w = pack_bf16x2(v[6], v[7]);
    *reinterpret_cast<uint4*>(p) = u;
  }
};
template <> struct Vec8<f16> {
  __device__ static __forceinline__ void load(const f16* p, float* v) {
    uint4 u = *reinterpret_cast<const uint4*>(p);
    const __half2* h = reinterpret_cast<const __half2*>(&u);
#pragma unroll
    for (int i = 0; i < 4; ++i) { float2 f = __half22float2(h[i]); v[2 * i] = f.x; v[2 * i + 1] = f.y; }
  }
  __device__ static __forceinline__ void store(f16* p, const float* v) {
    uint4 u;
    __half2* h = reinterpret_cast<__half2*>(&u);
#pragma unroll
    for (int i = 0; i < 4; ++i) h[i] = __floats2half2_rn(v[2 * i], v[2 * i + 1]);
    *reinterpret_cast<uint4*>(p) = u;
  }
};
template <> struct Vec8<float> {
  __device__ static __forceinline__ void load(const float* p, float* v) {
    float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  __device__ static __forceinline__ void store(float* p, const float* v) {
    reinterpret_cast<float4*>(p)[0] = make_float4(v[0], v[1], v[2], v[3]);
    reinterpret_cast<float4*>(p)[1] = make_float4(v[4], v[5], v[6], v[7]);
  }
};

// 8-wide store of a streaming output at element e of base: wt = write-through (sc1) for bf16 --
// the bytes leave the XCD's L2 as written instead of in the end-of-kernel write-back the next
// dependent launch waits for (the conv epilogues' st_out does the same); plain otherwise.
template <typename T>
__device__ __forceinline__ void st8(T* __restrict__ base, long e, const float* v, int wt) {
  if constexpr (sizeof(T) == 2) {
    if (wt) {
      const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)0xFFFFFFFF, 0x00020000);
      typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
      uint4 u;
      Vec8<T>::store(reinterpret_cast<T*>(&u), v);
      u32x4v w = {u.x, u.y, u.z, u.w};
      __builtin_amdgcn_raw_buffer_store_b128(w, r, (uint32_t)(e * 2), 0, 16);
      return;
    }
  }
  Vec8<T>::store(base + e, v);
}

// Per-channel statistics producers (conv epilogues, BN-backward reductions) add their
// per-workgroup partial sums with fp32 atomics into at most kStatSlots rows (row = block index
// mod rows, spreading contention); the fp64 finalize/reduce kernel sums the rows and
// re-zeroes them.  Replaces per-workgroup slabs + a compaction pass.
constexpr int kStatSlots = 64;
// upper bound on the rows of a (non-deterministic) slot buffer: large-M convolutions spread
// their workgroups over more rows (fewer adders per address; conv_igemm.py slot_rows)
constexpr int kMaxStatRows = 16384;

// Deterministic mode (--deterministic): every statistics producer writes slot = its block
// index WITHOUT wrapping (the Python side sizes the slot buffer to >= the block count), so
// each slot address has exactly one writer and the fp32 atomic add onto a zeroed slot is
// exact; the fp64 finalize then sums the rows in a fixed order.  Split-K reducers sum every
// split's partials in split order.  Result: bitwise-repeatable steps.
inline int& deterministic_flag() {
  static int f = 0;
  return f;
}
inline void set_deterministic(bool on) { deterministic_flag() = on ? 1 : 0; }
// conv epilogues: write-through (sc1) output stores (conv_igemm_impl.h st_out)
inline int& conv_write_through_flag() {
  static int f = 0;
  return f;
}
inline bool conv_write_through() { return conv_write_through_flag() != 0; }
// cost-probe switches of the conv kernels (never set in training: scripts/conv_probe2.py)
inline int& conv_debug_flags_ref() {
  static int f = 0;
  return f;
}
inline int conv_debug_flags() { return conv_debug_flags_ref(); }
inline bool deterministic() { return deterministic_flag() != 0; }
// slot index mask for a launch whose slot buffer holds `rows` rows (nblocks: the launch's
// block count along the slot axis)
inline unsigned stat_slot_mask(int rows, long nblocks) {
  if (!deterministic()) {
    // rows: a power of two (fewer for small grids: less for the finalize to read)
    FDT_CHECK(rows >= 1 && rows <= kMaxStatRows && (rows & (rows - 1)) == 0, "statistics slot rows");
    return (unsigned)(rows - 1);
  }
  FDT_CHECK(nblocks <= rows, "deterministic mode: statistics slot buffer smaller than the block count");
  return 0xFFFFFFFFu;
}

// ---------------------------------------------------------------- wave reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---------------------------------------------------------------- activations
// act codes shared with Python: 0 = identity, 1 = ReLU, 2 = CELU(alpha)
enum Act : int { kActNone = 0, kActRelu = 1, kActCelu = 2 };

__device__ __forceinline__ float act_fwd(float z, int act, float alpha) {
  if (act == kActRelu) return fmaxf(z, 0.f);
  if (act == kActCelu) return z > 0.f ? z : alpha * (__expf(z / alpha) - 1.f);
  return z;
}
// derivative expressed through the pre-activation z
__device__ __forceinline__ float act_grad(float z, int act, float alpha) {
  if (act == kActRelu) return z > 0.f ? 1.f : 0.f;
  if (act == kActCelu) return z > 0.f ? 1.f : __expf(z / alpha);
  return 1.f;
}

// Counter-based RNG (splitmix64 finaliser): stateless, identical in forward/backward,
// graph-replay safe when the seed/offset live in device memory.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ float u01(uint64_t h) {  // [0,1)
  return (float)(h >> 40) * (1.0f / 16777216.0f);
}

}  // namespace fdt
