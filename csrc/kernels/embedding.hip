// Token + position + segment embedding sum (reference transformer.py:150-156):
//     out[b,l,:] = (tok[ids[b,l]] + pos[pos_ids[l]] + seg[types[b,l]]) * scale
// Forward: one wave per (b,l) row, 16-B loads from the three fp32 tables, one store.
// Backward: see embedding_bwd_kernel (token rows by atomics, segment rows via LDS, position
// rows by a deterministic reduction over the batch).
// Indices are clamped into range on the device (a bad token id must not fault the GPU).
#include "common.h"

namespace fdt {

__device__ __forceinline__ int clampi(int v, int n) { return v < 0 ? 0 : (v >= n ? n - 1 : v); }

__global__ __launch_bounds__(256) void embedding_fwd_kernel(const int* __restrict__ ids, const int* __restrict__ types,
                                                            const int* __restrict__ pos_ids, const float* __restrict__ tok,
                                                            const float* __restrict__ pos, const float* __restrict__ seg,
                                                            float* __restrict__ out, long rows, int L, int d, float scale,
                                                            int vt, int vp, int vs) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int l = (int)(row % L);
  const float* a = tok + (long)clampi(ids[row], vt) * d;
  const float* b = pos + (long)clampi(pos_ids[l], vp) * d;
  const float* c = seg + (long)clampi(types[row], vs) * d;
  float* o = out + row * d;
  for (int e = lane * 4; e < d; e += 256) {
    float4 x = *reinterpret_cast<const float4*>(a + e);
    float4 y = *reinterpret_cast<const float4*>(b + e);
    float4 z = *reinterpret_cast<const float4*>(c + e);
    *reinterpret_cast<float4*>(o + e) =
        make_float4((x.x + y.x + z.x) * scale, (x.y + y.y + z.y) * scale, (x.z + y.z + z.z) * scale,
                    (x.w + y.w + z.w) * scale);
  }
}

// Backward, contention-aware (the naive form -- three float atomics per element of every
// row -- serialises on the 3-row segment table and the padding token's row):
//  * token table: whole-row 256-B atomics, skipped for rows whose gradient is exactly zero
//    (padding positions under a true key mask carry none);
//  * segment table (vs rows, tiny): per-workgroup LDS accumulation (ds_add_f32), one flush
//    of vs*d global atomics per workgroup;
//  * position table: a separate deterministic column reduction over the batch
//    (embedding_pos_bwd_kernel), no atomics.
constexpr int kEmbRowsPerBlock = 64;
constexpr int kEmbMaxSegLds = 8 * 1024;  // floats of LDS for the segment accumulators

__global__ __launch_bounds__(256) void embedding_bwd_kernel(const float* __restrict__ g, const int* __restrict__ ids,
                                                            const int* __restrict__ types, float* __restrict__ gt,
                                                            float* __restrict__ gs, long rows, int d, float scale,
                                                            int vt, int vs) {
  __shared__ float seg[kEmbMaxSegLds];
  const bool seg_lds = vs * d <= kEmbMaxSegLds;
  for (int i = threadIdx.x; seg_lds && i < vs * d; i += 256) seg[i] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long r0 = (long)blockIdx.x * kEmbRowsPerBlock;
  for (int k = w; k < kEmbRowsPerBlock; k += 4) {
    const long row = r0 + k;
    if (row >= rows) break;
    const float* gr = g + row * d;
    bool nz = false;
    for (int e = lane; e < d; e += 64) nz |= gr[e] != 0.f;
    if (!__any(nz)) continue;  // wave-uniform: an all-zero row adds nothing
    float* a = gt + (long)clampi(ids[row], vt) * d;
    const int t = clampi(types[row], vs);
    for (int e = lane; e < d; e += 64) {
      const float v = gr[e] * scale;
      atomicAdd(a + e, v);
      if (seg_lds) atomicAdd(&seg[t * d + e], v);
      else atomicAdd(gs + (long)t * d + e, v);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; seg_lds && i < vs * d; i += 256)
    if (seg[i] != 0.f) atomicAdd(gs + i, seg[i]);
}

// gp[pos_ids[l]] += scale * sum_b g[b, l, :]  (one thread per (l, e); fixed summation order)
__global__ __launch_bounds__(256) void embedding_pos_bwd_kernel(const float* __restrict__ g, const int* __restrict__ pos_ids,
                                                                float* __restrict__ gp, int B, int L, int d, float scale,
                                                                int vp) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)L * d) return;
  const int l = (int)(i / d), e = (int)(i - (long)l * d);
  float acc = 0.f;
  for (int b = 0; b < B; ++b) acc += g[((long)b * L + l) * d + e];
  atomicAdd(gp + (long)clampi(pos_ids[l], vp) * d + e, acc * scale);  // distinct rows for arange ids
}

void embedding_fwd(uint64_t ids, uint64_t types, uint64_t pos_ids, uint64_t tok, uint64_t pos, uint64_t seg,
                   uint64_t out, int B, int L, int d, float scale, int vt, int vp, int vs, uint64_t stream) {
  FDT_CHECK(d % 256 == 0, "embedding: d must be a multiple of 256");
  long rows = (long)B * L;
  if (rows == 0) return;
  embedding_fwd_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, as_stream(stream)>>>(
      P<const int>(ids), P<const int>(types), P<const int>(pos_ids), P<const float>(tok), P<const float>(pos),
      P<const float>(seg), P<float>(out), rows, L, d, scale, vt, vp, vs);
  FDT_LAUNCH_CHECK();
}

void embedding_bwd(uint64_t g, uint64_t ids, uint64_t types, uint64_t pos_ids, uint64_t gt, uint64_t gp, uint64_t gs,
                   int B, int L, int d, float scale, int vt, int vp, int vs, uint64_t stream) {
  long rows = (long)B * L;
  if (rows == 0) return;
  embedding_bwd_kernel<<<(unsigned)((rows + kEmbRowsPerBlock - 1) / kEmbRowsPerBlock), 256, 0, as_stream(stream)>>>(
      P<const float>(g), P<const int>(ids), P<const int>(types), P<float>(gt), P<float>(gs), rows, d, scale, vt, vs);
  FDT_LAUNCH_CHECK();
  embedding_pos_bwd_kernel<<<(unsigned)(((long)L * d + 255) / 256), 256, 0, as_stream(stream)>>>(
      P<const float>(g), P<const int>(pos_ids), P<float>(gp), B, L, d, scale, vp);
  FDT_LAUNCH_CHECK();
}

}  // namespace fdt
