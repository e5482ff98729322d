// Token + position + segment embedding sum (reference transformer.py:150-156):
//     out[b,l,:] = (tok[ids[b,l]] + pos[pos_ids[l]] + seg[types[b,l]]) * scale
// Forward: one wave per (b,l) row, 16-B loads from the three fp32 tables, one store.
// Backward: float atomics into the three fp32 gradient tables, each wave-instruction a
// contiguous 256-B row segment (the full-rate atomic shape on MI355X, ~1.3 TB/s).
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

__global__ __launch_bounds__(256) void embedding_bwd_kernel(const float* __restrict__ g, const int* __restrict__ ids,
                                                            const int* __restrict__ types, const int* __restrict__ pos_ids,
                                                            float* __restrict__ gt, float* __restrict__ gp,
                                                            float* __restrict__ gs, long rows, int L, int d, float scale,
                                                            int vt, int vp, int vs) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int l = (int)(row % L);
  float* a = gt + (long)clampi(ids[row], vt) * d;
  float* b = gp + (long)clampi(pos_ids[l], vp) * d;
  float* c = gs + (long)clampi(types[row], vs) * d;
  const float* gr = g + row * d;
  for (int e = lane; e < d; e += 64) {
    float v = gr[e] * scale;
    atomicAdd(a + e, v);
    atomicAdd(b + e, v);
    atomicAdd(c + e, v);
  }
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
  embedding_bwd_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, as_stream(stream)>>>(
      P<const float>(g), P<const int>(ids), P<const int>(types), P<const int>(pos_ids), P<float>(gt), P<float>(gp),
      P<float>(gs), rows, L, d, scale, vt, vp, vs);
  FDT_LAUNCH_CHECK();
}

}  // namespace fdt
