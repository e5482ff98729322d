// Per-kernel floor inside a HIP graph on MI355X: how long does a chain of small dependent
// kernels take per link?  Decides whether a tiny kernel (the BN statistics finalize: 1-32
// workgroups reading 64 slot rows) is worth folding into its neighbour.
//   hipcc -O3 --offload-arch=gfx950 tools/launch_floor.hip -o tools/launch_floor && ./tools/launch_floor
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void empty_k(float* p, int flag) {
  if (flag == 12345) p[threadIdx.x] = 1.f;
}

// finalize-shaped: `rows` x C fp32 slots summed per channel (64 channels per 256-thread block,
// 4 waves over the rows), result written, slots re-zeroed
__global__ __launch_bounds__(256) void fin_k(float* part, int rows, int C, float* out) {
  __shared__ float sm[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, c = blockIdx.x * 64 + lane;
  float a = 0.f;
  for (int r = w; r < rows; r += 4) {
    a += part[(long)r * C + c];
    part[(long)r * C + c] = 0.f;
  }
  sm[w][lane] = a;
  __syncthreads();
  if (w == 0) out[c] = sm[0][lane] + sm[1][lane] + sm[2][lane] + sm[3][lane];
}

// streaming elementwise kernel over n floats (a "real" neighbour)
__global__ __launch_bounds__(256) void axpy_k(const float4* __restrict__ x, float4* __restrict__ y, long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    float4 v = x[i];
    v.x *= 1.0001f; v.y *= 1.0001f; v.z *= 1.0001f; v.w *= 1.0001f;
    y[i] = v;
  }
}

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) { std::printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } \
  } while (0)

template <typename F>
static int graph_time(const char* name, int n, F body) {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < n; ++i) body(s, i);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, s));
  const int reps = 5;
  for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  std::printf("%-44s %8.2f us per kernel (%d kernels, graph)\n", name, ms * 1e3 / reps / n, n);
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipStreamDestroy(s));
  return 0;
}

int main() {
  float *p, *part, *out;
  CK(hipMalloc(&p, 256L << 20));
  CK(hipMalloc(&part, 64L * 2048 * 4));
  CK(hipMalloc(&out, 2048 * 4));
  CK(hipMemset(part, 0, 64L * 2048 * 4));
  const int n = 400;
  graph_time("empty, 1 workgroup", n, [&](hipStream_t s, int) { empty_k<<<1, 64, 0, s>>>(p, 0); });
  graph_time("empty, 2048 workgroups", n, [&](hipStream_t s, int) { empty_k<<<2048, 256, 0, s>>>(p, 0); });
  graph_time("finalize-shaped, C=256 (4 wg)", n, [&](hipStream_t s, int) { fin_k<<<4, 256, 0, s>>>(part, 64, 256, out); });
  graph_time("finalize-shaped, C=2048 (32 wg)", n, [&](hipStream_t s, int) { fin_k<<<32, 256, 0, s>>>(part, 64, 2048, out); });
  const long nv = (8L << 20) / 16;  // 8 MB in, 8 MB out
  graph_time("axpy 8 MB (alone)", n, [&](hipStream_t s, int) {
    axpy_k<<<1024, 256, 0, s>>>((const float4*)p, (float4*)(p + (32L << 20)), nv);
  });
  graph_time("axpy 8 MB + finalize C=256 (pairs)", n, [&](hipStream_t s, int i) {
    if (i & 1) fin_k<<<4, 256, 0, s>>>(part, 64, 256, out);
    else axpy_k<<<1024, 256, 0, s>>>((const float4*)p, (float4*)(p + (32L << 20)), nv);
  });
  return 0;
}
