// Counter calibration microkernels for the per-kernel roofline tables (scripts/pmc_table.py):
// kernels of KNOWN bytes / MFMA FLOPs, run under rocprofv3 --pmc to measure
//   * bytes per FETCH_SIZE unit for 16-, 8- and 4-byte-per-lane streaming reads (the
//     guide's "FETCH_SIZE counts half of a 16-B/lane stream" checked in-repo, plus the
//     widths the conv / wgrad kernels also issue),
//   * bytes per WRITE_SIZE unit for 16-B/lane streaming stores,
//   * FLOPs per SQ_VALU_MFMA_BUSY_CYCLES for v_mfma_f32_32x32x16_bf16, and the effective
//     shader clock of a long MFMA-bound dispatch (GRBM_GUI_ACTIVE / 8 / duration).
// Buffers are 1 GiB (4x the 256 MiB Infinity Cache), so reads come from HBM.
//   hipcc -O3 --offload-arch=gfx950 tools/pmc_calib.hip -o build/pmc_calib
//   ./build/pmc_calib   -> one line per kernel: name, bytes or FLOPs, elapsed
#include <hip/hip_runtime.h>

#include <cstdio>

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <typename V>
__global__ __launch_bounds__(256) void read_k(const V* __restrict__ src, long n, unsigned* __restrict__ sink) {
  unsigned acc = 0;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const V v = src[i];
    const unsigned* u = reinterpret_cast<const unsigned*>(&v);
#pragma unroll
    for (int k = 0; k < (int)(sizeof(V) / 4); ++k) acc ^= u[k];
  }
  if (acc == 0x9e3779b9u) sink[blockIdx.x] = acc;  // data-dependent, never taken for zeros
}

__global__ __launch_bounds__(256) void copy16_k(const uint4* __restrict__ src, uint4* __restrict__ dst, long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) dst[i] = src[i];
}

__global__ __launch_bounds__(256) void write16_k(uint4* __restrict__ dst, long n) {
  const uint4 v = make_uint4(threadIdx.x, blockIdx.x, 1, 2);
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) dst[i] = v;
}

// 4 independent accumulator chains per wave, `iters` x 4 MFMAs of 32x32x16 (32768 FLOP each)
__global__ __launch_bounds__(256) void mfma_k(float* __restrict__ out, int iters) {
  bf16x8_t a, b;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    a[k] = (short)(0x3f80 + (threadIdx.x & 7));
    b[k] = (short)(0x3f80 - k);
  }
  f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c3, 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
  out[(long)blockIdx.x * 256 + threadIdx.x] = s;
}

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      return 1;                                                                \
    }                                                                          \
  } while (0)

int main() {
  const long bytes = 1L << 30;
  char *a, *b;
  unsigned* sink;
  float* fo;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMalloc(&sink, 1 << 20));
  CK(hipMalloc(&fo, 64L << 20));
  CK(hipMemset(a, 0, bytes));
  CK(hipMemset(b, 0, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int grid = 256 * 16;
  auto timed = [&](const char* name, double amount, const char* unit, auto launch) {
    launch();  // warm
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("%-10s %14.0f %-5s %9.3f ms  %8.2f %s/s\n", name, amount, unit, ms, amount / (ms * 1e-3) / 1e12,
                unit[0] == 'B' ? "TB" : "TFLOP");
    return 0;
  };
  timed("read16", (double)bytes, "B", [&] { read_k<uint4><<<grid, 256>>>((const uint4*)a, bytes / 16, sink); });
  timed("read8", (double)bytes, "B", [&] { read_k<uint2><<<grid, 256>>>((const uint2*)a, bytes / 8, sink); });
  timed("read4", (double)bytes, "B", [&] { read_k<unsigned><<<grid, 256>>>((const unsigned*)a, bytes / 4, sink); });
  timed("write16", (double)bytes, "B", [&] { write16_k<<<grid, 256>>>((uint4*)b, bytes / 16); });
  timed("copy16", 2.0 * bytes, "B", [&] { copy16_k<<<grid, 256>>>((const uint4*)a, (uint4*)b, bytes / 16); });
  const int mgrid = 256 * 8, iters = 4096;
  const double flop = (double)mgrid * 4 /*waves*/ * iters * 4 /*mfma*/ * 32768.0;
  timed("mfma", flop, "FLOP", [&] { mfma_k<<<mgrid, 256>>>(fo, iters); });
  CK(hipDeviceSynchronize());
  return 0;
}
