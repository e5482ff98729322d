// Workgroup dispatch-rate probe: time an (almost) empty 256-thread kernel over grid sizes
// and dynamic-LDS sizes, to separate launch/dispatch limits from memory limits.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(256) void empty_k(float* out, int flag) {
  extern __shared__ float lds[];
  if (flag == 12345) { lds[threadIdx.x] = 1.f; __syncthreads(); out[blockIdx.x] = lds[threadIdx.x ^ 1]; }
}
__global__ __launch_bounds__(256) void store_k(uint4* out, int per_block_vec) {
  // each block writes per_block_vec uint4 (16 B) per thread, contiguous
  uint4 v = make_uint4(threadIdx.x, blockIdx.x, 0, 0);
  uint4* p = out + (size_t)blockIdx.x * per_block_vec * 256;
  for (int i = 0; i < per_block_vec; ++i) p[i * 256 + threadIdx.x] = v;
}
int main() {
  float* out; hipMalloc(&out, 1 << 28);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipFuncSetAttribute((const void*)empty_k, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
  for (int lds : {0, 16384, 38912, 65536}) {
    for (int g : {4096, 16384, 65536}) {
      empty_k<<<g, 256, lds>>>(out, 0);
      hipDeviceSynchronize();
      hipEventRecord(a);
      for (int r = 0; r < 10; ++r) empty_k<<<g, 256, lds>>>(out, 0);
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      printf("empty lds=%6d grid=%6d: %7.2f us  (%.1f WG/us)\n", lds, g, ms * 100, g / (ms * 100));
    }
  }
  // pure store bandwidth: 512 MB written as blocks of 32 KB (the conv epilogue's tile)
  for (int vec : {8, 32}) {
    int g = (256 << 20) / (vec * 256 * 16);
    store_k<<<g, 256>>>((uint4*)out, vec);
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int r = 0; r < 10; ++r) store_k<<<g, 256>>>((uint4*)out, vec);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    printf("store 256 MB per launch, %d KB/block, grid %d: %.1f us = %.2f TB/s\n", vec * 4, g, ms * 100,
           (256.0 * (1 << 20)) / (ms * 1e-4) / 1e12);
  }
  return 0;
}
