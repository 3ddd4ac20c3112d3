// Calibration: sustained v_mfma_i32_16x16x64_i8 rate with register operands (no memory in the loop),
// 4 waves per block, `blocks_per_cu` x 256 CUs, each wave issuing 32 independent MFMAs per iteration.
// hipcc --offload-arch=gfx950 -O3 mfma_rate.hip -o mfma_rate && ./mfma_rate
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v4i __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256, 2) void mfma_loop(const int* in, int* out, int iters) {
  v4i a = {in[threadIdx.x & 63], in[(threadIdx.x + 1) & 63], 3, 4};
  v4i b = {in[(threadIdx.x + 2) & 63], 5, 6, 7};
  v4i acc[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) acc[i] = v4i{i, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 32; ++i) acc[i] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, acc[i], 0, 0, 0);
  }
  int x = 0;
#pragma unroll
  for (int i = 0; i < 32; ++i) x ^= acc[i][0] ^ acc[i][1] ^ acc[i][2] ^ acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

int main() {
  int *in, *out;
  hipMalloc(&in, 64 * sizeof(int));
  hipMemset(in, 1, 64 * sizeof(int));
  const int blocks = 512, iters = 2000;
  hipMalloc(&out, blocks * 256 * sizeof(int));
  hipEvent_t s, e;
  hipEventCreate(&s);
  hipEventCreate(&e);
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(s);
    hipLaunchKernelGGL(mfma_loop, dim3(blocks), dim3(256), 0, 0, in, out, iters);
    hipEventRecord(e);
    hipEventSynchronize(e);
    float ms;
    hipEventElapsedTime(&ms, s, e);
    const double ops = 2.0 * 16 * 16 * 64 * 32.0 * iters * (blocks * 4.0);
    printf("mfma_i32_16x16x64_i8: %.3f ms  %.1f TOPS  (%.1f%% of 5033)\n", ms, ops / ms / 1e9, ops / ms / 1e9 / 5033 * 100);
  }
  return 0;
}
