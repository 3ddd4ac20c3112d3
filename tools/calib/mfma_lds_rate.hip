// Calibration: MFMA rate when each wave also reads its next fragments from LDS (10 x 16 B per lane per
// 32 MFMAs, register double buffer, no barrier), same occupancy as the GEMM (4 waves, 2 blocks/CU).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v4i __attribute__((ext_vector_type(4)));

template <int NREAD, int SYNC>
__global__ __launch_bounds__(256, 2) void loop(const int* in, int* out, int iters) {
  __shared__ __attribute__((aligned(16))) int lds[16384];
  for (int i = threadIdx.x; i < 16384; i += 256) lds[i] = in[i & 63] + i;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  v4i acc[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) acc[i] = v4i{i, 0, 0, 0};
  v4i fa[NREAD], fb[NREAD];
#pragma unroll
  for (int i = 0; i < NREAD; ++i) fa[i] = *reinterpret_cast<const v4i*>(lds + 4 * (lane + 64 * i));
  auto step = [&](v4i (&cur)[NREAD], v4i (&nxt)[NREAD], int it) __attribute__((always_inline)) {
    __builtin_amdgcn_s_waitcnt(0xC07F);
    if (SYNC) __syncthreads();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < NREAD; ++i)
      nxt[i] = *reinterpret_cast<const v4i*>(lds + ((4 * (lane + 64 * i) + 1024 * (it & 3)) & 16383));
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int s = 0; s < 8; ++s)
        acc[r * 8 + s] = __builtin_amdgcn_mfma_i32_16x16x64_i8(cur[r % NREAD], cur[(4 + s) % NREAD], acc[r * 8 + s], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  };
  for (int it = 0; it < iters; it += 2) {
    step(fa, fb, it);
    step(fb, fa, it + 1);
  }
  int x = 0;
#pragma unroll
  for (int i = 0; i < 32; ++i) x ^= acc[i][0] ^ acc[i][1] ^ acc[i][2] ^ acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

template <int NREAD, int SYNC>
void run(const int* in, int* out) {
  const int blocks = 512, iters = 2000;
  hipEvent_t s, e;
  (void)hipEventCreate(&s);
  (void)hipEventCreate(&e);
  for (int rep = 0; rep < 2; ++rep) {
    (void)hipEventRecord(s);
    hipLaunchKernelGGL((loop<NREAD, SYNC>), dim3(blocks), dim3(256), 0, 0, in, out, iters);
    (void)hipEventRecord(e);
    (void)hipEventSynchronize(e);
    float ms;
    (void)hipEventElapsedTime(&ms, s, e);
    const double ops = 2.0 * 16 * 16 * 64 * 32.0 * iters * (blocks * 4.0);
    if (rep) printf("reads/32mfma=%2d barrier=%d: %.3f ms  %.1f TOPS (%.1f%% of 5033)\n", NREAD, SYNC, ms, ops / ms / 1e9,
                    ops / ms / 1e9 / 5033 * 100);
  }
}

int main() {
  int *in, *out;
  (void)hipMalloc(&in, 64 * sizeof(int));
  (void)hipMemset(in, 1, 64 * sizeof(int));
  (void)hipMalloc(&out, 512 * 256 * sizeof(int));
  run<8, 0>(in, out);
  run<10, 0>(in, out);
  run<10, 1>(in, out);
  run<12, 1>(in, out);
  return 0;
}
