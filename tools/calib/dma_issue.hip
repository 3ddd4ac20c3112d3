// Calibration: what one vector-memory wave-instruction of the GEMM pipelines costs the issuing wave under load.
// Each wave of BPC 256-thread blocks per CU issues P 1-KiB pieces per iteration from an L2-resident 1 MiB source
// (per-lane 16 B, 64 lanes contiguous), then waits for them; s_memtime stamps around the issue and around the
// wait. MODE 0: global_load_lds_dwordx4 (LDS-DMA, M0 = the wave's LDS slot), MODE 1: global_load_dwordx4 into
// VGPRs. Per-wave sums go to a device array through vector stores; the host prints cycles per piece at issue,
// cycles per iteration, and the bytes per cycle per CU that the loop moved.
//   hipcc --offload-arch=gfx950 -O3 -o tools/_diag/dma_issue tools/calib/dma_issue.hip && tools/_diag/dma_issue
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));

template <int MODE, int P>
__global__ __launch_bounds__(256) void dma_loop(const int8_t* __restrict__ src, uint32_t mask, int iters,
                                                unsigned long long* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) int8_t lds[32768];  // 8 KiB (8 pieces) per wave
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lbase = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)(lds + wave * 8192));
  uint32_t off = ((blockIdx.x * 4 + wave) * 8192u) & mask;
  unsigned long long t_issue = 0, t_wait = 0;
  v4i sink = {0, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
    v4i r[P];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const int8_t* a = src + ((off + p * 1024u) & mask) + lane * 16;
      if (MODE == 0) {
        uint32_t keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\t"
            "s_mov_b32 m0, %2\n\t"
            "s_nop 0\n\t"
            "global_load_lds_dwordx4 %1, off\n\t"
            "s_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(a), "s"(lbase + p * 1024u)
            : "memory");
      } else {
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r[p]) : "v"(a) : "memory");
      }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long t2 = __builtin_amdgcn_s_memtime();
    if (MODE == 1) {
#pragma unroll
      for (int p = 0; p < P; ++p) {
        asm volatile("" : "+v"(r[p]));
        sink ^= r[p];
      }
    }
    t_issue += t1 - t0;
    t_wait += t2 - t1;
    off = (off + 37u * 1024u) & mask;
  }
  if (lane == 0) {
    const int w = blockIdx.x * 4 + wave;
    out[3 * w] = t_issue;
    out[3 * w + 1] = t_wait;
    out[3 * w + 2] = (unsigned long long)(sink[0] ^ sink[1] ^ sink[2] ^ sink[3]) & 1ull;
  }
}

template <int MODE, int P>
void run(const int8_t* src, uint32_t mask, int bpc, int cus, unsigned long long* dout) {
  const int iters = 2000;
  const int grid = cus * bpc;
  hipEvent_t s, e;
  (void)hipEventCreate(&s);
  (void)hipEventCreate(&e);
  float ms = 0.f;
  for (int rep = 0; rep < 2; ++rep) {
    (void)hipEventRecord(s);
    hipLaunchKernelGGL((dma_loop<MODE, P>), dim3(grid), dim3(256), 0, 0, src, mask, iters, dout);
    (void)hipEventRecord(e);
    (void)hipEventSynchronize(e);
    (void)hipEventElapsedTime(&ms, s, e);
  }
  std::vector<unsigned long long> h(3 * (size_t)grid * 4);
  (void)hipMemcpy(h.data(), dout, h.size() * 8, hipMemcpyDeviceToHost);
  double issue = 0, wait = 0;
  for (int w = 0; w < grid * 4; ++w) {
    issue += (double)h[3 * w];
    wait += (double)h[3 * w + 1];
  }
  issue /= (double)grid * 4 * iters;
  wait /= (double)grid * 4 * iters;
  const double cyc = issue + wait;                      // per iteration per wave
  const double bytes_cu = (double)bpc * 4 * P * 1024;   // per iteration per CU
  const double chip = (double)grid * 4 * P * 1024 * iters / (ms * 1e-3) / 1e12;
  printf("%-5s P=%d blocks/CU=%d  issue %7.1f cyc/piece  wait %7.1f cyc  iter %7.1f cyc  %6.1f B/cyc/CU  %6.2f TB/s\n",
         MODE == 0 ? "lds" : "vgpr", P, bpc, issue / P, wait, cyc, bytes_cu / cyc, chip);
}


// The same loop on waves 0-3 of a 512-thread block while waves 4-7 (one per SIMD beside each loader) run
// back-to-back v_mfma_i32_16x16x64_i8 on registers: the issue cost of a piece beside a matrix wave, and the
// matrix wave's cycles per MFMA beside a loader (out[3 w + 2] = MFMAs issued by a matrix wave).
template <int MODE, int P>
__global__ __launch_bounds__(512) void dma_mfma_loop(const int8_t* __restrict__ src, uint32_t mask, int iters,
                                                     unsigned long long* __restrict__ out, int mfma_per_iter) {
  __shared__ __attribute__((aligned(16))) int8_t lds[32768];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int w = blockIdx.x * 8 + wave;
  if (wave >= 4) {
    v4i acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = v4i{i + lane, 1, 2, 3};
    const v4i a = {lane, 3, 5, 7}, b = {7, lane, 3, 1};
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it)
      for (int k = 0; k < mfma_per_iter; k += 8) {
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, acc[i], 0, 0, 0);
      }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    int x = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) x ^= acc[i][0] ^ acc[i][1] ^ acc[i][2] ^ acc[i][3];
    if (lane == 0) {
      out[3 * w] = t1 - t0;
      out[3 * w + 1] = (unsigned long long)(x & 1);
      out[3 * w + 2] = (unsigned long long)iters * mfma_per_iter;
    }
    return;
  }
  const uint32_t lbase = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)(lds + wave * 8192));
  uint32_t off = ((blockIdx.x * 4 + wave) * 8192u) & mask;
  unsigned long long t_issue = 0, t_wait = 0;
  v4i sink = {0, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
    v4i r[P];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const int8_t* a = src + ((off + p * 1024u) & mask) + lane * 16;
      if (MODE == 0) {
        uint32_t keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\t"
            "s_mov_b32 m0, %2\n\t"
            "s_nop 0\n\t"
            "global_load_lds_dwordx4 %1, off\n\t"
            "s_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(a), "s"(lbase + p * 1024u)
            : "memory");
      } else {
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r[p]) : "v"(a) : "memory");
      }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long t2 = __builtin_amdgcn_s_memtime();
    if (MODE == 1) {
#pragma unroll
      for (int p = 0; p < P; ++p) {
        asm volatile("" : "+v"(r[p]));
        sink ^= r[p];
      }
    }
    t_issue += t1 - t0;
    t_wait += t2 - t1;
    off = (off + 37u * 1024u) & mask;
  }
  if (lane == 0) {
    out[3 * w] = t_issue;
    out[3 * w + 1] = t_wait;
    out[3 * w + 2] = (unsigned long long)(sink[0] ^ sink[1] ^ sink[2] ^ sink[3]) & 1ull;
  }
}

template <int MODE, int P>
void run_partner(const int8_t* src, uint32_t mask, int cus, unsigned long long* dout, int mfma_per_iter) {
  const int iters = 2000;
  const int grid = cus;  // one 512-thread block per CU
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL((dma_mfma_loop<MODE, P>), dim3(grid), dim3(512), 0, 0, src, mask, iters, dout, mfma_per_iter);
    (void)hipDeviceSynchronize();
  }
  std::vector<unsigned long long> h(3 * (size_t)grid * 8);
  (void)hipMemcpy(h.data(), dout, h.size() * 8, hipMemcpyDeviceToHost);
  double issue = 0, wait = 0, mcyc = 0, mcount = 0;
  for (int b = 0; b < grid; ++b)
    for (int wv = 0; wv < 8; ++wv) {
      const size_t w = (size_t)b * 8 + wv;
      if (wv < 4) {
        issue += (double)h[3 * w];
        wait += (double)h[3 * w + 1];
      } else {
        mcyc += (double)h[3 * w];
        mcount += (double)h[3 * w + 2];
      }
    }
  issue /= (double)grid * 4 * iters;
  wait /= (double)grid * 4 * iters;
  printf("%-5s P=%d beside MFMA (%3d per loader iteration): issue %7.1f cyc/piece  wait %7.1f cyc  | MFMA wave %6.2f cyc/mfma\n",
         MODE == 0 ? "lds" : "vgpr", P, mfma_per_iter, issue / P, wait, mcyc / mcount);
}

template <int MODE>
void sweep(const int8_t* src, uint32_t mask, int cus, unsigned long long* dout) {
  for (int bpc : {1, 2, 4}) {
    run<MODE, 1>(src, mask, bpc, cus, dout);
    run<MODE, 2>(src, mask, bpc, cus, dout);
    run<MODE, 4>(src, mask, bpc, cus, dout);
    run<MODE, 8>(src, mask, bpc, cus, dout);
  }
}

int main() {
  int dev = 0, cus = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const size_t n = 1 << 20;  // 1 MiB source: L2-resident on every XCD
  int8_t* src = nullptr;
  unsigned long long* dout = nullptr;
  if (hipMalloc(&src, n + 4096) != hipSuccess || hipMalloc(&dout, 3 * 8 * (size_t)cus * 8 * 4) != hipSuccess) {
    printf("alloc failed\n");
    return 1;
  }
  (void)hipMemset(src, 1, n + 4096);
  printf("CUs %d; s_memtime cycles; source 1 MiB (L2-resident), 2000 iterations\n", cus);
  sweep<0>(src, (uint32_t)(n - 1) & ~15u, cus, dout);
  sweep<1>(src, (uint32_t)(n - 1) & ~15u, cus, dout);
  const uint32_t m = (uint32_t)(n - 1) & ~15u;
  for (int k : {32, 64}) {
    run_partner<0, 2>(src, m, cus, dout, k);
    run_partner<0, 4>(src, m, cus, dout, k);
    run_partner<1, 2>(src, m, cus, dout, k);
    run_partner<1, 4>(src, m, cus, dout, k);
  }
  (void)hipFree(src);
  (void)hipFree(dout);
  return 0;
}
