// Phase-timing instrumentation for diagnostic builds only (tools/gemm_stamps.py builds with
// -DQVIT_GEMM_STAMPS, tools/attn_bench.py --stamps with -DQVIT_ATT_STAMPS). The shipping library is
// compiled without either define: every hook below is then an empty macro / empty inline member and
// the reader entry points do not exist (they are not part of include/qvit_hip.h).
//
// Each wave accumulates s_memtime deltas per phase in registers and lane 0 adds them into a device
// array once per wave; the host reads the array back with the qvit_*_stamps(host, reset) readers.
#pragma once

#include "qvit_common.h"

// ---- persistent GEMM (gemm_w4a8.hip): 0 prologue, 1 DMA issue, 2 stage wait,
//      3 fragment reads + MFMA issue, 4 epilogue, 5 step-top drain, 6 LayerNorm job
//      (EPI_RESID_LN), [7] wave count
#ifdef QVIT_GEMM_STAMPS
namespace {
__device__ unsigned long long qvit_gemm_stamp_sums[8];
}  // namespace
#define QVIT_STAMP_DECL                               \
  unsigned long long st_acc[7] = {0, 0, 0, 0, 0, 0, 0}; \
  unsigned long long st_prev = __builtin_amdgcn_s_memtime();
#define QVIT_STAMP(i)                                             \
  do {                                                            \
    const unsigned long long st_t = __builtin_amdgcn_s_memtime(); \
    st_acc[i] += st_t - st_prev;                                  \
    st_prev = st_t;                                               \
  } while (0)
#define QVIT_STAMP_FLUSH                                                                           \
  do {                                                                                             \
    if (lane == 0) {                                                                               \
      for (int st_i = 0; st_i < 7; ++st_i) atomicAdd(&qvit_gemm_stamp_sums[st_i], st_acc[st_i]); \
      atomicAdd(&qvit_gemm_stamp_sums[7], 1ull);                                                   \
    }                                                                                              \
  } while (0)
#define QVIT_GEMM_STAMP_READER                                                                   \
  extern "C" int qvit_gemm_stamps(unsigned long long* host8, int reset) {                       \
    if (reset) {                                                                                 \
      const unsigned long long z[8] = {};                                                        \
      return qvit_hip_status(hipMemcpyToSymbol(HIP_SYMBOL(qvit_gemm_stamp_sums), z, sizeof(z))); \
    }                                                                                            \
    return qvit_hip_status(                                                                      \
        hipMemcpyFromSymbol(host8, HIP_SYMBOL(qvit_gemm_stamp_sums), 8 * sizeof(unsigned long long))); \
  }
#else
#define QVIT_STAMP_DECL
#define QVIT_STAMP(i) \
  do {                \
  } while (0)
#define QVIT_STAMP_FLUSH \
  do {                   \
  } while (0)
#ifndef QVIT_GEMM_LSTAMPS
#define QVIT_GEMM_STAMP_READER
#endif
#endif

// ---- light variant (-DQVIT_GEMM_LSTAMPS): three stamps per TILE, none per stage, so the main loop's timing
//      is left alone: [0] tile head (stage-0 wait), [1] main loop incl. the tail steps, [2] epilogue,
//      [3] wave lifetime in shader cycles (s_memtime), [4] the same in 100 MHz ticks (s_memrealtime: the
//      in-kernel clock is [3] / [4] * 100 MHz), [5] tiles, [7] waves
#ifdef QVIT_GEMM_LSTAMPS
namespace {
__device__ unsigned long long qvit_gemm_stamp_sums[8];
}  // namespace
#define QVIT_LSTAMP_DECL                                          \
  unsigned long long lst_acc[3] = {0, 0, 0};                      \
  unsigned long long lst_tiles = 0;                               \
  const unsigned long long lst_t0 = __builtin_amdgcn_s_memtime(); \
  const unsigned long long lst_r0 = __builtin_amdgcn_s_memrealtime(); \
  unsigned long long lst_prev = lst_t0;
#define QVIT_LSTAMP(i)                                             \
  do {                                                             \
    const unsigned long long lst_t = __builtin_amdgcn_s_memtime(); \
    lst_acc[i] += lst_t - lst_prev;                                \
    lst_prev = lst_t;                                              \
    if ((i) == 2) ++lst_tiles;                                     \
  } while (0)
#define QVIT_LSTAMP_FLUSH                                                                            \
  do {                                                                                               \
    const unsigned long long lst_t1 = __builtin_amdgcn_s_memtime();                                  \
    const unsigned long long lst_r1 = __builtin_amdgcn_s_memrealtime();                              \
    if (lane == 0) {                                                                                 \
      for (int st_i = 0; st_i < 3; ++st_i) atomicAdd(&qvit_gemm_stamp_sums[st_i], lst_acc[st_i]);    \
      atomicAdd(&qvit_gemm_stamp_sums[3], lst_t1 - lst_t0);                                          \
      atomicAdd(&qvit_gemm_stamp_sums[4], lst_r1 - lst_r0);                                          \
      atomicAdd(&qvit_gemm_stamp_sums[5], lst_tiles);                                                \
      atomicAdd(&qvit_gemm_stamp_sums[7], 1ull);                                                     \
    }                                                                                                \
  } while (0)
#define QVIT_GEMM_STAMP_READER                                                                   \
  extern "C" int qvit_gemm_stamps(unsigned long long* host8, int reset) {                       \
    if (reset) {                                                                                 \
      const unsigned long long z[8] = {};                                                        \
      return qvit_hip_status(hipMemcpyToSymbol(HIP_SYMBOL(qvit_gemm_stamp_sums), z, sizeof(z))); \
    }                                                                                            \
    return qvit_hip_status(                                                                      \
        hipMemcpyFromSymbol(host8, HIP_SYMBOL(qvit_gemm_stamp_sums), 8 * sizeof(unsigned long long))); \
  }
#else
#define QVIT_LSTAMP_DECL
#define QVIT_LSTAMP(i) \
  do {                 \
  } while (0)
#define QVIT_LSTAMP_FLUSH \
  do {                    \
  } while (0)
#endif

// ---- attention bodies (attn_common.h): 0 block wait + DMA issue, 1 scores, 2 softmax, 3 PV,
//      4 epilogue, 5 query-block reads, [15] wave count
//      (-DQVIT_ATT_LSTAMPS: the same buckets without the fused kernel's per-k-step marks 7 and 8, so only the unit's
//      phase boundaries are stamped: projection (9), epilogue (6), attention (0), store (4))
#if defined(QVIT_ATT_LSTAMPS) && !defined(QVIT_ATT_STAMPS)
#define QVIT_ATT_STAMPS
#define QVIT_ATT_LIGHT 1
#else
#define QVIT_ATT_LIGHT 0
#endif
namespace qvit_attn {
#ifdef QVIT_ATT_STAMPS
static __device__ unsigned long long qvit_att_stamp_sums[16];
struct Stamps {
  unsigned long long a[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long prev = __builtin_amdgcn_s_memtime();
  QVIT_DEV void mark(int i) {
    if (QVIT_ATT_LIGHT && (i == 7 || i == 8)) return;
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    a[i] += t - prev;
    prev = t;
  }
  QVIT_DEV void flush() {
    if ((threadIdx.x & 63) == 0) {
      for (int i = 0; i < 10; ++i) atomicAdd(&qvit_att_stamp_sums[i], a[i]);
      atomicAdd(&qvit_att_stamp_sums[15], 1ull);
    }
  }
};
#else
struct Stamps {
  QVIT_DEV void mark(int) {}
  QVIT_DEV void flush() {}
};
#endif
}  // namespace qvit_attn

#ifdef QVIT_ATT_STAMPS
#define QVIT_ATT_STAMP_READER(fn)                                                                            \
  extern "C" int fn(unsigned long long* host8, int reset) {                                                  \
    if (reset) {                                                                                             \
      const unsigned long long z[16] = {};                                                                   \
      return qvit_hip_status(hipMemcpyToSymbol(HIP_SYMBOL(qvit_attn::qvit_att_stamp_sums), z, sizeof(z))); \
    }                                                                                                        \
    return qvit_hip_status(                                                                                  \
        hipMemcpyFromSymbol(host8, HIP_SYMBOL(qvit_attn::qvit_att_stamp_sums), 16 * sizeof(unsigned long long))); \
  }
#else
#define QVIT_ATT_STAMP_READER(fn)
#endif
