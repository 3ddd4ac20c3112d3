// Weight-stationary int8-code GEMM for the Mlp.fc1 shape class (quant_layers.py:495-499 under vit_model.py:172):
//   codes[m, n] = q_next(GELU(d_a d_w sum_k A[m, k] W[n, k] + bias[n]))     (or without the GELU)
// the same arithmetic as gemm_kernel<W4, EPI_I8(_GELU)> (gemm_w4a8.hip), bit for bit, on a different schedule.
//
// Why a second schedule: in gemm_kernel every 64-deep stage is a workgroup barrier plus four LDS-DMA pieces per wave,
// and the int8 epilogue's VALU competes with the SIMD partner's 16x16x64 MFMAs, each of which holds the SIMD's vector
// issue for half of its cycles. Measured per tile and wave (round 5, light stamps): 20.9 k cycles of main loop for
// 6.1 k of own MFMA, 9.8 k of epilogue for ~950 VALU. Here:
//   * one 512-thread workgroup per CU holds a 32 NTN-row panel of the weights for the whole launch, unpacked to
//     16x-scaled int8 in LDS once (NKC x NTN x 2 fragments of 1 KiB, lane-linear: conflict-free ds_read_b128);
//   * the 32 workgroups of an XCD hold the 32 panels of N (N = 32 x 32 NTN: fc1 of ViT-B 3072 = 32 x 96, ViT-L
//     4096 = 32 x 128) and walk the XCD's share of the rows in the same order, so every activation row is fetched
//     into the XCD's L2 once and read by all 32 CUs from there;
//   * each wave owns 64-row tiles (rows 64 i .. + 63, i = its XCD range's wave-tiles w, w + 8, ...) and streams their
//     activation fragments straight from global memory into registers, two 64-deep stages ahead (no LDS-DMA, no
//     barrier: the waves of a CU never wait for each other after the weight fill). The activations come in the
//     MFMA operand order (QVIT_ACT_T32, written by the producing LayerNorm, qvit_layernorm_quant_i8_t32): every
//     fragment load is one contiguous KiB. (Loaded from row-major codes, each lane of a fragment load is its own
//     row, 63 L1 accesses per instruction: the texture path was 78 % busy and the k-loop ran at 4.7x its MFMA
//     time, round-5 PMC and stamps.)
//   * v_mfma_i32_32x32x32_i8 (32 cycles, holds vector issue for 8): the SIMD partner's epilogue VALU gets three
//     quarters of the issue slots instead of half.
// Operand maps (tools/calib/mfma_i8_32x32_maps.hip, exact): lane l holds A[l & 31][16 (l >> 5) + j] and
// B[16 (l >> 5) + j][l & 31]; D register r = row (r & 3) + 8 (r >> 2) + 4 (l >> 5), column l & 31. A = weights: the
// panel's MFMA row i holds weight row 32 u + p(i), p(i) = 16 ((i >> 2) & 1) + 4 (i >> 3) + (i & 3), so lane (m, h)
// ends with the 16 consecutive columns 32 u + 16 h .. + 15 of its token m: one 16-B code store per accumulator.
// The k order inside a 32-deep step is the same for A and B (the contraction is an exact integer sum).
#include <type_traits>

#include "qvit_common.h"

// Diagnostic builds only (-DQVIT_GEMM_WS_STAMPS, tools/gemm_stamps.py --ws): per wave, s_memtime sums of [0] the
// k-loops, [1] the epilogues, [2] the weight fill, [3] the wave's lifetime in shader cycles and [4] in 100 MHz ticks
// (s_memrealtime), [5] tiles, [7] waves. Three stamps per tile, none inside the k-loop.
#ifdef QVIT_GEMM_WS_STAMPS
namespace {
__device__ unsigned long long qvit_ws_stamp_sums[8];
}
#define WS_STAMP(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#else
#define WS_STAMP(v)
#endif

namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int WS_WAVES = 8;
#ifndef QVIT_WS_PD
#define QVIT_WS_PD 2
#endif
constexpr int PD = QVIT_WS_PD;  // 64-deep activation stages loaded ahead of the one computing
// stages loaded as one group: the loads of a group touch each 128-B line of its rows back to back (pairs of 64-B
// stage chunks), so the L1 serves all but the first of them; loaded one stage at a time a line's second half was
// evicted before its turn (the k-loop ran at 4.7x its MFMA time, round-5 stamps)
#ifndef QVIT_WS_GS
#define QVIT_WS_GS 2
#endif
constexpr int GS = QVIT_WS_GS;
constexpr int WS_NT = WS_WAVES * 64;
constexpr int WS_TBL_BYTES = 17408;                       // code table region (<= 2174 buckets, as gemm_kernel)
constexpr int WS_TABLE_MAX_NB = (WS_TBL_BYTES - 16) / 8;

template <int NTN, int NKC>
struct WsGeo {
  static constexpr int FRAGS = NKC * NTN * 2;             // 1-KiB weight fragments (stage, 32-row tile, k half)
  static constexpr int WBYTES = FRAGS * 1024;
  static constexpr int BIAS = NTN * 32 * 4;
  static constexpr int LDS = WBYTES + WS_TBL_BYTES + BIAS + 64;
  static_assert(LDS <= 163840, "LDS budget");
};

struct WsArgs {
  const float* d_act;
  const float* d_wt;
  const float* bias;
  int out_qtype;
  const float* out_d;
  const float* out_qm;
  const float* out_t;
  int out_levels;
  const int8_t* table;
};

QVIT_DEV uint32_t nib16_lo(uint32_t p) { return (p << 4) & 0xF0F0F0F0u; }
QVIT_DEV uint32_t nib16_hi(uint32_t p) { return p & 0xF0F0F0F0u; }

// packed row of weight row n in the qvit_pack_weight image (inside each 64-row group the 2-bit fields [3:2] and
// [5:4] are swapped: an involution) and the byte offset of its 8-B chunk c (16 k) in k-stage st
QVIT_DEV uint32_t w4_image_offset(int n, int st, int c, int nk) {
  const int rho = (n & ~63) | (((n >> 2) & 3) << 4) | (((n >> 4) & 3) << 2) | (n & 3);
  const int r = rho & 255;
  return (uint32_t)(((rho >> 8) * nk + st) * 8192) + (uint32_t)(r * 32 + 8 * (c ^ (((r >> 3) & 1) << 1)));
}

template <int NTN, int NKC, int EPI>
__global__ __launch_bounds__(WS_NT, 1) void gemm_ws_kernel(const int8_t* __restrict__ A, int M,
                                                           const int8_t* __restrict__ Wp, int8_t* __restrict__ C,
                                                           int64_t ldc, int panels, WsArgs ep) {
  using G = WsGeo<NTN, NKC>;
  constexpr int PW = 32 * NTN;  // panel width (weight rows)
  __shared__ __attribute__((aligned(16))) int8_t smem[G::LDS];
  int8_t* wl = smem;
  int8_t* tbl = smem + G::WBYTES;
  float* bias_l = reinterpret_cast<float*>(tbl + WS_TBL_BYTES);
  QParams* qp_l = reinterpret_cast<QParams*>(tbl + WS_TBL_BYTES + G::BIAS);

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
#ifdef QVIT_GEMM_WS_STAMPS
  const unsigned long long st_t0 = __builtin_amdgcn_s_memtime(), st_r0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long st_loop = 0, st_epi = 0, st_fill = 0, st_tiles = 0;
#endif
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, team = gridDim.x >> 3;
  const int groups = team / panels;
  if (slot >= groups * panels) return;  // (team not a multiple of the panel count: surplus workgroups idle)
  const int pnl = slot % panels, grp = slot / panels;
  const int n0 = pnl * PW;

  // ---- this wave's 64-row tiles: XCD x owns wave-tiles [xlo, xhi) of ceil(M / 64), its group a contiguous part
  const int nwt = (M + 63) >> 6;
  const int xlo = (int)((int64_t)xcd * nwt / 8), xhi = (int)((int64_t)(xcd + 1) * nwt / 8);
  const int glo = xlo + (int)((int64_t)(xhi - xlo) * grp / groups);
  const int ghi = xlo + (int)((int64_t)(xhi - xlo) * (grp + 1) / groups);
  int ti = glo + wave;
  const bool has_tiles = ti < ghi;  // (waves without a tile still take part in the weight fill)

  const int lane = tid & 63;
  const int lr = lane & 31, lh = lane >> 5;
  // T32 activations: the 1-KiB block of rows 32 mb .. + 31, k 32 kb .. + 31 at (mb KB32 + kb) KiB, lane l's 16 B at
  // 16 l (rows past M exist in the padded buffer: loaded, never stored); per tile one uniform offset
  const uint32_t kb32 = (uint32_t)(NKC * 2);
  const uint32_t lane16 = (uint32_t)lane * 16u;
  auto aoffs = [&](int i, uint32_t (&o)[2]) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < 2; ++t) o[t] = __builtin_amdgcn_readfirstlane((uint32_t)(2 * i + t) * kb32 * 1024u);
  };
  const int8_t* wlane = wl + lane * 16;
  auto wload = [&](int s, v4i (&w)[NTN][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < NTN; ++u)
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) w[u][kh] = *reinterpret_cast<const v4i*>(wlane + ((s * NTN + u) * 2 + kh) * 1024);
  };

  v16i acc[2][NTN];
  // activation stages of a tile (the k-loop is straight-line code, so each stage's fragments are their own values:
  // three stages live at a time), xs[NKC], xs[NKC + 1] = the next tile's stages 0, 1, carried over
  v4i xs[NKC + PD][2][2];
  v4i wf[2][NTN][2];
  uint32_t ao[2];
  aoffs(ti, ao);
  // (t, stage, k half) order: one row tile's accesses to the same lines are adjacent
  auto agroup = [&](const uint32_t (&o)[2], int s0, int slot0) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int g = 0; g < GS; ++g)
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
          xs[slot0 + g][t][kh] =
              *reinterpret_cast<const v4i*>(A + o[t] + (uint32_t)((2 * (s0 + g) + kh) * 1024) + lane16);
  };
  static_assert(NKC % GS == 0 && PD % GS == 0, "stage groups");
  // the first tile's first stages load while the weights are filled in
  if (has_tiles) {
#pragma unroll
    for (int s = 0; s < PD; s += GS) agroup(ao, s, s);
  }

  // ---- once per launch: the panel's weights (int4 image -> 16x-scaled int8, lane-linear fragments), its bias, the
  // quantizer's code table and scalars
  {
    constexpr int SLOTS = G::FRAGS * 64;  // 16-B fragment slots
    constexpr int PER = SLOTS / WS_NT;
    static_assert(SLOTS % WS_NT == 0, "fill slots per thread");
    uint2 p[PER];  // all of a thread's loads in flight together
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int q = tid + j * WS_NT;
      const int f = q >> 6, l = q & 63;
      const int kh = f & 1, u = (f >> 1) % NTN, st = (f >> 1) / NTN;
      const int i = l & 31, h = l >> 5;
      const int n = n0 + 32 * u + 16 * ((i >> 2) & 1) + 4 * (i >> 3) + (i & 3);
      p[j] = *reinterpret_cast<const uint2*>(Wp + w4_image_offset(n, st, 2 * kh + h, NKC));
    }
#pragma unroll
    for (int j = 0; j < PER; ++j)
      *reinterpret_cast<v4i*>(wl + (tid + j * WS_NT) * 16) =
          v4i{(int)nib16_lo(p[j].x), (int)nib16_hi(p[j].x), (int)nib16_lo(p[j].y), (int)nib16_hi(p[j].y)};
    for (int j = tid; j < PW; j += WS_NT) bias_l[j] = ep.bias ? ep.bias[n0 + j] : 0.f;
  }
  bool use_table = false;
  float t_c0 = 0.f, t_invw = 0.f, t_top = 0.f;
  if (ep.table != nullptr) {
    const EpiTableHdr hd = *reinterpret_cast<const EpiTableHdr*>(ep.table);
    use_table = hd.valid != 0 && hd.nb >= 1 && hd.nb <= WS_TABLE_MAX_NB;
    t_c0 = hd.c0;
    t_invw = hd.inv_w;
    t_top = epi_top(hd.nb);
    if (use_table)
      for (int i = tid; i < (16 + 8 * hd.nb + 15) / 16; i += WS_NT)
        reinterpret_cast<v4i*>(tbl)[i] = reinterpret_cast<const v4i*>(ep.table)[i];
  }
  if (!use_table && tid == 0) *qp_l = load_qparams(ep.out_qtype, ep.out_d, ep.out_qm, ep.out_t, ep.out_levels);
  // W4 accumulators hold 16 acc: the 1/16 rides in alpha (exact), as in gemm_kernel
  const float alpha = (*ep.d_act) * (*ep.d_wt) * 0.0625f;
  __syncthreads();  // the only workgroup barrier
#ifdef QVIT_GEMM_WS_STAMPS
  st_fill = __builtin_amdgcn_s_memtime() - st_t0;
#endif
  if (!has_tiles) return;

  auto tile = [&](int i, int inext) __attribute__((always_inline)) {
    WS_STAMP(st_a);
    uint32_t an[2];
    aoffs(inext, an);
    wload(0, wf[0]);
#pragma unroll
    for (int s = 0; s < NKC; ++s) {
      // stages s + PD .. + GS - 1 (past the tile's end: the next tile's first stages)
      if (s % GS == 0) {
        if (s + PD < NKC) agroup(ao, s + PD, s + PD);
        else agroup(an, s + PD - NKC, s + PD);
      }
      if (s + 1 < NKC) wload(s + 1, wf[(s + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
      const v4i(&x)[2][2] = xs[s];
      const v4i(&w)[NTN][2] = wf[s & 1];
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int u = 0; u < NTN; ++u)
#pragma unroll
          for (int t = 0; t < 2; ++t)
            acc[t][u] = __builtin_amdgcn_mfma_i32_32x32x32_i8(w[u][kh], x[t][kh],
                                                              (s == 0 && kh == 0) ? v16i{} : acc[t][u], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    ao[0] = an[0];
    ao[1] = an[1];
#pragma unroll
    for (int s = 0; s < PD; ++s)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int kh = 0; kh < 2; ++kh) xs[s][t][kh] = xs[NKC + s][t][kh];

    // ---- epilogue: lane (token 64 i + 32 t + lr, h) holds columns n0 + 32 u + 16 h .. + 15 of acc[t][u]
    WS_STAMP(st_b);
    __builtin_amdgcn_s_setprio(1);
    auto store16 = [&](int t, int u, const uint32_t (&wd)[4]) __attribute__((always_inline)) {
      const int m = 64 * i + 32 * t + lr;
      if (m < M) *reinterpret_cast<uint4*>(C + (int64_t)m * ldc + n0 + 32 * u + 16 * lh) = make_uint4(wd[0], wd[1], wd[2], wd[3]);
    };
    if (use_table) {
      // the 2 NTN groups g = (u, t) of 16 codes, software-pipelined: group g + 1's 16 table lookups are issued
      // before group g's selects and store, so each group's LDS latency runs under the previous group's VALU
      const int8_t* ent = tbl + sizeof(EpiTableHdr);
      float v[2][16];
      uint2 e[2][16];
      auto look = [&](int g, int b) __attribute__((always_inline)) {
        const int u = g >> 1, t = g & 1;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 bq = *reinterpret_cast<const float4*>(bias_l + 32 * u + 16 * lh + 4 * q);
          const float bb[4] = {bq.x, bq.y, bq.z, bq.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[b][4 * q + j] = fmaf(alpha, (float)acc[t][u][4 * q + j], bb[j]);
            e[b][4 * q + j] = *epi_entry(ent, v[b][4 * q + j], t_c0, t_invw, t_top);
          }
        }
      };
      look(0, 0);
#pragma unroll
      for (int g = 0; g < 2 * NTN; ++g) {
        if (g + 1 < 2 * NTN) look(g + 1, (g + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);
        const int b = g & 1;
        uint32_t wd[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          epi_select_byte<0>(wd[q], v[b][4 * q], __uint_as_float(e[b][4 * q].x), e[b][4 * q].y);
          epi_select_byte<1>(wd[q], v[b][4 * q + 1], __uint_as_float(e[b][4 * q + 1].x), e[b][4 * q + 1].y);
          epi_select_byte<2>(wd[q], v[b][4 * q + 2], __uint_as_float(e[b][4 * q + 2].x), e[b][4 * q + 2].y);
          epi_select_byte<3>(wd[q], v[b][4 * q + 3], __uint_as_float(e[b][4 * q + 3].x), e[b][4 * q + 3].y);
        }
        store16(g & 1, g >> 1, wd);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {  // no valid table: the per-element quantizer (rare; same function as gemm_kernel's staged path)
      const QParams qp = *qp_l;
#pragma unroll
      for (int u = 0; u < NTN; ++u)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          uint32_t wd[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            float k[4];
            bool need[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              float vv = fmaf(alpha, (float)acc[t][u][4 * q + j], bias_l[32 * u + 16 * lh + 4 * q + j]);
              if (EPI == QVIT_EPI_I8_GELU) vv = gelu_ref(vv);
              k[j] = quant_fast(vv, qp, need[j]);
              if (need[j]) k[j] = quant_fixup(vv, qp);
            }
            wd[q] = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) wd[q] |= ((uint32_t)(uint8_t)to_i8_sat(k[j])) << (8 * j);
          }
          store16(t, u, wd);
        }
    }
    __builtin_amdgcn_s_setprio(0);
#ifdef QVIT_GEMM_WS_STAMPS
    WS_STAMP(st_c);
    st_loop += st_b - st_a;
    st_epi += st_c - st_b;
    ++st_tiles;
#endif
  };
  for (;;) {
    const int tn = ti + WS_WAVES;
    const int inext = tn < ghi ? tn : ti;  // (no next tile: its prefetch re-reads this one's rows, unused)
    tile(ti, inext);
    if (tn >= ghi) break;
    ti = tn;
  }
#ifdef QVIT_GEMM_WS_STAMPS
  const unsigned long long st_t1 = __builtin_amdgcn_s_memtime(), st_r1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0) {
    atomicAdd(&qvit_ws_stamp_sums[0], st_loop);
    atomicAdd(&qvit_ws_stamp_sums[1], st_epi);
    atomicAdd(&qvit_ws_stamp_sums[2], st_fill);
    atomicAdd(&qvit_ws_stamp_sums[3], st_t1 - st_t0);
    atomicAdd(&qvit_ws_stamp_sums[4], st_r1 - st_r0);
    atomicAdd(&qvit_ws_stamp_sums[5], st_tiles);
    atomicAdd(&qvit_ws_stamp_sums[7], 1ull);
  }
#endif
}

template <int NTN, int NKC>
int ws_launch(int epi, const int8_t* A, int64_t M, const void* Wp, int64_t N, void* C, int64_t ldc, const WsArgs& ep,
              hipStream_t stream) {
  const int panels = (int)(N / (32 * NTN));
  const int8_t* w = reinterpret_cast<const int8_t*>(Wp);
  int8_t* c = reinterpret_cast<int8_t*>(C);
  if (epi == QVIT_EPI_I8_GELU)
    hipLaunchKernelGGL((gemm_ws_kernel<NTN, NKC, QVIT_EPI_I8_GELU>), dim3(256), dim3(WS_NT), 0, stream, A, (int)M, w, c,
                       ldc, panels, ep);
  else
    hipLaunchKernelGGL((gemm_ws_kernel<NTN, NKC, QVIT_EPI_I8>), dim3(256), dim3(WS_NT), 0, stream, A, (int)M, w, c,
                       ldc, panels, ep);
  return qvit_hip_status(hipGetLastError());
}

}  // namespace

#ifdef QVIT_GEMM_WS_STAMPS
extern "C" int qvit_gemm_ws_stamps(unsigned long long* host8, int reset) {
  if (reset) {
    const unsigned long long z[8] = {};
    return qvit_hip_status(hipMemcpyToSymbol(HIP_SYMBOL(qvit_ws_stamp_sums), z, sizeof(z)));
  }
  return qvit_hip_status(hipMemcpyFromSymbol(host8, HIP_SYMBOL(qvit_ws_stamp_sums), 8 * sizeof(unsigned long long)));
}
#endif

extern "C" int qvit_gemm_a32_fits(int64_t K, int wfmt, int64_t N, int64_t npad, int epilogue) {
  if (wfmt != QVIT_W4 || (epilogue != QVIT_EPI_I8 && epilogue != QVIT_EPI_I8_GELU) || N != npad) return 0;
  return (K == 768 || K == 1024) && N == 32 * 96;
}

extern "C" int qvit_gemm_a32(const int8_t* A, int64_t M, int64_t K, const void* Wp, int wfmt, int64_t N, int64_t npad,
                             const float* d_act, const float* d_wt, const float* bias, int epilogue, void* C,
                             int64_t ldc, int out_qtype, const float* out_d, const float* out_qm, const float* out_t,
                             int out_levels, const void* epi_table, hipStream_t stream) {
  if (!A || !Wp || !C || !d_act || !d_wt) return QVIT_ENULL;
  if (!qvit_gemm_a32_fits(K, wfmt, N, npad, epilogue)) return QVIT_EINVAL;
  if (M < 0 || M > INT32_MAX / 2 || ldc < N) return QVIT_EINVAL;
  if ((M + 63) / 64 * 64 * K > (int64_t)0xFFFFFFFF) return QVIT_EINVAL;  // 32-bit activation offsets
  const int q = out_qtype & 0xff;
  if (q != QVIT_QT_LINEAR && q != QVIT_QT_NONLINEAR && q != QVIT_QT_ULTRA_ACT) return QVIT_EINVAL;
  if (q == QVIT_QT_ULTRA_ACT ? (out_levels < 1 || out_levels > 127) : (!out_d || !out_qm)) return QVIT_EINVAL;
  if ((((uintptr_t)A) & 15) || (((uintptr_t)Wp) & 15) || (ldc % 16) || (((uintptr_t)C) & 15)) return QVIT_EALIGN;
  if ((bias && (((uintptr_t)bias) & 15)) || (epi_table && (((uintptr_t)epi_table) & 15))) return QVIT_EALIGN;
  if (M == 0) return QVIT_OK;
  const WsArgs ep{d_act, d_wt, bias, out_qtype, out_d, out_qm, out_t, out_levels,
                  reinterpret_cast<const int8_t*>(epi_table)};
  const int8_t* a = reinterpret_cast<const int8_t*>(A);
  if (K == 768) return ws_launch<3, 12>(epilogue, a, M, Wp, N, C, ldc, ep, stream);
  return ws_launch<3, 16>(epilogue, a, M, Wp, N, C, ldc, ep, stream);
}
