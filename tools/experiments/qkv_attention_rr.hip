// EXPERIMENT (round 4), not built into the library: the role-alternating fused qkv + attention kernel
// (qkv_attn_rr_kernel below; the rest of the file is the shipping qkv_attention.hip of that time). It is correct
// (tests/test_gpu_attention.py -k qkv_attention: 23 passed) and slower than the shipping kernel: ViT-B b256 shape,
// random data (tools/attn_bench.py --fused), one box: 424-449 us i8 vs 275 us; in the model 398 vs ~230 us.
// Diagnostic builds on the same box: projection half idle (attention + tile-12 projection only) 359 us; attention
// half idle (projection only) 226 us. Both halves are latency-bound: without the LDS-DMA ring, weight and
// activation fragments stream into registers one k-step ahead, which the 256-register budget (144 projection
// accumulators) cannot deepen; the attention half, with one query tile in flight per wave, exposes the
// S -> softmax -> P.V chain of every key block. See DESIGN.md section 8.
// Fused qkv projection + attention core of Attention.forward (vit_model.py:126-152) for the fused block:
//   qkv = QuantizeLinear(x_codes)  ->  softmax(q k^T * scale) v  ->  proj's activation quantizer
// with q, k, v never leaving the chip. One persistent workgroup (8 waves) per CU walks (image, head)
// units; per unit:
//   1. projection: wave w computes the 192 q|k|v features of its token tiles {2 w', 2 w' + 1} (w' = w
//      rotated by unit) on v_mfma_i32_16x16x64_i8, as a GEMM-style pipeline: the head's three 64-row weight groups
//      of each 64-deep k-step are LDS-DMA'd (global_load_lds, 6 x 1 KiB, no register staging) from the
//      GEMM's pre-tiled int4 image into a 4-slot ring three k-steps ahead; activation fragments go global
//      -> registers three k-steps ahead; one counted vmcnt + barrier per k-step; the MFMAs of k-step s run
//      while the packed weight fragments of k-step s+1 are read from LDS, each unpacked to 16x-scaled int8
//      right before its two MFMAs;
//   2. epilogue: v = (d_a d_w acc + bias) * in_scale split into fp16 hi/lo exactly as
//      qvit_gemm_qkv_split does; q stays in registers (one permlane16 swap turns the two tiles into the
//      32-query tile's S^T B operands), k and v go to resident LDS images (208 rows, XOR-swizzled);
//   3. attention on v_mfma_f32_32x32x16_f16 (one 32-query tile per wave): the 7 key blocks of 32 with no
//      barrier (K/V resident), block kb + 1's scores issued ahead of block kb's online softmax, P·V, and
//      the output quantizer through its code table (same arithmetic as qvit_attention_split except the
//      order of the terms inside the q·k, P·V and row sums, and a running max kept an integer).
// The next unit's first weight k-steps (ring) and activation k-steps (registers) load while the current
// unit's attention runs. N <= 208.
#include "attn32.h"

#include <algorithm>
#include <type_traits>


namespace {

using namespace qvit_attn;

constexpr int FW = 8;                     // waves
constexpr int FT = FW * 64;               // threads
constexpr int TPW = 2;                    // token / query tiles per wave
constexpr int MAXN = FW * TPW * 16 > 208 ? 208 : FW * TPW * 16;
constexpr int IROWS = 208;                // rows of each K/V image (13 tiles)
constexpr int IMGF = IROWS * 128;         // 26 KiB per fp16 image
constexpr int KV_BYTES = 4 * IMGF + 2048; // K hi, K lo, V hi, V lo + zero rows past V lo (last key block)
constexpr int WGRP = 2048;                // one 64-row weight group of one k-step: 64 rows x 32 B (int4 image)
constexpr int WSLOT = 3 * WGRP;           // q, k, v groups of one k-step: 6 DMA pieces
constexpr int WRING = 4;                  // slots: k-step s computes from slot s % 4, s + 1 is read, s + 2, s + 3 land
constexpr int WDIST = WRING - 1;          // weight k-steps issued ahead
constexpr int XRING = 4;                  // activation register ring (k-steps s .. s + 3)
constexpr int TOPCNT = 2 + 3 * (WDIST - 2);  // vmem ops a wave issues after its DMA piece of k-step s + 1
constexpr int IMG4_STEP = 256 * 32;       // bytes of one (256-row tile, k-step) of the int4 weight image
constexpr int TBL = 8192;                 // code table (<= 1022 buckets)
constexpr int BIAS_MAX = 9216;            // fp32 bias of the qkv layer (<= 2304 features: H * 64 <= 768)
constexpr int LDS_TOTAL = KV_BYTES + WRING * WSLOT + TBL + BIAS_MAX;
static_assert(LDS_TOTAL <= 163840, "LDS budget");

typedef int v4i __attribute__((ext_vector_type(4)));

// int4 codes as 16x-scaled int8 MFMA operands: a nibble in the high half of a byte reads as the signed
// byte 16 w exactly, so the high nibbles need a mask and the low ones a shift and a mask
QVIT_DEV uint32_t nib16_lo(uint32_t p) { return (p << 4) & 0xF0F0F0F0u; }
QVIT_DEV uint32_t nib16_hi(uint32_t p) { return p & 0xF0F0F0F0u; }
// (the empty volatile asm pins the unpack where it is written: without it the IR passes hoist every
// fragment's unpack to the top of the k-step, 48 live registers instead of 4)
QVIT_DEV v4i unpack16(uint2 p) {
  asm volatile("" : "+v"(p));
  return v4i{(int)nib16_lo(p.x), (int)nib16_hi(p.x), (int)nib16_lo(p.y), (int)nib16_hi(p.y)};
}

// NKC: the number of 64-deep k-steps when fixed at compile time (12: K = 768, the ViT-B qkv; ViT-L's
// H * 64 = 1024 exceeds QKV_ATT_MAX_C and takes the split path), which unrolls the projection loop
// completely; 0: K / 64 at run time (K % 256 == 0, e.g. 256, 512 or 1024 with <= 12 heads)
template <int OUT, int NKC>
__global__ __launch_bounds__(FT, 1) void qkv_attn_kernel(
    const int8_t* __restrict__ A, int K, int64_t lda, const int8_t* __restrict__ Wp, int npad,
    const float* __restrict__ d_act, const float* __restrict__ d_wt, const float* __restrict__ bias, int B, int N,
    int H, float scale, float in_scale, void* __restrict__ out, int64_t ldo, int out_qtype, const float* out_d,
    const float* out_qm, const float* out_t, int out_levels, const int8_t* __restrict__ epi_table) {
  __shared__ __attribute__((aligned(16))) int8_t smem[LDS_TOTAL];
  int8_t* kv = smem;
  int8_t* wring = smem + KV_BYTES;
  int8_t* tbl = wring + WRING * WSLOT;
  float* bias_l = reinterpret_cast<float*>(tbl + TBL);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int C = H * 64;
  const int nk = NKC > 0 ? NKC : K / 64;

  // ---- per-workgroup setup: scalars, bias, code table, the zero rows past V lo -----------------------
  const float alpha = (*d_act) * (*d_wt);
  QParams qp{};
  EpiLds tb{nullptr, 0.f, 0.f, 0.f};
  if (OUT == 1) {
    qp = load_qparams(out_qtype, out_d, out_qm, out_t, out_levels);
    if (epi_table != nullptr) {
      const EpiTableHdr hd = *reinterpret_cast<const EpiTableHdr*>(epi_table);
      if (hd.valid != 0 && hd.nb >= 1 && 16 + 8 * hd.nb <= TBL) {
        for (int k = tid; k < (16 + 8 * hd.nb + 15) / 16; k += FT)
          reinterpret_cast<uint4*>(tbl)[k] = reinterpret_cast<const uint4*>(epi_table)[k];
        tb = EpiLds{tbl + sizeof(EpiTableHdr), hd.c0, hd.inv_w, epi_top(hd.nb)};
      }
    }
  }
  // in_scale is a power of two: (alpha acc + b) s == alpha s acc + b s exactly, so it is folded in here
  for (int k = tid; k < 3 * C; k += FT) bias_l[k] = bias ? bias[k] * in_scale : 0.f;
  // the accumulators hold 16 acc (16x-scaled int4 operands): float(16 acc) = 16 float(acc) exactly (|16 acc| <
  // 2^24), so the 1/16 rides in the scale instead of a shift per element — the same fp32 values
  const float alpha_s = alpha * in_scale * 0.0625f;
  // K / V images start zeroed (rows a unit does not write are then always finite), plus the zero rows
  for (int k = tid; k < KV_BYTES / 16; k += FT) reinterpret_cast<uint4*>(kv)[k] = make_uint4(0, 0, 0, 0);

  // ---- units of this workgroup: XCD x owns a contiguous range (the heads of an image share its L2) ----
  const int nunits = B * H;
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, team = gridDim.x >> 3;
  const int per = nunits >> 3, rem = nunits & 7;
  const int ulo = xcd * per + (xcd < rem ? xcd : rem);
  const int uhi = ulo + per + (xcd < rem ? 1 : 0);
  const int my_units = (uhi - ulo - slot + team - 1) / team;  // unit j: ulo + slot + j * team
  const int ntile = (N + 15) / 16;
  const int64_t M = (int64_t)B * N;

  // ---- operand sources of a unit ---------------------------------------------------------------------
  // activations: this lane's rows of the wave's two token tiles as 32-bit byte offsets from A (the launcher
  // checks B N lda < 2^32); weights: the wave's 1-KiB piece of each k-step's 6 (piece i = half i & 1 of
  // group i >> 1: q, k, v), a wave-uniform byte offset from Wp at k-step 0. Waves 6, 7 re-issue pieces 4, 5
  // (the same bytes to the same place), so every wave issues one per k-step and the counted waits are
  // uniform. Units past the end repeat the last one (their loads are never used).
  const int pc = wave < 6 ? wave : wave - 2;
  const uint32_t lds_w = __builtin_amdgcn_readfirstlane(lds_addr(wring) + (uint32_t)((pc >> 1) * WGRP + (pc & 1) * 1024));
  struct Src {
    uint32_t a[TPW];
    uint32_t w;
  };
  auto unit_src = [&](int j, Src& sr) __attribute__((always_inline)) {
    j = j < my_units ? j : my_units - 1;
    const int unit = ulo + slot + j * team;
    const int b = unit / H, h = unit - b * H;
    const int wr = (wave + unit) & (FW - 1);
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt) {
      int64_t m = (int64_t)b * N + 16 * (2 * wr + tt) + fr;
      m = m < M ? m : M - 1;  // tokens past the image: rows of the next one (masked); clamp at the end
      sr.a[tt] = (uint32_t)(m * lda) + (uint32_t)(16 * fq);
    }
    const int feat = (pc >> 1) * C + 64 * h;
    sr.w = __builtin_amdgcn_readfirstlane((uint32_t)((feat >> 8) * nk) * (uint32_t)IMG4_STEP +
                                          (uint32_t)(((feat & 255) >> 6) * WGRP + (pc & 1) * 1024));
  };
  const uint32_t lane16 = 16u * (uint32_t)lane;
  // weight k-step s of a unit -> ring slot rs: this wave's DMA piece
  auto dma_piece = [&](const Src& sr, int s, int rs) __attribute__((always_inline)) {
    dma16s(Wp + sr.w + (uint32_t)s * (uint32_t)IMG4_STEP, lane16, lds_w + (uint32_t)(rs * WSLOT));
  };
  // activation loads walk one running offset per tile (+64 B per k-step, reset to the next unit's rows when
  // the stream crosses into it), advanced by asm so the compiler cannot precompute (and hold) every
  // k-step's address. They are ordinary loads: the compiler tracks their registers and places their
  // vmcnt waits (counting only its own loads, so at least as strict as needed; the DMA pieces it cannot
  // see are waited for explicitly at each k-step's top, which already covers these loads).
  v4i xa[XRING][TPW];
  uint32_t aoff[TPW];
  auto act_load = [&](v4i& xd, int tt) __attribute__((always_inline)) {
    xd = *reinterpret_cast<const v4i*>(A + (size_t)aoff[tt]);
    asm volatile("v_add_u32_e32 %0, 64, %0" : "+v"(aoff[tt]));
  };
  auto act_next = [&](v4i (&xd)[TPW]) __attribute__((always_inline)) {
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt) act_load(xd[tt], tt);
  };
  // packed weight fragment (group p, 16-row tile r) of ring slot rs: the int4 image's swizzle
  // (quant_kernels.hip packed_offset<W4>), conflict-free ds_read_b64; one base register, the rest immediates
  const int8_t* wbase = wring + fr * 32 + ((fq ^ (((fr >> 3) & 1) << 1)) << 3);
  auto wfrag = [&](int rs, int f) __attribute__((always_inline)) {
    return *reinterpret_cast<const uint2*>(wbase + rs * WSLOT + (f >> 2) * WGRP + (f & 3) * 512);
  };

  // attention fragment offsets (attend32): K row reads of key lane & 31, chunk 4 h + c; V^T transposed reads,
  // lane 4 k + p of 16-lane group G supplies row 4 (G >> 1) + k, dims 32 dt + 16 (G & 1) + 4 p
  int koffs[4], voffs[2];
#pragma unroll
  for (int c = 0; c < 4; ++c) koffs[c] = koff(lane & 31, 4 * (lane >> 5) + c);
  // (V's offsets carry the V hi image's start, hidden from the compiler: with 2 IMGF in the immediates the
  // later blocks' offsets pass 64 KiB, and every block then needs base registers of its own)
#pragma unroll
  for (int dt = 0; dt < 2; ++dt) {
    voffs[dt] = 2 * IMGF + v32off(4 * (fq >> 1) + (fr >> 2), 2 * (32 * dt + 16 * (fq & 1) + 4 * (fr & 3)));
    asm volatile("" : "+v"(voffs[dt]));
  }
  const float sl2 = scale * LOG2E / (in_scale * in_scale);
  const bool st16 = ((ldo & 15) == 0) && ((((uintptr_t)out) & 15) == 0);
  Stamps sp;

  if (my_units <= 0) return;  // uniform per workgroup; no barrier has been reached yet
  Src cur, nxt;
  unit_src(0, cur);
  unit_src(1, nxt);
  // prologue: weight k-steps 0, 1 of the first unit, activation k-steps 0, 1, 2
#pragma unroll
  for (int t = 0; t < WDIST; ++t) dma_piece(cur, t, t);
  aoff[0] = cur.a[0];
  aoff[1] = cur.a[1];
  act_next(xa[0]);
  act_next(xa[1]);
  act_next(xa[2]);
  for (int j = 0; j < my_units; ++j) {
    const int unit = ulo + slot + j * team;
    const int b = unit / H, h = unit - b * H;
    const int wr = (wave + unit) & (FW - 1);
    bool tv[TPW];
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt) tv[tt] = 2 * wr + tt < ntile;
    const int nt = (tv[0] ? 1 : 0) + (tv[1] ? 1 : 0);

    // ---- 1. projection ---------------------------------------------------------------------------
    // unit head: everything issued before (the previous unit's output stores included) has landed, the
    // ring slots of k-steps 0 and 1 are complete for every wave; read k-step 0's weight fragments
    __builtin_amdgcn_s_waitcnt(0xC07F);
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    v4i acc[TPW][12];
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt)
#pragma unroll
      for (int f = 0; f < 12; ++f) acc[tt][f] = v4i{0, 0, 0, 0};
    uint2 wfr[12];
    // k-step s (ring slot and activation slot q = s % 4: nk % 4 == 0, so every unit starts at slot 0 and the
    // slot indices are compile-time constants in the 4-step groups):
    //   top (s > 0): this wave's DMA piece of k-step s + 1 landed (TOPCNT = the activation loads and DMA
    //   pieces issued after it may be in flight, which also covers the activations of k-step s), then the
    //   barrier: k-step s + 1's slot is complete for everyone, and every wave is past k-step s - 1, the last
    //   reader of slot (s + 3) % 4;
    //   issue: weight k-step s + 3 -> slot (s + 3) % 4, activation k-step s + 3 -> register slot (s + 3) % 4
    //   (past the unit's end: the next unit's k-steps 0, 1, 2);
    //   MFMAs of k-step s: fragment f + 1 is unpacked while f's two MFMAs run, and each packed fragment is
    //   replaced by k-step s + 1's right after its MFMAs.
    // two: 2 when both of the wave's token tiles {2 wr, 2 wr + 1} are inside the image, else 1 (the second
    // tile's MFMAs are skipped; N = 197 has 13 tiles). The order inside a k-step is pinned (sched_barrier); the DMA piece and the two
    // activation loads go between the first fragments' MFMAs in that order (the next top's count).
    auto kstep = [&](auto two, int s, int q) __attribute__((always_inline)) {
      __builtin_amdgcn_sched_barrier(0);
      if (s > 0) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(TOPCNT) : "memory");
      __builtin_amdgcn_sched_barrier(0);
      sp.mark(7);
      const int rd = (q + WDIST) & 3, rn = (q + 1) & 3;
      const bool more = s + 1 < nk;
      v4i wc = unpack16(wfr[0]);
#pragma unroll
      for (int f = 0; f < 12; ++f) {
        if (decltype(two)::value >= 1) acc[0][f] = __builtin_amdgcn_mfma_i32_16x16x64_i8(wc, xa[q][0], acc[0][f], 0, 0, 0);
        if (decltype(two)::value == 2) acc[1][f] = __builtin_amdgcn_mfma_i32_16x16x64_i8(wc, xa[q][1], acc[1][f], 0, 0, 0);
        if (f < 11) wc = unpack16(wfr[f + 1]);
        if (more) wfr[f] = wfrag(rn, f);
        if (f == 0) {  // weight k-step s + 3 (past the unit's end: the next unit's 0, 1, 2)
          if (s + WDIST < nk) dma_piece(cur, s + WDIST, rd);
          else dma_piece(nxt, s + WDIST - nk, rd);
        }
        if (f == 2) {  // activation k-step s + 3 (past the unit's end: the next unit's 0, 1, 2)
          if (s + 3 == nk) {
            aoff[0] = nxt.a[0];
            aoff[1] = nxt.a[1];
          }
          act_load(xa[(q + 3) & 3][0], 0);
        }
        if (f == 4) act_load(xa[(q + 3) & 3][1], 1);
        __builtin_amdgcn_sched_barrier(0);
      }
      sp.mark(8);
    };
    // with NKC the k-steps of a unit are straight-line code
    // (k-step 0's weight fragments are read inside each variant: values read before the branch would stay
    // live across both of its structurized arms)
    auto kloop = [&](auto two) __attribute__((always_inline)) {
#pragma unroll
      for (int f = 0; f < 12; ++f) wfr[f] = wfrag(0, f);
      if constexpr (NKC > 0) {
#pragma unroll
        for (int s = 0; s < NKC; s += 4) {
          kstep(two, s, 0);
          kstep(two, s + 1, 1);
          kstep(two, s + 2, 2);
          kstep(two, s + 3, 3);
        }
      } else {
        for (int s = 0; s < nk; s += 4) {
          kstep(two, s, 0);
          kstep(two, s + 1, 1);
          kstep(two, s + 2, 2);
          kstep(two, s + 3, 3);
        }
      }
    };
    if (nt == 2) kloop(std::integral_constant<int, 2>{});
    else kloop(std::integral_constant<int, 1>{});  // (a third, MFMA-free variant for nt == 0 spills)
    cur = nxt;
    unit_src(j + 2, nxt);
    sp.mark(9);

    // ---- 2. epilogue: q -> registers, k / v -> LDS images -----------------------------------------
    // acc[tt][4p + r][jj] = feature 64h + 16 fq + 4 r + jj of group p (q, k, v) for token 16 tile + fr
    h8 qh[TPW][2], ql[TPW][2];
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt) {
      const int row = 16 * (2 * wr + tt) + fr;  // token / key row of the images
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        float x[16];
        const float4* bl = reinterpret_cast<const float4*>(bias_l + p * C + 64 * h + 16 * fq);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float4 b4 = bl[r];
          const float bb[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
          for (int jj = 0; jj < 4; ++jj)
            x[4 * r + jj] = fmaf(alpha_s, (float)acc[tt][4 * p + r][jj], bb[jj]);
        }
        h8 hi0, lo0, hi1, lo1;
        float xa0[8], xa1[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) { xa0[e] = x[e]; xa1[e] = x[8 + e]; }
        split8(xa0, hi0, lo0);
        split8(xa1, hi1, lo1);
        if (p == 0) {
          qh[tt][0] = hi0; ql[tt][0] = lo0; qh[tt][1] = hi1; ql[tt][1] = lo1;
        } else if (tv[tt]) {
          if (p == 1) {
            *reinterpret_cast<h8*>(kv + koff(row, 2 * fq)) = hi0;
            *reinterpret_cast<h8*>(kv + koff(row, 2 * fq + 1)) = hi1;
            *reinterpret_cast<h8*>(kv + IMGF + koff(row, 2 * fq)) = lo0;
            *reinterpret_cast<h8*>(kv + IMGF + koff(row, 2 * fq + 1)) = lo1;
          } else {
            *reinterpret_cast<h8*>(kv + 2 * IMGF + v32off(row, 32 * fq)) = hi0;
            *reinterpret_cast<h8*>(kv + 2 * IMGF + v32off(row, 32 * fq + 16)) = hi1;
            *reinterpret_cast<h8*>(kv + 3 * IMGF + v32off(row, 32 * fq)) = lo0;
            *reinterpret_cast<h8*>(kv + 3 * IMGF + v32off(row, 32 * fq + 16)) = lo1;
          }
        }
      }
    }
    // K / V images complete: LDS writes retired + barrier, without the vmcnt(0) of __syncthreads (the next
    // unit's DMA pieces and activation loads stay in flight under the attention)
    __builtin_amdgcn_s_waitcnt(0xC07F);
    asm volatile("s_barrier" ::: "memory");
    sp.mark(9);

    // ---- 3. attention over the resident K / V ------------------------------------------------------
    // q as the 32-query tile's B operands: lane group G (tile G & 1, dims 32 (G >> 1) .. + 31) takes the
    // 16 dims it lacks from group G ^ 1 (permlane16 swap: even groups trade their tile-1 words, odd groups
    // their tile-0 words); q32h[c] = dims 32 h + 8 c .. + 7
    h8 q32h[4], q32l[4];
    {
      auto xch = [&](const h8& t0, const h8& t1, h8& first, h8& second) __attribute__((always_inline)) {
        const u4 x = __builtin_bit_cast(u4, t0), y = __builtin_bit_cast(u4, t1);
        u4 f, g;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const auto w = __builtin_amdgcn_permlane16_swap(x[d], y[d], false, false);
          f[d] = w[0];
          g[d] = w[1];
        }
        first = __builtin_bit_cast(h8, f);
        second = __builtin_bit_cast(h8, g);
      };
      xch(qh[0][0], qh[1][0], q32h[0], q32h[2]);
      xch(qh[0][1], qh[1][1], q32h[1], q32h[3]);
      xch(ql[0][0], ql[1][0], q32l[0], q32l[2]);
      xch(ql[0][1], ql[1][1], q32l[1], q32l[3]);
    }
    float m = -INFINITY, l = 0.f;  // running max (log2 units; an integer once set), sum
    f16x o[2] = {};
    const int nkb = (N + KB - 1) / KB;
    const int nfull = N / KB;  // full key blocks, then the last (masked when N % 32 != 0)
    // software-pipelined: block kb + 1's scores are issued before block kb's softmax, so the matrix core
    // runs them while this wave's softmax issues
    // With 7 key blocks (N 193 .. 224: ViT @ 224, N = 197) the block loop is straight-line code and every
    // LDS offset an immediate; otherwise two blocks per iteration with ping-pong score registers (no copy of
    // the loop-carried scores).
    if (nt > 0) {
      auto last = [&](int kb, const f16x& sc) __attribute__((always_inline)) {
        if (nfull < nkb) softmax_pv32<true, IMGF>(kv + kb * KB * 128, sc, m, l, o, voffs, kb * KB, N, sl2);
        else softmax_pv32<false, IMGF>(kv + kb * KB * 128, sc, m, l, o, voffs, kb * KB, N, sl2);
      };
      f16x sa = scores32<IMGF>(kv, q32h, q32l, koffs);
      if (nkb == 7) {
#pragma unroll
        for (int kb = 0; kb < 6; ++kb) {
          const f16x sb = scores32<IMGF>(kv + (kb + 1) * KB * 128, q32h, q32l, koffs);
          softmax_pv32<false, IMGF>(kv + kb * KB * 128, sa, m, l, o, voffs, kb * KB, N, sl2);
          sa = sb;
        }
        last(6, sa);
      } else {
        int kb = 0;
        for (; kb + 2 < nkb; kb += 2) {
          const f16x sb = scores32<IMGF>(kv + (kb + 1) * KB * 128, q32h, q32l, koffs);
          softmax_pv32<false, IMGF>(kv + kb * KB * 128, sa, m, l, o, voffs, kb * KB, N, sl2);
          sa = scores32<IMGF>(kv + (kb + 2) * KB * 128, q32h, q32l, koffs);
          softmax_pv32<false, IMGF>(kv + (kb + 1) * KB * 128, sb, m, l, o, voffs, (kb + 1) * KB, N, sl2);
        }
        if (kb + 1 < nkb) {
          const f16x sb = scores32<IMGF>(kv + (kb + 1) * KB * 128, q32h, q32l, koffs);
          softmax_pv32<false, IMGF>(kv + kb * KB * 128, sa, m, l, o, voffs, kb * KB, N, sl2);
          last(kb + 1, sb);
        } else {
          last(kb, sa);
        }
      }
    }
    sp.mark(0);
    attend_store32<OUT>(tv, l, o, wr, N, b, h, in_scale, out, ldo, qp, tb, st16);
    sp.mark(4);
  }
  sp.flush();
}

// ======================================================================================================
// Role-alternating form for 13 token tiles (N = 193 .. 208: every ViT @ 224 with 16-pixel patches, N = 197).
// The two halves of the workgroup (waves 0-3 and 4-7: one wave of each on every SIMD) take turns. In step t
// half P = t & 1 projects token tiles 0 .. 11 of unit t while half Q attends unit t - 1 from the resident K / V
// images and projects unit t's last token tile (12) on the side; so every SIMD pairs a projection wave with an
// attention wave, and the matrix pipe runs one wave's MFMAs while the other issues softmax, unpack and epilogue
// VALU. After one barrier (unit t - 1's K / V images are no longer read) both halves write unit t's K / V images
// (P tiles 0 .. 11, Q tile 12, whose q goes to a small staging image) and Q finishes tile 12 of unit t - 1; after
// the second barrier the halves swap roles: P attends unit t with its own tiles' q still in registers.
// No barrier inside either phase: every wave streams its own weight fragments and activation rows from the
// L1 / L2 straight into registers (a head's 6 KiB weight k-step is read by the CU's four projection waves; the
// L1 serves the repeats), so the k-loop needs no LDS ring and no shared hand-off.
// Per wave gw = 0..3 of a half: projection of token tiles 3 gw .. 3 gw + 2 (36 MFMAs per k-step), or attention of
// query tiles 3 gw .. 3 gw + 2 over the 7 key blocks, tile 12 over key blocks kb = gw (mod 4) (the four partial
// (o, max, sum) sets are combined after the barrier) and fragments 3 gw .. 3 gw + 2 of tile 12's projection of
// the next unit: both roles carry about the same matrix work per SIMD (6.9 k / 9.0-9.4 k MFMA cycles per unit).
// Attention body: attn_common.h attend() (16x16x32 fp16, 3 passes); the K image's 16-B chunk 2 g + c holds dims
// 16 g + 8 c .. + 7, which is where a projection lane (token fr, lane group g) already has its q, so q needs no
// lane movement; rows are XOR-swizzled (kswz) so the ds_read_b128 of every lane group is conflict-free.
namespace rr {
constexpr int W = 8;                       // waves (2 halves of 4)
constexpr int NT = W * 64;
constexpr int NTILE = 13;                  // token tiles
constexpr int NKB = 7;                     // key blocks of 32 (208 / 32, rounded up)
constexpr int ROWS = 208;                  // rows of each K / V image
constexpr int IMGB = ROWS * 128;           // one fp16 image: 26 KiB
constexpr int KV = 4 * IMGB + 2048;        // K hi, K lo, V hi, V lo + zero rows past V lo
constexpr int Q12 = 2 * 16 * 128;          // tile 12's q, hi and lo images [16 rows][64 dims]
constexpr int CMBF = 18;                   // per lane of a tile-12 partial: o (16 floats), m, l
constexpr int CMB = 4 * CMBF * 64 * 4;
constexpr int TBLB = 8192;                 // code table (<= 1022 buckets)
constexpr int BIASB = 9216;                // fp32 bias of the qkv layer (<= 2304 features)
constexpr int LDS = KV + Q12 + CMB + TBLB + BIASB;
static_assert(LDS <= 163840, "LDS budget");
// (IMG4_STEP: bytes of one (256-row tile, k-step) of the int4 weight image, as above)

// K image: row r, 16-B chunk ch at chunk ch ^ kswz(r). With chunk 2 g + c the ds_read_b128 lane groups
// ({0-3, 12-15, 20-27}, ...) each cover 16 distinct 16-B bank slots (exhaustive check)
QVIT_DEV int kswz(int r) { return (r & 6) | ((r >> 3) & 1); }
QVIT_DEV int krow(int r, int ch) { return r * 128 + 16 * (ch ^ kswz(r)); }

typedef _Float16 h4 __attribute__((ext_vector_type(4)));
// fp16 hi / lo of 4 values (the same arithmetic as attn_common.h split8)
QVIT_DEV void split4(const float (&x)[4], uint2& hi, uint2& lo) {
  h4 h, l;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    h[i] = (_Float16)x[i];
    l[i] = (_Float16)(x[i] - (float)h[i]);
  }
  hi = __builtin_bit_cast(uint2, h);
  lo = __builtin_bit_cast(uint2, l);
}

// LDS writes of this wave retired, then the workgroup barrier (global stores and loads stay in flight)
QVIT_DEV void lds_barrier() {
  __builtin_amdgcn_s_waitcnt(0xC07F);
  asm volatile("s_barrier" ::: "memory");
}

// Operand stream of a wave's projection share of one unit: this lane's 8-B fragment of weight rows (group p,
// 16-row tile r) of the head at k-step s of the pre-tiled int4 image (uniform group base + lane offset), and its
// 16-B activation fragment of a token tile's row (uniform tile base + lane offset).
struct ProjSrc {
  const int8_t* wb[3];   // group p's 64-row block of the head at k-step 0
  uint32_t wlane;        // row pr, 16-k chunk pq, the image's chunk swizzle
  uint32_t alane;        // row pr, 16-k chunk pq of a token tile
  QVIT_DEV uint2 w(int p, int r, int s) const {
    return *reinterpret_cast<const uint2*>(wb[p] + (size_t)s * IMG4_STEP + r * 512 + wlane);
  }
  QVIT_DEV v4i a(const int8_t* tile_base, int s) const {
    return *reinterpret_cast<const v4i*>(tile_base + 64 * s + alane);
  }
};
QVIT_DEV ProjSrc proj_src(const int8_t* Wp, int C, int h, int nk, int pr, int pq, int64_t lda) {
  ProjSrc ps;
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    const int feat = p * C + 64 * h;
    ps.wb[p] = Wp + ((int64_t)((feat >> 8) * nk) * IMG4_STEP + (feat & 255) * 32);
  }
  ps.wlane = (uint32_t)(pr * 32 + ((pq ^ (((pr >> 3) & 1) << 1)) << 3));
  ps.alane = (uint32_t)(pr * lda + 16 * pq);
  return ps;
}

// x = (d_a d_w acc + bias) * in_scale for 4 features (16x-scaled int4 accumulators: alpha_s carries the 1/16),
// as fp16 hi / lo
QVIT_DEV void qkv_value4(const v4i& acc, const float* bias4, float alpha_s, uint2& hi, uint2& lo) {
  const float4 b4 = *reinterpret_cast<const float4*>(bias4);
  const float x[4] = {fmaf(alpha_s, (float)acc[0], b4.x), fmaf(alpha_s, (float)acc[1], b4.y),
                      fmaf(alpha_s, (float)acc[2], b4.z), fmaf(alpha_s, (float)acc[3], b4.w)};
  split4(x, hi, lo);
}
}  // namespace rr

template <int OUT, int NKC>
__global__ __launch_bounds__(rr::NT, 1) void qkv_attn_rr_kernel(
    const int8_t* __restrict__ A, int K, int64_t lda, const int8_t* __restrict__ Wp, int npad,
    const float* __restrict__ d_act, const float* __restrict__ d_wt, const float* __restrict__ bias, int B, int N,
    int H, float scale, float in_scale, void* __restrict__ out, int64_t ldo, int out_qtype, const float* out_d,
    const float* out_qm, const float* out_t, int out_levels, const int8_t* __restrict__ epi_table) {
  using namespace rr;
  __shared__ __attribute__((aligned(16))) int8_t smem[LDS];
  int8_t* kv = smem;
  int8_t* q12 = smem + KV;
  float* cmb = reinterpret_cast<float*>(q12 + Q12);
  int8_t* tbl = reinterpret_cast<int8_t*>(cmb) + CMB;
  float* bias_l = reinterpret_cast<float*>(tbl + TBLB);
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int half = wave >> 2, gw = wave & 3;
  const int C = H * 64;
  const int nk = NKC > 0 ? NKC : K / 64;

  // ---- per-workgroup setup (as qkv_attn_kernel) -----------------------------------------------------------
  const float alpha = (*d_act) * (*d_wt);
  // the output quantizer's code table -> LDS (header included; valid = 0 there when there is none): the
  // attention branch re-reads its geometry and the quantizer scalars where it stores, so none of them stays
  // live through the projection
  if (OUT == 1) {
    bool have = false;
    if (epi_table != nullptr) {
      const EpiTableHdr hd = *reinterpret_cast<const EpiTableHdr*>(epi_table);
      if (hd.valid != 0 && hd.nb >= 1 && 16 + 8 * hd.nb <= TBLB) {
        for (int k = tid; k < (16 + 8 * hd.nb + 15) / 16; k += NT)
          reinterpret_cast<uint4*>(tbl)[k] = reinterpret_cast<const uint4*>(epi_table)[k];
        have = true;
      }
    }
    if (!have && tid == 0) reinterpret_cast<EpiTableHdr*>(tbl)->valid = 0;
  }
  for (int k = tid; k < 3 * C; k += NT) bias_l[k] = bias ? bias[k] * in_scale : 0.f;
  const float alpha_s = alpha * in_scale * 0.0625f;   // 16x-scaled int4 operands (qkv_attn_kernel)
  for (int k = tid; k < KV / 16; k += NT) reinterpret_cast<uint4*>(kv)[k] = make_uint4(0, 0, 0, 0);

  const int nunits = B * H;
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, team = gridDim.x >> 3;
  const int per = nunits >> 3, rem = nunits & 7;
  const int ulo = xcd * per + (xcd < rem ? xcd : rem);
  const int uhi = ulo + per + (xcd < rem ? 1 : 0);
  const int my_units = (uhi - ulo - slot + team - 1) / team;  // unit j: ulo + slot + j * team
  const int64_t M = (int64_t)B * N;
  const float sl2 = scale * LOG2E / (in_scale * in_scale);
  const bool st16 = ((ldo & 15) == 0) && ((((uintptr_t)out) & 15) == 0);
  Stamps sp;

  if (my_units <= 0) return;  // uniform per workgroup; no barrier reached yet
  __syncthreads();            // setup visible

  // Steps 0 .. my_units, two barriers each. Half h projects unit t in the steps t = h (mod 2) and attends it in
  // step t + 1, so one loop iteration of a half covers the projection of a unit and its attention (q stays in
  // registers within the iteration). Half 1 enters at t = -1: its step 0 only projects unit 0's tile 12.
  for (int t = half ? -1 : 0; t <= my_units; t += 2) {
    h8 qh[3][2], ql[3][2];   // q of the wave's three query tiles of unit t
    // ==================== step t: projection of unit t, token tiles 3 gw .. 3 gw + 2 ===========================
    if (t == my_units) {
      lds_barrier();
      lds_barrier();
      break;                  // (step t + 1 does not exist)
    }
    if (t >= 0) {
      const int unit = ulo + slot + t * team;
      const int b = unit / H, h = unit - b * H;
      // per-lane values from an opaque lane id: recomputed here, not hoisted out of the unit loop (the
      // projection holds 144 accumulators and its operand stream; nothing else may stay live through it)
      const int ln = lane_opaque();
      const int pr = ln & 15, pq = ln >> 4;
      const ProjSrc ps = proj_src(Wp, C, h, nk, pr, pq, lda);
      const int8_t* ab = A + (int64_t)(b * N + 48 * gw) * lda;   // rows of tiles 3 gw .. 3 gw + 2 (inside image b)
      v4i acc[3][12];
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int f = 0; f < 12; ++f) acc[i][f] = v4i{0, 0, 0, 0};
      // k-step s: its activation rows and weight fragments are in registers; k-step s + 1's activations are
      // loaded at its top, and each weight fragment of k-step s + 1 right after the MFMAs that consume the same
      // fragment of k-step s (into the same registers: one k-step of latency cover for every load)
      uint2 wf[12];
      v4i xa[3];
#pragma unroll
      for (int f = 0; f < 12; ++f) wf[f] = ps.w(f >> 2, f & 3, 0);
#pragma unroll
      for (int i = 0; i < 3; ++i) xa[i] = ps.a(ab + (int64_t)(16 * i) * lda, 0);
      auto kstep = [&](int s, bool more) __attribute__((always_inline)) {
        v4i xn[3];
        if (more) {
#pragma unroll
          for (int i = 0; i < 3; ++i) xn[i] = ps.a(ab + (int64_t)(16 * i) * lda, s + 1);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int f = 0; f < 12; ++f) {
          const v4i wc = unpack16(wf[f]);
#pragma unroll
          for (int i = 0; i < 3; ++i) acc[i][f] = __builtin_amdgcn_mfma_i32_16x16x64_i8(wc, xa[i], acc[i][f], 0, 0, 0);
          if (more) wf[f] = ps.w(f >> 2, f & 3, s + 1);
          __builtin_amdgcn_sched_barrier(0);
        }
        if (more) {
#pragma unroll
          for (int i = 0; i < 3; ++i) xa[i] = xn[i];
        }
      };
      if constexpr (NKC > 0) {
#pragma unroll
        for (int s = 0; s < NKC; ++s) kstep(s, s + 1 < NKC);
      } else {
        for (int s = 0; s < nk - 1; ++s) kstep(s, true);
        kstep(nk - 1, false);
      }
      sp.mark(8);
      lds_barrier();  // the attending half is done with unit t - 1's K / V images
      sp.mark(7);
      // ---- epilogue: K / V images, the wave's own q -> registers (kept into its attention step) -------------
      // acc[i][4 p + r][jj] = feature 64 h + 16 pq + 4 r + jj of group p for token 16 tile + pr
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int row = 16 * (3 * gw + i) + pr;
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          uint2 hi[4], lo[4];
#pragma unroll
          for (int r = 0; r < 4; ++r)
            qkv_value4(acc[i][4 * p + r], bias_l + p * C + 64 * h + 16 * pq + 4 * r, alpha_s, hi[r], lo[r]);
          const h8 hi0 = __builtin_bit_cast(h8, make_uint4(hi[0].x, hi[0].y, hi[1].x, hi[1].y));
          const h8 hi1 = __builtin_bit_cast(h8, make_uint4(hi[2].x, hi[2].y, hi[3].x, hi[3].y));
          const h8 lo0 = __builtin_bit_cast(h8, make_uint4(lo[0].x, lo[0].y, lo[1].x, lo[1].y));
          const h8 lo1 = __builtin_bit_cast(h8, make_uint4(lo[2].x, lo[2].y, lo[3].x, lo[3].y));
          if (p == 0) {
            qh[i][0] = hi0; ql[i][0] = lo0; qh[i][1] = hi1; ql[i][1] = lo1;
          } else if (p == 1) {
            *reinterpret_cast<h8*>(kv + krow(row, 2 * pq)) = hi0;
            *reinterpret_cast<h8*>(kv + krow(row, 2 * pq + 1)) = hi1;
            *reinterpret_cast<h8*>(kv + IMGB + krow(row, 2 * pq)) = lo0;
            *reinterpret_cast<h8*>(kv + IMGB + krow(row, 2 * pq + 1)) = lo1;
          } else {
            *reinterpret_cast<h8*>(kv + 2 * IMGB + voff(row, 32 * pq)) = hi0;
            *reinterpret_cast<h8*>(kv + 2 * IMGB + voff(row, 32 * pq + 16)) = hi1;
            *reinterpret_cast<h8*>(kv + 3 * IMGB + voff(row, 32 * pq)) = lo0;
            *reinterpret_cast<h8*>(kv + 3 * IMGB + voff(row, 32 * pq + 16)) = lo1;
          }
        }
      }
      lds_barrier();  // unit t's K / V images and tile-12 q complete
      sp.mark(9);
    }
    {
      // ============ step t + 1: attention of unit t (+ tile 12's projection fragments 3 gw .. + 2 of unit t + 1) ===
      const bool att = t >= 0;               // (half 1's first step: tile 12 of unit 0 only)
      const bool pnext = t + 1 < my_units;   // unit t + 1 exists: project its tile-12 share on the side
      const int unit = ulo + slot + (att ? t : 0) * team;
      const int b = unit / H, h = unit - b * H;
      const int unit_n = ulo + slot + (pnext ? t + 1 : t) * team;
      const int bn = unit_n / H, hn = unit_n - bn * H;
      const int ln = lane_opaque();
      const int fr = ln & 15, fq = ln >> 4;
      int koffs[2][2], voffs[4];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int c = 0; c < 2; ++c) koffs[kt][c] = krow(16 * kt + fr, 2 * fq + c);
      // the V image and its transposed reads are attend()'s (attn_common.h fragment_offsets, voff)
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) voffs[dt] = voff(4 * fq + (fr >> 2), 2 * (16 * dt + 4 * (fr & 3)));
      // tile 12 of unit t: fragments f = 3 gw + i (group f >> 2, 16-row tile f & 3), token rows 192 + fr (rows past
      // the image are the next one's, finite and masked; clamped at the end of the batch)
      const ProjSrc ps = proj_src(Wp, C, hn, nk, fr, fq, lda);
      int64_t m12 = (int64_t)bn * N + 192 + fr;
      m12 = m12 < M ? m12 : M - 1;
      const int8_t* a12 = A + m12 * lda + 16 * fq;
      v4i acc12[3] = {v4i{0, 0, 0, 0}, v4i{0, 0, 0, 0}, v4i{0, 0, 0, 0}};
      uint2 w3[3];
      v4i x12;
      if (pnext) {
#pragma unroll
        for (int i = 0; i < 3; ++i) w3[i] = ps.w((3 * gw + i) >> 2, (3 * gw + i) & 3, 0);
        x12 = *reinterpret_cast<const v4i*>(a12);
      }
      auto kstep12 = [&](int s) __attribute__((always_inline)) {
        if (!pnext || s >= nk) return;
        const bool more = s + 1 < nk;
        v4i xn = x12;
        if (more) xn = *reinterpret_cast<const v4i*>(a12 + 64 * (s + 1));
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          acc12[i] = __builtin_amdgcn_mfma_i32_16x16x64_i8(unpack16(w3[i]), x12, acc12[i], 0, 0, 0);
          if (more) w3[i] = ps.w((3 * gw + i) >> 2, (3 * gw + i) & 3, s + 1);
        }
        x12 = xn;
      };

      sp.mark(5);
      if (!att) {  // (pnext holds: my_units >= 1)
        for (int s = 0; s < nk; ++s) kstep12(s);
      } else {
      // one query tile at a time over the 7 key blocks (only one tile's o, max and sum live: the K / V fragments
      // are re-read from LDS per tile), then tile 12 over this wave's key blocks; the tile-12 k-steps of the next
      // unit ride between the blocks: k-step n after main block n (n < 21), any further ones after the loop
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        float m[1] = {-INFINITY}, l[1] = {0.f};
        f4 o[1][4] = {{f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}}};
        const h8 qa[1][2] = {{qh[i][0], qh[i][1]}}, qb[1][2] = {{ql[i][0], ql[i][1]}};
#pragma unroll 1
        for (int kb = 0; kb < NKB - 1; ++kb) {
          attend<1, IMGB, false>(1, false, kv + kb * KB * 128, qa, qb, m, l, o, koffs, voffs, kb * KB + 4 * fq, N, sl2,
                                 sp);
          kstep12(i * NKB + kb);
        }
        attend<1, IMGB, false>(1, true, kv + (NKB - 1) * KB * 128, qa, qb, m, l, o, koffs, voffs,
                               (NKB - 1) * KB + 4 * fq, N, sl2, sp);
        kstep12(i * NKB + NKB - 1);
        QParams qp{};
        EpiLds tb{nullptr, 0.f, 0.f, 0.f};
        if (OUT == 1) {  // (re-read per tile: nothing of the quantizer stays live through the key blocks)
          const EpiTableHdr hd = *reinterpret_cast<const EpiTableHdr*>(tbl);
          if (hd.valid != 0) tb = EpiLds{tbl + sizeof(EpiTableHdr), hd.c0, hd.inv_w, epi_top(hd.nb)};
          else qp = load_qparams(out_qtype, out_d, out_qm, out_t, out_levels);
        }
        const bool tv[1] = {true};
        attend_store<OUT, 1>(tv, l, o, 3 * gw + i, 1, 0, N, b, h, in_scale, out, ldo, qp, tb, st16);
      }
      for (int s = 3 * NKB; s < nk; ++s) kstep12(s);
      // tile 12 over key blocks kb = gw (mod 4): q from the staging images; this wave's partial (o, max, sum)
      {
        h8 qa[1][2], qb[1][2];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          qa[0][c] = lds_h8(q12, fr * 128 + 32 * fq + 16 * c);
          qb[0][c] = lds_h8(q12 + 2048, fr * 128 + 32 * fq + 16 * c);
        }
        float m[1] = {-INFINITY}, l[1] = {0.f};
        f4 o[1][4] = {{f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}}};
        for (int kb = gw; kb < NKB; kb += 4)
          attend<1, IMGB, false>(1, kb == NKB - 1, kv + kb * KB * 128, qa, qb, m, l, o, koffs, voffs, kb * KB + 4 * fq, N,
                                 sl2, sp);
        float* cw = cmb + gw * CMBF * 64 + ln;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) cw[(4 * dt + jj) * 64] = o[0][dt][jj];
        cw[16 * 64] = m[0];
        cw[17 * 64] = l[0];
      }
      }
      sp.mark(0);
      lds_barrier();
      sp.mark(4);
      // ---- tile 12 of unit t: combine the four partials; wave gw finishes dims 16 gw .. 16 gw + 15 -----------
      if (att) {
        float mw[4], M2 = -INFINITY;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          mw[w] = cmb[(w * CMBF + 16) * 64 + ln];
          M2 = fmax_nn(M2, mw[w]);
        }
        f4 oc = f4{0.f, 0.f, 0.f, 0.f};
        float lc = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const float sc = __builtin_amdgcn_exp2f(mw[w] - M2);
          const float* cw = cmb + w * CMBF * 64 + ln;
          const f4 ow = f4{cw[(4 * gw) * 64], cw[(4 * gw + 1) * 64], cw[(4 * gw + 2) * 64], cw[(4 * gw + 3) * 64]};
          oc += ow * sc;
          lc += cw[17 * 64] * sc;
        }
        const float inv = 1.f / (xsum(lc) * in_scale);
        const int q = 192 + fr;
        const int64_t row = (int64_t)b * N + q;
        if (OUT == 0) {
          if (q < N)
            *reinterpret_cast<f4*>(reinterpret_cast<float*>(out) + row * ldo + h * HD + 16 * gw + 4 * fq) = oc * inv;
        } else {
          uint32_t word = 0;
          const EpiTableHdr hd = *reinterpret_cast<const EpiTableHdr*>(tbl);
          if (hd.valid != 0) {
            const int8_t* ent = tbl + sizeof(EpiTableHdr);
            const float top = epi_top(hd.nb);
            float v[4];
            uint2 e[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              v[j] = oc[j] * inv;
              e[j] = *epi_entry(ent, v[j], hd.c0, hd.inv_w, top);
            }
            epi_select_byte<0>(word, v[0], __uint_as_float(e[0].x), e[0].y);
            epi_select_byte<1>(word, v[1], __uint_as_float(e[1].x), e[1].y);
            epi_select_byte<2>(word, v[2], __uint_as_float(e[2].x), e[2].y);
            epi_select_byte<3>(word, v[3], __uint_as_float(e[3].x), e[3].y);
          } else {
            const QParams qp = load_qparams(out_qtype, out_d, out_qm, out_t, out_levels);
            word = quant_word_ool(oc[0] * inv, oc[1] * inv, oc[2] * inv, oc[3] * inv, qp);
          }
          if (q < N)
            *reinterpret_cast<uint32_t*>(reinterpret_cast<int8_t*>(out) + row * ldo + h * HD + 16 * gw + 4 * fq) = word;
        }
      }
      // ---- tile 12 of unit t: this wave's fragments -> K / V images and the q staging image ------------------
      if (pnext) {
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const int f = 3 * gw + i, p = f >> 2, r = f & 3;
          uint2 hi, lo;
          qkv_value4(acc12[i], bias_l + p * C + 64 * hn + 16 * fq + 4 * r, alpha_s, hi, lo);
          const int row = 192 + fr;
          int8_t* dh;
          int imgs;
          if (p == 0) {
            dh = q12 + fr * 128 + 32 * fq + 8 * r;
            imgs = 2048;
          } else if (p == 1) {
            dh = kv + krow(row, 2 * fq + (r >> 1)) + 8 * (r & 1);
            imgs = IMGB;
          } else {
            dh = kv + 2 * IMGB + voff(row, 32 * fq + 8 * r);
            imgs = IMGB;
          }
          *reinterpret_cast<uint2*>(dh) = hi;
          *reinterpret_cast<uint2*>(dh + imgs) = lo;
        }
      }
      lds_barrier();
      sp.mark(6);
    }
  }
  sp.flush();
}

}  // namespace

extern "C" int qvit_qkv_attention(const int8_t* A, int64_t B, int64_t N, int64_t K, int64_t lda, const void* Wp,
                                  int wfmt, int64_t npad, const float* d_act, const float* d_wt, const float* bias,
                                  int64_t H, int64_t head_dim, float scale, float in_scale, int out_mode, void* out,
                                  int64_t ldo, int out_qtype, const float* out_d, const float* out_qm,
                                  const float* out_t, int out_levels, const void* epi_table, hipStream_t stream) {
  if (!A || !Wp || !out || !d_act || !d_wt) return QVIT_ENULL;
  if (wfmt != QVIT_W4 || head_dim != 64) return QVIT_EINVAL;
  if (B < 0 || N <= 0 || N > MAXN || H <= 0 || K <= 0 || K % 256 || K > 65536 || lda < K) return QVIT_EINVAL;
  if (npad < 3 * H * 64 || npad % 256 || 3 * H * 64 * 4 > BIAS_MAX || ldo < H * 64) return QVIT_EINVAL;
  if (B * N > INT32_MAX / 2 || !(in_scale > 0.f)) return QVIT_EINVAL;
  // the kernel addresses A and Wp with 32-bit byte offsets from the base pointers
  if (B * N * lda > (int64_t)0xFFFFFFFF - 64 || npad * K / 2 > (int64_t)0xFFFFFFFF) return QVIT_EINVAL;
  if ((lda % 16) || (((uintptr_t)A) & 15) || (((uintptr_t)Wp) & 15)) return QVIT_EALIGN;
  if (epi_table && (((uintptr_t)epi_table) & 15)) return QVIT_EALIGN;
  if (out_mode == QVIT_ATT_F32) {
    if ((ldo % 4) || (((uintptr_t)out) & 15)) return QVIT_EALIGN;
  } else if (out_mode == QVIT_ATT_I8) {
    if ((ldo % 4) || (((uintptr_t)out) & 3)) return QVIT_EALIGN;
    const int q = out_qtype & 0xff;
    if (q != QVIT_QT_LINEAR && q != QVIT_QT_NONLINEAR && q != QVIT_QT_ULTRA_ACT) return QVIT_EINVAL;
    if (q == QVIT_QT_ULTRA_ACT ? (out_levels < 1 || out_levels > 127) : (!out_d || !out_qm)) return QVIT_EINVAL;
  } else {
    return QVIT_EINVAL;
  }
  if (B == 0) return QVIT_OK;
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                hipSuccess || n <= 0)
      n = 256;
    return n;
  }();
  const int64_t grid = std::max<int64_t>(8, (int64_t)cus / 8 * 8);  // one workgroup per CU, a multiple of 8
  const int8_t* w = reinterpret_cast<const int8_t*>(Wp);
  const int8_t* tab = reinterpret_cast<const int8_t*>(epi_table);
#define QVIT_QA_LAUNCH_K(KERN, OUTV, NKV, TAB)                                                                  \
  hipLaunchKernelGGL((KERN<OUTV, NKV>), dim3((unsigned)grid), dim3(FT), 0, stream, A, (int)K, lda, w, (int)npad,   \
                     d_act, d_wt, bias, (int)B, (int)N, (int)H, scale, in_scale, out, ldo, out_qtype, out_d, out_qm, \
                     out_t, out_levels, TAB)
  if ((N + 15) / 16 == rr::NTILE) {  // 13 token tiles (ViT @ 224): the role-alternating kernel
    if (out_mode == QVIT_ATT_F32) {
      if (K == 768) QVIT_QA_LAUNCH_K(qkv_attn_rr_kernel, 0, 12, nullptr);
      else QVIT_QA_LAUNCH_K(qkv_attn_rr_kernel, 0, 0, nullptr);
    } else {
      if (K == 768) QVIT_QA_LAUNCH_K(qkv_attn_rr_kernel, 1, 12, tab);
      else QVIT_QA_LAUNCH_K(qkv_attn_rr_kernel, 1, 0, tab);
    }
    return qvit_hip_status(hipGetLastError());
  }
#undef QVIT_QA_LAUNCH_K
#define QVIT_QA_LAUNCH(OUTV, NKV, TAB)                                                                          \
  hipLaunchKernelGGL((qkv_attn_kernel<OUTV, NKV>), dim3((unsigned)grid), dim3(FT), 0, stream, A, (int)K, lda, w,    \
                     (int)npad, d_act, d_wt, bias, (int)B, (int)N, (int)H, scale, in_scale, out, ldo, out_qtype,   \
                     out_d, out_qm, out_t, out_levels, TAB)
  if (out_mode == QVIT_ATT_F32) {
    if (K == 768) QVIT_QA_LAUNCH(0, 12, nullptr);
    else QVIT_QA_LAUNCH(0, 0, nullptr);
  } else {
    if (K == 768) QVIT_QA_LAUNCH(1, 12, tab);
    else QVIT_QA_LAUNCH(1, 0, tab);
  }
#undef QVIT_QA_LAUNCH
  return qvit_hip_status(hipGetLastError());
}

QVIT_ATT_STAMP_READER(qvit_qkv_att_stamps)  // diag_stamps.h: -DQVIT_ATT_STAMPS builds only
