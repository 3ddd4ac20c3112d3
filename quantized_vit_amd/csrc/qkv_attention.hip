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
constexpr int XRING = 4;                  // activation register ring (k-steps s .. s + 3)
// vmem ops a wave issues after its DMA piece of k-step s + 2 (s odd): the activation loads of k-steps s + 1, s + 2
constexpr int TOPCNT = 2 * 2;
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
  // projection plan. Wave wr (the wave index rotated by unit) owns the token tiles {2 wr, 2 wr + 1}: their q go to
  // its registers (the 32-query tile it attends), their k, v to the LDS images. Waves wr, wr + 4 share a SIMD, so
  // with 13 token tiles (N = 193 .. 208, ViT @224) the SIMDs carry 4, 4, 3 and 2 (+ an idle wave's pass) tiles and
  // the two busiest set the pace. Balanced plan: the second tile of wr = 4 and wr = 5 (tiles 9, 11) is split by
  // features at the 8-feature chunk boundary of k: the owner computes fragments 0 .. 5 (q and the first half of
  // k), the otherwise idle wave wr = 7 computes fragments 6 .. 11 (the rest of k and v) of both tiles and writes
  // them to the images itself. MFMAs per k-step on the busiest SIMD: 48 -> 42.
  const bool bal = ntile == 13;
  auto ptile = [&](int wr_, int tt) -> int { return (bal && wr_ == 7) ? (tt ? 11 : 9) : 2 * wr_ + tt; };

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
      int64_t m = (int64_t)b * N + 16 * ptile(wr, tt) + fr;
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
  // prologue: weight k-steps 0 .. 3 of the first unit, activation k-steps 0, 1, 2
#pragma unroll
  for (int t = 0; t < WRING; ++t) dma_piece(cur, t, t);
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
    // projection ranges of the wave's two tiles: 1 all fragments, 2 fragments 0 .. 5, 3 fragments 6 .. 11, 0 none
    const int pmode = (bal && wr == 7) ? 3 : (bal && (wr == 4 || wr == 5)) ? 2 : (nt == 2) ? 0 : 1;
    const int prange[TPW] = {pmode == 3 ? 3 : 1, pmode == 0 ? 1 : pmode == 2 ? 2 : pmode == 3 ? 3 : 0};

    // ---- 1. projection ---------------------------------------------------------------------------
    // unit head: everything issued before (the previous unit's output stores included) has landed, the
    // ring slots of k-steps 0 .. 3 are complete for every wave; read k-step 0's weight fragments
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
    //   top (s odd; one barrier per two k-steps): this wave's DMA pieces of k-steps s + 1 and s + 2 landed
    //   (TOPCNT = the activation loads issued after them may be in flight, which also covers the activations
    //   of k-step s), then the barrier: the slots of k-steps s + 1 (read during k-step s) and s + 2 (read
    //   during k-step s + 1, before the next barrier) are complete for everyone, and every wave is past
    //   k-step s - 1, the last reader of slots (s + 3) % 4 (k-step s - 1's) and (s + 4) % 4 (k-step s's);
    //   issue (s odd): weight k-steps s + 3, s + 4 -> their slots; every k-step: activation k-step s + 3 ->
    //   register slot (s + 3) % 4 (past the unit's end: the next unit's k-steps; at k-step 0 the unit head's
    //   vmcnt(0) + barrier already cover k-steps 1 .. 3);
    //   MFMAs of k-step s: fragment f + 1 is unpacked while f's two MFMAs run, and each packed fragment is
    //   replaced by k-step s + 1's right after its MFMAs.
    // two: 2 when both of the wave's token tiles {2 wr, 2 wr + 1} are inside the image, else 1 (the second
    // tile's MFMAs are skipped; N = 197 has 13 tiles). The order inside a k-step is pinned (sched_barrier); the DMA pieces (odd k-steps) and the
    // two activation loads go between the first fragments' MFMAs in that order (the next top's count).
    auto kstep = [&](auto r0, auto r1, int s, int q) __attribute__((always_inline)) {
      constexpr int R0 = decltype(r0)::value, R1 = decltype(r1)::value;
      constexpr auto inr = [](int R, int f) constexpr { return R == 1 || (R == 2 && f < 6) || (R == 3 && f >= 6); };
      constexpr auto used = [=](int f) constexpr { return inr(R0, f) || inr(R1, f); };
      constexpr int F0 = (R0 == 3 && R1 != 1 && R1 != 2) ? 6 : 0;  // first fragment used
      __builtin_amdgcn_sched_barrier(0);
      if (q & 1) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(TOPCNT) : "memory");
      __builtin_amdgcn_sched_barrier(0);
      sp.mark(7);
      const int rn = (q + 1) & 3;
      const bool more = s + 1 < nk;
      v4i wc = unpack16(wfr[F0]);
#pragma unroll
      for (int f = 0; f < 12; ++f) {
        if (inr(R0, f)) acc[0][f] = __builtin_amdgcn_mfma_i32_16x16x64_i8(wc, xa[q][0], acc[0][f], 0, 0, 0);
        if (inr(R1, f)) acc[1][f] = __builtin_amdgcn_mfma_i32_16x16x64_i8(wc, xa[q][1], acc[1][f], 0, 0, 0);
        if (f < 11 && used(f + 1)) wc = unpack16(wfr[f + 1]);
        if (more) wfr[f] = wfrag(rn, f);
        if (f == 0 && (q & 1)) {  // weight k-steps s + 3, s + 4 (past the unit's end: the next unit's 0 .. 3)
#pragma unroll
          for (int d = 3; d <= 4; ++d) {
            if (s + d < nk) dma_piece(cur, s + d, (q + d) & 3);
            else dma_piece(nxt, s + d - nk, (q + d) & 3);
          }
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
    auto kloop = [&](auto r0, auto r1) __attribute__((always_inline)) {
#pragma unroll
      for (int f = 0; f < 12; ++f) wfr[f] = wfrag(0, f);
      if constexpr (NKC > 0) {
#pragma unroll
        for (int s = 0; s < NKC; s += 4) {
          kstep(r0, r1, s, 0);
          kstep(r0, r1, s + 1, 1);
          kstep(r0, r1, s + 2, 2);
          kstep(r0, r1, s + 3, 3);
        }
      } else {
        for (int s = 0; s < nk; s += 4) {
          kstep(r0, r1, s, 0);
          kstep(r0, r1, s + 1, 1);
          kstep(r0, r1, s + 2, 2);
          kstep(r0, r1, s + 3, 3);
        }
      }
    };
    using IC1 = std::integral_constant<int, 1>;
    if (pmode == 0) kloop(IC1{}, IC1{});
    else if (pmode == 2) kloop(IC1{}, std::integral_constant<int, 2>{});
    else if (pmode == 3) kloop(std::integral_constant<int, 3>{}, std::integral_constant<int, 3>{});
    else kloop(IC1{}, std::integral_constant<int, 0>{});  // (a third, MFMA-free variant for nt == 0 spills)
    cur = nxt;
    unit_src(j + 2, nxt);
    sp.mark(9);

    // ---- 2. epilogue: q -> registers, k / v -> LDS images -----------------------------------------
    // acc[tt][4p + r][jj] = feature 64h + 16 fq + 4 r + jj of group p (q, k, v) for token 16 tile + fr
    h8 qh[TPW][2], ql[TPW][2];
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt) {
      const int row = 16 * ptile(wr, tt) + fr;  // token / key row of the images
      const bool pv = ptile(wr, tt) < ntile;     // (the projection's tile: wr = 7's are 9 and 11 when balanced)
      const bool lo_half = prange[tt] == 1 || prange[tt] == 2, hi_half = prange[tt] == 1 || prange[tt] == 3;
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
        } else if (pv) {
          if (p == 1) {
            if (lo_half) {  // fragments 4, 5: features 16 fq .. + 7 of k
              *reinterpret_cast<h8*>(kv + koff(row, 2 * fq)) = hi0;
              *reinterpret_cast<h8*>(kv + IMGF + koff(row, 2 * fq)) = lo0;
            }
            if (hi_half) {  // fragments 6, 7: features 16 fq + 8 .. + 15
              *reinterpret_cast<h8*>(kv + koff(row, 2 * fq + 1)) = hi1;
              *reinterpret_cast<h8*>(kv + IMGF + koff(row, 2 * fq + 1)) = lo1;
            }
          } else if (hi_half) {
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
    sp.mark(6);

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
