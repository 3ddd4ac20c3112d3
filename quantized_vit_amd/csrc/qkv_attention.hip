// Fused qkv projection + attention core of Attention.forward (vit_model.py:126-152) for the fused block:
//   qkv = QuantizeLinear(x_codes)  ->  softmax(q k^T * scale) v  ->  proj's activation quantizer
// with q, k, v never leaving the chip. One persistent workgroup (8 waves) per CU walks (image, head)
// units; per unit:
//   1. projection: wave w computes the 192 q|k|v features of its token tiles {w', w'+8} (w' = w rotated
//      by unit) on v_mfma_i32_16x16x64_i8, as a GEMM-style pipeline: the head's three 64-row weight groups
//      of each 64-deep k-step are LDS-DMA'd (global_load_lds, 6 x 1 KiB, no register staging) from the
//      GEMM's pre-tiled int4 image into a 4-slot ring three k-steps ahead; activation fragments go global
//      -> registers three k-steps ahead; one counted vmcnt + barrier per k-step; the MFMAs of k-step s run
//      while the packed weight fragments of k-step s+1 are read from LDS, each unpacked to 16x-scaled int8
//      right before its two MFMAs;
//   2. epilogue: v = (d_a d_w acc + bias) * in_scale split into fp16 hi/lo exactly as
//      qvit_gemm_qkv_split does; q stays in registers as the wave's own S^T B-operand fragments (the
//      contraction runs over the head dims in the order the accumulators hold them: lane group g owns
//      dims 16g .. 16g+15), k and v go to resident LDS images (208 rows, XOR-swizzled);
//   3. attention: the 7 key blocks of 32 with no barrier (K/V resident), online softmax, P·V, and the
//      output quantizer through its code table (attn_common.h, same arithmetic as qvit_attention_split
//      except the order of the dims inside each q·k sum).
// The next unit's first weight k-steps (ring) and activation k-steps (registers) load while the current
// unit's attention runs. N <= 208.
#include "attn_common.h"

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

// Online-softmax update of one key block for the fused kernel's NTV (1 or 2) query tiles: attn_common.h's
// attend with the branches taken out of the block body. The tile count and the mask (last block only)
// are template parameters, and one ballot per block decides the deferred rescale for all tiles (a tile
// whose own max did not move past its bound is rescaled along, to max(m, block max): still within 2^8
// of every score), so the P computation and the P.V products of both tiles form one branch-free region
// the scheduler can interleave.
template <int NTV, bool MASK>
QVIT_DEV void attend_f(const int8_t* st, const h8 (&qh)[TPW][2], const h8 (&ql)[TPW][2], float (&m)[TPW],
                       float (&l)[TPW], f4 (&o)[TPW][4], const int (&koffs)[2][2], const int (&voffs)[4], int kbase,
                       int N, float sl2) {
  f4 s[NTV][2];
  // the last block's second 16 keys all past N (N % 32 in 1..16): their scores are masked, skip them
  const bool half = MASK && (kbase & ~31) + 16 >= N;  // kbase = block start + 4 g, g < 4
  {
    h8 kh[2][2], kl[2][2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        if (kt == 1 && half) continue;
        kh[kt][c] = lds_h8(st, koffs[kt][c]);
        kl[kt][c] = lds_h8(st + IMGF, koffs[kt][c]);
      }
#pragma unroll
    for (int i = 0; i < NTV; ++i)
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        s[i][kt] = f4{0.f, 0.f, 0.f, 0.f};
        if (kt == 1 && half) continue;  // wave-uniform
#pragma unroll
        for (int c = 0; c < 2; ++c) s[i][kt] = mfma3(kh[kt][c], kl[kt][c], qh[i][c], ql[i][c], s[i][kt]);
      }
  }
  // V fragments of the block issued before the softmax (they land while it runs)
  h8 vh[4], vl[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    vh[dt] = join(tr_read(st + 2 * IMGF, voffs[dt]), tr_read(st + 2 * IMGF, voffs[dt] + 16 * 128));
    vl[dt] = join(tr_read(st + 3 * IMGF, voffs[dt]), tr_read(st + 3 * IMGF, voffs[dt] + 16 * 128));
  }
  float r[NTV][8], bm[NTV];
  bool grow = false;
#pragma unroll
  for (int i = 0; i < NTV; ++i) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      r[i][e] = s[i][e >> 2][e & 3];
      if (MASK) r[i][e] = (kbase + 16 * (e >> 2) + (e & 3) < N) ? r[i][e] : -INFINITY;
    }
    const float b0 = fmax_nn(fmax_nn(fmax_nn(r[i][0], r[i][1]), fmax_nn(r[i][2], r[i][3])),
                             fmax_nn(fmax_nn(r[i][4], r[i][5]), fmax_nn(r[i][6], r[i][7])));
    bm[i] = xmax(b0) * sl2;
    grow |= bm[i] > m[i] + 8.f;
  }
  // deferred running max (attn_common.h attend): moved only when some query's block max exceeds it by
  // more than 8 in log2 units, so P <= 2^8 (exact in the fp16 hi/lo split)
  if (__builtin_amdgcn_ballot_w64(grow) != 0) {
#pragma unroll
    for (int i = 0; i < NTV; ++i) {
      const float mn = fmax_nn(m[i], bm[i]);
      const float alpha = __builtin_amdgcn_exp2f(m[i] - mn);
      l[i] *= alpha;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[i][dt] = o[i][dt] * alpha;
      m[i] = mn;
    }
  }
  h8 ph[NTV], pl[NTV];
#pragma unroll
  for (int i = 0; i < NTV; ++i) {
    const float nm = -m[i];
    float x[8];
    float ps = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      x[e] = __builtin_amdgcn_exp2f(fmaf(r[i][e], sl2, nm));
      ps += x[e];
    }
    l[i] += ps;
    split8(x, ph[i], pl[i]);
  }
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int i = 0; i < NTV; ++i) o[i][dt] = mfma3(vh[dt], vl[dt], ph[i], pl[i], o[i][dt]);
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
      int64_t m = (int64_t)b * N + 16 * (wr + FW * tt) + fr;
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

  int koffs[2][2], voffs[4];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int c = 0; c < 2; ++c) koffs[kt][c] = koff(16 * kt + fr, 2 * fq + c);  // dims 16g + 8c .. +7
  {
    const int vq = fr >> 2, vp = fr & 3;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) voffs[dt] = voff(4 * fq + vq, 2 * (16 * dt + 4 * vp));
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
    for (int tt = 0; tt < TPW; ++tt) tv[tt] = wr + FW * tt < ntile;
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
    // TWO: the wave's second token tile is inside the image (otherwise its MFMAs are skipped: 3 of the 16
    // tiles of N = 197). The order inside a k-step is pinned (sched_barrier); the DMA piece and the two
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
        acc[0][f] = __builtin_amdgcn_mfma_i32_16x16x64_i8(wc, xa[q][0], acc[0][f], 0, 0, 0);
        if (decltype(two)::value) acc[1][f] = __builtin_amdgcn_mfma_i32_16x16x64_i8(wc, xa[q][1], acc[1][f], 0, 0, 0);
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
    if (tv[1]) kloop(std::true_type{});
    else kloop(std::false_type{});
    cur = nxt;
    unit_src(j + 2, nxt);
    sp.mark(9);

    // ---- 2. epilogue: q -> registers, k / v -> LDS images -----------------------------------------
    // acc[tt][4p + r][jj] = feature 64h + 16 fq + 4 r + jj of group p (q, k, v) for token 16 tile + fr
    h8 qh[TPW][2], ql[TPW][2];
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt) {
      const int row = 16 * (wr + FW * tt) + fr;  // token / key row of the images
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
            *reinterpret_cast<h8*>(kv + 2 * IMGF + voff(row, 32 * fq)) = hi0;
            *reinterpret_cast<h8*>(kv + 2 * IMGF + voff(row, 32 * fq + 16)) = hi1;
            *reinterpret_cast<h8*>(kv + 3 * IMGF + voff(row, 32 * fq)) = lo0;
            *reinterpret_cast<h8*>(kv + 3 * IMGF + voff(row, 32 * fq + 16)) = lo1;
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
    float m[TPW], l[TPW];
    f4 o[TPW][4];
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt) {
      m[tt] = -INFINITY;
      l[tt] = 0.f;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[tt][dt] = f4{0.f, 0.f, 0.f, 0.f};
    }
    const int nkb = (N + KB - 1) / KB;
    // full key blocks, then the last (masked when N % 32 != 0); one straight-line body per tile count
    const int nfull = N / KB;
    auto attend_all = [&](auto ntv) __attribute__((always_inline)) {
      constexpr int NTV = decltype(ntv)::value;
      for (int kb = 0; kb < nfull; ++kb)
        attend_f<NTV, false>(kv + kb * KB * 128, qh, ql, m, l, o, koffs, voffs, kb * KB + 4 * fq, N, sl2);
      if (nfull < nkb)
        attend_f<NTV, true>(kv + nfull * KB * 128, qh, ql, m, l, o, koffs, voffs, nfull * KB + 4 * fq, N, sl2);
    };
    if (nt == 2) attend_all(std::integral_constant<int, 2>{});
    else if (nt == 1) attend_all(std::integral_constant<int, 1>{});
    sp.mark(0);
    attend_store<OUT, TPW>(tv, l, o, wr, FW, 0, N, b, h, in_scale, out, ldo, qp, tb, st16);
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

#ifdef QVIT_ATT_STAMPS
extern "C" int qvit_qkv_att_stamps(unsigned long long* host8, int reset) {
  if (reset) {
    const unsigned long long z[16] = {};
    return qvit_hip_status(hipMemcpyToSymbol(HIP_SYMBOL(qvit_attn::qvit_att_stamp_sums), z, sizeof(z)));
  }
  return qvit_hip_status(
      hipMemcpyFromSymbol(host8, HIP_SYMBOL(qvit_attn::qvit_att_stamp_sums), 16 * sizeof(unsigned long long)));
}
#endif
