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

// ---- attention on v_mfma_f32_32x32x16_f16 --------------------------------------------------------------
// A wave's two 16-query tiles are one 32-query tile (query r < 16: tile 0, else tile 1, token r & 15). Per key
// block of 32: S^T = K . Q^T (keys x queries, 4 dim chunks x 3 passes), then O^T += V^T . P^T (2 32-dim tiles x
// 2 key chunks x 3 passes): 24 MFMAs that hold the SIMD's vector issue 8 of 32 cycles each, instead of 48
// 16x16x32 ones that hold it 8 of 16 (the phase is issue-bound). A lane (r = lane & 31, h = lane >> 5) owns
// query r: S^T's accumulator holds its scores of keys (e & 3) + 8 (e >> 2) + 4 h (e < 16), the other 16 are
// in lane ^ 32, so a row max / sum is 15 in-lane steps and one permlane32 swap.
// The contraction orders: the q . k sum of MFMA chunk c runs over dims 32 h + 8 c + j (K's 16-B chunk 4 h + c,
// the layout koff already has); the P . V sum over chunk kc takes S^T's registers 8 kc .. 8 kc + 7 as its
// B operand with no lane movement, so element j of half h is key 16 kc + 8 (j >> 2) + 4 h + (j & 3), and V^T
// is read (ds_read_b64_tr_b16) in that same key order.
typedef float f16x __attribute__((ext_vector_type(16)));

QVIT_DEV f16x mfma3w(h8 ah, h8 al, h8 bh, h8 bl, f16x c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, c, 0, 0, 0);
  return c;
}

// V image of the fused kernel: 128-B rows, 16-B chunks XOR-swizzled by row bits 1 and 2 only, so the transposed
// reads of 4 consecutive rows x 64 B (one 32-lane pass) cover all 64 banks, and a read 8, 16 or 32 rows further
// keeps the same swizzle (an immediate offset); the epilogue's 16-B writes are 2-way
QVIT_DEV int v32off(int r, int byte) { return r * 128 + (byte ^ (((((r >> 1) & 1) << 2) | ((r >> 2) & 1)) << 4)); }

// P's fp16 hi/lo split with the same values as attn_common.h split8 (hi = RNE f16 of x; lo = RNE f16 of the
// exact f32 x - hi) in fewer VALU: lo comes from v_fma_mix{lo,hi}_f16 (-hi as an f16 source, x as f32, one
// rounding of the exact difference) instead of cvt f16 -> f32, subtract and cvt back. The asm carries its own
// wait states: s_nop 0 first (x is fresh from v_exp: transcendental -> VALU use), s_nop 1 last (its results
// are MFMA operands: VALU write -> MFMA read).
QVIT_DEV void split8_mix(const float (&x)[8], h8& hi, h8& lo) {
#pragma unroll
  for (int i = 0; i < 8; ++i) hi[i] = (_Float16)x[i];
  const u4 hw = __builtin_bit_cast(u4, hi);
  u4 lw;
  asm("s_nop 0\n\t"
      "v_fma_mixlo_f16 %0, -%4, 1.0, %8 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %0, -%4, 1.0, %9 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixlo_f16 %1, -%5, 1.0, %10 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %1, -%5, 1.0, %11 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixlo_f16 %2, -%6, 1.0, %12 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %2, -%6, 1.0, %13 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixlo_f16 %3, -%7, 1.0, %14 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %3, -%7, 1.0, %15 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
      "s_nop 1"
      : "=&v"(lw[0]), "=&v"(lw[1]), "=&v"(lw[2]), "=&v"(lw[3])
      : "v"(hw[0]), "v"(hw[1]), "v"(hw[2]), "v"(hw[3]), "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]), "v"(x[4]),
        "v"(x[5]), "v"(x[6]), "v"(x[7]));
  lo = __builtin_bit_cast(h8, lw);
}

QVIT_DEV float bits_f(uint32_t u) { return __uint_as_float(u); }
QVIT_DEV float pair_max(float v) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmax_nn(bits_f(a[0]), bits_f(a[1]));
}
QVIT_DEV float pair_sum(float v) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return bits_f(a[0]) + bits_f(a[1]);
}

// S^T of one key block (st: the block's first K hi row)
QVIT_DEV f16x scores32(const int8_t* st, const h8 (&qh)[4], const h8 (&ql)[4], const int (&koffs)[4]) {
  h8 kh[4], kl[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    kh[c] = lds_h8(st, koffs[c]);
    kl[c] = lds_h8(st + IMGF, koffs[c]);
  }
  f16x s = {};
#pragma unroll
  for (int c = 0; c < 4; ++c) s = mfma3w(kh[c], kl[c], qh[c], ql[c], s);
  return s;
}

// Online-softmax update of one key block from its scores s. Deferred running max as in attn_common.h
// attend: m moves only when the block max exceeds it by more than 8 (log2 units), so P <= 2^8 is exact in
// the fp16 hi/lo split. MASK: the block holds keys >= N (the last block only).
template <bool MASK>
QVIT_DEV void softmax_pv32(const int8_t* st, const f16x& s, float& m, float& l, f16x (&o)[2],
                           const int (&voffs)[2], int kbase, int N, float sl2) {
  // the last block's keys 16 .. 31 all past N (N % 32 in 1 .. 16): their P are 0, skip their V reads and P.V
  const bool half = MASK && kbase + 16 >= N;
  // V fragments of the block issued before the softmax (they land while it runs)
  h8 vh[2][2], vl[2][2];
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int kc = 0; kc < 2; ++kc) {
      if (kc == 1 && half) continue;  // wave-uniform
      const int o0 = voffs[dt] + 16 * kc * 128;  // voffs includes the V hi image's 2 IMGF
      vh[dt][kc] = join(tr_read(st, o0), tr_read(st, o0 + 8 * 128));
      vl[dt][kc] = join(tr_read(st + IMGF, o0), tr_read(st + IMGF, o0 + 8 * 128));
    }
  float r[16];
  const int h4 = 4 * ((threadIdx.x >> 5) & 1);
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    r[e] = s[e];
    if (MASK) r[e] = (kbase + (e & 3) + 8 * (e >> 2) + h4 < N) ? r[e] : -INFINITY;
  }
  // 16 scores -> one max in 8 v_maximum3_f32
  float t[5];
#pragma unroll
  for (int e = 0; e < 5; ++e) t[e] = fmax_nn(fmax_nn(r[3 * e], r[3 * e + 1]), r[3 * e + 2]);
  const float b0 = fmax_nn(fmax_nn(fmax_nn(t[0], t[1]), t[2]), fmax_nn(fmax_nn(t[3], t[4]), r[15]));
  const float bm = pair_max(b0) * sl2;
  // deferred rescale (rare after the first block). The running max is kept an integer (ceil), so alpha is a
  // power of two and the rescale is an exact v_ldexp_f32 per accumulator: scalar, where a compiler multiply is
  // SLP-packed into v_pk_mul_f32 (packed f32 VALU beside the MFMAs costs several times its issue slot)
  if (__builtin_amdgcn_ballot_w64(bm > m + 8.f) != 0) {
    const float mn = __builtin_ceilf(fmax_nn(m, bm));
    const int k = (int)fmax_nn(m - mn, -256.f);  // the first block (m = -inf) scales the zero o, l by 2^-256
    l = __builtin_amdgcn_ldexpf(l, k);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      o[0][e] = __builtin_amdgcn_ldexpf(o[0][e], k);
      o[1][e] = __builtin_amdgcn_ldexpf(o[1][e], k);
    }
    m = mn;
  }
  const float nm = -m;
  float x[2][8];
  float ps = 0.f;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    x[e >> 3][e & 7] = __builtin_amdgcn_exp2f(fmaf(r[e], sl2, nm));
    ps += x[e >> 3][e & 7];
  }
  l += ps;
  h8 ph[2], pl[2];
  split8_mix(x[0], ph[0], pl[0]);
  split8_mix(x[1], ph[1], pl[1]);
#pragma unroll
  for (int kc = 0; kc < 2; ++kc) {
    if (kc == 1 && half) continue;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) o[dt] = mfma3w(vh[dt][kc], vl[dt][kc], ph[kc], pl[kc], o[dt]);
  }
}

// Normalise and write the wave's 32 queries: fp32 rows, or the next layer's int8 codes. o[dt][4 g + j] is dim
// 32 dt + 8 g + 4 h + j of the lane's query; with st16 the two halves trade words (permlane32) so that each
// lane stores 16 contiguous codes per 32-dim tile (half h: dims 32 dt + 16 h .. + 15).
template <int OUT>
QVIT_DEV void attend_store32(const bool (&tv)[TPW], float l, const f16x (&o)[2], int wr, int N, int b, int h,
                             float in_scale, void* out, int64_t ldo, const QParams& qp, const EpiLds& tb, bool st16) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 31, hh = lane >> 5;
  const int tile = r >> 4;
  const float inv = 1.f / (pair_sum(l) * in_scale);
  const int q = 16 * (2 * wr + tile) + (r & 15);
  const bool ok = (tile ? tv[1] : tv[0]) && q < N;
  const int64_t row = (int64_t)b * N + q;
  if (OUT == 0) {
    if (!ok) return;
    float* dst = reinterpret_cast<float*>(out) + row * ldo + h * HD + 4 * hh;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<f4*>(dst + 32 * dt + 8 * g) =
            f4{o[dt][4 * g], o[dt][4 * g + 1], o[dt][4 * g + 2], o[dt][4 * g + 3]} * inv;
    return;
  }
  uint32_t wd[2][4];
#pragma unroll
  for (int dt = 0; dt < 2; ++dt) {
    if (tb.ent != nullptr) {
      float v[4][4];
      uint2 e[4][4];
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[g][j] = o[dt][4 * g + j] * inv;
          e[g][j] = *epi_entry(tb.ent, v[g][j], tb.c0, tb.inv_w, tb.top);
        }
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        epi_select_byte<0>(wd[dt][g], v[g][0], __uint_as_float(e[g][0].x), e[g][0].y);
        epi_select_byte<1>(wd[dt][g], v[g][1], __uint_as_float(e[g][1].x), e[g][1].y);
        epi_select_byte<2>(wd[dt][g], v[g][2], __uint_as_float(e[g][2].x), e[g][2].y);
        epi_select_byte<3>(wd[dt][g], v[g][3], __uint_as_float(e[g][3].x), e[g][3].y);
      }
    } else {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float k[4];
        bool need[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) k[j] = quant_fast(o[dt][4 * g + j] * inv, qp, need[j]);
        if (need[0] | need[1] | need[2] | need[3]) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (need[j]) k[j] = quant_fixup(o[dt][4 * g + j] * inv, qp);
        }
        uint32_t word = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) word |= ((uint32_t)(uint8_t)to_i8_sat(k[j])) << (8 * j);
        wd[dt][g] = word;
      }
    }
  }
  int8_t* dst = reinterpret_cast<int8_t*>(out) + row * ldo + h * HD;
  if (st16) {
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      const auto a = __builtin_amdgcn_permlane32_swap(wd[dt][0], wd[dt][2], false, false);
      const auto c = __builtin_amdgcn_permlane32_swap(wd[dt][1], wd[dt][3], false, false);
      if (ok) *reinterpret_cast<uint4*>(dst + 32 * dt + 16 * hh) = make_uint4(a[0], a[1], c[0], c[1]);
    }
  } else if (ok) {
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) *reinterpret_cast<uint32_t*>(dst + 32 * dt + 8 * g + 4 * hh) = wd[dt][g];
  }
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
        if (nfull < nkb) softmax_pv32<true>(kv + kb * KB * 128, sc, m, l, o, voffs, kb * KB, N, sl2);
        else softmax_pv32<false>(kv + kb * KB * 128, sc, m, l, o, voffs, kb * KB, N, sl2);
      };
      f16x sa = scores32(kv, q32h, q32l, koffs);
      if (nkb == 7) {
#pragma unroll
        for (int kb = 0; kb < 6; ++kb) {
          const f16x sb = scores32(kv + (kb + 1) * KB * 128, q32h, q32l, koffs);
          softmax_pv32<false>(kv + kb * KB * 128, sa, m, l, o, voffs, kb * KB, N, sl2);
          sa = sb;
        }
        last(6, sa);
      } else {
        int kb = 0;
        for (; kb + 2 < nkb; kb += 2) {
          const f16x sb = scores32(kv + (kb + 1) * KB * 128, q32h, q32l, koffs);
          softmax_pv32<false>(kv + kb * KB * 128, sa, m, l, o, voffs, kb * KB, N, sl2);
          sa = scores32(kv + (kb + 2) * KB * 128, q32h, q32l, koffs);
          softmax_pv32<false>(kv + (kb + 1) * KB * 128, sb, m, l, o, voffs, (kb + 1) * KB, N, sl2);
        }
        if (kb + 1 < nkb) {
          const f16x sb = scores32(kv + (kb + 1) * KB * 128, q32h, q32l, koffs);
          softmax_pv32<false>(kv + kb * KB * 128, sa, m, l, o, voffs, kb * KB, N, sl2);
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
