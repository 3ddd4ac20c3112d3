// The 32x32 attention body of the fused qkv + attention kernel (qkv_attention.hip, K / V resident for the whole
// sequence). IMGS is the byte distance between a key block's hi and lo images. (A streaming split-operand
// kernel on this body, K / V key blocks through an LDS ring, was measured slower than attention.hip's
// attn_split_kernel on ViT-L: DESIGN.md section 8.)
#pragma once
#include "attn_common.h"

namespace qvit_attn {

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

QVIT_DEV float bits_f(uint32_t u) { return __uint_as_float(u); }
QVIT_DEV float pair_max(float v) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmax_nn(bits_f(a[0]), bits_f(a[1]));
}
QVIT_DEV float pair_sum(float v) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return bits_f(a[0]) + bits_f(a[1]);
}

// S^T of one key block (st: the block's first K hi row; the K lo image IMGS bytes further)
template <int IMGS>
QVIT_DEV f16x scores32(const int8_t* st, const h8 (&qh)[4], const h8 (&ql)[4], const int (&koffs)[4]) {
  h8 kh[4], kl[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    kh[c] = lds_h8(st, koffs[c]);
    kl[c] = lds_h8(st + IMGS, koffs[c]);
  }
  f16x s = {};
#pragma unroll
  for (int c = 0; c < 4; ++c) s = mfma3w(kh[c], kl[c], qh[c], ql[c], s);
  return s;
}

// Online-softmax update of one key block from its scores s. Deferred running max as in attn_common.h
// attend: m moves only when the block max exceeds it by more than 8 (log2 units), so P <= 2^8 is exact in
// the fp16 hi/lo split. MASK: the block holds keys >= N (the last block only).
template <bool MASK, int IMGS>
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
      const int o0 = voffs[dt] + 16 * kc * 128;  // voffs includes the V hi image's offset (2 IMGS)
      vh[dt][kc] = join(tr_read(st, o0), tr_read(st, o0 + 8 * 128));
      vl[dt][kc] = join(tr_read(st + IMGS, o0), tr_read(st + IMGS, o0 + 8 * 128));
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
QVIT_DEV void attend_store32(const bool (&tv)[2], float l, const f16x (&o)[2], int wr, int N, int b, int h,
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

}  // namespace qvit_attn
