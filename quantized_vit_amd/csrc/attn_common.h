// Shared pieces of the attention kernels (attention.hip, qkv_attention.hip): fp16 hi/lo operand
// images, the 3-pass fp16 MFMA product, the online-softmax block update and the output epilogue.
#pragma once
#include "diag_stamps.h"
#include "qvit_common.h"

namespace qvit_attn {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef short s8v __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned int u4 __attribute__((ext_vector_type(4)));

constexpr int HD = 64;          // head dim (the only one supported)
constexpr int KB = 32;          // keys per block
constexpr int IMG = KB * HD * 2;       // one fp16 image of a key block: 4 KiB
constexpr float LOG2E = 1.4426950408889634f;

QVIT_DEV int koff(int r, int c) { return r * 128 + 16 * (c ^ ((r >> 1) & 7)); }
QVIT_DEV int voff(int r, int byte) { return r * 128 + 32 * ((byte >> 5) ^ ((r >> 1) & 3)) + (byte & 31); }

QVIT_DEV void split8(const float (&x)[8], h8& hi, h8& lo) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const _Float16 h = (_Float16)x[i];
    hi[i] = h;
    lo[i] = (_Float16)(x[i] - (float)h);
  }
}

// P's fp16 hi/lo split with the same values as split8 (hi = RNE f16 of x; lo = RNE f16 of the
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

QVIT_DEV h8 lds_h8(const int8_t* base, int off) { return *reinterpret_cast<const h8*>(base + off); }

QVIT_DEV s4v tr_read(const int8_t* base, int off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s4v*)(uintptr_t)(const __attribute__((address_space(3))) void*)(base + off));
}

QVIT_DEV h8 join(s4v a, s4v b) {
  const s8v s = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(h8, s);
}

QVIT_DEV f4 mfma3(h8 ah, h8 al, h8 bh, h8 bl, f4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, c, 0, 0, 0);
  return c;
}

// Cross-lane max / sum over the 4 lane groups g (xor 16, xor 32) with the gfx950 permlane swaps (VALU,
// no LDS round trip); the sums add in the same order as a butterfly of shuffles.
// (scores are never NaN: IEEE maximum, v_maximum3_f32 on gfx950, needs none of fmaxf's operand quieting)
QVIT_DEV float fmax_nn(float a, float b) { return __builtin_elementwise_maximum(a, b); }
QVIT_DEV float xmax(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmax_nn(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmax_nn(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
QVIT_DEV float xsum(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// Stamps (phase timing of diagnostic builds; empty in the library): diag_stamps.h.

// Online-softmax update of one key block (KB keys in the LDS images at st) for a wave's first NT query
// tiles, in three phases that keep the live fragments small (2 waves per SIMD leave 256 registers):
//   1. S^T = K . Q^T for every tile (K fragments live only here);
//   2. the softmax of every tile: running max / sum, P split to fp16 hi/lo in place of the scores;
//   3. O^T += V^T . P^T one 16-dim slice at a time (one V fragment pair live).
// No branches between the tiles: the softmax of tile i runs while the matrix core finishes the later
// tiles' scores, and the first slices' PV products overlap the last softmaxes.
// s[i][kt][j] = S^T[key kbase + 16 kt + j][query of the lane]; scores in log2 units (sl2).
// MASK: the block holds keys >= N (the last block only).
// T: query tiles per wave (arrays); IMGS: byte distance between the K hi, K lo, V hi and V lo images.
template <int T, int IMGS = IMG, bool VEARLY = false>
QVIT_DEV void attend(int nt, bool mask, const int8_t* st, const h8 (&qh)[T][2], const h8 (&ql)[T][2], float (&m)[T],
                     float (&l)[T], f4 (&o)[T][4], const int (&koffs)[2][2], const int (&voffs)[4], int kbase,
                     int N, float sl2, Stamps& sp) {
  constexpr int NT = T;
  f4 s[NT][2];
  // the last block's second 16 keys all past N (N % 32 in 1..16): their scores are masked, skip them
  const bool half = mask && (kbase & ~31) + 16 >= N;  // kbase = block start + 4 g, g < 4
  {
    h8 kh[2][2], kl[2][2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        if (kt == 1 && half) continue;
        kh[kt][c] = lds_h8(st, koffs[kt][c]);
        kl[kt][c] = lds_h8(st + IMGS, koffs[kt][c]);
      }
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        s[i][kt] = f4{0.f, 0.f, 0.f, 0.f};
        if (i >= nt) continue;                 // wave-uniform: the wave has nt tiles
        if (kt == 1 && half) continue;        // wave-uniform
#pragma unroll
        for (int c = 0; c < 2; ++c) s[i][kt] = mfma3(kh[kt][c], kl[kt][c], qh[i][c], ql[i][c], s[i][kt]);
      }
  }
  sp.mark(1);
  // VEARLY: the V fragments of the whole block are issued before the softmax and land while it runs, so
  // the P.V products never wait on an LDS round trip (read per 16-dim slice, each slice waits on one);
  // it costs 32 registers, which the split kernel (4 query tiles per wave) does not have
  h8 vh[4], vl[4];
  if (VEARLY) {
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      vh[dt] = join(tr_read(st + 2 * IMGS, voffs[dt]), tr_read(st + 2 * IMGS, voffs[dt] + 16 * 128));
      vl[dt] = join(tr_read(st + 3 * IMGS, voffs[dt]), tr_read(st + 3 * IMGS, voffs[dt] + 16 * 128));
    }
  }
  h8 ph[NT], pl[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    if (i >= nt) continue;
    float x[8];
    // raw scores of this lane's query; sl2 (> 0) goes into the exponent's fma: the max of the scaled
    // scores is sl2 times the max of the raw ones (rounding is monotone)
    float r[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) r[e] = s[i][e >> 2][e & 3];
    if (mask) {  // wave-uniform: the last key block only
#pragma unroll
      for (int e = 0; e < 8; ++e) r[e] = (kbase + 16 * (e >> 2) + (e & 3) < N) ? r[e] : -INFINITY;
    }
    float bm = fmax_nn(fmax_nn(fmax_nn(r[0], r[1]), fmax_nn(r[2], r[3])), fmax_nn(fmax_nn(r[4], r[5]), fmax_nn(r[6], r[7])));
    bm = xmax(bm) * sl2;
    // deferred max: the running max moves only when some query's block max exceeds it by more than 8
    // (log2 units), so P <= 2^8 (exact in the fp16 hi/lo split) and o, l are rescaled only then; a query
    // whose max did not grow gets alpha = exp2(0) = 1 exactly
    if (__builtin_amdgcn_ballot_w64(bm > m[i] + 8.f) != 0) {
      const float mn = fmax_nn(m[i], bm);
      const float alpha = __builtin_amdgcn_exp2f(m[i] - mn);
      l[i] *= alpha;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[i][dt] = o[i][dt] * alpha;
      m[i] = mn;
    }
    const float nm = -m[i];
    float ps = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      x[e] = __builtin_amdgcn_exp2f(fmaf(r[e], sl2, nm));
      ps += x[e];
    }
    l[i] += ps;
    split8_mix(x, ph[i], pl[i]);
  }
  sp.mark(2);
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    if (!VEARLY) {
      vh[dt] = join(tr_read(st + 2 * IMGS, voffs[dt]), tr_read(st + 2 * IMGS, voffs[dt] + 16 * 128));
      vl[dt] = join(tr_read(st + 3 * IMGS, voffs[dt]), tr_read(st + 3 * IMGS, voffs[dt] + 16 * 128));
    }
#pragma unroll
    for (int i = 0; i < NT; ++i)
      if (i < nt) o[i][dt] = mfma3(vh[dt], vl[dt], ph[i], pl[i], o[i][dt]);
  }
  sp.mark(3);
}

// The int8 epilogue's code table in LDS (qvit_epi_table_build with QVIT_EPI_I8 semantics), if any.
struct EpiLds {
  const int8_t* ent;  // entries (header excluded), nullptr -> per-element quantizer
  float c0, inv_w, top;  // table geometry (EpiTableHdr, epi_top)
};

// 4x4 transpose between the lane groups g (lanes 16g..16g+15) and the 4 registers: afterwards lane g
// holds what lane k held in register g, as w[k] (two permlane32 swaps, then two permlane16 swaps).
QVIT_DEV void transpose_groups(uint32_t (&w)[4]) {
  auto a = __builtin_amdgcn_permlane32_swap(w[0], w[2], false, false);
  auto b = __builtin_amdgcn_permlane32_swap(w[1], w[3], false, false);
  w[0] = a[0]; w[2] = a[1]; w[1] = b[0]; w[3] = b[1];
  auto c = __builtin_amdgcn_permlane16_swap(w[0], w[1], false, false);
  auto d = __builtin_amdgcn_permlane16_swap(w[2], w[3], false, false);
  w[0] = c[0]; w[1] = c[1]; w[2] = d[0]; w[3] = d[1];
}

// Normalise and write a wave's query tiles: fp32 rows, or the next layer's int8 codes. With st16 the
// codes of a row leave as one 16-B store per lane (lane group g: columns 16g .. 16g+15 of the head).
// Tile i of the wave is query tile qtile0 + tstride * i of the group starting at q0.
template <int OUT, int T>
QVIT_DEV void attend_store(const bool (&tv)[T], const float (&l)[T], const f4 (&o)[T][4], int qtile0, int tstride,
                           int q0, int N, int b, int h, float in_scale, void* out, int64_t ldo, const QParams& qp,
                           const EpiLds& tb, bool st16) {
  const int lane = threadIdx.x & 63;
  const int fr = lane & 15, g = lane >> 4;
#pragma unroll
  for (int i = 0; i < T; ++i) {
    if (!tv[i]) continue;  // wave-uniform
    const float inv = 1.f / (xsum(l[i]) * in_scale);
    const int q = q0 + 16 * (qtile0 + tstride * i) + fr;
    const int64_t row = (int64_t)b * N + q;
    if (OUT == 0) {
      if (q >= N) continue;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int col = h * HD + 16 * dt + 4 * g;
        *reinterpret_cast<f4*>(reinterpret_cast<float*>(out) + row * ldo + col) = o[i][dt] * inv;
      }
      continue;
    }
    uint32_t wd[4];
    if (tb.ent != nullptr) {
      float v[4][4];
      uint2 e[4][4];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[dt][j] = o[i][dt][j] * inv;
          e[dt][j] = *epi_entry(tb.ent, v[dt][j], tb.c0, tb.inv_w, tb.top);
        }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        epi_select_byte<0>(wd[dt], v[dt][0], __uint_as_float(e[dt][0].x), e[dt][0].y);
        epi_select_byte<1>(wd[dt], v[dt][1], __uint_as_float(e[dt][1].x), e[dt][1].y);
        epi_select_byte<2>(wd[dt], v[dt][2], __uint_as_float(e[dt][2].x), e[dt][2].y);
        epi_select_byte<3>(wd[dt], v[dt][3], __uint_as_float(e[dt][3].x), e[dt][3].y);
      }
    } else {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const f4 v = o[i][dt] * inv;
        float k[4];
        bool need[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) k[j] = quant_fast(v[j], qp, need[j]);
        if (need[0] | need[1] | need[2] | need[3]) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (need[j]) k[j] = quant_fixup(v[j], qp);
        }
        uint32_t word = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) word |= ((uint32_t)(uint8_t)to_i8_sat(k[j])) << (8 * j);
        wd[dt] = word;
      }
    }
    int8_t* dst = reinterpret_cast<int8_t*>(out) + row * ldo + h * HD;
    if (st16) {
      transpose_groups(wd);
      if (q < N) *reinterpret_cast<uint4*>(dst + 16 * g) = make_uint4(wd[0], wd[1], wd[2], wd[3]);
    } else if (q < N) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) *reinterpret_cast<uint32_t*>(dst + 16 * dt + 4 * g) = wd[dt];
    }
  }
}

QVIT_DEV void fragment_offsets(int (&koffs)[2][2], int (&voffs)[4]) {
  const int lane = threadIdx.x & 63;
  const int fr = lane & 15, g = lane >> 4;
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int c = 0; c < 2; ++c) koffs[kt][c] = koff(16 * kt + fr, g + 4 * c);
  const int vq = fr >> 2, vp = fr & 3;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) voffs[dt] = voff(4 * g + vq, 2 * (16 * dt + 4 * vp));
}


}  // namespace qvit_attn
