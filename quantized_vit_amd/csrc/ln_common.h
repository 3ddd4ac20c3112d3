// LayerNorm + activation quantizer of one row held by one wave (Block.norm1 / norm2, vit_model.py:193,206-207,
// eps 1e-6, followed by the next layer's quantize_act, quant_layers.py:356-381). Shared by the standalone
// kernel (quant_kernels.hip layernorm_quant_*) and the residual GEMM with the LayerNorm fused behind it
// (gemm_w4a8.hip EPI_F32_RESID_LN), so both produce bit-identical codes: lane l holds columns 4 (l + 64 i) .. + 3
// of the row (i < NV), the sums are reduced in the same order, and y = (x - mean) * rstd * gamma + beta.
#pragma once
#include "qvit_common.h"

QVIT_DEV float wave_sum_fast(float v) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(b[0]) + __uint_as_float(b[1]);
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xf, 0xf, false));  // row_ror:8
  v += __shfl_xor(v, 4, 64);
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xf, 0xf, false));   // xor 2
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xf, 0xf, false));   // xor 1
  return v;
}

// The row's code words: word[i] holds the codes of columns 4 (lane + 64 i) .. + 3 (byte j = column + j); only
// the words with 4 (lane + 64 i) < cols are meaningful. gb(i, g, b) supplies gamma / beta of those columns.
// ent != nullptr: the quantizer's code table (qvit_epi_table_build, EPI_I8) at ent; else the direct quantizer.
// MODE: 0 = either (ent decides at run time), 1 = table only (ent != nullptr), 2 = direct quantizer only
template <int NV, class GB, int MODE = 0>
QVIT_DEV void ln_quant_row(const float4 (&v)[NV], int lane, int cols, float eps, GB gb, const int8_t* ent, float c0,
                           float inv_w, float top, const QParams& p, uint32_t (&word)[NV]) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  const float mean = wave_sum_fast(s) / (float)cols;
  float s2 = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = 4 * (lane + 64 * i);
    if (c < cols) {
      const float a = v[i].x - mean, b = v[i].y - mean, cc = v[i].z - mean, dd = v[i].w - mean;
      s2 += (a * a + b * b) + (cc * cc + dd * dd);
    }
  }
  const float var = wave_sum_fast(s2) / (float)cols;
  const float rstd = 1.0f / sqrtf(var + eps);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = 4 * (lane + 64 * i);
    word[i] = 0;
    if (c < cols) {
      float4 gv, bv;
      gb(i, gv, bv);
      const float y[4] = {(v[i].x - mean) * rstd * gv.x + bv.x, (v[i].y - mean) * rstd * gv.y + bv.y,
                          (v[i].z - mean) * rstd * gv.z + bv.z, (v[i].w - mean) * rstd * gv.w + bv.w};
      uint32_t w;
      if (MODE == 1 || (MODE == 0 && ent != nullptr)) {
        uint2 e[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) e[j] = *epi_entry(ent, y[j], c0, inv_w, top);
        epi_select_byte<0>(w, y[0], __uint_as_float(e[0].x), e[0].y);
        epi_select_byte<1>(w, y[1], __uint_as_float(e[1].x), e[1].y);
        epi_select_byte<2>(w, y[2], __uint_as_float(e[2].x), e[2].y);
        epi_select_byte<3>(w, y[3], __uint_as_float(e[3].x), e[3].y);
      } else {
        w = (uint32_t)(uint8_t)to_i8_sat(quant_code(y[0], p)) | ((uint32_t)(uint8_t)to_i8_sat(quant_code(y[1], p)) << 8) |
            ((uint32_t)(uint8_t)to_i8_sat(quant_code(y[2], p)) << 16) |
            ((uint32_t)(uint8_t)to_i8_sat(quant_code(y[3], p)) << 24);
      }
      word[i] = w;
    }
  }
}
