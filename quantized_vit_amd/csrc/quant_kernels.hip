// Memory-bound quantizer kernels of libqvit_hip.so (gfx950):
//   activation -> int8 codes, fp32 fake-quant, weight -> packed int4/int8 operand,
//   conv im2col -> codes, LayerNorm -> codes, bias padding.
// Every kernel reads its fp32 input once and writes int8 once (16 B per lane where the layout
// allows), so the bound is HBM bandwidth: 5 bytes moved per element.
#include "qvit_common.h"
#include "ln_common.h"

#include <algorithm>

namespace {

constexpr int kThreads = 256;

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

inline int grid_for(int64_t work, int threads) {
  int64_t g = cdiv(work, threads);
  const int64_t cap = 256 * 16;  // 16 blocks per CU, grid-stride beyond
  return (int)(g < cap ? (g > 0 ? g : 1) : cap);
}

// ---- activation quantizer: one thread = 16 columns of one row -> one 16-byte store ----------
__global__ __launch_bounds__(kThreads) void quantize_act_kernel(
    const float* __restrict__ x, int64_t rows, int64_t cols, int64_t ldx, int qtype,
    const float* d, const float* qm, const float* t, int levels, int8_t* __restrict__ codes,
    int64_t ldc, int64_t kpad) {
  const QParams p = load_qparams(qtype, d, qm, t, levels);
  const int64_t chunks_per_row = kpad / 16;
  const int64_t total = rows * chunks_per_row;
  const bool vec = ((ldx & 3) == 0) && ((((uintptr_t)x) & 15) == 0);
  for (int64_t id = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; id < total;
       id += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = id / chunks_per_row;
    const int64_t c0 = (id - r * chunks_per_row) * 16;
    const float* src = x + r * ldx + c0;
    float v[16];
    if (vec && c0 + 16 <= cols) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float4 f = *reinterpret_cast<const float4*>(src + 4 * i);
        v[4 * i + 0] = f.x; v[4 * i + 1] = f.y; v[4 * i + 2] = f.z; v[4 * i + 3] = f.w;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = (c0 + i < cols) ? src[i] : 0.f;
    }
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint32_t acc = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int8_t k = to_i8_sat(quant_code(v[4 * i + b], p));
        acc |= ((uint32_t)(uint8_t)k) << (8 * b);
      }
      w[i] = acc;
    }
    *reinterpret_cast<uint4*>(codes + r * ldc + c0) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

__global__ __launch_bounds__(kThreads) void fake_quant_kernel(const float* __restrict__ x, int64_t n,
                                                              int qtype, const float* d,
                                                              const float* qm, const float* t,
                                                              int levels, float* __restrict__ y) {
  const QParams p = load_qparams(qtype, d, qm, t, levels);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    y[i] = fake_quant_value(x[i], p);
  }
}

__global__ __launch_bounds__(kThreads) void gelu_kernel(const float* __restrict__ x, int64_t n, float* __restrict__ y) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = gelu_ref(x[i]);
}

// ---- weight quantizer + operand packing ------------------------------------------------------
// Packed row rho holds weight row perm(rho): inside each 64-row group swap bits [3:2] and [5:4].
__device__ __forceinline__ int64_t perm_row(int64_t rho) {
  const int64_t lo = rho & 3, r = (rho >> 2) & 3, q = (rho >> 4) & 3;
  return (rho & ~int64_t(63)) | (r << 4) | (q << 2) | lo;
}

// Packed weight format = the GEMM's LDS images, pre-tiled: for n-block nb (256 packed rows) and k-stage
// st (64 k), one contiguous tile of 256 rows x 32 B (W4) / 64 B (W8); inside a tile, row r holds its 8-B
// (W4) / 16-B (W8) chunk c at position c ^ (((r >> 3) & 1) << 1) (W4) / c ^ (((r >> 2) & 1) << 1) (W8),
// the bank-conflict-free swizzle of the fragment reads. The GEMM stages a tile with contiguous 1-KiB
// LDS-DMA pieces (whole cache lines). Byte offset of the 4 (W4) / 8 (W8) bytes holding k0 .. k0+7:
template <int WFMT>
__device__ __forceinline__ int64_t packed_offset(int64_t rho, int64_t k0, int64_t kpad) {
  constexpr int ROWB = (WFMT == QVIT_W4) ? 32 : 64;  // bytes per row per stage
  const int64_t nb = rho >> 8, r = rho & 255, st = k0 >> 6, kk = k0 & 63;
  const int64_t tile = (nb * (kpad >> 6) + st) * (256 * ROWB);
  if (WFMT == QVIT_W4) {
    const int64_t c = kk >> 4;                                  // 8-B chunk (16 k)
    return tile + r * ROWB + 8 * (c ^ (((r >> 3) & 1) << 1)) + ((kk & 15) >> 1);
  } else {
    const int64_t c = kk >> 4;                                  // 16-B chunk (16 k)
    return tile + r * ROWB + 16 * (c ^ (((r >> 2) & 1) << 1)) + (kk & 15);
  }
}

template <int WFMT>
__global__ __launch_bounds__(kThreads) void pack_weight_kernel(
    const float* __restrict__ w, int64_t n, int64_t k, int64_t ldw, int qtype, const float* d,
    const float* qm, const float* t, void* __restrict__ packed, int64_t npad, int64_t kpad,
    int32_t* overflow) {
  const QParams p = load_qparams(qtype, d, qm, t, 0);
  // one thread = 8 consecutive k of one packed row
  const int64_t words_per_row = kpad / 8;
  const int64_t total = npad * words_per_row;
  for (int64_t id = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; id < total;
       id += (int64_t)gridDim.x * blockDim.x) {
    const int64_t rho = id / words_per_row;
    const int64_t k0 = (id - rho * words_per_row) * 8;
    const int64_t row = perm_row(rho);
    int kc[8];
    bool bad = false;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float v = 0.f;
      if (row < n && k0 + i < k) v = w[row * ldw + k0 + i];
      const float c = quant_code(v, p);
      const float lim_lo = (WFMT == QVIT_W4) ? -8.f : -128.f;
      const float lim_hi = (WFMT == QVIT_W4) ? 7.f : 127.f;
      bad |= !(c >= lim_lo && c <= lim_hi);
      kc[i] = (int)fminf(fmaxf(c, lim_lo), lim_hi);
    }
    if (bad && overflow) atomicOr(overflow, 1);
    if (WFMT == QVIT_W4) {
      uint32_t word = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        word |= ((uint32_t)(kc[b] & 0xF)) << (8 * b);
        word |= ((uint32_t)(kc[b + 4] & 0xF)) << (8 * b + 4);
      }
      *reinterpret_cast<uint32_t*>(reinterpret_cast<int8_t*>(packed) + packed_offset<QVIT_W4>(rho, k0, kpad)) = word;
    } else {
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        lo |= ((uint32_t)(uint8_t)(int8_t)kc[b]) << (8 * b);
        hi |= ((uint32_t)(uint8_t)(int8_t)kc[b + 4]) << (8 * b);
      }
      uint2* dst = reinterpret_cast<uint2*>(reinterpret_cast<int8_t*>(packed) + packed_offset<QVIT_W8>(rho, k0, kpad));
      *dst = make_uint2(lo, hi);
    }
  }
}

__global__ __launch_bounds__(kThreads) void pad_bias_kernel(const float* __restrict__ bias, int64_t n,
                                                            float* __restrict__ out, int64_t npad) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < npad;
       i += (int64_t)gridDim.x * blockDim.x) {
    out[i] = (bias != nullptr && i < n) ? bias[i] : 0.f;
  }
}

// ---- conv input -> im2col codes ----------------------------------------------------------------
// I: the index type of the element arithmetic (int when every extent fits: 64-bit divisions cost more than
// the quantizer per 16-element chunk)
template <typename I>
__global__ __launch_bounds__(kThreads) void im2col_quant_kernel(
    const float* __restrict__ x, int64_t B_, int64_t C_, int64_t H_, int64_t W_, int kh, int kw,
    int sh, int sw, int ph, int pw, int dh, int dw, int64_t OH_, int64_t OW_, int qtype,
    const float* d, const float* qm, const float* t, int levels, int8_t* __restrict__ codes,
    int64_t ldc_, int64_t kpad_) {
  const I B = (I)B_, C = (I)C_, H = (I)H_, W = (I)W_, OH = (I)OH_, OW = (I)OW_, ldc = (I)ldc_, kpad = (I)kpad_;
  const QParams p = load_qparams(qtype, d, qm, t, levels);
  const I K = C * kh * kw;
  const I chunks_per_row = kpad / 16;
  const I rows = B * OH * OW;
  const I total = rows * chunks_per_row;
  // patchify fast path: a 16-wide chunk is 16 consecutive pixels of one input row
  const bool patch16 = (kw % 16 == 0) && dw == 1 && pw == 0 && ph == 0 && (W % 4 == 0) &&
                       (sw % 4 == 0) && ((((uintptr_t)x) & 15) == 0);
  for (I id = blockIdx.x * (I)blockDim.x + threadIdx.x; id < total;
       id += (I)gridDim.x * blockDim.x) {
    const I r = id / chunks_per_row;
    const I c0 = (id - r * chunks_per_row) * 16;
    const I b = r / (OH * OW);
    const I rem = r - b * OH * OW;
    const I oh = rem / OW, ow = rem - (rem / OW) * OW;
    float v[16];
    if (patch16 && c0 + 16 <= K) {
      const I ci = c0 / (kh * kw);
      const I r2 = c0 - ci * kh * kw;
      const I ih = r2 / kw, iw = r2 - ih * kw;
      const I y = oh * sh + ih * dh;
      const I xx = ow * sw + iw;
      const float* src = x + ((b * C + ci) * H + y) * W + xx;
      if (y < H && xx + 16 <= W) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float4 f = *reinterpret_cast<const float4*>(src + 4 * i);
          v[4 * i + 0] = f.x; v[4 * i + 1] = f.y; v[4 * i + 2] = f.z; v[4 * i + 3] = f.w;
        }
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = (y < H && xx + i < W) ? src[i] : 0.f;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const I kk = c0 + i;
        float val = 0.f;
        if (kk < K) {
          const I ci = kk / (kh * kw);
          const I r2 = kk - ci * kh * kw;
          const I ih = r2 / kw, iw = r2 - ih * kw;
          const I y = oh * sh - ph + ih * dh;
          const I xx = ow * sw - pw + iw * dw;
          if (y >= 0 && y < H && xx >= 0 && xx < W) val = x[((b * C + ci) * H + y) * W + xx];
        }
        v[i] = val;
      }
    }
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint32_t acc = 0;
#pragma unroll
      for (int bb = 0; bb < 4; ++bb) {
        const int8_t k = to_i8_sat(quant_code(v[4 * i + bb], p));
        acc |= ((uint32_t)(uint8_t)k) << (8 * bb);
      }
      w[i] = acc;
    }
    *reinterpret_cast<uint4*>(codes + r * ldc + c0) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// ---- LayerNorm + quantizer: one wave per row ----------------------------------------------------
QVIT_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Register-resident row: cols % 4 == 0, cols <= 256 * NV. One HBM read of the row, two-pass
// statistics from registers (mean, then sum of squared deviations), one int8 write.
template <int NV>
__global__ __launch_bounds__(kThreads) void layernorm_quant_reg_kernel(
    const float* __restrict__ x, int64_t rows, int64_t cols, int64_t ldx, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, int qtype, const float* d, const float* qm, const float* t,
    int levels, int8_t* __restrict__ codes, int64_t ldc, int64_t kpad) {
  const QParams p = load_qparams(qtype, d, qm, t, levels);
  const int lane = threadIdx.x & 63;
  const int64_t r = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  if (r >= rows) return;
  const float* xr = x + r * ldx;
  float4 v[NV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int64_t c = 4 * (lane + 64 * i);
    v[i] = (c < cols) ? *reinterpret_cast<const float4*>(xr + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  }
  const float mean = wave_sum(s) / (float)cols;
  float s2 = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int64_t c = 4 * (lane + 64 * i);
    if (c < cols) {
      const float a = v[i].x - mean, b = v[i].y - mean, cc = v[i].z - mean, dd = v[i].w - mean;
      s2 += (a * a + b * b) + (cc * cc + dd * dd);
    }
  }
  const float var = wave_sum(s2) / (float)cols;
  const float rstd = 1.0f / sqrtf(var + eps);
  int8_t* cr = codes + r * ldc;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int64_t c = 4 * (lane + 64 * i);
    if (c < cols) {
      const float4 g = gamma ? *reinterpret_cast<const float4*>(gamma + c) : make_float4(1.f, 1.f, 1.f, 1.f);
      const float4 b = beta ? *reinterpret_cast<const float4*>(beta + c) : make_float4(0.f, 0.f, 0.f, 0.f);
      const float y0 = (v[i].x - mean) * rstd * g.x + b.x;
      const float y1 = (v[i].y - mean) * rstd * g.y + b.y;
      const float y2 = (v[i].z - mean) * rstd * g.z + b.z;
      const float y3 = (v[i].w - mean) * rstd * g.w + b.w;
      const uint32_t word = (uint32_t)(uint8_t)to_i8_sat(quant_code(y0, p)) |
                            ((uint32_t)(uint8_t)to_i8_sat(quant_code(y1, p)) << 8) |
                            ((uint32_t)(uint8_t)to_i8_sat(quant_code(y2, p)) << 16) |
                            ((uint32_t)(uint8_t)to_i8_sat(quant_code(y3, p)) << 24);
      *reinterpret_cast<uint32_t*>(cr + c) = word;
    }
  }
  for (int64_t c = cols + lane; c < kpad; c += 64) cr[c] = 0;
}

// The same butterfly (xor 32, 16, 8, 4, 2, 1; identical sums in every lane) with the exact-xor steps on
// permlane swaps and DPP instead of LDS shuffles.

// Persistent register-resident LayerNorm + quantizer (cols % 4 == 0, cols <= 256 * NV): each wave walks
// rows wave, wave + nwaves, ... with the next row's load in flight while the current row is finished;
// gamma/beta, the quantizer scalars and the code table (QVIT_EPI_I8 semantics, nullable) are read once
// per workgroup. Same arithmetic as layernorm_quant_reg_kernel, row for row.
constexpr int LN_TBL_BYTES = 16384;
// T32: codes in the 32x32x32 MFMA operand order of qvit_gemm_a32 (QVIT_ACT_T32): column c of row r at
// ((r >> 5) (kpad >> 5) + (c >> 5)) * 1024 + ((r & 31) + 32 ((c >> 4) & 1)) * 16 + (c & 15); a lane's 4-code word
// stays 4 contiguous bytes (4 | c)
QVIT_DEV int64_t t32_offset(int64_t r, int64_t c, int64_t kpad) {
  return ((r >> 5) * (kpad >> 5) + (c >> 5)) * 1024 + ((r & 31) + 32 * ((c >> 4) & 1)) * 16 + (c & 15);
}
template <int NV, bool T32 = false>
__global__ __launch_bounds__(kThreads, 1) void layernorm_quant_persist_kernel(
    const float* __restrict__ x, int64_t rows, int64_t cols, int64_t ldx, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, int qtype, const float* d, const float* qm, const float* t,
    int levels, int8_t* __restrict__ codes, int64_t ldc, int64_t kpad, const int8_t* __restrict__ table) {
  // code table, then gamma and beta as float4 rows (read per row from LDS: held in registers they would
  // cost 8 NV VGPRs and a wave per SIMD of occupancy)
  __shared__ __attribute__((aligned(16))) int8_t tl[LN_TBL_BYTES + 2 * 4096];
  float4* gbl = reinterpret_cast<float4*>(tl + LN_TBL_BYTES);
  const QParams p = load_qparams(qtype, d, qm, t, levels);
  const int lane = threadIdx.x & 63;
  const int tid = threadIdx.x;
  const int64_t nwaves = ((int64_t)gridDim.x * kThreads) >> 6;
  int64_t r = (blockIdx.x * (int64_t)kThreads + tid) >> 6;
  float4 v[NV];
  auto load_row = [&](int64_t rr, float4 (&dst)[NV]) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int64_t c = 4 * (lane + 64 * i);
      dst[i] = (rr < rows && c < cols) ? *reinterpret_cast<const float4*>(x + rr * ldx + c)
                                       : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  load_row(r, v);  // the first row is in flight while the table is staged
  const int8_t* ent = nullptr;
  float c0 = 0.f, inv_w = 0.f, top = 0.f;
  if (table != nullptr) {
    const EpiTableHdr hd = *reinterpret_cast<const EpiTableHdr*>(table);
    if (hd.valid != 0 && hd.nb >= 1 && 16 + 8 * hd.nb <= LN_TBL_BYTES) {
      for (int k = tid; k < (16 + 8 * hd.nb + 15) / 16; k += kThreads)
        reinterpret_cast<uint4*>(tl)[k] = reinterpret_cast<const uint4*>(table)[k];
      ent = tl + sizeof(EpiTableHdr);
      c0 = hd.c0;
      inv_w = hd.inv_w;
      top = epi_top(hd.nb);
    }
  }
  for (int k = tid; k < 64 * NV; k += kThreads) {
    const int64_t c = 4 * k;
    gbl[k] = (gamma && c < cols) ? *reinterpret_cast<const float4*>(gamma + c) : make_float4(1.f, 1.f, 1.f, 1.f);
    gbl[256 + k] = (beta && c < cols) ? *reinterpret_cast<const float4*>(beta + c) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __syncthreads();
  for (; r < rows; r += nwaves) {
    float4 vn[NV];
    load_row(r + nwaves, vn);
    uint32_t word[NV];
    ln_quant_row<NV>(v, lane, (int)cols, eps,
                     [&](int i, float4& gv, float4& bv) {
                       gv = gbl[lane + 64 * i];
                       bv = gbl[256 + lane + 64 * i];
                     },
                     ent, c0, inv_w, top, p, word);
    if constexpr (T32) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int64_t c = 4 * (lane + 64 * i);
        if (c < cols) *reinterpret_cast<uint32_t*>(codes + t32_offset(r, c, kpad)) = word[i];
      }
      for (int64_t c = cols + lane; c < kpad; c += 64) codes[t32_offset(r, c, kpad)] = 0;
    } else {
      int8_t* cr = codes + r * ldc;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int64_t c = 4 * (lane + 64 * i);
        if (c < cols) *reinterpret_cast<uint32_t*>(cr + c) = word[i];
      }
      for (int64_t c = cols + lane; c < kpad; c += 64) cr[c] = 0;
    }
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = vn[i];
  }
}

// General rows (any cols / stride): re-reads the row from cache for each pass.
__global__ __launch_bounds__(kThreads) void layernorm_quant_kernel(
    const float* __restrict__ x, int64_t rows, int64_t cols, int64_t ldx,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps, int qtype,
    const float* d, const float* qm, const float* t, int levels, int8_t* __restrict__ codes,
    int64_t ldc, int64_t kpad) {
  const QParams p = load_qparams(qtype, d, qm, t, levels);
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t r = wave; r < rows; r += nwaves) {
    const float* xr = x + r * ldx;
    float s = 0.f;
    for (int64_t c = lane; c < cols; c += 64) s += xr[c];
    const float mean = wave_sum(s) / (float)cols;
    float s2 = 0.f;
    for (int64_t c = lane; c < cols; c += 64) {
      const float a = xr[c] - mean;
      s2 += a * a;
    }
    const float var = wave_sum(s2) / (float)cols;
    const float rstd = 1.0f / sqrtf(var + eps);
    int8_t* cr = codes + r * ldc;
    for (int64_t c = lane; c < cols; c += 64) {
      float y = (xr[c] - mean) * rstd;
      if (gamma) y = y * gamma[c];
      if (beta) y = y + beta[c];
      cr[c] = to_i8_sat(quant_code(y, p));
    }
    for (int64_t c = cols + lane; c < kpad; c += 64) cr[c] = 0;
  }
}

}  // namespace

extern "C" {

const char* qvit_strerror(int code) {
  switch (code) {
    case QVIT_OK: return "ok";
    case QVIT_EINVAL: return "invalid argument (size, stride or enum)";
    case QVIT_EALIGN: return "pointer or leading dimension not aligned as required";
    case QVIT_ENULL: return "required pointer is NULL";
    default: break;
  }
  if (code <= QVIT_EHIP) return hipGetErrorString((hipError_t)(QVIT_EHIP - code));
  return "unknown qvit status";
}

const char* qvit_version(void) { return "qvit_hip 0.1 gfx950"; }

static bool qtype_ok(int qtype) {
  const int q = qtype & 0xff;
  return (qtype & ~(0xff | QVIT_QT_FORCE_CAREFUL)) == 0 &&
         (q == QVIT_QT_LINEAR || q == QVIT_QT_NONLINEAR || q == QVIT_QT_ULTRA_ACT);
}

static bool qptrs_ok(int qtype, const float* d, const float* qm, int levels) {
  if ((qtype & 0xff) == QVIT_QT_ULTRA_ACT) return levels >= 1 && levels <= 127;
  return d != nullptr && qm != nullptr;
}

int qvit_quantize_act_i8(const float* x, int64_t rows, int64_t cols, int64_t ldx, int qtype,
                         const float* d_quant, const float* q_m, const float* t_quant, int levels,
                         int8_t* codes, int64_t ldc, int64_t kpad, hipStream_t stream) {
  if (!x || !codes) return QVIT_ENULL;
  if (!qtype_ok(qtype) || !qptrs_ok(qtype, d_quant, q_m, levels)) return QVIT_EINVAL;
  if (rows < 0 || cols < 0 || ldx < cols || kpad < cols || kpad % 16 || ldc < kpad) return QVIT_EINVAL;
  if ((ldc % 16) || (((uintptr_t)codes) & 15)) return QVIT_EALIGN;
  if (rows == 0 || kpad == 0) return QVIT_OK;
  const int64_t work = rows * (kpad / 16);
  hipLaunchKernelGGL(quantize_act_kernel, dim3(grid_for(work, kThreads)), dim3(kThreads), 0, stream,
                     x, rows, cols, ldx, qtype, d_quant, q_m, t_quant, levels, codes, ldc, kpad);
  return qvit_hip_status(hipGetLastError());
}

int qvit_fake_quant_f32(const float* x, int64_t n, int qtype, const float* d_quant,
                        const float* q_m, const float* t_quant, int levels, float* y,
                        hipStream_t stream) {
  if (!x || !y) return QVIT_ENULL;
  if (!qtype_ok(qtype) || !qptrs_ok(qtype, d_quant, q_m, levels)) return QVIT_EINVAL;
  if (n < 0) return QVIT_EINVAL;
  if (n == 0) return QVIT_OK;
  hipLaunchKernelGGL(fake_quant_kernel, dim3(grid_for(n, kThreads)), dim3(kThreads), 0, stream, x,
                     n, qtype, d_quant, q_m, t_quant, levels, y);
  return qvit_hip_status(hipGetLastError());
}

int qvit_gelu_f32(const float* x, int64_t n, float* y, hipStream_t stream) {
  if (!x || !y) return QVIT_ENULL;
  if (n < 0) return QVIT_EINVAL;
  if (n == 0) return QVIT_OK;
  hipLaunchKernelGGL(gelu_kernel, dim3(grid_for(n, kThreads)), dim3(kThreads), 0, stream, x, n, y);
  return qvit_hip_status(hipGetLastError());
}

int qvit_pack_weight(const float* w, int64_t n, int64_t k, int64_t ldw, int qtype,
                     const float* d_quant, const float* q_m, const float* t_quant, int wfmt,
                     void* packed, int64_t npad, int64_t kpad, int32_t* overflow,
                     hipStream_t stream) {
  if (!w || !packed) return QVIT_ENULL;
  const int q = qtype & 0xff;
  if (!qtype_ok(qtype) || q == QVIT_QT_ULTRA_ACT || !d_quant || !q_m) return QVIT_EINVAL;
  if (wfmt != QVIT_W4 && wfmt != QVIT_W8) return QVIT_EINVAL;
  if (n <= 0 || k <= 0 || ldw < k || npad < n || kpad < k) return QVIT_EINVAL;
  if (npad % QVIT_TILE_N || kpad % QVIT_TILE_K) return QVIT_EINVAL;
  if (((uintptr_t)packed) & 15) return QVIT_EALIGN;
  const int64_t work = npad * (kpad / 8);
  if (wfmt == QVIT_W4) {
    hipLaunchKernelGGL(pack_weight_kernel<QVIT_W4>, dim3(grid_for(work, kThreads)), dim3(kThreads),
                       0, stream, w, n, k, ldw, qtype, d_quant, q_m, t_quant, packed, npad, kpad,
                       overflow);
  } else {
    hipLaunchKernelGGL(pack_weight_kernel<QVIT_W8>, dim3(grid_for(work, kThreads)), dim3(kThreads),
                       0, stream, w, n, k, ldw, qtype, d_quant, q_m, t_quant, packed, npad, kpad,
                       overflow);
  }
  return qvit_hip_status(hipGetLastError());
}

int qvit_pad_bias(const float* bias, int64_t n, float* out, int64_t npad, hipStream_t stream) {
  if (!out) return QVIT_ENULL;
  if (n < 0 || npad < n) return QVIT_EINVAL;
  if (npad == 0) return QVIT_OK;
  hipLaunchKernelGGL(pad_bias_kernel, dim3(grid_for(npad, kThreads)), dim3(kThreads), 0, stream,
                     bias, n, out, npad);
  return qvit_hip_status(hipGetLastError());
}

int qvit_im2col_quant_i8(const float* x, int64_t B, int64_t C, int64_t H, int64_t W, int kh,
                         int kw, int sh, int sw, int ph, int pw, int dh, int dw, int qtype,
                         const float* d_quant, const float* q_m, const float* t_quant, int levels,
                         int8_t* codes, int64_t ldc, int64_t kpad, hipStream_t stream) {
  if (!x || !codes) return QVIT_ENULL;
  if (!qtype_ok(qtype) || !qptrs_ok(qtype, d_quant, q_m, levels)) return QVIT_EINVAL;
  if (B < 0 || C <= 0 || H <= 0 || W <= 0 || kh <= 0 || kw <= 0 || sh <= 0 || sw <= 0 || ph < 0 ||
      pw < 0 || dh <= 0 || dw <= 0)
    return QVIT_EINVAL;
  const int64_t OH = (H + 2 * ph - (int64_t)dh * (kh - 1) - 1) / sh + 1;
  const int64_t OW = (W + 2 * pw - (int64_t)dw * (kw - 1) - 1) / sw + 1;
  const int64_t K = C * kh * kw;
  if (OH <= 0 || OW <= 0 || kpad < K || kpad % 16 || ldc < kpad) return QVIT_EINVAL;
  if ((ldc % 16) || (((uintptr_t)codes) & 15)) return QVIT_EALIGN;
  if (B == 0) return QVIT_OK;
  const int64_t work = B * OH * OW * (kpad / 16);
  const int64_t lim = (int64_t)INT32_MAX - 2 * (int64_t)256 * 16 * kThreads;  // headroom for the grid stride
  if (work < lim && B * C * H * W < lim && B * OH * OW * ldc < lim)
    hipLaunchKernelGGL(im2col_quant_kernel<int>, dim3(grid_for(work, kThreads)), dim3(kThreads), 0, stream,
                       x, B, C, H, W, kh, kw, sh, sw, ph, pw, dh, dw, OH, OW, qtype, d_quant, q_m,
                       t_quant, levels, codes, ldc, kpad);
  else
    hipLaunchKernelGGL(im2col_quant_kernel<int64_t>, dim3(grid_for(work, kThreads)), dim3(kThreads), 0, stream,
                       x, B, C, H, W, kh, kw, sh, sw, ph, pw, dh, dw, OH, OW, qtype, d_quant, q_m,
                       t_quant, levels, codes, ldc, kpad);
  return qvit_hip_status(hipGetLastError());
}

int qvit_layernorm_quant_i8(const float* x, int64_t rows, int64_t cols, int64_t ldx,
                            const float* gamma, const float* beta, float eps, int qtype,
                            const float* d_quant, const float* q_m, const float* t_quant,
                            int levels, int8_t* codes, int64_t ldc, int64_t kpad,
                            const void* code_table, hipStream_t stream) {
  if (!x || !codes) return QVIT_ENULL;
  if (code_table && (((uintptr_t)code_table) & 15)) return QVIT_EALIGN;
  if (!qtype_ok(qtype) || !qptrs_ok(qtype, d_quant, q_m, levels)) return QVIT_EINVAL;
  if (rows < 0 || cols <= 0 || ldx < cols || kpad < cols || ldc < kpad) return QVIT_EINVAL;
  if (((ldc & 3) != 0) || (((uintptr_t)codes) & 3)) return QVIT_EALIGN;
  if (rows == 0) return QVIT_OK;
  const bool reg = ((cols & 3) == 0) && ((ldx & 3) == 0) && ((((uintptr_t)x) & 15) == 0) &&
                   (!gamma || (((uintptr_t)gamma) & 15) == 0) && (!beta || (((uintptr_t)beta) & 15) == 0);
  const int nv = (int)((cols + 255) / 256);
  const dim3 grid((unsigned)((rows + 3) / 4));
  if (reg && nv <= 4) {  // persistent: as many workgroups as are co-resident, the table read once per workgroup
    static const int cus = [] {
      int dev = 0, n = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
        n = 256;
      return n;
    }();
    // workgroups per CU that are resident together (registers bound it: 5 at NV = 3); a grid past that
    // leaves a second, partly filled round of workgroups behind the first
    auto resident = [](const void* fn) {
      int n = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, kThreads, 0) != hipSuccess || n <= 0) n = 4;
      return std::min(n, 8);
    };
    const int8_t* tab = reinterpret_cast<const int8_t*>(code_table);
#define QVIT_LN_P(NV)                                                                                               \
  do {                                                                                                              \
    static const int per_cu = resident(reinterpret_cast<const void*>(&layernorm_quant_persist_kernel<NV>));         \
    const int64_t pg = std::min<int64_t>((rows + 3) / 4, (int64_t)per_cu * cus);                                    \
    hipLaunchKernelGGL(layernorm_quant_persist_kernel<NV>, dim3((unsigned)pg), dim3(kThreads), 0, stream, x, rows, \
                       cols, ldx, gamma, beta, eps, qtype, d_quant, q_m, t_quant, levels, codes, ldc, kpad, tab);   \
  } while (0)
    if (nv <= 1) QVIT_LN_P(1);
    else if (nv <= 2) QVIT_LN_P(2);
    else if (nv <= 3) QVIT_LN_P(3);
    else QVIT_LN_P(4);
#undef QVIT_LN_P
    return qvit_hip_status(hipGetLastError());
  }
#define QVIT_LN_REG(NV)                                                                                   \
  hipLaunchKernelGGL(layernorm_quant_reg_kernel<NV>, grid, dim3(kThreads), 0, stream, x, rows, cols, ldx, \
                     gamma, beta, eps, qtype, d_quant, q_m, t_quant, levels, codes, ldc, kpad)
  if (reg && nv <= 1) QVIT_LN_REG(1);
  else if (reg && nv <= 2) QVIT_LN_REG(2);
  else if (reg && nv <= 3) QVIT_LN_REG(3);
  else if (reg && nv <= 4) QVIT_LN_REG(4);
  else if (reg && nv <= 8) QVIT_LN_REG(8);
  else
    hipLaunchKernelGGL(layernorm_quant_kernel, dim3(grid_for(rows * 64, kThreads)), dim3(kThreads), 0, stream, x,
                       rows, cols, ldx, gamma, beta, eps, qtype, d_quant, q_m, t_quant, levels, codes, ldc, kpad);
#undef QVIT_LN_REG
  return qvit_hip_status(hipGetLastError());
}

int qvit_layernorm_quant_i8_t32(const float* x, int64_t rows, int64_t cols, int64_t ldx, const float* gamma,
                                const float* beta, float eps, int qtype, const float* d_quant, const float* q_m,
                                const float* t_quant, int levels, int8_t* codes, int64_t kpad, const void* code_table,
                                hipStream_t stream) {
  if (!x || !codes) return QVIT_ENULL;
  if (code_table && (((uintptr_t)code_table) & 15)) return QVIT_EALIGN;
  if (!qtype_ok(qtype) || !qptrs_ok(qtype, d_quant, q_m, levels)) return QVIT_EINVAL;
  if (rows < 0 || cols <= 0 || cols > 1024 || (cols & 3) || ldx < cols || kpad < cols || (kpad & 63)) return QVIT_EINVAL;
  if ((ldx & 3) || (((uintptr_t)x) & 15) || (gamma && (((uintptr_t)gamma) & 15)) || (beta && (((uintptr_t)beta) & 15)) ||
      (((uintptr_t)codes) & 15))
    return QVIT_EALIGN;
  if (rows == 0) return QVIT_OK;
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                hipSuccess || n <= 0)
      n = 256;
    return n;
  }();
  auto resident = [](const void* fn) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, kThreads, 0) != hipSuccess || n <= 0) n = 4;
    return std::min(n, 8);
  };
  const int8_t* tab = reinterpret_cast<const int8_t*>(code_table);
  const int nv = (int)((cols + 255) / 256);
#define QVIT_LN_T(NV)                                                                                             \
  do {                                                                                                            \
    static const int per_cu = resident(reinterpret_cast<const void*>(&layernorm_quant_persist_kernel<NV, true>)); \
    const int64_t pg = std::min<int64_t>((rows + 3) / 4, (int64_t)per_cu * cus);                                  \
    hipLaunchKernelGGL((layernorm_quant_persist_kernel<NV, true>), dim3((unsigned)pg), dim3(kThreads), 0, stream,  \
                       x, rows, cols, ldx, gamma, beta, eps, qtype, d_quant, q_m, t_quant, levels, codes, kpad,    \
                       kpad, tab);                                                                                \
  } while (0)
  if (nv <= 1) QVIT_LN_T(1);
  else if (nv <= 2) QVIT_LN_T(2);
  else if (nv <= 3) QVIT_LN_T(3);
  else QVIT_LN_T(4);
#undef QVIT_LN_T
  return qvit_hip_status(hipGetLastError());
}

}  // extern "C"
