// Quantized contraction for QuantizeLinear / QuantizeConv2d (quant_layers.py:495-499,575-587):
//   C[m, n] = epilogue( sum_k A[m, k] * W[n, k] ),  A = int8 activation codes, W = int4/int8 weight
//   codes, exact int32 accumulation on v_mfma_i32_16x16x64_i8 (gfx950).
//
// Geometry (one workgroup = 256 threads = 4 waves):
//   block tile 128 (n) x 128 (m), BK = 128 k per stage, two LDS stages (64 KiB) -> 2 blocks / CU.
//   Waves form 2 (n) x 2 (m); each wave owns 64 n x 64 m = 4 x 4 MFMA tiles of 16 x 16.
//   MFMA operand "A" (16 rows) = weights, operand "B" (16 cols) = activations, so the
//   accumulator lane holds 4 consecutive weight rows of one activation row; the packer's row
//   permutation (qvit_pack_weight) turns the 4 x 4 repeats into 16 consecutive output features.
// Staging: activations and packed weights are register-staged (global_load_dwordx4) one stage
//   ahead; int4 weights are sign-extended to int8 on the way into LDS (once per block, shared
//   by both waves that read them). LDS rows are 128 B with the 16-B chunk index XOR-swizzled by
//   (row >> 1) & 7, which makes the ds_read_b128 fragment reads conflict-free.
// Grid: one block per output tile, blockIdx remapped so consecutive tiles (same activation
//   panel, different weight panels) land on the same XCD / L2.
#include "qvit_common.h"

namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

constexpr int BN = 128;      // weight rows per block
constexpr int BM = 128;      // activation rows per block
constexpr int BK = 128;      // k per stage (bytes of int8 per LDS row)
constexpr int NT = 256;      // threads per block
constexpr int TILE_BYTES = BN * BK;  // 16 KiB per operand per stage

QVIT_DEV uint32_t sext4_lo(uint32_t p) {
  const uint32_t x = p & 0x0F0F0F0Fu;
  return ((x ^ 0x08080808u) + 0x78787878u) ^ 0x80808080u;
}
QVIT_DEV uint32_t sext4_hi(uint32_t p) {
  const uint32_t x = (p >> 4) & 0x0F0F0F0Fu;
  return ((x ^ 0x08080808u) + 0x78787878u) ^ 0x80808080u;
}

// byte offset of 16-byte chunk c of LDS row `row`
QVIT_DEV int lds_off(int row, int c) { return row * BK + ((c ^ ((row >> 1) & 7)) << 4); }

struct EpiArgs {
  const float* d_act;
  const float* d_wt;
  const float* bias;
  int out_qtype;
  const float* out_d;
  const float* out_qm;
  const float* out_t;
  int out_levels;
};

template <int WFMT, int EPI>
__global__ __launch_bounds__(NT, 2) void gemm_kernel(const int8_t* __restrict__ A, int M, int K,
                                                     int64_t lda, const void* __restrict__ Wp,
                                                     int N, int npad, void* __restrict__ C,
                                                     int64_t ldc, EpiArgs ep) {
  __shared__ __attribute__((aligned(16))) int8_t smem[2 * 2 * TILE_BYTES];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wn = wave & 1;   // weight-row half of the tile
  const int wm = wave >> 1;  // activation-row half of the tile

  // ---- tile assignment with a bijective XCD remap ----------------------------------------
  const int nb_n = npad / BN;
  const int nb_m = (M + BM - 1) / BM;
  const int nblk = nb_n * nb_m;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nblk >> 3, r8 = nblk & 7;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tile_n = lid % nb_n;
  const int tile_m = lid / nb_n;
  const int n0 = tile_n * BN;
  const int m0 = tile_m * BM;

  // ---- global -> register staging addresses ------------------------------------------------
  // activations: 4 x 16 B per thread; row = (tid >> 3) + 32 i, chunk = tid & 7
  const int xa_c = tid & 7;
  const int8_t* xsrc[4];
  int xdst[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (tid >> 3) + 32 * i;
    int gm = m0 + row;
    gm = gm < M ? gm : M - 1;  // clamp the tail: loaded, never stored
    xsrc[i] = A + (int64_t)gm * lda + xa_c * 16;
    xdst[i] = lds_off(row, xa_c);
  }
  // weights
  constexpr int WLOADS = (WFMT == QVIT_W4) ? 2 : 4;
  const int8_t* wsrc[WLOADS];
  int wdst0[WLOADS], wdst1[WLOADS];
  const int64_t wrow_bytes = (WFMT == QVIT_W4) ? (int64_t)K / 2 : (int64_t)K;
#pragma unroll
  for (int i = 0; i < WLOADS; ++i) {
    if (WFMT == QVIT_W4) {
      const int id = tid + NT * i;
      const int row = id >> 2, c4 = id & 3;
      wsrc[i] = reinterpret_cast<const int8_t*>(Wp) + (int64_t)(n0 + row) * wrow_bytes + c4 * 16;
      wdst0[i] = lds_off(row, 2 * c4);
      wdst1[i] = lds_off(row, 2 * c4 + 1);
    } else {
      const int row = (tid >> 3) + 32 * i;
      wsrc[i] = reinterpret_cast<const int8_t*>(Wp) + (int64_t)(n0 + row) * wrow_bytes + xa_c * 16;
      wdst0[i] = lds_off(row, xa_c);
      wdst1[i] = 0;
    }
  }

  v4u xr[4];
  v4u wr[WLOADS];

  auto gload = [&](int kt) {
    const int64_t kx = (int64_t)kt * BK;
    const int64_t kw = (WFMT == QVIT_W4) ? kx / 2 : kx;
#pragma unroll
    for (int i = 0; i < 4; ++i) xr[i] = *reinterpret_cast<const v4u*>(xsrc[i] + kx);
#pragma unroll
    for (int i = 0; i < WLOADS; ++i) wr[i] = *reinterpret_cast<const v4u*>(wsrc[i] + kw);
  };
  auto lstore = [&](int stage) {
    int8_t* sx = smem + stage * 2 * TILE_BYTES;
    int8_t* sw = sx + TILE_BYTES;
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<v4u*>(sx + xdst[i]) = xr[i];
#pragma unroll
    for (int i = 0; i < WLOADS; ++i) {
      if (WFMT == QVIT_W4) {
        const v4u p = wr[i];
        *reinterpret_cast<v4u*>(sw + wdst0[i]) =
            v4u{sext4_lo(p.x), sext4_hi(p.x), sext4_lo(p.y), sext4_hi(p.y)};
        *reinterpret_cast<v4u*>(sw + wdst1[i]) =
            v4u{sext4_lo(p.z), sext4_hi(p.z), sext4_lo(p.w), sext4_hi(p.w)};
      } else {
        *reinterpret_cast<v4u*>(sw + wdst0[i]) = wr[i];
      }
    }
  };

  v4i acc[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int s = 0; s < 4; ++s) acc[r][s] = v4i{0, 0, 0, 0};

  // fragment read offsets: row = base + 16 r + (lane & 15), chunk = 4 kk + (lane >> 4)
  const int fr = lane & 15;
  const int fq = lane >> 4;
  const int wrow0 = wn * 64 + fr;
  const int xrow0 = wm * 64 + fr;

  const int nk = K / BK;
  auto compute = [&](int cur) {
    const int8_t* sx = smem + cur * 2 * TILE_BYTES;
    const int8_t* sw = sx + TILE_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      v4i wf[4], xf[4];
#pragma unroll
      for (int r = 0; r < 4; ++r)
        wf[r] = *reinterpret_cast<const v4i*>(sw + lds_off(wrow0 + 16 * r, 4 * kk + fq));
#pragma unroll
      for (int s = 0; s < 4; ++s)
        xf[s] = *reinterpret_cast<const v4i*>(sx + lds_off(xrow0 + 16 * s, 4 * kk + fq));
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int s = 0; s < 4; ++s)
          acc[r][s] = __builtin_amdgcn_mfma_i32_16x16x64_i8(wf[r], xf[s], acc[r][s], 0, 0, 0);
    }
  };
  gload(0);
  lstore(0);
  __syncthreads();
  // steady state: prefetch stage kt+1 into registers, compute stage kt, write kt+1 to LDS
  for (int kt = 0; kt < nk - 1; ++kt) {
    const int cur = kt & 1;
    gload(kt + 1);
    compute(cur);
    lstore(cur ^ 1);
    __syncthreads();
  }
  compute((nk - 1) & 1);

  // ---- epilogue -------------------------------------------------------------------------------
  // acc[r][s][j] is C[m = m0 + 64 wm + 16 s + fr][n = n0 + 64 wn + 16 fq + 4 r + j]
  const int nbase = n0 + wn * 64 + 16 * fq;
  const bool nfull = nbase + 16 <= N;
  if (EPI == QVIT_EPI_I32) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int m = m0 + wm * 64 + 16 * s + fr;
      if (m >= M) continue;
      int32_t* dst = reinterpret_cast<int32_t*>(C) + (int64_t)m * ldc + nbase;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (nfull) {
          *reinterpret_cast<v4i*>(dst + 4 * r) = acc[r][s];
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (nbase + 4 * r + j < N) dst[4 * r + j] = acc[r][s][j];
        }
      }
    }
    return;
  }

  const float alpha = (*ep.d_act) * (*ep.d_wt);
  float bv[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) bv[i] = 0.f;
  if (ep.bias != nullptr) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float4 b4 = *reinterpret_cast<const float4*>(ep.bias + nbase + 4 * r);
      bv[4 * r + 0] = b4.x; bv[4 * r + 1] = b4.y; bv[4 * r + 2] = b4.z; bv[4 * r + 3] = b4.w;
    }
  }

  if (EPI == QVIT_EPI_F32 || EPI == QVIT_EPI_F32_RESID) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int m = m0 + wm * 64 + 16 * s + fr;
      if (m >= M) continue;
      float* dst = reinterpret_cast<float*>(C) + (int64_t)m * ldc + nbase;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = alpha * (float)acc[r][s][j] + bv[4 * r + j];
        if (nfull) {
          float4* d4 = reinterpret_cast<float4*>(dst + 4 * r);
          if (EPI == QVIT_EPI_F32_RESID) {
            const float4 old = *d4;
            o[0] += old.x; o[1] += old.y; o[2] += old.z; o[3] += old.w;
          }
          *d4 = make_float4(o[0], o[1], o[2], o[3]);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (nbase + 4 * r + j < N) {
              if (EPI == QVIT_EPI_F32_RESID) dst[4 * r + j] += o[j];
              else dst[4 * r + j] = o[j];
            }
          }
        }
      }
    }
    return;
  }

  // int8-code epilogues: the next layer's quantizer applied to (optionally GELU of) the output
  const QParams qp = load_qparams(ep.out_qtype, ep.out_d, ep.out_qm, ep.out_t, ep.out_levels);
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int m = m0 + wm * 64 + 16 * s + fr;
    if (m >= M) continue;
    int8_t* dst = reinterpret_cast<int8_t*>(C) + (int64_t)m * ldc + nbase;
    uint32_t words[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      uint32_t wv = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float v = alpha * (float)acc[r][s][j] + bv[4 * r + j];
        if (EPI == QVIT_EPI_I8_GELU) v = gelu_erf(v);
        wv |= ((uint32_t)(uint8_t)to_i8_sat(quant_code(v, qp))) << (8 * j);
      }
      words[r] = wv;
    }
    if (nfull) {
      *reinterpret_cast<uint4*>(dst) = make_uint4(words[0], words[1], words[2], words[3]);
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (nbase + i < N) dst[i] = (int8_t)((words[i >> 2] >> (8 * (i & 3))) & 0xff);
    }
  }
}

template <int WFMT, int EPI>
int launch(const int8_t* A, int64_t M, int64_t K, int64_t lda, const void* Wp, int64_t N,
           int64_t npad, void* C, int64_t ldc, const EpiArgs& ep, hipStream_t stream) {
  const int64_t nblk = (npad / BN) * ((M + BM - 1) / BM);
  hipLaunchKernelGGL((gemm_kernel<WFMT, EPI>), dim3((unsigned)nblk), dim3(NT), 0, stream, A, (int)M,
                     (int)K, lda, Wp, (int)N, (int)npad, C, ldc, ep);
  return qvit_hip_status(hipGetLastError());
}

template <int WFMT>
int dispatch_epi(int epilogue, const int8_t* A, int64_t M, int64_t K, int64_t lda, const void* Wp,
                 int64_t N, int64_t npad, void* C, int64_t ldc, const EpiArgs& ep,
                 hipStream_t stream) {
  switch (epilogue) {
    case QVIT_EPI_F32: return launch<WFMT, QVIT_EPI_F32>(A, M, K, lda, Wp, N, npad, C, ldc, ep, stream);
    case QVIT_EPI_F32_RESID:
      return launch<WFMT, QVIT_EPI_F32_RESID>(A, M, K, lda, Wp, N, npad, C, ldc, ep, stream);
    case QVIT_EPI_I8_GELU:
      return launch<WFMT, QVIT_EPI_I8_GELU>(A, M, K, lda, Wp, N, npad, C, ldc, ep, stream);
    case QVIT_EPI_I8: return launch<WFMT, QVIT_EPI_I8>(A, M, K, lda, Wp, N, npad, C, ldc, ep, stream);
    case QVIT_EPI_I32: return launch<WFMT, QVIT_EPI_I32>(A, M, K, lda, Wp, N, npad, C, ldc, ep, stream);
    default: return QVIT_EINVAL;
  }
}

}  // namespace

extern "C" int qvit_gemm(const int8_t* A, int64_t M, int64_t K, int64_t lda, const void* Wp,
                         int wfmt, int64_t N, int64_t npad, const float* d_act, const float* d_wt,
                         const float* bias, int epilogue, void* C, int64_t ldc, int out_qtype,
                         const float* out_d, const float* out_qm, const float* out_t,
                         int out_levels, hipStream_t stream) {
  if (!A || !Wp || !C) return QVIT_ENULL;
  if (wfmt != QVIT_W4 && wfmt != QVIT_W8) return QVIT_EINVAL;
  if (M < 0 || K <= 0 || K % BK || lda < K || N <= 0 || npad < N || npad % BN) return QVIT_EINVAL;
  if (M > INT32_MAX / 2 || npad > INT32_MAX / 2 || K > (1 << 24)) return QVIT_EINVAL;
  if ((lda % 16) || (((uintptr_t)A) & 15) || (((uintptr_t)Wp) & 15)) return QVIT_EALIGN;
  const bool i8out = epilogue == QVIT_EPI_I8 || epilogue == QVIT_EPI_I8_GELU;
  if (epilogue < QVIT_EPI_F32 || epilogue > QVIT_EPI_I32) return QVIT_EINVAL;
  if (ldc < N) return QVIT_EINVAL;
  if (i8out) {
    if ((ldc % 16) || (((uintptr_t)C) & 15)) return QVIT_EALIGN;
    const int q = out_qtype & 0xff;
    if (q != QVIT_QT_LINEAR && q != QVIT_QT_NONLINEAR && q != QVIT_QT_ULTRA_ACT) return QVIT_EINVAL;
    if (q == QVIT_QT_ULTRA_ACT ? (out_levels < 1 || out_levels > 127) : (!out_d || !out_qm))
      return QVIT_EINVAL;
  } else {
    if ((ldc % 4) || (((uintptr_t)C) & 15)) return QVIT_EALIGN;
  }
  if (epilogue != QVIT_EPI_I32 && (!d_act || !d_wt)) return QVIT_ENULL;
  if (bias && (((uintptr_t)bias) & 15)) return QVIT_EALIGN;
  if (M == 0) return QVIT_OK;
  EpiArgs ep{d_act, d_wt, bias, out_qtype, out_d, out_qm, out_t, out_levels};
  if (wfmt == QVIT_W4) return dispatch_epi<QVIT_W4>(epilogue, A, M, K, lda, Wp, N, npad, C, ldc, ep, stream);
  return dispatch_epi<QVIT_W8>(epilogue, A, M, K, lda, Wp, N, npad, C, ldc, ep, stream);
}
