// Fused qkv projection + attention core of Attention.forward (vit_model.py:126-152) for the fused block:
//   qkv = QuantizeLinear(x_codes)  ->  softmax(q k^T * scale) v  ->  proj's activation quantizer
// with q, k, v never leaving the chip. One persistent workgroup (8 waves) per CU walks (image, head)
// units; per unit:
//   1. projection: wave w computes the 192 q|k|v features of its token tiles {w', w'+8} (w' = w rotated
//      by unit) on v_mfma_i32_16x16x64_i8: activation codes come straight from global into registers
//      (two k-steps ahead), the head's three 64-row weight groups (pre-tiled int4 images of the qkv
//      GEMM's weights) through a 3-slot LDS ring (register-staged, one barrier per k-step);
//   2. epilogue: v = (d_a d_w acc + bias) * in_scale split into fp16 hi/lo exactly as
//      qvit_gemm_qkv_split does; q stays in registers as the wave's own S^T B-operand fragments (the
//      contraction runs over the head dims in the order the accumulators hold them: lane group g owns
//      dims 16g .. 16g+15), k and v go to resident LDS images (208 rows, XOR-swizzled);
//   3. attention: the 7 key blocks of 32 with no barrier (K/V resident), online softmax, P·V, and the
//      output quantizer through its code table (attn_common.h, same arithmetic as qvit_attention_split
//      except the order of the dims inside each q·k sum).
// The next unit's first two k-steps are loaded while the current unit's attention runs. N <= 208.
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
constexpr int WSLOT = 3 * 4096;           // q, k, v 64-row weight groups of one k-step, unpacked to int8
constexpr int WRING = 3;
#ifndef QVIT_QA_SKIP
#define QVIT_QA_SKIP 1
#endif
#ifndef QVIT_QA_PAIR
#define QVIT_QA_PAIR 1
#endif
constexpr int TBL = 8192;                 // code table (<= 1022 buckets)
constexpr int BIAS_MAX = 9216;            // fp32 bias of the qkv layer (<= 2304 features: H * 64 <= 768)
constexpr int LDS_TOTAL = KV_BYTES + WRING * WSLOT + TBL + BIAS_MAX;
static_assert(LDS_TOTAL <= 163840, "LDS budget");

QVIT_DEV uint32_t nib16_lo(uint32_t p) { return (p << 4) & 0xF0F0F0F0u; }
QVIT_DEV uint32_t nib16_hi(uint32_t p) { return p & 0xF0F0F0F0u; }
typedef int v4i __attribute__((ext_vector_type(4)));

// NKC: the number of 64-deep k-steps when fixed at compile time (12: K = 768, the ViT-B qkv; ViT-L's
// H * 64 = 1024 exceeds QKV_ATT_MAX_C and takes the split path), which unrolls the projection loop
// completely; 0: K / 64 at run time (other K, e.g. 512 or 1024 with <= 12 heads)
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
  const int total = my_units > 0 ? my_units * nk : 0;
  const int ntile = (N + 15) / 16;
  const int64_t M = (int64_t)B * N;

  // ---- operand stream: global k-step g = j * nk + s; register ring slot = s % 4 (nk % 4 == 0), so the
  // slot of every unrolled step is a compile-time constant and loads stay in flight 3 steps ------------
  v4i xa[4][TPW];   // activation fragments
  v4i wst[4];       // this wave's 1-KiB piece of a weight slot (waves 0..5)
  // per-unit operand sources (this lane's activation rows, this wave's weight piece), computed once per
  // unit; units past the end repeat the last one (its loads are never used)
  struct Src {
    const int8_t* a[TPW];
    const int8_t* w;
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
      sr.a[tt] = A + m * lda + 16 * fq;
    }
    const int p = wave < 6 ? (wave >> 1) : 2;  // weight group (q, k, v); waves 6, 7 load a copy, never written
    const int feat = p * C + 64 * h;
    sr.w = Wp + (int64_t)(feat >> 8) * nk * 8192 + ((feat & 255) >> 6) * 2048 + (wave & 1) * 1024 + 16 * lane;
  };
  // k-step s of a unit: the same three loads on every path, so they stay in flight
  auto load_step = [&](const Src& sr, int s, v4i (&xd)[TPW], v4i& wd) __attribute__((always_inline)) {
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt) xd[tt] = *reinterpret_cast<const v4i*>(sr.a[tt] + 64 * s);
    wd = *reinterpret_cast<const v4i*>(sr.w + (int64_t)s * 8192);
  };
  // the staging wave unpacks its 16 packed bytes (two 8-B fragment chunks) into the 16x-scaled int8 MFMA
  // operands once, at twice the packed offset, so the 8 waves that read a fragment do no unpacking
  auto write_w = [&](int g, const v4i& wd) __attribute__((always_inline)) {
    if (g >= total || wave >= 6) return;
    const v4i u0 = v4i{(int)nib16_lo(wd[0]), (int)nib16_hi(wd[0]), (int)nib16_lo(wd[1]), (int)nib16_hi(wd[1])};
    const v4i u1 = v4i{(int)nib16_lo(wd[2]), (int)nib16_hi(wd[2]), (int)nib16_lo(wd[3]), (int)nib16_hi(wd[3])};
    int8_t* d = wring + (g % WRING) * WSLOT + (wave >> 1) * 4096 + (wave & 1) * 2048 + 32 * lane;
    *reinterpret_cast<v4i*>(d) = u0;
    *reinterpret_cast<v4i*>(d + 16) = u1;
  };
  // weight fragment of row tile r of group p: the GEMM's pre-tiled group image (wn = 0), offsets doubled
  const int woff = 2 * (fr * 32 + ((fq ^ (((fr >> 3) & 1) << 1)) << 3));

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
  load_step(cur, 0, xa[0], wst[0]);
  load_step(cur, 1, xa[1], wst[1]);
  load_step(cur, 2, xa[2], wst[2]);
  write_w(0, wst[0]);
  int g = 0;
  for (int j = 0; j < my_units; ++j) {
    const int unit = ulo + slot + j * team;
    const int b = unit / H, h = unit - b * H;
    const int wr = (wave + unit) & (FW - 1);
    bool tv[TPW];
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt) tv[tt] = wr + FW * tt < ntile;
    const int nt = (tv[0] ? 1 : 0) + (tv[1] ? 1 : 0);

    // ---- 1. projection ---------------------------------------------------------------------------
    v4i acc[TPW][12];
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt)
#pragma unroll
      for (int f = 0; f < 12; ++f) acc[tt][f] = v4i{0, 0, 0, 0};
    // k-step s (ring slot q = s % 4, compile-time after unrolling). The two waves of a SIMD (w, w + 4)
    // take opposite orders around the one barrier per k-step, so that one issues its MFMAs while the
    // other issues its loads and weight staging: waves 0-3 compute first and stage the slot they fill
    // (g + 1) after their MFMAs, waves 4-7 stage first. Either order writes slot g + 1 after barrier
    // g - 1 (its last reader, step g - 2, is done) and before barrier g + 1 (its first read).
    auto issue = [&](int s, int q) __attribute__((always_inline)) {
      if (s + 3 < nk) load_step(cur, s + 3, xa[(q + 3) & 3], wst[(q + 3) & 3]);
      else load_step(nxt, s + 3 - nk, xa[(q + 3) & 3], wst[(q + 3) & 3]);
      sp.mark(5);
      write_w(g + 1, wst[(q + 1) & 3]);
      sp.mark(6);
    };
    // TWO: the wave's second token tile is inside the image (otherwise its MFMAs are skipped: 3 of the 16
    // tiles of N = 197)
    auto mma = [&](auto two, int q) __attribute__((always_inline)) {
      const int8_t* ws = wring + (g % WRING) * WSLOT;
      v4i wfr[12];
#pragma unroll
      for (int f = 0; f < 12; ++f) wfr[f] = *reinterpret_cast<const v4i*>(ws + (f >> 2) * 4096 + woff + (f & 3) * 16 * 64);
#pragma unroll
      for (int f = 0; f < 12; ++f) {
        const v4i wf = wfr[f];
        acc[0][f] = __builtin_amdgcn_mfma_i32_16x16x64_i8(wf, xa[q][0], acc[0][f], 0, 0, 0);
        if (decltype(two)::value) acc[1][f] = __builtin_amdgcn_mfma_i32_16x16x64_i8(wf, xa[q][1], acc[1][f], 0, 0, 0);
      }
      sp.mark(8);
    };
    auto kstep = [&](auto first, auto two, int s, int q) __attribute__((always_inline)) {
      if (!decltype(first)::value) {
        issue(s, q);
        __syncthreads();
        sp.mark(7);
        mma(two, q);
      } else {
        __syncthreads();
        sp.mark(7);
        mma(two, q);
        issue(s, q);
      }
      ++g;
    };
    // with NKC the k-steps of a unit are straight-line code: a loop back-edge carrying the register ring's
    // in-flight loads makes hipcc wait vmcnt(0) at the loop head, draining the prefetch every 4 k-steps
    auto kloop = [&](auto first, auto two) __attribute__((always_inline)) {
      if constexpr (NKC > 0) {
#pragma unroll
        for (int s = 0; s < NKC; s += 4) {
          kstep(first, two, s, 0);
          kstep(first, two, s + 1, 1);
          kstep(first, two, s + 2, 2);
          kstep(first, two, s + 3, 3);
        }
      } else {
        for (int s = 0; s < nk; s += 4) {
          kstep(first, two, s, 0);
          kstep(first, two, s + 1, 1);
          kstep(first, two, s + 2, 2);
          kstep(first, two, s + 3, 3);
        }
      }
    };
    const bool first = QVIT_QA_PAIR && wave < 4;
    if (first && (QVIT_QA_SKIP == 0 || tv[1])) kloop(std::true_type{}, std::true_type{});
    else if (first) kloop(std::true_type{}, std::false_type{});
    else if (QVIT_QA_SKIP == 0 || tv[1]) kloop(std::false_type{}, std::true_type{});
    else kloop(std::false_type{}, std::false_type{});
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
    __syncthreads();  // K / V images complete
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
    if (nt > 0) {
      for (int kb = 0; kb < nkb; ++kb)
        attend<TPW, IMGF, true>(nt, (kb + 1) * KB > N, kv + kb * KB * 128, qh, ql, m, l, o, koffs, voffs, kb * KB + 4 * fq,
                          N, sl2, sp);
    }
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
