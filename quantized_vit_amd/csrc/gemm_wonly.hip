// Weight-only QuantizeLinear.forward (quant_layers.py:495-499 with quant_mode = WEIGHT_ONLY, the reference's
// default mode, quant_model.py:23): quantize_act is the identity (:356-358), so the layer is
//   y = F.linear(x, quantize_weight(W), b) = x @ (d_w k)^T + b,   x fp32, k the int4 / int8 weight codes.
// Here y = (d_w / s) * (x @ (s k)^T) + b on v_mfma_f32_16x16x32_bf16, with the codes read from the packed
// image qvit_pack_weight writes for qvit_gemm (s = 16 for int4: the nibble in the high half of its byte).
// Exactness: x = x1 + x2 + x3 with x1 = x truncated to bf16, x2 = (x - x1) truncated, x3 = x - x1 - x2 (each
// difference is exact in fp32 and x3 has at most 8 significant bits, so x3 is a bf16 exactly); s k has at
// most 7 significant bits, so every product x_i (s k) is exact in fp32 and the three passes sum x k with fp32
// accumulation — an fp32 GEMM of x and k, the order of the K-term sum aside. One multiply by d_w / s (s a
// power of two) and the bias add follow, as in the reference's fp32 F.linear on the fake-quant weight.
//
// Geometry: one workgroup (4 waves) per 64 (x rows) x 256 (weight rows) tile; wave w owns weight rows
// [64 w, 64 w + 64) and all 64 x rows: 4 x 4 MFMA tiles of 16 x 16. K advances in 64-deep stages through
// two LDS buffers: per stage each thread loads 16 fp32 of one x row (4 x 16 B) and its slice of the packed
// weight stage (the GEMM's LDS image, 8 KiB int4 / 16 KiB int8) into registers while the current stage
// computes, then splits the x values into three bf16 planes (rows padded to 144 B: conflict-free
// ds_read_b128 fragment reads) and writes both to the other buffer; one barrier per stage.
// MFMA operands: A = weights (16 rows), B = x (16 rows): lane (fr = l & 15, fq = l >> 4) pairs weight byte b of
// its packed fragment with x column 16 fq + b of the stage (the qvit_gemm pairing), chunk c = bytes 8c .. 8c+7.
// D[n][m]: acc[r][s][j] = y[m0 + 16 s + fr][n0 + 64 w + 16 fq + 4 r + j] (the packed rows are pre-permuted).
// Wider codes (levels beyond int8, e.g. the reference's default num_bits = 16): balanced base-256 digits,
// QVIT_W16 k = 256 h + l (|k| <= 32639), QVIT_W24 k = 65536 a + 256 h + l (|k| < 2^23; 16-bit layers whose
// saturation code is 32768), every digit in [-128, 127], one QVIT_W8 image per digit, most significant first.
// 65536 a, 256 h and l are bf16 exactly, every product with an x term is exact in fp32, the digits' terms stay
// within about |k| (balanced: no cancellation beyond a factor 2), and one accumulator takes them all (three
// MFMAs per x term and digit).
// Convolution (qvit_conv_wonly: weight-only QuantizeConv2d, UltraNet's Conv2d_Q): an implicit GEMM, the x row of
// output pixel m = (b, oy, ox) being its input patch in the weight's flattening order k = (c kh + ky) kw + kx,
// gathered from the NCHW input while the stage loads (zero outside the image and for k >= C kh kw), so no patch
// matrix is ever written; the epilogue stores y straight into the NCHW output (plane n of image b).
// Few tiles (small M, e.g. one image): the K stages are split over `splits` workgroups per tile, each writing
// its raw fp32 partial to a workspace, and wonly_reduce_kernel sums the partials in split order (deterministic)
// and applies d_w / s and the bias.
#include <algorithm>

#include "qvit_common.h"

namespace {

typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef int v4i __attribute__((ext_vector_type(4)));

constexpr int WO_BM = 64;        // x rows per tile
constexpr int WO_BN = 256;       // weight rows per tile (one packed tile_n)
constexpr int WO_BK = 64;        // k per stage
constexpr int WO_PITCH = 144;    // bytes per x-plane row: 64 bf16 + 16 pad
constexpr int WO_PLANE = WO_BM * WO_PITCH;
constexpr int WO_XBYTES = 3 * WO_PLANE;

template <int WFMT>
struct WoGeo {
  static constexpr int WROW = WFMT == QVIT_W4 ? 32 : 64;  // packed bytes per weight row per stage (per image)
  static constexpr int PARTS = WFMT == QVIT_W24 ? 3 : WFMT == QVIT_W16 ? 2 : 1;  // digit images
  static constexpr int WBYTES = WO_BN * WROW;              // one image's stage
  static constexpr int WPER = PARTS * WBYTES / 256 / 16;   // 16-B pieces per thread per stage
  static constexpr int STAGE = WO_XBYTES + PARTS * WBYTES;
  static constexpr int MINB = WFMT == QVIT_W4 ? 2 : 1;
};

QVIT_DEV uint32_t nib16_lo(uint32_t p) { return (p << 4) & 0xF0F0F0F0u; }
QVIT_DEV uint32_t nib16_hi(uint32_t p) { return p & 0xF0F0F0F0u; }
QVIT_DEV uint32_t hi16(float a, float b) {  // bf16 bits of a (low half) and b (high half); both exact bf16 values
  return (__float_as_uint(a) >> 16) | (__float_as_uint(b) & 0xFFFF0000u);
}
// four signed bytes -> four bf16 of mul * byte, exact (mul a power of two)
QVIT_DEV void bytes_bf16(uint32_t d, uint32_t& lo, uint32_t& hi, float mul) {
  const uint32_t u = d ^ 0x80808080u;  // unsigned byte = signed + 128
  const float f0 = ((float)(u & 0xff) - 128.f) * mul, f1 = ((float)((u >> 8) & 0xff) - 128.f) * mul;
  const float f2 = ((float)((u >> 16) & 0xff) - 128.f) * mul, f3 = ((float)(u >> 24) - 128.f) * mul;
  lo = hi16(f0, f1);
  hi = hi16(f2, f3);
}
// convolution geometry (CONV kernels); L = OH OW output pixels per image, kreal = C kh kw
struct WoConv {
  int C, H, W, kh, kw, sh, sw, ph, pw, dh, dw, OW, L, kreal;
};
QVIT_DEV float trunc_bf16(float x) { return __uint_as_float(__float_as_uint(x) & 0xFFFF0000u); }

template <int WFMT, bool CONV>
__global__ __launch_bounds__(256, WoGeo<WFMT>::MINB) void gemm_wonly_kernel(
    const float* __restrict__ X, int M, int K, int64_t ldx, const int8_t* __restrict__ Wp, int N, int npad,
    const float* __restrict__ d_wt, const float* __restrict__ bias, float* __restrict__ Y, int64_t ldy, int splits,
    float* __restrict__ part, const WoConv cg) {
  using G = WoGeo<WFMT>;
  __shared__ __attribute__((aligned(16))) int8_t smem[2 * G::STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;

  // tile: XCD x (blocks x, x + 8, ...) walks a contiguous range, weight tiles fastest, so the tiles of one
  // x panel share an L2
  const int nb_n = npad / WO_BN;
  const int ntiles = nb_n * ((M + WO_BM - 1) / WO_BM);
  int t, sp = 0;
  if (splits > 1) {  // (tile, split) = (b / splits, b % splits)
    t = (int)blockIdx.x / splits;
    sp = (int)blockIdx.x - t * splits;
  } else {
    const int per = (ntiles + 7) >> 3;
    t = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
  }
  if (t >= ntiles) return;
  const int m0 = (t / nb_n) * WO_BM, tn = t % nb_n, n0 = tn * WO_BN;
  const int nk = K / WO_BK;
  const int ks0 = (int)((int64_t)sp * nk / splits), ks1 = (int)((int64_t)(sp + 1) * nk / splits);

  // this thread's loads: x row m0 + (tid >> 2), columns 16 (tid & 3) .. + 15 of the stage; weight pieces
  const int xr = tid >> 2, xq = tid & 3;
  const int xm = (m0 + xr < M) ? m0 + xr : M - 1;  // rows past M: a valid row, never stored
  const float* xsrc = X + (int64_t)xm * ldx + 16 * xq;
  // CONV: this row's image and the input position of its patch's top-left tap
  const float* img = X;
  int iy0 = 0, ix0 = 0;
  if (CONV) {
    const int b = xm / cg.L, p = xm - b * cg.L, oy = p / cg.OW;
    img = X + (int64_t)b * cg.C * cg.H * cg.W;
    iy0 = oy * cg.sh - cg.ph;
    ix0 = (p - oy * cg.OW) * cg.sw - cg.pw;
  }
  // (W16 / W24: piece i from digit image i / WPP, each image npad K bytes)
  constexpr int WPP = G::WPER / G::PARTS;
  const int8_t* wsrc = Wp + (int64_t)tn * nk * G::WBYTES + tid * 16 * WPP;
  const int64_t wpart = (int64_t)npad * K;
  f4 xv[4];
  v4i wv[G::WPER];
  auto load = [&](int kt) __attribute__((always_inline)) {
    if (CONV) {  // the 16 taps k0 .. k0 + 15 of the patch, (c, ky, kx) stepped along
      const int k0 = kt * WO_BK + 16 * xq, khw = cg.kh * cg.kw;
      int c = k0 / khw, r = k0 - c * khw, ky = r / cg.kw, kx = r - ky * cg.kw;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int iy = iy0 + ky * cg.dh, ix = ix0 + kx * cg.dw;
        float v = 0.f;
        if (k0 + i < cg.kreal && (unsigned)iy < (unsigned)cg.H && (unsigned)ix < (unsigned)cg.W)
          v = img[((int64_t)c * cg.H + iy) * cg.W + ix];
        xv[i >> 2][i & 3] = v;
        if (++kx == cg.kw) {
          kx = 0;
          if (++ky == cg.kh) {
            ky = 0;
            ++c;
          }
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) xv[i] = *reinterpret_cast<const f4*>(xsrc + kt * WO_BK + 4 * i);
    }
#pragma unroll
    for (int i = 0; i < G::WPER; ++i)
      wv[i] = *reinterpret_cast<const v4i*>(wsrc + (i / WPP) * wpart + (int64_t)kt * G::WBYTES + 16 * (i % WPP));
  };
  // split and store into buffer b: plane p row xr, bf16 columns 16 xq .. + 15 (32 B)
  auto store = [&](int b) __attribute__((always_inline)) {
    int8_t* base = smem + b * G::STAGE;
    uint32_t p1[8], p2[8], p3[8];
#pragma unroll
    for (int e = 0; e < 16; e += 2) {
      const float a = xv[e >> 2][e & 3], c = xv[(e + 1) >> 2][(e + 1) & 3];
      const float a1 = trunc_bf16(a), c1 = trunc_bf16(c);
      const float ar = a - a1, cr = c - c1;  // exact
      const float a2 = trunc_bf16(ar), c2 = trunc_bf16(cr);
      const float a3 = ar - a2, c3 = cr - c2;  // exact, <= 8 significant bits
      p1[e >> 1] = hi16(a1, c1);
      p2[e >> 1] = hi16(a2, c2);
      p3[e >> 1] = hi16(a3, c3);
    }
    int8_t* d = base + xr * WO_PITCH + 32 * xq;
    *reinterpret_cast<uint4*>(d) = make_uint4(p1[0], p1[1], p1[2], p1[3]);
    *reinterpret_cast<uint4*>(d + 16) = make_uint4(p1[4], p1[5], p1[6], p1[7]);
    *reinterpret_cast<uint4*>(d + WO_PLANE) = make_uint4(p2[0], p2[1], p2[2], p2[3]);
    *reinterpret_cast<uint4*>(d + WO_PLANE + 16) = make_uint4(p2[4], p2[5], p2[6], p2[7]);
    *reinterpret_cast<uint4*>(d + 2 * WO_PLANE) = make_uint4(p3[0], p3[1], p3[2], p3[3]);
    *reinterpret_cast<uint4*>(d + 2 * WO_PLANE + 16) = make_uint4(p3[4], p3[5], p3[6], p3[7]);
#pragma unroll
    for (int i = 0; i < G::WPER; ++i)
      *reinterpret_cast<v4i*>(base + WO_XBYTES + (i / WPP) * G::WBYTES + tid * 16 * WPP + 16 * (i % WPP)) = wv[i];
  };

  // fragment offsets: weights as qvit_gemm's read_frags (XOR-swizzled packed image), x planes row 16 s + fr
  const int woff = (WFMT == QVIT_W4) ? (64 * wave + fr) * G::WROW + ((fq ^ (((fr >> 3) & 1) << 1)) << 3)
                                     : (64 * wave + fr) * G::WROW + ((fq ^ (((fr >> 2) & 1) << 1)) << 4);
  const int xoff = fr * WO_PITCH + 32 * fq;

  f4 acc[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int s = 0; s < 4; ++s) acc[r][s] = f4{0.f, 0.f, 0.f, 0.f};

  load(ks0);
  store(0);
  __syncthreads();
  for (int kt = ks0; kt < ks1; ++kt) {
    const int cur = (kt - ks0) & 1;
    if (kt + 1 < ks1) load(kt + 1);  // lands while this stage computes
    const int8_t* base = smem + cur * G::STAGE;
    // the wave's weight fragments of this stage as bf16: wb[q][r][c] = bytes 8c .. 8c + 7 of fragment r of
    // digit image q, times 256^(PARTS - 1 - q)
    bf8 wb[G::PARTS][4][2];
#pragma unroll
    for (int q = 0; q < G::PARTS; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int8_t* wp = base + WO_XBYTES + q * G::WBYTES + woff + r * 16 * G::WROW;
        v4i wf;
        if (WFMT == QVIT_W4) {
          const uint2 p = *reinterpret_cast<const uint2*>(wp);
          wf = v4i{(int)nib16_lo(p.x), (int)nib16_hi(p.x), (int)nib16_lo(p.y), (int)nib16_hi(p.y)};
        } else {
          wf = *reinterpret_cast<const v4i*>(wp);
        }
        uint32_t h[8];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          bytes_bf16((uint32_t)wf[e], h[2 * e], h[2 * e + 1], G::PARTS - 1 - q == 2 ? 65536.f : G::PARTS - 1 - q == 1 ? 256.f : 1.f);
        wb[q][r][0] = __builtin_bit_cast(bf8, make_uint4(h[0], h[1], h[2], h[3]));
        wb[q][r][1] = __builtin_bit_cast(bf8, make_uint4(h[4], h[5], h[6], h[7]));
      }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int8_t* xp = base + xoff + s * 16 * WO_PITCH + 16 * c;
        bf8 xs[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) xs[p] = *reinterpret_cast<const bf8*>(xp + p * WO_PLANE);
#pragma unroll
        for (int q = 0; q < G::PARTS; ++q)
#pragma unroll
          for (int p = 0; p < 3; ++p)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              acc[r][s] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[q][r][c], xs[p], acc[r][s], 0, 0, 0);
      }
    }
    if (kt + 1 < ks1) store(cur ^ 1);  // the other buffer: its last reader finished a barrier ago
    __syncthreads();
  }

  if (splits > 1) {  // raw partial -> part[sp][m][n] (n < npad, m < M)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int m = m0 + 16 * s + fr;
      if (m >= M) continue;
      float* pr = part + ((int64_t)sp * M + m) * npad + n0 + 64 * wave + 16 * fq;
#pragma unroll
      for (int r = 0; r < 4; ++r) *reinterpret_cast<f4*>(pr + 4 * r) = acc[r][s];
    }
    return;
  }
  // epilogue: y = (d_w / s) acc + bias, 16 contiguous columns per lane and row (4 x 16-B stores)
  const float alpha = (*d_wt) * (WFMT == QVIT_W4 ? 0.0625f : 1.f);
  const int nb = n0 + 64 * wave + 16 * fq;
  float bcol[16];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const f4 b4 = bias ? *reinterpret_cast<const f4*>(bias + nb + 4 * r) : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; ++j) bcol[4 * r + j] = b4[j];
  }
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int m = m0 + 16 * s + fr;
    if (m >= M) continue;
    if (CONV) {  // NCHW: y[b][n][p], 16 lanes of a row group storing consecutive pixels of one plane
      const int b = m / cg.L;
      float* yp = Y + ((int64_t)b * N * cg.L + (m - b * cg.L));
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = nb + 4 * r + j;
          if (n < N) yp[(int64_t)n * cg.L] = fmaf(alpha, acc[r][s][j], bcol[4 * r + j]);
        }
      continue;
    }
    float* yr = Y + (int64_t)m * ldy + nb;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      f4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = fmaf(alpha, acc[r][s][j], bcol[4 * r + j]);
      const int n = nb + 4 * r;
      if (n + 4 <= N) {
        *reinterpret_cast<f4*>(yr + 4 * r) = o;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (n + j < N) yr[4 * r + j] = o[j];
      }
    }
  }
}

// y[m][n] = (d_w / s) sum_sp part[sp][m][n] + bias[n], the partials summed in split order
template <int WFMT>
__global__ __launch_bounds__(256) void wonly_reduce_kernel(const float* __restrict__ part, int splits, int M, int N,
                                                            int npad, const float* __restrict__ d_wt,
                                                            const float* __restrict__ bias, float* __restrict__ Y,
                                                            int64_t ldy, int L) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // one 4-column group per thread
  const int gpr = npad / 4;
  if (i >= (int64_t)M * gpr) return;
  const int m = (int)(i / gpr), n = 4 * (int)(i - (int64_t)m * gpr);
  if (n >= N) return;
  f4 a = *reinterpret_cast<const f4*>(part + (int64_t)m * npad + n);
  for (int sp = 1; sp < splits; ++sp) a += *reinterpret_cast<const f4*>(part + ((int64_t)sp * M + m) * npad + n);
  const float alpha = (*d_wt) * (WFMT == QVIT_W4 ? 0.0625f : 1.f);
  if (L > 0) {  // NCHW output of a convolution (L pixels per plane)
    const int b = m / L;
    float* yp = Y + ((int64_t)b * N * L + (m - b * L));
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (n + j < N) yp[(int64_t)(n + j) * L] = fmaf(alpha, a[j], bias ? bias[n + j] : 0.f);
    return;
  }
  float* yr = Y + (int64_t)m * ldy + n;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (n + j < N) yr[j] = fmaf(alpha, a[j], bias ? bias[n + j] : 0.f);
}

// ---- narrow convolution (N <= 64 output channels, UltraNet's Conv2d_Q layers) -----------------------------------
// The wide kernel's 256-row weight tile is 75-94 % padding for 16-64 output channels. Here all N features (NT
// MFMA tiles of 16) of all K stages sit in LDS for the workgroup's lifetime (loaded once, re-ordered from the packed
// image so that LDS row f = feature f), with a table of every tap's input offset, and each WAVE then runs on its own,
// with no barrier and no LDS staging of the patches: a wave tile is 16 output pixels, lane (fr, fq) gathers the 16
// consecutive taps 64 st + 16 fq .. + 15 of pixel fr itself (straight into its MFMA operand registers, split into
// the three bf16 terms there), and the wave walks its tiles with the next (tile, stage)'s taps loaded while the
// current one computes. MFMAs, their operands and their order per accumulator (stage, chunk c, bf16 term p) are the
// wide kernel's, so the results are bit-identical to it (tests/test_gpu_ultra_modules.py::
// test_conv_wonly_narrow_equals_wide). Stages past C kh kw are skipped.
// EPI 0: y = (d_w / s) acc + bias; EPI 1 (qvit_conv_wonly_bn_act, Conv2d_Q -> BatchNorm2d(eval) ->
// activation_quantize_fn): z = fma(y, alpha_n, shift_n) (one rounding; alpha, shift: the fold ultra_bn_fold computes,
// the fused network's BN step, whose mul + add the compiler contracts the same way) -> round(clamp(z, 0, 1) levels) /
// levels.
constexpr int NW_WMAX = 24 * 1024;                     // weight panel bytes
constexpr int NW_KMAX = 1024;                          // taps in the offset table (C kh kw <= 1024)
constexpr int NW_WAVES = 4;

bool g_wonly_narrow = true;

// PAIR (C kh kw <= 32, one stage whose taps 32 .. 63 are all zero, e.g. UltraNet's layer 0): lanes fq = 2, 3 gather
// a SECOND 16-pixel tile's taps 0 .. 31 instead of zeros, and one v_permlane32_swap per operand register turns the
// gathered registers into both tiles' operands (upper half zero): half the gather instructions per pixel.
template <int WFMT, int NT, int EPI, bool PAIR>
__global__ __launch_bounds__(NW_WAVES * 64) void conv_wonly_narrow_kernel(
    const float* __restrict__ X, int M, int nke, const int8_t* __restrict__ Wp, int N,
    const float* __restrict__ d_wt, const float* __restrict__ bias, const float* __restrict__ bn_a,
    const float* __restrict__ bn_s, float levels, float* __restrict__ Y, const WoConv cg) {
  using G = WoGeo<WFMT>;
  constexpr int NF = 16 * NT;                          // feature rows held
  __shared__ __attribute__((aligned(16))) int8_t w_l[NW_WMAX];    // [stage][NF rows][WROW]
  __shared__ __attribute__((aligned(16))) int2 tap_l[NW_KMAX];    // tap k: {input offset, dy << 16 | dx}
  __shared__ float par_l[3][64];                                  // bias, BN alpha, BN shift
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;

  // ---- workgroup setup: weight panel (LDS row f of stage st = packed row rho(f), the inverse of perm_row inside
  // the first 64-row group, chunks re-swizzled from rho's position to f's), tap table, epilogue parameters
  {
    constexpr int CH = G::WROW / 4;                    // 8 (W4) / 16 (W8) bytes per chunk
    const int units = nke * NF * 4;
    for (int u = tid; u < units; u += NW_WAVES * 64) {
      const int c = u & 3, f = (u >> 2) % NF, st = (u >> 2) / NF;
      const int rho = 16 * ((f >> 2) & 3) + 4 * (f >> 4) + (f & 3);
      const int sw_src = WFMT == QVIT_W4 ? ((rho >> 3) & 1) << 1 : ((rho >> 2) & 1) << 1;
      const int sw_dst = WFMT == QVIT_W4 ? ((f >> 3) & 1) << 1 : ((f >> 2) & 1) << 1;
      const int8_t* src = Wp + (int64_t)st * G::WBYTES + rho * G::WROW + CH * (c ^ sw_src);
      int8_t* dst = w_l + (st * NF + f) * G::WROW + CH * (c ^ sw_dst);
      if (CH == 8) *reinterpret_cast<uint2*>(dst) = *reinterpret_cast<const uint2*>(src);
      else *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(src);
    }
    const int khw = cg.kh * cg.kw;
    for (int k = tid; k < nke * WO_BK; k += NW_WAVES * 64) {
      int2 e = make_int2(0, 0x7fff0000);               // past C kh kw: dy out of range (zero tap)
      if (k < cg.kreal) {
        const int c = k / khw, r = k - c * khw, ky = r / cg.kw, kx = r - ky * cg.kw;
        const int dy = ky * cg.dh, dx = kx * cg.dw;
        e = make_int2((c * cg.H + dy) * cg.W + dx, (dy << 16) | dx);
      }
      tap_l[k] = e;
    }
    for (int f = tid; f < 64; f += NW_WAVES * 64) {
      par_l[0][f] = (bias && f < N) ? bias[f] : 0.f;
      par_l[1][f] = (EPI == 1 && f < N) ? bn_a[f] : 0.f;
      par_l[2][f] = (EPI == 1 && f < N) ? bn_s[f] : 0.f;
    }
  }
  __syncthreads();

  constexpr int TPU = PAIR ? 2 : 1;                    // 16-pixel tiles per unit
  const int ntiles = (M + 16 * TPU - 1) / (16 * TPU);  // wave units
  const int gw = (int)blockIdx.x * NW_WAVES + wave, tw = (int)gridDim.x * NW_WAVES;
  const int my = ntiles > gw ? (ntiles - 1 - gw) / tw + 1 : 0;
  const int units = my * nke;
  // the load side: this lane's pixel of the tile being loaded
  int64_t lbase = 0;
  int iy0 = 0, ix0 = 0;
  bool mval = false;
  float xv[16];
  auto load = [&](int u) __attribute__((always_inline)) {
    const int i = u / nke, st = u - i * nke;
    if (st == 0) {
      const int m = ((gw + i * tw) * TPU + (PAIR ? fq >> 1 : 0)) * 16 + fr;
      mval = m < M;
      const int mm = mval ? m : M - 1;
      const int b = mm / cg.L, p = mm - b * cg.L, oy = p / cg.OW;
      iy0 = oy * cg.sh - cg.ph;
      ix0 = (p - oy * cg.OW) * cg.sw - cg.pw;
      lbase = (int64_t)b * cg.C * cg.H * cg.W + (int64_t)iy0 * cg.W + ix0;
    }
    const int2* tp = tap_l + st * WO_BK + 16 * (PAIR ? fq & 1 : fq);
#pragma unroll
    for (int e = 0; e < 16; e += 2) {
      const int4 t2 = *reinterpret_cast<const int4*>(tp + e);   // taps e, e + 1
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int off = h ? t2.z : t2.x, dd = h ? t2.w : t2.y;
        const int dy = dd >> 16, dx = dd & 0xffff;
        const bool ok = mval && (unsigned)(iy0 + dy) < (unsigned)cg.H && (unsigned)(ix0 + dx) < (unsigned)cg.W;
        float v = 0.f;
        if (ok) v = X[lbase + off];  // (exec-masked: padding and taps past C kh kw issue no request)
        xv[e + h] = v;
      }
    }
  };

  const int woff = (WFMT == QVIT_W4) ? fr * G::WROW + ((fq ^ (((fr >> 3) & 1) << 1)) << 3)
                                     : fr * G::WROW + ((fq ^ (((fr >> 2) & 1) << 1)) << 4);
  const float alpha = (*d_wt) * (WFMT == QVIT_W4 ? 0.0625f : 1.f);
  f4 acc[TPU][NT];
#pragma unroll
  for (int q = 0; q < TPU; ++q)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[q][t] = f4{0.f, 0.f, 0.f, 0.f};

  if (units > 0) load(0);
  for (int u = 0; u < units; ++u) {
    const int i = u / nke, st = u - i * nke;
    // this unit's taps as the three exact bf16 terms (the wide kernel's split), chunk c = taps 8 c .. 8 c + 7
    bf8 xs[3][2], xt[PAIR ? 3 : 1][2];
    {
      uint32_t p1[8], p2[8], p3[8];
#pragma unroll
      for (int e = 0; e < 16; e += 2) {
        const float a = xv[e], c = xv[e + 1];
        const float a1 = trunc_bf16(a), c1 = trunc_bf16(c);
        const float ar = a - a1, cr = c - c1;
        const float a2 = trunc_bf16(ar), c2 = trunc_bf16(cr);
        const float a3 = ar - a2, c3 = cr - c2;
        p1[e >> 1] = hi16(a1, c1);
        p2[e >> 1] = hi16(a2, c2);
        p3[e >> 1] = hi16(a3, c3);
      }
      if constexpr (PAIR) {  // lanes 32 .. 63 hold the second tile: split into {lo, 0} and {hi, 0}
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          uint32_t a1[4], a2[4], a3[4], b1[4], b2[4], b3[4];
#pragma unroll
          for (int d = 0; d < 4; ++d) {
            const auto w1 = __builtin_amdgcn_permlane32_swap(p1[4 * c + d], 0u, false, false);
            const auto w2 = __builtin_amdgcn_permlane32_swap(p2[4 * c + d], 0u, false, false);
            const auto w3 = __builtin_amdgcn_permlane32_swap(p3[4 * c + d], 0u, false, false);
            a1[d] = w1[0]; b1[d] = w1[1];
            a2[d] = w2[0]; b2[d] = w2[1];
            a3[d] = w3[0]; b3[d] = w3[1];
          }
          xs[0][c] = __builtin_bit_cast(bf8, make_uint4(a1[0], a1[1], a1[2], a1[3]));
          xs[1][c] = __builtin_bit_cast(bf8, make_uint4(a2[0], a2[1], a2[2], a2[3]));
          xs[2][c] = __builtin_bit_cast(bf8, make_uint4(a3[0], a3[1], a3[2], a3[3]));
          xt[0][c] = __builtin_bit_cast(bf8, make_uint4(b1[0], b1[1], b1[2], b1[3]));
          xt[1][c] = __builtin_bit_cast(bf8, make_uint4(b2[0], b2[1], b2[2], b2[3]));
          xt[2][c] = __builtin_bit_cast(bf8, make_uint4(b3[0], b3[1], b3[2], b3[3]));
        }
      } else {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          xs[0][c] = __builtin_bit_cast(bf8, make_uint4(p1[4 * c], p1[4 * c + 1], p1[4 * c + 2], p1[4 * c + 3]));
          xs[1][c] = __builtin_bit_cast(bf8, make_uint4(p2[4 * c], p2[4 * c + 1], p2[4 * c + 2], p2[4 * c + 3]));
          xs[2][c] = __builtin_bit_cast(bf8, make_uint4(p3[4 * c], p3[4 * c + 1], p3[4 * c + 2], p3[4 * c + 3]));
        }
      }
    }
    if (u + 1 < units) load(u + 1);  // lands while this unit computes
    bf8 wb[NT][2];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int8_t* wp = w_l + (st * NF + 16 * t) * G::WROW + woff;
      v4i wf;
      if (WFMT == QVIT_W4) {
        const uint2 p = *reinterpret_cast<const uint2*>(wp);
        wf = v4i{(int)nib16_lo(p.x), (int)nib16_hi(p.x), (int)nib16_lo(p.y), (int)nib16_hi(p.y)};
      } else {
        wf = *reinterpret_cast<const v4i*>(wp);
      }
      uint32_t h[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) bytes_bf16((uint32_t)wf[e], h[2 * e], h[2 * e + 1], 1.f);
      wb[t][0] = __builtin_bit_cast(bf8, make_uint4(h[0], h[1], h[2], h[3]));
      wb[t][1] = __builtin_bit_cast(bf8, make_uint4(h[4], h[5], h[6], h[7]));
    }
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          acc[0][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[t][c], xs[p][c], acc[0][t], 0, 0, 0);
          if constexpr (PAIR)
            acc[PAIR ? 1 : 0][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[t][c], xt[PAIR ? p : 0][c],
                                                                            acc[PAIR ? 1 : 0][t], 0, 0, 0);
        }
    if (st == nke - 1) {
      // epilogue of the unit's tiles: lane (fr, fq) holds features 16 t + 4 fq + j of pixel fr
#pragma unroll
      for (int q = 0; q < TPU; ++q) {
        const int m = ((gw + i * tw) * TPU + q) * 16 + fr;
        if (m < M) {
          const int b = m / cg.L;
          float* yp = Y + ((int64_t)b * N * cg.L + (m - b * cg.L));
#pragma unroll
          for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int n = 16 * t + 4 * fq + j;
              float y = fmaf(alpha, acc[q][t][j], par_l[0][n]);
              if (EPI == 1) {
                const float z = fmaf(y, par_l[1][n], par_l[2][n]);
                y = rintf(fminf(fmaxf(z, 0.f), 1.f) * levels) / levels;
              }
              if (n < N) yp[(int64_t)n * cg.L] = y;
            }
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[q][t] = f4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
}

// the narrow schedule's stage count and feature tiles, or 0 when it does not apply
struct NarrowGeo {
  int nke, nt;
};
NarrowGeo narrow_geo(int wfmt, int64_t N, int64_t npad, int64_t K, const WoConv& cg) {
  if (!g_wonly_narrow || (wfmt != QVIT_W4 && wfmt != QVIT_W8) || N > 64 || npad < 64) return {0, 0};
  // the tap table holds each tap's input offset (c H + dy) W + dx as an int32 and dy, dx in 16 bits each, with
  // dy = 0x7fff marking a zero tap (never inside the image: iy0 + 0x7fff >= H for every iy0 >= -ph); layers past
  // these bounds take the wide schedule, which computes the offsets in 64 bits
  const int64_t dy_max = (int64_t)cg.dh * (cg.kh - 1), dx_max = (int64_t)cg.dw * (cg.kw - 1);
  if (cg.H >= 32767 || cg.W >= 32767 || dy_max >= 32767 || dx_max >= 32767) return {0, 0};
  if ((int64_t)cg.ph + cg.H > 32767) return {0, 0};
  if ((int64_t)cg.C * cg.H * cg.W + dy_max * cg.W + dx_max > INT32_MAX) return {0, 0};
  const int64_t kreal = cg.kreal;
  const int nke = (int)((kreal + WO_BK - 1) / WO_BK);
  const int nt = (int)((N + 15) / 16);
  const int wrow = wfmt == QVIT_W4 ? 32 : 64;
  const int64_t wbytes = (int64_t)nke * 16 * nt * wrow;
  if (nke < 1 || nke > K / WO_BK || wbytes > NW_WMAX || nke * WO_BK > NW_KMAX) return {0, 0};
  return {nke, nt};
}

template <int EPI>
int narrow_launch(const NarrowGeo& g, const float* X, int64_t M, const int8_t* w, int wfmt, int64_t N,
                  const float* d_wt, const float* bias, const float* bn_a, const float* bn_s, float levels, float* Y,
                  const WoConv& cg, hipStream_t stream) {
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                hipSuccess || n <= 0)
      n = 256;
    return n;
  }();
  // wave units of 16 (PAIR: 32) pixels; resident workgroups (8 per CU), no more than the units need
  const bool pair = cg.kreal <= 32;
  const int64_t wtiles = (M + (pair ? 31 : 15)) / (pair ? 32 : 16);
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((wtiles + NW_WAVES - 1) / NW_WAVES,
                                                                         8 * (int64_t)cus));
#define QVIT_NW2(F, T, PR)                                                                                        \
  hipLaunchKernelGGL((conv_wonly_narrow_kernel<F, T, EPI, PR>), dim3(grid), dim3(NW_WAVES * 64), 0, stream, X,      \
                     (int)M, g.nke, w, (int)N, d_wt, bias, bn_a, bn_s, levels, Y, cg)
#define QVIT_NW(F, T)     \
  if (pair) {             \
    QVIT_NW2(F, T, true); \
  } else {                \
    QVIT_NW2(F, T, false); \
  }
#define QVIT_NW_T(F)      \
  switch (g.nt) {         \
    case 1: QVIT_NW(F, 1); break; \
    case 2: QVIT_NW(F, 2); break; \
    case 3: QVIT_NW(F, 3); break; \
    default: QVIT_NW(F, 4); break; \
  }
  if (wfmt == QVIT_W4) {
    QVIT_NW_T(QVIT_W4)
  } else {
    QVIT_NW_T(QVIT_W8)
  }
#undef QVIT_NW_T
#undef QVIT_NW
#undef QVIT_NW2
  return qvit_hip_status(hipGetLastError());
}

// shared launch of the GEMM (CONV = false) and the implicit-GEMM convolution (CONV = true); arguments checked
template <bool CONV>
int wonly_launch(const float* X, int64_t M, int64_t K, int64_t ldx, const void* Wp, int wfmt, int64_t N, int64_t npad,
                 const float* d_wt, const float* bias, float* Y, int64_t ldy, float* workspace, int64_t workspace_bytes,
                 const WoConv& cg, hipStream_t stream) {
  const int64_t ntiles = (npad / WO_BN) * ((M + WO_BM - 1) / WO_BM);
  if (ntiles > INT32_MAX / 2) return QVIT_EINVAL;
  if (CONV) {  // few output channels: the narrow schedule
    const NarrowGeo g = narrow_geo(wfmt, N, npad, K, cg);
    if (g.nke > 0)
      return narrow_launch<0>(g, X, M, reinterpret_cast<const int8_t*>(Wp), wfmt, N, d_wt, bias, nullptr, nullptr,
                              0.f, Y, cg, stream);
  }
  // fewer tiles than half the CUs: split the K stages so that about 256 workgroups run (when the workspace
  // holds the partials)
  const int64_t nk = K / WO_BK;
  int64_t splits = 1;
  if (ntiles < 128 && nk >= 2 && workspace && !(((uintptr_t)workspace) & 15)) {
    splits = std::min<int64_t>(nk, (256 + ntiles - 1) / ntiles);
    while (splits > 1 && splits * M * npad * 4 > workspace_bytes) --splits;
  }
  const int64_t grid = splits > 1 ? ntiles * splits : (ntiles + 7) / 8 * 8;
  const int8_t* w = reinterpret_cast<const int8_t*>(Wp);
#define QVIT_WO_LAUNCH(F)                                                                                    \
  hipLaunchKernelGGL((gemm_wonly_kernel<F, CONV>), dim3((unsigned)grid), dim3(256), 0, stream, X, (int)M, (int)K,  \
                     ldx, w, (int)N, (int)npad, d_wt, bias, Y, ldy, (int)splits, workspace, cg)
  if (wfmt == QVIT_W4) QVIT_WO_LAUNCH(QVIT_W4);
  else if (wfmt == QVIT_W8) QVIT_WO_LAUNCH(QVIT_W8);
  else if (wfmt == QVIT_W16) QVIT_WO_LAUNCH(QVIT_W16);
  else QVIT_WO_LAUNCH(QVIT_W24);
#undef QVIT_WO_LAUNCH
  if (splits > 1) {
    const int64_t groups = M * (npad / 4);
    const unsigned rg = (unsigned)((groups + 255) / 256);
    const int L = CONV ? cg.L : 0;
    if (wfmt == QVIT_W4)
      hipLaunchKernelGGL(wonly_reduce_kernel<QVIT_W4>, dim3(rg), dim3(256), 0, stream, workspace, (int)splits, (int)M,
                         (int)N, (int)npad, d_wt, bias, Y, ldy, L);
    else  // (W8 / W16 / W24 accumulators are unscaled)
      hipLaunchKernelGGL(wonly_reduce_kernel<QVIT_W8>, dim3(rg), dim3(256), 0, stream, workspace, (int)splits, (int)M,
                         (int)N, (int)npad, d_wt, bias, Y, ldy, L);
  }
  return qvit_hip_status(hipGetLastError());
}

}  // namespace

extern "C" int qvit_gemm_wonly(const float* X, int64_t M, int64_t K, int64_t ldx, const void* Wp, int wfmt,
                               int64_t N, int64_t npad, const float* d_wt, const float* bias, float* Y, int64_t ldy,
                               float* workspace, int64_t workspace_bytes, hipStream_t stream) {
  if (!X || !Wp || !Y || !d_wt) return QVIT_ENULL;
  if (wfmt != QVIT_W4 && wfmt != QVIT_W8 && wfmt != QVIT_W16 && wfmt != QVIT_W24) return QVIT_EINVAL;
  if (M < 0 || K <= 0 || K % QVIT_TILE_K || ldx < K || N <= 0 || npad < N || npad % WO_BN || ldy < N)
    return QVIT_EINVAL;
  if (M > INT32_MAX / 2 || npad > INT32_MAX / 2 || K > (1 << 24)) return QVIT_EINVAL;
  if ((ldx % 4) || (((uintptr_t)X) & 15) || (((uintptr_t)Wp) & 15)) return QVIT_EALIGN;
  if ((ldy % 4) || (((uintptr_t)Y) & 15) || (bias && (((uintptr_t)bias) & 15))) return QVIT_EALIGN;
  if (M == 0) return QVIT_OK;
  return wonly_launch<false>(X, M, K, ldx, Wp, wfmt, N, npad, d_wt, bias, Y, ldy, workspace, workspace_bytes,
                             WoConv{}, stream);
}

namespace {

// the argument checks of the convolution entries; fills cg and M
int conv_args(const float* X, int64_t B, int64_t C, int64_t H, int64_t W, int kh, int kw, int sh, int sw, int ph,
              int pw, int dh, int dw, const void* Wp, int wfmt, int64_t N, int64_t npad, int64_t K, const float* d_wt,
              const float* bias, float* Y, WoConv& cg, int64_t& M) {
  if (!X || !Wp || !Y || !d_wt) return QVIT_ENULL;
  if (wfmt != QVIT_W4 && wfmt != QVIT_W8 && wfmt != QVIT_W16 && wfmt != QVIT_W24) return QVIT_EINVAL;
  if (B < 0 || C <= 0 || H <= 0 || W <= 0 || kh <= 0 || kw <= 0 || sh <= 0 || sw <= 0 || ph < 0 || pw < 0 ||
      dh <= 0 || dw <= 0)
    return QVIT_EINVAL;
  if (C > INT32_MAX || H > INT32_MAX || W > INT32_MAX || B * C * H * W > (int64_t)1 << 40) return QVIT_EINVAL;
  const int64_t OH = (H + 2 * ph - (int64_t)dh * (kh - 1) - 1) / sh + 1;
  const int64_t OW = (W + 2 * pw - (int64_t)dw * (kw - 1) - 1) / sw + 1;
  const int64_t kreal = C * kh * kw;
  if (H + 2 * ph < (int64_t)dh * (kh - 1) + 1 || W + 2 * pw < (int64_t)dw * (kw - 1) + 1) return QVIT_EINVAL;
  if (K <= 0 || K % QVIT_TILE_K || K < kreal || K > (1 << 24) || N <= 0 || npad < N || npad % WO_BN ||
      npad > INT32_MAX / 2)
    return QVIT_EINVAL;
  M = B * OH * OW;
  if (M > INT32_MAX / 2 || OH * OW > INT32_MAX / 2) return QVIT_EINVAL;
  if ((((uintptr_t)Wp) & 15) || (bias && (((uintptr_t)bias) & 15))) return QVIT_EALIGN;
  cg = WoConv{(int)C, (int)H, (int)W, kh, kw, sh, sw, ph, pw, dh, dw, (int)OW, (int)(OH * OW), (int)kreal};
  return QVIT_OK;
}

}  // namespace

extern "C" int qvit_conv_wonly(const float* X, int64_t B, int64_t C, int64_t H, int64_t W, int kh, int kw, int sh,
                               int sw, int ph, int pw, int dh, int dw, const void* Wp, int wfmt, int64_t N,
                               int64_t npad, int64_t K, const float* d_wt, const float* bias, float* Y,
                               float* workspace, int64_t workspace_bytes, hipStream_t stream) {
  WoConv cg{};
  int64_t M = 0;
  const int st = conv_args(X, B, C, H, W, kh, kw, sh, sw, ph, pw, dh, dw, Wp, wfmt, N, npad, K, d_wt, bias, Y, cg, M);
  if (st != QVIT_OK) return st;
  if (M == 0) return QVIT_OK;
  return wonly_launch<true>(X, M, K, K, Wp, wfmt, N, npad, d_wt, bias, Y, N, workspace, workspace_bytes, cg, stream);
}

extern "C" int qvit_conv_wonly_bn_act(const float* X, int64_t B, int64_t C, int64_t H, int64_t W, int kh, int kw,
                                      int sh, int sw, int ph, int pw, int dh, int dw, const void* Wp, int wfmt,
                                      int64_t N, int64_t npad, int64_t K, const float* d_wt, const float* bias,
                                      const float* bn_alpha, const float* bn_shift, int a_levels, float* Y,
                                      hipStream_t stream) {
  WoConv cg{};
  int64_t M = 0;
  const int st = conv_args(X, B, C, H, W, kh, kw, sh, sw, ph, pw, dh, dw, Wp, wfmt, N, npad, K, d_wt, bias, Y, cg, M);
  if (st != QVIT_OK) return st;
  if (!bn_alpha || !bn_shift) return QVIT_ENULL;
  if (a_levels < 1 || a_levels > 127) return QVIT_EINVAL;
  const NarrowGeo g = narrow_geo(wfmt, N, npad, K, cg);
  // (N > 64, W16 / W24, a weight panel past NW_WMAX, or offsets past the tap table's bounds: unfused modules)
  if (g.nke == 0) return QVIT_EINVAL;
  if (M == 0) return QVIT_OK;
  return narrow_launch<1>(g, X, M, reinterpret_cast<const int8_t*>(Wp), wfmt, N, d_wt, bias, bn_alpha, bn_shift,
                          (float)a_levels, Y, cg, stream);
}

extern "C" int qvit_conv_wonly_narrow(int enable) {
  const int prev = g_wonly_narrow ? 1 : 0;
  if (enable >= 0) g_wonly_narrow = enable != 0;
  return prev;
}
