// UltraNet 4-bit path (reference `4-bit quantization/`): quant_ultra.py weight/activation quantizers and
// Conv2d_Q (:8-91), and the conv -> BatchNorm2d(eval) -> activation_quantize_fn -> MaxPool2d blocks and
// YOLO decode of mymodel.py:23-144.
//
// Integer view: weight codes k_w = rne(tanh(w)/max|tanh(w)| * 7) (value k_w/7),
// activation codes k_a = rne(clamp(x,0,1) * 15) (value k_a/15), so a conv on codes is an exact int32
// contraction acc = sum k_a k_w with conv value acc/105. BN in eval mode is the per-channel affine
// y = x * alpha + beta with alpha = gamma / sqrt(var + eps), beta = bias - mean * alpha (the order torch's
// CPU batch_norm uses), and the next code is rne(clamp(y,0,1) * 15). MaxPool2d(2,2) commutes with the
// monotone quantizer, so pooling runs on codes, fused into the producing conv's epilogue.
//
// Kernels:
//   ultra_wmax / ultra_wcodes : the weight quantizer (two passes: max|tanh|, then codes in the conv
//                               kernel's K order (ky, kx, c)).
//   ultra_bn_fold             : per-channel (alpha, beta) on the device.
//   ultra_conv0               : layer 0 (float image input, 3 -> 16, 3x3): direct fp32 conv on the
//                               VALU (27 taps), fused BN + quantizer + 2x2 max pool; NCHW in, NHWC codes out.
//   ultra_conv                : layers 1..8: implicit GEMM on v_mfma_i32_16x16x64_i8 over NHWC codes.
//                               Block = 4 waves, 16x16 output pixels (each MFMA column tile is a 4x4
//                               pixel patch, so a 2x2 pool window is lanes p, p^1, p^4, p^5), all output
//                               channels; the (16+ks-1)^2 x Cin halo tile and the whole [Cout][9 Cin]
//                               weight image sit in LDS (weights loaded once per persistent block); the
//                               K loop runs over 64-deep chunks of (tap, channel); epilogue = BN + quantizer
//                               (+ pool) -> NHWC codes, or (head) acc/105 + bias -> fp32 NHWC.
//   yolo_decode               : YOLOLayer eval decode (mymodel.py:47-60) from the head's NHWC output.
#include "qvit_common.h"

namespace {

typedef int v4i __attribute__((ext_vector_type(4)));

// ---- weight quantizer ----------------------------------------------------------------------------
__global__ void ultra_wmax_kernel(const float* __restrict__ w, int64_t n, unsigned* __restrict__ maxbits) {
  float m = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    m = fmaxf(m, fabsf(tanhf(w[i])));
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) atomicMax(maxbits, __float_as_uint(m));  // m >= 0: bit order == value order
}

// codes[o][k], k = (ky * ks + kx) * cin + c, rows >= cout and columns >= ks*ks*cin zero
__global__ void ultra_wcodes_kernel(const float* __restrict__ w, int cout, int cin, int ks,
                                    const unsigned* __restrict__ maxbits, float n, int8_t* __restrict__ codes,
                                    int kpad, int cout_pad, float* __restrict__ values) {
  const int64_t total = (int64_t)cout_pad * kpad;
  const float m = __uint_as_float(*maxbits);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int o = (int)(i / kpad), k = (int)(i % kpad);
    int8_t code = 0;
    if (o < cout && k < ks * ks * cin) {
      const int tap = k / cin, c = k % cin;
      const int64_t src = (((int64_t)o * cin + c) * ks + tap / ks) * ks + tap % ks;
      const float t = tanhf(w[src]);
      const float kq = rintf((t / m) * n);  // quant_ultra.py:52-55 + :20: round((tanh(w)/max) * n)
      code = (int8_t)kq;
      if (values) values[src] = kq / n;     // the reference's value round(.) / n, original layout
    }
    codes[i] = code;
  }
}

__global__ void ultra_bn_fold_kernel(const float* gamma, const float* beta, const float* mean, const float* var,
                                     float eps, int n, float* alpha, float* shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  const float invstd = 1.0f / sqrtf(__fadd_rn(var[c], eps));
  const float a = __fmul_rn(invstd, gamma ? gamma[c] : 1.f);
  alpha[c] = a;
  shift[c] = __fsub_rn(beta ? beta[c] : 0.f, __fmul_rn(mean[c], a));
}

QVIT_DEV int act_code(float x, float alpha, float shift, float levels) {
  const float y = __fadd_rn(__fmul_rn(x, alpha), shift);
  return (int)rintf(fminf(fmaxf(y, 0.f), 1.f) * levels);
}

// ---- layer 0: float image, 3 -> 16 channels, 3x3 pad 1, BN + quantizer + 2x2 pool ----------------
// One thread per pooled pixel (a 4x4x3 input window held in registers, 2x2 pre-pool pixels). The weights
// (fake-quant values k/7, [16][3][3][3] as the reference lays them out) are read with wave-uniform
// indices, so they arrive through scalar loads and feed the FMAs as SGPR operands; pixel pairs along x
// run as packed fp32 FMAs. The output-channel loop is not unrolled, which keeps the register count low
// enough for several waves per SIMD (the kernel waits on image loads, not on math).
constexpr int C0_IN = 3, C0_OUT = 16, C0_K = C0_IN * 9;
typedef float f2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void ultra_conv0_kernel(const float* __restrict__ img, int B, int H, int W,
                                                          const float* __restrict__ wvals,
                                                          const float* __restrict__ alpha,
                                                          const float* __restrict__ shift, float levels,
                                                          int8_t* __restrict__ out) {
  const int Ho = H / 2, Wo = W / 2;
  const int64_t total = (int64_t)B * Ho * Wo;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int xo = (int)(i % Wo);
    const int yo = (int)((i / Wo) % Ho);
    const int b = (int)(i / ((int64_t)Wo * Ho));
    float win[C0_IN][4][4];
#pragma unroll
    for (int c = 0; c < C0_IN; ++c)
#pragma unroll
      for (int dy = 0; dy < 4; ++dy)
#pragma unroll
        for (int dx = 0; dx < 4; ++dx) {
          const int y = 2 * yo - 1 + dy, x = 2 * xo - 1 + dx;
          win[c][dy][dx] = (y >= 0 && y < H && x >= 0 && x < W) ? img[(((int64_t)b * C0_IN + c) * H + y) * W + x] : 0.f;
        }
    uint32_t words[4] = {0, 0, 0, 0};
#pragma unroll 1
    for (int o = 0; o < C0_OUT; ++o) {
      const float* wo = wvals + o * C0_K;  // [c][ky][kx], wave-uniform
      f2 acc0 = {0.f, 0.f}, acc1 = {0.f, 0.f};  // pre-pool rows 0 and 1, pixels (x, x+1)
#pragma unroll
      for (int c = 0; c < C0_IN; ++c)
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) {
            const float wv = wo[(c * 3 + ky) * 3 + kx];
            const f2 w2 = {wv, wv};
            acc0 = __builtin_elementwise_fma(f2{win[c][ky][kx], win[c][ky][kx + 1]}, w2, acc0);
            acc1 = __builtin_elementwise_fma(f2{win[c][ky + 1][kx], win[c][ky + 1][kx + 1]}, w2, acc1);
          }
      const float al = alpha[o], sh = shift[o];
      const int best = max(max(act_code(acc0.x, al, sh, levels), act_code(acc0.y, al, sh, levels)),
                           max(act_code(acc1.x, al, sh, levels), act_code(acc1.y, al, sh, levels)));
      const uint32_t v = (uint32_t)best << (8 * (o & 3));
      if ((o >> 2) == 0) words[0] |= v;
      else if ((o >> 2) == 1) words[1] |= v;
      else if ((o >> 2) == 2) words[2] |= v;
      else words[3] |= v;
    }
    *reinterpret_cast<uint4*>(out + i * C0_OUT) = make_uint4(words[0], words[1], words[2], words[3]);
  }
}

// ---- integer deploy (quantization.py:24-31,68-89; ultranet_param_gen.py) --------------------------------
// The FPGA flow's integer form of conv -> BN -> activation quantizer: with per-channel inc_q, bias_q from
// bn_act_quantize_int and S = w_bit - 1 + in_bit + l_shift,
//   code = clamp(round((acc * inc_q + bias_q) / 2^S), 0, 2^out_bit - 1),   round = half up ((x + 2^(S-1)) >> S)
// in 64-bit integer arithmetic (acc * inc_q can exceed 32 bits). The accelerator's own rounding is not in
// the reference (its HLS source is absent): parity for this formula is unpinned beyond the oracle's
// restatement of the same expression.
QVIT_DEV int int_code(int acc, int inc, int bias, int sbits, int levels) {
  const long long v = ((long long)acc * inc + bias + (1ll << (sbits - 1))) >> sbits;
  return (int)(v < 0 ? 0 : (v > levels ? levels : v));
}

// Layer 0 of the integer deploy: uint8 image NCHW (in_bit 8), weight codes [16][3][3][3] (reference layout),
// int32 accumulation, integer threshold, 2x2 max pool on the codes -> NHWC codes [B][H/2][W/2][16].
__global__ __launch_bounds__(256) void ultra_conv0_int_kernel(const uint8_t* __restrict__ img, int B, int H, int W,
                                                              const int8_t* __restrict__ wcodes,
                                                              const int* __restrict__ inc,
                                                              const int* __restrict__ bias, int sbits, int levels,
                                                              int8_t* __restrict__ out) {
  const int Ho = H / 2, Wo = W / 2;
  const int64_t total = (int64_t)B * Ho * Wo;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int xo = (int)(i % Wo);
    const int yo = (int)((i / Wo) % Ho);
    const int b = (int)(i / ((int64_t)Wo * Ho));
    int win[C0_IN][4][4];
#pragma unroll
    for (int c = 0; c < C0_IN; ++c)
#pragma unroll
      for (int dy = 0; dy < 4; ++dy)
#pragma unroll
        for (int dx = 0; dx < 4; ++dx) {
          const int y = 2 * yo - 1 + dy, x = 2 * xo - 1 + dx;
          win[c][dy][dx] = (y >= 0 && y < H && x >= 0 && x < W) ? img[(((int64_t)b * C0_IN + c) * H + y) * W + x] : 0;
        }
    uint32_t words[4] = {0, 0, 0, 0};
#pragma unroll 1
    for (int o = 0; o < C0_OUT; ++o) {
      const int8_t* wo = wcodes + o * C0_K;  // [c][ky][kx], wave-uniform
      int a00 = 0, a01 = 0, a10 = 0, a11 = 0;
#pragma unroll
      for (int c = 0; c < C0_IN; ++c)
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) {
            const int wv = wo[(c * 3 + ky) * 3 + kx];
            a00 += wv * win[c][ky][kx];
            a01 += wv * win[c][ky][kx + 1];
            a10 += wv * win[c][ky + 1][kx];
            a11 += wv * win[c][ky + 1][kx + 1];
          }
      const int ic = inc[o], bc = bias[o];
      const int best = max(max(int_code(a00, ic, bc, sbits, levels), int_code(a01, ic, bc, sbits, levels)),
                           max(int_code(a10, ic, bc, sbits, levels), int_code(a11, ic, bc, sbits, levels)));
      const uint32_t v = (uint32_t)best << (8 * (o & 3));
      if ((o >> 2) == 0) words[0] |= v;
      else if ((o >> 2) == 1) words[1] |= v;
      else if ((o >> 2) == 2) words[2] |= v;
      else words[3] |= v;
    }
    *reinterpret_cast<uint4*>(out + i * C0_OUT) = make_uint4(words[0], words[1], words[2], words[3]);
  }
}

// ---- layers 1..8: implicit GEMM conv on MFMA ------------------------------------------------------
constexpr int TS = 16;  // output tile 16 x 16 (pre-pool) pixels

template <int CIN, int KS, int COUT>
struct ConvGeo {
  static constexpr int KDIM = KS * KS * CIN;
  static constexpr int KPAD = (KDIM + 63) / 64 * 64;
  static constexpr int WSTR = KPAD + 32;  // weight row pitch: conflict-free ds_read_b128 A fragments
  static constexpr int HT = TS + KS - 1;  // halo tile side
  static constexpr int HALO = HT * HT * CIN;
  static constexpr int LDS = COUT * WSTR + HALO;
  static constexpr int NCT = COUT / 16;
};

// OUT: 0 = BN + quantizer codes (POOL: + 2x2 max pool), 1 = acc/den + bias fp32,
//      2 = integer deploy threshold (alpha / shift hold int32 inc_q / bias_q, sbits = S; POOL as for 0)
template <int CIN, int KS, int COUT, int POOL, int OUT>
__global__ __launch_bounds__(256, 2) void ultra_conv_kernel(const int8_t* __restrict__ in, int B, int H, int W,
                                                            const int8_t* __restrict__ wcodes, int kpad_in,
                                                            float den, const float* __restrict__ alpha,
                                                            const float* __restrict__ shift, float levels,
                                                            int cout_real, void* __restrict__ out, int ldo,
                                                            int sbits) {
  using G = ConvGeo<CIN, KS, COUT>;
  __shared__ __attribute__((aligned(16))) int8_t smem[G::LDS];
  int8_t* wl = smem;
  int8_t* halo = smem + COUT * G::WSTR;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int p = lane & 15, g = lane >> 4;
  const int py = p >> 2, px = p & 3;

  // weights -> LDS once per block (rows >= real cout are zero in the packed image)
  for (int i = tid; i < COUT * (G::KPAD / 16); i += 256) {
    const int o = i / (G::KPAD / 16), c16 = i % (G::KPAD / 16);
    *reinterpret_cast<v4i*>(wl + o * G::WSTR + 16 * c16) =
        *reinterpret_cast<const v4i*>(wcodes + (int64_t)o * kpad_in + 16 * c16);
  }
  float al[G::NCT][4], sh[G::NCT][4];
  int iinc[G::NCT][4], ibias[G::NCT][4];
#pragma unroll
  for (int ct = 0; ct < G::NCT; ++ct)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int o = 16 * ct + 4 * g + j;
      al[ct][j] = (OUT == 0 && o < cout_real) ? alpha[o] : 0.f;
      sh[ct][j] = (OUT != 2 && o < cout_real) ? shift[o] : 0.f;  // OUT == 1: shift = bias
      iinc[ct][j] = (OUT == 2 && o < cout_real) ? reinterpret_cast<const int*>(alpha)[o] : 0;
      ibias[ct][j] = (OUT == 2 && o < cout_real) ? reinterpret_cast<const int*>(shift)[o] : 0;
    }

  const int tiles_y = (H + TS - 1) / TS, tiles_x = (W + TS - 1) / TS;
  const int64_t ntiles = (int64_t)B * tiles_y * tiles_x;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int tx0 = (int)(t % tiles_x) * TS;
    const int ty0 = (int)((t / tiles_x) % tiles_y) * TS;
    const int b = (int)(t / ((int64_t)tiles_x * tiles_y));
    __syncthreads();  // previous tile's halo reads are done
    constexpr int CH16 = CIN / 16;
    for (int i = tid; i < G::HT * G::HT * CH16; i += 256) {
      const int cc = i % CH16, hx = (i / CH16) % G::HT, hy = i / (CH16 * G::HT);
      const int y = ty0 - KS / 2 + hy, x = tx0 - KS / 2 + hx;
      v4i v = {0, 0, 0, 0};
      if (y >= 0 && y < H && x >= 0 && x < W)
        v = *reinterpret_cast<const v4i*>(in + (((int64_t)b * H + y) * W + x) * CIN + 16 * cc);
      *reinterpret_cast<v4i*>(halo + (hy * G::HT + hx) * CIN + 16 * cc) = v;
    }
    __syncthreads();

    v4i acc[4][G::NCT];
#pragma unroll
    for (int pt = 0; pt < 4; ++pt)
#pragma unroll
      for (int ct = 0; ct < G::NCT; ++ct) acc[pt][ct] = v4i{0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < G::KPAD / 64; ++j) {
      const int kk = 64 * j + 16 * g;
      const int tap = kk / CIN, c0 = kk % CIN;
      const bool kv = tap < KS * KS;
      const int kty = kv ? tap / KS : 0, ktx = kv ? tap % KS : 0;
      v4i a[G::NCT], bf[4];
#pragma unroll
      for (int ct = 0; ct < G::NCT; ++ct) a[ct] = *reinterpret_cast<const v4i*>(wl + (16 * ct + p) * G::WSTR + kk);
#pragma unroll
      for (int pt = 0; pt < 4; ++pt) {
        const int hy = 4 * wave + py + kty, hx = 4 * pt + px + ktx;
        bf[pt] = *reinterpret_cast<const v4i*>(halo + (hy * G::HT + hx) * CIN + c0);
        if (!kv) bf[pt] = v4i{0, 0, 0, 0};
      }
#pragma unroll
      for (int pt = 0; pt < 4; ++pt)
#pragma unroll
        for (int ct = 0; ct < G::NCT; ++ct)
          acc[pt][ct] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[ct], bf[pt], acc[pt][ct], 0, 0, 0);
    }

    // epilogue: acc[pt][ct][j] = conv[b][cout 16 ct + 4 g + j][y = ty0 + 4 wave + py][x = tx0 + 4 pt + px]
    const int y = ty0 + 4 * wave + py;
#pragma unroll
    for (int pt = 0; pt < 4; ++pt) {
      const int x = tx0 + 4 * pt + px;
#pragma unroll
      for (int ct = 0; ct < G::NCT; ++ct) {
        const int o0 = 16 * ct + 4 * g;
        if (OUT == 1) {
          if (y < H && x < W) {
            float* dst = reinterpret_cast<float*>(out) + (((int64_t)b * H + y) * W + x) * ldo;
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (o0 + j < cout_real) dst[o0 + j] = __fadd_rn((float)acc[pt][ct][j] / den, sh[ct][j]);
          }
        } else {
          int code[4];
#pragma unroll
          for (int j = 0; j < 4; ++j)
            code[j] = (OUT == 2) ? int_code(acc[pt][ct][j], iinc[ct][j], ibias[ct][j], sbits, (int)levels)
                                 : act_code((float)acc[pt][ct][j] / den, al[ct][j], sh[ct][j], levels);
          if (POOL) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              code[j] = max(code[j], __shfl_xor(code[j], 1));
              code[j] = max(code[j], __shfl_xor(code[j], 4));
            }
          }
          const uint32_t word = (uint32_t)code[0] | ((uint32_t)code[1] << 8) | ((uint32_t)code[2] << 16) |
                                ((uint32_t)code[3] << 24);
          if (POOL) {
            const int Ho = H / 2, Wo = W / 2;
            if ((p & 5) == 0 && (y >> 1) < Ho && (x >> 1) < Wo && o0 < cout_real)
              *reinterpret_cast<uint32_t*>(reinterpret_cast<int8_t*>(out) +
                                           (((int64_t)b * Ho + (y >> 1)) * Wo + (x >> 1)) * ldo + o0) = word;
          } else if (y < H && x < W && o0 < cout_real) {
            *reinterpret_cast<uint32_t*>(reinterpret_cast<int8_t*>(out) + (((int64_t)b * H + y) * W + x) * ldo + o0) =
                word;
          }
        }
      }
    }
  }
}

// ---- YOLOLayer decode (mymodel.py:47-60) -----------------------------------------------------------
__global__ void yolo_decode_kernel(const float* __restrict__ head, int B, int ny, int nx, int na, int no, int ldh,
                                   const float* __restrict__ anchors, float stride, float* __restrict__ io,
                                   float* __restrict__ pout) {
  const int64_t total = (int64_t)B * na * ny * nx * no;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int o = (int)(i % no);
    const int x = (int)((i / no) % nx);
    const int y = (int)((i / ((int64_t)no * nx)) % ny);
    const int a = (int)((i / ((int64_t)no * nx * ny)) % na);
    const int b = (int)(i / ((int64_t)no * nx * ny * na));
    // p[b][a][y][x][o] = head_nchw[b][a*no + o][y][x] = head_nhwc[b][y][x][a*no + o]
    const float v = head[(((int64_t)b * ny + y) * nx + x) * ldh + a * no + o];
    pout[i] = v;
    float r;
    if (o < 2) {
      r = __fadd_rn(1.f / (1.f + expf(-v)), (float)(o == 0 ? x : y));
      r = __fmul_rn(r, stride);
    } else if (o < 4) {
      const float awh = anchors[2 * a + (o - 2)] / stride;  // anchor_vec = anchors / stride
      r = __fmul_rn(__fmul_rn(expf(v), awh), stride);
    } else {
      r = 1.f / (1.f + expf(-v));
    }
    io[i] = r;
  }
}

int grid_cap(int64_t work, int per = 256) {
  int64_t g = (work + per - 1) / per;
  if (g > 256 * 16) g = 256 * 16;
  return (int)(g < 1 ? 1 : g);
}

template <int CIN, int KS, int COUT, int POOL, int OUT>
int launch_conv(const int8_t* in, int B, int H, int W, const int8_t* w, int kpad, float den, const float* alpha,
                const float* shift, float levels, int cout_real, void* out, int ldo, hipStream_t stream,
                int sbits = 0) {
  using G = ConvGeo<CIN, KS, COUT>;
  if (kpad < G::KPAD) return QVIT_EINVAL;
  const int64_t ntiles = (int64_t)B * ((H + TS - 1) / TS) * ((W + TS - 1) / TS);
  const int grid = (int)(ntiles < 256 * 8 ? ntiles : 256 * 8);
  hipLaunchKernelGGL((ultra_conv_kernel<CIN, KS, COUT, POOL, OUT>), dim3(grid), dim3(256), 0, stream, in, B, H, W,
                     w, kpad, den, alpha, shift, levels, cout_real, out, ldo, sbits);
  return qvit_hip_status(hipGetLastError());
}

}  // namespace

extern "C" int qvit_ultra_weight_codes(const float* w, int64_t cout, int64_t cin, int64_t ks, int w_bit,
                                       int8_t* codes, int64_t kpad, int64_t cout_pad, float* values,
                                       unsigned* workspace, hipStream_t stream) {
  if (!w || !codes || !workspace) return QVIT_ENULL;
  if (cout <= 0 || cin <= 0 || ks <= 0 || cout_pad < cout || kpad < ks * ks * cin) return QVIT_EINVAL;
  if (w_bit < 2 || w_bit > 8) return QVIT_EINVAL;  // quant_ultra.py:33 (1 and 32 are not integer paths)
  if (cout_pad * kpad > INT32_MAX) return QVIT_EINVAL;
  const int64_t n = cout * cin * ks * ks;
  hipError_t e = hipMemsetAsync(workspace, 0, sizeof(unsigned), stream);
  if (e != hipSuccess) return qvit_hip_status(e);
  hipLaunchKernelGGL(ultra_wmax_kernel, dim3(grid_cap(n)), dim3(256), 0, stream, w, n, workspace);
  hipLaunchKernelGGL(ultra_wcodes_kernel, dim3(grid_cap(cout_pad * kpad)), dim3(256), 0, stream, w, (int)cout,
                     (int)cin, (int)ks, workspace, (float)((1 << (w_bit - 1)) - 1), codes, (int)kpad, (int)cout_pad,
                     values);
  return qvit_hip_status(hipGetLastError());
}

extern "C" int qvit_ultra_bn_fold(const float* gamma, const float* beta, const float* mean, const float* var,
                                  float eps, int64_t n, float* alpha, float* shift, hipStream_t stream) {
  if (!mean || !var || !alpha || !shift) return QVIT_ENULL;
  if (n <= 0 || n > (1 << 20)) return QVIT_EINVAL;
  hipLaunchKernelGGL(ultra_bn_fold_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, gamma, beta, mean,
                     var, eps, (int)n, alpha, shift);
  return qvit_hip_status(hipGetLastError());
}

extern "C" int qvit_ultra_conv0(const float* img, int64_t B, int64_t H, int64_t W, const float* wvals,
                                const float* alpha, const float* shift, int a_bit, int8_t* out, hipStream_t stream) {
  if (!img || !wvals || !alpha || !shift || !out) return QVIT_ENULL;
  if (B < 0 || H < 2 || W < 2 || a_bit < 1 || a_bit > 7) return QVIT_EINVAL;
  if ((((uintptr_t)out) & 15)) return QVIT_EALIGN;
  if (B * H * W > INT32_MAX) return QVIT_EINVAL;
  if (B == 0) return QVIT_OK;
  const int64_t work = B * (H / 2) * (W / 2);
  hipLaunchKernelGGL(ultra_conv0_kernel, dim3(grid_cap(work)), dim3(256), 0, stream, img, (int)B, (int)H, (int)W,
                     wvals, alpha, shift, (float)((1 << a_bit) - 1), out);
  return qvit_hip_status(hipGetLastError());
}

extern "C" int qvit_ultra_conv(const int8_t* in, int64_t B, int64_t H, int64_t W, int64_t cin, int64_t ks,
                               const int8_t* wcodes, int64_t kpad, int64_t cout, int w_bit, int a_bit,
                               const float* alpha, const float* shift, int mode, void* out, int64_t ldo,
                               hipStream_t stream) {
  if (!in || !wcodes || !shift || !out) return QVIT_ENULL;
  if (B < 0 || H < 1 || W < 1 || cout < 1 || ldo < cout || w_bit < 2 || w_bit > 8 || a_bit < 1 || a_bit > 7)
    return QVIT_EINVAL;
  if (mode != QVIT_ULTRA_CODES && mode != QVIT_ULTRA_CODES_POOL && mode != QVIT_ULTRA_F32) return QVIT_EINVAL;
  if (mode != QVIT_ULTRA_F32 && !alpha) return QVIT_ENULL;
  if (mode == QVIT_ULTRA_CODES_POOL && ((H | W) & 1)) return QVIT_EINVAL;
  if ((((uintptr_t)in) & 15) || (((uintptr_t)wcodes) & 15) || (kpad % 16)) return QVIT_EALIGN;
  if (mode != QVIT_ULTRA_F32 && (ldo % 4 || (((uintptr_t)out) & 3) || cout % 4)) return QVIT_EALIGN;
  if (B * H * W > INT32_MAX) return QVIT_EINVAL;
  if (B == 0) return QVIT_OK;
  const float den = (float)(((1 << (w_bit - 1)) - 1) * ((1 << a_bit) - 1));
  const float lv = (float)((1 << a_bit) - 1);
  const int b = (int)B, h = (int)H, w = (int)W, co = (int)cout, ld = (int)ldo, kp = (int)kpad;
#define QVIT_ULTRA_CASE(CI, K, CO)                                                                                  \
  if (cin == CI && ks == K && cout <= CO && cout > CO - 16) {                                                     \
    if (mode == QVIT_ULTRA_CODES_POOL)                                                                            \
      return launch_conv<CI, K, CO, 1, 0>(in, b, h, w, wcodes, kp, den, alpha, shift, lv, co, out, ld, stream);    \
    if (mode == QVIT_ULTRA_CODES)                                                                                 \
      return launch_conv<CI, K, CO, 0, 0>(in, b, h, w, wcodes, kp, den, alpha, shift, lv, co, out, ld, stream);    \
    return launch_conv<CI, K, CO, 0, 1>(in, b, h, w, wcodes, kp, den, alpha, shift, lv, co, out, ld, stream);      \
  }
  QVIT_ULTRA_CASE(16, 3, 32)
  QVIT_ULTRA_CASE(32, 3, 64)
  QVIT_ULTRA_CASE(64, 3, 64)
  QVIT_ULTRA_CASE(64, 1, 48)
#undef QVIT_ULTRA_CASE
  return QVIT_EINVAL;  // shapes outside UltraNetQua's layer set
}

extern "C" int qvit_ultra_conv0_int(const uint8_t* img, int64_t B, int64_t H, int64_t W, const int8_t* wcodes,
                                    const int32_t* inc, const int32_t* bias, int shift_bits, int out_bit, int8_t* out,
                                    hipStream_t stream) {
  if (!img || !wcodes || !inc || !bias || !out) return QVIT_ENULL;
  if (B < 0 || H < 2 || W < 2 || shift_bits < 1 || shift_bits > 40 || out_bit < 1 || out_bit > 7) return QVIT_EINVAL;
  if ((((uintptr_t)out) & 15)) return QVIT_EALIGN;
  if (B * H * W > INT32_MAX) return QVIT_EINVAL;
  if (B == 0) return QVIT_OK;
  const int64_t work = B * (H / 2) * (W / 2);
  hipLaunchKernelGGL(ultra_conv0_int_kernel, dim3(grid_cap(work)), dim3(256), 0, stream, img, (int)B, (int)H, (int)W,
                     wcodes, inc, bias, shift_bits, (1 << out_bit) - 1, out);
  return qvit_hip_status(hipGetLastError());
}

extern "C" int qvit_ultra_conv_int(const int8_t* in, int64_t B, int64_t H, int64_t W, int64_t cin, int64_t ks,
                                   const int8_t* wcodes, int64_t kpad, int64_t cout, const int32_t* inc,
                                   const int32_t* bias, int shift_bits, int out_bit, int pool, int8_t* out, int64_t ldo,
                                   hipStream_t stream) {
  if (!in || !wcodes || !inc || !bias || !out) return QVIT_ENULL;
  if (B < 0 || H < 1 || W < 1 || cout < 1 || ldo < cout || shift_bits < 1 || shift_bits > 40 || out_bit < 1 ||
      out_bit > 7)
    return QVIT_EINVAL;
  if (pool && ((H | W) & 1)) return QVIT_EINVAL;
  if ((((uintptr_t)in) & 15) || (((uintptr_t)wcodes) & 15) || (kpad % 16)) return QVIT_EALIGN;
  if (ldo % 4 || (((uintptr_t)out) & 3) || cout % 4 || (((uintptr_t)inc) & 3) || (((uintptr_t)bias) & 3))
    return QVIT_EALIGN;
  if (B * H * W > INT32_MAX) return QVIT_EINVAL;
  if (B == 0) return QVIT_OK;
  const float lv = (float)((1 << out_bit) - 1);
  const float* fi = reinterpret_cast<const float*>(inc);
  const float* fb = reinterpret_cast<const float*>(bias);
  const int b = (int)B, h = (int)H, w = (int)W, co = (int)cout, ld = (int)ldo, kp = (int)kpad;
#define QVIT_ULTRA_INT_CASE(CI, K, CO)                                                                               \
  if (cin == CI && ks == K && cout <= CO && cout > CO - 16) {                                                      \
    if (pool)                                                                                                      \
      return launch_conv<CI, K, CO, 1, 2>(in, b, h, w, wcodes, kp, 1.f, fi, fb, lv, co, out, ld, stream, shift_bits); \
    return launch_conv<CI, K, CO, 0, 2>(in, b, h, w, wcodes, kp, 1.f, fi, fb, lv, co, out, ld, stream, shift_bits);   \
  }
  QVIT_ULTRA_INT_CASE(16, 3, 32)
  QVIT_ULTRA_INT_CASE(32, 3, 64)
  QVIT_ULTRA_INT_CASE(64, 3, 64)
#undef QVIT_ULTRA_INT_CASE
  return QVIT_EINVAL;  // shapes outside UltraNetQua's quantized layer set
}

extern "C" int qvit_yolo_decode(const float* head, int64_t B, int64_t ny, int64_t nx, int64_t na, int64_t no,
                                int64_t ldh, const float* anchors, float stride, float* io, float* p,
                                hipStream_t stream) {
  if (!head || !anchors || !io || !p) return QVIT_ENULL;
  if (B < 0 || ny < 1 || nx < 1 || na < 1 || no < 5 || ldh < na * no || !(stride > 0.f)) return QVIT_EINVAL;
  if (B == 0) return QVIT_OK;
  hipLaunchKernelGGL(yolo_decode_kernel, dim3(grid_cap(B * na * ny * nx * no)), dim3(256), 0, stream, head, (int)B,
                     (int)ny, (int)nx, (int)na, (int)no, (int)ldh, anchors, stride, io, p);
  return qvit_hip_status(hipGetLastError());
}
