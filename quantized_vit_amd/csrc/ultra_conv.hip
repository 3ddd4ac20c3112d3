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
//   ultra_conv0_mfma          : layer 0 (float image input, 3 -> 16, 3x3): implicit GEMM on
//                               v_mfma_f32_16x16x32_f16 with fp16 hi/lo operand splits (fp32-class products),
//                               fused BN + quantizer + 2x2 max pool; NCHW in, NHWC codes out.
//   ultra_conv0_int_mfma      : the same layer of the integer deploy (uint8 image) on v_mfma_i32_16x16x64_i8.
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

// acc / den for an integer accumulator |acc| < 2^24 and the small integer den = (2^(w-1) - 1)(2^a - 1): the
// reciprocal product with one exact FMA residual correction (3 VALU instead of the IEEE divide's ~10); the
// per-layer kernels and the fused tail use the same form, so their codes agree bit for bit
QVIT_DEV float acc_div(int acc, float den, float rden) {
  const float x = (float)acc;
  const float q0 = x * rden;
  return fmaf(fmaf(-q0, den, x), rden, q0);
}

QVIT_DEV int act_code(float x, float alpha, float shift, float levels) {
  const float y = __fadd_rn(__fmul_rn(x, alpha), shift);
  return (int)rintf(fminf(fmaxf(y, 0.f), 1.f) * levels);
}

// ---- layer 0: 3 -> 16 channels, 3x3 pad 1, BN + quantizer + 2x2 pool -------------------------------
constexpr int C0_OUT = 16;

// ---- layer 0 on the matrix cores --------------------------------------------------------------------
// The same conv as an implicit GEMM on v_mfma_f32_16x16x32_f16: A = 16 pixels (a 4x4 patch) x K taps, B = K x
// the 16 output channels' weights, D[pixel][channel]. fp32 operands are exact sums of two fp16
// (x = hi + lo, hi = RNE f16 of x, lo = RNE f16 of the exact x - hi: 22 significant bits) and the conv is
// hi.hi + hi.lo + lo.hi with fp32 accumulation — the fp32 conv to ~2^-22 relative (the dropped lo.lo term),
// the order of the 27-term sum aside. K order: 8-value groups g = lane >> 4 of two 4-channel pixel records (tap
// (ky, kx); channel 3 a zero-weight pad). Chunk 0 = the 8 taps other than (2, 2): g < 3 = row g, kx 0 and 1;
// g = 3 = kx 2, rows 0 and 1; its three passes are three MFMAs. Chunk 1 = tap (2, 2) with all three passes in one
// MFMA: g = 0 is (x hi, x lo) against (w hi, w hi), g = 1 is (x hi, -) against (w lo, 0), g = 2, 3 zero weights.
// 4 MFMAs per patch. (v_mfma_f32_16x16x16_f16 for a half-empty chunk gave wrong accumulator reads: the compiler
// placed VALU reads of its result too early on gfx950.) The image tile is
// staged once per tile as fp16 hi / lo planes of 4-channel pixels (8 B), so every pixel fragment is two 8-B LDS
// reads and the hi / lo split runs once per input pixel instead of once per tap. The patch's row order puts
// one 2x2 pool window in each lane's four D rows (row 4 G + j = window G, position j), so lane (window G,
// channel n) pools in registers: BN is monotone in the accumulator (increasing for alpha >= 0, decreasing
// below), so the pooled BN output is BN of the max (or min) accumulator, and the quantizer (monotone) runs
// once per pooled value — the same code as pooling the four codes.
// Tile staging: halo row hy = image row ty0 - 1 + hy, halo column hx = image column tx0 - 4 + hx (40 columns:
// the conv reads hx = 3 .. 37), loaded as 4-pixel quads (one float4 / uchar4 per channel: 18 x 10 quads, one per
// thread of the first 180) and written as four 4-channel pixel records.
constexpr int C0_TY = 16, C0_TX = 32;                 // pre-pool output tile
constexpr int C0_HY = C0_TY + 2, C0_HX = C0_TX + 8;   // halo rows, columns
constexpr int C0_HPIX = C0_HY * C0_HX;
constexpr int C0_PLANE = C0_HPIX * 8;                 // fp16 x 4 channels per pixel
constexpr int C0_QUADS = C0_HY * C0_HX / 4;           // 180 <= 256
static_assert(C0_QUADS <= 256, "one quad per thread");
typedef _Float16 c0h8 __attribute__((ext_vector_type(8)));
typedef _Float16 c0h4 __attribute__((ext_vector_type(4)));
typedef float c0f4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

QVIT_DEV float fmax_nn(float a, float b) { return __builtin_elementwise_maximum(a, b); }
// Tiles of this persistent block: with a grid that is a multiple of 8, XCD x (blocks x, x + 8, ...) owns a
// contiguous tile range, so the tiles in flight on one XCD are neighbours whose halo rows share 128-B lines
// in that XCD's L2 (walking t = blockIdx + k grid put x-neighbours on different XCDs: layer 0 fetched 3.2x
// its input from HBM). Tile k of this block: lo + slot + k team while < hi.
struct TileWalk {
  int lo, hi, slot, team;
};
QVIT_DEV TileWalk tile_walk(int ntiles) {
  TileWalk w{0, ntiles, (int)blockIdx.x, (int)gridDim.x};
  if ((gridDim.x & 7) == 0) {
    const int xcd = blockIdx.x & 7, per = ntiles >> 3, rem = ntiles & 7;
    w.lo = xcd * per + (xcd < rem ? xcd : rem);
    w.hi = w.lo + per + (xcd < rem ? 1 : 0);
    w.slot = blockIdx.x >> 3;
    w.team = gridDim.x >> 3;
  }
  return w;
}
QVIT_DEV _Float16 hi_h(float x) { return (_Float16)x; }
// codes of lanes 4k .. 4k + 3 (channels n .. n + 3) as one word in lane 4k (DPP quad permutes)
QVIT_DEV uint32_t pack_quad(int code) {
  const uint32_t c1 = (uint32_t)__builtin_amdgcn_update_dpp(0, code, 0x39, 0xf, 0xf, false);  // quad lane + 1
  const uint32_t c2 = (uint32_t)__builtin_amdgcn_update_dpp(0, code, 0x4E, 0xf, 0xf, false);  // + 2
  const uint32_t c3 = (uint32_t)__builtin_amdgcn_update_dpp(0, code, 0x93, 0xf, 0xf, false);  // + 3
  return ((uint32_t)code & 0xff) | ((c1 & 0xff) << 8) | ((c2 & 0xff) << 16) | (c3 << 24);
}
QVIT_DEV _Float16 lo_h(float x) { return (_Float16)(x - (float)(_Float16)x); }  // x - hi is exact in fp32

// patches per MFMA group and workgroups per CU of the layer-0 kernel: one patch at a time holds 64 VGPRs, so
// LDS (23 KiB per workgroup) rather than registers bounds residency at 7 workgroups per CU; 4 patches per group
// at 4 workgroups per CU (round-3 build): 344-353 us vs 283-286 us at b256 (profiles/r03_conv0_occupancy_ab.txt)
constexpr int C0_G = 1;     // patches per MFMA group
constexpr int C0_WAVE_OUT = 2 * (C0_TX / 2) * C0_OUT;  // a wave's pooled codes per tile: 512 B
constexpr int C0_OCC = 6;   // workgroups per CU
template <bool VEC>
__global__ __launch_bounds__(256, C0_OCC) void ultra_conv0_mfma_kernel(const float* __restrict__ img, int B, int H, int W,
                                                               const float* __restrict__ wvals,
                                                               const float* __restrict__ alpha,
                                                               const float* __restrict__ shift, float levels,
                                                               int8_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) int8_t smem[2][2 * C0_PLANE];
  __shared__ __attribute__((aligned(16))) int8_t codes_l[4][C0_WAVE_OUT];  // each wave's pooled codes of a tile
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n = lane & 15, g = lane >> 4;
  // A row n = pixel (2 ((n >> 2) >> 1) + ((n & 3) >> 1), 2 ((n >> 2) & 1) + (n & 1)) of the 4x4 patch
  const int py = 2 * (n >> 3) + ((n >> 1) & 1), px = 2 * ((n >> 2) & 1) + (n & 1);
  const int Ho = H / 2, Wo = W / 2;
  // this lane's code byte of patch pq: pooled row g >> 1, pooled column 2 pq + (g & 1), channel n
  int8_t* cw = codes_l[wave] + ((g >> 1) * (C0_TX / 2) + (g & 1)) * C0_OUT + n;

  // B operands: weights [o = n][c][ky][kx] split hi / lo in the K order above; record r (0, 1) of group g is tap
  // (ky, kx) = g < 3 ? (g, r) : (r, 2)
  // A channel whose BN decreases in the accumulator (alpha < 0) gets its B column negated: the hi / lo split
  // and every product and sum are sign-symmetric, so its accumulators come out exactly negated, the max of
  // them is minus the min of the true ones, and (-alpha) (-min) = alpha min. One max pool for every lane.
  const float al = alpha[n], sh = shift[n];
  const bool up = !(al < 0.f);  // BN increasing in the accumulator
  const float alp = up ? al : -al;
  c0h8 wh0, wl0, wc1;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int r = j >> 2, c = j & 3;
    const int ky = g < 3 ? g : r, kx = g < 3 ? r : 2;
    const float w = c < 3 ? wvals[((n * 3 + c) * 3 + ky) * 3 + kx] : 0.f;
    wh0[j] = up ? hi_h(w) : -hi_h(w);
    wl0[j] = up ? lo_h(w) : -lo_h(w);
    const float w22 = c < 3 ? wvals[((n * 3 + c) * 3 + 2) * 3 + 2] : 0.f;
    const _Float16 c1 = g == 0 ? hi_h(w22) : (g == 1 && r == 0) ? lo_h(w22) : (_Float16)0;
    wc1[j] = up ? c1 : -c1;
  }
  // both BN constants arrive here, before the loop: a use inside the loop would otherwise carry a vmcnt(0) that
  // also drains the next tile's halo prefetch at the first patch
  asm volatile("" ::"v"(alp), "v"(sh));

  const int tiles_y = (H + C0_TY - 1) / C0_TY, tiles_x = (W + C0_TX - 1) / C0_TX;
  const int ntiles = B * tiles_y * tiles_x;
  const int64_t HW = (int64_t)H * W;
  // tile t = (b tiles_y + ty) tiles_x + tx as (b, ty, tx); the walk advances t by a fixed team, so the
  // coordinates advance by the team's own with carries (no division per tile)
  struct TPos {
    int b, ty, tx;
  };
  auto tpos = [&](int t) __attribute__((always_inline)) {
    const int row = t / tiles_x;
    return TPos{row / tiles_y, row - (row / tiles_y) * tiles_y, t - row * tiles_x};
  };
  // this thread's halo quad (hy, 4 qx .. 4 qx + 3) of tile t -> registers (zero outside the image)
  const int qy = tid / (C0_HX / 4), qx = tid - qy * (C0_HX / 4);
  c0f4 xin[3];
  auto load_tile = [&](const TPos& p) __attribute__((always_inline)) {
    if (tid >= C0_QUADS) return;
    const int b = p.b, ty0 = p.ty * C0_TY, tx0 = p.tx * C0_TX;
    const float* base = img + (int64_t)b * 3 * HW;
    const int y = ty0 - 1 + qy, x = tx0 - 4 + 4 * qx;
    const bool row = y >= 0 && y < H;
    if (VEC) {  // W % 4 == 0: a quad is wholly inside or outside the row
      const bool ok = row && x >= 0 && x < W;
      const int64_t off = ok ? (int64_t)y * W + x : 0;
#pragma unroll
      for (int c = 0; c < 3; ++c)
        xin[c] = ok ? *reinterpret_cast<const c0f4*>(base + c * HW + off) : c0f4{0.f, 0.f, 0.f, 0.f};
    } else {
#pragma unroll
      for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool ok = row && x + e >= 0 && x + e < W;
          xin[c][e] = ok ? base[c * HW + (int64_t)y * W + x + e] : 0.f;
        }
    }
  };
  auto stage_tile = [&](int8_t* buf) __attribute__((always_inline)) {
    if (tid >= C0_QUADS) return;
    c0h8 hi[2], lo[2];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        hi[e >> 1][4 * (e & 1) + c] = hi_h(xin[c][e]);
        lo[e >> 1][4 * (e & 1) + c] = lo_h(xin[c][e]);
      }
      hi[e >> 1][4 * (e & 1) + 3] = 0;
      lo[e >> 1][4 * (e & 1) + 3] = 0;
    }
    int8_t* d = buf + 32 * tid;  // pixel (qy, 4 qx) = halo pixel 4 tid
    *reinterpret_cast<c0h8*>(d) = hi[0];
    *reinterpret_cast<c0h8*>(d + 16) = hi[1];
    *reinterpret_cast<c0h8*>(d + C0_PLANE) = lo[0];
    *reinterpret_cast<c0h8*>(d + C0_PLANE + 16) = lo[1];
  };

  const TileWalk tw = tile_walk(ntiles);
  int t = tw.lo + tw.slot;
  if (t >= tw.hi) return;
  TPos cur = tpos(t);
  const TPos step = tpos(tw.team);
  auto advance = [&](TPos p) __attribute__((always_inline)) {
    p.tx += step.tx;
    if (p.tx >= tiles_x) p.tx -= tiles_x, p.ty += 1;
    p.ty += step.ty;
    if (p.ty >= tiles_y) p.ty -= tiles_y, p.b += 1;
    p.b += step.b;
    return p;
  };
  load_tile(cur);
  stage_tile(smem[0]);
  __syncthreads();
  // the wave's pooled codes of a tile (2 rows x 16 columns x 16 channels) leave as 16-B pixels, 16 lanes per
  // 256-B output row; the wave reads back only what it wrote (its LDS operations complete in order). Issued
  // after the next tile's halo loads: a store ahead of them would make their issue wait for its completion.
  auto flush = [&](int b, int ty0, int tx0) __attribute__((always_inline)) {
    __builtin_amdgcn_wave_barrier();
    if (lane < 32) {
      const int yo = ((ty0 + 4 * wave) >> 1) + (lane >> 4), xo = (tx0 >> 1) + (lane & 15);
      const uint4 v = *reinterpret_cast<const uint4*>(codes_l[wave] + lane * C0_OUT);
      if (yo < Ho && xo < Wo) *reinterpret_cast<uint4*>(out + (((int64_t)b * Ho + yo) * Wo + xo) * C0_OUT) = v;
    }
    __builtin_amdgcn_wave_barrier();
  };
  int pb = 0, pty = 0, ptx = 0;  // the previous tile, its codes still in codes_l
  for (int it = 0; t < tw.hi; t += tw.team, ++it) {
    const int8_t* buf = smem[it & 1];
    const int tn = t + tw.team;
    const TPos nxt = advance(cur);
    if (tn < tw.hi) load_tile(nxt);  // lands while this tile computes
    if (it > 0) flush(pb, pty, ptx);
    const int b = cur.b, ty0 = cur.ty * C0_TY, tx0 = cur.tx * C0_TX;
    pb = b, pty = ty0, ptx = tx0;
    cur = nxt;
    // A fragment records (halo pixel of tap (ky, kx): row 4 wave + py + ky, column px + kx + 3, + 4 per patch):
    // chunk 0 records r0, r1 of group g; chunk 1 = tap (2, 2) hi, then its lo (g = 0) or hi again
    auto rec = [&](int ky, int kx) { return buf + ((4 * wave + py + ky) * C0_HX + px + kx + 3) * 8; };
    const int8_t* r0 = g < 3 ? rec(g, 0) : rec(0, 2);
    const int8_t* r1 = g < 3 ? rec(g, 1) : rec(1, 2);
    const int8_t* c0 = rec(2, 2);
    const int8_t* c1 = rec(2, 2) + (g == 0 ? C0_PLANE : 0);
    // C0_G patches at a time (their MFMA chains interleaved; with one, the other resident waves cover the
    // chain latency)
#pragma unroll
    for (int pq = 0; pq < C0_TX / 4; pq += C0_G) {
      c0h8 h0[C0_G], l0[C0_G], x1[C0_G];
      c0f4 acc[C0_G];
      auto pair = [](const int8_t* a, const int8_t* b) {
        return __builtin_shufflevector(*reinterpret_cast<const c0h4*>(a), *reinterpret_cast<const c0h4*>(b), 0, 1, 2, 3,
                                       4, 5, 6, 7);
      };
#pragma unroll
      for (int q = 0; q < C0_G; ++q) {
        const int o = 32 * (pq + q);
        h0[q] = pair(r0 + o, r1 + o);
        l0[q] = pair(r0 + C0_PLANE + o, r1 + C0_PLANE + o);
        x1[q] = pair(c0 + o, c1 + o);
        acc[q] = c0f4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int q = 0; q < C0_G; ++q) acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(h0[q], wh0, acc[q], 0, 0, 0);
#pragma unroll
      for (int q = 0; q < C0_G; ++q) acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(x1[q], wc1, acc[q], 0, 0, 0);
#pragma unroll
      for (int q = 0; q < C0_G; ++q) acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(l0[q], wh0, acc[q], 0, 0, 0);
#pragma unroll
      for (int q = 0; q < C0_G; ++q) acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(h0[q], wl0, acc[q], 0, 0, 0);
      // acc[q][j] = conv[pixel 4 g + j of patch pq + q][channel n]: window g's four pixels
#pragma unroll
      for (int q = 0; q < C0_G; ++q) {
        const float mx = fmax_nn(fmax_nn(acc[q][0], acc[q][1]), fmax_nn(acc[q][2], acc[q][3]));
        const float y = __fadd_rn(__fmul_rn(mx, alp), sh);
        const int code = (int)rintf(__builtin_amdgcn_fmed3f(y, 0.f, 1.f) * levels);
        cw[2 * (pq + q) * C0_OUT] = (int8_t)code;
      }
      // one patch at a time (without the fence the scheduler hoists later patches' fragment reads: spills)
      __builtin_amdgcn_sched_barrier(0);
    }
    if (tn < tw.hi) stage_tile(smem[(it + 1) & 1]);  // the other buffer: its last reader finished a barrier ago
    __syncthreads();
  }
  flush(pb, pty, ptx);
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

// Layer 0 of the integer deploy on v_mfma_i32_16x16x64_i8: the same tiling, pixel order and in-lane pool as
// ultra_conv0_mfma_kernel, exact in int32. The uint8 image is staged as x - 128 (int8, 4-channel pixels), and
// 128 * sum(w) per channel is added back to the accumulator; K = one 64-deep chunk, group g = kernel row g
// (g < 3; group 3 zero weights), 16 values = kx 0..3 x c 0..3 (kx = 3, c = 3 zero-weight pads). The 2x2 pool
// takes the max (inc >= 0) or min (inc < 0) accumulator before the threshold, which is monotone in acc * inc.
constexpr int C0I_PLANE = C0_HPIX * 4;  // int8 x 4 channels per pixel

template <bool VEC>
__global__ __launch_bounds__(256, 4) void ultra_conv0_int_mfma_kernel(const uint8_t* __restrict__ img, int B, int H,
                                                                   int W, const int8_t* __restrict__ wcodes,
                                                                   const int* __restrict__ inc,
                                                                   const int* __restrict__ bias, int sbits,
                                                                   int levels, int8_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) int8_t smem[2][C0I_PLANE];
  __shared__ __attribute__((aligned(16))) int8_t codes_l[4][C0_WAVE_OUT];  // each wave's pooled codes of a tile
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n = lane & 15, g = lane >> 4;
  const int py = 2 * (n >> 3) + ((n >> 1) & 1), px = 2 * ((n >> 2) & 1) + (n & 1);  // A row n (as the float kernel)
  const int Ho = H / 2, Wo = W / 2;
  int8_t* cw = codes_l[wave] + ((g >> 1) * (C0_TX / 2) + (g & 1)) * C0_OUT + n;  // as the float kernel

  v4i wa;  // B operand: channel n, kernel row g, (kx, c) = (i >> 2, i & 3) for byte i
  {
    int8_t wb[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int kx = i >> 2, c = i & 3;
      wb[i] = (g < 3 && kx < 3 && c < 3) ? wcodes[((n * 3 + c) * 3 + g) * 3 + kx] : (int8_t)0;
    }
    wa = __builtin_bit_cast(v4i, wb);
  }
  // 128 sum(w) of channel n: the MFMA of an all-ones A with the weights
  const v4i ones = v4i{0x01010101, 0x01010101, 0x01010101, 0x01010101};
  const int wsum = 128 * __builtin_amdgcn_mfma_i32_16x16x64_i8(ones, wa, v4i{0, 0, 0, 0}, 0, 0, 0)[0];
  const int ic = inc[n], bc = bias[n];
  asm volatile("" ::"v"(ic), "v"(bc));  // both arrive before the loop (see the float kernel)

  const int tiles_y = (H + C0_TY - 1) / C0_TY, tiles_x = (W + C0_TX - 1) / C0_TX;
  const int ntiles = B * tiles_y * tiles_x;
  const int64_t HW = (int64_t)H * W;
  struct TPos {
    int b, ty, tx;
  };
  auto tpos = [&](int t) __attribute__((always_inline)) {
    const int row = t / tiles_x;
    return TPos{row / tiles_y, row - (row / tiles_y) * tiles_y, t - row * tiles_x};
  };
  // this thread's halo quad (as the float kernel): per channel 4 bytes, staged as x - 128 in 4-channel pixels
  const int qy = tid / (C0_HX / 4), qx = tid - qy * (C0_HX / 4);
  uint32_t xin[3];
  auto load_tile = [&](const TPos& p) __attribute__((always_inline)) {
    if (tid >= C0_QUADS) return;
    const int b = p.b, ty0 = p.ty * C0_TY, tx0 = p.tx * C0_TX;
    const uint8_t* base = img + (int64_t)b * 3 * HW;
    const int y = ty0 - 1 + qy, x = tx0 - 4 + 4 * qx;
    const bool row = y >= 0 && y < H;
    if (VEC) {
      const bool ok = row && x >= 0 && x < W;
      const int64_t off = ok ? (int64_t)y * W + x : 0;
#pragma unroll
      for (int c = 0; c < 3; ++c) xin[c] = ok ? *reinterpret_cast<const uint32_t*>(base + c * HW + off) : 0u;
    } else {
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        uint32_t w = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool ok = row && x + e >= 0 && x + e < W;
          w |= (uint32_t)(ok ? base[c * HW + (int64_t)y * W + x + e] : 0) << (8 * e);
        }
        xin[c] = w;
      }
    }
  };
  auto stage_tile = [&](int8_t* buf) __attribute__((always_inline)) {
    if (tid >= C0_QUADS) return;
    // pixel e of the quad: bytes (c0, c1, c2, 0) - 128 each (the pad byte becomes 0 again below)
    v4i rec;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t p = ((xin[0] >> (8 * e)) & 0xff) | (((xin[1] >> (8 * e)) & 0xff) << 8) |
                         (((xin[2] >> (8 * e)) & 0xff) << 16);
      rec[e] = (int)((p ^ 0x00808080u));  // x - 128 as int8 == x ^ 0x80 for 0 <= x <= 255
    }
    *reinterpret_cast<v4i*>(buf + 16 * tid) = rec;
  };

  const TileWalk tw = tile_walk(ntiles);
  int t = tw.lo + tw.slot;
  if (t >= tw.hi) return;
  TPos cur = tpos(t);
  const TPos step = tpos(tw.team);
  auto advance = [&](TPos p) __attribute__((always_inline)) {
    p.tx += step.tx;
    if (p.tx >= tiles_x) p.tx -= tiles_x, p.ty += 1;
    p.ty += step.ty;
    if (p.ty >= tiles_y) p.ty -= tiles_y, p.b += 1;
    p.b += step.b;
    return p;
  };
  load_tile(cur);
  stage_tile(smem[0]);
  __syncthreads();
  auto flush = [&](int b, int ty0, int tx0) __attribute__((always_inline)) {  // as the float kernel
    __builtin_amdgcn_wave_barrier();
    if (lane < 32) {
      const int yo = ((ty0 + 4 * wave) >> 1) + (lane >> 4), xo = (tx0 >> 1) + (lane & 15);
      const uint4 v = *reinterpret_cast<const uint4*>(codes_l[wave] + lane * C0_OUT);
      if (yo < Ho && xo < Wo) *reinterpret_cast<uint4*>(out + (((int64_t)b * Ho + yo) * Wo + xo) * C0_OUT) = v;
    }
    __builtin_amdgcn_wave_barrier();
  };
  int pb = 0, pty = 0, ptx = 0;
  for (int it = 0; t < tw.hi; t += tw.team, ++it) {
    const int8_t* buf = smem[it & 1];
    const int tn = t + tw.team;
    const TPos nxt = advance(cur);
    if (tn < tw.hi) load_tile(nxt);
    if (it > 0) flush(pb, pty, ptx);
    pb = cur.b, pty = cur.ty * C0_TY, ptx = cur.tx * C0_TX;
    cur = nxt;
    // A fragment: pixels px .. px + 3 of kernel row g (group 3 re-reads row 2: zero weights)
    const int8_t* bb = buf + ((4 * wave + py + (g < 3 ? g : 2)) * C0_HX + px + 3) * 4;
#pragma unroll
    for (int pq = 0; pq < C0_TX / 4; pq += 2) {
      v4i acc[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(bb + 16 * (pq + q));
        const v4i xb = v4i{(int)src[0], (int)src[1], (int)src[2], (int)src[3]};
        acc[q] = __builtin_amdgcn_mfma_i32_16x16x64_i8(xb, wa, v4i{0, 0, 0, 0}, 0, 0, 0);
      }
      // acc[q][j] + 128 sum(w) = conv[pixel 4 g + j of patch pq + q][channel n]
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int mx = max(max(acc[q][0], acc[q][1]), max(acc[q][2], acc[q][3]));
        const int mn = min(min(acc[q][0], acc[q][1]), min(acc[q][2], acc[q][3]));
        cw[2 * (pq + q) * C0_OUT] = (int8_t)int_code((ic < 0 ? mn : mx) + wsum, ic, bc, sbits, levels);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (tn < tw.hi) stage_tile(smem[(it + 1) & 1]);
    __syncthreads();
  }
  flush(pb, pty, ptx);
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
// minimum resident workgroups per CU by input width (register budget): CIN 32 at 3 instead of 2 (168 VGPRs, no
// spills): conv2 114-116 -> 96-98 us at b256 (profiles/r03_conv0_occupancy_ab.txt)
constexpr int UC_MINB16 = 2, UC_MINB32 = 3;
// zeros for the LDS-DMA of halo pixels outside the image
__device__ __attribute__((aligned(16))) int4 qvit_ultra_zero16 = {0, 0, 0, 0};

// STG (pooled code layers whose output rows are whole 16-B groups, cout == COUT): the halo of tile t + 1 is
// LDS-DMA'd into the second halo buffer while tile t computes (no register staging: zeros for pixels outside
// the image come from a zero line), and the pooled codes leave through a per-wave LDS image as one 16-B
// buffer store per lane, so each wave has exactly one vector-memory operation younger than the halo it waits for.
template <int CIN, int KS, int COUT, int POOL, int OUT, bool STG>
__global__ __launch_bounds__(256, STG ? 2 : CIN == 32 ? UC_MINB32 : CIN == 16 ? UC_MINB16 : 2) void ultra_conv_kernel(const int8_t* __restrict__ in, int B, int H, int W,
                                                            const int8_t* __restrict__ wcodes, int kpad_in,
                                                            float den, const float* __restrict__ alpha,
                                                            const float* __restrict__ shift, float levels,
                                                            int cout_real, void* __restrict__ out, int ldo,
                                                            int sbits) {
  using G = ConvGeo<CIN, KS, COUT>;
  const float rden = 1.f / den;
  constexpr bool STAGED = STG && POOL != 0 && OUT != 1;
  constexpr int HALO16 = (G::HALO + 15) / 16 * 16;
  constexpr int WOUT = 2 * (TS / 2) * COUT;  // a wave's pooled codes per tile (2 rows x 8 columns)
  __shared__ __attribute__((aligned(16))) int8_t smem[COUT * G::WSTR + HALO16 + (STAGED ? HALO16 + 4 * WOUT : 0)];
  int8_t* wl = smem;
  int8_t* halo = smem + COUT * G::WSTR;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int p = lane & 15, g = lane >> 4;
  // SW (pooled code layers): pixels are the MFMA A rows in the order of ultra_conv0_mfma_kernel (row 4 G + j =
  // pool window G, position j), weights the B columns, so D[pixel][channel] puts each 2x2 window in one lane:
  // the pool runs in registers on the accumulators (BN and the quantizer are monotone in them) and the
  // quantizer once per pooled value. Otherwise A = weights, B = pixels (p = 4 py + px), D[channel][pixel].
  constexpr bool SW = POOL != 0 && OUT != 1;
  const int py = SW ? 2 * (p >> 3) + ((p >> 1) & 1) : p >> 2;
  const int px = SW ? 2 * ((p >> 2) & 1) + (p & 1) : p & 3;

  // weights -> LDS once per block (rows >= real cout are zero in the packed image). STAGED with the BN path
  // (OUT 0): the row of a channel whose BN decreases in the accumulator (alpha < 0) is stored negated (codes are
  // in [-127, 127]), so its accumulators come out exactly negated and the pooled BN input is their max for every
  // lane (acc_div is odd, and (-x)(-alpha) = x alpha): no min pool, no select (as ultra_conv0_mfma_kernel).
  // (The unstaged pooled form, UltraNet's CIN 64 layer, measured slower with it: +4 %, profiles/r06_ultranet_bn_sign_fold_ab.txt)
  constexpr bool NEG = STAGED && OUT == 0;
  static_assert(!NEG || COUT <= 64, "one channel per lane of the sign ballot");
  // bit o: channel o's BN decreases (one ballot per wave, so the staging loop reads no alpha)
  const uint64_t negmask = NEG ? __ballot(lane < cout_real && alpha[lane < cout_real ? lane : 0] < 0.f) : 0;
  for (int i = tid; i < COUT * (G::KPAD / 16); i += 256) {
    const int o = i / (G::KPAD / 16), c16 = i % (G::KPAD / 16);
    v4i w = *reinterpret_cast<const v4i*>(wcodes + (int64_t)o * kpad_in + 16 * c16);
    if (NEG && ((negmask >> o) & 1)) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {  // bytewise two's-complement negation: ~b + 1 without carries across bytes
        const uint32_t t = ~(uint32_t)w[k];
        w[k] = (int)(((t & 0x7f7f7f7fu) + 0x01010101u) ^ (t & 0x80808080u));
      }
    }
    *reinterpret_cast<v4i*>(wl + o * G::WSTR + 16 * c16) = w;
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
  // SW: this lane's channel 16 ct + p
  float als[G::NCT], shs[G::NCT];
  int iincs[G::NCT], ibiass[G::NCT];
#pragma unroll
  for (int ct = 0; ct < G::NCT; ++ct) {
    const int o = 16 * ct + p;
    als[ct] = (SW && OUT == 0 && o < cout_real) ? (NEG ? fabsf(alpha[o]) : alpha[o]) : 0.f;  // NEG: sign in the weights
    shs[ct] = (SW && OUT == 0 && o < cout_real) ? shift[o] : 0.f;
    iincs[ct] = (SW && OUT == 2 && o < cout_real) ? reinterpret_cast<const int*>(alpha)[o] : 0;
    ibiass[ct] = (SW && OUT == 2 && o < cout_real) ? reinterpret_cast<const int*>(shift)[o] : 0;
    // arrived before the loop: a first use inside it would carry a compiler vmcnt(0) that drains the halo DMA
    if (STG) asm volatile("" ::"v"(als[ct]), "v"(shs[ct]), "v"(iincs[ct]), "v"(ibiass[ct]));
  }

  const int tiles_y = (H + TS - 1) / TS, tiles_x = (W + TS - 1) / TS;
  const int64_t ntiles = (int64_t)B * tiles_y * tiles_x;
  const TileWalk tw = tile_walk((int)ntiles);

  // the implicit-GEMM contraction of one tile from the halo image hb
  auto conv_tile = [&](const int8_t* hb, v4i (&acc)[4][G::NCT]) __attribute__((always_inline)) {
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
        bf[pt] = *reinterpret_cast<const v4i*>(hb + (hy * G::HT + hx) * CIN + c0);
        if (!kv) bf[pt] = v4i{0, 0, 0, 0};
      }
#pragma unroll
      for (int pt = 0; pt < 4; ++pt)
#pragma unroll
        for (int ct = 0; ct < G::NCT; ++ct)
          acc[pt][ct] = SW ? __builtin_amdgcn_mfma_i32_16x16x64_i8(bf[pt], a[ct], acc[pt][ct], 0, 0, 0)
                           : __builtin_amdgcn_mfma_i32_16x16x64_i8(a[ct], bf[pt], acc[pt][ct], 0, 0, 0);
    }
  };

  if constexpr (STAGED) {
    int8_t* halo1 = halo + HALO16;
    int8_t* codes_w = halo1 + HALO16 + wave * WOUT;
    // DMA of tile t's halo into hb: 1-KiB pieces i = wave, wave + 4, ...; lane L of piece i fills bytes
    // 1024 i + 16 L of the image (hy, hx, channel chunk), past the image end the lanes are masked off
    constexpr int NPIECE = (G::HALO + 1023) / 1024;
    auto issue_halo = [&](int t, int8_t* hb) __attribute__((always_inline)) {
      const int row = t / tiles_x, b = row / tiles_y;
      const int tx0 = (t - row * tiles_x) * TS, ty0 = (row - b * tiles_y) * TS;
      const uint32_t lb = lds_addr(hb);
#pragma unroll
      for (int i = 0; i < NPIECE; ++i) {
        if ((i & 3) != wave) continue;  // wave-uniform
        const int o = 1024 * i + 16 * lane;
        if (o < G::HALO) {
          const int hy = o / (G::HT * CIN), r = o - hy * (G::HT * CIN);
          const int hx = r / CIN, c = r - hx * CIN;
          const int y = ty0 - KS / 2 + hy, x = tx0 - KS / 2 + hx;
          const void* src = (y >= 0 && y < H && x >= 0 && x < W)
                                ? static_cast<const void*>(in + (((int64_t)b * H + y) * W + x) * CIN + c)
                                : static_cast<const void*>(&qvit_ultra_zero16);
          dma16(src, __builtin_amdgcn_readfirstlane(lb + 1024 * i));
        }
      }
    };
    const int Ho = H / 2, Wo = W / 2;
    // this lane's code byte for (patch pt, channel tile ct): pooled row g >> 1, column 2 pt + (g & 1), channel
    // 16 ct + p; the flush: lane l stores channels 16 (l % (COUT / 16)) .. + 15 of pooled pixel l / (COUT / 16)
    int8_t* cw = codes_w + ((g >> 1) * (TS / 2) + (g & 1)) * COUT + p;
    constexpr int CG = COUT / 16;  // 16-B groups per pooled pixel
    int t = tw.lo + tw.slot;
    if (t < tw.hi) issue_halo(t, halo);
    for (int it = 0; t < tw.hi; t += tw.team, ++it) {
      // tile t's halo landed for every wave (the only younger operation of a wave is its previous flush store),
      // every wave is done with the other buffer (the previous tile) and with its codes image
      __builtin_amdgcn_s_waitcnt(0xC07F);
      if (it == 0) asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(1)\n\ts_barrier" ::: "memory");
      const int tn = t + tw.team;
      if (tn < tw.hi) issue_halo(tn, (it & 1) ? halo : halo1);
      const int row = t / tiles_x, b = row / tiles_y;
      const int tx0 = (t - row * tiles_x) * TS, ty0 = (row - b * tiles_y) * TS;
      v4i acc[4][G::NCT];
      conv_tile((it & 1) ? halo1 : halo, acc);
#pragma unroll
      for (int pt = 0; pt < 4; ++pt)
#pragma unroll
        for (int ct = 0; ct < G::NCT; ++ct) {
          const v4i v = acc[pt][ct];
          const int vmax = max(max(v[0], v[1]), max(v[2], v[3]));
          const int vmin = min(min(v[0], v[1]), min(v[2], v[3]));
          const int code = (OUT == 2) ? int_code(iincs[ct] < 0 ? vmin : vmax, iincs[ct], ibiass[ct], sbits, (int)levels)
                                      : act_code(acc_div(NEG || !(als[ct] < 0.f) ? vmax : vmin, den, rden), als[ct], shs[ct], levels);
          cw[2 * pt * COUT + 16 * ct] = (int8_t)code;
        }
      __builtin_amdgcn_wave_barrier();
      {
        const int q = lane / CG, cc = lane - q * CG;  // pooled pixel q (row q >> 3, column q & 7), group cc
        const int yo = ((ty0 + 4 * wave) >> 1) + (q >> 3), xo = (tx0 >> 1) + (q & 7);
        const bool ok = lane < 16 * CG && yo < Ho && xo < Wo;
        const v4i v = ok ? *reinterpret_cast<const v4i*>(codes_w + lane * 16) : v4i{0, 0, 0, 0};
        int8_t* ob = reinterpret_cast<int8_t*>(out) + (int64_t)b * Ho * Wo * ldo;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(ob, (short)0, Ho * Wo * ldo, 0x00020000);
        const int off = ok ? (yo * Wo + xo) * ldo + 16 * cc : (int)0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, off, 0, 0);
      }
      __builtin_amdgcn_wave_barrier();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return;
  }

  for (int64_t t = tw.lo + tw.slot; t < tw.hi; t += tw.team) {
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
    conv_tile(halo, acc);

    if constexpr (SW) {
      // acc[pt][ct][j] = conv[b][cout 16 ct + p][pool window g of patch pt, position j]
      const int Ho = H / 2, Wo = W / 2;
      const int yo = ((ty0 + 4 * wave) >> 1) + (g >> 1);
#pragma unroll
      for (int pt = 0; pt < 4; ++pt) {
        const int xo = ((tx0 + 4 * pt) >> 1) + (g & 1);
#pragma unroll
        for (int ct = 0; ct < G::NCT; ++ct) {
          const v4i v = acc[pt][ct];
          const int vmax = max(max(v[0], v[1]), max(v[2], v[3]));
          const int vmin = min(min(v[0], v[1]), min(v[2], v[3]));
          const int code = (OUT == 2) ? int_code(iincs[ct] < 0 ? vmin : vmax, iincs[ct], ibiass[ct], sbits, (int)levels)
                                      : act_code(acc_div(NEG || !(als[ct] < 0.f) ? vmax : vmin, den, rden), als[ct], shs[ct], levels);
          const uint32_t word = pack_quad(code);  // channels 16 ct + p .. + 3 in lane p = 4k
          const int o = 16 * ct + p;
          if ((p & 3) == 0 && yo < Ho && xo < Wo && o < cout_real)
            *reinterpret_cast<uint32_t*>(reinterpret_cast<int8_t*>(out) + (((int64_t)b * Ho + yo) * Wo + xo) * ldo + o) =
                word;
        }
      }
      continue;
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
              if (o0 + j < cout_real) dst[o0 + j] = __fadd_rn(acc_div(acc[pt][ct][j], den, rden), sh[ct][j]);
          }
        } else {
          int code[4];
#pragma unroll
          for (int j = 0; j < 4; ++j)
            code[j] = (OUT == 2) ? int_code(acc[pt][ct][j], iinc[ct][j], ibias[ct][j], sbits, (int)levels)
                                 : act_code(acc_div(acc[pt][ct][j], den, rden), al[ct][j], sh[ct][j], levels);
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

// YOLOLayer eval decode of one head value v = p[..][o] of anchor a at grid cell (x, y) (mymodel.py:56-59)
QVIT_DEV float yolo_io(float v, int o, int a, int x, int y, const float* __restrict__ anchors, float stride) {
  if (o < 2) return __fmul_rn(__fadd_rn(1.f / (1.f + expf(-v)), (float)(o == 0 ? x : y)), stride);
  if (o < 4) return __fmul_rn(__fmul_rn(expf(v), anchors[2 * a + (o - 2)] / stride), stride);  // anchor_vec = anchors / stride
  return 1.f / (1.f + expf(-v));
}

// ---- layers.16-28 in one launch: conv4 .. conv7 (64 -> 64, 3x3, BN + quantizer) and the 1x1 head ---------------
// At 416 x 416 these five layers run on 26 x 26 maps: per image 43 KB of codes in and out of each layer, so as
// separate launches they are latency-bound (≈ 28 µs each for ≈ 2.5 µs of MFMA work at b256). Here one workgroup
// (8 waves) owns one image: its codes stay in LDS through all five layers, in two zero-bordered [H + 2][W + 2][64]
// images used in turn (the border is the 3x3 conv's zero padding), and each layer's weight codes are staged in
// LDS before it runs. The arithmetic is ultra_conv_kernel's (A = weights, B = 16 pixels of a 4 x 4 patch, exact
// int32 accumulation, the same BN + quantizer and head epilogues), so the outputs are bit-identical to the
// per-layer launches. Maps up to 26 x 26 (LDS: 2 x 50 KiB images + 38 KiB of weights).
constexpr int TL_MAX = 26;
// image rows of (W + 2) pixels x 64 B plus 32 B: a row pitch of 8 (mod 16) dwords puts the 16 pixels of a 4 x 4
// patch read by one ds_read_b128 lane group on distinct banks (a multiple of 64 dwords gave 2-way conflicts)
constexpr int TL_RPAD = 32;
constexpr int TL_IMG = (TL_MAX + 2) * ((TL_MAX + 2) * 64 + TL_RPAD);  // 51 072 B
constexpr int TL_WSTR = 9 * 64 + 32;                       // 3x3 weight row pitch (conflict-free b128 reads)
constexpr int TL_HSTR = 64 + 32;                           // head weight row pitch
constexpr int TL_PW = ((TL_MAX + 3) / 4) * ((TL_MAX + 3) / 4) / 8 + 1;  // 4 x 4 patches per wave (7 at 26 x 26)
struct TailArgs {
  const int8_t* w[4];
  const float* alpha[4];
  const float* shift[4];
};

// DEC: the YOLO decode of the head output (qvit_yolo_decode's arithmetic) into io / p instead of the fp32 head
struct TailDecode {
  const float* anchors;
  int na, no;
  float stride;
  float* io;
  float* p;
};
template <bool DEC>
__global__ __launch_bounds__(512, 1) void ultra_tail_kernel(const int8_t* __restrict__ in, int H, int W, TailArgs ta,
                                                            int kpad, const int8_t* __restrict__ hw, int hkpad,
                                                            const float* __restrict__ hbias, int hout, float den,
                                                            float levels, float* __restrict__ out, int ldo,
                                                            TailDecode dec) {
  __shared__ __attribute__((aligned(16))) int8_t smem[2 * TL_IMG + 64 * TL_WSTR];
  __shared__ __attribute__((aligned(16))) float bn_l[4][2][64];  // every layer's BN alpha / shift
  int8_t* imgA = smem;
  int8_t* imgB = smem + TL_IMG;
  int8_t* wl = smem + 2 * TL_IMG;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int p = lane & 15, g = lane >> 4;
  const int b = blockIdx.x;
  const float rden = 1.f / den;
  const int RP = (W + 2) * 64 + TL_RPAD;  // image row pitch (bytes)
  const int PX = (W + 3) / 4, NP = ((H + 3) / 4) * PX;
  // P / PX as a multiply-shift (exact for P < 64, PX <= 7: the fractional parts of P / PX stay below 6 / 7)
  const int pinv = (65536 + PX - 1) / PX;
  auto pdiv = [&](int P) __attribute__((always_inline)) { return (P * pinv) >> 16; };

  // zero both images (borders), then the input codes into A's interior
  for (int i = tid; i < 2 * TL_IMG / 16; i += 512) reinterpret_cast<v4i*>(smem)[i] = v4i{0, 0, 0, 0};
  __syncthreads();
  {  // all of a thread's input pieces in flight at once (a rolled loop waited for each in turn)
    constexpr int IPT = (TL_MAX * TL_MAX * 4 + 511) / 512;
    v4i v[IPT];
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
      const int i = tid + 512 * k;
      if (i < H * W * 4) v[k] = *reinterpret_cast<const v4i*>(in + (int64_t)b * H * W * 64 + 16 * i);
    }
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
      const int i = tid + 512 * k, pix = i >> 2, c16 = i & 3, y = pix / W, x = pix - (pix / W) * W;
      if (i < H * W * 4) *reinterpret_cast<v4i*>(imgA + (y + 1) * RP + (x + 1) * 64 + 16 * c16) = v[k];
    }
  }
  // a layer's weight codes pass through registers: the next layer's are loaded while the current one computes
  // (64 x 576 B = 4.5 16-B pieces per thread), and written to LDS once every wave is done with the current ones
  constexpr int WPT = (64 * 36 + 511) / 512;
  v4i wpre[WPT];
  // head: the 1x1 head's 48 x 64-B rows instead of a 3x3 layer's 64 x 576-B rows. Each load and its wait (put_w) have
  // one call site in the layer loop, selected by `head` rather than by two branches: with two sites the compiler
  // gave the prefetch registers two homes and copied one into the other before the wait, i.e. before the data had
  // landed (found by tools/asm_load_check.py)
  auto fetch_w = [&](const int8_t* w, bool head, int kp) __attribute__((always_inline)) {
    const int per = head ? 4 : 36, rows = head ? 48 : 64;
#pragma unroll
    for (int k = 0; k < WPT; ++k) {
      const int i = tid + 512 * k, o = head ? i >> 2 : i / 36, c16 = i - o * per;
      // (issued from asm: the compiler would drain an ordinary load before the patch loop that it outlives)
      const int8_t* src = w + (int64_t)(i < rows * per ? o : 0) * kp + 16 * (i < rows * per ? c16 : 0);
      asm volatile("; qvit_asm_load\n\tglobal_load_dwordx4 %0, %1, off" : "=v"(wpre[k]) : "v"(src) : "memory");
    }
  };
  auto put_w = [&](bool head) __attribute__((always_inline)) {
    const int per = head ? 4 : 36, rows = head ? 48 : 64, stride = head ? TL_HSTR : TL_WSTR;
    static_assert(WPT == 5, "the wait's operand list");
    asm volatile("s_waitcnt vmcnt(0)\n\t; qvit_pin %0 %1 %2 %3 %4"
                 : "+v"(wpre[0]), "+v"(wpre[1]), "+v"(wpre[2]), "+v"(wpre[3]), "+v"(wpre[4])::"memory");
#pragma unroll
    for (int k = 0; k < WPT; ++k) {
      const int i = tid + 512 * k, o = head ? i >> 2 : i / 36, c16 = i - o * per;
      if (i < rows * per) *reinterpret_cast<v4i*>(wl + o * stride + 16 * c16) = wpre[k];
    }
  };
  if (tid < 4 * 64) {
    const int l = tid >> 6, c = tid & 63;
    bn_l[l][0][c] = ta.alpha[l][c];
    bn_l[l][1][c] = ta.shift[l][c];
  }
  fetch_w(ta.w[0], false, kpad);
  put_w(false);
  __syncthreads();

  for (int l = 0; l < 4; ++l) {
    const int8_t* src = (l & 1) ? imgB : imgA;
    int8_t* dst = (l & 1) ? imgA : imgB;
    const bool head = l == 3;
    fetch_w(head ? hw : ta.w[l < 3 ? l + 1 : 3], head, head ? hkpad : kpad);  // lands while this layer computes
    // the wave's patches P = wave + 8 k (k < TL_PW) all at once: each weight fragment read feeds TL_PW patches
    v4i acc[TL_PW][4];
#pragma unroll
    for (int k = 0; k < TL_PW; ++k)
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) acc[k][ct] = v4i{0, 0, 0, 0};
    // pixel of this lane in patch k (recomputed where used: arrays of them would stay live across the taps)
    auto pix = [&](int k, int& py, int& px) __attribute__((always_inline)) {
      const int P = wave + 8 * k < NP ? wave + 8 * k : wave;
      const int pr = pdiv(P);
      py = 4 * pr + (p >> 2);
      px = 4 * (P - pr * PX) + (p & 3);
    };
    // this lane's pixel of each patch as an LDS byte offset (pixels past the map, the last patches' overhang,
    // read a valid pixel and are never stored)
    int poff[TL_PW];
#pragma unroll
    for (int k = 0; k < TL_PW; ++k) {
      int py, px;
      pix(k, py, px);
      poff[k] = (py < H ? py : H - 1) * RP + (px < W ? px : W - 1) * 64 + 16 * g;
    }
#pragma unroll
    for (int j = 0; j < 9; ++j) {  // tap j = (ky, kx); lane group g: channels 16 g .. 16 g + 15
      const int ky = j / 3, kx = j - 3 * (j / 3);
      v4i a[4];
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) a[ct] = *reinterpret_cast<const v4i*>(wl + (16 * ct + p) * TL_WSTR + 64 * j + 16 * g);
#pragma unroll
      for (int k = 0; k < TL_PW; ++k) {
        if (wave + 8 * k >= NP) continue;  // wave-uniform
        const v4i bf = *reinterpret_cast<const v4i*>(src + poff[k] + ky * RP + kx * 64);
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) acc[k][ct] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[ct], bf, acc[k][ct], 0, 0, 0);
      }
    }
    // acc[k][ct][j] = conv[channel 16 ct + 4 g + j][pixel (py, px)] -> codes into dst's interior
#pragma unroll
    for (int k = 0; k < TL_PW; ++k) {
      int py, px;
      pix(k, py, px);
      if (wave + 8 * k >= NP || py >= H || px >= W) continue;
      int8_t* d = dst + (py + 1) * RP + (px + 1) * 64 + 4 * g;
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        const float4 al = *reinterpret_cast<const float4*>(&bn_l[l][0][16 * ct + 4 * g]);
        const float4 sh = *reinterpret_cast<const float4*>(&bn_l[l][1][16 * ct + 4 * g]);
        const uint32_t word = (uint32_t)act_code(acc_div(acc[k][ct][0], den, rden), al.x, sh.x, levels) |
                              ((uint32_t)act_code(acc_div(acc[k][ct][1], den, rden), al.y, sh.y, levels) << 8) |
                              ((uint32_t)act_code(acc_div(acc[k][ct][2], den, rden), al.z, sh.z, levels) << 16) |
                              ((uint32_t)act_code(acc_div(acc[k][ct][3], den, rden), al.w, sh.w, levels) << 24);
        *reinterpret_cast<uint32_t*>(d + 16 * ct) = word;
      }
    }
    __syncthreads();  // every read of this layer's weights and source image done, dst complete
    put_w(head);
    __syncthreads();
  }

  // head (1x1, 64 -> hout <= 48, bias, fp32 NHWC out) from image A (conv7's output)
  for (int pi = wave; pi < NP; pi += 8) {
    const int pr = pdiv(pi);
    const int py = 4 * pr + (p >> 2), px = 4 * (pi - pr * PX) + (p & 3);
    const int y = py < H ? py : H - 1, x = px < W ? px : W - 1;
    const v4i bf = *reinterpret_cast<const v4i*>(imgA + (y + 1) * RP + (x + 1) * 64 + 16 * g);
    v4i acc[3];
#pragma unroll
    for (int ct = 0; ct < 3; ++ct)
      acc[ct] = __builtin_amdgcn_mfma_i32_16x16x64_i8(*reinterpret_cast<const v4i*>(wl + (16 * ct + p) * TL_HSTR + 16 * g), bf,
                                                      v4i{0, 0, 0, 0}, 0, 0, 0);
    if (py >= H || px >= W) continue;
    float* o = out + ((int64_t)b * H * W + py * W + px) * ldo;
#pragma unroll
    for (int ct = 0; ct < 3; ++ct)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = 16 * ct + 4 * g + j;
        if (c >= hout) continue;
        const float v = __fadd_rn(acc_div(acc[ct][j], den, rden), hbias[c]);
        if (DEC) {  // p[b][a][y][x][o] = head channel a no + o, io its decode
          const int a = c / dec.no, oo = c - a * dec.no;
          const int64_t i = ((((int64_t)b * dec.na + a) * H + py) * W + px) * dec.no + oo;
          dec.p[i] = v;
          dec.io[i] = yolo_io(v, oo, a, px, py, dec.anchors, dec.stride);
        } else {
          o[c] = v;
        }
      }
  }
}

// ---- YOLOLayer decode (mymodel.py:47-60) -----------------------------------------------------------
// (32-bit index arithmetic: the launcher checks the element count fits; 64-bit divisions cost more than the
// decode itself)
__global__ void yolo_decode_kernel(const float* __restrict__ head, int B, int ny, int nx, int na, int no, int ldh,
                                   const float* __restrict__ anchors, float stride, float* __restrict__ io,
                                   float* __restrict__ pout) {
  const uint32_t total = (uint32_t)B * na * ny * nx * no;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    uint32_t r0 = i;
    const int o = (int)(r0 % (uint32_t)no);
    r0 /= (uint32_t)no;
    const int x = (int)(r0 % (uint32_t)nx);
    r0 /= (uint32_t)nx;
    const int y = (int)(r0 % (uint32_t)ny);
    r0 /= (uint32_t)ny;
    const int a = (int)(r0 % (uint32_t)na);
    const int b = (int)(r0 / (uint32_t)na);
    // p[b][a][y][x][o] = head_nchw[b][a*no + o][y][x] = head_nhwc[b][y][x][a*no + o]
    const float v = head[(((int64_t)b * ny + y) * nx + x) * ldh + a * no + o];
    pout[i] = v;
    io[i] = yolo_io(v, o, a, x, y, anchors, stride);
  }
}

// persistent grid: every block resident at once (CUs x occupancy), at most one per tile
template <class K>
int64_t resident_grid(K kernel, int64_t ntiles) {
  int dev = 0, cus = 0, occ = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                              hipSuccess || cus <= 0)
    cus = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel, 256, 0) != hipSuccess || occ <= 0) occ = 1;
  return std::max<int64_t>(1, std::min<int64_t>(ntiles, (int64_t)cus * occ));
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
  // the staged pooled path: whole 16-B output groups (cout == COUT, 16-B rows) and an image of codes that a
  // 32-bit buffer offset reaches
  // (CIN 64: two halo buffers and the weights leave room for one workgroup per CU; that layer keeps the
  // synchronous halo at two workgroups)
  const bool stg = CIN <= 32 && POOL != 0 && OUT != 1 && cout_real == COUT && (ldo % 16) == 0 &&
                   (((uintptr_t)out) & 15) == 0 &&
                   (int64_t)(H / 2) * (W / 2) * ldo < ((int64_t)1 << 31);
  if constexpr (CIN <= 32 && POOL != 0 && OUT != 1) {
    if (stg) {
      hipLaunchKernelGGL((ultra_conv_kernel<CIN, KS, COUT, POOL, OUT, true>), dim3(grid), dim3(256), 0, stream, in, B,
                         H, W, w, kpad, den, alpha, shift, levels, cout_real, out, ldo, sbits);
      return qvit_hip_status(hipGetLastError());
    }
  }
    hipLaunchKernelGGL((ultra_conv_kernel<CIN, KS, COUT, POOL, OUT, false>), dim3(grid), dim3(256), 0, stream, in, B,
                       H, W, w, kpad, den, alpha, shift, levels, cout_real, out, ldo, sbits);
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
  // persistent over 16 x 32 tiles
  const int64_t ntiles = B * ((H + C0_TY - 1) / C0_TY) * ((W + C0_TX - 1) / C0_TX);
  if (ntiles > INT32_MAX) return QVIT_EINVAL;
  const float levels = (float)((1 << a_bit) - 1);
  if ((W % 4) == 0 && (((uintptr_t)img) & 15) == 0) {  // 16-B quad loads
    const int64_t grid = resident_grid(ultra_conv0_mfma_kernel<true>, ntiles);
    hipLaunchKernelGGL(ultra_conv0_mfma_kernel<true>, dim3((unsigned)grid), dim3(256), 0, stream, img, (int)B, (int)H,
                       (int)W, wvals, alpha, shift, levels, out);
  } else {
    const int64_t grid = resident_grid(ultra_conv0_mfma_kernel<false>, ntiles);
    hipLaunchKernelGGL(ultra_conv0_mfma_kernel<false>, dim3((unsigned)grid), dim3(256), 0, stream, img, (int)B, (int)H,
                       (int)W, wvals, alpha, shift, levels, out);
  }
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

extern "C" int qvit_ultra_tail(const int8_t* in, int64_t B, int64_t H, int64_t W, const int8_t* const* wcodes,
                               int64_t kpad, const float* const* alpha, const float* const* shift,
                               const int8_t* hcodes, int64_t hkpad, const float* hbias, int64_t hout, int w_bit,
                               int a_bit, float* out, int64_t ldo, const float* anchors, int64_t na, int64_t no,
                               float stride, float* io, float* p, hipStream_t stream) {
  const bool dec = io != nullptr;
  if (!in || !wcodes || !alpha || !shift || !hcodes || !hbias) return QVIT_ENULL;
  if (dec ? (!p || !anchors) : !out) return QVIT_ENULL;
  if (dec && (na < 1 || no < 5 || na * no != hout || !(stride > 0.f))) return QVIT_EINVAL;
  for (int l = 0; l < 4; ++l)
    if (!wcodes[l] || !alpha[l] || !shift[l]) return QVIT_ENULL;
  if (B < 0 || H < 1 || W < 1 || H > TL_MAX || W > TL_MAX || hout < 1 || hout > 48 || (!dec && ldo < hout))
    return QVIT_EINVAL;
  if (kpad < 9 * 64 || hkpad < 64 || w_bit < 2 || w_bit > 8 || a_bit < 1 || a_bit > 7) return QVIT_EINVAL;
  if (B > INT32_MAX) return QVIT_EINVAL;
  if ((((uintptr_t)in) & 15) || (kpad % 16) || (hkpad % 16) || (((uintptr_t)hcodes) & 15)) return QVIT_EALIGN;
  for (int l = 0; l < 4; ++l)
    if (((uintptr_t)wcodes[l]) & 15) return QVIT_EALIGN;
  if (B == 0) return QVIT_OK;
  TailArgs ta;
  for (int l = 0; l < 4; ++l) {
    ta.w[l] = wcodes[l];
    ta.alpha[l] = alpha[l];
    ta.shift[l] = shift[l];
  }
  const float den = (float)(((1 << (w_bit - 1)) - 1) * ((1 << a_bit) - 1));
  const float lv = (float)((1 << a_bit) - 1);
  const TailDecode td{anchors, (int)na, (int)no, stride, io, p};
  if (dec)
    hipLaunchKernelGGL(ultra_tail_kernel<true>, dim3((unsigned)B), dim3(512), 0, stream, in, (int)H, (int)W, ta,
                       (int)kpad, hcodes, (int)hkpad, hbias, (int)hout, den, lv, out, (int)ldo, td);
  else
    hipLaunchKernelGGL(ultra_tail_kernel<false>, dim3((unsigned)B), dim3(512), 0, stream, in, (int)H, (int)W, ta,
                       (int)kpad, hcodes, (int)hkpad, hbias, (int)hout, den, lv, out, (int)ldo, td);
  return qvit_hip_status(hipGetLastError());
}

extern "C" int qvit_ultra_conv0_int(const uint8_t* img, int64_t B, int64_t H, int64_t W, const int8_t* wcodes,
                                    const int32_t* inc, const int32_t* bias, int shift_bits, int out_bit, int8_t* out,
                                    hipStream_t stream) {
  if (!img || !wcodes || !inc || !bias || !out) return QVIT_ENULL;
  if (B < 0 || H < 2 || W < 2 || shift_bits < 1 || shift_bits > 40 || out_bit < 1 || out_bit > 7) return QVIT_EINVAL;
  if ((((uintptr_t)out) & 15)) return QVIT_EALIGN;
  if (B * H * W > INT32_MAX) return QVIT_EINVAL;
  if (B == 0) return QVIT_OK;
  const int64_t ntiles = B * ((H + C0_TY - 1) / C0_TY) * ((W + C0_TX - 1) / C0_TX);
  if (ntiles > INT32_MAX) return QVIT_EINVAL;
  if ((W % 4) == 0 && (((uintptr_t)img) & 3) == 0) {  // 4-B quad loads
    const int64_t grid = resident_grid(ultra_conv0_int_mfma_kernel<true>, ntiles);
    hipLaunchKernelGGL(ultra_conv0_int_mfma_kernel<true>, dim3((unsigned)grid), dim3(256), 0, stream, img, (int)B,
                       (int)H, (int)W, wcodes, inc, bias, shift_bits, (1 << out_bit) - 1, out);
  } else {
    const int64_t grid = resident_grid(ultra_conv0_int_mfma_kernel<false>, ntiles);
    hipLaunchKernelGGL(ultra_conv0_int_mfma_kernel<false>, dim3((unsigned)grid), dim3(256), 0, stream, img, (int)B,
                       (int)H, (int)W, wcodes, inc, bias, shift_bits, (1 << out_bit) - 1, out);
  }
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
  if (B * na * ny * nx * no > (int64_t)INT32_MAX) return QVIT_EINVAL;  // the kernel's 32-bit element index
  if (B == 0) return QVIT_OK;
  hipLaunchKernelGGL(yolo_decode_kernel, dim3(grid_cap(B * na * ny * nx * no)), dim3(256), 0, stream, head, (int)B,
                     (int)ny, (int)nx, (int)na, (int)no, (int)ldh, anchors, stride, io, p);
  return qvit_hip_status(hipGetLastError());
}
