// Fused multi-head attention core of Attention.forward (vit_model.py:126-152):
//   q, k, v = qkv.reshape(B, N, 3, H, hd).permute(2, 0, 3, 1, 4)
//   out     = softmax((q @ k^T) * scale) @ v          -> [B, N, H * hd]
// optionally followed by the next QuantizeLinear's activation quantizer (proj's act quantizer,
// quant_layers.py:41-69 / 137-161), so the kernel writes int8 codes that feed the proj GEMM directly.
//
// Arithmetic: the reference runs these matmuls in fp32. Each fp32 operand x is split into
// fp16 hi = f16(x) and lo = f16(x - hi) (x - hi is exact in fp32), and every product is formed as
// hi*hi + hi*lo + lo*hi on v_mfma_f32_16x16x32_f16 with fp32 accumulation: the dropped lo*lo term and
// the rounding of lo leave ~2^-22 relative error per product (fp32-class). The caller passes a power-of-
// two in_scale that keeps |x * in_scale| inside the fp16 range (quant_layers.py derives it from the
// qkv GEMM's output bound); it is undone exactly in the softmax exponent and the output.
//
// Work split: one workgroup (4 waves) per (image, head, group of <= 256 queries); wave w owns the
// 16-query tiles w, w+4, w+8, w+12 of its group. Keys stream through LDS in blocks of 32 (register
// prefetch of block j+1 while block j is computed, double-buffered LDS images of K and V, hi and lo).
// Orientation: S^T = K . Q^T (keys on MFMA rows), so after the MFMA each lane holds 8 scores of ONE
// query (lane & 15) and the softmax row statistics need only two cross-lane steps; those scores,
// split to fp16, are directly the B operand of O^T = V^T . P^T (the k order inside a 32-key step is
// permuted identically on both sides). V^T fragments come from row-major V images through
// ds_read_b64_tr_b16. Online softmax (running max / sum per query) over the key blocks.
// LDS images (128-B rows of 64 fp16), XOR-swizzled, conflict-free for every read and write:
//   K: 16-B chunk c of row r at c ^ ((r >> 1) & 7)        (ds_read_b128 A fragments)
//   V: 32-B block b of row r at b ^ ((r >> 1) & 3)        (ds_read_b64_tr_b16 transposed reads)
#include "qvit_common.h"

namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef short s8v __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned int u4 __attribute__((ext_vector_type(4)));

constexpr int HD = 64;          // head dim (the only one supported)
constexpr int KB = 32;          // keys per block
constexpr int NWAVES = 4;
constexpr int QTW = 4;          // query tiles per wave
constexpr int QG = NWAVES * QTW * 16;  // queries per workgroup (256)
constexpr int IMG = KB * HD * 2;       // one fp16 image of a key block: 4 KiB
constexpr int STAGE = 4 * IMG;         // K hi, K lo, V hi, V lo
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

QVIT_DEV float xmax(float v) {
  v = fmaxf(v, __shfl_xor(v, 16));
  return fmaxf(v, __shfl_xor(v, 32));
}
QVIT_DEV float xsum(float v) {
  v += __shfl_xor(v, 16);
  return v + __shfl_xor(v, 32);
}

template <int OUT>  // 0: fp32 output, 1: int8 codes of the next layer's activation quantizer
__global__ __launch_bounds__(256, 2) void attn_kernel(const float* __restrict__ qkv, int N, int H, int64_t ldq,
                                                      float scale, float in_scale, void* __restrict__ out,
                                                      int64_t ldo, int out_qtype, const float* out_d,
                                                      const float* out_qm, const float* out_t, int out_levels) {
  __shared__ __attribute__((aligned(16))) int8_t smem[2 * STAGE];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15;  // query (S^T column) / key row of an A fragment / dim row of V^T
  const int g = lane >> 4;

  const int ngroups = (N + QG - 1) / QG;
  const int bid = blockIdx.x;
  const int grp = bid % ngroups;
  const int bh = bid / ngroups;
  const int h = bh % H;
  const int b = bh / H;
  const int C = H * HD;
  const float* base = qkv + (int64_t)b * N * ldq;
  const float* qcol = base + h * HD;
  const float* kcol = base + C + h * HD;
  const float* vcol = base + 2 * C + h * HD;

  // ---- Q^T fragments (B operand): lane holds Q[q][8g .. 8g+7] (+32) ------------------------------
  const int q0 = grp * QG;
  h8 qh[QTW][2], ql[QTW][2];
  bool tv[QTW];
#pragma unroll
  for (int i = 0; i < QTW; ++i) {
    const int tile = wave + NWAVES * i;
    tv[i] = q0 + 16 * tile < N;  // wave-uniform
    int q = q0 + 16 * tile + fr;
    q = q < N ? q : N - 1;       // padded queries read a valid row; never stored
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      float x[8];
      const f4* src = reinterpret_cast<const f4*>(qcol + (int64_t)q * ldq + 32 * c + 8 * g);
      const f4 a = src[0], bq = src[1];
#pragma unroll
      for (int j = 0; j < 4; ++j) { x[j] = a[j] * in_scale; x[4 + j] = bq[j] * in_scale; }
      split8(x, qh[i][c], ql[i][c]);
    }
  }

  // ---- key-block staging: thread -> key row tid >> 3 (0..31), 8-dim chunk tid & 7 ------------------
  const int srow = tid >> 3, schunk = tid & 7;
  f4 pk[2], pv[2];
  auto load_block = [&](int kb) {
    const int key = kb * KB + srow;
    if (key < N) {
      const f4* ks = reinterpret_cast<const f4*>(kcol + (int64_t)key * ldq + 8 * schunk);
      const f4* vs = reinterpret_cast<const f4*>(vcol + (int64_t)key * ldq + 8 * schunk);
      pk[0] = ks[0]; pk[1] = ks[1];
      pv[0] = vs[0]; pv[1] = vs[1];
    } else {
      pk[0] = pk[1] = pv[0] = pv[1] = f4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto store_block = [&](int buf) {
    int8_t* st = smem + buf * STAGE;
    float x[8];
    h8 hi, lo;
#pragma unroll
    for (int j = 0; j < 4; ++j) { x[j] = pk[0][j] * in_scale; x[4 + j] = pk[1][j] * in_scale; }
    split8(x, hi, lo);
    *reinterpret_cast<h8*>(st + koff(srow, schunk)) = hi;
    *reinterpret_cast<h8*>(st + IMG + koff(srow, schunk)) = lo;
#pragma unroll
    for (int j = 0; j < 4; ++j) { x[j] = pv[0][j] * in_scale; x[4 + j] = pv[1][j] * in_scale; }
    split8(x, hi, lo);
    *reinterpret_cast<h8*>(st + 2 * IMG + voff(srow, 16 * schunk)) = hi;
    *reinterpret_cast<h8*>(st + 3 * IMG + voff(srow, 16 * schunk)) = lo;
  };

  // per-lane fragment offsets
  int koffs[2][2];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int c = 0; c < 2; ++c) koffs[kt][c] = koff(16 * kt + fr, g + 4 * c);
  const int vq = fr >> 2, vp = fr & 3;
  int voffs[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) voffs[dt] = voff(4 * g + vq, 2 * (16 * dt + 4 * vp));

  // softmax state and O^T accumulators: o[i][dt][j] = O^T[16 dt + 4 g + j][query of lane]
  const float sl2 = scale * LOG2E / (in_scale * in_scale);
  float m[QTW], l[QTW];
  f4 o[QTW][4];
#pragma unroll
  for (int i = 0; i < QTW; ++i) {
    m[i] = -INFINITY;
    l[i] = 0.f;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[i][dt] = f4{0.f, 0.f, 0.f, 0.f};
  }

  const int nkb = (N + KB - 1) / KB;
  load_block(0);
  store_block(0);
  __syncthreads();
  for (int kb = 0; kb < nkb; ++kb) {
    if (kb + 1 < nkb) load_block(kb + 1);
    const int8_t* st = smem + (kb & 1) * STAGE;
    h8 kh[2][2], kl[2][2], vh[4], vl[4];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        kh[kt][c] = lds_h8(st, koffs[kt][c]);
        kl[kt][c] = lds_h8(st + IMG, koffs[kt][c]);
      }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      vh[dt] = join(tr_read(st + 2 * IMG, voffs[dt]), tr_read(st + 2 * IMG, voffs[dt] + 16 * 128));
      vl[dt] = join(tr_read(st + 3 * IMG, voffs[dt]), tr_read(st + 3 * IMG, voffs[dt] + 16 * 128));
    }
    const int kbase = kb * KB + 4 * g;
#pragma unroll
    for (int i = 0; i < QTW; ++i) {
      if (!tv[i]) continue;  // wave-uniform
      f4 s[2];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        s[kt] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < 2; ++c) s[kt] = mfma3(kh[kt][c], kl[kt][c], qh[i][c], ql[i][c], s[kt]);
      }
      // s[kt][j] = S^T[key kbase + 16 kt + j][query]; scores in log2 units
      float x[8];
      float bm = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float v = (kbase + 16 * kt + j < N) ? s[kt][j] * sl2 : -INFINITY;
          x[4 * kt + j] = v;
          bm = fmaxf(bm, v);
        }
      bm = xmax(bm);
      const float mn = fmaxf(m[i], bm);
      const float alpha = __builtin_amdgcn_exp2f(m[i] - mn);
      float ps = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        x[e] = __builtin_amdgcn_exp2f(x[e] - mn);
        ps += x[e];
      }
      l[i] = l[i] * alpha + ps;
      m[i] = mn;
      h8 ph, pl;
      split8(x, ph, pl);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[i][dt] = mfma3(vh[dt], vl[dt], ph, pl, o[i][dt] * alpha);
    }
    if (kb + 1 < nkb) {
      __syncthreads();  // every wave is done with buffer (kb + 1) & 1 (used by block kb - 1)
      store_block((kb + 1) & 1);
    }
    __syncthreads();
  }

  // ---- epilogue: normalise, write fp32 or the next layer's int8 codes ----------------------------
  QParams qp;
  if (OUT == 1) qp = load_qparams(out_qtype, out_d, out_qm, out_t, out_levels);
#pragma unroll
  for (int i = 0; i < QTW; ++i) {
    if (!tv[i]) continue;
    const float inv = 1.f / (xsum(l[i]) * in_scale);
    const int q = q0 + 16 * (wave + NWAVES * i) + fr;
    if (q >= N) continue;
    const int64_t row = (int64_t)b * N + q;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int col = h * HD + 16 * dt + 4 * g;
      f4 v = o[i][dt] * inv;
      if (OUT == 0) {
        *reinterpret_cast<f4*>(reinterpret_cast<float*>(out) + row * ldo + col) = v;
      } else {
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
        *reinterpret_cast<uint32_t*>(reinterpret_cast<int8_t*>(out) + row * ldo + col) = word;
      }
    }
  }
}

}  // namespace

extern "C" int qvit_attention(const float* qkv, int64_t B, int64_t N, int64_t H, int64_t head_dim, int64_t ldq,
                              float scale, float in_scale, int out_mode, void* out, int64_t ldo, int out_qtype,
                              const float* out_d, const float* out_qm, const float* out_t, int out_levels,
                              hipStream_t stream) {
  if (!qkv || !out) return QVIT_ENULL;
  if (head_dim != HD) return QVIT_EINVAL;
  if (B < 0 || N <= 0 || H <= 0 || ldq < 3 * H * HD || ldo < H * HD) return QVIT_EINVAL;
  if (B * N > INT32_MAX || N > (1 << 20) || !(in_scale > 0.f)) return QVIT_EINVAL;
  if ((ldq % 4) || (((uintptr_t)qkv) & 15)) return QVIT_EALIGN;
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
  const int64_t ngroups = (N + QG - 1) / QG;
  const int64_t nblk = B * H * ngroups;
  if (nblk > INT32_MAX) return QVIT_EINVAL;
  if (out_mode == QVIT_ATT_F32)
    hipLaunchKernelGGL(attn_kernel<0>, dim3((unsigned)nblk), dim3(256), 0, stream, qkv, (int)N, (int)H, ldq, scale,
                       in_scale, out, ldo, out_qtype, out_d, out_qm, out_t, out_levels);
  else
    hipLaunchKernelGGL(attn_kernel<1>, dim3((unsigned)nblk), dim3(256), 0, stream, qkv, (int)N, (int)H, ldq, scale,
                       in_scale, out, ldo, out_qtype, out_d, out_qm, out_t, out_levels);
  return qvit_hip_status(hipGetLastError());
}
