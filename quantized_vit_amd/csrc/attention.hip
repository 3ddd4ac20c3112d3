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
#include "attn_common.h"

#include <algorithm>

namespace {

using namespace qvit_attn;

constexpr int NWAVES = 4;
constexpr int QTW = 4;          // query tiles per wave
constexpr int QG = NWAVES * QTW * 16;  // queries per workgroup (256)
constexpr int STAGE = 4 * IMG;         // K hi, K lo, V hi, V lo

QVIT_DEV void attend_n(int nt, bool mask, const int8_t* st, const h8 (&qh)[QTW][2], const h8 (&ql)[QTW][2],
                       float (&m)[QTW], float (&l)[QTW], f4 (&o)[QTW][4], const int (&koffs)[2][2],
                       const int (&voffs)[4], int kbase, int N, float sl2, Stamps& sp) {
  attend<QTW>(nt, mask, st, qh, ql, m, l, o, koffs, voffs, kbase, N, sl2, sp);
}

// ---- fp32 qkv input (the unfused module path) -------------------------------------------------------
template <int OUT>  // 0: fp32 output, 1: int8 codes of the next layer's activation quantizer
__global__ __launch_bounds__(256, 2) void attn_kernel(const float* __restrict__ qkv, int N, int H, int64_t ldq,
                                                      float scale, float in_scale, void* __restrict__ out,
                                                      int64_t ldo, int out_qtype, const float* out_d,
                                                      const float* out_qm, const float* out_t, int out_levels) {
  __shared__ __attribute__((aligned(16))) int8_t smem[2 * STAGE];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15;
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

  int koffs[2][2], voffs[4];
  fragment_offsets(koffs, voffs);

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

  int nt = 0;  // valid tiles of this wave (a prefix of i = 0..3)
#pragma unroll
  for (int i = 0; i < QTW; ++i) nt += tv[i] ? 1 : 0;
  const int nkb = (N + KB - 1) / KB;
  load_block(0);
  store_block(0);
  __syncthreads();
  for (int kb = 0; kb < nkb; ++kb) {
    if (kb + 1 < nkb) load_block(kb + 1);
    Stamps sp;
    attend_n(nt, (kb + 1) * KB > N, smem + (kb & 1) * STAGE, qh, ql, m, l, o, koffs, voffs, kb * KB + 4 * g, N,
             sl2, sp);
    if (kb + 1 < nkb) {
      __syncthreads();  // every wave is done with buffer (kb + 1) & 1 (used by block kb - 1)
      store_block((kb + 1) & 1);
    }
    __syncthreads();
  }
  QParams qp{};
  if (OUT == 1) qp = load_qparams(out_qtype, out_d, out_qm, out_t, out_levels);
  const bool st16 = ((ldo & 15) == 0) && ((((uintptr_t)out) & 15) == 0);
  attend_store<OUT, QTW>(tv, l, o, wave, NWAVES, q0, N, b, h, in_scale, out, ldo, qp, EpiLds{nullptr, 0.f, 0.f, 0.f},
                         st16);
}

// ---- split fp16 input (the fused block path) --------------------------------------------------------
// q, k, v arrive pre-scaled and pre-split by the qkv GEMM (qvit_gemm_qkv_split): hi and lo planes of
// layout [B][3H][N][64] fp16, so a key block's four LDS images (K hi/lo, V hi/lo; 32 rows x 128 B) are
// copied by LDS-DMA straight from global memory, the swizzle applied on the source side. A ring of
// SRING blocks keeps SRING - 1 blocks (48 KiB per workgroup) in flight: a head's keys stream while the
// previous block is computed, with no register staging and no conversion in this kernel.
constexpr int SRING = 4;

template <int N_>
QVIT_DEV void block_sync() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N_) : "memory");
}

// Persistent: workgroup w walks the units (image, head, group of <= QG queries) w, w + grid, ... Each
// unit is a run of ring blocks in one stream: nqb query blocks (64 queries: hi and lo images in the K
// layout, wave w reads its tile from each) and then nkb key blocks. Block p + 3 is issued as soon as
// block p is waited for, across unit boundaries, so the next unit's queries and first keys land while the
// current unit finishes. Every global load of the loop is an LDS-DMA (the quantizer scalars are read
// before the stream starts), so the only vmcnt waits are the counted stage waits; the output stores of a
// unit's epilogue do join the count and are drained by the next wait.
constexpr int QB = 64;  // queries per query block
constexpr int TBL_BYTES = 16384;  // int8 epilogue code table (<= 2046 buckets): 2 x (64 + 16) KiB per CU

template <int OUT>
__global__ __launch_bounds__(256, 2) void attn_split_kernel(const _Float16* __restrict__ hi,
                                                            const _Float16* __restrict__ lo, int N, int H, int nunits,
                                                            float scale, float in_scale, void* __restrict__ out,
                                                            int64_t ldo, int out_qtype, const float* out_d,
                                                            const float* out_qm, const float* out_t, int out_levels,
                                                            const int8_t* __restrict__ epi_table) {
  __shared__ __attribute__((aligned(16))) int8_t smem[SRING * STAGE + (OUT == 1 ? TBL_BYTES : 0)];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15;
  const int g = lane >> 4;

  QParams qp{};
  EpiLds tb{nullptr, 0.f, 0.f, 0.f};
  if (OUT == 1) {
    qp = load_qparams(out_qtype, out_d, out_qm, out_t, out_levels);
    if (epi_table != nullptr) {  // the code table -> LDS, once per workgroup
      const EpiTableHdr hd = *reinterpret_cast<const EpiTableHdr*>(epi_table);
      if (hd.valid != 0 && hd.nb >= 1 && 16 + 8 * hd.nb <= TBL_BYTES) {
        int8_t* tl = smem + SRING * STAGE;
        for (int k = tid; k < (16 + 8 * hd.nb + 15) / 16; k += 256)
          reinterpret_cast<uint4*>(tl)[k] = reinterpret_cast<const uint4*>(epi_table)[k];
        tb = EpiLds{tl + sizeof(EpiTableHdr), hd.c0, hd.inv_w, epi_top(hd.nb)};
      }
    }
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): nothing of the compiler's own is pending below
  const bool st16 = ((ldo & 15) == 0) && ((((uintptr_t)out) & 15) == 0);

  const int ngroups = (N + QG - 1) / QG;
  const int nqb = (N < QG ? (N + QB - 1) / QB : QG / QB);
  const int nkb = (N + KB - 1) / KB;
  const int per = nqb + nkb;
  // units of this workgroup: with a grid that is a multiple of 8, XCD x (blocks x, x + 8, ...) owns a contiguous
  // unit range, so the query groups of one (image, head) stream the same K / V through one XCD's L2 instead of
  // fetching it once per XCD; otherwise units blockIdx + j * grid
  const bool xcd_map = (gridDim.x & 7) == 0;
  const int team = xcd_map ? (int)gridDim.x >> 3 : (int)gridDim.x;
  const int slot = xcd_map ? (int)blockIdx.x >> 3 : (int)blockIdx.x;
  int ulo = 0, uhi = nunits;
  if (xcd_map) {
    const int xcd = blockIdx.x & 7, per8 = nunits >> 3, rem = nunits & 7;
    ulo = xcd * per8 + (xcd < rem ? xcd : rem);
    uhi = ulo + per8 + (xcd < rem ? 1 : 0);
  }
  const int my_units = (uhi - ulo - slot + team - 1) / team;  // unit j: ulo + slot + j * team
  const int total = my_units * per;
  const int64_t plane = (int64_t)N * HD;

  const uint32_t lds0 = lds_addr(smem);
  // DMA of stream block p into ring slot p % SRING
  auto issue = [&](int p) {
    const int j = p / per, idx = p - j * per;
    const int unit = ulo + slot + j * team;
    const int grp = unit % ngroups, bh = unit / ngroups;
    const int h = bh % H, b = bh / H;
    const int64_t qoff = ((int64_t)b * 3 * H + h) * plane;
    const uint32_t base = __builtin_amdgcn_readfirstlane(lds0 + (p & (SRING - 1)) * STAGE);
    if (idx < nqb) {  // query block: rows 16w .. 16w+15 of the hi and lo images (K layout)
#pragma unroll
      for (int pc = 0; pc < 2; ++pc) {
        const int r = 16 * wave + 8 * pc + (lane >> 3);
        int q = grp * QG + idx * QB + r;
        q = q < N ? q : N - 1;
        const int kc = ((lane & 7) ^ ((r >> 1) & 7)) << 4;
        const int64_t e = qoff + (int64_t)q * HD;
        const uint32_t d = base + (16 * wave + 8 * pc) * 128;
        dma16(reinterpret_cast<const int8_t*>(hi + e) + kc, __builtin_amdgcn_readfirstlane(d));
        dma16(reinterpret_cast<const int8_t*>(lo + e) + kc, __builtin_amdgcn_readfirstlane(d + QB * 128));
      }
    } else {          // key block: rows 8w .. 8w+7 of K hi, K lo, V hi, V lo
      const int kb = idx - nqb;
      const int r = 8 * wave + (lane >> 3);
      const int sc = lane & 7;
      int key = kb * KB + r;
      key = key < N ? key : N - 1;  // keys past N: a valid row, masked out of the softmax
      const int kc = (sc ^ ((r >> 1) & 7)) << 4;
      const int vb = (((sc >> 1) ^ ((r >> 1) & 3)) << 5) | ((sc & 1) << 4);
      const int64_t ke = qoff + H * plane + (int64_t)key * HD;
      const int64_t ve = ke + H * plane;
      const uint32_t d = base + wave * 1024;
      dma16(reinterpret_cast<const int8_t*>(hi + ke) + kc, __builtin_amdgcn_readfirstlane(d));
      dma16(reinterpret_cast<const int8_t*>(lo + ke) + kc, __builtin_amdgcn_readfirstlane(d + IMG));
      dma16(reinterpret_cast<const int8_t*>(hi + ve) + vb, __builtin_amdgcn_readfirstlane(d + 2 * IMG));
      dma16(reinterpret_cast<const int8_t*>(lo + ve) + vb, __builtin_amdgcn_readfirstlane(d + 3 * IMG));
    }
  };
  // block p landed for every wave (4 DMAs per wave per block; up to two younger blocks in flight) and
  // every wave is done with block p - 1, whose slot block p + 3 takes
  auto sync = [&](int p) {
    const int ahead = total - 1 - p;
    if (ahead >= 2) block_sync<8>();
    else if (ahead == 1) block_sync<4>();
    else block_sync<0>();
    if (p + 3 < total) issue(p + 3);
  };

  int koffs[2][2], voffs[4];
  fragment_offsets(koffs, voffs);
  const float sl2 = scale * LOG2E / (in_scale * in_scale);

  Stamps sp;
  for (int p = 0; p < 3 && p < total; ++p) issue(p);
  int p = 0;
  for (int j = 0; j < my_units; ++j) {
    const int unit = ulo + slot + j * team;
    const int grp = unit % ngroups, bh = unit / ngroups;
    const int h = bh % H, b = bh / H;
    const int q0 = grp * QG;
    const int wr = (wave + unit) & (NWAVES - 1);  // the wave owning a 4th tile rotates by unit
    h8 qh[QTW][2], ql[QTW][2];
    int nt = 0;
#pragma unroll
    for (int i = 0; i < QTW; ++i) {
      if (i < nqb) {
        sp.mark(4);
        sync(p);
        sp.mark(0);
        const int8_t* st = smem + (p & (SRING - 1)) * STAGE;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int off = koff(16 * wr + fr, g + 4 * c);
          qh[i][c] = lds_h8(st, off);
          ql[i][c] = lds_h8(st + QB * 128, off);
        }
        ++p;
      } else {  // no such query block: zeros (the tile is skipped or discarded)
        qh[i][0] = qh[i][1] = ql[i][0] = ql[i][1] = h8{};
      }
      nt += (i < nqb && q0 + 16 * (wr + NWAVES * i) < N) ? 1 : 0;
    }
    float m[QTW], l[QTW];
    f4 o[QTW][4];
#pragma unroll
    for (int i = 0; i < QTW; ++i) {
      m[i] = -INFINITY;
      l[i] = 0.f;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[i][dt] = f4{0.f, 0.f, 0.f, 0.f};
    }
    sp.mark(5);
    for (int kb = 0; kb < nkb; ++kb, ++p) {
      sync(p);
      sp.mark(0);
      attend_n(nt, (kb + 1) * KB > N, smem + (p & (SRING - 1)) * STAGE, qh, ql, m, l, o, koffs, voffs,
               kb * KB + 4 * g, N, sl2, sp);
    }
    bool tv[QTW];
#pragma unroll
    for (int i = 0; i < QTW; ++i) tv[i] = i < nt;
    attend_store<OUT, QTW>(tv, l, o, wr, NWAVES, q0, N, b, h, in_scale, out, ldo, qp, tb, st16);
  }
  sp.mark(4);
  sp.flush();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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

extern "C" int qvit_attention_split(const void* qkv_hi, const void* qkv_lo, int64_t B, int64_t N, int64_t H,
                                    int64_t head_dim, float scale, float in_scale, int out_mode, void* out,
                                    int64_t ldo, int out_qtype, const float* out_d, const float* out_qm,
                                    const float* out_t, int out_levels, const void* epi_table,
                                    hipStream_t stream) {
  if (!qkv_hi || !qkv_lo || !out) return QVIT_ENULL;
  if (epi_table && (((uintptr_t)epi_table) & 15)) return QVIT_EALIGN;
  if (head_dim != HD) return QVIT_EINVAL;
  if (B < 0 || N <= 0 || H <= 0 || ldo < H * HD) return QVIT_EINVAL;
  if (B * N > INT32_MAX || N > (1 << 20) || !(in_scale > 0.f)) return QVIT_EINVAL;
  if ((((uintptr_t)qkv_hi) & 15) || (((uintptr_t)qkv_lo) & 15)) return QVIT_EALIGN;
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
  const _Float16* hi = reinterpret_cast<const _Float16*>(qkv_hi);
  const _Float16* lo = reinterpret_cast<const _Float16*>(qkv_lo);
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                hipSuccess || n <= 0)
      n = 256;
    return n;
  }();
  const int64_t grid = std::min<int64_t>(nblk, 2 * (int64_t)cus);  // two resident workgroups per CU
  if (out_mode == QVIT_ATT_F32)
    hipLaunchKernelGGL(attn_split_kernel<0>, dim3((unsigned)grid), dim3(256), 0, stream, hi, lo, (int)N, (int)H,
                       (int)nblk, scale, in_scale, out, ldo, out_qtype, out_d, out_qm, out_t, out_levels,
                       nullptr);
  else
    hipLaunchKernelGGL(attn_split_kernel<1>, dim3((unsigned)grid), dim3(256), 0, stream, hi, lo, (int)N, (int)H,
                       (int)nblk, scale, in_scale, out, ldo, out_qtype, out_d, out_qm, out_t, out_levels,
                       reinterpret_cast<const int8_t*>(epi_table));
  return qvit_hip_status(hipGetLastError());
}

QVIT_ATT_STAMP_READER(qvit_att_stamps)  // diag_stamps.h: -DQVIT_ATT_STAMPS builds only
