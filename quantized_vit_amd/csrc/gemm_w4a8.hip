// Quantized contraction for QuantizeLinear / QuantizeConv2d (quant_layers.py:495-499,575-587):
//   C[m, n] = epilogue( sum_k A[m, k] * W[n, k] ),  A = int8 activation codes, W = int4/int8 weight
//   codes, exact int32 accumulation on v_mfma_i32_16x16x64_i8 (gfx950).
//
// Geometry (one workgroup = 256 threads = 4 waves, 2 workgroups per CU):
//   block tile 256 (n, weights) x 128 (m, activations); k advances in 64-deep stages.
//   Wave w owns weight rows [64w, 64w+64) and all 128 activation rows: 4 x 8 MFMA tiles of 16x16.
//   MFMA operand "A" (16 rows) = weights, operand "B" (16 cols) = activations.
// Pipeline: a 3-slot LDS ring of stages (16 KiB each for int4 weights, RING below). Both operands go
//   HBM/L2 -> LDS with global_load_lds_dwordx4 (issued from inline asm: no VGPRs, no ds_write, and
//   no compiler-inserted vmcnt drains) two stages ahead; one counted `s_waitcnt vmcnt` + barrier per
//   stage; the MFMA fragments of stage k+1 are read from LDS while the MFMAs of stage k run.
//   int4 weights stay packed in LDS and are sign-extended after the ds_read_b64 fragment read
//   (each unpacked fragment feeds 8 MFMAs).
// LDS images are XOR-swizzled through the per-lane SOURCE address (the DMA writes lane-linear), so
//   all fragment reads are bank-conflict free:
//   activations (64-B rows):  16-B chunk c of row r at c ^ (((r >> 2) & 1) << 1)   (ds_read_b128)
//   W4 weights  (32-B rows):   8-B chunk c of row r at c ^ (((r >> 3) & 1) << 1)   (ds_read_b64)
//   W8 weights  (64-B rows):  as activations.
// Epilogue: accumulators are staged through LDS (32 rows at a time per wave) and written back by a
//   rolled loop in which 16 lanes own one contiguous 64-column row segment: 256-B coalesced fp32
//   rows, 64-B int8 code rows, one inlined copy of the (GELU +) quantizer per element slot.
// Grid: one block per output tile; blockIdx is remapped so that consecutive tiles (same activation
//   panel, different weight panels) share an XCD and its L2.
#include <cmath>
#include <cstddef>
#include <type_traits>

#include "diag_stamps.h"
#include "ln_common.h"
#include "qvit_common.h"

namespace {

typedef int v4i __attribute__((ext_vector_type(4)));

// internal epilogue of qvit_gemm_resid_ln: QVIT_EPI_F32_RESID (stores written through, sc1) and, behind the last
// of a row block's tiles, LayerNorm + the next layer's activation quantizer of that block's rows
constexpr int EPI_RESID_LN = 16;

constexpr int BN = 256;    // weight rows per tile
constexpr int BK = 64;     // k per stage
constexpr int KTILE = 128; // the API's K granularity (QVIT_TILE_K): stages come in pairs
constexpr int RING = 3;    // LDS stages
#ifndef QVIT_GEMM_ALEAD
#define QVIT_GEMM_ALEAD 2
#endif
// register-weight GEMMs (L2 below): activation stages in flight ahead of the one being read (ring of ALEAD + 2)
constexpr int ALEAD = QVIT_GEMM_ALEAD;
static_assert(ALEAD == 2 || ALEAD == 3, "the tail steps are written out for 2 or 3");
// stages in flight ahead of the one being computed: 2 (the tail steps of a tile issue the next
// tile's stages 0 and 1; the steady steps issue stage kt + 2)
constexpr int EPI_LD = 68; // staged accumulator row pitch (ints): 64 + 4 pad
constexpr int EPI_ROWS = 16;                            // rows staged per pass per wave
constexpr int EPI_WAVE_BYTES = EPI_ROWS * EPI_LD * 4;   // 4352

// WM = waves along m: WM = 1 -> 4 waves, tile 256 (n) x 128 (m). The LDS holds the operand ring and a
// separate epilogue region (accumulator staging, or the int8 code table), so a block's epilogue never
// touches the ring and the DMA of its next tile's first stages proceeds underneath it.
template <int WFMT, int WM>
struct Geo {
  static constexpr int NT = 256 * WM;
  static constexpr int NWAVES = 4 * WM;
  static constexpr int BM = 128 * WM;
  static constexpr int XBYTES = BM * BK;                        // 8 KiB activation tile per stage
  static constexpr int WROW = (WFMT == QVIT_W4) ? BK / 2 : BK;  // bytes per weight row per stage
  static constexpr int WBYTES = BN * WROW;                      // 8 KiB (W4) / 16 KiB (W8)
  static constexpr int STAGE = XBYTES + WBYTES;
  static constexpr int RING_BYTES = RING * STAGE;
  static constexpr int EPI_BYTES = NWAVES * EPI_WAVE_BYTES;     // 17 KiB: staging, or a table of <= 2174 buckets
  static constexpr int BIAS_BYTES = BN * 4;                     // the tile's bias, DMA'd at its head
  static constexpr int QP_BYTES = 64;                           // the output quantizer's scalars
  static constexpr int LDS = RING_BYTES + EPI_BYTES + BIAS_BYTES + QP_BYTES;
  static constexpr int XPIECES = XBYTES / 1024 / NWAVES;        // 1-KiB DMA pieces per wave
  static constexpr int WPIECES = WBYTES / 1024 / NWAVES;
  static constexpr int DMA_PER_STAGE = XPIECES + WPIECES;       // per wave
  static constexpr int MIN_BLOCKS = (WFMT == QVIT_W4 && WM == 1) ? 2 : 1;
  static constexpr int TABLE_MAX_NB = (EPI_BYTES - 16) / 8;
};

// int4 weights as int8 MFMA operands scaled by 16: a nibble moved to the high half of its byte reads as
// the signed byte 16 w exactly (w in [-8, 7]), so the unpack is a mask (high nibbles) or a shift and a
// mask (low nibbles). The accumulators then hold 16 acc (|16 w a| <= 16256: no overflow for K <= 65536)
// and are shifted back exactly before the epilogue.
QVIT_DEV uint32_t nib16_lo(uint32_t p) { return (p << 4) & 0xF0F0F0F0u; }
QVIT_DEV uint32_t nib16_hi(uint32_t p) { return p & 0xF0F0F0F0u; }

// A lane's 32-B weight slice of a stage as two 16-B register loads from a wave-uniform base (the register-weight
// path): issued from asm, so the compiler's wait-count model never drains the asm-issued activation DMA for them;
// the counted stage waits cover them (2 per stage and wave, as the 2 weight DMA pieces they replace)
QVIT_DEV void ldw32(v4i& a, v4i& b, const void* sbase, uint32_t voff) {
  asm volatile("; qvit_asm_load\n\t"
               "global_load_dwordx4 %0, %2, %3\n\t"
               "global_load_dwordx4 %1, %2, %3 offset:16"
               : "=&v"(a), "=&v"(b)
               : "v"(voff), "s"(sbase)
               : "memory");
}

// The int8 register image (QVIT_W8R): a lane's four 16-B fragments of a stage, already unpacked to 16x-scaled int8
// (16 w, exactly the operand the W4 paths unpack to), as four loads from a wave-uniform base
QVIT_DEV void ldw64(v4i& a, v4i& b, v4i& c, v4i& d, const void* sbase, uint32_t voff) {
  asm volatile("; qvit_asm_load\n\t"
               "global_load_dwordx4 %0, %4, %5\n\t"
               "global_load_dwordx4 %1, %4, %5 offset:16\n\t"
               "global_load_dwordx4 %2, %4, %5 offset:32\n\t"
               "global_load_dwordx4 %3, %4, %5 offset:48"
               : "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(d)
               : "v"(voff), "s"(sbase)
               : "memory");
}

// The register-weight image (QVIT_W4R) of a packed QVIT_W4 weight: in every (tile_n, k-stage) chunk of 8 KiB, wave
// w's 2 KiB hold lane l's four 8-B fragments (rows 64 w + 16 r + (l & 15), logical k-chunk l >> 4, r = 0..3)
// contiguously at 32 l, so that a wave's weight slice of a stage is two fully coalesced 16-B loads per lane.
__global__ void pack_w4r_kernel(const int8_t* __restrict__ src, int8_t* __restrict__ dst, int64_t nunits) {
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= nunits) return;
  const int64_t c = u >> 10;
  const int w = (int)(u >> 8) & 3, ln = (int)(u >> 2) & 63, r = (int)u & 3;
  const int lfr = ln & 15, lfq = ln >> 4;
  const int row = 64 * w + 16 * r + lfr;
  *reinterpret_cast<uint2*>(dst + c * 8192 + w * 2048 + ln * 32 + r * 8) =
      *reinterpret_cast<const uint2*>(src + c * 8192 + row * 32 + ((lfq ^ (((lfr >> 3) & 1) << 1)) << 3));
}

// The int8 register image (QVIT_W8R) of a packed QVIT_W4 weight: every (tile_n, k-stage) chunk of the W4 image (8 KiB)
// becomes 16 KiB in which wave w's 4 KiB hold lane l's four 16-B MFMA operands (rows 64 w + 16 r + (l & 15), logical
// k-chunk l >> 4, r = 0..3, each nibble as the byte 16 w) contiguously at 64 l: the main loop loads them with four
// coalesced 16-B loads per stage and lane and feeds them to the MFMAs with no unpack.
__global__ void pack_w8r_kernel(const int8_t* __restrict__ src, int8_t* __restrict__ dst, int64_t nunits) {
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= nunits) return;
  const int64_t c = u >> 10;
  const int w = (int)(u >> 8) & 3, ln = (int)(u >> 2) & 63, r = (int)u & 3;
  const int lfr = ln & 15, lfq = ln >> 4;
  const int row = 64 * w + 16 * r + lfr;
  const uint2 p = *reinterpret_cast<const uint2*>(src + c * 8192 + row * 32 + ((lfq ^ (((lfr >> 3) & 1) << 1)) << 3));
  *reinterpret_cast<uint4*>(dst + c * 16384 + w * 4096 + ln * 64 + r * 16) =
      make_uint4(nib16_lo(p.x), nib16_hi(p.x), nib16_lo(p.y), nib16_hi(p.y));
}

// Wait until at most N of this wave's DMAs are in flight, retire its LDS reads, then barrier.
// The LDS drain is the builtin (lgkmcnt(0) = 0xC07F on gfx9) so the compiler's wait-count model sees
// it and does not re-drain lgkmcnt when the next stage's fragment reads are in flight.
template <int N>
QVIT_DEV void stage_sync() {
  __builtin_amdgcn_s_waitcnt(0xC07F);
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

struct EpiArgs {
  const float* d_act;
  const float* d_wt;
  const float* bias;
  int out_qtype;
  const float* out_d;
  const float* out_qm;
  const float* out_t;
  int out_levels;
  const int8_t* table;  // optional code table for the I8 epilogues (qvit_epi_table_build)
  int seq;              // QKV_SPLIT: rows per image
  float inv_seq;        // 1 / seq (row -> image with an exact correction)
  float in_scale;       // QKV_SPLIT: power-of-two operand scale
  _Float16* lo;         // QKV_SPLIT: lo plane (C is the hi plane)
  // EPI_RESID_LN: LayerNorm (gamma, beta, eps) of the finished rows + the next quantizer -> codes
  const float* ln_gamma;
  const float* ln_beta;
  float ln_eps;
  const int8_t* ln_table;  // its code table (EPI_I8 semantics), nullable
  int8_t* ln_codes;
  int64_t ln_ldc;
  int ln_kpad;
  int* ln_cnt;             // arrivals per 128-row block (zeroed by qvit_gemm_resid_ln before the launch)
};

// ---- code table of the int8 epilogues --------------------------------------------------------------
// The epilogue's output code as a function of its fp32 pre-activation v = alpha*acc + bias,
//   F(v) = quant_code(gelu_ref(v))  (EPI_I8_GELU)   or   quant_code(v)  (EPI_I8),
// is piecewise constant with at most 2L+1 values. Buckets of uniform width in v, each narrower than the
// smallest distance between two change points of F, hold (threshold, code below, code above):
//   F(v) = v >= thr ? hi : lo      for every v the index formula maps to that bucket,
// and the range [v_lo, v_lo + nb w) is chosen so F is constant beyond either end (the clamped index
// then still reads the right code). The table is built on the device by bisection with the very same F
// the direct epilogue evaluates, and validated (both ends constant, no bucket whose end codes differ
// by more than one); an invalid table makes the epilogue fall back to the direct computation.
QVIT_DEV float epi_F(float v, int gelu, const QParams& qp) { return quant_code(gelu ? gelu_ref(v) : v, qp); }

// float <-> totally ordered int key (for bisection over representable floats)
QVIT_DEV int fkey(float f) {
  const int i = __float_as_int(f);
  return i >= 0 ? i : (int)(0x80000000u - (unsigned)i);
}
QVIT_DEV float funkey(int k) { return __int_as_float(k >= 0 ? k : (int)(0x80000000u - (unsigned)k)); }

__global__ void epi_table_kernel(int gelu, int out_qtype, const float* out_d, const float* out_qm, const float* out_t,
                                 int out_levels, float c0, float inv_w, int nb, int8_t* table) {
  const QParams qp = load_qparams(out_qtype, out_d, out_qm, out_t, out_levels);
  EpiTableHdr* hdr = reinterpret_cast<EpiTableHdr*>(table);
  EpiTableEnt* ent = reinterpret_cast<EpiTableEnt*>(table + sizeof(EpiTableHdr));
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const float C = c0 + 8388608.f;  // epi_bucket_bits
  const float top = epi_top(nb);
  if (j == 0) {
    hdr->c0 = C;
    hdr->inv_w = inv_w;
    hdr->nb = nb;
  }
  if (j >= nb) return;
  // smallest float mapped to bucket >= j, and the largest float of bucket j
  auto first_at_least = [&](int b) {
    int lo = fkey(-3.0e38f), hi = fkey(3.0e38f);
    while (lo < hi) {
      const int mid = lo + ((hi - lo) >> 1);
      if (epi_bucket(funkey(mid), C, inv_w, top) >= b) hi = mid;
      else lo = mid + 1;
    }
    return lo;
  };
  const int ks = (j == 0) ? fkey(-3.0e38f) : first_at_least(j);
  const int ke = (j == nb - 1) ? fkey(3.0e38f) : first_at_least(j + 1) - 1;
  const float cs = epi_F(funkey(ks), gelu, qp), ce = epi_F(funkey(ke), gelu, qp);
  bool ok = fabsf(cs - ce) <= 1.f && !(isnan(cs) || isnan(ce));
  float thr = INFINITY;
  if (cs != ce) {  // the one change point inside the bucket: first v whose code differs from cs
    int lo = ks, hi = ke;
    while (lo < hi) {
      const int mid = lo + ((hi - lo) >> 1);
      if (epi_F(funkey(mid), gelu, qp) != cs) hi = mid;
      else lo = mid + 1;
    }
    thr = funkey(lo);
  }
  if (j == 0 || j == nb - 1) {  // F must be constant beyond the table's ends
    const float far = epi_F(j == 0 ? -1.0e30f : 1.0e30f, gelu, qp);
    if (far != (j == 0 ? cs : ce)) ok = false;
  }
  EpiTableEnt e;
  e.thr = thr;
  e.lo = to_i8_sat(cs);
  e.hi = to_i8_sat(ce);
  e.pad = 0;
  ent[j] = e;
  if (!ok) atomicAnd(&hdr->valid, 0);
}


template <int WFMT>
struct Frags {
  v4i x[8];
  uint2 w4[4];  // W4: packed 16 nibbles per lane
  v4i wq[4];    // W4R: the four fragments as loaded (wq[0..1]); W8R: the four int8 operands
  v4i w8[4];    // W8: 16 bytes per lane
};

// Residual rows of EPI_RESID_LN are handed to another workgroup inside the launch (the LayerNorm behind the
// last tile of a row block): written through with sc1 stores, read back with sc1 loads, the hand-off an agent-scope
// counter after every storing wave's vmcnt(0) (MI355X_MICROARCH.md, inter-workgroup visibility, Valid forms)
// (the sc1 store is a compiler-visible buffer store, so the hazard recognizer pads what follows it; C + 4 M ldc
// < 2^31 bytes, checked by the launcher)
template <bool SC1>
QVIT_DEV void st_resid(float* dst, float4 o, const float* C0, int M, int64_t ldc) {
  if constexpr (SC1) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(C0), (short)0,
                                                                        (int)((int64_t)M * ldc * 4), 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(f4v{o.x, o.y, o.z, o.w}, r, (int)((dst - C0) * 4), 0, 16);
  } else {
    *reinterpret_cast<float4*>(dst) = o;
  }
}

// Persistent kernel: gridDim.x = a multiple of 8 (blocks are dispatched round-robin over the 8 XCDs);
// XCD x's blocks share the contiguous tile range [lo_x, hi_x) (tile_n fastest, so the tiles in flight on
// one XCD share their activation panels in its L2), block slot s of the XCD walks lo_x + s + i * team.
// The operand stages form one stream across the block's tiles: the last two steps of a tile issue the
// DMA of the next tile's first two stages, so the pipeline never drains between tiles.
//
// RW (register weights): each wave's 64 weight rows are its own, so they come straight into registers, one stage
// ahead of their MFMAs, instead of through an LDS-DMA piece and a fragment read; the activations stay on the LDS-DMA
// ring. RW 1 = QVIT_W4R (two 16-B loads per stage and lane, unpacked like the LDS form; round 5: fc1 -2.6 % in the
// model, same box), RW 2 = QVIT_W8R (the same operands already unpacked: four 16-B loads, no unpack VALU).
//
// L2 (register weights, K >= 256): the activation stream runs two stages ahead instead of one, through a 4-slot ring
// of activation-only slots (8 KiB; the weight half of a slot is unused with register weights): step kt issues stage
// kt + 3's pieces and waits for stage kt + 1's, so a stage has two steps to land instead of one. The same barriers,
// reads and MFMAs per step; LDS 32 KiB of ring instead of 48.
template <int WFMT, int EPI, int WM, int RW, bool L2 = false>
__global__ __launch_bounds__((Geo<WFMT, WM>::NT), (Geo<WFMT, WM>::MIN_BLOCKS)) void gemm_kernel(
    const int8_t* __restrict__ A, int M, int K, int64_t lda, const int8_t* __restrict__ Wp, int N, int npad,
    void* __restrict__ C, int64_t ldc, EpiArgs ep) {
  using G = Geo<WFMT, WM>;
  constexpr int BM = G::BM;
  constexpr int XBYTES = G::XBYTES;
  constexpr bool I8OUT = (EPI == QVIT_EPI_I8 || EPI == QVIT_EPI_I8_GELU);
  static_assert(!L2 || RW != 0, "the two-ahead activation ring is for register weights");
  constexpr int RINGN = L2 ? ALEAD + 2 : RING;            // ring slots
  constexpr int SLOT = L2 ? XBYTES : G::STAGE;            // bytes per slot
  constexpr int RING_B = RINGN * SLOT;
  __shared__ __attribute__((aligned(16))) int8_t smem[RING_B + G::EPI_BYTES + G::BIAS_BYTES + G::QP_BYTES];
  int8_t* epi_lds = smem + RING_B;
  const float* bias_l = reinterpret_cast<const float*>(smem + RING_B + G::EPI_BYTES);
  QParams* qp_l = reinterpret_cast<QParams*>(smem + RING_B + G::EPI_BYTES + G::BIAS_BYTES);
  const bool has_bias = (EPI != QVIT_EPI_I32) && ep.bias != nullptr;
  constexpr bool REGW = RW != 0;
  static_assert(!RW || (WFMT == QVIT_W4 && WM == 1), "register weights: the W4 4-wave tile");
  constexpr int WREG = RW == 2 ? 4 : 2;                        // register loads per stage and wave (REGW)
  constexpr int WIMG = RW == 2 ? 2 * G::WBYTES : G::WBYTES;   // weight image bytes per (tile_n, stage)

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave & 3;   // weight rows [64 wn, 64 wn + 64)
  const int wm = wave >> 2;  // activation rows [128 wm, 128 wm + 128)
  const int fr = lane & 15;
  const int fq = lane >> 4;

  // ---- this block's tiles ---------------------------------------------------------------------
  const int nb_n = npad / BN;
  const int ntiles = nb_n * ((M + BM - 1) / BM);
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, team = gridDim.x >> 3;
  const int per = ntiles >> 3, rem = ntiles & 7;
  const int lo = xcd * per + (xcd < rem ? xcd : rem);
  const int hi = lo + per + (xcd < rem ? 1 : 0);
  int t = lo + slot;
  if (t >= hi) return;

  // epilogue scalars and the code table are set up before the main loop
  // W4 accumulators hold 16 acc exactly: the float epilogues fold the 1/16 into alpha, which gives the very
  // same fp32 results (float(16 acc) = 16 float(acc), and alpha/16 is exact), one shift per element cheaper
  float alpha = 0.f;
  if (EPI != QVIT_EPI_I32) alpha = (*ep.d_act) * (*ep.d_wt) * (WFMT == QVIT_W4 ? 0.0625f : 1.f);
  bool use_table = false;
  float t_c0 = 0.f, t_invw = 0.f, t_top = 0.f;  // wave-uniform (SGPRs)
  int t_nb = 1;
  if (I8OUT && ep.table != nullptr) {
    const EpiTableHdr h = *reinterpret_cast<const EpiTableHdr*>(ep.table);
    use_table = h.valid != 0 && h.nb <= G::TABLE_MAX_NB;
    t_c0 = h.c0;
    t_invw = h.inv_w;
    t_nb = h.nb;
    t_top = epi_top(h.nb);
    if (use_table) {  // -> the epilogue region, once per block (made visible by the first stage sync)
      const v4i* src = reinterpret_cast<const v4i*>(ep.table);
      for (int i = tid; i < (16 + 8 * t_nb + 15) / 16; i += G::NT) reinterpret_cast<v4i*>(epi_lds)[i] = src[i];
    }
  }
  // the direct quantizer's scalars: derived once (double-precision exp/log) and kept in LDS, so
  // nothing of it stays live across the main loop
  if (I8OUT && !use_table && tid == 0) *qp_l = load_qparams(ep.out_qtype, ep.out_d, ep.out_qm, ep.out_t, ep.out_levels);

  // ---- LDS-DMA sources (per lane) of a tile -----------------------------------------------------
  // activations: wave w stages rows [32w, 32w+32) as 2 pieces of 16 rows x 64 B (swizzle on the source)
  // weights: the packed (tile_n, stage) tile is the LDS image itself, staged as contiguous 1-KiB pieces
  constexpr int WROWS_PER_PIECE = 1024 / G::WROW;
  constexpr int WROWS_PER_WAVE = BN / G::NWAVES;
  const int nk = K / BK;  // even, >= 2
  // The per-lane parts of the DMA sources are tile-invariant: piece j of wave w stages the tile's rows
  // 32 w + 16 j + (lane >> 2), 16-B chunk (lane & 3) swizzled by row bit 2 (= lane bit 4, as 32 w + 16 j has no bit
  // below 4), so the lane offset (lane >> 2) lda + chunk is one value for every piece, wave and whole tile; the row
  // base m0 + 32 w + 16 j and the stage's k offset ride in the SGPR base (a 64-bit scalar add per piece, no VALU).
  // Only a tail tile (rows past M, clamped to M - 1 so no read leaves A) computes per-lane row offsets. The lane
  // offsets (DMA sources, fragment reads, weight slices) are computed at each tile head from an opaque lane id, so
  // none of them is live across the epilogue (the int8-code epilogues need every register of the budget) and a
  // stage does no per-lane address arithmetic.
  // PEEL (the fp32 / int32 epilogues on the W4 images): the tile's first stage accumulates onto zero (peeled)
  // instead of clearing the accumulators (the peeled copy of the step does not fit the W8R registers).
  constexpr bool PEEL = !I8OUT && RW != 2;
  uint32_t wlane = 0;
  auto tile_w = [&](int tt) -> uint32_t {
    return __builtin_amdgcn_readfirstlane((uint32_t)(tt % nb_n) * (uint32_t)(nk * WIMG));
  };
  auto tile_m0 = [&](int tt) -> int { return __builtin_amdgcn_readfirstlane((tt / nb_n) * BM); };
  auto lane_a = [&](int ln) -> uint32_t {
    return (uint32_t)(ln >> 2) * (uint32_t)lda + (uint32_t)(((ln & 3) ^ (((ln >> 4) & 1) << 1)) << 4);
  };
  uint32_t alane = 0;
  const uint32_t lds0 = lds_addr(smem);
  auto issue = [&](int m0, uint32_t wt, int kt, int rslot) __attribute__((always_inline)) {
    const uint32_t sx = lds0 + (uint32_t)(rslot * SLOT);
    const uint32_t sw = sx + XBYTES;
    if (m0 + BM <= M) {
      const int8_t* abase = A + (int64_t)(m0 + 32 * wave) * lda + kt * BK;
#pragma unroll
      for (int j = 0; j < G::XPIECES; ++j)
        dma16s(abase + (int64_t)(16 * j) * lda, alane, __builtin_amdgcn_readfirstlane(sx + (32 * wave + 16 * j) * BK));
    } else {
      const int ln = lane_opaque();
#pragma unroll
      for (int j = 0; j < G::XPIECES; ++j) {
        const int row = 32 * wave + 16 * j + (ln >> 2);
        int gm = m0 + row;
        gm = gm < M ? gm : M - 1;  // clamp the tail: staged, never stored
        const uint32_t a = (uint32_t)gm * (uint32_t)lda + (uint32_t)(((ln & 3) ^ (((row >> 2) & 1) << 1)) * 16);
        dma16s(A + kt * BK, a, __builtin_amdgcn_readfirstlane(sx + (32 * wave + 16 * j) * BK));
      }
    }
    if constexpr (!REGW) {
      const uint32_t wl = wlane;
      const int8_t* wbase = Wp + wt + (uint32_t)kt * G::WBYTES + (uint32_t)(wave * (G::WPIECES * 1024));
      // (piece j's 1-KiB step rides in the SGPR base: an instruction offset would move the LDS address too)
#pragma unroll
      for (int j = 0; j < G::WPIECES; ++j)
        dma16s(wbase + j * 1024, wl, __builtin_amdgcn_readfirstlane(sw + (WROWS_PER_WAVE * wave + WROWS_PER_PIECE * j) * G::WROW));
    }
  };
  // REGW: this wave's weight slice of stage kt -> f.wq (issued one stage ahead of its MFMAs: the stage wait of the
  // next step, which counts 4 younger operations, covers it)
  auto issue_w = [&](uint32_t wt, int kt, Frags<WFMT>& f) __attribute__((always_inline)) {
    if constexpr (RW == 1) {
      const int8_t* wbase = Wp + wt + (uint32_t)kt * WIMG + (uint32_t)(wave * (WIMG / 4));
      ldw32(f.wq[0], f.wq[1], wbase, wlane * 2u);
    } else if constexpr (RW == 2) {
      const int8_t* wbase = Wp + wt + (uint32_t)kt * WIMG + (uint32_t)(wave * (WIMG / 4));
      ldw64(f.wq[0], f.wq[1], f.wq[2], f.wq[3], wbase, wlane * 4u);
    }
  };
  // the loads of f.wq have landed (a counted wait above): tied here, so no use of them is scheduled earlier
  auto pin = [&](Frags<WFMT>& f) __attribute__((always_inline)) {
    if constexpr (RW == 1) asm volatile("; qvit_pin %0 %1" : "+v"(f.wq[0]), "+v"(f.wq[1]));
    if constexpr (RW == 2)
      asm volatile("; qvit_pin %0 %1 %2 %3" : "+v"(f.wq[0]), "+v"(f.wq[1]), "+v"(f.wq[2]), "+v"(f.wq[3]));
  };
  // per-lane fragment offsets inside a stage (set at each tile head; one add per stage moves them to the slot)
  int xoff = 0, woff = 0;
  auto lane_offsets = [&](int ln) __attribute__((always_inline)) {
    const int lfr = ln & 15, lfq = ln >> 4;
    xoff = (128 * wm + lfr) * BK + ((lfq ^ (((lfr >> 2) & 1) << 1)) << 4);
    woff = (WFMT == QVIT_W4) ? (64 * wn + lfr) * G::WROW + ((lfq ^ (((lfr >> 3) & 1) << 1)) << 3)
                             : (64 * wn + lfr) * G::WROW + ((lfq ^ (((lfr >> 2) & 1) << 1)) << 4);
    wlane = (uint32_t)ln * 16u;
    alane = lane_a(ln);
  };
  auto read_frags = [&](int rslot, Frags<WFMT>& f) {
    const int8_t* sx = smem + rslot * SLOT;
    const int8_t* sw = sx + XBYTES;
#pragma unroll
    for (int s = 0; s < 8; ++s) f.x[s] = *reinterpret_cast<const v4i*>(sx + xoff + s * 16 * BK);
    if constexpr (!REGW) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (WFMT == QVIT_W4)
          f.w4[r] = *reinterpret_cast<const uint2*>(sw + woff + r * 16 * G::WROW);
        else
          f.w8[r] = *reinterpret_cast<const v4i*>(sw + woff + r * 16 * G::WROW);
      }
    }
  };

  v4i acc[4][8];
  // ZERO: the tile's first stage accumulates onto 0 (no register clearing per tile)
  auto mfma_stage = [&](const Frags<WFMT>& f, auto zeroc) __attribute__((always_inline)) {
    constexpr bool ZERO = decltype(zeroc)::value;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      v4i wf;
      if constexpr (RW == 2) {
        wf = f.wq[r];
      } else if (WFMT == QVIT_W4) {
        uint2 p = f.w4[r];
        if constexpr (REGW) {
          const v4i q = f.wq[r >> 1];
          p = (r & 1) ? make_uint2((uint32_t)q[2], (uint32_t)q[3]) : make_uint2((uint32_t)q[0], (uint32_t)q[1]);
        }
        wf = v4i{(int)nib16_lo(p.x), (int)nib16_hi(p.x), (int)nib16_lo(p.y), (int)nib16_hi(p.y)};
      } else {
        wf = f.w8[r];
      }
#pragma unroll
      for (int s = 0; s < 8; ++s)
        acc[r][s] = __builtin_amdgcn_mfma_i32_16x16x64_i8(wf, f.x[s], ZERO ? v4i{0, 0, 0, 0} : acc[r][s], 0, 0, 0);
    }
  };

  // One pipeline step: stage kt is in registers (cur); bring stage kt+1 into registers (nxt).
  // The phases are fenced (sched_barrier) and the LDS drain at the top is compiler-visible, so the
  // fragment reads of stage kt+1 overlap the MFMAs of stage kt with no wait between them.
  // memory operations per stage and wave: the activation pieces + the weight pieces (LDS) or register loads
  constexpr int D = G::XPIECES + (REGW ? WREG : G::WPIECES);
  auto step_core = [&](Frags<WFMT>& cur, Frags<WFMT>& nxt, int next_slot, bool read,
                       auto zeroc) __attribute__((always_inline)) {
    if (read) read_frags(next_slot, nxt);
    __builtin_amdgcn_sched_barrier(0);
    mfma_stage(cur, zeroc);
    __builtin_amdgcn_sched_barrier(0);
  };

  // ---- EPI_RESID_LN: arrival of this tile at its row block; the last of the block's nb_n tiles runs the
  // LayerNorm + quantizer of its <= 128 rows (wave w: rows m0 + w + 4 i), reading every column back with sc1
  // loads (the other tiles were written through by other workgroups, possibly on other XCDs)
  auto ln_after_tile = [&](int m0) __attribute__((always_inline)) {
    int* flag = reinterpret_cast<int*>(qp_l);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 residual stores have landed
    __builtin_amdgcn_s_waitcnt(0xC07F);
    asm volatile("s_barrier" ::: "memory");
    if (tid == 0) {
      const int old = __hip_atomic_fetch_add(ep.ln_cnt + m0 / BM, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = old == nb_n - 1 ? 1 : 0;  // counters zeroed by the launcher
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    asm volatile("s_barrier" ::: "memory");
    if (*flag == 0) return;  // workgroup-uniform
    // the quantizer's code table -> the epilogue region (its staging is done: every wave passed the barrier)
    const int8_t* ent = nullptr;
    float c0 = 0.f, inv_w = 0.f, top = 0.f;
    QParams qp{};
    if (ep.ln_table != nullptr) {
      const EpiTableHdr h = *reinterpret_cast<const EpiTableHdr*>(ep.ln_table);
      if (h.valid != 0 && h.nb >= 1 && h.nb <= G::TABLE_MAX_NB) {
        const v4i* src = reinterpret_cast<const v4i*>(ep.ln_table);
        for (int i = tid; i < (16 + 8 * h.nb + 15) / 16; i += G::NT) reinterpret_cast<v4i*>(epi_lds)[i] = src[i];
        ent = epi_lds + sizeof(EpiTableHdr);
        c0 = h.c0;
        inv_w = h.inv_w;
        top = epi_top(h.nb);
      }
    }
    if (ent == nullptr) qp = load_qparams(ep.out_qtype, ep.out_d, ep.out_qm, ep.out_t, ep.out_levels);
    const int ln = lane_opaque();
    const int cols = N;
    float4 gam[4], bet[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = 4 * (ln + 64 * i);
      const bool in = c < cols;
      gam[i] = (in && ep.ln_gamma) ? *reinterpret_cast<const float4*>(ep.ln_gamma + c) : make_float4(1.f, 1.f, 1.f, 1.f);
      bet[i] = (in && ep.ln_beta) ? *reinterpret_cast<const float4*>(ep.ln_beta + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    asm volatile("s_barrier" ::: "memory");  // the table is in place
    // sc1 buffer loads (compiler-tracked) of a row's columns 4 (lane + 64 i) .. + 3; zero past the row; rows past
    // M read row M - 1. Wave w owns rows m0 + w + 4 i; they are taken 8 at a time with all 8 rows' loads in flight
    // together (the accumulator registers are free here), so the block's 128 rows cost 4 memory latencies.
    typedef float f4v __attribute__((ext_vector_type(4)));
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<void*>(static_cast<const void*>(C)), (short)0, (int)((int64_t)M * ldc * 4), 0x00020000);
    // wave w: rows m0 + w + 4 i (i < 32), three per loop iteration from a 3-deep register ring, each row's loads
    // issued two rows ahead; the rolled loop keeps the job's code small (an unrolled job thrashed the I-cache)
    auto job = [&](auto nvc, auto modec) __attribute__((always_inline)) {
      constexpr int NV = decltype(nvc)::value;
      constexpr int MODE = decltype(modec)::value;
      const int rend = (m0 + BM < M ? m0 + BM : M);
      auto ld = [&](int r, f4v (&t)[NV]) __attribute__((always_inline)) {
        const int rr = r < M ? r : M - 1;
#pragma unroll
        for (int i = 0; i < NV; ++i) {
          const int c = 4 * (ln + 64 * i);
          t[i] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)(((int64_t)rr * ldc + (c < cols ? c : 0)) * 4), 0, 16);
        }
      };
      auto row = [&](int r, const f4v (&t)[NV]) __attribute__((always_inline)) {
        float4 v[NV];
#pragma unroll
        for (int i = 0; i < NV; ++i)
          v[i] = (4 * (ln + 64 * i) < cols) ? make_float4(t[i][0], t[i][1], t[i][2], t[i][3])
                                            : make_float4(0.f, 0.f, 0.f, 0.f);
        uint32_t word[NV];
        auto gb = [&](int i, float4& g, float4& bb) {
          g = gam[i];
          bb = bet[i];
        };
        ln_quant_row<NV, decltype(gb), MODE>(v, ln, cols, ep.ln_eps, gb, ent, c0, inv_w, top, qp, word);
        if (r < rend) {
          int8_t* cr = ep.ln_codes + (int64_t)r * ep.ln_ldc;
#pragma unroll
          for (int i = 0; i < NV; ++i) {
            const int c = 4 * (ln + 64 * i);
            if (c < cols) *reinterpret_cast<uint32_t*>(cr + c) = word[i];
          }
          for (int c = cols + ln; c < ep.ln_kpad; c += 64) cr[c] = 0;
        }
      };
      f4v t0[NV], t1[NV], t2[NV];
      const int r0 = m0 + wave;
      ld(r0, t0);
      ld(r0 + 4, t1);
#pragma unroll 1
      for (int r = r0; r < rend; r += 12) {
        ld(r + 8, t2);
        row(r, t0);
        ld(r + 12, t0);
        row(r + 4, t1);
        ld(r + 16, t1);
        row(r + 8, t2);
      }
    };
    // (the direct quantizer, for a missing or invalid table, is the rare slow path: one row in flight, NV 4)
    if (ent == nullptr) job(std::integral_constant<int, 4>{}, std::integral_constant<int, 2>{});
    else if (cols <= 768) job(std::integral_constant<int, 3>{}, std::integral_constant<int, 1>{});
    else job(std::integral_constant<int, 4>{}, std::integral_constant<int, 1>{});
  };

  // prologue: the first tile's stages 0 and 1 (the Src values are scoped to one tile: nothing of them is
  // carried across a loop iteration)
  int g = 0;  // global stage counter of this block (ring slot = g % RINGN)
  {
    lane_offsets(lane_opaque());
    const int am0 = tile_m0(t);
    const uint32_t w0 = tile_w(t);
    issue(am0, w0, 0, 0);
    issue(am0, w0, 1, 1);
    if constexpr (L2)
      for (int j = 2; j <= ALEAD; ++j) issue(am0, w0, j, j);
  }
  Frags<WFMT> fa, fb;
  QVIT_STAMP_DECL
  QVIT_LSTAMP_DECL
  for (;;) {
    const int tnext = t + team;
    const bool has_next = tnext < hi;
    const int m0 = tile_m0(t), n0 = (t % nb_n) * BN;
    if (nk == 2 || !PEEL) {  // (K = 128: no steady step, the tail's first stage is the tile's first)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int s = 0; s < 8; ++s) acc[r][s] = v4i{0, 0, 0, 0};
    }

    if constexpr (L2) {
    // AL-ahead activation stream (AL = ALEAD: 2, or 3 in -DQVIT_GEMM_ALEAD=3 builds). Memory operations in issue
    // order (XP = G::XPIECES activation pieces, WREG weight loads per stage and wave): step kt issues w(kt + 1), then
    // act(kt + AL + 1) (this tile's, or in the tail steps nk-AL-1 .. nk-1 the next tile's stages 0 .. AL, or nothing).
    // Step kt needs w(kt) (issued by step kt - 1, or the head for kt = 0) and act(kt + 1) (older than w(kt)): its
    // wait leaves in flight exactly what was issued after w(kt) - step kt - 1's activation pieces and step kt's
    // operations - so vmcnt(2 XP + WREG) in the steady steps, less where a step issues nothing of a kind.
    // Ring slot safety (AL + 2 slots): act(kt + AL + 1) lands in the slot of stage kt - 1, whose fragments every wave
    // read in step kt - 2, before the barrier of step kt - 1.
    constexpr int XP = G::XPIECES;
    QVIT_STAMP(5);
    const uint32_t cw = tile_w(t);
    const int ln = lane_opaque();
    lane_offsets(ln);
    issue_w(cw, 0, fa);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    stage_sync<ALEAD * XP + WREG>();  // act(0): at most act(1 .. AL) and w(0) are younger and still in flight
    QVIT_STAMP(0);
    QVIT_LSTAMP(0);
    if (has_bias && wave == 0)
      dma16(ep.bias + n0 + ln * 4, __builtin_amdgcn_readfirstlane(lds0 + RING_B + G::EPI_BYTES));
    read_frags(g % RINGN, fa);
    // one step of this tile's stream: stage kt computes from cur, stage kt + 1's fragments are read into nxt
    auto lstep = [&](int kt, Frags<WFMT>& cur, Frags<WFMT>& nxt, auto zeroc) __attribute__((always_inline)) {
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_sched_barrier(0);
      issue_w(cw, kt + 1, nxt);
      issue(m0, cw, kt + ALEAD + 1, (g + kt + ALEAD + 1) % RINGN);
      QVIT_STAMP(1);
      stage_sync<2 * XP + WREG>();
      pin(cur);
      QVIT_STAMP(2);
      step_core(cur, nxt, (g + kt + 1) % RINGN, true, zeroc);
      QVIT_STAMP(3);
    };
    // step 0 (accumulators start at zero when PEEL): needs act(1), w(0); younger: w(1), act(AL + 1)
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_sched_barrier(0);
    issue_w(cw, 1, fb);
    issue(m0, cw, ALEAD + 1, (g + ALEAD + 1) % RINGN);
    QVIT_STAMP(1);
    stage_sync<XP + WREG>();
    pin(fa);
    QVIT_STAMP(2);
    if constexpr (PEEL) step_core(fa, fb, (g + 1) % RINGN, true, std::true_type{});
    else step_core(fa, fb, (g + 1) % RINGN, true, std::false_type{});
    QVIT_STAMP(3);
    // steady steps 1 .. nk-AL-2 (nk is even, so their count has AL's parity): an odd count starts with step 1
    // alone, then pairs (stage kt in cur = kt odd ? fb : fa)
    int kt = 1;
    if constexpr (ALEAD & 1) {
      lstep(1, fb, fa, std::false_type{});
      kt = 2;
      for (; kt + 1 <= nk - ALEAD - 2; kt += 2) {
        lstep(kt, fa, fb, std::false_type{});
        lstep(kt + 1, fb, fa, std::false_type{});
      }
    } else {
      for (; kt + 1 <= nk - ALEAD - 2; kt += 2) {
        lstep(kt, fb, fa, std::false_type{});
        lstep(kt + 1, fa, fb, std::false_type{});
      }
    }
    // tail steps j = 0 .. AL (kt = nk - AL - 1 + j): the next tile's stage j, if any; the weight load goes out before
    // the branch, so every path from a load to its use holds a covering wait (tools/asm_load_check.py)
    const uint32_t nw = has_next ? tile_w(tnext) : 0u;
    const int nm0 = has_next ? tile_m0(tnext) : 0;
    auto tstep = [&](auto jc, Frags<WFMT>& cur, Frags<WFMT>& nxt) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      const int tk = nk - ALEAD - 1 + j;
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (j < ALEAD) issue_w(cw, tk + 1, nxt);
      // younger than w(tk): the previous step's activation pieces (always issued before the tail, else only with a
      // next tile), this step's weights and activation pieces
      constexpr int NW = j < ALEAD ? WREG : 0;
      if (has_next) {
        issue(nm0, nw, j, (g + nk + j) % RINGN);
        if constexpr (j < ALEAD) stage_sync<2 * XP + NW>();
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * XP) : "memory");
      } else {
        if constexpr (j < ALEAD) stage_sync<(j == 0 ? XP : 0) + NW>();
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      pin(cur);
      step_core(cur, nxt, (g + tk + 1) % RINGN, j < ALEAD, std::false_type{});
    };
    if constexpr (ALEAD & 1) {   // nk - AL - 1 even: the tail starts in fa
      tstep(std::integral_constant<int, 0>{}, fa, fb);
      tstep(std::integral_constant<int, 1>{}, fb, fa);
      tstep(std::integral_constant<int, 2>{}, fa, fb);
      tstep(std::integral_constant<int, 3>{}, fb, fa);
    } else {
      tstep(std::integral_constant<int, 0>{}, fb, fa);
      tstep(std::integral_constant<int, 1>{}, fa, fb);
      tstep(std::integral_constant<int, 2>{}, fb, fa);
    }
    QVIT_STAMP(3);
    QVIT_LSTAMP(1);
    } else {
    // head: stage 0 of this tile landed (stage 1 may still be in flight); every wave is past the
    // previous tile's epilogue, so the tile's bias can be DMA'd into its LDS slot (1 KiB, wave 0;
    // older than every later stage DMA, so the counted stage waits cover it)
    QVIT_STAMP(5);
    const uint32_t cw = tile_w(t);
    const int ln = lane_opaque();
    lane_offsets(ln);
    issue_w(cw, 0, fa);  // REGW: stage 0's weights (covered by the first stage wait below the head)
    __builtin_amdgcn_s_waitcnt(0xC07F);
    stage_sync<D>();
    QVIT_STAMP(0);
    QVIT_LSTAMP(0);
    {
      if (has_bias && wave == 0)
        dma16(ep.bias + n0 + ln * 4, __builtin_amdgcn_readfirstlane(lds0 + RING_B + G::EPI_BYTES));
    }
    read_frags(g % RINGN, fa);
    // steady steps kt = 0 .. nk-3: issue this tile's stage kt+2 (the first one peeled: zero accumulators)
    int kt = 0;
    if (PEEL && nk > 2) {
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_sched_barrier(0);
      issue(m0, cw, 2, (g + 2) % RINGN);
      issue_w(cw, 1, fb);
      QVIT_STAMP(1);
      stage_sync<D>();
      pin(fa);
      QVIT_STAMP(2);
      step_core(fa, fb, (g + 1) % RING, true, std::true_type{});
      QVIT_STAMP(3);
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_sched_barrier(0);
      issue(m0, cw, 3, (g + 3) % RINGN);
      issue_w(cw, 2, fa);
      QVIT_STAMP(1);
      stage_sync<D>();
      pin(fb);
      QVIT_STAMP(2);
      step_core(fb, fa, (g + 2) % RING, true, std::false_type{});
      QVIT_STAMP(3);
      kt = 2;
    }
    for (; kt < nk - 2; kt += 2) {
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_sched_barrier(0);
      issue(m0, cw, kt + 2, (g + kt + 2) % RINGN);
      issue_w(cw, kt + 1, fb);
      QVIT_STAMP(1);
      stage_sync<D>();
      pin(fa);
      QVIT_STAMP(2);
      step_core(fa, fb, (g + kt + 1) % RING, true, std::false_type{});
      QVIT_STAMP(3);
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_sched_barrier(0);
      issue(m0, cw, kt + 3, (g + kt + 3) % RINGN);
      issue_w(cw, kt + 2, fa);
      QVIT_STAMP(1);
      stage_sync<D>();
      pin(fb);
      QVIT_STAMP(2);
      step_core(fb, fa, (g + kt + 2) % RING, true, std::false_type{});
      QVIT_STAMP(3);
    }
    // tail kt = nk-2, nk-1: issue the next tile's stages 0, 1
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_sched_barrier(0);
    const uint32_t nw = has_next ? tile_w(tnext) : 0u;
    const int nm0 = has_next ? tile_m0(tnext) : 0;
    // (REGW: the last stage's weights go out before the branches, so every path from their load to their pin
    // holds a covering wait - tools/asm_load_check.py walks all of them - and the counts are those of the steady
    // steps: with a next tile, stage_sync<D> leaves exactly the weights and the next tile's stage-0 pieces in flight)
    issue_w(cw, nk - 1, fb);
    if (has_next) {
      issue(nm0, nw, 0, (g + nk) % RINGN);
      stage_sync<D>();
    } else {
      stage_sync<REGW ? WREG : 0>();
    }
    pin(fa);
    step_core(fa, fb, (g + nk - 1) % RING, true, std::false_type{});
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_sched_barrier(0);
    if (has_next) {
      issue(nm0, nw, 1, (g + nk + 1) % RINGN);
      // the last stage's weights (younger: the next tile's stage-1 pieces)
      if constexpr (REGW) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::XPIECES) : "memory");
    } else {
      if constexpr (REGW) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    pin(fb);
    step_core(fb, fa, 0, false, std::false_type{});
    QVIT_STAMP(3);
    QVIT_LSTAMP(1);

    }

    if (WFMT == QVIT_W4 && EPI == QVIT_EPI_I32) {  // 16 acc -> acc (exact arithmetic shift)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int sr = 0; sr < 8; ++sr)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[r][sr][j] >>= 4;
    }
    {
    // ---- epilogue (epilogue LDS region only; the next tile's DMA streams underneath) -----------
    // acc[r][s][j] = C[m0 + 128 wm + 16 s + fr][n0 + 64 wn + 16 fq + 4 r + j] (weight rows pre-permuted)
    const int el = lane_opaque();
    // the int8 epilogue (VALU + LDS lookups) runs at raised wave priority: the co-resident block's
    // main loop keeps the matrix pipe busy either way, and the epilogue no longer loses every issue
    // arbitration to it (fc1: -9 % time; the fp32 epilogues wait on memory and gain nothing)
    if (I8OUT) __builtin_amdgcn_s_setprio(1);
    const int efr = el & 15, efq = el >> 4;
    if (I8OUT && use_table) {
      // register path: lane (fr, fq) owns the 16 consecutive columns [nbase, nbase+16) of rows
      // m0 + 16 s + fr, so each accumulator row leaves as one 16-B code store
      const int8_t* tlb = epi_lds + sizeof(EpiTableHdr);  // 8-B entries {thr, lo | hi << 8}
      const int nbase = n0 + 64 * wn + 16 * efq;
      float bcol[16];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float4 b = make_float4(0.f, 0.f, 0.f, 0.f);
        if (has_bias) b = *reinterpret_cast<const float4*>(bias_l + (nbase - n0) + 4 * r);
        bcol[4 * r] = b.x; bcol[4 * r + 1] = b.y; bcol[4 * r + 2] = b.z; bcol[4 * r + 3] = b.w;
      }
      // 16-B row stores when every row segment is whole and aligned (kernel-uniform); else byte stores
      const bool fast16 = ((ldc & 15) == 0) && ((((uintptr_t)C) & 15) == 0) && ((N & 15) == 0);
      // software-pipelined over the 8 rows: row sr + 1's 16 lookups are issued before row sr's are resolved, so
      // each row's LDS latency runs under the previous row's selects and store (the fragment registers of the
      // main loop are free here: two rows of values and entries fit beside the accumulators)
      float v[2][4][4];
      uint2 e[2][4][4];
      auto look = [&](int sr, int b) __attribute__((always_inline)) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[b][r][j] = fmaf(alpha, (float)acc[r][sr][j], bcol[4 * r + j]);
            e[b][r][j] = *epi_entry(tlb, v[b][r][j], t_c0, t_invw, t_top);
          }
      };
      look(0, 0);
#pragma unroll
      for (int sr = 0; sr < 8; ++sr) {
        const int cb = sr & 1;
        if (sr + 1 < 8) look(sr + 1, cb ^ 1);
        __builtin_amdgcn_sched_barrier(0);
        const int m = m0 + 128 * wm + 16 * sr + efr;
        uint32_t wd[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          epi_select_byte<0>(wd[r], v[cb][r][0], __uint_as_float(e[cb][r][0].x), e[cb][r][0].y);
          epi_select_byte<1>(wd[r], v[cb][r][1], __uint_as_float(e[cb][r][1].x), e[cb][r][1].y);
          epi_select_byte<2>(wd[r], v[cb][r][2], __uint_as_float(e[cb][r][2].x), e[cb][r][2].y);
          epi_select_byte<3>(wd[r], v[cb][r][3], __uint_as_float(e[cb][r][3].x), e[cb][r][3].y);
        }
        int8_t* dst = reinterpret_cast<int8_t*>(C) + (int64_t)m * ldc + nbase;
        if (fast16) {
          if (m < M && nbase < N) *reinterpret_cast<uint4*>(dst) = make_uint4(wd[0], wd[1], wd[2], wd[3]);
        } else if (m < M) {
#pragma unroll
          for (int q = 0; q < 16; ++q)
            if (nbase + q < N) dst[q] = (int8_t)((wd[q >> 2] >> (8 * (q & 3))) & 0xff);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    } else if (EPI == QVIT_EPI_F32_RESID || EPI == EPI_RESID_LN) {
      // C += alpha acc + bias: 16 rows per pass through the wave's staging area, 16 lanes per 64-column
      // row segment; the residual rows of pass sr + 1 are loaded while pass sr is staged and stored, so
      // the read-modify-write pays one memory latency per tile instead of one per row
      int* stg = reinterpret_cast<int*>(epi_lds + wave * EPI_WAVE_BYTES);
      const int prow = el >> 4, pcol = 4 * (el & 15);
      const int n = n0 + 64 * wn + pcol;
      const bool nfull = n + 4 <= N;
      float4 b4 = make_float4(0.f, 0.f, 0.f, 0.f);
      if (has_bias) b4 = *reinterpret_cast<const float4*>(bias_l + (n - n0));
      float* Cf = reinterpret_cast<float*>(C);
      float4 old[2][4];
      if (m0 + BM <= M && n0 + BN <= N) {
        // whole tile: the residual rows are loaded by inline asm, which the compiler does not track,
        // and waited for with exact counts (pass sr's loads are older than the previous pass's 4 stores
        // and the next pass's 4 loads), so neither the loads of pass sr + 1 nor the stores in flight are
        // drained at every pass, as the compiler's own vmcnt(0) would (the DMA ring is in flight)
        typedef float f4v __attribute__((ext_vector_type(4)));
        f4v ov0[4], ov1[4];
        auto ld = [&](int sr, f4v (&ov)[4]) __attribute__((always_inline)) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float* src = Cf + (int64_t)(m0 + 128 * wm + 16 * sr + 4 * i + prow) * ldc + n;
            asm volatile("; qvit_asm_load\n\tglobal_load_dwordx4 %0, %1, off" : "=v"(ov[i]) : "v"(src) : "memory");
          }
        };
        auto pass = [&](int sr, f4v (&ov)[4]) __attribute__((always_inline)) {
          __builtin_amdgcn_s_waitcnt(0xC07F);
#pragma unroll
          for (int r = 0; r < 4; ++r)
            *reinterpret_cast<v4i*>(stg + efr * EPI_LD + 16 * efq + 4 * r) = acc[r][sr];
          __builtin_amdgcn_s_waitcnt(0xC07F);
          __builtin_amdgcn_wave_barrier();
          // tie the wait to the loaded registers, so no use of them is scheduled above it
          if (sr == 0 || sr == 7)
            asm volatile("s_waitcnt vmcnt(4)\n\t; qvit_pin %0 %1 %2 %3"
                         : "+v"(ov[0]), "+v"(ov[1]), "+v"(ov[2]), "+v"(ov[3]) :: "memory");
          else
            asm volatile("s_waitcnt vmcnt(8)\n\t; qvit_pin %0 %1 %2 %3"
                         : "+v"(ov[0]), "+v"(ov[1]), "+v"(ov[2]), "+v"(ov[3]) :: "memory");
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int row = 4 * i + prow;
            const int m = m0 + 128 * wm + 16 * sr + row;
            const v4i a4 = *reinterpret_cast<const v4i*>(stg + row * EPI_LD + pcol);
            float4 o = make_float4(alpha * (float)a4[0] + b4.x, alpha * (float)a4[1] + b4.y,
                                   alpha * (float)a4[2] + b4.z, alpha * (float)a4[3] + b4.w);
            o.x += ov[i][0]; o.y += ov[i][1]; o.z += ov[i][2]; o.w += ov[i][3];
            st_resid<EPI == EPI_RESID_LN>(Cf + (int64_t)m * ldc + n, o, Cf, M, ldc);
          }
        };
        ld(0, ov0);
#pragma unroll
        for (int sr = 0; sr < 8; sr += 2) {
          ld(sr + 1, ov1);
          pass(sr, ov0);
          if (sr + 2 < 8) ld(sr + 2, ov0);
          pass(sr + 1, ov1);
        }
      } else {
      auto load_old = [&](int sr, float4 (&ov)[4]) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = m0 + 128 * wm + 16 * sr + 4 * i + prow;
          ov[i] = (m < M && nfull) ? *reinterpret_cast<const float4*>(Cf + (int64_t)m * ldc + n)
                                   : make_float4(0.f, 0.f, 0.f, 0.f);
        }
      };
      load_old(0, old[0]);
#pragma unroll
      for (int sr = 0; sr < 8; ++sr) {
        if (sr + 1 < 8) load_old(sr + 1, old[(sr + 1) & 1]);
        __builtin_amdgcn_s_waitcnt(0xC07F);
#pragma unroll
        for (int r = 0; r < 4; ++r)
          *reinterpret_cast<v4i*>(stg + efr * EPI_LD + 16 * efq + 4 * r) = acc[r][sr];
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = 4 * i + prow;
          const int m = m0 + 128 * wm + 16 * sr + row;
          const v4i a4 = *reinterpret_cast<const v4i*>(stg + row * EPI_LD + pcol);
          if (m < M) {
            float4 o = make_float4(alpha * (float)a4[0] + b4.x, alpha * (float)a4[1] + b4.y,
                                   alpha * (float)a4[2] + b4.z, alpha * (float)a4[3] + b4.w);
            float* dst = Cf + (int64_t)m * ldc + n;
            if (nfull) {
              const float4 ov = old[sr & 1][i];
              o.x += ov.x; o.y += ov.y; o.z += ov.z; o.w += ov.w;
              st_resid<EPI == EPI_RESID_LN>(dst, o, Cf, M, ldc);
            } else {
              const float v[4] = {o.x, o.y, o.z, o.w};
              for (int j = 0; j < 4; ++j)
                if (n + j < N) dst[j] = dst[j] + v[j];
            }
          }
        }
      }
      }
    } else if (EPI == QVIT_EPI_QKV_SPLIT) {
      // fp16 hi/lo planes: 8 lanes per 64-column head-plane row, 8 columns (16 B of hi, 16 B of lo) each
      int* stg = reinterpret_cast<int*>(epi_lds + wave * EPI_WAVE_BYTES);
      const int prow = el >> 3, pcol = 8 * (el & 7);
      const int nw = n0 + 64 * wn;  // the wave's head plane (N % 64 == 0: all valid or none)
      float bb[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) bb[j] = has_bias ? bias_l[nw - n0 + pcol + j] : 0.f;
      const int64_t pstride = (int64_t)ep.seq * 64;
#pragma unroll
      for (int sr = 0; sr < 8; ++sr) {
        __builtin_amdgcn_s_waitcnt(0xC07F);
#pragma unroll
        for (int r = 0; r < 4; ++r)
          *reinterpret_cast<v4i*>(stg + efr * EPI_LD + 16 * efq + 4 * r) = acc[r][sr];
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int row = 8 * i + prow;
          const int m = m0 + 128 * wm + 16 * sr + row;
          const v4i a0 = *reinterpret_cast<const v4i*>(stg + row * EPI_LD + pcol);
          const v4i a1 = *reinterpret_cast<const v4i*>(stg + row * EPI_LD + pcol + 4);
          if (m < M && nw < N) {
            int bimg = (int)((float)m * ep.inv_seq);
            bimg -= (bimg * ep.seq > m) ? 1 : 0;
            bimg += ((bimg + 1) * ep.seq <= m) ? 1 : 0;
            const int tok = m - bimg * ep.seq;
            const int64_t e = ((int64_t)bimg * (N >> 6) + (nw >> 6)) * pstride + (int64_t)tok * 64 + pcol;
            uint32_t hw[4], lw[4];
#pragma unroll
            for (int j = 0; j < 8; j += 2) {
              const int a_0 = (j < 4) ? a0[j] : a1[j - 4], a_1 = (j < 4) ? a0[j + 1] : a1[j - 3];
              const float x0 = (alpha * (float)a_0 + bb[j]) * ep.in_scale;
              const float x1 = (alpha * (float)a_1 + bb[j + 1]) * ep.in_scale;
              const _Float16 h0 = (_Float16)x0, h1 = (_Float16)x1;
              const _Float16 l0 = (_Float16)(x0 - (float)h0), l1 = (_Float16)(x1 - (float)h1);
              hw[j >> 1] = (uint32_t)__builtin_bit_cast(uint16_t, h0) | ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
              lw[j >> 1] = (uint32_t)__builtin_bit_cast(uint16_t, l0) | ((uint32_t)__builtin_bit_cast(uint16_t, l1) << 16);
            }
            *reinterpret_cast<uint4*>(reinterpret_cast<_Float16*>(C) + e) = make_uint4(hw[0], hw[1], hw[2], hw[3]);
            *reinterpret_cast<uint4*>(ep.lo + e) = make_uint4(lw[0], lw[1], lw[2], lw[3]);
          }
        }
      }
    } else {
      // staged path: 16 accumulator rows at a time through this wave's own staging area, then 16 lanes
      // own one contiguous 64-column row segment (256-B fp32 rows / 64-B code rows); wave-local only
      int* stg = reinterpret_cast<int*>(epi_lds + wave * EPI_WAVE_BYTES);
      const int prow = el >> 4;          // row 4 i + prow of the staged 16
      const int pcol = 4 * (el & 15);    // 4 consecutive columns of the wave's 64
      const int n = n0 + 64 * wn + pcol;
      const bool nfull = n + 4 <= N;
      float4 b4 = make_float4(0.f, 0.f, 0.f, 0.f);
      if (has_bias) b4 = *reinterpret_cast<const float4*>(bias_l + (n - n0));
      QParams qp;
      if (I8OUT) qp = *qp_l;
#pragma unroll
      for (int sr = 0; sr < 8; ++sr) {
        __builtin_amdgcn_s_waitcnt(0xC07F);  // the previous pass's staged reads are done
#pragma unroll
        for (int r = 0; r < 4; ++r)
          *reinterpret_cast<v4i*>(stg + efr * EPI_LD + 16 * efq + 4 * r) = acc[r][sr];
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
#pragma unroll 1
        for (int i = 0; i < 4; ++i) {
          const int row = 4 * i + prow;
          const int m = m0 + 128 * wm + 16 * sr + row;
          const v4i a4 = *reinterpret_cast<const v4i*>(stg + row * EPI_LD + pcol);
          if (m < M) {
            if (EPI == QVIT_EPI_I32) {
              int32_t* dst = reinterpret_cast<int32_t*>(C) + (int64_t)m * ldc + n;
              if (nfull) {
                *reinterpret_cast<v4i*>(dst) = a4;
              } else {
                for (int j = 0; j < 4; ++j)
                  if (n + j < N) dst[j] = a4[j];
              }
            } else if (EPI == QVIT_EPI_F32 || EPI == QVIT_EPI_F32_RESID) {
              float4 o = make_float4(alpha * (float)a4[0] + b4.x, alpha * (float)a4[1] + b4.y,
                                     alpha * (float)a4[2] + b4.z, alpha * (float)a4[3] + b4.w);
              float* dst = reinterpret_cast<float*>(C) + (int64_t)m * ldc + n;
              if (nfull) {
                if (EPI == QVIT_EPI_F32_RESID) {
                  const float4 old = *reinterpret_cast<const float4*>(dst);
                  o.x += old.x; o.y += old.y; o.z += old.z; o.w += old.w;
                }
                *reinterpret_cast<float4*>(dst) = o;
              } else {
                const float ov[4] = {o.x, o.y, o.z, o.w};
                for (int j = 0; j < 4; ++j)
                  if (n + j < N) dst[j] = (EPI == QVIT_EPI_F32_RESID) ? dst[j] + ov[j] : ov[j];
              }
            } else {
              const float bb[4] = {b4.x, b4.y, b4.z, b4.w};
              float v[4], k[4];
              bool need[4];
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                v[j] = alpha * (float)a4[j] + bb[j];
                if (EPI == QVIT_EPI_I8_GELU) v[j] = gelu_ref(v[j]);
                k[j] = quant_fast(v[j], qp, need[j]);
              }
              if (__any(need[0] | need[1] | need[2] | need[3])) {  // rare: near-tie elements
#pragma unroll
                for (int j = 0; j < 4; ++j)
                  if (need[j]) k[j] = quant_fixup(v[j], qp);
              }
              uint32_t word = 0;
#pragma unroll
              for (int j = 0; j < 4; ++j) word |= ((uint32_t)(uint8_t)to_i8_sat(k[j])) << (8 * j);
              int8_t* dst = reinterpret_cast<int8_t*>(C) + (int64_t)m * ldc + n;
              if (nfull) {
                *reinterpret_cast<uint32_t*>(dst) = word;
              } else {
                for (int j = 0; j < 4; ++j)
                  if (n + j < N) dst[j] = (int8_t)((word >> (8 * j)) & 0xff);
              }
            }
          }
        }
      }
    }
    }
    if (I8OUT) __builtin_amdgcn_s_setprio(0);
    QVIT_STAMP(4);
    QVIT_LSTAMP(2);
    if constexpr (EPI == EPI_RESID_LN) {
      ln_after_tile(m0);
      QVIT_STAMP(6);
    }
    if (!has_next) break;
    t = tnext;
    g += nk;
  }
  QVIT_STAMP_FLUSH;
  QVIT_LSTAMP_FLUSH;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int device_cus() {
  static int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                hipSuccess || n <= 0)
      n = 256;
    return n;
  }();
  return cus;
}

#ifndef QVIT_GEMM_L2
#define QVIT_GEMM_L2 1
#endif
constexpr bool GEMM_L2 = QVIT_GEMM_L2 != 0;  // (diagnostic builds: -DQVIT_GEMM_L2=0 for the one-ahead ring)

template <int WFMT, int EPI, int RW = 0>
int launch(const int8_t* A, int64_t M, int64_t K, int64_t lda, const void* Wp, int64_t N, int64_t npad,
           void* C, int64_t ldc, const EpiArgs& ep, hipStream_t stream) {
  constexpr int WMV = 1;   // (a second W4 tile width was measured slower in round 3: DESIGN.md section 8)
  using G = Geo<WFMT, WMV>;
  // the kernel addresses A and Wp as 32-bit byte offsets from the base pointers: rows are launched in
  // chunks whose A span stays below 2^32 (one chunk for every ViT / UltraNet shape)
  const int64_t span = (int64_t)0xFFFFFFFF - K;
  int64_t rows = span / lda / G::BM * G::BM;
  if (rows < G::BM || npad * (K / (WFMT == QVIT_W4 && RW != 2 ? 2 : 1)) > span) return QVIT_EINVAL;
  if (EPI == QVIT_EPI_QKV_SPLIT && rows < M) return QVIT_EINVAL;  // its row -> (image, token) map is global
  const int64_t esize = (EPI == QVIT_EPI_I8 || EPI == QVIT_EPI_I8_GELU) ? 1 : 4;
  for (int64_t m0 = 0; m0 < M; m0 += rows) {
    const int64_t mc = (M - m0 < rows) ? M - m0 : rows;
    const int64_t ntiles = (npad / BN) * ((mc + G::BM - 1) / G::BM);
    // resident blocks, a multiple of 8 (one team per XCD), no more than the tiles need
    int64_t grid = (int64_t)device_cus() * G::MIN_BLOCKS / 8 * 8;
    const int64_t need = (ntiles + 7) / 8 * 8;
    if (grid > need) grid = need;
    if (grid < 8) grid = 8;
    void* Cc = reinterpret_cast<int8_t*>(C) + (EPI == QVIT_EPI_QKV_SPLIT ? 0 : m0 * ldc * esize);
    EpiArgs epc = ep;
    if (EPI == EPI_RESID_LN) {  // this chunk's row blocks and code rows
      epc.ln_cnt = ep.ln_cnt + m0 / G::BM;
      epc.ln_codes = ep.ln_codes + m0 * ep.ln_ldc;
    }
    // register weights and K >= 256 (4 stages or more per tile): the two-ahead activation ring
    if (RW != 0 && K / BK >= ALEAD + 2 && GEMM_L2)
      hipLaunchKernelGGL((gemm_kernel<WFMT, EPI, WMV, RW, RW != 0>), dim3((unsigned)grid), dim3(G::NT), 0, stream,
                         A + m0 * lda, (int)mc, (int)K, lda, reinterpret_cast<const int8_t*>(Wp), (int)N, (int)npad, Cc,
                         ldc, epc);
    else
      hipLaunchKernelGGL((gemm_kernel<WFMT, EPI, WMV, RW>), dim3((unsigned)grid), dim3(G::NT), 0, stream,
                         A + m0 * lda, (int)mc, (int)K, lda, reinterpret_cast<const int8_t*>(Wp), (int)N, (int)npad, Cc,
                         ldc, epc);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return qvit_hip_status(e);
  }
  return QVIT_OK;
}

template <int WFMT, int RW = 0>
int dispatch_epi(int epilogue, const int8_t* A, int64_t M, int64_t K, int64_t lda, const void* Wp, int64_t N,
                 int64_t npad, void* C, int64_t ldc, const EpiArgs& ep, hipStream_t stream) {
  switch (epilogue) {
    case QVIT_EPI_F32: return launch<WFMT, QVIT_EPI_F32, RW>(A, M, K, lda, Wp, N, npad, C, ldc, ep, stream);
    case QVIT_EPI_F32_RESID: return launch<WFMT, QVIT_EPI_F32_RESID, RW>(A, M, K, lda, Wp, N, npad, C, ldc, ep, stream);
    case QVIT_EPI_I8_GELU: return launch<WFMT, QVIT_EPI_I8_GELU, RW>(A, M, K, lda, Wp, N, npad, C, ldc, ep, stream);
    case QVIT_EPI_I8: return launch<WFMT, QVIT_EPI_I8, RW>(A, M, K, lda, Wp, N, npad, C, ldc, ep, stream);
    case QVIT_EPI_I32: return launch<WFMT, QVIT_EPI_I32, RW>(A, M, K, lda, Wp, N, npad, C, ldc, ep, stream);
    case QVIT_EPI_QKV_SPLIT:
      return launch<WFMT, QVIT_EPI_QKV_SPLIT, RW>(A, M, K, lda, Wp, N, npad, C, ldc, ep, stream);
    default: return QVIT_EINVAL;
  }
}

}  // namespace

extern "C" int qvit_epi_table_build(int epilogue, int out_qtype, const float* out_d, const float* out_qm,
                                    const float* out_t, int out_levels, float v_lo, float w, int64_t nb, void* table,
                                    hipStream_t stream) {
  if (!table) return QVIT_ENULL;
  if (epilogue != QVIT_EPI_I8 && epilogue != QVIT_EPI_I8_GELU) return QVIT_EINVAL;
  if (nb < 1 || nb > QVIT_EPI_TABLE_MAX_NB || !(w > 0.f) || !std::isfinite(v_lo) || !std::isfinite(v_lo + w * nb))
    return QVIT_EINVAL;
  const int q = out_qtype & 0xff;
  if (q != QVIT_QT_LINEAR && q != QVIT_QT_NONLINEAR && q != QVIT_QT_ULTRA_ACT) return QVIT_EINVAL;
  if (q == QVIT_QT_ULTRA_ACT ? (out_levels < 1 || out_levels > 127) : (!out_d || !out_qm)) return QVIT_EINVAL;
  if (((uintptr_t)table) & 15) return QVIT_EALIGN;
  const int one = 1;
  hipError_t e = hipMemcpyAsync(reinterpret_cast<int8_t*>(table) + offsetof(EpiTableHdr, valid), &one, sizeof(int),
                                hipMemcpyHostToDevice, stream);
  if (e != hipSuccess) return qvit_hip_status(e);
  hipLaunchKernelGGL(epi_table_kernel, dim3((unsigned)((nb + 63) / 64)), dim3(64), 0, stream,
                     epilogue == QVIT_EPI_I8_GELU ? 1 : 0, out_qtype, out_d, out_qm, out_t, out_levels,
                     -(v_lo * (1.0f / w)), 1.0f / w, (int)nb, reinterpret_cast<int8_t*>(table));
  return qvit_hip_status(hipGetLastError());
}

extern "C" int qvit_pack_weight_w4r(const void* packed, int64_t npad, int64_t kpad, void* out, hipStream_t stream) {
  if (!packed || !out) return QVIT_ENULL;
  if (npad <= 0 || npad % BN || kpad <= 0 || kpad % KTILE || npad > INT32_MAX / 2 || kpad > 65536) return QVIT_EINVAL;
  if ((((uintptr_t)packed) & 15) || (((uintptr_t)out) & 15)) return QVIT_EALIGN;
  if (packed == out) return QVIT_EINVAL;  // not in place
  const int64_t units = npad * kpad / 16;  // 8-B slices (npad kpad / 2 bytes)
  hipLaunchKernelGGL(pack_w4r_kernel, dim3((unsigned)((units + 255) / 256)), dim3(256), 0, stream,
                     reinterpret_cast<const int8_t*>(packed), reinterpret_cast<int8_t*>(out), units);
  return qvit_hip_status(hipGetLastError());
}

extern "C" int qvit_pack_weight_w8r(const void* packed, int64_t npad, int64_t kpad, void* out, hipStream_t stream) {
  if (!packed || !out) return QVIT_ENULL;
  if (npad <= 0 || npad % BN || kpad <= 0 || kpad % KTILE || npad > INT32_MAX / 2 || kpad > 65536) return QVIT_EINVAL;
  if ((((uintptr_t)packed) & 15) || (((uintptr_t)out) & 15)) return QVIT_EALIGN;
  if (packed == out) return QVIT_EINVAL;  // not in place
  const int64_t units = npad * kpad / 16;  // 8-B source slices -> 16-B operands (npad kpad bytes out)
  hipLaunchKernelGGL(pack_w8r_kernel, dim3((unsigned)((units + 255) / 256)), dim3(256), 0, stream,
                     reinterpret_cast<const int8_t*>(packed), reinterpret_cast<int8_t*>(out), units);
  return qvit_hip_status(hipGetLastError());
}

extern "C" int qvit_gemm(const int8_t* A, int64_t M, int64_t K, int64_t lda, const void* Wp, int wfmt, int64_t N,
                         int64_t npad, const float* d_act, const float* d_wt, const float* bias, int epilogue,
                         void* C, int64_t ldc, int out_qtype, const float* out_d, const float* out_qm,
                         const float* out_t, int out_levels, const void* epi_table, hipStream_t stream) {
  if (!A || !Wp || !C) return QVIT_ENULL;
  if (wfmt != QVIT_W4 && wfmt != QVIT_W4R && wfmt != QVIT_W8R && wfmt != QVIT_W8) return QVIT_EINVAL;
  if (M < 0 || K <= 0 || K % KTILE || lda < K || N <= 0 || npad < N || npad % BN) return QVIT_EINVAL;
  if (M > INT32_MAX / 2 || npad > INT32_MAX / 2 || K > (1 << 24)) return QVIT_EINVAL;
  if (wfmt != QVIT_W8 && K > 65536) return QVIT_EINVAL;  // 16x-scaled int32 accumulation bound
  if ((lda % 16) || (((uintptr_t)A) & 15) || (((uintptr_t)Wp) & 15)) return QVIT_EALIGN;
  if (epilogue < QVIT_EPI_F32 || epilogue > QVIT_EPI_I32) return QVIT_EINVAL;
  const bool i8out = epilogue == QVIT_EPI_I8 || epilogue == QVIT_EPI_I8_GELU;
  if (ldc < N) return QVIT_EINVAL;
  if (i8out) {
    if ((ldc % 4) || (((uintptr_t)C) & 3)) return QVIT_EALIGN;
    const int q = out_qtype & 0xff;
    if (q != QVIT_QT_LINEAR && q != QVIT_QT_NONLINEAR && q != QVIT_QT_ULTRA_ACT) return QVIT_EINVAL;
    if (q == QVIT_QT_ULTRA_ACT ? (out_levels < 1 || out_levels > 127) : (!out_d || !out_qm)) return QVIT_EINVAL;
  } else {
    if ((ldc % 4) || (((uintptr_t)C) & 15)) return QVIT_EALIGN;
  }
  if (epilogue != QVIT_EPI_I32 && (!d_act || !d_wt)) return QVIT_ENULL;
  if (bias && (((uintptr_t)bias) & 15)) return QVIT_EALIGN;
  if (M == 0) return QVIT_OK;
  if (epi_table && (((uintptr_t)epi_table) & 15)) return QVIT_EALIGN;
  EpiArgs ep{d_act, d_wt, bias, out_qtype, out_d, out_qm, out_t, out_levels,
             (i8out ? reinterpret_cast<const int8_t*>(epi_table) : nullptr), 1, 1.f, 1.f, nullptr};
  if (wfmt == QVIT_W4) return dispatch_epi<QVIT_W4>(epilogue, A, M, K, lda, Wp, N, npad, C, ldc, ep, stream);
  if (wfmt == QVIT_W4R) return dispatch_epi<QVIT_W4, 1>(epilogue, A, M, K, lda, Wp, N, npad, C, ldc, ep, stream);
  if (wfmt == QVIT_W8R) return dispatch_epi<QVIT_W4, 2>(epilogue, A, M, K, lda, Wp, N, npad, C, ldc, ep, stream);
  return dispatch_epi<QVIT_W8>(epilogue, A, M, K, lda, Wp, N, npad, C, ldc, ep, stream);
}

extern "C" int qvit_gemm_resid_ln(const int8_t* A, int64_t M, int64_t K, int64_t lda, const void* Wp, int wfmt,
                                  int64_t N, int64_t npad, const float* d_act, const float* d_wt, const float* bias,
                                  float* C, int64_t ldc, const float* gamma, const float* beta, float eps,
                                  int out_qtype, const float* out_d, const float* out_qm, const float* out_t,
                                  int out_levels, const void* ln_table, int8_t* codes, int64_t ldcodes,
                                  int64_t kpad_codes, int32_t* counters, hipStream_t stream) {
  if (!A || !Wp || !C || !codes || !counters || !d_act || !d_wt) return QVIT_ENULL;
  if (wfmt != QVIT_W4 && wfmt != QVIT_W8) return QVIT_EINVAL;
  if (M < 0 || K <= 0 || K % KTILE || lda < K || N <= 0 || N > 1024 || N % 4 || npad < N || npad % BN)
    return QVIT_EINVAL;
  if (M > INT32_MAX / 2 || K > (1 << 24) || (wfmt == QVIT_W4 && K > 65536)) return QVIT_EINVAL;
  if (ldc < N || kpad_codes < N || ldcodes < kpad_codes || M * ldc * 4 > 0x7FFFFFFF) return QVIT_EINVAL;
  if ((lda % 16) || (((uintptr_t)A) & 15) || (((uintptr_t)Wp) & 15)) return QVIT_EALIGN;
  if ((ldc % 4) || (((uintptr_t)C) & 15) || (ldcodes % 4) || (((uintptr_t)codes) & 3)) return QVIT_EALIGN;
  if ((((uintptr_t)counters) & 3) || (bias && (((uintptr_t)bias) & 15))) return QVIT_EALIGN;
  if ((gamma && (((uintptr_t)gamma) & 15)) || (beta && (((uintptr_t)beta) & 15))) return QVIT_EALIGN;
  if (ln_table && (((uintptr_t)ln_table) & 15)) return QVIT_EALIGN;
  const int q = out_qtype & 0xff;
  if (q != QVIT_QT_LINEAR && q != QVIT_QT_NONLINEAR && q != QVIT_QT_ULTRA_ACT) return QVIT_EINVAL;
  if (q == QVIT_QT_ULTRA_ACT ? (out_levels < 1 || out_levels > 127) : (!out_d || !out_qm)) return QVIT_EINVAL;
  if (M == 0) return QVIT_OK;
  // fresh arrival counters for this launch (the hand-off never depends on earlier launches)
  const hipError_t ez = hipMemsetAsync(counters, 0, (size_t)((M + 127) / 128) * sizeof(int32_t), stream);
  if (ez != hipSuccess) return qvit_hip_status(ez);
  EpiArgs ep{d_act, d_wt, bias, out_qtype, out_d, out_qm, out_t, out_levels, nullptr, 1, 1.f, 1.f, nullptr,
             gamma, beta, eps, reinterpret_cast<const int8_t*>(ln_table), codes, ldcodes, (int)kpad_codes,
             reinterpret_cast<int*>(counters)};
  if (wfmt == QVIT_W4) return launch<QVIT_W4, EPI_RESID_LN>(A, M, K, lda, Wp, N, npad, C, ldc, ep, stream);
  return launch<QVIT_W8, EPI_RESID_LN>(A, M, K, lda, Wp, N, npad, C, ldc, ep, stream);
}

QVIT_GEMM_STAMP_READER  // diag_stamps.h: exists only in -DQVIT_GEMM_STAMPS builds

extern "C" int qvit_gemm_qkv_split(const int8_t* A, int64_t M, int64_t K, int64_t lda, const void* Wp, int wfmt,
                                   int64_t N, int64_t npad, const float* d_act, const float* d_wt, const float* bias,
                                   int64_t seq, float in_scale, void* qkv_hi, void* qkv_lo, hipStream_t stream) {
  if (!A || !Wp || !qkv_hi || !qkv_lo || !d_act || !d_wt) return QVIT_ENULL;
  if (wfmt != QVIT_W4 && wfmt != QVIT_W4R && wfmt != QVIT_W8R && wfmt != QVIT_W8) return QVIT_EINVAL;
  if (M < 0 || K <= 0 || K % KTILE || lda < K || N <= 0 || N % 64 || npad < N || npad % BN) return QVIT_EINVAL;
  if (M > INT32_MAX / 2 || npad > INT32_MAX / 2 || K > (1 << 24)) return QVIT_EINVAL;
  if (seq <= 0 || seq > (1 << 20) || M % seq || !(in_scale > 0.f)) return QVIT_EINVAL;
  if (wfmt != QVIT_W8 && K > 65536) return QVIT_EINVAL;
  if ((lda % 16) || (((uintptr_t)A) & 15) || (((uintptr_t)Wp) & 15)) return QVIT_EALIGN;
  if ((((uintptr_t)qkv_hi) & 15) || (((uintptr_t)qkv_lo) & 15)) return QVIT_EALIGN;
  if (bias && (((uintptr_t)bias) & 15)) return QVIT_EALIGN;
  if (M == 0) return QVIT_OK;
  EpiArgs ep{d_act, d_wt, bias, 0, nullptr, nullptr, nullptr, 0, nullptr, (int)seq, 1.0f / (float)seq, in_scale,
             reinterpret_cast<_Float16*>(qkv_lo)};
  if (wfmt == QVIT_W4)
    return launch<QVIT_W4, QVIT_EPI_QKV_SPLIT>(A, M, K, lda, Wp, N, npad, qkv_hi, N, ep, stream);
  if (wfmt == QVIT_W4R)
    return launch<QVIT_W4, QVIT_EPI_QKV_SPLIT, 1>(A, M, K, lda, Wp, N, npad, qkv_hi, N, ep, stream);
  if (wfmt == QVIT_W8R)
    return launch<QVIT_W4, QVIT_EPI_QKV_SPLIT, 2>(A, M, K, lda, Wp, N, npad, qkv_hi, N, ep, stream);
  return launch<QVIT_W8, QVIT_EPI_QKV_SPLIT>(A, M, K, lda, Wp, N, npad, qkv_hi, N, ep, stream);
}
