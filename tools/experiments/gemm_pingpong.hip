// Experiment (round 4, not built into the library): the ping-pong schedule for the int8-code GEMM epilogues
// (fc1), as it ran inside quantized_vit_amd/csrc/gemm_w4a8.hip (it uses that file's Geo, Frags, EpiArgs, epilogue
// helpers and launcher; to rebuild it, paste it back above device_cus() and route the I8 / I8_GELU launches of
// launch() to it). Bit-identical to gemm_kernel (tests/test_gpu_gemm_pp.py at the time), and slower: fc1
// 182-219 us in the model vs 124-131 us, 205-234 us vs 145-169 us in tools/gemm_bench.py
// (profiles/r04_gemm_pingpong_ab.txt).
// ---- ping-pong schedule for the int8 code epilogues (fc1: QVIT_EPI_I8_GELU) ----------------------------
// One 512-thread workgroup per CU, two halves of 4 waves (waves 0-3, 4-7) that share the CU's 4 SIMDs: one wave
// of each half per SIMD. Each wave of a half owns the same 64 weight rows x 128 activation rows of a tile as a
// wave of gemm_kernel. The workgroup's tiles are computed alternately, tile j by half j & 1, in intervals of one
// 64-deep k-stage separated by workgroup barriers. In interval i (stage i of the workgroup's stage stream, nk
// stages per tile):
//   the computing half  issues the LDS-DMA of its own weight rows of stage i + PP_LEAD, runs stage i's MFMAs and
//                       streams stage i + 1's fragments into the registers they free;
//   the other half      issues the activation rows of stage i + PP_LEAD (and, with a tile's stage 0, the tile's
//                       bias) and runs one 16-row chunk of its previous tile's epilogue (chunks 0..7 in the
//                       period's first 8 intervals);
//   at the barrier      every wave has retired its LDS reads and its VMEM ops older than the previous interval,
//                       so stages <= i + 2 are in LDS when interval i + 1 starts.
// So each SIMD pairs one matrix wave with one memory / VALU wave throughout (MI355X_MICROARCH.md, two waves per
// SIMD), where gemm_kernel's two independent co-resident blocks drift into lockstep and contend for the matrix pipe
// and the DMA issue together. Ring: PP_LEAD slots, stage i + PP_LEAD takes stage i's slot, whose fragments were
// read in interval i - 1. The last tile's epilogue runs after the stream, without barriers.
// Requirements (checked by the launcher): nk = K / 64 >= PP_CHUNKS + PP_LEAD (a tile's bias DMA, issued with its
// stage 0 PP_LEAD intervals ahead, must follow the last chunk that reads the slot of the tile two before), N % 16
// == 0, ldc % 16 == 0, C 16-B aligned, M * ldc < 2^31 (the code rows are written by buffer stores; rows >= M and
// columns >= N go to an out-of-range offset and are dropped, so every chunk issues exactly one store per lane and
// the VMEM counts stay static).
constexpr int PP_NT = 512;
constexpr int PP_CHUNKS = 8;  // epilogue chunks per tile (16 activation rows each)
#ifndef QVIT_PP_LEAD
#define QVIT_PP_LEAD 4
#endif
#ifndef QVIT_PP_SPLIT
#define QVIT_PP_SPLIT 0
#endif
// interval i issues stage i + PP_LEAD; the ring holds PP_LEAD stages (W8 stages are 24 KiB: at most 4 fit)
template <int WFMT>
constexpr int pp_lead() { return (WFMT == QVIT_W8 && QVIT_PP_LEAD > 4) ? 4 : QVIT_PP_LEAD; }

template <int WFMT, int EPI>
__global__ __launch_bounds__(PP_NT, 1) void gemm_pp_kernel(const int8_t* __restrict__ A, int M, int K, int64_t lda,
                                                           const int8_t* __restrict__ Wp, int N, int npad,
                                                           void* __restrict__ C, int64_t ldc, EpiArgs ep) {
  using G = Geo<WFMT, 1>;
  constexpr int BM = G::BM;  // 128
  constexpr int XBYTES = G::XBYTES;
  static_assert(EPI == QVIT_EPI_I8 || EPI == QVIT_EPI_I8_GELU, "int8 code epilogues only");
  constexpr int PP_LEAD = pp_lead<WFMT>();
  constexpr int PP_RING = PP_LEAD;
  constexpr int RING_BYTES = PP_RING * G::STAGE;
  constexpr int BIAS_OFF = RING_BYTES + G::EPI_BYTES;  // two 1-KiB bias slots (tile j: slot j & 1)
  constexpr int QP_OFF = BIAS_OFF + 2 * G::BIAS_BYTES;
  __shared__ __attribute__((aligned(16))) int8_t smem[QP_OFF + G::QP_BYTES];
  int8_t* epi_lds = smem + RING_BYTES;
  QParams* qp_l = reinterpret_cast<QParams*>(smem + QP_OFF);
  const bool has_bias = ep.bias != nullptr;

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int half = wave >> 2;
  const int wq = wave & 3;  // weight rows [64 wq, 64 wq + 64) of the tile

  // ---- the workgroup's tiles: XCD-contiguous ranges as in gemm_kernel, tile j = lo + slot + j * team ----------
  const int nb_n = npad / BN;
  const int ntiles = nb_n * ((M + BM - 1) / BM);
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, team = gridDim.x >> 3;
  const int per = ntiles >> 3, rem = ntiles & 7;
  const int lo = xcd * per + (xcd < rem ? xcd : rem);
  const int hi = lo + per + (xcd < rem ? 1 : 0);
  if (lo + slot >= hi) return;  // workgroup-uniform
  const int ntl = (hi - lo - slot + team - 1) / team;
  const int nk = K / BK;
  const int nstages = ntl * nk;

  const float alpha = (*ep.d_act) * (*ep.d_wt) * (WFMT == QVIT_W4 ? 0.0625f : 1.f);
  bool use_table = false;
  float t_c0 = 0.f, t_invw = 0.f, t_top = 0.f;
  if (ep.table != nullptr) {
    const EpiTableHdr h = *reinterpret_cast<const EpiTableHdr*>(ep.table);
    use_table = h.valid != 0 && h.nb <= G::TABLE_MAX_NB;
    t_c0 = h.c0;
    t_invw = h.inv_w;
    t_top = epi_top(h.nb);
    if (use_table) {
      const v4i* src = reinterpret_cast<const v4i*>(ep.table);
      for (int i = tid; i < (16 + 8 * h.nb + 15) / 16; i += PP_NT) reinterpret_cast<v4i*>(epi_lds)[i] = src[i];
    }
  }
  if (!use_table && tid == 0) *qp_l = load_qparams(ep.out_qtype, ep.out_d, ep.out_qm, ep.out_t, ep.out_levels);
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the compiler's own loads are done before the counted stream

  // ---- LDS-DMA of stream stage (tile index j, stage kt) by wave wq of the issuing half ----------------------
  constexpr int WROWS_PER_PIECE = 1024 / G::WROW;
  constexpr int WROWS_PER_WAVE = BN / 4;
  const uint32_t lds0 = lds_addr(smem);
  auto tile_of = [&](int j) { return lo + slot + j * team; };
  // parts: 1 = the activation pieces (+ the tile's bias with its stage 0), 2 = this wave's weight rows
  auto issue = [&](int j, int kt, int rslot, int parts) __attribute__((always_inline)) {
    const int tt = tile_of(j);
    const int m0 = (tt / nb_n) * BM;
    const uint32_t wbase = (uint32_t)(tt % nb_n) * (uint32_t)(nk * G::WBYTES);
    const uint32_t sx = lds0 + (uint32_t)(rslot * G::STAGE);
    const uint32_t sw = sx + XBYTES;
    const uint32_t kx = (uint32_t)kt * BK;
    const int ln = lane_opaque();
    if (parts & 1) {
#pragma unroll
      for (int p = 0; p < 2; ++p) {  // activations: rows 32 wq + 16 p .. + 15, swizzled on the source
        const int row = 32 * wq + 16 * p + (ln >> 2);
        int gm = m0 + row;
        gm = gm < M ? gm : M - 1;
        const uint32_t lg = (uint32_t)(((ln & 3) ^ (((row >> 2) & 1) << 1)) * 16);
        dma16s(A, (uint32_t)gm * (uint32_t)lda + lg + kx, __builtin_amdgcn_readfirstlane(sx + (32 * wq + 16 * p) * BK));
      }
      if (kt == 0 && wq == 0 && has_bias)  // the tile's bias (npad floats, qvit_pad_bias) into slot j & 1
        dma16(ep.bias + (tt % nb_n) * BN + ln * 4, __builtin_amdgcn_readfirstlane(lds0 + BIAS_OFF + (j & 1) * G::BIAS_BYTES));
    }
    if (parts & 2) {
      const uint32_t wt = wbase + (uint32_t)kt * G::WBYTES + (uint32_t)(wq * (G::WPIECES * 1024) + ln * 16);
#pragma unroll
      for (int p = 0; p < G::WPIECES; ++p)
        dma16s(Wp, wt + p * 1024, __builtin_amdgcn_readfirstlane(sw + (WROWS_PER_WAVE * wq + WROWS_PER_PIECE * p) * G::WROW));
    }
  };
  // VMEM ops one issue() puts in flight for this wave (wave-uniform)
  auto issued = [&](int kt, int parts) {
    return ((parts & 1) ? 2 + ((kt == 0 && wq == 0 && has_bias) ? 1 : 0) : 0) + ((parts & 2) ? G::WPIECES : 0);
  };

  // fragments of the stage being computed: x[s] (activation rows 16 s .. + 15), wp[r] (weight rows 16 r .. + 15,
  // packed); a stage's MFMAs stream the next stage's fragments into the same registers as they free them
  typedef typename std::conditional<WFMT == QVIT_W4, uint2, v4i>::type WFrag;
  v4i xf[8];
  WFrag wp[4];
  auto frag_off = [&](int& xoff, int& woff) __attribute__((always_inline)) {
    const int ln = lane_opaque();
    const int lfr = ln & 15, lfq = ln >> 4;
    xoff = lfr * BK + ((lfq ^ (((lfr >> 2) & 1) << 1)) << 4);
    woff = (WFMT == QVIT_W4) ? (64 * wq + lfr) * G::WROW + ((lfq ^ (((lfr >> 3) & 1) << 1)) << 3)
                             : (64 * wq + lfr) * G::WROW + ((lfq ^ (((lfr >> 2) & 1) << 1)) << 4);
  };
  auto read_all = [&](int rslot) __attribute__((always_inline)) {
    int xoff, woff;
    frag_off(xoff, woff);
    const int8_t* sx = smem + rslot * G::STAGE;
    const int8_t* sw = sx + XBYTES;
#pragma unroll
    for (int r = 0; r < 4; ++r) wp[r] = *reinterpret_cast<const WFrag*>(sw + woff + r * 16 * G::WROW);
#pragma unroll
    for (int q = 0; q < 8; ++q) xf[q] = *reinterpret_cast<const v4i*>(sx + xoff + q * 16 * BK);
  };
  v4i acc[4][8];
  auto zero_acc = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int s = 0; s < 8; ++s) acc[r][s] = v4i{0, 0, 0, 0};
  };
  // MFMAs of the stage in registers; the fragments of ring slot nslot replace them as they are consumed (an
  // activation fragment after its 4 MFMAs, the weights up front into 8 / 16 spare registers)
  auto stage_stream = [&](int nslot) __attribute__((always_inline)) {
    int xoff, woff;
    frag_off(xoff, woff);
    const int8_t* sx = smem + nslot * G::STAGE;
    const int8_t* sw = sx + XBYTES;
    WFrag wn[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) wn[r] = *reinterpret_cast<const WFrag*>(sw + woff + r * 16 * G::WROW);
    v4i wf[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if constexpr (WFMT == QVIT_W4) {
        const uint2 pw = wp[r];
        wf[r] = v4i{(int)nib16_lo(pw.x), (int)nib16_hi(pw.x), (int)nib16_lo(pw.y), (int)nib16_hi(pw.y)};
      } else {
        wf[r] = wp[r];
      }
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[r][q] = __builtin_amdgcn_mfma_i32_16x16x64_i8(wf[r], xf[q], acc[r][q], 0, 0, 0);
      xf[q] = *reinterpret_cast<const v4i*>(sx + xoff + q * 16 * BK);
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) wp[r] = wn[r];
  };

  // end of an interval: LDS reads retired, VMEM ops of earlier intervals retired (N = this interval's), barrier
  auto sync_n = [&](int n) __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(0xC07F);
#define QVIT_PP_WAIT(k) \
  case k: asm volatile("s_waitcnt vmcnt(" #k ")\n\ts_barrier" ::: "memory"); break;
    switch (n) {
      QVIT_PP_WAIT(0) QVIT_PP_WAIT(1) QVIT_PP_WAIT(2) QVIT_PP_WAIT(3) QVIT_PP_WAIT(4) QVIT_PP_WAIT(5)
      QVIT_PP_WAIT(6) QVIT_PP_WAIT(7) QVIT_PP_WAIT(8) QVIT_PP_WAIT(9) QVIT_PP_WAIT(10) QVIT_PP_WAIT(11)
      QVIT_PP_WAIT(12) QVIT_PP_WAIT(13) QVIT_PP_WAIT(14)
      default: asm volatile("s_waitcnt vmcnt(15)\n\ts_barrier" ::: "memory"); break;
    }
#undef QVIT_PP_WAIT
    __builtin_amdgcn_sched_barrier(0);
  };
  // VMEM ops this wave issued in each of the previous PP_LEAD - 3 intervals: their stages are read later than the
  // next interval, so they may stay in flight across this interval's barrier; everything older is retired at it
  constexpr int NH = PP_LEAD > 3 ? PP_LEAD - 3 : 1;
  int hist[NH];
#pragma unroll
  for (int k = 0; k < NH; ++k) hist[k] = 0;
  auto sync_iv = [&](int n) __attribute__((always_inline)) {
    int out = n;
    if constexpr (PP_LEAD > 3) {
#pragma unroll
      for (int k = 0; k < NH; ++k) out += hist[k];
#pragma unroll
      for (int k = 0; k + 1 < NH; ++k) hist[k] = hist[k + 1];
      hist[NH - 1] = n;
    }
    sync_n(out);
  };

  // ---- one epilogue chunk: rows 16 sr .. 16 sr + 15 of tile j (this half's last computed tile) -------------
  // lane (fr, fq) owns the 16 consecutive columns [n0 + 64 wq + 16 fq, + 16) of row m0 + 16 sr + fr (the weight
  // rows are pre-permuted so acc[r][sr][j] is column 16 fq + 4 r + j of them): one 16-B buffer store per lane
  const __amdgpu_buffer_rsrc_t crs =
      __builtin_amdgcn_make_buffer_rsrc(C, (short)0, (int)((int64_t)M * ldc), 0x00020000);
  auto chunk = [&](auto src, int j) __attribute__((always_inline)) {
    constexpr int sr = decltype(src)::value;
    const int el = lane_opaque();  // (re-derived per chunk: no lane-dependent address stays live across intervals)
    const int efr = el & 15, efq = el >> 4;
    const int tt = tile_of(j);
    const int m = (tt / nb_n) * BM + 16 * sr + efr;
    const int nbase = (tt % nb_n) * BN + 64 * wq + 16 * efq;
    uint32_t wd[4];
    const int8_t* tlb = epi_lds + sizeof(EpiTableHdr);
    if (use_table) {
      // the 16 columns' bias from the tile's LDS slot, per chunk (nothing of the epilogue stays live across the
      // intervals, where the register budget belongs to the matrix half's fragments)
      float bcol[16];
      const float* bl = reinterpret_cast<const float*>(smem + BIAS_OFF + (j & 1) * G::BIAS_BYTES) + 64 * wq + 16 * efq;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float4 b = make_float4(0.f, 0.f, 0.f, 0.f);
        if (has_bias) b = *reinterpret_cast<const float4*>(bl + 4 * r);
        bcol[4 * r] = b.x; bcol[4 * r + 1] = b.y; bcol[4 * r + 2] = b.z; bcol[4 * r + 3] = b.w;
      }
      float v[4][4];
      uint2 e[4][4];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          v[r][q] = fmaf(alpha, (float)acc[r][sr][q], bcol[4 * r + q]);
          e[r][q] = *epi_entry(tlb, v[r][q], t_c0, t_invw, t_top);
        }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        epi_select_byte<0>(wd[r], v[r][0], __uint_as_float(e[r][0].x), e[r][0].y);
        epi_select_byte<1>(wd[r], v[r][1], __uint_as_float(e[r][1].x), e[r][1].y);
        epi_select_byte<2>(wd[r], v[r][2], __uint_as_float(e[r][2].x), e[r][2].y);
        epi_select_byte<3>(wd[r], v[r][3], __uint_as_float(e[r][3].x), e[r][3].y);
      }
    } else {
      // no valid table: the direct (GELU +) quantizer, a rolled loop over the lane's 16 values staged through the
      // (then unused) table region, 4352 B per wave of the half
      int* stg = reinterpret_cast<int*>(epi_lds + wq * EPI_WAVE_BYTES) + efr * EPI_LD + 16 * efq;
      const float* bl = reinterpret_cast<const float*>(smem + BIAS_OFF + (j & 1) * G::BIAS_BYTES) + 64 * wq + 16 * efq;
#pragma unroll
      for (int r = 0; r < 4; ++r) *reinterpret_cast<v4i*>(stg + 4 * r) = acc[r][sr];
      const QParams qp = *qp_l;
      uint32_t word = 0;
#pragma unroll 1
      for (int q = 0; q < 16; ++q) {
        float x = fmaf(alpha, (float)stg[q], has_bias ? bl[q] : 0.f);
        if (EPI == QVIT_EPI_I8_GELU) x = gelu_ref(x);
        word |= ((uint32_t)(uint8_t)to_i8_sat(quant_code(x, qp))) << (8 * (q & 3));
        if ((q & 3) == 3) {
          stg[q >> 2] = (int)word;  // the 4 codes of stg[q - 3 .. q], read above
          word = 0;
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) wd[r] = (uint32_t)stg[r];
    }
    const int off = (m < M && nbase < N) ? (int)((int64_t)m * ldc + nbase) : (int)0x80000000;
    typedef int i4v __attribute__((ext_vector_type(4)));
    __builtin_amdgcn_raw_buffer_store_b128(i4v{(int)wd[0], (int)wd[1], (int)wd[2], (int)wd[3]}, crs, off, 0, 0);
  };

  // ---- prologue: half 1 (the loading half of interval 0) issues stages 0, 1, 2; stages 0, 1 landed ----------
  if (half == 1) {
#pragma unroll
    for (int k = 0; k < PP_LEAD; ++k) issue(0, k, k, 3);
    sync_n((PP_LEAD - 2) * issued(2, 3));  // stages 0, 1 landed
    // stages 3 .. PP_LEAD - 1 count as issued in intervals 3 - PP_LEAD .. -1 (stage s is retired by the end of
    // interval s - 2)
    if constexpr (PP_LEAD > 3) {
#pragma unroll
      for (int k = 0; k < NH; ++k) hist[k] = issued(3 + k, 3);
    }
  } else {
    sync_n(0);
    zero_acc();
    read_all(0);
  }

  // the issue cursor: stage i + PP_LEAD of interval i, as (tile index, stage, ring slot)
  int ij = 0, ikt = PP_LEAD, islot = 0;  // tile 0 (nk >= 12), slot PP_LEAD % PP_RING
  auto issue_next = [&](int i, int parts) __attribute__((always_inline)) {  // -> VMEM ops issued
    int n = 0;
    if (i + PP_LEAD < nstages) {
      issue(ij, ikt, islot, parts);
      n = issued(ikt, parts);
    }
    return n;
  };
  auto advance = [&]() __attribute__((always_inline)) {
    if (++ikt == nk) { ikt = 0; ++ij; }
    islot = islot == PP_RING - 1 ? 0 : islot + 1;
  };

  // compute period p: tile p, stages i0 .. i0 + nk - 1 (stage i0's fragments in registers at the start); the last
  // interval also streams in a slot past the tile, whose bytes are never used
  auto compute_period = [&](int p) __attribute__((always_inline)) {
    int rs = (p * nk + 1) % PP_RING;
    for (int kt = 0; kt < nk; ++kt) {
      __builtin_amdgcn_sched_barrier(0);
      const int n = issue_next(p * nk + kt, QVIT_PP_SPLIT ? 2 : 0);  // (SPLIT: its weight rows of stage i + PP_LEAD)
      advance();
      __builtin_amdgcn_sched_barrier(0);
      stage_stream(rs);
      rs = rs == PP_RING - 1 ? 0 : rs + 1;
      sync_iv(n);
    }
  };
  // load period p: the other half computes tile p; this half issues stages p nk + 3 .. and (EPION) writes tile
  // p - 1 in chunks; its last interval reads this half's next tile's stage-0 fragments (unconditionally, so that
  // they are dead through the period; past the last tile the slot's bytes are never used)
  auto load_period = [&](auto epion, int p) __attribute__((always_inline)) {
    constexpr bool EPION = decltype(epion)::value;
    const int i0 = p * nk;
    auto interval = [&](auto src, int kt) __attribute__((always_inline)) {
      constexpr int sr = decltype(src)::value;  // chunk index, or -1
      const int n = issue_next(i0 + kt, QVIT_PP_SPLIT ? 1 : 3);
      advance();
      if constexpr (EPION && sr >= 0) {
        chunk(std::integral_constant<int, sr>{}, p - 1);
        sync_iv(n + 1);
      } else {
        sync_iv(n);
      }
    };
    interval(std::integral_constant<int, 0>{}, 0);
    interval(std::integral_constant<int, 1>{}, 1);
    interval(std::integral_constant<int, 2>{}, 2);
    interval(std::integral_constant<int, 3>{}, 3);
    interval(std::integral_constant<int, 4>{}, 4);
    interval(std::integral_constant<int, 5>{}, 5);
    interval(std::integral_constant<int, 6>{}, 6);
    interval(std::integral_constant<int, 7>{}, 7);
    zero_acc();  // tile p - 1 is written; the accumulators start this half's next tile
    for (int kt = PP_CHUNKS; kt < nk - 1; ++kt) interval(std::integral_constant<int, -1>{}, kt);
    const int n = issue_next(i0 + nk - 1, QVIT_PP_SPLIT ? 1 : 3);
    advance();
    read_all((i0 + nk) % PP_RING);
    sync_iv(n);
  };
  // each half's period sequence as straight-line code (compute, load, compute, ...; half 1 starts with a load
  // period without epilogue), so the accumulators flow compute -> epilogue -> zero -> compute with no
  // control-flow merge of differently allocated copies
  auto run = [&](auto hc) __attribute__((always_inline)) {
    constexpr int H = decltype(hc)::value;
    int p = 0;
    if constexpr (H == 1) {
      load_period(std::false_type{}, 0);
      p = 1;
      if (p >= ntl) return;
    }
    for (;;) {
      compute_period(p);
      if (p + 1 >= ntl) {  // this half computed the last tile: its epilogue, after the stream (no barriers)
        chunk(std::integral_constant<int, 0>{}, p);
        chunk(std::integral_constant<int, 1>{}, p);
        chunk(std::integral_constant<int, 2>{}, p);
        chunk(std::integral_constant<int, 3>{}, p);
        chunk(std::integral_constant<int, 4>{}, p);
        chunk(std::integral_constant<int, 5>{}, p);
        chunk(std::integral_constant<int, 6>{}, p);
        chunk(std::integral_constant<int, 7>{}, p);
        return;
      }
      load_period(std::true_type{}, p + 1);
      p += 2;
      if (p >= ntl) return;
    }
  };
  if (half == 0) run(std::integral_constant<int, 0>{});
  else run(std::integral_constant<int, 1>{});
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

