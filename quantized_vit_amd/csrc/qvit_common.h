// Device-side helpers shared by every kernel of libqvit_hip.so (gfx950 only).
//
// The quantizer here is the integer restatement of the reference's fake quantizers:
//   SymQuantizerLinear.forward    OTO/quantization/quant_layers.py:137-161
//   SymQuantizerNonLinear.forward OTO/quantization/quant_layers.py:41-69
//   activation_quantize_fn        4-bit quantization/quant_ultra.py:59-73
// The reference returns v = sgn(x) * (d * rne(p(|x|) / d)) with p(a) = a (linear) or
// exp(t*log(a)) (nonlinear), zero where |x| <= 0 and d*rne(p_sat/d) where |x| >= q_m. We return
// the integer k with v = d * k, so a contraction of two quantized tensors is d_a*d_w*sum(k_a*k_w).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/qvit_hip.h"

#define QVIT_DEV __device__ __forceinline__

// Test-only flag OR-ed into qtype: disables the guarded fast path, so every element goes through
// the careful (IEEE division + ocml exp/log) sequence. Results must be identical either way.
#define QVIT_QT_FORCE_CAREFUL 0x100

// fp32 log / exp rounded from double precision: the correctly rounded fp32 result except for
// double-rounding ties (~2^-29). torch's CPU kernels (Sleef u10) return the correctly rounded
// value for all but ~0.1% (log) / ~0.3% (exp) of inputs, so this matches the reference far more
// often than the fp32 ocml sequence (v_log_f32/v_exp_f32 based, a few ulp).
QVIT_DEV float log_cr(float a) { return (float)log((double)a); }
QVIT_DEV float exp_cr(float a) { return (float)exp((double)a); }


struct QParams {
  int qtype;      // QVIT_QT_*
  int careful;    // 1 -> always take the careful path
  float d;        // d_quant
  float inv_d;    // 1/d (fast path only)
  float qm;       // q_m (signed: the reference compares |x| >= q_m)
  float t;        // t_quant (nonlinear)
  float L;        // saturation code rne(p_sat / d)
  float levels;   // ULTRA_ACT: 2^b - 1
};

// Loads the per-tensor scalars from device memory and derives the saturation level exactly as
// the reference: range_pow = |q_m - q_s| (linear, :154) or exp(t*log(|q_m - q_s| + 1e-6)) (:62).
QVIT_DEV QParams load_qparams(int qtype, const float* d, const float* qm, const float* t, int levels) {
  QParams p;
  p.careful = (qtype & QVIT_QT_FORCE_CAREFUL) ? 1 : 0;
  p.qtype = qtype & 0xff;
  p.levels = (float)levels;
  p.d = 1.f; p.inv_d = 1.f; p.qm = 0.f; p.t = 1.f; p.L = 0.f;
  if (p.qtype == QVIT_QT_ULTRA_ACT) return p;
  p.d = *d;
  p.qm = *qm;
  p.t = (t != nullptr) ? *t : 1.f;
  p.inv_d = 1.f / p.d;
  if (p.qtype == QVIT_QT_LINEAR) {
    p.L = rintf(fabsf(p.qm) / p.d);
  } else {
    p.L = rintf(exp_cr(p.t * log_cr(fabsf(p.qm) + 1e-6f)) / p.d);
  }
  return p;
}

// Careful magnitude code for 0 < a < q_m: the reference's op sequence
//   exp(t * log(a)) (fp32 values at every step), IEEE fp32 division, round-half-even.
// Out of line: it runs for a small fraction of elements (near rounding ties), and inlining its
// double-precision exp/log into every unrolled call site bloats kernels past the I-cache.
__device__ __noinline__ float code_mag_careful_ool(float a, int linear, float t, float d) {
  float pw = linear ? a : exp_cr(t * log_cr(a));
  return rintf(pw / d);
}
QVIT_DEV float code_mag_careful(float a, const QParams& p) {
  return code_mag_careful_ool(a, p.qtype == QVIT_QT_LINEAR, p.t, p.d);
}

// Guarded fast path, branch-free: an approximate quotient q; if q is provably far from a rounding
// tie (x.5) the rounded result equals the careful one. Otherwise `need` is set and the caller runs
// code_mag_careful for that element (rare: ~1e-4 of elements). Error budget: q carries <= ~3 ulp
// (linear) or (|t ln a| + 3) ulp (nonlinear) of relative error; the margin is 8x that.
// Returns the signed code (integer-valued float); x == 0 and NaN give 0.
QVIT_DEV float quant_fast(float x, const QParams& p, bool& need) {
  if (p.qtype == QVIT_QT_ULTRA_ACT) {
    // uniform_quantize(clamp(x,0,1)) with n = 2^b - 1: round(c * n) (quant_ultra.py:18-19,71)
    need = false;
    return rintf(fminf(fmaxf(x, 0.f), 1.f) * p.levels);
  }
  const float a = fabsf(x);
  float q, relerr;
  if (p.qtype == QVIT_QT_LINEAR) {
    q = a * p.inv_d;
    relerr = 32.f * 1.1920929e-7f;
  } else {
    // |t * ln(a)| bound from the binary exponent (no transcendental on the t == 1 path)
    const float eb = fabsf(p.t) * (float)(abs(__builtin_amdgcn_frexp_expf(a)) + 1);
    const float pw = (p.t == 1.f) ? a : __builtin_amdgcn_exp2f(p.t * __builtin_amdgcn_logf(a));
    q = pw * p.inv_d;
    relerr = (eb * 0.6931472f + 4.f) * 8.f * 1.1920929e-7f;
  }
  const float f = q - floorf(q);
  const bool in_range = (a < p.qm) && (a > 0.f);
  const bool tiny = (p.qtype == QVIT_QT_NONLINEAR) && !(a > 1e-30f);  // hw log2 flushes denormals
  need = in_range && ((fabsf(f - 0.5f) <= fabsf(q) * relerr + 1e-37f) || tiny || p.careful);
  float k = (a >= p.qm) ? p.L : rintf(q);  // saturation mask (:67, :159)
  k = copysignf(k, x);                     // output = sign(input) * output (:68, :160)
  return (a > 0.f) ? k : 0.f;              // zero mask (:66, :158); NaN -> 0
}

// Careful result for an element flagged by quant_fast.
QVIT_DEV float quant_fixup(float x, const QParams& p) {
  return copysignf(code_mag_careful(fabsf(x), p), x);
}

// Signed code k (as an integer-valued float), v_ref = d * k.
QVIT_DEV float quant_code(float x, const QParams& p) {
  bool need;
  const float k = quant_fast(x, p, need);
  return need ? quant_fixup(x, p) : k;
}

// The reference's fp32 fake-quant value for the same element (d * k, rounded once in fp32,
// then the sign applied) — used by qvit_fake_quant_f32.
QVIT_DEV float fake_quant_value(float x, const QParams& p) {
  if (p.qtype == QVIT_QT_ULTRA_ACT) {
    return quant_code(x, p) / p.levels;      // round(c*n)/n
  }
  // sign(x) * fl(d * rne(p/d)) == fl(d * (sign(x) * rne(p/d))): multiplying by +-1 is exact.
  return p.d * quant_code(x, p);
}

QVIT_DEV int8_t to_i8_sat(float k) {
  k = fminf(fmaxf(k, -127.f), 127.f);
  return (int8_t)(int)k;
}


// ---- code tables of the int8 epilogues (qvit_epi_table_build; GEMM and attention epilogues) ----------
// header (16 B) + nb entries {thr, lo | hi << 8} (8 B each); see gemm_w4a8.hip for the construction.
struct EpiTableHdr {
  float c0;     // C = 2^23 + (-v_lo * inv_w), rounded: see epi_bucket_bits
  float inv_w;
  int nb;
  int valid;
};
struct EpiTableEnt {
  float thr;
  int8_t lo, hi;
  int16_t pad;
};
// Bucket of v: f = med3(fma(v, inv_w, C), 2^23, 2^23 + nb - 1). In [2^23, 2^24) a float's ulp is 1, so the
// fma itself rounds to the bucket index, which then sits in f's low mantissa bits: bits(f) = 0x4B000000 + j.
// Monotone in v (the builder's bisection relies on it); one FMA and one med3, no float->int conversion,
// and the entry's byte offset is one shift-add of bits(f).
// 2^23 + nb - 1 from its bit pattern (integer add: stays on the scalar unit for a uniform nb)
QVIT_DEV float epi_top(int nb) { return __int_as_float(0x4B000000 + nb - 1); }
QVIT_DEV uint32_t epi_bucket_bits(float v, float C, float inv_w, float top) {
  return __float_as_uint(__builtin_amdgcn_fmed3f(fmaf(v, inv_w, C), 8388608.f, top));
}
QVIT_DEV int epi_bucket(float v, float C, float inv_w, float top) {
  return (int)(epi_bucket_bits(v, C, inv_w, top) - 0x4B000000u);
}
// v's 8-B entry in an LDS-resident table whose entries start at `ent`
QVIT_DEV const uint2* epi_entry(const int8_t* ent, float v, float C, float inv_w, float top) {
  return reinterpret_cast<const uint2*>(ent + ((epi_bucket_bits(v, C, inv_w, top) << 3) - (0x4B000000u << 3)));
}

// wd.byte[J] = (v >= thr) ? byte 1 of lohi : byte 0 of lohi (J = 0 also zeroes bytes 1..3):
// a v_cmp and one SDWA v_cndmask that writes the selected byte in place.
template <int J>
QVIT_DEV void epi_select_byte(uint32_t& wd, float v, float thr, uint32_t lohi) {
  if (J == 0)
    asm("v_cmp_ge_f32_e32 vcc, %1, %2\n\t"
        "v_cndmask_b32_sdwa %0, %3, %3, vcc dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_1"
        : "=v"(wd) : "v"(v), "v"(thr), "v"(lohi) : "vcc");
  else if (J == 1)
    asm("v_cmp_ge_f32_e32 vcc, %1, %2\n\t"
        "v_cndmask_b32_sdwa %0, %3, %3, vcc dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0 src1_sel:BYTE_1"
        : "+v"(wd) : "v"(v), "v"(thr), "v"(lohi) : "vcc");
  else if (J == 2)
    asm("v_cmp_ge_f32_e32 vcc, %1, %2\n\t"
        "v_cndmask_b32_sdwa %0, %3, %3, vcc dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0 src1_sel:BYTE_1"
        : "+v"(wd) : "v"(v), "v"(thr), "v"(lohi) : "vcc");
  else
    asm("v_cmp_ge_f32_e32 vcc, %1, %2\n\t"
        "v_cndmask_b32_sdwa %0, %3, %3, vcc dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0 src1_sel:BYTE_1"
        : "+v"(wd) : "v"(v), "v"(thr), "v"(lohi) : "vcc");
}


// SLEEF's single-precision exp, 1-ulp variant (Sleef_expf*_u10, the `xexpf` kernel torch links statically):
// Cody-Waite reduction by ln 2 in two fp32 parts, a degree-6 polynomial in fma steps, and the scale by 2^q
// as two power-of-two multiplies. Every step is one IEEE fp32 operation, so the device value equals the
// CPU's bit for bit (pinned by tests/test_gpu_kats.py::test_gelu_bit_exact_all_floats).
QVIT_DEV float pow2i_f(int q) { return __int_as_float((q + 0x7f) << 23); }
QVIT_DEV float sleef_expf_u10(float d) {
#pragma clang fp contract(off)
  // q = rint(d / ln 2), clamped only where the result is overridden below (|d| > 104)
  const float fq = fminf(fmaxf(rintf(d * 1.442695040888963407359924681001892137426645954152985934135449406931f),
                               -256.f), 256.f);
  const int q = (int)fq;
  float s = fmaf(fq, -0.693145751953125f, d);
  s = fmaf(fq, -1.428606765330187045e-06f, s);
  float u = 0.000198527617612853646278381f;
  u = fmaf(u, s, 0.00139304355252534151077271f);
  u = fmaf(u, s, 0.00833336077630519866943359f);
  u = fmaf(u, s, 0.0416664853692054748535156f);
  u = fmaf(u, s, 0.166666671633720397949219f);
  u = fmaf(u, s, 0.5f);
  u = 1.0f + fmaf(s * s, u, s);
  u = (u * pow2i_f(q >> 1)) * pow2i_f(q - (q >> 1));
  u = (d < -104.f) ? 0.f : u;
  return (d > 100.f) ? INFINITY : u;
}

// nn.GELU() (approximate='none', vit_model.py:242,173) exactly as torch's ATen CPU kernel computes it
// (GeluKernelImpl, vectorized branch): (x * 0.5) * (1 + erf(x * M_SQRT1_2)) with Vectorized<float>::erf =
// Abramowitz-Stegun 7.1.26: sign(u) * fma(-exp(-u*u) * t, r(t), 1), t = 1 / fma(0.3275911, |u|, 1) (IEEE
// division), r a degree-4 Horner polynomial in fma steps, exp = SLEEF expf u10. Bit-identical to the oracle's
// GELU (oracle/quant_oracle.py:gelu) on every fp32 input. Used by the int8-epilogue code tables and the
// direct epilogue; the per-element cost is irrelevant there (the tables are built once per quantizer).
QVIT_DEV float gelu_ref(float x) {
#pragma clang fp contract(off)
  const float u = x * 0.70710678118654752440f;
  const float t = 1.0f / fmaf(0.3275911f, fabsf(u), 1.0f);
  float r = fmaf(1.061405429f, t, -1.453152027f);
  r = fmaf(r, t, 1.421413741f);
  r = fmaf(r, t, -0.284496736f);
  r = fmaf(r, t, 0.254829592f);
  const float e = sleef_expf_u10(-(u * u));
  const float erf_abs = fmaf(-e * t, r, 1.0f);
  return (x * 0.5f) * (1.0f + copysignf(erf_abs, u));
}

// Lane id from a volatile asm: values derived from it are recomputed where used instead of being
// hoisted out of the tile / unit loop (which would keep them live across the register-bound main loop).
QVIT_DEV int lane_opaque() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

// ---- LDS-DMA and asm-issued global loads (GEMM and fused-attention pipelines) ------------------------
QVIT_DEV uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// One 1-KiB LDS-DMA piece: 64 lanes x 16 B from per-lane global addresses to lds_base + 16*lane.
// Issued from asm so the compiler neither counts it nor drains vmcnt for it; M0 is saved/restored.
QVIT_DEV void dma16(const void* gsrc, uint32_t lds_base) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_base)
      : "memory");
}

// The same from a wave-uniform SGPR base + a per-lane 32-bit byte offset (the global "saddr" form): no
// 64-bit per-lane address arithmetic and no VGPR pair holding a base pointer across the main loop.
QVIT_DEV void dma16s(const void* sbase, uint32_t voff, uint32_t lds_base) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %2\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(lds_base)
      : "memory");
}

static inline int qvit_hip_status(hipError_t e) {
  return e == hipSuccess ? QVIT_OK : (QVIT_EHIP - (int)e);
}
