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
    p.L = rintf(expf(p.t * logf(fabsf(p.qm) + 1e-6f)) / p.d);
  }
  return p;
}

// Careful magnitude code for 0 < a < q_m: the reference's op sequence in fp32 with IEEE division
// (hipcc default: correctly rounded fp32 divide) and ocml exp/log.
QVIT_DEV float code_mag_careful(float a, const QParams& p) {
  float pw = (p.qtype == QVIT_QT_LINEAR) ? a : expf(p.t * logf(a));
  return rintf(pw / p.d);
}

// Guarded fast path: an approximate quotient q; if q is provably far from a rounding boundary
// (x.5) the rounded result equals the careful one, otherwise fall back to the careful sequence.
// Error budget: q carries <= ~3 ulp (linear) or (|t ln a| + 3) ulp (nonlinear) of relative error;
// the margin below is 8x that, so both paths round identically whenever the fast one is taken.
QVIT_DEV float code_mag(float a, const QParams& p) {
  if (p.careful) return code_mag_careful(a, p);
  float q, relerr;
  if (p.qtype == QVIT_QT_LINEAR) {
    q = a * p.inv_d;
    relerr = 32.f * 1.1920929e-7f;
  } else {
    if (!(a > 1e-30f)) return code_mag_careful(a, p);  // hw log2 flushes denormals
    float lg = __builtin_amdgcn_logf(a);                 // v_log_f32 (log2)
    float e = p.t * lg;
    float pw = (p.t == 1.f) ? a : __builtin_amdgcn_exp2f(e);  // v_exp_f32
    q = pw * p.inv_d;
    relerr = (fabsf(e) * 0.6931472f + 4.f) * 8.f * 1.1920929e-7f;
  }
  float aq = fabsf(q);
  float f = aq - floorf(aq);
  if (fabsf(f - 0.5f) > aq * relerr + 1e-37f) return rintf(q);
  return code_mag_careful(a, p);
}

// Signed code k (as an integer-valued float), v_ref = d * k.
QVIT_DEV float quant_code(float x, const QParams& p) {
  if (p.qtype == QVIT_QT_ULTRA_ACT) {
    // uniform_quantize(clamp(x,0,1)) with n = 2^b - 1: round(c * n) (quant_ultra.py:18-19,71)
    float c = fminf(fmaxf(x, 0.f), 1.f);
    return rintf(c * p.levels);
  }
  float a = fabsf(x);
  float k;
  if (a >= p.qm) {
    k = p.L;                     // output[input_abs >= q_m] = d*round(range_pow/d)   (:67, :159)
  } else if (a > 0.f) {
    k = code_mag(a, p);
  } else {
    k = 0.f;                     // output[input_abs <= q_s] = 0                      (:66, :158)
  }
  // output = sign(input) * output (:68, :160); sign(0) = 0. NaN inputs map to 0.
  return (x > 0.f) ? k : ((x < 0.f) ? -k : 0.f);
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

// nn.GELU() (approximate='none'): x * 0.5 * (1 + erf(x / sqrt(2)))   (vit_model.py:242,173)
QVIT_DEV float gelu_erf(float x) {
  return x * 0.5f * (1.0f + erff(x * 0.70710678118654752440f));
}

static inline int qvit_hip_status(hipError_t e) {
  return e == hipSuccess ? QVIT_OK : (QVIT_EHIP - (int)e);
}
