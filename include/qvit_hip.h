/*
 * qvit_hip.h — C-ABI of libqvit_hip.so, the MI355X (gfx950) implementation of the
 * 4-bit QuantizeLinear / QuantizeConv2d forward path of LongAoTianxia/Quantized_ViT.
 *
 * Every entry point replaces one step of the reference's fake-quant forward
 * (paths relative to the reference checkout; OTO = QViT_with_GETA/only_train_once):
 *
 *   qvit_quantize_act_i8      OTO/quantization/quant_layers.py:356-381 (QuantizeMixin.quantize_act)
 *                             -> SymQuantizerLinear.forward :137-161 / SymQuantizerNonLinear.forward :41-69,
 *                             emitted as integer codes k (value = d * k) instead of fake-quant floats;
 *                             also 4-bit quantization/quant_ultra.py:59-73 (activation_quantize_fn).
 *   qvit_fake_quant_f32       the same quantizers emitting the reference's fp32 fake-quant values
 *                             (used when a layer's level count does not fit int8, e.g. num_bits > 8).
 *   qvit_pack_weight          quant_layers.py:332-354 (QuantizeMixin.quantize_weight) + the GEMM operand
 *                             layout: codes packed int4 (8 per u32) or int8, rows padded/permuted.
 *   qvit_im2col_quant_i8      quant_layers.py:575-587 (QuantizeConv2d.forward): the conv input patches
 *                             quantized to codes, K-order (c, kh, kw) = the reference weight flattening.
 *   qvit_layernorm_quant_i8   vit_model.py:193,206-207 (Block.norm1/norm2, eps 1e-6) fused with the next
 *                             QuantizeLinear's quantize_act (quant_layers.py:497-498).
 *   qvit_gemm                 quant_layers.py:499 (nn.functional.linear on fake-quant operands) as an
 *                             int8 x int4/int8 -> int32 MFMA contraction with a fused epilogue:
 *                             d_act * d_wt * acc + bias, optionally + residual (vit_model.py:206-207),
 *                             or GELU (vit_model.py:173) + the next layer's activation quantizer.
 *   qvit_gemm_wonly           quant_layers.py:495-499 in the default WEIGHT_ONLY mode (quant_model.py:23): fp32
 *                             activations x int4/int8 weight codes on bf16 MFMA (x split into three exact
 *                             bf16 terms), d_wt * acc + bias — F.linear(x, quantize_weight(W), b).
 *   qvit_conv_wonly           quant_layers.py:575-587 (QuantizeConv2d.forward, WEIGHT_ONLY) and quant_ultra.py:85-89
 *                             (Conv2d_Q.forward): the same contraction as an implicit GEMM over the NCHW input
 *                             (patches gathered in the kernel), NCHW fp32 out — F.conv2d(x, quantize_weight(W), b).
 *   qvit_ultra_*              4-bit quantization/quant_ultra.py:8-91 + mymodel.py:62-144 (UltraNet: weight
 *                             codes, BN folding, fused conv+BN+quantizer+maxpool blocks, the 26 x 26 tail of
 *                             the network in one launch, YOLO decode).
 *   qvit_attention            vit_model.py:133-149 (Attention.forward between qkv and proj):
 *                             softmax(q k^T * scale) v per (image, head), fp32 out or fused with the
 *                             proj layer's quantize_act (quant_layers.py:497) -> int8 codes.
 *
 * Conventions
 *   - Plain pointers and sizes only. All pointers are device pointers (hipMalloc'd / torch CUDA
 *     tensors) unless stated otherwise. Every entry point is stream-ordered on `stream`, never
 *     synchronises the host, never allocates, and is safe to capture into a hipGraph.
 *   - Quantizer parameters are per-tensor device scalars (float[1]): d_quant, q_m, t_quant, exactly the
 *     reference's nn.Parameter([1]) tensors (quant_layers.py:315-325). t_quant may be NULL for the
 *     linear quantizer. Reading them on the device keeps the host free of .item() syncs.
 *   - Return value: 0 on success; QVIT_E* (< 0) on a rejected argument; QVIT_EHIP - hipError_t
 *     when a launch fails. qvit_strerror() maps a code to text.
 */
#ifndef QVIT_HIP_H
#define QVIT_HIP_H

#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---------------------------------------------------------------------- */
#define QVIT_OK          0
#define QVIT_EINVAL     -1   /* bad size / stride / enum */
#define QVIT_EALIGN     -2   /* pointer or leading dimension not aligned as required */
#define QVIT_ENULL      -3   /* required pointer is NULL */
#define QVIT_EHIP    -1000   /* QVIT_EHIP - (int)hipError_t */

/* ---- quantizer kinds (QuantizationType, quant_layers.py:20-24; quant_ultra.py) ---------- */
#define QVIT_QT_LINEAR      0  /* SymQuantizerLinear / DGEQuantizer forward: k = sgn(x) rne(|x|/d) */
#define QVIT_QT_NONLINEAR   1  /* SymQuantizerNonLinear: k = sgn(x) rne(exp(t log|x|)/d)          */
#define QVIT_QT_ULTRA_ACT   2  /* quant_ultra activation_quantize_fn: k = rne(clamp(x,0,1) (2^b-1)),
                                  d_quant = NULL, the level count 2^b-1 is passed as `levels`      */

/* ---- GEMM weight storage ---------------------------------------------------------------- */
#define QVIT_W4 4   /* int4 codes, 8 per uint32 (see qvit_pack_weight for the nibble order) */
#define QVIT_W8 8   /* int8 codes                                                           */
#define QVIT_W4R 40 /* qvit_gemm / qvit_gemm_qkv_split only: QVIT_W4 codes in the register-weight image
                       (qvit_pack_weight_w4r); same results, each wave's weight rows loaded into registers */
#define QVIT_W8R 80 /* qvit_gemm / qvit_gemm_qkv_split only: QVIT_W4 codes in the int8 register image
                       (qvit_pack_weight_w8r); same results, no unpack in the main loop, twice the bytes  */
#define QVIT_W16 16 /* qvit_gemm_wonly only: codes |k| <= 32639 as balanced base-256 digits k = 256 h + l, h and l
                       in [-128, 127], two QVIT_W8 images of npad * kpad bytes (h, then l; qvit_pack_weight)  */
#define QVIT_W24 24 /* the same with three digits k = 65536 a + 256 h + l (|k| < 2^23, e.g. 16-bit layers whose
                       saturation code is 32768): three QVIT_W8 images, a, h, l                               */

/* ---- GEMM epilogues ----------------------------------------------------------------------- */
#define QVIT_EPI_F32        0  /* C[m,n]  = d_act d_wt acc + bias[n]                 (fp32)          */
#define QVIT_EPI_F32_RESID  1  /* C[m,n] += d_act d_wt acc + bias[n]                 (fp32, in place) */
#define QVIT_EPI_I8_GELU    2  /* C[m,n]  = q_next(gelu(d_act d_wt acc + bias[n]))  (int8 codes)    */
#define QVIT_EPI_I8         3  /* C[m,n]  = q_next(d_act d_wt acc + bias[n])        (int8 codes)    */
#define QVIT_EPI_I32        4  /* C[m,n]  = acc                                      (int32, exact)  */
#define QVIT_EPI_QKV_SPLIT  5  /* fp16 hi/lo planes of in_scale (d_act d_wt acc + bias[n]); only via
                                  qvit_gemm_qkv_split (qvit_gemm rejects it)                        */

/* ---- qvit_ultra_conv epilogues (UltraNet, 4-bit quantization/mymodel.py) -------------------- */
#define QVIT_ULTRA_CODES       0  /* codes = rne(clamp(bn(acc/den), 0, 1) (2^a_bit-1))       (uint codes) */
#define QVIT_ULTRA_CODES_POOL  1  /* the same followed by MaxPool2d(2, 2)                    (uint codes) */
#define QVIT_ULTRA_F32         2  /* out = acc/den + bias (shift = bias)                      (fp32)       */

/* ---- qvit_attention output modes -------------------------------------------------------------- */
#define QVIT_ATT_F32        0  /* out = softmax(q k^T * scale) v                     (fp32)          */
#define QVIT_ATT_I8         1  /* out = q_next(softmax(q k^T * scale) v)             (int8 codes)    */

/* Tile geometry the packed operands must be padded to. */
#define QVIT_TILE_N  256   /* weight rows (out features) are padded to a multiple of this  */
#define QVIT_TILE_K  128   /* the reduction dim is padded to a multiple of this (zeros)    */

const char* qvit_strerror(int code);
/* Library version / build tag, e.g. "qvit_hip 0.1 gfx950". Host pointer, static storage. */
const char* qvit_version(void);

/*
 * Activation quantizer -> int8 codes (value = d_quant * code).
 *   x      : fp32 [rows][ldx], first `cols` columns used
 *   codes  : int8 [rows][ldc]; columns [cols, kpad) are written with 0 (kpad <= ldc, kpad % 16 == 0)
 *   qtype  : QVIT_QT_*; levels is only read for QVIT_QT_ULTRA_ACT.
 * Codes saturate at +-127 (the caller rejects layers whose level count exceeds 127).
 * Replaces quant_layers.py:356-381 (+ :41-69 / :137-161) and quant_ultra.py:66-73.
 */
int qvit_quantize_act_i8(const float* x, int64_t rows, int64_t cols, int64_t ldx,
                         int qtype, const float* d_quant, const float* q_m, const float* t_quant,
                         int levels, int8_t* codes, int64_t ldc, int64_t kpad, hipStream_t stream);

/*
 * Fake-quant fp32 values exactly as the reference returns them (y = sgn(x) * (d * rne(...)),
 * saturation and zero masks in the reference's order). Elementwise over n contiguous floats.
 * Replaces SymQuantizerLinear/NonLinear.forward (quant_layers.py:41-69,137-161) when a layer's
 * levels do not fit the integer path.
 */
int qvit_fake_quant_f32(const float* x, int64_t n, int qtype, const float* d_quant,
                        const float* q_m, const float* t_quant, int levels, float* y,
                        hipStream_t stream);

/*
 * y = GELU(x) elementwise over n contiguous floats: nn.GELU() (QViT_with_GETA/vit_model.py:173,242), bit-identical
 * to torch's ATen CPU kernel (erf as Abramowitz-Stegun 7.1.26 with SLEEF's expf, IEEE division) — the same
 * function the QVIT_EPI_I8_GELU epilogue evaluates. For the Mlp path outside the fused block, and for tests.
 */
int qvit_gelu_f32(const float* x, int64_t n, float* y, hipStream_t stream);

/*
 * Weight quantizer + GEMM operand packing (QuantizeMixin.quantize_weight, quant_layers.py:332-354).
 *   w      : fp32 [n][ldw], first k columns used (nn.Linear weight [out,in]; a conv weight
 *            [Cout,Cin,kh,kw] is passed as [Cout][Cin*kh*kw]).
 *   wfmt   : QVIT_W4 -> packed uint32 [npad][kpad/8]; QVIT_W8 -> int8 [npad][kpad].
 *            npad % QVIT_TILE_N == 0, kpad % QVIT_TILE_K == 0, npad >= n, kpad >= k; padding = 0.
 *   Row order: within every 64-row group the two 2-bit fields of the row index are swapped
 *   (packed row (r<<4)|(q<<2)|j holds weight row (q<<4)|(r<<2)|j) so that each GEMM lane ends up
 *   owning 16 consecutive output features.  W4 nibble order inside each uint32 covering
 *   k0..k0+7: byte b holds k0+b in bits [0,4) and k0+4+b in bits [4,8), two's complement.
 *   overflow (int32[1], device, may be NULL): atomically set to 1 if any code does not fit wfmt.
 */
int qvit_pack_weight(const float* w, int64_t n, int64_t k, int64_t ldw, int qtype,
                     const float* d_quant, const float* q_m, const float* t_quant, int wfmt,
                     void* packed, int64_t npad, int64_t kpad, int32_t* overflow,
                     hipStream_t stream);

/*
 * The register-weight image (QVIT_W4R) of a QVIT_W4 image from qvit_pack_weight: the same npad * kpad / 2 bytes,
 * re-ordered so that in every (256-row tile, 64-deep k stage) chunk of 8 KiB the GEMM lane l of wave w finds its
 * four 8-byte fragments (rows 64 w + 16 r + (l & 15) of the tile, r = 0..3, k bytes 8 (l >> 4) .. + 7 of the
 * stage) contiguously at byte 2048 w + 32 l. npad % QVIT_TILE_N == 0, kpad % QVIT_TILE_K == 0, kpad <= 65536;
 * out must not alias packed. qvit_gemm with wfmt QVIT_W4R on it gives the QVIT_W4 results byte for byte (same
 * accumulation order); it loads each wave's weights straight into registers instead of through LDS.
 * Replaces nothing in the reference: a second storage form of quantize_weight's codes (quant_layers.py:332-354).
 */
int qvit_pack_weight_w4r(const void* packed, int64_t npad, int64_t kpad, void* out, hipStream_t stream);

/*
 * The int8 register image (QVIT_W8R) of a QVIT_W4 image from qvit_pack_weight: npad * kpad bytes (twice the W4
 * image). In every (256-row tile, 64-deep k stage) chunk of 16 KiB the GEMM lane l of wave w finds its four 16-byte
 * MFMA operands (rows 64 w + 16 r + (l & 15) of the tile, r = 0..3, k 16 (l >> 4) .. + 15 of the stage, each code
 * as the byte 16 k) contiguously at byte 4096 w + 64 l. Same argument rules as qvit_pack_weight_w4r. qvit_gemm with
 * wfmt QVIT_W8R on it gives the QVIT_W4 results byte for byte (same operands, same accumulation order) with no int4
 * unpack in the main loop.
 * Replaces nothing in the reference: a third storage form of quantize_weight's codes (quant_layers.py:332-354).
 */
int qvit_pack_weight_w8r(const void* packed, int64_t npad, int64_t kpad, void* out, hipStream_t stream);

/*
 * Pads a bias vector to npad floats (zeros past n; bias may be NULL -> all zeros).
 */
int qvit_pad_bias(const float* bias, int64_t n, float* out, int64_t npad, hipStream_t stream);

/*
 * Conv input -> quantized im2col codes for QuantizeConv2d (quant_layers.py:575-587), groups == 1.
 *   x      : fp32 NCHW [B][C][H][W] contiguous
 *   codes  : int8 [B*OH*OW][ldc], row (b, oh, ow), column (c, ih, iw) = c*kh*kw + ih*kw + iw;
 *            columns [C*kh*kw, kpad) zero. Zero-padding of the image quantizes to code 0, as in
 *            the reference (quantize_act runs before F.conv2d pads).
 */
int qvit_im2col_quant_i8(const float* x, int64_t B, int64_t C, int64_t H, int64_t W,
                         int kh, int kw, int sh, int sw, int ph, int pw, int dh, int dw,
                         int qtype, const float* d_quant, const float* q_m, const float* t_quant,
                         int levels, int8_t* codes, int64_t ldc, int64_t kpad, hipStream_t stream);

/*
 * LayerNorm (biased variance, eps) followed by the next layer's activation quantizer.
 *   x : fp32 [rows][ldx] (D = cols), gamma/beta fp32 [cols] (may be NULL -> 1 / 0)
 *   codes : int8 [rows][ldc], columns [cols, kpad) zero.
 *   code_table : nullable, 16-B aligned; a qvit_epi_table_build table (QVIT_EPI_I8 semantics) of the
 *            same quantizer, used only if valid and <= 2046 buckets (results never depend on it).
 */
int qvit_layernorm_quant_i8(const float* x, int64_t rows, int64_t cols, int64_t ldx,
                            const float* gamma, const float* beta, float eps,
                            int qtype, const float* d_quant, const float* q_m,
                            const float* t_quant, int levels,
                            int8_t* codes, int64_t ldc, int64_t kpad,
                            const void* code_table, hipStream_t stream);

/*
 * Quantized contraction C = epilogue(A_codes @ W_codes^T).
 *   A      : int8 codes [M][lda], K valid columns; K % QVIT_TILE_K == 0 (and K <= 65536 for QVIT_W4), lda % 16 == 0,
 *            A 16-byte aligned, columns past the true in-features must be 0 (the quantizers
 *            above write them so).
 *   Wp     : packed weights from qvit_pack_weight (wfmt, npad rows, kpad == K), or with wfmt QVIT_W4R the
 *            qvit_pack_weight_w4r image of a QVIT_W4 one (same results).
 *   N      : true out features (<= npad); outputs for n >= N are not written.
 *   d_act, d_wt : device float[1] scales; bias : device float[npad] (padded) or NULL.
 *   C      : fp32 / int8 / int32 [M][ldc] per epilogue; ldc % 4 == 0 (fp32/int32), % 16 (int8).
 *   For QVIT_EPI_I8*: the next layer's quantizer (out_qtype, out_d, out_qm, out_t, out_levels) and an
 *   optional code table (qvit_epi_table_build, NULL -> per-element evaluation).
 */
int qvit_gemm(const int8_t* A, int64_t M, int64_t K, int64_t lda,
              const void* Wp, int wfmt, int64_t N, int64_t npad,
              const float* d_act, const float* d_wt, const float* bias,
              int epilogue, void* C, int64_t ldc,
              int out_qtype, const float* out_d, const float* out_qm, const float* out_t,
              int out_levels, const void* epi_table, hipStream_t stream);

/*
 * QVIT_ACT_T32: activation codes in the operand order of the int8 32x32x32 matrix instruction, the input of
 * qvit_gemm_a32. An [M][kpad] code matrix (kpad % 64 == 0) is stored as 1-KiB blocks of 32 rows x 32 columns,
 * block (r / 32, c / 32) at byte (r / 32 * kpad / 32 + c / 32) * 1024; inside it, 16-byte group
 * (r % 32) + 32 * ((c / 16) % 2) holds columns c - c % 16 .. + 15 of row r. Buffers hold ceil(M / 64) * 64 rows
 * (rows past M are never stored).
 *
 * qvit_layernorm_quant_i8_t32: qvit_layernorm_quant_i8 (vit_model.py:206-207 norm2 + the fc1 layer's quantize_act,
 *   quant_layers.py:356-381) with the codes written in QVIT_ACT_T32 order: cols % 4 == 0, cols <= 1024,
 *   kpad % 64 == 0, x / gamma / beta / codes 16-byte aligned. Same codes as qvit_layernorm_quant_i8, byte for byte.
 * qvit_gemm_a32: qvit_gemm with the activations in QVIT_ACT_T32 order, for the int8-code epilogues of Mlp.fc1
 *   (quant_layers.py:495-499 under vit_model.py:172: GELU + fc2's quantizer): a weight-stationary schedule (each
 *   CU holds one 96-row panel of the int4 weights in LDS for the whole launch) on int8 32x32x32 MFMA. Same codes
 *   as qvit_gemm on the row-major codes, byte for byte. Shapes: qvit_gemm_a32_fits (wfmt QVIT_W4, epilogue
 *   QVIT_EPI_I8 / QVIT_EPI_I8_GELU, N == npad == 3072, K == 768 or 1024) returns 1, else the call is QVIT_EINVAL.
 *   C: int8 [M][ldc], ldc % 16 == 0, 16-byte aligned.
 */
int qvit_layernorm_quant_i8_t32(const float* x, int64_t rows, int64_t cols, int64_t ldx, const float* gamma,
                                const float* beta, float eps, int qtype, const float* d_quant, const float* q_m,
                                const float* t_quant, int levels, int8_t* codes, int64_t kpad,
                                const void* code_table, hipStream_t stream);
int qvit_gemm_a32_fits(int64_t K, int wfmt, int64_t N, int64_t npad, int epilogue);
int qvit_gemm_a32(const int8_t* A, int64_t M, int64_t K, const void* Wp, int wfmt, int64_t N, int64_t npad,
                  const float* d_act, const float* d_wt, const float* bias, int epilogue, void* C, int64_t ldc,
                  int out_qtype, const float* out_d, const float* out_qm, const float* out_t, int out_levels,
                  const void* epi_table, hipStream_t stream);

/*
 * Weight-only QuantizeLinear.forward (quant_layers.py:495-499, quant_mode WEIGHT_ONLY: quantize_act is the
 * identity, :356-358): Y[m, n] = d_wt * sum_k X[m, k] k_w[n, k] + bias[n] with fp32 X.
 *   X      : fp32 [M][ldx], K valid columns; K % QVIT_TILE_K == 0 (pad X with zero columns to the packed
 *            kpad), ldx % 4 == 0, X 16-byte aligned.
 *   Wp     : packed weights from qvit_pack_weight (wfmt QVIT_W4 / QVIT_W8, npad rows, kpad == K), or QVIT_W16 /
 *            QVIT_W24: the QVIT_W8 images of the balanced base-256 digits back to back (levels beyond int8).
 *   d_wt   : device float[1]; bias : device float[npad] (padded) or NULL.
 *   Y      : fp32 [M][ldy], ldy % 4 == 0, 16-byte aligned; outputs for n >= N are not written.
 *   workspace : optional device buffer (16-byte aligned, workspace_bytes long) for small M: with fewer tiles
 *            than half the CUs the K range is split over several workgroups whose fp32 partials
 *            (splits * M * npad floats) are then summed in a fixed order; NULL -> no split.
 * fp32-GEMM accuracy: X is split into three bf16 terms whose sum is X exactly, every product with a code is
 * exact in fp32, accumulation is fp32 (the order of the K-term sum differs from the reference's GEMM).
 */
int qvit_gemm_wonly(const float* X, int64_t M, int64_t K, int64_t ldx, const void* Wp, int wfmt,
                    int64_t N, int64_t npad, const float* d_wt, const float* bias, float* Y, int64_t ldy,
                    float* workspace, int64_t workspace_bytes, hipStream_t stream);

/*
 * Weight-only convolution (QuantizeConv2d.forward, quant_layers.py:575-587, quant_mode WEIGHT_ONLY; UltraNet's
 * Conv2d_Q.forward, quant_ultra.py:85-89, whose quantize_fn values are k / (2^(w_bit-1) - 1)):
 *   Y[b][n][oy][ox] = d_wt * sum_{c,ky,kx} X[b][c][oy sh - ph + ky dh][ox sw - pw + kx dw] k_w[n][(c kh + ky) kw + kx]
 *                     + bias[n]   (zero padding; groups = 1)
 *   X      : fp32 NCHW [B][C][H][W], contiguous (any alignment).
 *   Wp     : qvit_pack_weight image of the codes [N][C kh kw] in the weight's flattening order (npad rows, kpad
 *            == K >= C kh kw columns, K % QVIT_TILE_K == 0); wfmt as qvit_gemm_wonly.
 *   d_wt, bias : as qvit_gemm_wonly.
 *   Y      : fp32 NCHW [B][N][OH][OW] contiguous, OH = (H + 2 ph - dh (kh - 1) - 1) / sh + 1 (OW alike).
 *   workspace : as qvit_gemm_wonly (split K for few output pixels).
 * The patch rows are never materialised: the kernel gathers them from X stage by stage. Same arithmetic as
 * qvit_gemm_wonly on the patch matrix.
 */
int qvit_conv_wonly(const float* X, int64_t B, int64_t C, int64_t H, int64_t W, int kh, int kw, int sh, int sw,
                    int ph, int pw, int dh, int dw, const void* Wp, int wfmt, int64_t N, int64_t npad, int64_t K,
                    const float* d_wt, const float* bias, float* Y, float* workspace, int64_t workspace_bytes,
                    hipStream_t stream);
/* N <= 64 output channels with QVIT_W4 / QVIT_W8 codes whose first ceil(C kh kw / 64) stages of 16 ceil(N / 16)
 * rows take at most 24 KiB (and C kh kw <= 1024, H, W < 32767) run the narrow schedule: weights and a tap-offset
 * table LDS-resident, every wave on its own 16-pixel tiles, no workspace used; bit-identical to the wide one.
 * qvit_conv_wonly_narrow(0 / 1) turns it off / on for the process (-1: query); returns the previous setting. */
int qvit_conv_wonly_narrow(int enable);

/*
 * Conv2d_Q -> BatchNorm2d (eval, running statistics) -> activation_quantize_fn in one launch (UltraNet's blocks,
 * reference mymodel.py:71-124 run module by module; quant_ultra.py:59-73, :76-91):
 *   Y = round(clamp(fma(y, bn_alpha[n], bn_shift[n]), 0, 1) * a_levels) / a_levels,  y = qvit_conv_wonly's value
 *   (one fused multiply-add with the fold qvit_ultra_bn_fold computes; IEEE division by a_levels = 2^a_bit - 1).
 *   Arguments as qvit_conv_wonly; bn_alpha, bn_shift: device float[N]; 1 <= a_levels <= 127.
 * Only for layers on the narrow schedule (QVIT_EINVAL otherwise: run the modules one by one).
 */
int qvit_conv_wonly_bn_act(const float* X, int64_t B, int64_t C, int64_t H, int64_t W, int kh, int kw, int sh,
                           int sw, int ph, int pw, int dh, int dw, const void* Wp, int wfmt, int64_t N, int64_t npad,
                           int64_t K, const float* d_wt, const float* bias, const float* bn_alpha,
                           const float* bn_shift, int a_levels, float* Y, hipStream_t stream);

/*
 * The residual contraction of a transformer block with the next LayerNorm behind it, in one launch:
 * replaces QuantizeLinear.forward of Attention.proj / Mlp.fc2 (quant_layers.py:495-499) + the residual add of
 * Block.forward (reference vit_model.py:202-208) + the following norm2 / next block's norm1 (vit_model.py:193,
 * 206-207) + the next layer's quantize_act (quant_layers.py:356-381), i.e. qvit_gemm(QVIT_EPI_F32_RESID) then
 * qvit_layernorm_quant_i8 on the same rows, with the same results.
 *   A .. ldc : as qvit_gemm with QVIT_EPI_F32_RESID (C += d_act d_wt acc + bias); N % 4 == 0, N <= 1024,
 *              M * ldc * 4 < 2^31.
 *   gamma, beta, eps, out_* , ln_table : the LayerNorm and the next quantizer, as qvit_layernorm_quant_i8
 *              (ln_table: its QVIT_EPI_I8 code table, nullable; used if valid and <= 2174 buckets).
 *   codes    : int8 [M][ldcodes], the LayerNorm codes of the updated rows, columns [N, kpad_codes) zero.
 *   counters : int32 [ceil(M / 128)] (one per 128-row block), scratch: the call zeroes it on `stream` before
 *              the launch, so no state carries over between launches; it must not be shared with a launch
 *              running concurrently on another stream.
 * The last of a row block's npad / 256 workgroups runs the LayerNorm of its rows; the residual rows are written
 * through (sc1) and read back with sc1 loads behind an agent-scope counter.
 */
int qvit_gemm_resid_ln(const int8_t* A, int64_t M, int64_t K, int64_t lda, const void* Wp, int wfmt,
                       int64_t N, int64_t npad, const float* d_act, const float* d_wt, const float* bias,
                       float* C, int64_t ldc, const float* gamma, const float* beta, float eps,
                       int out_qtype, const float* out_d, const float* out_qm, const float* out_t,
                       int out_levels, const void* ln_table, int8_t* codes, int64_t ldcodes,
                       int64_t kpad_codes, int32_t* counters, hipStream_t stream);

/*
 * Code table for the int8 epilogues (optional `epi_table` of qvit_gemm; 16-byte aligned,
 * QVIT_EPI_TABLE_BYTES(nb) bytes). The output code of QVIT_EPI_I8 / QVIT_EPI_I8_GELU is a piecewise
 * constant function of the pre-activation v = d_act d_wt acc + bias; the table holds it exactly over
 * nb uniform buckets of width w starting at v_lo (w must be below the smallest distance between two
 * of its change points, and the function constant beyond both ends). The device builds it by bisection
 * with the epilogue's own arithmetic and validates it; qvit_gemm uses it only if valid (else the
 * direct per-element evaluation runs), so results never depend on the choice of (v_lo, w, nb).
 */
#define QVIT_EPI_TABLE_MAX_NB 3800
#define QVIT_EPI_TABLE_BYTES(nb) ((16 + 8 * (nb) + 1023) / 1024 * 1024)  /* staged in 1-KiB pieces */
int qvit_epi_table_build(int epilogue, int out_qtype, const float* out_d, const float* out_qm,
                         const float* out_t, int out_levels, float v_lo, float w, int64_t nb,
                         void* table, hipStream_t stream);

/*
 * Attention core between the qkv and proj QuantizeLinear layers of Attention.forward
 * (reference vit_model.py:133-149): out = softmax((q @ k^T) * scale) @ v per (image, head),
 * written as [B*N][ldo] with column h*head_dim + d (the reference's transpose(1, 2).reshape).
 *   qkv      : fp32 [B*N][ldq], row = [q | k | v], each H*head_dim wide (qkv.reshape(B,N,3,H,hd)).
 *   head_dim : 64 (the only supported head size); scale: qk_scale (head_dim ** -0.5 by default).
 *   in_scale : power of two applied to q, k, v before their fp16 hi/lo split (keeps |x * in_scale|
 *              < 65504; undone exactly), 1.0 for ordinary activations.
 *   out_mode : QVIT_ATT_F32 -> fp32 out (ldo % 4 == 0, 16-B aligned);
 *              QVIT_ATT_I8  -> int8 codes of the next layer's activation quantizer
 *              (out_qtype, out_d, out_qm, out_t, out_levels as in qvit_gemm), ldo % 4 == 0.
 * fp32 matmuls are formed from fp16 hi/lo products with fp32 accumulation (~2^-22 relative error).
 */
/*
 * UltraNet (reference `4-bit quantization/`: quant_ultra.py:8-91, mymodel.py:23-144).
 * Weight codes k_w = rne(tanh(w)/max|tanh(w)| * (2^(w_bit-1)-1)) (weight_quantize_fn, quant_ultra.py:30-56),
 * activation codes k_a = rne(clamp(x,0,1) * (2^a_bit-1)) (activation_quantize_fn :59-73), so a
 * Conv2d_Q on codes is the int32 contraction acc with value acc / den, den = (2^(w_bit-1)-1)(2^a_bit-1).
 *
 * qvit_ultra_weight_codes: w fp32 [cout][cin][ks][ks] -> codes int8 [cout_pad][kpad] in K order
 *   (ky, kx, c), zero padded; values (nullable) = the reference's fake-quant weight k_w/(2^(w_bit-1)-1)
 *   in w's own layout; workspace = device unsigned[1] (max |tanh| scratch).
 * qvit_ultra_bn_fold: BatchNorm2d eval constants alpha = gamma/sqrt(var+eps), shift = beta - mean*alpha.
 * qvit_ultra_conv0: layer 0 (mymodel.py:73-77): float image NCHW [B][3][H][W] -> conv 3x3 pad 1 with the
 *   fake-quant weights (wvals [16][3][3][3], the `values` output of qvit_ultra_weight_codes)
 *   -> BN (alpha, shift) -> activation quantizer -> MaxPool2d(2,2);
 *   out = codes NHWC [B][H/2][W/2][16], 16-byte aligned.
 * qvit_ultra_conv: layers 1..8: in = codes NHWC [B][H][W][cin] (16-B aligned), ks in {1, 3} (pad ks/2),
 *   wcodes [round_up(cout,16)][kpad] from qvit_ultra_weight_codes; mode QVIT_ULTRA_* ; out NHWC with
 *   row (pixel) pitch ldo: codes (ldo % 4 == 0) or fp32 (the 1x1 head, shift = its bias).
 *   Supported (cin, ks, cout): (16,3,17..32), (32,3,49..64), (64,3,49..64), (64,1,33..48).
 * qvit_yolo_decode: YOLOLayer eval decode (mymodel.py:47-60) of the head output NHWC [B][ny][nx][ldh]
 *   (channel a*no + o) with anchors (device float [na][2]) and stride -> io and p, both
 *   [B][na][ny][nx][no] (io.view(bs, -1, no) is the reference's first output).
 */
int qvit_ultra_weight_codes(const float* w, int64_t cout, int64_t cin, int64_t ks, int w_bit,
                            int8_t* codes, int64_t kpad, int64_t cout_pad, float* values,
                            unsigned* workspace, hipStream_t stream);
int qvit_ultra_bn_fold(const float* gamma, const float* beta, const float* mean, const float* var,
                       float eps, int64_t n, float* alpha, float* shift, hipStream_t stream);
int qvit_ultra_conv0(const float* img, int64_t B, int64_t H, int64_t W, const float* wvals,
                     const float* alpha, const float* shift, int a_bit, int8_t* out, hipStream_t stream);
int qvit_ultra_conv(const int8_t* in, int64_t B, int64_t H, int64_t W, int64_t cin, int64_t ks,
                    const int8_t* wcodes, int64_t kpad, int64_t cout, int w_bit, int a_bit,
                    const float* alpha, const float* shift, int mode, void* out, int64_t ldo,
                    hipStream_t stream);
/*
 * qvit_ultra_tail: UltraNetQua.layers.16-28 (mymodel.py:104-124: four Conv2d_Q 64 -> 64 3x3 + BatchNorm2d +
 *   activation_quantize_fn blocks, then the 1x1 Conv2d_Q head with bias) in one launch, one workgroup per image
 *   with the maps resident in LDS. Same results as qvit_ultra_conv(QVIT_ULTRA_CODES) four times and
 *   qvit_ultra_conv(QVIT_ULTRA_F32) once, bit for bit.
 *   in      : codes NHWC [B][H][W][64], H, W <= 26 (UltraNet @416: 26 x 26), 16-byte aligned.
 *   wcodes, alpha, shift : HOST arrays of 4 device pointers (layers 4..7): weight codes [64][kpad] in K order
 *             (ky, kx, c) (qvit_ultra_weight_codes, kpad >= 576, % 16), BN alpha / shift [64] (qvit_ultra_bn_fold).
 *   hcodes  : head codes [48][hkpad] (hkpad >= 64); hbias device float[hout], hout <= 48.
 *   out     : fp32 NHWC [B][H][W][ldo], channels < hout written (io == NULL), or
 *   anchors, na, no, stride, io, p : with io != NULL the YOLOLayer decode of qvit_yolo_decode is applied in the
 *             kernel instead (hout == na * no; io, p [B][na][H][W][no]; out unused and may be NULL).
 */
int qvit_ultra_tail(const int8_t* in, int64_t B, int64_t H, int64_t W, const int8_t* const* wcodes, int64_t kpad,
                    const float* const* alpha, const float* const* shift, const int8_t* hcodes, int64_t hkpad,
                    const float* hbias, int64_t hout, int w_bit, int a_bit, float* out, int64_t ldo,
                    const float* anchors, int64_t na, int64_t no, float stride, float* io, float* p,
                    hipStream_t stream);
/*
 * UltraNet integer deploy (reference `4-bit quantization/`: quantization.py:24-31,68-89,
 * qnn_param_reader.py:58-85, ultranet_param_gen.py:14-22 — the FPGA flow's integer parameters):
 *   code = clamp(round((acc * inc_q[o] + bias_q[o]) / 2^S), 0, 2^out_bit - 1), round half up, 64-bit
 *   intermediate, S = w_bit - 1 + in_bit + l_shift; inc_q / bias_q from bn_act_quantize_int (host side).
 *   Replaces the accelerator's conv + BN + activation stage (its HLS source is absent from the reference;
 *   the rounding shown is the float path's round(), restated in integers: parity unpinned beyond it).
 * qvit_ultra_conv0_int: layer 0 on uint8 pixels NCHW [B][3][H][W] (in_bit 8), weight codes [16][3][3][3]
 *   (reference layout, weight_quantize_int) -> 2x2 max-pooled codes NHWC [B][H/2][W/2][16] (16-B aligned).
 * qvit_ultra_conv_int: layers 1..7 as qvit_ultra_conv (same input / weight layouts and shapes, 3x3 only)
 *   with the integer threshold; pool != 0 adds MaxPool2d(2, 2) on the codes.
 */
int qvit_ultra_conv0_int(const uint8_t* img, int64_t B, int64_t H, int64_t W, const int8_t* wcodes,
                         const int32_t* inc, const int32_t* bias, int shift_bits, int out_bit, int8_t* out,
                         hipStream_t stream);
int qvit_ultra_conv_int(const int8_t* in, int64_t B, int64_t H, int64_t W, int64_t cin, int64_t ks,
                        const int8_t* wcodes, int64_t kpad, int64_t cout, const int32_t* inc, const int32_t* bias,
                        int shift_bits, int out_bit, int pool, int8_t* out, int64_t ldo, hipStream_t stream);
int qvit_yolo_decode(const float* head, int64_t B, int64_t ny, int64_t nx, int64_t na, int64_t no,
                     int64_t ldh, const float* anchors, float stride, float* io, float* p,
                     hipStream_t stream);

int qvit_attention(const float* qkv, int64_t B, int64_t N, int64_t H, int64_t head_dim, int64_t ldq,
                   float scale, float in_scale, int out_mode, void* out, int64_t ldo,
                   int out_qtype, const float* out_d, const float* out_qm, const float* out_t,
                   int out_levels, hipStream_t stream);

/*
 * The qkv projection feeding qvit_attention_split (fused block path; replaces the fp32 qkv of
 * Attention.forward, vit_model.py:130-137, with the operand form the attention kernel consumes).
 * The value x = d_act d_wt acc + bias[n] is computed exactly as QVIT_EPI_F32 does, scaled by the power
 * of two in_scale and split into fp16 hi = f16(x s), lo = f16(x s - hi), stored head-major:
 *   qkv_hi / qkv_lo : fp16 [B][N / 64][seq][64], B = M / seq, plane p = n / 64 (q heads, k heads,
 *                     v heads), element (b, p, t, n % 64) for row m = b seq + t; 16-B aligned.
 * A, Wp, d_act, d_wt, bias as qvit_gemm; N % 64 == 0, M % seq == 0.
 */
int qvit_gemm_qkv_split(const int8_t* A, int64_t M, int64_t K, int64_t lda,
                        const void* Wp, int wfmt, int64_t N, int64_t npad,
                        const float* d_act, const float* d_wt, const float* bias,
                        int64_t seq, float in_scale, void* qkv_hi, void* qkv_lo, hipStream_t stream);

/*
 * qvit_attention on the split operands of qvit_gemm_qkv_split (planes [B][3H][N][64], in_scale the
 * same power of two): identical arithmetic; K/V blocks stream into LDS by DMA with no conversion.
 * epi_table (QVIT_ATT_I8 only, nullable): a qvit_epi_table_build table with QVIT_EPI_I8 semantics for
 * the output quantizer (<= 2046 buckets; used only if valid, results never depend on it).
 */
int qvit_attention_split(const void* qkv_hi, const void* qkv_lo, int64_t B, int64_t N, int64_t H,
                         int64_t head_dim, float scale, float in_scale, int out_mode, void* out,
                         int64_t ldo, int out_qtype, const float* out_d, const float* out_qm,
                         const float* out_t, int out_levels, const void* epi_table, hipStream_t stream);

/*
 * Fused qkv projection + attention core (vit_model.py:130-152) for the fused block: the qkv
 * QuantizeLinear (qvit_gemm_qkv_split semantics: d_act d_wt acc + bias, scaled by in_scale, split to
 * fp16 hi/lo) and qvit_attention_split in one kernel, q/k/v never written to HBM.
 *   A    : activation codes [B*N][lda] (K valid columns, K % 256 == 0, K <= 65536), N <= 208 tokens, H*64 <= 768;
 *   Wp   : the qkv layer's packed int4 weights (qvit_pack_weight, wfmt QVIT_W4, npad rows), bias [npad];
 *   out  : as qvit_attention_split (QVIT_ATT_F32 / QVIT_ATT_I8 + optional code table epi_table).
 * The dims of each q.k sum are added in a different order than in qvit_attention_split (fp32-level
 * differences only).
 */
int qvit_qkv_attention(const int8_t* A, int64_t B, int64_t N, int64_t K, int64_t lda, const void* Wp,
                       int wfmt, int64_t npad, const float* d_act, const float* d_wt, const float* bias,
                       int64_t H, int64_t head_dim, float scale, float in_scale, int out_mode, void* out,
                       int64_t ldo, int out_qtype, const float* out_d, const float* out_qm,
                       const float* out_t, int out_levels, const void* epi_table, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* QVIT_HIP_H */
