// magpie_oracle — CPU restatement of the reference's decode path and nano-codec.
//
// *** TEST INFRASTRUCTURE. *** Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load this library, and only as the checker / the timed CPU
// baseline. The product (libmagpie_hip.so) never links or calls it.
//
// Parity status: the reference's arithmetic lives in ggml (unpinned, absent here),
// its weights and golden tensors are absent. This oracle is
// pinned only by the weight-independent known answers the reference holds (the FSQ
// tables of tests/test_codec_fsq.cpp:41-74, the codec shape progression of
// docs/CODEC_ARCHITECTURE.md:186-196, token-id constants of magpie.h:70-73) —
// everything else is "parity unpinned" against real ggml. See DESIGN.md §Oracle.
#ifndef MAGPIE_ORACLE_H
#define MAGPIE_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_model orc_model;
typedef struct orc_codec orc_codec;

// acc64=1: every dot/LN/softmax accumulates in double, tensors stored f32 (the
// parity judge). acc64=0: f32 accumulation in 8 SIMD lanes (ggml-CPU-like speed;
// used for the CPU baseline timing). gelu_f16=1 applies ggml-CPU's fp16 GELU table
// semantics (A.7, assumed). n_threads<=0 keeps the OpenMP default.
void orc_set_mode(int acc64, int gelu_f16, int n_threads);

orc_model *orc_load(const char *gguf_path);
// Weight mode 1 = this build's bf16 decode path (no reference file format: the
// reference converter writes F32/F16/Q8_0/Q4_0): in decode steps (BOS included)
// the projections qkv/o/ff1/ff2 of every decoder layer, the LT layer's FFN
// (ff1/ff2) and the 8 LT output projections use bf16-rounded weights and
// bf16-rounded input activations (ggml's BF16 mul_mat semantics), f32/f64
// accumulation. Encoder, prefill, cross-attention, LT in_proj and the LT layer's
// attention (q|k|v, o_net: the build computes it through load-time f32 tables)
// stay f32. 0 = as stored (Q8_0/F16
// tensors dequantised to f32, f32 activations). Weight mode 2 = ggml's Q8_0
// mul_mat for every Q8_0 tensor of the file, everywhere it is used (encoder,
// XA K/V, prefill, decode steps, LT): the activation row is quantised to Q8_0
// (quantize_row_q8_0_ref), per-block integer dots scaled by d_w*d_a (SURVEY A.7,
// assumed); Q4_0 tensors the same way with q - 8 (vec_dot_q4_0_q8_0); -1 if the
// file has no Q8_0 / Q4_0 tensor. Weight mode 3 = ggml's F16 mul_mat for every F16
// tensor of the file, everywhere (encoder incl. its k=3 conv FFN, XA q/kv/o,
// prefill, decode steps, LT in_proj/layer/heads): src1 rounded to f16, products
// exact, f32/f64 accumulation; -1 if the file has no F16 tensor.
int orc_set_weight_mode(orc_model *m, int mode);
/* SA cache rounded to bf16 on append (MP_KV_BF16); process-wide, default off. */
void orc_set_kv_bf16(int on);
void orc_free(orc_model *m);
int orc_dec_layers(const orc_model *m);

// magpie_synthesize_codes_graph_reuse (magpie.cpp:4063-4432) at temperature 0.
// Returns n_frames (>=0) or <0 on error. codes_out: [max_steps][8] frame-major.
// margins_out (nullable): [max_steps][8] top1-top2 gap of the masked logits.
// hidden_out (nullable): [max_steps+1][768] decoder hidden after every step (BOS first).
// timing_out (nullable): [0]=preamble ms (encoder+XA+prefill), [1]=decode ms (BOS+loop).
int orc_synthesize(orc_model *m, const int32_t *tokens, int n_tokens, int speaker_id, int max_steps,
                   int ignore_eos, int32_t *codes_out, float *margins_out, float *hidden_out,
                   double *timing_out);

// Same with the reference's temperature/top-k sampling (sample_top_k,
// magpie.cpp:1072-1109). Draws use this repo's counter-based stream
// u(seed, stream, step, codebook) (see magpie_oracle.c); stream = batch slot.
// margins_out then holds min(argmax gap, distance of u to the chosen interval).
// emit_eos = 1: the EOS frame is emitted too (the streaming loop, magpie.cpp:4800-4806).
int orc_synthesize_ex(orc_model *m, const int32_t *tokens, int n_tokens, int speaker_id, int max_steps,
                      int ignore_eos, float temperature, int top_k, uint64_t seed, int stream, int emit_eos,
                      int32_t *codes_out, float *margins_out, float *hidden_out, double *timing_out);

// Teacher-forced run of the same loop for exactly n_frames frames: at every
// codebook decision the oracle records ITS OWN pick (codes_out) and margin, then
// continues with forced[step][cb] (the codes of the run under test, [n_frames][8]),
// so every decision of a GPU run is checked against the oracle, not only those
// before the first near-tie. EOS does not stop the loop (the forced run decides).
int orc_synthesize_forced(orc_model *m, const int32_t *tokens, int n_tokens, int speaker_id, int n_frames,
                          int ignore_eos, float temperature, int top_k, uint64_t seed, int stream,
                          const int32_t *forced, int32_t *codes_out, float *margins_out, float *hidden_out);

// magpie_local_transformer_sample_all (magpie.cpp:1113-1317) for one hidden[768]:
// sampled[8], argmax[8] (nullable), margins[8] (nullable).
int orc_lt_sample(orc_model *m, const float *hidden, float temperature, int top_k, int forbid_eos, uint64_t seed,
                  int stream, int step, int32_t *sampled, int32_t *argmax, float *margins);

// Component entry points used by unit tests.
float orc_draw_u(uint64_t seed, int stream, int step, int cb);
int orc_sample_top_k(const float *logits, int n, float temperature, int top_k, float u, float *margin);
int orc_encode(orc_model *m, const int32_t *tokens, int n_tokens, float *enc_out /*[T][768]*/);
// ggml Q8_0 mul_mat of raw GGUF Q8_0 blocks ([N][K], 34 B per 32 weights) with x[K].
int orc_q8_matvec(const uint8_t *blocks, int N, int K, const float *x, float *y);
// ggml's quantize_row_q8_0 (the oracle's restatement, the same function its Q8_0
// mul_mat uses): x[K] -> q[K] int8, d[K/32] (fp16 values as f32).
int orc_q8_quantize_row(const float *x, int K, int8_t *q, float *d);
// The exact integer block dots of raw GGUF blocks (type 8 = Q8_0, 2 = Q4_0 as q - 8)
// [N][K] with one quantised activation row aq[K]: dots[N][K/32].
int orc_qblock_dots(const uint8_t *blocks, int type, int N, int K, const int8_t *aq, int32_t *dots);

orc_codec *orc_codec_load(const char *gguf_path);
void orc_codec_free(orc_codec *c);
// magpie_codec_decode (nano-codec.cpp:758-845). codes: [8][n_frames] cb-major.
// f16_operands=1 rounds conv_1d operands to fp16 as ggml's F16 im2col does (A.7).
int orc_codec_decode(orc_codec *c, const int32_t *codes, int n_frames, float *audio_out, int f16_operands);
// Residual-conv rounding order: 0 (default) = the reference's (sum + b) + x
// (nano-codec.cpp:454-462, 568-599); 1 = (x + sum) + b, the order this build's kernels use
// (accumulators initialised with the residual, bias after; mp_codec.hip MP_RESINIT).
void orc_codec_set_resinit(orc_codec *c, int on);
// fsq_dequantize_cpu (nano-codec.cpp:721-752): latent [32][n_frames] (time fastest).
void orc_fsq(const int32_t *codes, int n_frames, float *latent);

#ifdef __cplusplus
}
#endif
#endif
