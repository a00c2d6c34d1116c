/*
 * magpie_hip.h — the C-ABI boundary of the MI355X-native decode path.
 *
 * Plain C, plain pointers and sizes, no torch/ggml types. Every entry point
 * replaces a piece of the reference's ggml-backed path in m1el/magpie-tts.cpp;
 * the reference symbol each one stands in for is cited next to it (file:line
 * under /root/reference). The C++ drop-in API (include/magpie.h) is a thin layer
 * over these functions; Python (ctypes) and other FFIs bind them directly (see
 * INTEGRATION.md).
 *
 * Conventions (mirroring the reference's error behaviour):
 *   - every int-returning call returns MP_OK (0) or a negative MP_ERR_* code and
 *     leaves a message for mp_hip_error(); the reference returns nullptr / an
 *     empty vector / -1 and prints to stderr.
 *   - all buffers are caller-owned host memory; one mp_dev == one GPU, used by one
 *     host thread at a time (the reference context is not thread-safe either,
 *     magpie.cpp:1129, 2364).
 */
#ifndef MAGPIE_HIP_H
#define MAGPIE_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MP_OK 0
#define MP_ERR_ARG (-1)
#define MP_ERR_HIP (-2)
#define MP_ERR_IO (-3)
#define MP_ERR_FORMAT (-4)
#define MP_ERR_STATE (-5)
#define MP_ERR_UNSUPPORTED (-6)

typedef struct mp_dev mp_dev;
typedef struct mp_codec mp_codec;

/* Inference parameters. The reference carries them on magpie_context
 * (temperature/top_k/speaker_id, magpie.h:298-306) and hparams.max_dec_steps
 * (magpie.h:76). */
typedef struct mp_params {
    float temperature;  /* < 0.01 => greedy argmax (magpie.cpp:1263-1264) */
    int top_k;          /* top-k of sample_top_k (magpie.cpp:1072-1109) */
    int max_dec_steps;  /* frame budget per utterance (magpie.h:76); <= 0 => 500 */
    int ignore_eos;     /* 1: EOS masked at every step (fixed-length bench mode) */
    uint64_t seed;      /* sampling RNG seed (reference: unseeded static mt19937, magpie.cpp:1129) */
    int trace_hidden;   /* 1: keep the decoder hidden state of every step (parity tests) */
    int stream_base;    /* draw stream of utterance b = stream_base + b (a sentence run alone with
                           stream_base = i draws exactly what slot i of a batch draws) */
    int emit_eos_frame; /* 1: the EOS frame's codes are emitted too, as the streaming loop does
                           (magpie.cpp:4800-4806); 0: dropped, as graph_reuse does (4349-4352) */
} mp_params;

typedef struct mp_timing {
    double preamble_ms;  /* encoder + XA K/V + 110-frame prefill (magpie.cpp:4081-4238) */
    double decode_ms;    /* BOS step + autoregressive loop (gen_time, magpie.cpp:4265,4409) */
    int frames_total;    /* frames produced over all utterances */
    int iterations;      /* decode iterations (graph replays) executed */
    double first_audio_ms; /* mp_hip_decode_stream: decode start -> first audio callback */
} mp_timing;

/* --- device + weights ---------------------------------------------------- */
int mp_hip_device_count(int *n);
/* the file of the HIP runtime this library's calls are bound to (dladdr of
 * hipGetDeviceCount as resolved from here): a process that also loads torch's
 * bundled copy must still run the kernels on /opt/rocm's (bench.py loads this
 * library first; tests/test_dist_cpu.py) */
const char *mp_hip_runtime_path(void);
/* replaces init_backend / ggml_backend_cuda_init (magpie.cpp:14-67) */
int mp_hip_init(int device, mp_dev **out);
/* replaces gguf_init_from_file + read_hparams + create_tensors + load_tensor_data
 * (magpie.cpp:73-121, 572-718, 781-880): parses the GGUF (F32/F16/Q8_0 tensors,
 * same names and layout) and uploads resident weights once. */
int mp_hip_load_model(mp_dev *dev, const char *gguf_path);
/* Weight modes of mp_hip_load_model_ex. AS_STORED streams the GGUF's weights
 * as f32 (F16/BF16/Q8_0 tensors are widened at load). BF16 additionally repacks
 * the decode-step projections (decoder qkv/o/ff1/ff2, LT FFN, LT heads) into
 * bf16 (MFMA fragments for the decoder and heads): half the bytes per frame,
 * activations rounded to bf16 like ggml's BF16 mul_mat; batches up to 16
 * (BASELINE configs 3-4). The preamble, cross-attention, LT in_proj and the LT
 * layer's attention (through load-time f32 tables, as AS_STORED computes it)
 * stay f32. No reference counterpart (the
 * reference converter writes F32/F16/Q8_0/Q4_0, convert_magpie_to_gguf.py:197-206). */
#define MP_WEIGHTS_AS_STORED 0
#define MP_WEIGHTS_BF16 1
/* Q8: the GGUF's Q8_0 tensors (the reference converter's Q8 file quantises the
 * attention, cross-attention and LT projections, convert_magpie_to_gguf.py:155-176)
 * stay int8 in HBM and are multiplied the way ggml multiplies Q8_0:
 * every activation row is quantised to Q8_0 (quantize_row_q8_0_ref) and each
 * 32-block contributes its exact integer dot times d_w*d_a — in the encoder, the
 * XA K/V precompute, the prefill, every decode step and the LT. F32 tensors (the
 * pos_ff convs) keep the f32 path. Batches up to 16 when every decode projection is
 * quantised (the reference converter's files), else 8 (mp_hip_max_batch). MP_ERR_UNSUPPORTED for a file
 * without Q8_0 tensors (BASELINE config 5). A Q4_0 file (convert_magpie_to_gguf.py:
 * 107-138) runs in this mode too: its blocks are repacked losslessly to int8 q - 8
 * with the same fp16 scale, so the same kernels compute ggml's vec_dot_q4_0_q8_0. */
#define MP_WEIGHTS_Q8 2
/* F16: an F16 GGUF (the converter's F16 file: the same projections plus the pos_ff
 * convs, convert_magpie_to_gguf.py:311-327) computed as ggml computes F16 mul_mat:
 * every projection's activation rounded to f16, products exact, f32 accumulation.
 * The decode-step projections (decoder qkv/o/ff1/ff2, LT in_proj/layer/heads) stream
 * their f16 weights on f16 MFMA (2 B/param); the preamble GEMMs round their operand;
 * the fused cross-attention rounds its query (LN(x)) to f16, and applies o_net to the
 * unrounded attention output (reassociated). Batches up to 16.
 * MP_ERR_UNSUPPORTED for a file whose projections are not F16. */
#define MP_WEIGHTS_F16 3
int mp_hip_load_model_ex(mp_dev *dev, const char *gguf_path, int weight_mode);
/* SA (self-attention) cache element type, applied from the next mp_hip_begin_batch.
 * F32 is the reference's graph-reuse cache (magpie.cpp:3313-3376, f32 K/V tensors).
 * BF16 stores every K and V row rounded to bf16 (round to nearest even) when it is
 * appended, in the 110-frame prefill and every decode step, and every attention
 * (prefill and decode) reads the rounded rows: half the cache bytes per step, which
 * at batch 16 are about as many as the bf16 weights. No reference counterpart; the
 * oracle's kv_bf16 mode restates it. Any weight mode. */
#define MP_KV_F32 0
#define MP_KV_BF16 1
int mp_hip_set_kv_mode(mp_dev *dev, int kv_mode);
/* Cross-attention form of the decode step, applied from the next mp_hip_begin_batch.
 * REASSOC: x += sum_t softmax_t(K'_t . LN(x)) V'_t with K' = W_q^T K, V' = W_o V
 * precomputed per utterance (reads 6 KB per text token and layer; fused into the
 * O-projection launch). DIRECT: q = W_q LN(x), attention over K, V, W_o (reads 1 KB
 * per text token and layer + q_net / o_net, 0.79 MB; two launches), the order
 * magpie.cpp:1713-1767 computes. AUTO (default): DIRECT when the batch's longest text
 * exceeds MP_XA_DIRECT_T tokens (where it reads fewer bytes), else REASSOC. The F16
 * weight mode is always REASSOC; the Q8_0 mode always direct (its quantised q_net /
 * o_net). A batch reproduces its utterances run alone when both use the same form. */
#define MP_XA_AUTO 0
#define MP_XA_REASSOC 1
#define MP_XA_DIRECT 2
#define MP_XA_DIRECT_T 160
int mp_hip_set_xa_mode(mp_dev *dev, int xa_mode);
int mp_hip_weight_mode(mp_dev *dev);
/* the largest batch mp_hip_begin_batch accepts for the loaded model: 16 in the
 * bf16 / F16 modes and for a Q8_0 / Q4_0 file whose decode projections are all
 * quantised, else 8 (negative MP_ERR_* without a model) */
int mp_hip_max_batch(mp_dev *dev);
int mp_hip_model_info(mp_dev *dev, int *dec_layers, int *enc_layers, size_t *weight_bytes);
/* replaces magpie_free (magpie.cpp:882-910) */
void mp_hip_free(mp_dev *dev);
const char *mp_hip_error(mp_dev *dev);

/* --- synthesis ------------------------------------------------------------ */
/* Per-utterance preamble for B independent utterances (1 <= B <= mp_hip_max_batch:
 * 16 in the bf16 / F16 modes and for a fully quantised Q8_0 / Q4_0 file, else 8): text encoder
 * (magpie_encode_text, magpie.cpp:2284-2374), cross-attention K/V
 * (magpie.cpp:4098-4136), baked speaker context + 110-frame prefill
 * (magpie.cpp:4138-4238). tokens: [B][tmax] row-major (padding ignored),
 * n_tokens: [B], speaker: [B] (0..4). */
int mp_hip_begin_batch(mp_dev *dev, const int32_t *tokens, const int32_t *n_tokens, const int32_t *speaker, int B,
                       int tmax, const mp_params *params);
/* The frame loop of magpie_synthesize_codes_graph_reuse (magpie.cpp:4245-4407)
 * for the whole batch: one hipGraph replay per frame. codes_out:
 * [B][max_dec_steps][8] frame-major (BOS excluded, as magpie.cpp:4416-4420);
 * n_frames: [B]. */
int mp_hip_decode(mp_dev *dev, int32_t *codes_out, int32_t *n_frames);
/* decoder hidden state after every step (BOS first): [B][max_dec_steps+1][768];
 * requires params.trace_hidden. */
int mp_hip_get_trace(mp_dev *dev, float *hidden);
/* magpie_encode_text (src/magpie.cpp:2284-2374): the text encoder alone (embedding +
 * positions, the encoder layers, final LN) for one utterance, into a private device
 * workspace; enc_out: host [n_tokens][768]. A batch in progress (mp_hip_begin_batch /
 * mp_hip_decode) is not touched. Returns MP_OK or a negative MP_ERR_*. */
int mp_hip_encode_text(mp_dev *dev, const int32_t *tokens, int n_tokens, float *enc_out);

/* Diagnostics: copy a per-batch device buffer to host after mp_hip_begin_batch /
 * mp_hip_decode. name: "enc_out" [NB][Tmax][768] (magpie_encode_text's output),
 * "xak"/"xav" [NB][L][Tmax][128] (XA K/V, magpie.cpp:1663-1711), "kc"/"vc"
 * [NB][L][max_seq][768] (SA cache), "x" [NB][768] (residual stream). Writes at
 * most `bytes`; returns the buffer's size in bytes (host may be NULL to query),
 * or a negative MP_ERR_*. */
int64_t mp_hip_debug_buffer(mp_dev *dev, const char *name, void *host, int64_t bytes);

/* Streaming variant of mp_hip_decode (magpie_synthesize_sentence_streaming's
 * frame loop, magpie.cpp:4762-4838, for every utterance of the batch): every
 * frames_per_chunk frames (<= 0: 4, magpie.h:621) each utterance's new frames are
 * decoded by `codec` as one stateless chunk (decode_frames_to_audio,
 * magpie.cpp:4458-4476; the last chunk may be shorter) and passed to on_audio in
 * frame order; returning 0 stops that utterance (4820-4824). Once an utterance
 * has ended (EOS, max_dec_steps or stopped) on_audio(utt, NULL, 0, user) is called
 * once. codes_out / n_frames / total_samples may be NULL. */
typedef int (*mp_audio_cb)(int utterance, const float *samples, int n_samples, void *user);
int mp_hip_decode_stream(mp_dev *dev, mp_codec *codec, int frames_per_chunk, mp_audio_cb on_audio, void *user,
                         int32_t *codes_out, int32_t *n_frames, int64_t *total_samples);

/* magpie_local_transformer_sample_all (magpie.cpp:1113-1317) for one normalised
 * decoder hidden vector [768]: sampled[8] and argmax[8] codes. Independent of any
 * batch in flight. Draws use stream -1 and a per-device call counter as the step. */
int mp_hip_lt_sample(mp_dev *dev, const float *hidden, float temperature, int top_k, int forbid_eos, uint64_t seed,
                     int32_t *sampled, int32_t *argmax);
int mp_hip_get_timing(mp_dev *dev, mp_timing *t);

/* --- measurement ---------------------------------------------------------- */
/* Ops of the captured decode iteration (valid after mp_hip_decode). */
int mp_hip_num_ops(mp_dev *dev);
const char *mp_hip_op_name(mp_dev *dev, int op);
/* algorithmic HBM bytes one launch of `op` moves (weights + activations) */
double mp_hip_op_bytes(mp_dev *dev, int op);
/* Re-launch one op of the iteration `reps` times back to back on the decode
 * stream (same arguments as in the captured graph), one hipEvent pair around
 * the whole run; returns the mean per-launch time in us (kernel + dispatch gap). */
int mp_hip_time_op(mp_dev *dev, int op, int reps, float *avg_us);
/* In-situ per-op timing: run `iters` whole decode iterations with every kernel
 * launched directly (not from the graph), each launch bracketed by a hipEvent
 * pair on the decode stream, so every op sees the caches a real frame leaves it
 * (weights streamed by the ops before it). avg_us[op] = mean per launch of op
 * (mp_hip_num_ops entries). Continues from the batch's current state; after
 * every utterance is done the iteration recomputes the same frame. */
int mp_hip_profile_ops(mp_dev *dev, int iters, float *avg_us);
/* mp_hip_profile_ops plus, per op, the time of an EMPTY event pair recorded right
 * after it (pair_us, nullable): avg_us - pair_us estimates the launch's own
 * duration without the event-pair overhead. */
int mp_hip_profile_ops_ex(mp_dev *dev, int iters, float *avg_us, float *pair_us);
/* Per-op duration from in-kernel timestamps (first wave start to last wave end
 * after its stores, s_memrealtime), eager launches of whole iterations with no
 * event in the stream: the launch's own time in the decode's cache state. -1 for
 * an op whose kernel records no timestamps. */
int mp_hip_profile_ops_ts(mp_dev *dev, int iters, float *avg_us);
/* Per-op duration from the kernel dispatch's own begin/end timestamps
 * (hipExtLaunchKernel start/stop events: the interval rocprofv3's kernel trace
 * reports), eager launches of whole iterations in the decode's cache state. */
int mp_hip_profile_ops_kev(mp_dev *dev, int iters, float *avg_us);

/* --- text front end (host) ---------------------------------------------------- */
/* magpie_tokenizer_init + magpie_tokenize (magpie.cpp:124-495): vocabulary and
 * pronunciation dictionary from the GGUF strings magpie.tokenizer.vocab / .dict.
 * mp_tokenize returns the token count (writing at most cap ids) or < 0. */
typedef struct mp_tokenizer mp_tokenizer;
int mp_tokenizer_load(const char *gguf_path, mp_tokenizer **out);
int mp_tokenize(mp_tokenizer *tok, const char *text, int32_t *out, int cap);
void mp_tokenizer_free(mp_tokenizer *tok);
/* magpie_split_sentences (magpie.cpp:4439-4480): byte offset/length of each
 * sentence (at most cap written); returns the sentence count or < 0. */
int mp_split_sentences(const char *text, int32_t *offsets, int32_t *lengths, int cap);

/* --- nano-codec ----------------------------------------------------------- */
/* replaces magpie_codec_init / magpie_codec_load (nano-codec.cpp:205-352) */
int mp_hip_codec_init(int device, const char *gguf_path, mp_codec **out);
/* replaces magpie_codec_decode (nano-codec.cpp:758-845): codes [8][n_frames]
 * codebook-major, audio_out [n_frames * 1024] samples in [-1, 1]. */
int mp_hip_codec_decode(mp_codec *c, const int32_t *codes, int n_frames, float *audio_out);
/* n_chunks independent chunks of chunk_frames frames in one launch sequence
 * (the CLI decodes stateless 32-frame chunks, magpie-tts.cpp:181-206):
 * codes [n_chunks][8][chunk_frames], audio_out [n_chunks][chunk_frames * 1024]. */
int mp_hip_codec_decode_chunks(mp_codec *c, const int32_t *codes, int n_chunks, int chunk_frames, float *audio_out);
/* device time (hipEvents) of the last decode's kernel sequence, ms */
int mp_hip_codec_last_ms(mp_codec *c, float *ms);
void mp_hip_codec_free(mp_codec *c);
const char *mp_hip_codec_error(mp_codec *c);

#ifdef __cplusplus
}
#endif
#endif /* MAGPIE_HIP_H */
