// magpie.h — drop-in C++ API of the MI355X-native Magpie decode path.
//
// Same function names, argument meaning, ownership and error behaviour as the
// reference header (/root/reference/src/magpie.h) for the hot path named in
// BASELINE.json: model init/free, magpie_synthesize_codes_graph_reuse and its
// aliases, magpie_local_transformer_sample_all, and the nano-codec
// init/decode/free. ggml types are gone from the public structs; everything
// below is implemented over the C-ABI in magpie_hip.h (one HIP device per
// context, no multi-backend dispatch).
//
// Also provided: the streaming API (magpie.h:596-648) and the text
// front end / tokenizer (magpie.h:86-110). Out of scope: graph-builder entry
// points (magpie_build_*) and the CLI.
#ifndef MAGPIE_H
#define MAGPIE_H

#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "magpie_hip.h"

// magpie.h:24-29 — kept for source compatibility. CUDA and AUTO select the single
// HIP device path; CPU and Metal requests are refused (magpie_model_load returns
// false with a message on stderr, magpie_init_with_backend nullptr): there is no
// CPU fallback by design.
enum magpie_backend_type {
    MAGPIE_BACKEND_CPU = 0,
    MAGPIE_BACKEND_CUDA = 1,
    MAGPIE_BACKEND_METAL = 2,
    MAGPIE_BACKEND_AUTO = 3,
};

// magpie.h:35-80 (same fields and defaults)
struct magpie_hparams {
    int32_t d_model = 768;
    int32_t d_ffn = 3072;
    int32_t d_head = 64;
    int32_t enc_layers = 6;
    int32_t enc_heads = 12;
    int32_t enc_kernel = 3;
    int32_t dec_layers = 12;
    int32_t dec_sa_heads = 12;
    int32_t dec_xa_heads = 1;
    int32_t dec_xa_d_head = 128;
    int32_t dec_kernel = 1;
    int32_t lt_dim = 256;
    int32_t lt_ffn_dim = 1024;
    int32_t lt_layers = 1;
    int32_t lt_heads = 1;
    int32_t text_vocab_size = 2380;
    int32_t num_codebooks = 8;
    int32_t codebook_size = 2016;
    int32_t vocab_per_cb = 2024;
    int32_t num_speakers = 5;
    int32_t context_frames = 110;
    int32_t text_bos_id = 2378;
    int32_t text_eos_id = 2379;
    int32_t audio_bos_id = 2016;
    int32_t audio_eos_id = 2017;
    int32_t max_dec_steps = 500;
    int32_t sample_rate = 22050;
    float eps = 1e-5f;
};

// magpie.h:86-104 (same fields)
struct magpie_tokenizer {
    std::vector<std::string> vocab;               // token id -> token string
    std::map<std::string, int32_t> token_to_id;   // token string -> id
    std::map<std::string, std::string> dict;      // word -> IPA pronunciation
    int32_t pad_id = -1;
    int32_t oov_id = -1;
    int32_t space_id = -1;
    int32_t bos_id = -1;
    int32_t eos_id = -1;
    bool loaded = false;
};
// magpie.h:107: magpie_tokenizer_init from an open GGUF's metadata (strings
// magpie.tokenizer.vocab / .dict, ids magpie.tokenizer.*). gguf_context is this
// library's own opaque, ggml-free GGUF handle: magpie_gguf_open / magpie_gguf_close.
struct gguf_context;
struct gguf_context *magpie_gguf_open(const char *gguf_path);  // nullptr + stderr on failure
void magpie_gguf_close(struct gguf_context *gguf_ctx);
bool magpie_tokenizer_init(magpie_tokenizer *tok, struct gguf_context *gguf_ctx);
// the same from a GGUF path (open, init, close)
bool magpie_tokenizer_load(magpie_tokenizer *tok, const char *gguf_path);
// magpie.h:110: normalise, lower-case, dictionary/IPA or letter fallback, BOS..EOS
std::vector<int32_t> magpie_tokenize(const magpie_tokenizer *tok, const std::string &text);

struct magpie_model {
    magpie_hparams hparams;
    magpie_tokenizer tokenizer;  // loaded by magpie_init when the GGUF carries one
    magpie_backend_type backend_type = MAGPIE_BACKEND_CUDA;
    mp_dev *dev = nullptr;  // resident weights + device state (replaces ggml ctx/buffers)
};

// magpie.h:265-287 — the per-call generation state, host side. The KV caches and
// the graph allocator live on the device (mp_dev) and are not exposed; the
// fields a caller can read are filled by the single-utterance synthesis calls:
// the last call's frames (frame-major, as returned) and its encoder output
// ([enc_seq_len][d_model], magpie_encode_text's copy, magpie.cpp:2364-2367).
struct magpie_state {
    std::vector<int32_t> generated_codes;
    int32_t n_generated_frames = 0;
    std::vector<float> encoder_output;
    int32_t enc_seq_len = 0;
    void reset() {
        generated_codes.clear();
        n_generated_frames = 0;
        encoder_output.clear();
        enc_seq_len = 0;
    }
};

// magpie.h:293-307 — same members, names and defaults; public inference settings
// kept as plain fields.
struct magpie_context {
    magpie_model model;
    magpie_state state;
    int n_threads;  // accepted, unused (the reference never applies it either, magpie.h:298)
    float temperature;
    int top_k;
    int speaker_id;
    struct magpie_codec *codec;
    // added: the reference's sampler is an unseeded static mt19937 (magpie.cpp:1129);
    // here every draw is u(seed, stream, step, codebook)
    uint64_t seed;
    // added: magpie_synthesize_streaming runs up to this many sentences as one device
    // batch (audio still delivered in sentence order, identical samples); 1 = one by one
    int max_parallel_sentences;
    magpie_context()
        : n_threads(4), temperature(0.7f), top_k(80), speaker_id(0), codec(nullptr), seed(0),
          max_parallel_sentences(8) {}
};

// magpie.h:310-313
struct magpie_sample_result {
    std::vector<int32_t> sampled_codes;
    std::vector<int32_t> argmax_codes;
};

// magpie.h:655-678 (codec hyperparameters, same defaults)
struct magpie_codec_hparams {
    int32_t sample_rate = 22050;
    int32_t num_codebooks = 8;
    int32_t codebook_size = 2016;
    int32_t hop_length = 1024;
    int32_t latent_dim = 32;
    int32_t fsq_levels[4] = {8, 7, 6, 6};
    int32_t pre_conv_kernel = 7;
    int32_t post_conv_kernel = 3;
    int32_t base_channels = 864;
    int32_t num_upsample_layers = 5;
    int32_t up_sample_rates[5] = {8, 8, 4, 2, 2};
    int32_t up_channels[5] = {432, 216, 108, 54, 27};
    int32_t resblock_kernel_sizes[3] = {3, 7, 11};
    int32_t resblock_dilations[3] = {1, 3, 5};
};

struct magpie_codec {
    magpie_codec_hparams hparams;
    magpie_backend_type backend_type = MAGPIE_BACKEND_CUDA;
    mp_codec *dev = nullptr;
};

// ---- API (magpie.h:320-329): nullptr on failure, diagnostics on stderr
magpie_context *magpie_init(const char *model_path);
magpie_context *magpie_init_with_backend(const char *model_path, magpie_backend_type backend);
void magpie_free(magpie_context *ctx);
const char *magpie_get_backend_name(magpie_context *ctx);
// magpie.h:332: load a GGUF's weights into `model` (on the device MAGPIE_DEVICE names).
// The file is loaded into a fresh device state that replaces model.dev only on success:
// a model already loaded is replaced by a successful load and left intact, weights and
// hparams, by a failed one. The weight mode is picked from the file as magpie_init does.
// false + stderr on failure. backend: AUTO / CUDA
// select the HIP device; MAGPIE_BACKEND_CPU and METAL are refused (false + stderr: this
// build has one backend). Ownership: model.dev belongs to the caller until handed to a
// context; release a standalone model with magpie_model_free (magpie_free releases a
// context's model).
bool magpie_model_load(const std::string &path, magpie_model &model, magpie_backend_type backend = MAGPIE_BACKEND_AUTO);
// Added: release the device state of a model loaded with magpie_model_load (no-op if none).
void magpie_model_free(magpie_model &model);

// magpie.h:555-558: run the text encoder for one utterance; ctx->state.encoder_output
// ([n_tokens][d_model]) and enc_seq_len receive its output, as in the reference
// (magpie.cpp:2284-2374). The encoder alone (mp_hip_encode_text, a private device
// workspace): a batch in progress on ctx is not touched.
bool magpie_encode_text(magpie_context *ctx, const int32_t *tokens, int n_tokens);

// ---- synthesis (magpie.h:571-595): frame-major codes [n_frames * 8], BOS
// excluded; empty vector on failure. All four names run the same device loop
// (the reference's legacy variants are superseded).
std::vector<int32_t> magpie_synthesize_codes(magpie_context *ctx, const int32_t *tokens, int n_tokens);
std::vector<int32_t> magpie_synthesize_codes_cached(magpie_context *ctx, const int32_t *tokens, int n_tokens);
std::vector<int32_t> magpie_synthesize_codes_optimized(magpie_context *ctx, const int32_t *tokens, int n_tokens);
std::vector<int32_t> magpie_synthesize_codes_graph_reuse(magpie_context *ctx, const int32_t *tokens, int n_tokens);

// Added: B independent utterances in one device batch; out[b]
// receives utterance b's codes. Returns false on failure.
bool magpie_synthesize_codes_batch(magpie_context *ctx, const int32_t *const *tokens, const int *n_tokens, int B,
                                   std::vector<int32_t> *out);

// ---- nano-codec (magpie.h:746-759)
magpie_codec *magpie_codec_init(const char *codec_path);
magpie_codec *magpie_codec_init_with_backend(const char *codec_path, magpie_backend_type backend);
void magpie_codec_free(magpie_codec *codec);
// magpie.h:753: load codec weights from a GGUF into `codec` (replacing any loaded ones)
bool magpie_codec_load(const std::string &path, magpie_codec &codec, magpie_backend_type backend = MAGPIE_BACKEND_AUTO);
// codes: [num_codebooks][n_frames] codebook-major; returns n_frames * 1024 samples
std::vector<float> magpie_codec_decode(magpie_codec *codec, const int32_t *codes, int n_frames);

// magpie.h:372-377: the 8-codebook local transformer for one normalised decoder
// hidden state [768] (sampled + argmax codes), on the device.
magpie_sample_result magpie_local_transformer_sample_all(magpie_context *ctx, const float *decoder_hidden,
                                                        float temperature, int top_k, bool forbid_eos = false);

// ---- streaming (magpie.h:596-648, same types, fields and defaults)
typedef bool (*magpie_audio_callback)(const float *samples, int n_samples, void *user_data);
typedef void (*magpie_progress_callback)(int frames_generated, int sentence_index, int total_sentences,
                                         void *user_data);
struct magpie_stream_params {
    float temperature = 0.7f;
    int top_k = 80;
    int speaker_id = 0;
    int frames_per_chunk = 4;
    bool sentence_chunking = true;
    magpie_audio_callback on_audio = nullptr;
    magpie_progress_callback on_progress = nullptr;
    void *user_data = nullptr;
};
std::vector<std::string> magpie_split_sentences(const char *text);
// total samples, or -1 on error
int magpie_synthesize_streaming(magpie_context *ctx, magpie_codec *codec, const char *text,
                                const magpie_stream_params &params);
int magpie_synthesize_sentence_streaming(magpie_context *ctx, magpie_codec *codec, const int32_t *tokens,
                                         int n_tokens, const magpie_stream_params &params);

// magpie.h:823 utility
bool magpie_is_eos(const std::vector<int32_t> &frame_codes, int32_t eos_id);

#endif  // MAGPIE_H
