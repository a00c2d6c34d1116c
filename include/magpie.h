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
// Out of scope here: graph-builder entry points
// (magpie_build_*), the tokenizer, streaming API and CLI.
#ifndef MAGPIE_H
#define MAGPIE_H

#include <cstdint>
#include <string>
#include <vector>

#include "magpie_hip.h"

// magpie.h:24-29 — kept for source compatibility; every value selects the single
// HIP device path (CPU/Metal requests are honoured as "the GPU" — there is no
// CPU fallback by design).
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

struct magpie_model {
    magpie_hparams hparams;
    magpie_backend_type backend_type = MAGPIE_BACKEND_CUDA;
    mp_dev *dev = nullptr;  // resident weights + device state (replaces ggml ctx/buffers)
};

// magpie.h:293-307 — public inference settings kept as plain fields.
struct magpie_context {
    magpie_model model;
    int n_threads;  // accepted, unused (the reference never applies it either, magpie.h:298)
    float temperature;
    int top_k;
    int speaker_id;
    struct magpie_codec *codec;
    uint64_t seed;  // added: the reference's sampler is an unseeded static mt19937 (magpie.cpp:1129)
    magpie_context() : n_threads(4), temperature(0.7f), top_k(80), speaker_id(0), codec(nullptr), seed(0) {}
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
// codes: [num_codebooks][n_frames] codebook-major; returns n_frames * 1024 samples
std::vector<float> magpie_codec_decode(magpie_codec *codec, const int32_t *codes, int n_frames);

// magpie.h:823 utility
bool magpie_is_eos(const std::vector<int32_t> &frame_codes, int32_t eos_id);

#endif  // MAGPIE_H
