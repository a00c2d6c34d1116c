// magpie_api.cpp — the reference's C++ entry points (include/magpie.h) over the
// C-ABI of magpie_hip.h. Host-only code; every arithmetic op runs in the HIP
// kernels behind mp_hip_*.
#include "../../include/magpie.h"

#include <cstdio>
#include <cstdlib>

static int env_device() {
    const char *s = getenv("MAGPIE_DEVICE");
    return s ? atoi(s) : 0;
}

magpie_context *magpie_init(const char *model_path) { return magpie_init_with_backend(model_path, MAGPIE_BACKEND_AUTO); }

// magpie_init_with_backend (magpie.cpp:781-880): nullptr + stderr on failure.
magpie_context *magpie_init_with_backend(const char *model_path, magpie_backend_type backend) {
    (void)backend;  // single HIP device path
    if (!model_path) return nullptr;
    magpie_context *ctx = new magpie_context();
    if (mp_hip_init(env_device(), &ctx->model.dev) != MP_OK) {
        fprintf(stderr, "magpie: no usable HIP device\n");
        delete ctx;
        return nullptr;
    }
    if (mp_hip_load_model(ctx->model.dev, model_path) != MP_OK) {
        fprintf(stderr, "magpie: failed to load '%s': %s\n", model_path, mp_hip_error(ctx->model.dev));
        mp_hip_free(ctx->model.dev);
        delete ctx;
        return nullptr;
    }
    int dec = 12, enc = 6;
    mp_hip_model_info(ctx->model.dev, &dec, &enc, nullptr);
    ctx->model.hparams.dec_layers = dec;
    ctx->model.hparams.enc_layers = enc;
    return ctx;
}

void magpie_free(magpie_context *ctx) {
    if (!ctx) return;
    if (ctx->model.dev) mp_hip_free(ctx->model.dev);
    delete ctx;
}

const char *magpie_get_backend_name(magpie_context *ctx) { return ctx && ctx->model.dev ? "HIP (gfx950)" : "none"; }

static mp_params params_of(const magpie_context *ctx) {
    mp_params p{};
    p.temperature = ctx->temperature;
    p.top_k = ctx->top_k;
    p.max_dec_steps = ctx->model.hparams.max_dec_steps;
    p.ignore_eos = 0;
    p.seed = ctx->seed;
    p.trace_hidden = 0;
    return p;
}

bool magpie_synthesize_codes_batch(magpie_context *ctx, const int32_t *const *tokens, const int *n_tokens, int B,
                                   std::vector<int32_t> *out) {
    if (!ctx || !ctx->model.dev || !tokens || !n_tokens || B < 1 || !out) return false;
    int tmax = 0;
    for (int b = 0; b < B; ++b) {
        if (!tokens[b] || n_tokens[b] <= 0) return false;
        tmax = std::max(tmax, n_tokens[b]);
    }
    std::vector<int32_t> tok((size_t)B * tmax, 0), nt(B), spk(B, ctx->speaker_id);
    for (int b = 0; b < B; ++b) {
        nt[b] = n_tokens[b];
        std::copy(tokens[b], tokens[b] + n_tokens[b], tok.begin() + (size_t)b * tmax);
    }
    const mp_params p = params_of(ctx);
    const int steps = p.max_dec_steps > 0 ? p.max_dec_steps : 500;
    if (mp_hip_begin_batch(ctx->model.dev, tok.data(), nt.data(), spk.data(), B, tmax, &p) != MP_OK) {
        fprintf(stderr, "magpie: %s\n", mp_hip_error(ctx->model.dev));
        return false;
    }
    std::vector<int32_t> codes((size_t)B * steps * 8), nf(B);
    if (mp_hip_decode(ctx->model.dev, codes.data(), nf.data()) != MP_OK) {
        fprintf(stderr, "magpie: %s\n", mp_hip_error(ctx->model.dev));
        return false;
    }
    for (int b = 0; b < B; ++b)
        out[b].assign(codes.begin() + (size_t)b * steps * 8, codes.begin() + (size_t)b * steps * 8 + (size_t)nf[b] * 8);
    return true;
}

// magpie_synthesize_codes_graph_reuse (magpie.cpp:4063-4432): empty on failure.
std::vector<int32_t> magpie_synthesize_codes_graph_reuse(magpie_context *ctx, const int32_t *tokens, int n_tokens) {
    if (!ctx || !tokens || n_tokens <= 0) {
        fprintf(stderr, "magpie_synthesize_codes_graph_reuse: invalid args\n");
        return {};
    }
    std::vector<int32_t> out;
    const int32_t *tp[1] = {tokens};
    const int nt[1] = {n_tokens};
    if (!magpie_synthesize_codes_batch(ctx, tp, nt, 1, &out)) return {};
    mp_timing t{};
    mp_hip_get_timing(ctx->model.dev, &t);
    const int n_frames = (int)out.size() / 8;
    fprintf(stderr, "magpie: [hip] %d audio frames in %.3f s (%.1f fps), preamble %.1f ms\n", n_frames,
            t.decode_ms / 1e3, t.decode_ms > 0 ? n_frames / (t.decode_ms / 1e3) : 0.0, t.preamble_ms);
    return out;
}
std::vector<int32_t> magpie_synthesize_codes(magpie_context *ctx, const int32_t *tokens, int n_tokens) {
    return magpie_synthesize_codes_graph_reuse(ctx, tokens, n_tokens);
}
std::vector<int32_t> magpie_synthesize_codes_cached(magpie_context *ctx, const int32_t *tokens, int n_tokens) {
    return magpie_synthesize_codes_graph_reuse(ctx, tokens, n_tokens);
}
std::vector<int32_t> magpie_synthesize_codes_optimized(magpie_context *ctx, const int32_t *tokens, int n_tokens) {
    return magpie_synthesize_codes_graph_reuse(ctx, tokens, n_tokens);
}

magpie_codec *magpie_codec_init(const char *codec_path) {
    return magpie_codec_init_with_backend(codec_path, MAGPIE_BACKEND_AUTO);
}
magpie_codec *magpie_codec_init_with_backend(const char *codec_path, magpie_backend_type backend) {
    (void)backend;
    if (!codec_path) return nullptr;
    magpie_codec *c = new magpie_codec();
    if (mp_hip_codec_init(env_device(), codec_path, &c->dev) != MP_OK) {
        fprintf(stderr, "magpie_codec: failed to load %s\n", codec_path);
        delete c;
        return nullptr;
    }
    return c;
}
void magpie_codec_free(magpie_codec *codec) {
    if (!codec) return;
    if (codec->dev) mp_hip_codec_free(codec->dev);
    delete codec;
}
// magpie_codec_decode (nano-codec.cpp:758-845): empty vector on failure.
std::vector<float> magpie_codec_decode(magpie_codec *codec, const int32_t *codes, int n_frames) {
    if (!codec || !codec->dev || !codes || n_frames <= 0) {
        fprintf(stderr, "magpie_codec_decode: invalid args\n");
        return {};
    }
    std::vector<float> audio((size_t)n_frames * codec->hparams.hop_length);
    if (mp_hip_codec_decode(codec->dev, codes, n_frames, audio.data()) != MP_OK) {
        fprintf(stderr, "magpie_codec_decode: %s\n", mp_hip_codec_error(codec->dev));
        return {};
    }
    return audio;
}

bool magpie_is_eos(const std::vector<int32_t> &frame_codes, int32_t eos_id) {
    for (int32_t c : frame_codes)
        if (c == eos_id) return true;
    return false;
}
