// magpie_api.cpp — the reference's C++ entry points (include/magpie.h) over the
// C-ABI of magpie_hip.h. Host-only code; every arithmetic op runs in the HIP
// kernels behind mp_hip_*.
#include "../../include/magpie.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>

static int env_device() {
    const char *s = getenv("MAGPIE_DEVICE");
    return s ? atoi(s) : 0;
}

magpie_context *magpie_init(const char *model_path) { return magpie_init_with_backend(model_path, MAGPIE_BACKEND_AUTO); }

// magpie_model_load (magpie.cpp:572-718 behind magpie.h:332): false + stderr on failure.
bool magpie_model_load(const std::string &path, magpie_model &model, magpie_backend_type backend) {
    if (backend == MAGPIE_BACKEND_CPU || backend == MAGPIE_BACKEND_METAL) {
        fprintf(stderr, "magpie: backend %s is not available in this build (HIP only)\n",
                backend == MAGPIE_BACKEND_CPU ? "CPU" : "Metal");
        return false;
    }
    // Always load into a fresh device state and swap it in only on success: a failed
    // reload leaves a model that was already loaded intact (weights and hparams).
    mp_dev *dev = nullptr;
    if (mp_hip_init(env_device(), &dev) != MP_OK) {
        fprintf(stderr, "magpie: no usable HIP device\n");
        return false;
    }
    // Weight mode (magpie_hip.h): a GGUF with Q8_0 / Q4_0 tensors runs them as ggml does
    // (MP_WEIGHTS_Q8), an F16 file with ggml's F16 semantics (MP_WEIGHTS_F16), any other
    // file as stored; MAGPIE_WEIGHTS=f32|bf16|q8|f16 overrides.
    const char *wm = getenv("MAGPIE_WEIGHTS");
    int mode = MP_WEIGHTS_Q8;
    bool forced = false;
    if (wm && *wm) {
        forced = true;
        mode = !strcmp(wm, "bf16")  ? MP_WEIGHTS_BF16
               : !strcmp(wm, "q8") ? MP_WEIGHTS_Q8
               : !strcmp(wm, "f16") ? MP_WEIGHTS_F16
                                    : MP_WEIGHTS_AS_STORED;
    }
    int rc = mp_hip_load_model_ex(dev, path.c_str(), mode);
    if (rc == MP_ERR_UNSUPPORTED && !forced)  // no block-quantised tensors: an F16 file?
        rc = mp_hip_load_model_ex(dev, path.c_str(), MP_WEIGHTS_F16);
    if (rc == MP_ERR_UNSUPPORTED && !forced)  // neither: as stored
        rc = mp_hip_load_model_ex(dev, path.c_str(), MP_WEIGHTS_AS_STORED);
    if (rc != MP_OK) {
        fprintf(stderr, "magpie: failed to load '%s': %s\n", path.c_str(), mp_hip_error(dev));
        mp_hip_free(dev);
        return false;
    }
    if (model.dev) mp_hip_free(model.dev);  // the replaced model
    model.dev = dev;
    int dec = 12, enc = 6;
    mp_hip_model_info(model.dev, &dec, &enc, nullptr);
    // the text front end rides in the same GGUF (magpie.cpp:853-858); optional
    model.tokenizer = magpie_tokenizer();
    if (!magpie_tokenizer_load(&model.tokenizer, path.c_str()))
        fprintf(stderr, "magpie: no tokenizer in '%s' (token-id entry points only)\n", path.c_str());
    model.hparams.dec_layers = dec;
    model.hparams.enc_layers = enc;
    return true;
}

void magpie_model_free(magpie_model &model) {
    if (model.dev) mp_hip_free(model.dev);
    model.dev = nullptr;
}

// magpie_init_with_backend (magpie.cpp:781-880): nullptr + stderr on failure.
magpie_context *magpie_init_with_backend(const char *model_path, magpie_backend_type backend) {
    if (!model_path) return nullptr;
    magpie_context *ctx = new magpie_context();
    if (!magpie_model_load(model_path, ctx->model, backend)) {
        if (ctx->model.dev) mp_hip_free(ctx->model.dev);
        delete ctx;
        return nullptr;
    }
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
    ctx->state.reset();
    if (!magpie_synthesize_codes_batch(ctx, tp, nt, 1, &out)) return {};
    // ctx->state as the reference leaves it: the encoder output of this utterance
    // (magpie.cpp:2364-2367) and the generated frames
    const long long eb = mp_hip_debug_buffer(ctx->model.dev, "enc_out", nullptr, 0);
    if (eb >= (long long)n_tokens * 768 * 4) {
        std::vector<float> enc((size_t)eb / 4);
        if (mp_hip_debug_buffer(ctx->model.dev, "enc_out", enc.data(), eb) == eb) {
            ctx->state.encoder_output.assign(enc.begin(), enc.begin() + (size_t)n_tokens * 768);
            ctx->state.enc_seq_len = n_tokens;
        }
    }
    ctx->state.generated_codes = out;
    ctx->state.n_generated_frames = (int32_t)(out.size() / 8);
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

// magpie_encode_text (magpie.cpp:2284-2374): the encoder output lands in ctx->state.
// Encoder only (mp_hip_encode_text): a batch in progress on this context is untouched.
bool magpie_encode_text(magpie_context *ctx, const int32_t *tokens, int n_tokens) {
    if (!ctx || !ctx->model.dev || !tokens || n_tokens <= 0) {
        fprintf(stderr, "magpie_encode_text: invalid args\n");
        return false;
    }
    std::vector<float> enc((size_t)n_tokens * 768);
    if (mp_hip_encode_text(ctx->model.dev, tokens, n_tokens, enc.data()) != MP_OK) {
        fprintf(stderr, "magpie_encode_text: %s\n", mp_hip_error(ctx->model.dev));
        return false;
    }
    ctx->state.encoder_output = std::move(enc);
    ctx->state.enc_seq_len = n_tokens;
    return true;
}

magpie_codec *magpie_codec_init(const char *codec_path) {
    return magpie_codec_init_with_backend(codec_path, MAGPIE_BACKEND_AUTO);
}
magpie_codec *magpie_codec_init_with_backend(const char *codec_path, magpie_backend_type backend) {
    (void)backend;
    if (!codec_path) return nullptr;
    magpie_codec *c = new magpie_codec();
    if (!magpie_codec_load(codec_path, *c, backend)) {
        delete c;
        return nullptr;
    }
    return c;
}
// magpie_codec_load (nano-codec.cpp:205-352 behind magpie.h:753)
bool magpie_codec_load(const std::string &path, magpie_codec &codec, magpie_backend_type backend) {
    (void)backend;
    if (codec.dev) {
        mp_hip_codec_free(codec.dev);
        codec.dev = nullptr;
    }
    if (mp_hip_codec_init(env_device(), path.c_str(), &codec.dev) != MP_OK) {
        fprintf(stderr, "magpie_codec: failed to load %s\n", path.c_str());
        codec.dev = nullptr;
        return false;
    }
    return true;
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

// magpie_local_transformer_sample_all (magpie.cpp:1113-1317) on the device.
magpie_sample_result magpie_local_transformer_sample_all(magpie_context *ctx, const float *decoder_hidden,
                                                        float temperature, int top_k, bool forbid_eos) {
    magpie_sample_result r;
    if (!ctx || !ctx->model.dev || !decoder_hidden) return r;
    int32_t smp[8], amx[8];
    if (mp_hip_lt_sample(ctx->model.dev, decoder_hidden, temperature, top_k, forbid_eos ? 1 : 0, ctx->seed, smp, amx) !=
        MP_OK) {
        fprintf(stderr, "magpie: local transformer failed: %s\n", mp_hip_error(ctx->model.dev));
        return r;  // empty: the reference's failure signal (sampled_codes.size() != 8)
    }
    r.sampled_codes.assign(smp, smp + 8);
    r.argmax_codes.assign(amx, amx + 8);
    return r;
}

// ---------------------------------------------------------------- streaming
// magpie_split_sentences (magpie.cpp:4439-4480), over mp_split_sentences
std::vector<std::string> magpie_split_sentences(const char *text) {
    std::vector<std::string> out;
    if (!text) return out;
    const int n = mp_split_sentences(text, nullptr, nullptr, 0);
    std::vector<int32_t> off(std::max(n, 0)), len(std::max(n, 0));
    mp_split_sentences(text, off.data(), len.data(), n);
    for (int i = 0; i < n; ++i) out.emplace_back(text + off[i], (size_t)len[i]);
    return out;
}

namespace {

// Runs one device batch of sentences through mp_hip_decode_stream and hands the
// audio to the caller's callback in sentence order: sentence `next` streams
// live, later ones are buffered until every earlier sentence has ended.
struct OrderedStream {
    const magpie_stream_params *prm;
    int B = 0, next = 0, sentence0 = 0, n_sentences = 1;
    std::vector<std::deque<std::vector<float>>> pending;
    std::vector<int> ended, stopped, frames;
    long long delivered = 0;

    bool deliver(int u, const float *x, int n) {
        delivered += n;
        frames[u] += n / 1024;
        bool go = prm->on_audio ? prm->on_audio(x, n, prm->user_data) : true;
        if (prm->on_progress) prm->on_progress(frames[u], 0, 1, prm->user_data);  // (4826-4828)
        return go;
    }
    void drain() {
        while (next < B) {
            auto &q = pending[next];
            while (!q.empty() && !stopped[next]) {
                std::vector<float> a = std::move(q.front());
                q.pop_front();
                if (!deliver(next, a.data(), (int)a.size())) stopped[next] = 1;
            }
            q.clear();
            if (!ended[next]) break;
            ++next;
        }
    }
    static int cb(int u, const float *x, int n, void *self_) {
        OrderedStream &s = *(OrderedStream *)self_;
        if (n == 0) {
            s.ended[u] = 1;
            s.drain();
            return 1;
        }
        if (s.stopped[u]) return 0;
        if (u == s.next) {
            if (!s.deliver(u, x, n)) { s.stopped[u] = 1; return 0; }
            return 1;
        }
        s.pending[u].emplace_back(x, x + n);
        return 1;  // a buffered sentence's stop is applied when it is delivered
    }
};

long long stream_batch(magpie_context *ctx, magpie_codec *codec, const std::vector<std::vector<int32_t>> &sents,
                       int sentence0, const magpie_stream_params &prm) {
    const int B = (int)sents.size();
    int tmax = 0;
    for (auto &t : sents) tmax = std::max(tmax, (int)t.size());
    std::vector<int32_t> tok((size_t)B * tmax, 0), nt(B), spk(B, prm.speaker_id);
    for (int b = 0; b < B; ++b) {
        nt[b] = (int32_t)sents[b].size();
        std::copy(sents[b].begin(), sents[b].end(), tok.begin() + (size_t)b * tmax);
    }
    mp_params p{};
    p.temperature = prm.temperature;
    p.top_k = prm.top_k;
    p.max_dec_steps = ctx->model.hparams.max_dec_steps;
    p.seed = ctx->seed;
    p.stream_base = sentence0;  // sentence i draws from stream i, batched or not
    p.emit_eos_frame = 1;       // the streaming loop emits the EOS frame (magpie.cpp:4800-4806)
    if (mp_hip_begin_batch(ctx->model.dev, tok.data(), nt.data(), spk.data(), B, tmax, &p) != MP_OK) {
        fprintf(stderr, "magpie: %s\n", mp_hip_error(ctx->model.dev));
        return -1;
    }
    OrderedStream os;
    os.prm = &prm;
    os.B = B;
    os.pending.resize(B);
    os.ended.assign(B, 0);
    os.stopped.assign(B, 0);
    os.frames.assign(B, 0);
    if (mp_hip_decode_stream(ctx->model.dev, codec->dev, prm.frames_per_chunk, OrderedStream::cb, &os, nullptr,
                             nullptr, nullptr) != MP_OK) {
        fprintf(stderr, "magpie: %s\n", mp_hip_error(ctx->model.dev));
        return -1;
    }
    os.drain();
    return os.delivered;
}

}  // namespace

// magpie_synthesize_sentence_streaming (magpie.cpp:4479-4840)
int magpie_synthesize_sentence_streaming(magpie_context *ctx, magpie_codec *codec, const int32_t *tokens,
                                         int n_tokens, const magpie_stream_params &params) {
    if (!ctx || !ctx->model.dev || !codec || !codec->dev || !tokens || n_tokens <= 0) return -1;
    ctx->temperature = params.temperature;  // as the reference does (4497-4499)
    ctx->top_k = params.top_k;
    ctx->speaker_id = params.speaker_id;
    const long long n = stream_batch(ctx, codec, {std::vector<int32_t>(tokens, tokens + n_tokens)}, 0, params);
    return n < 0 ? -1 : (int)n;
}

// magpie_synthesize_streaming (magpie.cpp:4843-4863). Sentences of the text run
// as device batches of up to ctx->max_parallel_sentences; the audio reaches on_audio
// in sentence order, sample for sample what the sentence-by-sentence loop gives.
int magpie_synthesize_streaming(magpie_context *ctx, magpie_codec *codec, const char *text,
                                const magpie_stream_params &params) {
    if (!ctx || !ctx->model.dev || !codec || !codec->dev || !text) return -1;
    std::vector<std::vector<int32_t>> sents;
    if (params.sentence_chunking) {
        std::vector<std::string> ss = magpie_split_sentences(text);
        if (ss.empty()) ss.push_back(text);
        for (auto &s : ss) {
            std::vector<int32_t> t = magpie_tokenize(&ctx->model.tokenizer, s);
            if (!t.empty()) sents.push_back(std::move(t));
        }
    } else {
        std::vector<int32_t> t = magpie_tokenize(&ctx->model.tokenizer, text);
        if (t.empty()) return -1;
        sents.push_back(std::move(t));
    }
    ctx->temperature = params.temperature;
    ctx->top_k = params.top_k;
    ctx->speaker_id = params.speaker_id;
    const int bmax = std::max(1, mp_hip_max_batch(ctx->model.dev));
    const int P = std::max(1, std::min(ctx->max_parallel_sentences, bmax));
    long long total = 0;
    for (size_t s0 = 0; s0 < sents.size(); s0 += P) {
        const size_t s1 = std::min(sents.size(), s0 + P);
        if (params.on_progress) params.on_progress(0, (int)s0, (int)sents.size(), params.user_data);
        const long long n = stream_batch(ctx, codec, {sents.begin() + s0, sents.begin() + s1}, (int)s0, params);
        if (n < 0) return -1;
        total += n;
    }
    return (int)total;
}
