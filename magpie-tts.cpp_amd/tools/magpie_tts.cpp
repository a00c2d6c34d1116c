// magpie-tts — command-line front end over the MI355X-native library, with the
// reference CLI's flags, defaults and output (src/magpie-tts.cpp:11-229): text ->
// tokens -> codes (graph-reuse decode loop) -> 32-frame stateless codec chunks ->
// 16-bit mono WAV at 22050 Hz. Extra flags: --stream (sentence-chunked streaming
// synthesis, magpie.cpp:4843-4863), --bf16 (bf16 decode projections), --seed.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/magpie.h"

namespace {

void usage(const char *prog) {
    fprintf(stderr,
            "Magpie TTS (MI355X / HIP)\n\nUsage: %s [options]\n\n"
            "  -m, --model PATH     model GGUF (default: weights/magpie-357m-f32.gguf)\n"
            "  -c, --codec PATH     codec GGUF (default: weights/nano-codec-f32.gguf)\n"
            "  -t, --text TEXT      text to synthesize (required)\n"
            "  -o, --output PATH    output WAV (default: output.wav)\n"
            "  -s, --speaker ID     speaker id (default: 0)\n"
            "  --temp FLOAT         sampling temperature (default: 0.7, 0 = greedy)\n"
            "  --top-k INT          top-k sampling (default: 80)\n"
            "  --seed N             sampling stream seed (default: 0)\n"
            "  --stream             sentence-chunked streaming synthesis (4-frame codec chunks)\n"
            "  --bf16               bf16 decode projections (MFMA)\n"
            "  -q, --quiet          minimal output\n"
            "  -h, --help           this help\n",
            prog);
}

// RIFF/WAVE, PCM 16-bit mono; samples clamped to [-1, 1] and scaled by 32767
// with truncation, as the reference writer does (magpie-tts.cpp:31-69).
bool write_wav(const char *path, const std::vector<float> &audio, int rate) {
    FILE *f = fopen(path, "wb");
    if (!f) return false;
    struct {
        char riff[4] = {'R', 'I', 'F', 'F'};
        int32_t riff_size;
        char wave[4] = {'W', 'A', 'V', 'E'};
        char fmt[4] = {'f', 'm', 't', ' '};
        int32_t fmt_size = 16;
        int16_t format = 1, channels = 1;
        int32_t rate, byte_rate;
        int16_t align = 2, bits = 16;
        char data[4] = {'d', 'a', 't', 'a'};
        int32_t data_size;
    } __attribute__((packed)) h;
    h.data_size = (int32_t)(audio.size() * 2);
    h.riff_size = 36 + h.data_size;
    h.rate = rate;
    h.byte_rate = rate * 2;
    std::vector<int16_t> pcm(audio.size());
    for (size_t i = 0; i < audio.size(); ++i) {
        const float s = audio[i] > 1.f ? 1.f : audio[i] < -1.f ? -1.f : audio[i];
        pcm[i] = (int16_t)(s * 32767.0f);
    }
    const bool ok = fwrite(&h, sizeof h, 1, f) == 1 && fwrite(pcm.data(), 2, pcm.size(), f) == pcm.size();
    return fclose(f) == 0 && ok;
}

bool collect(const float *x, int n, void *user) {
    auto *v = (std::vector<float> *)user;
    v->insert(v->end(), x, x + n);
    return true;
}

}  // namespace

int main(int argc, char **argv) {
    const char *model = "weights/magpie-357m-f32.gguf", *codec_path = "weights/nano-codec-f32.gguf";
    const char *text = nullptr, *out = "output.wav";
    int speaker = 0, top_k = 80;
    float temp = 0.7f;
    unsigned long long seed = 0;
    bool quiet = false, stream = false, bf16 = false;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto val = [&](const char *what) -> const char * {
            if (++i >= argc) {
                fprintf(stderr, "Error: %s requires a value\n", what);
                exit(1);
            }
            return argv[i];
        };
        if (a == "-h" || a == "--help") { usage(argv[0]); return 0; }
        else if (a == "-m" || a == "--model") model = val("--model");
        else if (a == "-c" || a == "--codec") codec_path = val("--codec");
        else if (a == "-t" || a == "--text") text = val("--text");
        else if (a == "-o" || a == "--output") out = val("--output");
        else if (a == "-s" || a == "--speaker") speaker = atoi(val("--speaker"));
        else if (a == "--temp") temp = (float)atof(val("--temp"));
        else if (a == "--top-k") top_k = atoi(val("--top-k"));
        else if (a == "--seed") seed = strtoull(val("--seed"), nullptr, 10);
        else if (a == "--stream") stream = true;
        else if (a == "--bf16") bf16 = true;
        else if (a == "-q" || a == "--quiet") quiet = true;
        else {
            fprintf(stderr, "Unknown option: %s\n", argv[i]);
            usage(argv[0]);
            return 1;
        }
    }
    if (!text) {
        fprintf(stderr, "Error: --text is required\n\n");
        usage(argv[0]);
        return 1;
    }
    if (bf16) setenv("MAGPIE_WEIGHTS", "bf16", 1);
    magpie_context *ctx = magpie_init(model);
    if (!ctx) {
        fprintf(stderr, "Error: Failed to load model from %s\n", model);
        return 1;
    }
    ctx->temperature = temp;
    ctx->top_k = top_k;
    ctx->speaker_id = speaker;
    ctx->seed = seed;
    magpie_codec *codec = magpie_codec_init(codec_path);
    if (!codec) {
        fprintf(stderr, "Error: Failed to load codec from %s\n", codec_path);
        magpie_free(ctx);
        return 1;
    }
    std::vector<float> audio;
    int rc = 0;
    if (stream) {
        magpie_stream_params sp;
        sp.temperature = temp;
        sp.top_k = top_k;
        sp.speaker_id = speaker;
        sp.on_audio = collect;
        sp.user_data = &audio;
        if (magpie_synthesize_streaming(ctx, codec, text, sp) < 0) rc = 1;
    } else {
        const std::vector<int32_t> tokens = magpie_tokenize(&ctx->model.tokenizer, text);
        if (tokens.empty()) {
            fprintf(stderr, "Error: Tokenization failed\n");
            rc = 1;
        } else {
            if (!quiet) fprintf(stderr, "Tokens: %zu\n", tokens.size());
            const std::vector<int32_t> codes = magpie_synthesize_codes_graph_reuse(ctx, tokens.data(), (int)tokens.size());
            const int n = (int)codes.size() / 8;
            if (codes.empty()) rc = 1;
            // stateless 32-frame codec chunks, frame-major -> codebook-major (magpie-tts.cpp:181-206)
            for (int c0 = 0; rc == 0 && c0 < n; c0 += 32) {
                const int f = std::min(32, n - c0);
                std::vector<int32_t> cb((size_t)8 * f);
                for (int t = 0; t < f; ++t)
                    for (int k = 0; k < 8; ++k) cb[(size_t)k * f + t] = codes[(size_t)(c0 + t) * 8 + k];
                const std::vector<float> a = magpie_codec_decode(codec, cb.data(), f);
                if (a.empty()) rc = 1;
                audio.insert(audio.end(), a.begin(), a.end());
            }
        }
    }
    if (rc == 0 && !write_wav(out, audio, 22050)) {
        fprintf(stderr, "Error: Failed to write %s\n", out);
        rc = 1;
    }
    if (rc == 0) {
        if (quiet) printf("%s\n", out);
        else fprintf(stderr, "Done! Generated %.2f seconds of audio.\n", audio.size() / 22050.0);
    }
    magpie_codec_free(codec);
    magpie_free(ctx);
    return rc;
}
