// api_probe — exercises the drop-in C++ entry points a reference caller may use
// beyond init/synthesize (src/magpie.h:332 magpie_model_load, 555-558
// magpie_encode_text, 753 magpie_codec_load) on the device, for
// tests/test_cli_gpu.py: prints one JSON line and writes the encoder output
// ([n_tokens][768] f32) to OUT.
// usage: magpie-api-probe MODEL.gguf CODEC.gguf OUT.bin TEXT
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/magpie.h"

int main(int argc, char **argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: %s MODEL.gguf CODEC.gguf OUT.bin TEXT\n", argv[0]);
        return 2;
    }
    magpie_model m;
    const bool loaded = magpie_model_load(std::string(argv[1]), m);
    const int dec_layers = m.hparams.dec_layers;
    magpie_model_free(m);
    magpie_model cpu;  // the CPU backend is refused (one HIP backend), without leaking a device
    const bool cpu_refused = !magpie_model_load(std::string(argv[1]), cpu, MAGPIE_BACKEND_CPU) && cpu.dev == nullptr;
    magpie_context *ctx = magpie_init(argv[1]);
    if (!ctx) return 1;
    const std::vector<int32_t> ids = magpie_tokenize(&ctx->model.tokenizer, argv[4]);
    const bool enc = magpie_encode_text(ctx, ids.data(), (int)ids.size());
    if (FILE *f = fopen(argv[3], "wb")) {
        fwrite(ctx->state.encoder_output.data(), sizeof(float), ctx->state.encoder_output.size(), f);
        fclose(f);
    }
    magpie_codec c;
    const bool cl = magpie_codec_load(std::string(argv[2]), c);
    std::vector<int32_t> codes(8 * 4, 0);
    const std::vector<float> audio = cl ? magpie_codec_decode(&c, codes.data(), 4) : std::vector<float>();
    if (c.dev) mp_hip_codec_free(c.dev);
    printf("{\"model_load\": %s, \"dec_layers\": %d, \"encode_text\": %s, \"enc_seq_len\": %d, \"n_tokens\": %d, "
           "\"tokens\": [",
           loaded ? "true" : "false", dec_layers, enc ? "true" : "false", ctx->state.enc_seq_len, (int)ids.size());
    for (size_t i = 0; i < ids.size(); ++i) printf("%s%d", i ? ", " : "", ids[i]);
    printf("], \"codec_load\": %s, \"codec_samples\": %d, \"cpu_backend_refused\": %s}\n", cl ? "true" : "false",
           (int)audio.size(), cpu_refused ? "true" : "false");
    magpie_free(ctx);
    return loaded && enc && cl ? 0 : 1;
}
