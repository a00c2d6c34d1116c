// mp_bench — native driver of the decode path (no Python), used for rocprofv3
// kernel traces and as a C++ mirror of the reference's tests/test_graph_reuse.cpp
// (wall-clock fps of magpie_synthesize_codes_graph_reuse).
//
// usage: mp_bench MODEL.gguf [frames=256] [batch=1] [reps=3] [tokens=64]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../include/magpie_hip.h"

int main(int argc, char **argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s MODEL.gguf [frames] [batch] [reps] [tokens]\n", argv[0]);
        return 2;
    }
    const int frames = argc > 2 ? atoi(argv[2]) : 256;
    const int B = argc > 3 ? atoi(argv[3]) : 1;
    const int reps = argc > 4 ? atoi(argv[4]) : 3;
    const int T = argc > 5 ? atoi(argv[5]) : 64;
    mp_dev *dev = nullptr;
    if (mp_hip_init(0, &dev) != MP_OK) { fprintf(stderr, "no HIP device\n"); return 1; }
    if (mp_hip_load_model(dev, argv[1]) != MP_OK) { fprintf(stderr, "%s\n", mp_hip_error(dev)); return 1; }
    std::vector<int32_t> tok((size_t)B * T), nt(B, T), spk(B);
    uint64_t s = 1000;
    for (int b = 0; b < B; ++b) {
        spk[b] = b % 5;
        for (int t = 0; t < T; ++t) {
            s = s * 6364136223846793005ull + 1442695040888963407ull;
            tok[(size_t)b * T + t] = t == 0 ? 2378 : t == T - 1 ? 2379 : (int)((s >> 33) % 96);
        }
    }
    mp_params p{};
    p.temperature = 0.f;
    p.top_k = 80;
    p.max_dec_steps = frames;
    p.ignore_eos = 1;
    if (mp_hip_begin_batch(dev, tok.data(), nt.data(), spk.data(), B, T, &p) != MP_OK) {
        fprintf(stderr, "%s\n", mp_hip_error(dev));
        return 1;
    }
    std::vector<int32_t> codes((size_t)B * frames * 8), nf(B);
    for (int r = 0; r < reps; ++r) {
        auto t0 = std::chrono::steady_clock::now();
        if (mp_hip_decode(dev, codes.data(), nf.data()) != MP_OK) { fprintf(stderr, "%s\n", mp_hip_error(dev)); return 1; }
        const double s_wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        mp_timing t{};
        mp_hip_get_timing(dev, &t);
        printf("rep %d: %d frames, decode %.3f ms (%.1f fps), wall %.3f ms, preamble %.2f ms\n", r, t.frames_total,
               t.decode_ms, t.frames_total / (t.decode_ms / 1e3), s_wall * 1e3, t.preamble_ms);
    }
    mp_hip_free(dev);
    return 0;
}
