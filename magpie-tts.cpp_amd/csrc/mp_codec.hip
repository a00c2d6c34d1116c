// Nano-codec decoder on gfx950 (placeholder until the conv kernels land).
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/magpie_hip.h"

struct mp_codec {
    int device = 0;
    std::string err;
};

extern "C" {
int mp_hip_codec_init(int device, const char *path, mp_codec **out) {
    (void)device; (void)path;
    if (out) *out = nullptr;
    return MP_ERR_UNSUPPORTED;
}
int mp_hip_codec_decode(mp_codec *c, const int32_t *codes, int n_frames, float *audio_out) {
    (void)c; (void)codes; (void)n_frames; (void)audio_out;
    return MP_ERR_UNSUPPORTED;
}
void mp_hip_codec_free(mp_codec *c) { delete c; }
const char *mp_hip_codec_error(mp_codec *c) { return c ? c->err.c_str() : "null mp_codec"; }
}
