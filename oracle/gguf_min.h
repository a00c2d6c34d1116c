// Minimal, dependency-free GGUF v3 reader for the CPU oracle (TEST INFRASTRUCTURE).
// Independent of the product's reader on purpose. Layout per
// scripts/convert_magpie_to_gguf.py:380-423 (header, KV pairs, tensor infos,
// 32-byte aligned data section).
#ifndef ORC_GGUF_MIN_H
#define ORC_GGUF_MIN_H
#include <stddef.h>
#include <stdint.h>

typedef struct {
    char name[128];
    int n_dims;
    int64_t ne[4];   // ggml order (ne[0] contiguous)
    int type;        // 0 F32, 1 F16, 8 Q8_0
    uint64_t offset; // relative to data section
} orc_tinfo;

typedef struct {
    char key[128];
    int type;
    uint64_t u;  // integer value (if integer type)
    double f;    // float value (if float type)
} orc_kv;

typedef struct {
    uint8_t *map;
    size_t size;
    uint64_t data_off;
    int n_tensors, n_kv;
    orc_tinfo *t;
    orc_kv *kv;
} orc_gguf;

int orc_gguf_open(orc_gguf *g, const char *path);
void orc_gguf_close(orc_gguf *g);
const orc_tinfo *orc_gguf_find(const orc_gguf *g, const char *name);
// Returns a freshly malloc'ed f32 copy (dequantising F16/Q8_0); NULL if absent.
float *orc_gguf_f32(const orc_gguf *g, const char *name, int64_t *n_out);
int64_t orc_gguf_u32(const orc_gguf *g, const char *key, int64_t def);
double orc_gguf_f32kv(const orc_gguf *g, const char *key, double def);
float orc_f16_to_f32(uint16_t h);
uint16_t orc_f32_to_f16(float f);

#endif
