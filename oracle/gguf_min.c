// Minimal GGUF v3 reader for the CPU oracle. TEST INFRASTRUCTURE ONLY.
// Format: scripts/convert_magpie_to_gguf.py:380-423; Q8_0 block = fp16 d + 32 x int8
// (scripts/convert_magpie_to_gguf.py:79-104).
#include "gguf_min.h"

#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

float orc_f16_to_f32(uint16_t h) {
    uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t exp = (h >> 10) & 0x1Fu, mant = h & 0x3FFu, x;
    if (exp == 0) {
        if (!mant) x = sign;
        else {
            exp = 127 - 15 + 1;
            while (!(mant & 0x400u)) { mant <<= 1; exp--; }
            mant &= 0x3FFu;
            x = sign | (exp << 23) | (mant << 13);
        }
    } else if (exp == 31) x = sign | 0x7F800000u | (mant << 13);
    else x = sign | ((exp - 15 + 127) << 23) | (mant << 13);
    float f;
    memcpy(&f, &x, 4);
    return f;
}

uint16_t orc_f32_to_f16(float f) {  // round to nearest even
    uint32_t x;
    memcpy(&x, &f, 4);
    uint32_t sign = (x >> 16) & 0x8000u, mant = x & 0x7FFFFFu;
    int32_t exp = (int32_t)((x >> 23) & 0xFF);
    if (exp == 0xFF) return (uint16_t)(sign | 0x7C00u | (mant ? 0x200u : 0));
    int32_t e = exp - 127 + 15;
    if (e >= 31) return (uint16_t)(sign | 0x7C00u);
    if (e <= 0) {
        if (e < -10) return (uint16_t)sign;
        mant |= 0x800000u;
        uint32_t shift = (uint32_t)(14 - e), half = mant >> shift;
        uint32_t rem = mant & ((1u << shift) - 1u), mid = 1u << (shift - 1);
        if (rem > mid || (rem == mid && (half & 1u))) half++;
        return (uint16_t)(sign | half);
    }
    uint32_t half = ((uint32_t)e << 10) | (mant >> 13), rem = mant & 0x1FFFu;
    if (rem > 0x1000u || (rem == 0x1000u && (half & 1u))) half++;
    return (uint16_t)(sign | half);
}

typedef struct { const uint8_t *p, *end; int err; } rd;
static uint64_t r_u64(rd *r) { uint64_t v = 0; if (r->p + 8 > r->end) { r->err = 1; return 0; } memcpy(&v, r->p, 8); r->p += 8; return v; }
static uint32_t r_u32(rd *r) { uint32_t v = 0; if (r->p + 4 > r->end) { r->err = 1; return 0; } memcpy(&v, r->p, 4); r->p += 4; return v; }
static void r_skip(rd *r, uint64_t n) { if (r->p + n > r->end) { r->err = 1; return; } r->p += n; }
static void r_str(rd *r, char *dst, size_t cap) {
    uint64_t n = r_u64(r);
    if (r->err || r->p + n > r->end) { r->err = 1; return; }
    if (dst) { size_t c = n < cap - 1 ? (size_t)n : cap - 1; memcpy(dst, r->p, c); dst[c] = 0; }
    r->p += n;
}
static const int k_scalar_size[13] = {1, 1, 2, 2, 4, 4, 4, 1, 0, 0, 8, 8, 8};

static void r_value(rd *r, int type, orc_kv *kv) {
    if (type == 8) { r_str(r, NULL, 0); return; }
    if (type == 9) {
        uint32_t et = r_u32(r);
        uint64_t n = r_u64(r);
        for (uint64_t i = 0; i < n && !r->err; ++i) r_value(r, (int)et, NULL);
        return;
    }
    if (type < 0 || type > 12) { r->err = 1; return; }
    const uint8_t *p = r->p;
    r_skip(r, (uint64_t)k_scalar_size[type]);
    if (!kv || r->err) return;
    switch (type) {
    case 0: kv->u = p[0]; break;
    case 1: kv->u = (uint64_t)(int64_t)(int8_t)p[0]; break;
    case 2: { uint16_t v; memcpy(&v, p, 2); kv->u = v; } break;
    case 3: { int16_t v; memcpy(&v, p, 2); kv->u = (uint64_t)(int64_t)v; } break;
    case 4: { uint32_t v; memcpy(&v, p, 4); kv->u = v; } break;
    case 5: { int32_t v; memcpy(&v, p, 4); kv->u = (uint64_t)(int64_t)v; } break;
    case 6: { float v; memcpy(&v, p, 4); kv->f = v; } break;
    case 7: kv->u = p[0]; break;
    case 10: case 11: memcpy(&kv->u, p, 8); break;
    case 12: memcpy(&kv->f, p, 8); break;
    }
}

int orc_gguf_open(orc_gguf *g, const char *path) {
    memset(g, 0, sizeof *g);
    int fd = open(path, O_RDONLY);
    if (fd < 0) return -1;
    struct stat st;
    if (fstat(fd, &st) != 0) { close(fd); return -1; }
    g->size = (size_t)st.st_size;
    g->map = mmap(NULL, g->size, PROT_READ, MAP_PRIVATE, fd, 0);
    close(fd);
    if (g->map == MAP_FAILED) { g->map = NULL; return -1; }
    rd r = {g->map, g->map + g->size, 0};
    if (g->size < 24 || memcmp(g->map, "GGUF", 4) != 0) { orc_gguf_close(g); return -2; }
    r.p += 4;
    if (r_u32(&r) != 3) { orc_gguf_close(g); return -3; }
    g->n_tensors = (int)r_u64(&r);
    g->n_kv = (int)r_u64(&r);
    g->t = calloc((size_t)g->n_tensors, sizeof(orc_tinfo));
    g->kv = calloc((size_t)g->n_kv, sizeof(orc_kv));
    for (int i = 0; i < g->n_kv && !r.err; ++i) {
        r_str(&r, g->kv[i].key, sizeof g->kv[i].key);
        g->kv[i].type = (int)r_u32(&r);
        r_value(&r, g->kv[i].type, &g->kv[i]);
    }
    uint32_t align = 32;
    for (int i = 0; i < g->n_kv; ++i)
        if (!strcmp(g->kv[i].key, "general.alignment")) align = (uint32_t)g->kv[i].u;
    for (int i = 0; i < g->n_tensors && !r.err; ++i) {
        orc_tinfo *t = &g->t[i];
        r_str(&r, t->name, sizeof t->name);
        t->n_dims = (int)r_u32(&r);
        for (int d = 0; d < 4; ++d) t->ne[d] = 1;
        for (int d = 0; d < t->n_dims && d < 4; ++d) t->ne[d] = (int64_t)r_u64(&r);
        t->type = (int)r_u32(&r);
        t->offset = r_u64(&r);
    }
    if (r.err) { orc_gguf_close(g); return -4; }
    uint64_t pos = (uint64_t)(r.p - g->map);
    g->data_off = (pos + align - 1) / align * align;
    return 0;
}

void orc_gguf_close(orc_gguf *g) {
    if (g->map) munmap(g->map, g->size);
    free(g->t);
    free(g->kv);
    memset(g, 0, sizeof *g);
}

const orc_tinfo *orc_gguf_find(const orc_gguf *g, const char *name) {
    for (int i = 0; i < g->n_tensors; ++i)
        if (!strcmp(g->t[i].name, name)) return &g->t[i];
    return NULL;
}

float *orc_gguf_f32(const orc_gguf *g, const char *name, int64_t *n_out) {
    const orc_tinfo *t = orc_gguf_find(g, name);
    if (!t) return NULL;
    int64_t n = t->ne[0] * t->ne[1] * t->ne[2] * t->ne[3];
    float *out = malloc((size_t)n * sizeof(float));
    const uint8_t *src = g->map + g->data_off + t->offset;
    if (t->type == 0) memcpy(out, src, (size_t)n * 4);
    else if (t->type == 1) {
        for (int64_t i = 0; i < n; ++i) { uint16_t h; memcpy(&h, src + 2 * i, 2); out[i] = orc_f16_to_f32(h); }
    } else if (t->type == 8) {
        for (int64_t b = 0; b < n / 32; ++b) {
            const uint8_t *blk = src + b * 34;
            uint16_t h; memcpy(&h, blk, 2);
            const float d = orc_f16_to_f32(h);
            for (int i = 0; i < 32; ++i) out[b * 32 + i] = (float)(int8_t)blk[2 + i] * d;
        }
    } else if (t->type == 2) {  // Q4_0 (dequantize_row_q4_0): byte j = q_j | q_{j+16} << 4, value (q - 8) d
        for (int64_t b = 0; b < n / 32; ++b) {
            const uint8_t *blk = src + b * 18;
            uint16_t h; memcpy(&h, blk, 2);
            const float d = orc_f16_to_f32(h);
            for (int j = 0; j < 16; ++j) {
                out[b * 32 + j] = (float)((int)(blk[2 + j] & 0x0F) - 8) * d;
                out[b * 32 + j + 16] = (float)((int)(blk[2 + j] >> 4) - 8) * d;
            }
        }
    } else { free(out); return NULL; }
    if (n_out) *n_out = n;
    return out;
}

int64_t orc_gguf_u32(const orc_gguf *g, const char *key, int64_t def) {
    for (int i = 0; i < g->n_kv; ++i)
        if (!strcmp(g->kv[i].key, key)) return (int64_t)g->kv[i].u;
    return def;
}

double orc_gguf_f32kv(const orc_gguf *g, const char *key, double def) {
    for (int i = 0; i < g->n_kv; ++i)
        if (!strcmp(g->kv[i].key, key)) return g->kv[i].f;
    return def;
}
