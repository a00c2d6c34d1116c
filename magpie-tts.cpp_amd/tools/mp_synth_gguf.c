// mp_synth_gguf — deterministic synthetic GGUF writer for Magpie-357M and the
// NeMo nano-codec, with the exact tensor names, shapes and dtypes the reference
// loader maps (magpie.cpp:572-672, nano-codec.cpp:84-199) and the file layout its
// converters emit (scripts/convert_magpie_to_gguf.py:380-423,
// scripts/convert_codec_to_gguf.py:230-280).
//
// No real weights exist offline, so every parity test and every
// bench runs on these files. The generator is counter-based: element i of tensor
// `name` depends only on (seed, name, i), so the GPU box regenerates identical
// bytes from the seed instead of shipping ~1 GB of weights.
//
// usage: mp_synth_gguf magpie|codec OUT.gguf [--seed S] [--dtype f32|q8_0|q4_0|f16]
//                      [--dec-layers N] [--enc-layers N] [--dec-pos P] [--eos-bias V]
//                      [--lt-head-scale K]  (LT output head weights N(0, (0.02 K)^2): decisive logits)
//                      [--audio-bos N]      (the 8 special audio ids from N, EOS = N + 1; default 2016)
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

enum { T_F32 = 0, T_F16 = 1, T_Q4_0 = 2, T_Q8_0 = 8 };
enum { KV_U32 = 4, KV_F32 = 6, KV_STR = 8 };

static uint64_t g_seed = 0x4D414750ull;  // "MAGP"
static float g_eos_bias = 0.f;            // test-only: added to out_proj[3].bias[audio_eos]
static int g_audio_bos = 2016;            // test-only (--audio-bos): the 8 special ids' first; EOS = +1
static float g_lt_head_scale = 1.f;       // LT output heads std = 0.02 * this

static uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
static uint64_t fnv1a64(const char *s) {
    uint64_t h = 0xcbf29ce484222325ull;
    for (; *s; ++s) { h ^= (unsigned char)*s; h *= 0x100000001b3ull; }
    return h;
}
static double unif(uint64_t key, uint64_t i) {  // [0,1)
    return (double)(splitmix64(key + i) >> 11) * (1.0 / 9007199254740992.0);
}
static double gauss(uint64_t key, uint64_t i) {
    double u1 = ((double)(splitmix64(key + 2 * i) >> 11) + 1.0) * (1.0 / 9007199254740992.0);
    double u2 = unif(key, 2 * i + 1);
    return sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
}

// float -> IEEE half, round-to-nearest-even (numpy astype(float16) semantics)
static uint16_t f32_to_f16(float f) {
    uint32_t x; memcpy(&x, &f, 4);
    uint32_t sign = (x >> 16) & 0x8000u;
    uint32_t mant = x & 0x7FFFFFu;
    int32_t exp = (int32_t)((x >> 23) & 0xFF);
    if (exp == 0xFF) return (uint16_t)(sign | 0x7C00u | (mant ? 0x200u : 0));
    int32_t e = exp - 127 + 15;
    if (e >= 31) return (uint16_t)(sign | 0x7C00u);
    if (e <= 0) {
        if (e < -10) return (uint16_t)sign;
        mant |= 0x800000u;
        uint32_t shift = (uint32_t)(14 - e);
        uint32_t half = mant >> shift;
        uint32_t rem = mant & ((1u << shift) - 1u), mid = 1u << (shift - 1);
        if (rem > mid || (rem == mid && (half & 1u))) half++;
        return (uint16_t)(sign | half);
    }
    uint32_t half = ((uint32_t)e << 10) | (mant >> 13);
    uint32_t rem = mant & 0x1FFFu;
    if (rem > 0x1000u || (rem == 0x1000u && (half & 1u))) half++;
    return (uint16_t)(sign | half);
}
static float f16_to_f32(uint16_t h) {
    uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t exp = (h >> 10) & 0x1Fu, mant = h & 0x3FFu, x;
    if (exp == 0) {
        if (!mant) x = sign;
        else { exp = 127 - 15 + 1; while (!(mant & 0x400u)) { mant <<= 1; exp--; } mant &= 0x3FFu; x = sign | (exp << 23) | (mant << 13); }
    } else if (exp == 31) x = sign | 0x7F800000u | (mant << 13);
    else x = sign | ((exp - 15 + 127) << 23) | (mant << 13);
    float f; memcpy(&f, &x, 4); return f;
}

// ---------------------------------------------------------------- tensor plan
typedef struct {
    char name[96];
    int n_dims;
    int64_t shape[4];  // PyTorch order
    int type;
    int init;          // see fill()
    float p0, p1;
    uint64_t offset;
} tdesc;

enum { I_NORMAL = 0, I_LNW = 1, I_ALPHA = 2, I_FIXED_BASE = 3, I_FIXED_LEVELS = 4 };

static tdesc *g_t = NULL;
static int g_nt = 0, g_cap = 0;

static void add(const char *name, int nd, int64_t a, int64_t b, int64_t c, int type, int init, float p0, float p1) {
    if (g_nt == g_cap) { g_cap = g_cap ? 2 * g_cap : 256; g_t = realloc(g_t, sizeof(tdesc) * (size_t)g_cap); }
    tdesc *t = &g_t[g_nt++];
    memset(t, 0, sizeof *t);
    snprintf(t->name, sizeof t->name, "%s", name);
    t->n_dims = nd; t->shape[0] = a; t->shape[1] = b; t->shape[2] = c;
    t->type = type; t->init = init; t->p0 = p0; t->p1 = p1;
}
static int64_t nel(const tdesc *t) { int64_t n = 1; for (int i = 0; i < t->n_dims; ++i) n *= t->shape[i]; return n; }
static uint64_t nbytes(const tdesc *t) {
    int64_t n = nel(t);
    if (t->type == T_Q8_0) return (uint64_t)(n / 32) * 34u;
    if (t->type == T_Q4_0) return (uint64_t)(n / 32) * 18u;
    if (t->type == T_F16) return (uint64_t)n * 2u;
    return (uint64_t)n * 4u;
}

// ---------------------------------------------------------------- metadata
typedef struct { char key[64]; int type; uint32_t u; float f; const char *s; } kv_t;
static kv_t g_kv[64];
static int g_nkv = 0;
static void kv_u32(const char *k, uint32_t v) { kv_t *e = &g_kv[g_nkv++]; snprintf(e->key, 64, "%s", k); e->type = KV_U32; e->u = v; }
static void kv_str(const char *k, const char *v) { kv_t *e = &g_kv[g_nkv++]; snprintf(e->key, 64, "%s", k); e->type = KV_STR; e->s = v; }

static void w_u32(FILE *f, uint32_t v) { fwrite(&v, 4, 1, f); }
static void w_i32(FILE *f, int32_t v) { fwrite(&v, 4, 1, f); }
static void w_u64(FILE *f, uint64_t v) { fwrite(&v, 8, 1, f); }
static void w_str(FILE *f, const char *s) { uint64_t n = strlen(s); w_u64(f, n); fwrite(s, 1, n, f); }

// ---------------------------------------------------------------- fill
static void fill_f32(const tdesc *t, float *dst) {
    const int64_t n = nel(t);
    const uint64_t key = fnv1a64(t->name) ^ splitmix64(g_seed);
    switch (t->init) {
    case I_NORMAL:
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < n; ++i) dst[i] = (float)(t->p0 * gauss(key, (uint64_t)i)); break;
    case I_LNW:    for (int64_t i = 0; i < n; ++i) dst[i] = (float)(1.0 + t->p0 * gauss(key, (uint64_t)i)); break;
    case I_ALPHA:  for (int64_t i = 0; i < n; ++i) dst[i] = (float)(t->p0 + (t->p1 - t->p0) * unif(key, (uint64_t)i)); break;
    case I_FIXED_BASE: { const float v[4] = {1, 8, 56, 336}; for (int64_t i = 0; i < n; ++i) dst[i] = v[i & 3]; } break;
    case I_FIXED_LEVELS: { const float v[4] = {8, 7, 6, 6}; for (int64_t i = 0; i < n; ++i) dst[i] = v[i & 3]; } break;
    }
    // EOS-forcing variant for the stop-logic tests: codebook 3 prefers audio EOS
    // once it is no longer forbidden (step >= 4, magpie.cpp:4325)
    if (g_eos_bias != 0.f && !strcmp(t->name, "local_transformer_out_projections.3.bias")) dst[g_audio_bos + 1] += g_eos_bias;
}

// Q8_0 exactly as scripts/convert_magpie_to_gguf.py:79-104 (numpy): fp16 scale =
// amax/127, q = round-half-even(x / f32(scale)), int8 wrap on overflow.
static void quant_q8_0(const float *x, int64_t n, uint8_t *out) {
    for (int64_t b = 0; b < n / 32; ++b) {
        const float *blk = x + b * 32;
        float amax = 0.f;
        for (int i = 0; i < 32; ++i) { float a = fabsf(blk[i]); if (a > amax) amax = a; }
        uint16_t hs = f32_to_f16(amax != 0.f ? amax / 127.0f : 0.f);
        float s = f16_to_f32(hs);
        uint8_t *o = out + b * 34;
        memcpy(o, &hs, 2);
        for (int i = 0; i < 32; ++i) {
            int q = 0;
            if (s != 0.f) q = (int)nearbyintf(blk[i] / s);
            o[2 + i] = (uint8_t)(int8_t)q;
        }
    }
}

// Q4_0 exactly as scripts/convert_magpie_to_gguf.py:107-138 (numpy): fp16 scale =
// amax/7, q = clip(round-half-even(x / f32(scale)), -8, 7) + 8, byte j = q_j | q_{j+16} << 4.
static void quant_q4_0(const float *x, int64_t n, uint8_t *out) {
    for (int64_t b = 0; b < n / 32; ++b) {
        const float *blk = x + b * 32;
        float amax = 0.f;
        for (int i = 0; i < 32; ++i) { float a = fabsf(blk[i]); if (a > amax) amax = a; }
        uint16_t hs = f32_to_f16(amax != 0.f ? amax / 7.0f : 0.f);
        float s = f16_to_f32(hs);
        uint8_t *o = out + b * 18, qv[32];
        memcpy(o, &hs, 2);
        for (int i = 0; i < 32; ++i) {
            int q = 0;
            if (s != 0.f) q = (int)nearbyintf(blk[i] / s);
            q = q < -8 ? -8 : q > 7 ? 7 : q;
            qv[i] = (uint8_t)(q + 8);
        }
        for (int j = 0; j < 16; ++j) o[2 + j] = (uint8_t)((qv[j] & 0x0F) | (qv[j + 16] << 4));
    }
}

static int should_q8(const char *name) {
    // scripts/convert_magpie_to_gguf.py:155-176 default patterns
    if (strstr(name, ".self_attention.qkv_net.weight") || strstr(name, ".self_attention.o_net.weight")) return 1;
    if (strstr(name, ".cross_attention.q_net.weight") || strstr(name, ".cross_attention.kv_net.weight") ||
        strstr(name, ".cross_attention.o_net.weight")) return 1;
    if (!strcmp(name, "final_proj.weight")) return 1;
    if (!strncmp(name, "local_transformer_out_projections.", 34) && strstr(name, ".weight")) return 1;
    if (!strcmp(name, "local_transformer_in_projection.weight")) return 1;
    return 0;  // pos_ff conv weights: inner dim 1 or 3 < 32 -> stay F32 (convert_magpie_to_gguf.py:311-320)
}
// F16 (convert_magpie_to_gguf.py:155-176, 311-322): the same pattern set plus the
// pos_ff conv weights (F16 has no block constraint), tensors of >= 256 elements
static int should_f16(const char *name) {
    if (strstr(name, ".pos_ff.proj.conv.weight") || strstr(name, ".pos_ff.o_net.conv.weight")) return 1;
    return should_q8(name);
}

// ---------------------------------------------------------------- plans
static void plan_magpie(int dtype, int dec_layers, int enc_layers, int dec_pos) {
    const float S = 0.02f;
    char nm[128];
#define MAT(nmv, a, b) add(nmv, 2, a, b, 1, T_F32, I_NORMAL, S, 0)
#define MAT3(nmv, a, b, c) add(nmv, 3, a, b, c, T_F32, I_NORMAL, S, 0)
#define VEC(nmv, a) add(nmv, 1, a, 1, 1, T_F32, I_NORMAL, S, 0)
#define LNW(nmv, a) add(nmv, 1, a, 1, 1, T_F32, I_LNW, S, 0)
    MAT("text_embedding.weight", 2380, 768);
    MAT("encoder.position_embeddings.weight", 4096, 768);
    for (int l = 0; l < enc_layers; ++l) {
        snprintf(nm, sizeof nm, "encoder.layers.%d.norm_self.weight", l); LNW(nm, 768);
        snprintf(nm, sizeof nm, "encoder.layers.%d.self_attention.qkv_net.weight", l); MAT(nm, 2304, 768);
        snprintf(nm, sizeof nm, "encoder.layers.%d.self_attention.o_net.weight", l); MAT(nm, 768, 768);
        snprintf(nm, sizeof nm, "encoder.layers.%d.norm_pos_ff.weight", l); LNW(nm, 768);
        snprintf(nm, sizeof nm, "encoder.layers.%d.pos_ff.proj.conv.weight", l); MAT3(nm, 3072, 768, 3);
        snprintf(nm, sizeof nm, "encoder.layers.%d.pos_ff.o_net.conv.weight", l); MAT3(nm, 768, 3072, 3);
    }
    LNW("encoder.norm_out.weight", 768);
    MAT("decoder.position_embeddings.weight", dec_pos, 768);
    for (int l = 0; l < dec_layers; ++l) {
        snprintf(nm, sizeof nm, "decoder.layers.%d.norm_self.weight", l); LNW(nm, 768);
        snprintf(nm, sizeof nm, "decoder.layers.%d.self_attention.qkv_net.weight", l); MAT(nm, 2304, 768);
        snprintf(nm, sizeof nm, "decoder.layers.%d.self_attention.o_net.weight", l); MAT(nm, 768, 768);
        snprintf(nm, sizeof nm, "decoder.layers.%d.norm_xattn_query.weight", l); LNW(nm, 768);
        snprintf(nm, sizeof nm, "decoder.layers.%d.cross_attention.q_net.weight", l); MAT(nm, 128, 768);
        snprintf(nm, sizeof nm, "decoder.layers.%d.cross_attention.kv_net.weight", l); MAT(nm, 256, 768);
        snprintf(nm, sizeof nm, "decoder.layers.%d.cross_attention.o_net.weight", l); MAT(nm, 768, 128);
        snprintf(nm, sizeof nm, "decoder.layers.%d.norm_xattn_memory.weight", l); LNW(nm, 768);
        snprintf(nm, sizeof nm, "decoder.layers.%d.norm_pos_ff.weight", l); LNW(nm, 768);
        snprintf(nm, sizeof nm, "decoder.layers.%d.pos_ff.proj.conv.weight", l); MAT3(nm, 3072, 768, 1);
        snprintf(nm, sizeof nm, "decoder.layers.%d.pos_ff.o_net.conv.weight", l); MAT3(nm, 768, 3072, 1);
    }
    LNW("decoder.norm_out.weight", 768);
    for (int c = 0; c < 8; ++c) { snprintf(nm, sizeof nm, "audio_embeddings.%d.weight", c); MAT(nm, 2024, 768); }
    MAT("baked_context_embedding.weight", 5, 110 * 768);
    MAT("final_proj.weight", 16192, 768);
    VEC("final_proj.bias", 16192);
    MAT("local_transformer_in_projection.weight", 256, 768);
    VEC("local_transformer_in_projection.bias", 256);
    MAT("local_transformer.position_embeddings.weight", 10, 256);
    LNW("local_transformer.layers.0.norm_self.weight", 256);
    MAT("local_transformer.layers.0.self_attention.qkv_net.weight", 768, 256);
    MAT("local_transformer.layers.0.self_attention.o_net.weight", 256, 256);
    LNW("local_transformer.layers.0.norm_pos_ff.weight", 256);
    MAT3("local_transformer.layers.0.pos_ff.proj.conv.weight", 1024, 256, 1);
    MAT3("local_transformer.layers.0.pos_ff.o_net.conv.weight", 256, 1024, 1);
    for (int c = 0; c < 8; ++c) {  // --lt-head-scale: wider logits, so greedy decisions are not near-ties
        snprintf(nm, sizeof nm, "local_transformer_out_projections.%d.weight", c);
        add(nm, 2, 2024, 256, 1, T_F32, I_NORMAL, S * g_lt_head_scale, 0);
        snprintf(nm, sizeof nm, "local_transformer_out_projections.%d.bias", c);
        add(nm, 1, 2024, 1, 1, T_F32, I_NORMAL, S, 0);
    }
    for (int i = 0; i < g_nt; ++i) {
        if ((dtype == T_Q8_0 || dtype == T_Q4_0) && should_q8(g_t[i].name) && nel(&g_t[i]) % 32 == 0)
            g_t[i].type = dtype;
        if (dtype == T_F16 && g_t[i].n_dims >= 2 && nel(&g_t[i]) >= 256 && should_f16(g_t[i].name)) g_t[i].type = T_F16;
    }
    // keys written by the converter (convert_magpie_to_gguf.py:207-230)
    kv_str("general.architecture", "magpie-tts");
    kv_str("general.name", "magpie-357m-synthetic");
    kv_u32("magpie.sample_rate", 22050);
    kv_u32("magpie.num_codebooks", 8);
    kv_u32("magpie.codebook_size", 2016);
    kv_u32("magpie.vocab_size_per_codebook", 2024);
    kv_u32("magpie.text_vocab_size", 2380);
    kv_u32("magpie.d_model", 768);
    kv_u32("magpie.d_ffn", 3072);
    kv_u32("magpie.encoder_layers", 6);
    kv_u32("magpie.decoder_layers", 12);
    kv_u32("magpie.text_bos_id", 2378);
    kv_u32("magpie.text_eos_id", 2379);
    // synthetic text front end (the real one ships NeMo's IPA vocabulary and CMU-style
    // dictionary as magpie.tokenizer.vocab / .dict): ids 0-25 upper-case letters
    // (out-of-dictionary fallback), 26-31 punctuation, IPA symbols (some multi-byte,
    // some two-symbol tokens for the longest-match rule), 93 space, 94 pad, 95 oov
    {
        static const char *ipa[] = {"a", "b", "d", "e", "f", "h", "i", "j", "k", "l", "m", "n", "o", "p", "r",
                                    "s", "t", "u", "v", "w", "z", "\xc9\x99" /*ə*/, "\xc9\xaa" /*ɪ*/,
                                    "\xca\x8a" /*ʊ*/, "\xc9\x9b" /*ɛ*/, "\xc3\xa6" /*æ*/, "\xc9\x91" /*ɑ*/,
                                    "\xc9\x94" /*ɔ*/, "\xca\x83" /*ʃ*/, "\xca\x92" /*ʒ*/, "\xce\xb8" /*θ*/,
                                    "\xc3\xb0" /*ð*/, "\xc5\x8b" /*ŋ*/, "\xcb\x88" /*ˈ*/, "\xcb\x8c" /*ˌ*/,
                                    "\xc9\xb9" /*ɹ*/, "\xc9\x9d" /*ɝ*/, "\xc9\x9a" /*ɚ*/, "o\xca\x8a" /*oʊ*/,
                                    "a\xc9\xaa" /*aɪ*/, "e\xc9\xaa" /*eɪ*/, "a\xca\x8a" /*aʊ*/,
                                    "\xc9\x94\xc9\xaa" /*ɔɪ*/, "t\xca\x83" /*tʃ*/, "d\xca\x92" /*dʒ*/, "'", "-"};
        static char vocab[4096];
        size_t n = 0;
        const int nipa = (int)(sizeof ipa / sizeof ipa[0]);
        for (int id = 0; id < 96; ++id) {
            char tok[32];
            if (id < 26) snprintf(tok, sizeof tok, "%c", 'A' + id);
            else if (id < 32) snprintf(tok, sizeof tok, "%c", ",.!?:;"[id - 26]);
            else if (id - 32 < nipa) snprintf(tok, sizeof tok, "%s", ipa[id - 32]);
            else if (id == 93) snprintf(tok, sizeof tok, " ");
            else if (id == 94) snprintf(tok, sizeof tok, "<pad>");
            else if (id == 95) snprintf(tok, sizeof tok, "<oov>");
            else snprintf(tok, sizeof tok, "<unused%d>", id);
            n += (size_t)snprintf(vocab + n, sizeof vocab - n, id ? "\n%s" : "%s", tok);
        }
        kv_str("magpie.tokenizer.vocab", vocab);
        kv_str("magpie.tokenizer.dict",
               "hello\th\xc9\x99\xcb\x88lo\xca\x8a\n"            /* həˈloʊ */
               "world\tw\xcb\x88\xc9\x9dld\n"                      /* wˈɝld */
               "the\t\xc3\xb0\xc9\x99\n"                           /* ðə */
               "and\t\xc3\xa6nd\n"                                  /* ænd */
               "twenty\tt w\xcb\x88\xc9\x9bnti\n"                  /* a space inside: no token, skipped */
               "four\tf\xcb\x88\xc9\x94\xc9\xb9\n"                /* fˈɔɹ */
               "dollars\td\xcb\x88\xc9\x91l\xc9\x9az\n"          /* dˈɑlɚz */
               "percent\tp\xc9\x9a\xcb\x88s\xc9\x9bnt\n"         /* pɚˈsɛnt */
               "first\tf\xcb\x88\xc9\x9dst\n"                      /* fˈɝst */
               "voice\tv\xcb\x88\xc9\x94\xc9\xaas\n"             /* vˈɔɪs */
               "joy\td\xca\x92\xcb\x88\xc9\x94\xc9\xaa\xe2\x82\xac");  /* dʒˈɔɪ + an unknown 3-byte char */
        kv_u32("magpie.tokenizer.space", 93);
        kv_u32("magpie.tokenizer.pad", 94);
        kv_u32("magpie.tokenizer.oov", 95);
    }
    kv_u32("magpie.audio_bos_id", (uint32_t)g_audio_bos);
    kv_u32("magpie.audio_eos_id", (uint32_t)g_audio_bos + 1);
    // keys the reader actually honours (magpie.cpp:85-120); only written when a
    // reduced test model deviates from the struct defaults
    if (dec_layers != 12) kv_u32("magpie.dec_layers", (uint32_t)dec_layers);
    if (enc_layers != 6) kv_u32("magpie.enc_layers", (uint32_t)enc_layers);
}

// Residual-block conv gain. 1/sqrt(C*k) (gain 1) makes the 45-conv residual
// stack of the synthetic codec chaotic: flipping the accumulation order alone
// moves the waveform by 6e-3. 0.6 keeps the signal healthy (std ~0.13) with
// rounding sensitivity ~3e-4, closer to a trained vocoder's conditioning.
#ifndef RB_GAIN
#define RB_GAIN 0.6
#endif

static void plan_codec(void) {
    char nm[128];
    const int chans[6] = {864, 432, 216, 108, 54, 27};
    const int rates[5] = {8, 8, 4, 2, 2};
    const int ks[3] = {3, 7, 11};
    add("dec.pre.weight", 3, 864, 32, 7, T_F32, I_NORMAL, (float)(1.0 / sqrt(32.0 * 7.0)), 0);
    add("dec.pre.bias", 1, 864, 1, 1, T_F32, I_NORMAL, 0.02f, 0);
    for (int i = 0; i < 5; ++i) {
        const int cin = chans[i], cout = chans[i + 1], K = 2 * rates[i];
        snprintf(nm, sizeof nm, "dec.act.%d.activation.snake_act.alpha", i);
        add(nm, 3, 1, cin / 2, 1, T_F32, I_ALPHA, 0.5f, 1.5f);
        snprintf(nm, sizeof nm, "dec.up.%d.c.weight", i);
        add(nm, 3, cin, 1, K, T_F32, I_NORMAL, 0.5f, 0);
        snprintf(nm, sizeof nm, "dec.up.%d.c.bias", i);
        add(nm, 1, cout, 1, 1, T_F32, I_NORMAL, 0.02f, 0);
        for (int j = 0; j < 3; ++j)
            for (int k = 0; k < 3; ++k) {
                const float ws = (float)(RB_GAIN / sqrt((double)cout * ks[j]));
                snprintf(nm, sizeof nm, "dec.rl.%d.rb.%d.rb.%d.in_act.alpha", i, j, k);
                add(nm, 3, 1, cout / 2, 1, T_F32, I_ALPHA, 0.5f, 1.5f);
                snprintf(nm, sizeof nm, "dec.rl.%d.rb.%d.rb.%d.in_conv.weight", i, j, k);
                add(nm, 3, cout, cout, ks[j], T_F32, I_NORMAL, ws, 0);
                snprintf(nm, sizeof nm, "dec.rl.%d.rb.%d.rb.%d.in_conv.bias", i, j, k);
                add(nm, 1, cout, 1, 1, T_F32, I_NORMAL, 0.02f, 0);
                snprintf(nm, sizeof nm, "dec.rl.%d.rb.%d.rb.%d.sk_act.alpha", i, j, k);
                add(nm, 3, 1, cout / 2, 1, T_F32, I_ALPHA, 0.5f, 1.5f);
                snprintf(nm, sizeof nm, "dec.rl.%d.rb.%d.rb.%d.sk_conv.weight", i, j, k);
                add(nm, 3, cout, cout, ks[j], T_F32, I_NORMAL, ws, 0);
                snprintf(nm, sizeof nm, "dec.rl.%d.rb.%d.rb.%d.sk_conv.bias", i, j, k);
                add(nm, 1, cout, 1, 1, T_F32, I_NORMAL, 0.02f, 0);
            }
    }
    add("dec.post_act.alpha", 3, 1, 13, 1, T_F32, I_ALPHA, 0.5f, 1.5f);
    // 0.2x: keeps the synthetic waveform out of tanh saturation (pre-tanh std ~0.35),
    // so waveform parity is measured where the output still depends on its input.
    add("dec.post.weight", 3, 1, 27, 3, T_F32, I_NORMAL, (float)(0.2 / sqrt(27.0 * 3.0)), 0);
    add("dec.post.bias", 1, 1, 1, 1, T_F32, I_NORMAL, 0.02f, 0);
    for (int i = 0; i < 8; ++i) {
        snprintf(nm, sizeof nm, "vq.fsqs.%d.dim_base_index", i);
        add(nm, 3, 1, 4, 1, T_F32, I_FIXED_BASE, 0, 0);
        snprintf(nm, sizeof nm, "vq.fsqs.%d.num_levels", i);
        add(nm, 3, 1, 4, 1, T_F32, I_FIXED_LEVELS, 0, 0);
    }
    kv_str("general.architecture", "nano-codec");
    kv_str("general.name", "nemo-nano-codec-22khz-synthetic");
    kv_u32("codec.sample_rate", 22050);
    kv_u32("codec.num_codebooks", 8);
    kv_u32("codec.codebook_size", 2016);
    kv_u32("codec.hop_length", 1024);
    kv_u32("codec.latent_dim", 32);
}

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s magpie|codec OUT.gguf [--seed S] [--dtype f32|q8_0|q4_0|f16] "
                        "[--dec-layers N] [--enc-layers N] [--dec-pos P] [--eos-bias V] [--lt-head-scale K] [--audio-bos N]\n", argv[0]);
        return 2;
    }
    const char *kind = argv[1], *out = argv[2];
    int dtype = T_F32, dec_layers = 12, enc_layers = 6, dec_pos = 2048;
    for (int i = 3; i + 1 < argc; i += 2) {
        if (!strcmp(argv[i], "--seed")) g_seed = strtoull(argv[i + 1], NULL, 0);
        else if (!strcmp(argv[i], "--dtype")) dtype = !strcmp(argv[i + 1], "q8_0")   ? T_Q8_0
                                                          : !strcmp(argv[i + 1], "q4_0") ? T_Q4_0
                                                          : !strcmp(argv[i + 1], "f16")  ? T_F16
                                                                                         : T_F32;
        else if (!strcmp(argv[i], "--dec-layers")) dec_layers = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "--enc-layers")) enc_layers = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "--dec-pos")) dec_pos = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "--eos-bias")) g_eos_bias = (float)atof(argv[i + 1]);
        else if (!strcmp(argv[i], "--audio-bos")) g_audio_bos = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "--lt-head-scale")) g_lt_head_scale = (float)atof(argv[i + 1]);
        else { fprintf(stderr, "unknown option %s\n", argv[i]); return 2; }
    }
    if (!strcmp(kind, "magpie")) plan_magpie(dtype, dec_layers, enc_layers, dec_pos);
    else if (!strcmp(kind, "codec")) plan_codec();
    else { fprintf(stderr, "unknown kind %s\n", kind); return 2; }

    uint64_t off = 0;
    for (int i = 0; i < g_nt; ++i) {
        off = (off + 31) & ~(uint64_t)31;
        g_t[i].offset = off;
        off += nbytes(&g_t[i]);
    }
    char tmp[4096];
    snprintf(tmp, sizeof tmp, "%s.tmp", out);
    FILE *f = fopen(tmp, "wb");
    if (!f) { perror(tmp); return 1; }
    fwrite("GGUF", 1, 4, f);
    w_u32(f, 3);
    w_u64(f, (uint64_t)g_nt);
    w_u64(f, (uint64_t)g_nkv);
    for (int i = 0; i < g_nkv; ++i) {
        w_str(f, g_kv[i].key);
        w_i32(f, g_kv[i].type);
        if (g_kv[i].type == KV_U32) w_u32(f, g_kv[i].u);
        else if (g_kv[i].type == KV_F32) fwrite(&g_kv[i].f, 4, 1, f);
        else w_str(f, g_kv[i].s);
    }
    for (int i = 0; i < g_nt; ++i) {
        const tdesc *t = &g_t[i];
        w_str(f, t->name);
        w_u32(f, (uint32_t)t->n_dims);
        for (int d = t->n_dims - 1; d >= 0; --d) w_u64(f, (uint64_t)t->shape[d]);  // ggml order
        w_i32(f, t->type);
        w_u64(f, t->offset);
    }
    long pos = ftell(f);
    while (pos % 32) { fputc(0, f); ++pos; }
    const uint64_t data_start = (uint64_t)pos;
    float *buf = NULL; uint8_t *qbuf = NULL; size_t cap = 0;
    for (int i = 0; i < g_nt; ++i) {
        const tdesc *t = &g_t[i];
        const int64_t n = nel(t);
        if ((size_t)n > cap) { cap = (size_t)n; buf = realloc(buf, cap * 4); qbuf = realloc(qbuf, cap * 4); }
        fill_f32(t, buf);
        while ((uint64_t)ftell(f) < data_start + t->offset) fputc(0, f);
        if (t->type == T_F32) fwrite(buf, 4, (size_t)n, f);
        else if (t->type == T_F16) {
            uint16_t *h = (uint16_t *)qbuf;
            for (int64_t k = 0; k < n; ++k) h[k] = f32_to_f16(buf[k]);
            fwrite(h, 2, (size_t)n, f);
        } else {
            if (t->type == T_Q4_0) quant_q4_0(buf, n, qbuf);
            else quant_q8_0(buf, n, qbuf);
            fwrite(qbuf, 1, nbytes(t), f);
        }
    }
    free(buf); free(qbuf);
    if (fclose(f) != 0) { perror("fclose"); return 1; }
    if (rename(tmp, out) != 0) { perror("rename"); return 1; }
    fprintf(stderr, "mp_synth_gguf: wrote %s (%d tensors, %.1f MB)\n", out, g_nt, (double)(data_start + off) / 1e6);
    return 0;
}
