// magpie_oracle.c — CPU restatement of m1el/magpie-tts.cpp's decode path and
// nano-codec decoder. *** TEST INFRASTRUCTURE ONLY *** (see magpie_oracle.h).
//
// Every function cites the reference lines it restates. Arithmetic spec:
// SURVEY.md Appendix A. Tensors are stored f32 between ops (as ggml does); the
// accumulation precision is selectable (orc_set_mode).
#include "magpie_oracle.h"

#include <math.h>
#include <omp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "gguf_min.h"

static int g_acc64 = 1;
static int g_gelu_f16 = 0;

void orc_set_mode(int acc64, int gelu_f16, int n_threads) {
    g_acc64 = acc64;
    g_gelu_f16 = gelu_f16;
    if (n_threads > 0) omp_set_num_threads(n_threads);
}

static double now_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

// ------------------------------------------------------------------ primitives
static double dot64(const float *a, const float *b, int n) {
    double s = 0.0;
    for (int i = 0; i < n; ++i) s += (double)a[i] * (double)b[i];
    return s;
}
static float dot32(const float *a, const float *b, int n) {
    float s[8] = {0};
    int i = 0;
    for (; i + 8 <= n; i += 8)
        for (int j = 0; j < 8; ++j) s[j] += a[i + j] * b[i + j];
    float r = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
    for (; i < n; ++i) r += a[i] * b[i];
    return r;
}
static inline double dotp(const float *a, const float *b, int n) { return g_acc64 ? dot64(a, b, n) : (double)dot32(a, b, n); }

// Y[m][n] = sum_k W[n][k] * X[m][k] (+ bias[n]); ggml_mul_mat(W, X) (+ ggml_add)
static void matmul(const float *W, const float *bias, const float *X, float *Y, int M, int N, int K) {
#pragma omp parallel for schedule(static) if ((long)N * K * M > 200000)
    for (int n = 0; n < N; ++n) {
        const float *w = W + (size_t)n * K;
        for (int m = 0; m < M; ++m) {
            double v = dotp(w, X + (size_t)m * K, K);
            if (bias) v += bias[n];
            Y[(size_t)m * N + n] = (float)v;
        }
    }
}

// ------------------------------------------------------------------ Q8_0 (weight mode 2)
// A Q8_0 tensor of the GGUF (scripts/convert_magpie_to_gguf.py:79-104: per 32
// weights an fp16 scale d and 32 int8 q, value q*d) kept as stored.
typedef struct {
    const float *w;  // the dequantised f32 copy this entry shadows (lookup key)
    int8_t *q;       // [N][K]
    float *d;        // [N][K/32] (fp16 values, exact in f32)
} q8w_t;

// ggml's Q8_0 mul_mat (assumed; ggml is absent here): the activation
// row is itself quantised to Q8_0 (quantize_row_q8_0_ref: d = amax/127,
// id = 1/d, q = roundf(x*id), d stored as fp16), then per block the exact
// integer dot is scaled by d_w*d_a and the blocks are summed
// (ggml_vec_dot_q8_0_q8_0: sumf += sumi*(d_w*d_a)).
static void quant_row_q8(const float *x, int K, int8_t *q, float *d) {
    for (int b = 0; b < K / 32; ++b) {
        float amax = 0.f;
        for (int j = 0; j < 32; ++j) amax = fmaxf(amax, fabsf(x[b * 32 + j]));
        const float dd = amax / 127.0f;
        const float id = dd != 0.f ? 1.0f / dd : 0.0f;
        d[b] = orc_f16_to_f32(orc_f32_to_f16(dd));
        for (int j = 0; j < 32; ++j) q[b * 32 + j] = (int8_t)roundf(x[b * 32 + j] * id);
    }
}

// the exact integer dot of one weight block with one activation block (the sumi of
// ggml_vec_dot_q8_0_q8_0 / vec_dot_q4_0_q8_0, Q4_0 weights as q - 8)
static int block_dot_q8(const int8_t *wq, const int8_t *aq) {
    int s = 0;
    for (int j = 0; j < 32; ++j) s += (int)wq[j] * (int)aq[j];
    return s;
}

// a GGUF tensor's Q8_0 (type 8: fp16 d + 32 int8) or Q4_0 (type 2: fp16 d + 16 bytes,
// byte j = q_j | q_{j+16} << 4, value (q - 8) d) blocks as int8 values + f32 scales
static void unpack_qblocks(const uint8_t *src, int type, int64_t n, int8_t *q, float *d) {
    for (int64_t b = 0; b < n / 32; ++b) {
        uint16_t h;
        if (type == 8) {
            memcpy(&h, src + b * 34, 2);
            memcpy(q + b * 32, src + b * 34 + 2, 32);
        } else {  // Q4_0 as ggml's vec_dot_q4_0_q8_0 reads it: (nibble - 8), same integer dot
            const uint8_t *blk = src + b * 18;
            memcpy(&h, blk, 2);
            for (int j = 0; j < 16; ++j) {
                q[b * 32 + j] = (int8_t)((blk[2 + j] & 0x0F) - 8);
                q[b * 32 + j + 16] = (int8_t)((blk[2 + j] >> 4) - 8);
            }
        }
        d[b] = orc_f16_to_f32(h);
    }
}

static void matmul_q8(const q8w_t *W, const float *bias, const float *X, float *Y, int M, int N, int K) {
    const int nb = K / 32;
    int8_t *xq = malloc((size_t)M * K);
    float *xd = malloc(sizeof(float) * (size_t)M * nb);
    for (int m = 0; m < M; ++m) quant_row_q8(X + (size_t)m * K, K, xq + (size_t)m * K, xd + (size_t)m * nb);
#pragma omp parallel for schedule(static) if ((long)N * K * M > 200000)
    for (int n = 0; n < N; ++n) {
        const int8_t *wq = W->q + (size_t)n * K;
        const float *wd = W->d + (size_t)n * nb;
        for (int m = 0; m < M; ++m) {
            const int8_t *aq = xq + (size_t)m * K;
            const float *ad = xd + (size_t)m * nb;
            double v64 = 0.0;
            float v32 = 0.f;
            for (int b = 0; b < nb; ++b) {
                const int s = block_dot_q8(wq + b * 32, aq + b * 32);
                if (g_acc64) v64 += (double)s * ((double)wd[b] * (double)ad[b]);
                else v32 += (float)s * (wd[b] * ad[b]);
            }
            float v = g_acc64 ? (float)v64 : v32;
            if (bias) v = v + bias[n];
            Y[(size_t)m * N + n] = v;
        }
    }
    free(xq);
    free(xd);
}

// f32 -> bf16 -> f32, round-to-nearest-even (ggml_compute_fp32_to_bf16)
static float bf16r(float x) {
    uint32_t u;
    memcpy(&u, &x, 4);
    if ((u & 0x7fffffff) > 0x7f800000) u = (u | 0x00400000) & 0xffff0000u;  // NaN stays NaN
    else u = (u + (0x7fff + ((u >> 16) & 1))) & 0xffff0000u;
    memcpy(&x, &u, 4);
    return x;
}
static float *bf16_copy(const float *w, size_t n) {
    float *r = malloc(sizeof(float) * n);
    for (size_t i = 0; i < n; ++i) r[i] = bf16r(w[i]);
    return r;
}

// ggml_norm(eps) * w (magpie.cpp:2237-2259): mean/var accumulated in double.
static void layernorm(const float *x, const float *w, float *y, int K, float eps) {
    double s = 0.0;
    for (int i = 0; i < K; ++i) s += x[i];
    const double mean = s / K;
    double v = 0.0;
    for (int i = 0; i < K; ++i) { double d = (double)x[i] - mean; v += d * d; }
    v /= K;
    if (g_acc64) {
        const double sc = 1.0 / sqrt(v + (double)eps);
        for (int i = 0; i < K; ++i) y[i] = (float)(((double)x[i] - mean) * sc * (double)w[i]);
    } else {
        const float sc = 1.0f / sqrtf((float)v + eps);
        for (int i = 0; i < K; ++i) y[i] = ((x[i] - (float)mean) * sc) * w[i];
    }
}
static void layernorm_rows(const float *x, const float *w, float *y, int M, int K, float eps) {
    for (int m = 0; m < M; ++m) layernorm(x + (size_t)m * K, w, y + (size_t)m * K, K, eps);
}

// ggml_gelu: tanh approximation (GELU_COEF_A = 0.044715, sqrt(2/pi)).
static float gelu1(float x) {
    if (g_gelu_f16) {  // ggml-CPU fp16 table semantics (A.7; assumed, unverifiable here)
        if (x <= -10.0f) return 0.0f;
        if (x >= 10.0f) return x;
        float xh = orc_f16_to_f32(orc_f32_to_f16(x));
        float r = 0.5f * xh * (1.0f + tanhf(0.79788456080286535588f * xh * (1.0f + 0.044715f * xh * xh)));
        return orc_f16_to_f32(orc_f32_to_f16(r));
    }
    if (g_acc64) {
        double d = x;
        return (float)(0.5 * d * (1.0 + tanh(0.79788456080286535588 * d * (1.0 + 0.044715 * d * d))));
    }
    return 0.5f * x * (1.0f + tanhf(0.79788456080286535588f * x * (1.0f + 0.044715f * x * x)));
}
static void gelu_inplace(float *x, size_t n) {
    for (size_t i = 0; i < n; ++i) x[i] = gelu1(x[i]);
}

// softmax(scale * s[0..n)) written back into p (ggml_scale + ggml_soft_max).
static void softmax_scaled(const double *s, double *p, int n, double scale) {
    double mx = -INFINITY;
    for (int j = 0; j < n; ++j) if (s[j] * scale > mx) mx = s[j] * scale;
    double sum = 0.0;
    for (int j = 0; j < n; ++j) { p[j] = exp(s[j] * scale - mx); sum += p[j]; }
    for (int j = 0; j < n; ++j) p[j] /= sum;
}

// One head of attention for one query: out[d] = sum_j softmax(q.k_j * scale) v_j[d].
// K/V rows at stride `ld` floats, head slice starts at the pointers.
static void attend(const float *q, const float *K, const float *V, int nkeys, int ld, int dh, double scale,
                   float *out, double *sbuf, double *pbuf) {
    for (int j = 0; j < nkeys; ++j) sbuf[j] = dotp(q, K + (size_t)j * ld, dh);
    softmax_scaled(sbuf, pbuf, nkeys, scale);
    for (int d = 0; d < dh; ++d) {
        double a = 0.0;
        for (int j = 0; j < nkeys; ++j) a += pbuf[j] * (double)V[(size_t)j * ld + d];
        out[d] = (float)a;
    }
}

// ------------------------------------------------------------------ model
typedef struct {
    float *norm_self, *qkv, *o, *norm_ff, *ff1, *ff2;  // encoder layer
} enc_layer;
typedef struct {
    float *norm_self, *qkv, *o, *norm_xq, *xq, *xkv, *xo, *norm_xmem, *norm_ff, *ff1, *ff2;
    float *qkv_h, *o_h, *ff1_h, *ff2_h;  // bf16-rounded copies (weight mode 1)
} dec_layer;

struct orc_model {
    int d, dff, enc_layers, dec_layers, enc_heads, dec_heads, xa_heads, xa_dh, enc_kernel;
    int lt_dim, lt_ffn, n_cb, vocab_cb, ctx_frames, n_spk;
    int text_bos, text_eos, audio_bos, audio_eos, max_dec_steps;
    float eps;
    int dec_pos_rows;
    float *text_emb, *enc_pos, *enc_norm_out, *dec_pos, *dec_norm_out, *baked;
    float *audio_emb[8];
    enc_layer *enc;
    dec_layer *dec;
    float *lt_in_w, *lt_in_b, *lt_pos, *lt_norm_self, *lt_qkv, *lt_o, *lt_norm_ff, *lt_ff1, *lt_ff2;
    float *lt_out_w[8], *lt_out_b[8];
    // weight mode 1 (bf16 decode projections): rounded copies, NULL in mode 0
    int half;
    float *lt_qkv_h, *lt_o_h, *lt_ff1_h, *lt_ff2_h, *lt_out_w_h[8];
    // weight mode 3 (an F16 file, ggml's F16 mul_mat): the tensors stored F16 (their
    // widened values are exact); every mul_mat with one rounds its src1 to f16
    int f16mode;
    const float **f16w;
    int n_f16, cap_f16;
    // weight mode 2 (ggml Q8_0 mul_mat for the file's Q8_0 tensors): the raw blocks
    int q8mode;
    q8w_t *q8;
    int n_q8, cap_q8;
    float **owned;
    int n_owned, cap_owned;
};

static int is_f16(const orc_model *m, const float *W) {
    if (!m->f16mode) return 0;
    for (int i = 0; i < m->n_f16; ++i)
        if (m->f16w[i] == W) return 1;
    return 0;
}
static float f16r(float x) { return orc_f16_to_f32(orc_f32_to_f16(x)); }
static float *f16_rows(const float *X, size_t n) {
    float *r = malloc(sizeof(float) * n);
    for (size_t i = 0; i < n; ++i) r[i] = f16r(X[i]);
    return r;
}

static const q8w_t *find_q8(const orc_model *m, const float *W) {
    if (!m->q8mode) return NULL;
    for (int i = 0; i < m->n_q8; ++i)
        if (m->q8[i].w == W) return &m->q8[i];
    return NULL;
}

// ggml_mul_mat(W, X) (+ bias) with W's stored type: Q8_0 tensors in weight
// mode 2 take ggml's quantised path, everything else the f32 dot.
static void mm(const orc_model *m, const float *W, const float *bias, const float *X, float *Y, int M, int N, int K) {
    const q8w_t *q = find_q8(m, W);
    if (q) { matmul_q8(q, bias, X, Y, M, N, K); return; }
    if (is_f16(m, W)) {  // ggml F16 mul_mat: src1 rounded to f16 (vec_dot_type F16), products exact in f32
        float *Xh = f16_rows(X, (size_t)M * K);
        matmul(W, bias, Xh, Y, M, N, K);
        free(Xh);
        return;
    }
    matmul(W, bias, X, Y, M, N, K);
}

// Projection in weight mode 1: bf16 weights x bf16-rounded activations,
// products exact, accumulated like matmul() (ggml's BF16 mul_mat rounds src1 to
// its vec_dot_type BF16 the same way). Wh == NULL: mm().
static void matmul_sel(const orc_model *m, const float *W, const float *Wh, const float *bias, const float *X, float *Y,
                       int M, int N, int K) {
    if (!Wh) { mm(m, W, bias, X, Y, M, N, K); return; }
    float *Xh = malloc(sizeof(float) * (size_t)M * K);
    for (size_t i = 0; i < (size_t)M * K; ++i) Xh[i] = bf16r(X[i]);
    matmul(Wh, bias, Xh, Y, M, N, K);
    free(Xh);
}

static float *take(orc_model *m, const orc_gguf *g, const char *name, int *ok) {
    float *p = orc_gguf_f32(g, name, NULL);
    if (!p) { fprintf(stderr, "oracle: missing tensor %s\n", name); *ok = 0; return NULL; }
    if (m->n_owned == m->cap_owned) {
        m->cap_owned = m->cap_owned ? 2 * m->cap_owned : 256;
        m->owned = realloc(m->owned, sizeof(float *) * (size_t)m->cap_owned);
    }
    m->owned[m->n_owned++] = p;
    const orc_tinfo *t = orc_gguf_find(g, name);
    if (t && t->type == 1) {  // F16: remembered for weight mode 3
        if (m->n_f16 == m->cap_f16) {
            m->cap_f16 = m->cap_f16 ? 2 * m->cap_f16 : 128;
            m->f16w = realloc(m->f16w, sizeof(float *) * (size_t)m->cap_f16);
        }
        m->f16w[m->n_f16++] = p;
    }
    if (t && (t->type == 8 || t->type == 2)) {  // keep the stored Q8_0 / Q4_0 blocks for weight mode 2
        const int64_t n = t->ne[0] * t->ne[1] * t->ne[2] * t->ne[3];
        const uint8_t *src = g->map + g->data_off + t->offset;
        if (m->n_q8 == m->cap_q8) {
            m->cap_q8 = m->cap_q8 ? 2 * m->cap_q8 : 64;
            m->q8 = realloc(m->q8, sizeof(q8w_t) * (size_t)m->cap_q8);
        }
        q8w_t *e = &m->q8[m->n_q8++];
        e->w = p;
        e->q = malloc((size_t)n);
        e->d = malloc(sizeof(float) * (size_t)(n / 32));
        unpack_qblocks(src, (int)t->type, n, e->q, e->d);
    }
    return p;
}

int orc_dec_layers(const orc_model *m) { return m->dec_layers; }

// read_hparams (magpie.cpp:73-121) + create_tensors name mapping (magpie.cpp:572-672)
orc_model *orc_load(const char *path) {
    orc_gguf g;
    if (orc_gguf_open(&g, path) != 0) { fprintf(stderr, "oracle: cannot open %s\n", path); return NULL; }
    orc_model *m = calloc(1, sizeof *m);
    m->d = (int)orc_gguf_u32(&g, "magpie.d_model", 768);
    m->dff = (int)orc_gguf_u32(&g, "magpie.d_ffn", 3072);
    m->enc_layers = (int)orc_gguf_u32(&g, "magpie.enc_layers", 6);
    m->enc_heads = (int)orc_gguf_u32(&g, "magpie.enc_heads", 12);
    m->enc_kernel = (int)orc_gguf_u32(&g, "magpie.enc_kernel", 3);
    m->dec_layers = (int)orc_gguf_u32(&g, "magpie.dec_layers", 12);
    m->dec_heads = (int)orc_gguf_u32(&g, "magpie.dec_sa_heads", 12);
    m->xa_heads = (int)orc_gguf_u32(&g, "magpie.dec_xa_heads", 1);
    m->xa_dh = (int)orc_gguf_u32(&g, "magpie.dec_xa_d_head", 128);
    m->lt_dim = (int)orc_gguf_u32(&g, "magpie.lt_dim", 256);
    m->lt_ffn = (int)orc_gguf_u32(&g, "magpie.lt_ffn_dim", 1024);
    m->n_cb = (int)orc_gguf_u32(&g, "magpie.num_codebooks", 8);
    m->vocab_cb = (int)orc_gguf_u32(&g, "magpie.vocab_per_cb", 2024);
    m->n_spk = (int)orc_gguf_u32(&g, "magpie.num_speakers", 5);
    m->ctx_frames = (int)orc_gguf_u32(&g, "magpie.context_frames", 110);
    m->text_bos = (int)orc_gguf_u32(&g, "magpie.text_bos_id", 2378);
    m->text_eos = (int)orc_gguf_u32(&g, "magpie.text_eos_id", 2379);
    m->audio_bos = (int)orc_gguf_u32(&g, "magpie.audio_bos_id", 2016);
    m->audio_eos = (int)orc_gguf_u32(&g, "magpie.audio_eos_id", 2017);
    m->max_dec_steps = (int)orc_gguf_u32(&g, "magpie.max_dec_steps", 500);
    m->eps = (float)orc_gguf_f32kv(&g, "magpie.eps", 1e-5);
    int ok = 1;
    char nm[160];
    m->text_emb = take(m, &g, "text_embedding.weight", &ok);
    m->enc_pos = take(m, &g, "encoder.position_embeddings.weight", &ok);
    m->enc = calloc((size_t)m->enc_layers, sizeof(enc_layer));
    for (int l = 0; l < m->enc_layers; ++l) {
        enc_layer *L = &m->enc[l];
#define T(field, suffix) snprintf(nm, sizeof nm, "encoder.layers.%d.%s", l, suffix); L->field = take(m, &g, nm, &ok)
        T(norm_self, "norm_self.weight");
        T(qkv, "self_attention.qkv_net.weight");
        T(o, "self_attention.o_net.weight");
        T(norm_ff, "norm_pos_ff.weight");
        T(ff1, "pos_ff.proj.conv.weight");
        T(ff2, "pos_ff.o_net.conv.weight");
#undef T
    }
    m->enc_norm_out = take(m, &g, "encoder.norm_out.weight", &ok);
    m->dec_pos = take(m, &g, "decoder.position_embeddings.weight", &ok);
    {
        const orc_tinfo *t = orc_gguf_find(&g, "decoder.position_embeddings.weight");
        m->dec_pos_rows = t ? (int)t->ne[1] : 0;
    }
    m->dec = calloc((size_t)m->dec_layers, sizeof(dec_layer));
    for (int l = 0; l < m->dec_layers; ++l) {
        dec_layer *L = &m->dec[l];
#define T(field, suffix) snprintf(nm, sizeof nm, "decoder.layers.%d.%s", l, suffix); L->field = take(m, &g, nm, &ok)
        T(norm_self, "norm_self.weight");
        T(qkv, "self_attention.qkv_net.weight");
        T(o, "self_attention.o_net.weight");
        T(norm_xq, "norm_xattn_query.weight");
        T(xq, "cross_attention.q_net.weight");
        T(xkv, "cross_attention.kv_net.weight");
        T(xo, "cross_attention.o_net.weight");
        T(norm_xmem, "norm_xattn_memory.weight");
        T(norm_ff, "norm_pos_ff.weight");
        T(ff1, "pos_ff.proj.conv.weight");
        T(ff2, "pos_ff.o_net.conv.weight");
#undef T
    }
    m->dec_norm_out = take(m, &g, "decoder.norm_out.weight", &ok);
    for (int c = 0; c < 8; ++c) {
        snprintf(nm, sizeof nm, "audio_embeddings.%d.weight", c);
        m->audio_emb[c] = take(m, &g, nm, &ok);
    }
    m->baked = take(m, &g, "baked_context_embedding.weight", &ok);
    m->lt_in_w = take(m, &g, "local_transformer_in_projection.weight", &ok);
    m->lt_in_b = take(m, &g, "local_transformer_in_projection.bias", &ok);
    m->lt_pos = take(m, &g, "local_transformer.position_embeddings.weight", &ok);
    m->lt_norm_self = take(m, &g, "local_transformer.layers.0.norm_self.weight", &ok);
    m->lt_qkv = take(m, &g, "local_transformer.layers.0.self_attention.qkv_net.weight", &ok);
    m->lt_o = take(m, &g, "local_transformer.layers.0.self_attention.o_net.weight", &ok);
    m->lt_norm_ff = take(m, &g, "local_transformer.layers.0.norm_pos_ff.weight", &ok);
    m->lt_ff1 = take(m, &g, "local_transformer.layers.0.pos_ff.proj.conv.weight", &ok);
    m->lt_ff2 = take(m, &g, "local_transformer.layers.0.pos_ff.o_net.conv.weight", &ok);
    for (int c = 0; c < 8; ++c) {
        snprintf(nm, sizeof nm, "local_transformer_out_projections.%d.weight", c);
        m->lt_out_w[c] = take(m, &g, nm, &ok);
        snprintf(nm, sizeof nm, "local_transformer_out_projections.%d.bias", c);
        m->lt_out_b[c] = take(m, &g, nm, &ok);
    }
    orc_gguf_close(&g);
    if (!ok || m->d != 768) { orc_free(m); return NULL; }
    return m;
}

static void free_half(orc_model *m) {
    for (int l = 0; l < m->dec_layers; ++l) {
        dec_layer *L = &m->dec[l];
        free(L->qkv_h); free(L->o_h); free(L->ff1_h); free(L->ff2_h);
        L->qkv_h = L->o_h = L->ff1_h = L->ff2_h = NULL;
    }
    free(m->lt_qkv_h); free(m->lt_o_h); free(m->lt_ff1_h); free(m->lt_ff2_h);
    m->lt_qkv_h = m->lt_o_h = m->lt_ff1_h = m->lt_ff2_h = NULL;
    for (int c = 0; c < 8; ++c) { free(m->lt_out_w_h[c]); m->lt_out_w_h[c] = NULL; }
    m->half = 0;
}

// SA cache element type (this build's MP_KV_BF16, include/magpie_hip.h): every K and V
// row rounded to bf16 (round to nearest even) as it is appended to the cache, in the
// 110-frame prefill and every decode step; attention reads the rounded rows.
static int g_kv_bf16 = 0;
void orc_set_kv_bf16(int on) { g_kv_bf16 = on != 0; }
static inline float round_bf16(float v) {
    uint32_t u;
    memcpy(&u, &v, 4);
    u = (u + 0x7FFFu + ((u >> 16) & 1u)) & 0xFFFF0000u;
    memcpy(&v, &u, 4);
    return v;
}

int orc_set_weight_mode(orc_model *m, int mode) {
    if (!m || mode < 0 || mode > 3) return -1;
    free_half(m);
    m->q8mode = 0;
    m->f16mode = 0;
    if (mode == 0) return 0;
    if (mode == 3) {  // ggml F16 semantics for the file's F16 tensors
        if (m->n_f16 == 0) return -1;
        m->f16mode = 1;
        return 0;
    }
    if (mode == 2) {  // ggml Q8_0 semantics for the file's Q8_0 tensors
        if (m->n_q8 == 0) return -1;
        m->q8mode = 1;
        return 0;
    }
    const int d = m->d, dff = m->dff, D = m->lt_dim, F = m->lt_ffn;
    for (int l = 0; l < m->dec_layers; ++l) {
        dec_layer *L = &m->dec[l];
        L->qkv_h = bf16_copy(L->qkv, (size_t)3 * d * d);
        L->o_h = bf16_copy(L->o, (size_t)d * d);
        L->ff1_h = bf16_copy(L->ff1, (size_t)dff * d);
        L->ff2_h = bf16_copy(L->ff2, (size_t)d * dff);
    }
    // the LT attention (q|k|v, o_net) stays f32 in this mode: the build computes it through
    // load-time f32 tables (lt_slot_kernel); its FFN and output heads are bf16
    m->lt_ff1_h = bf16_copy(m->lt_ff1, (size_t)F * D);
    m->lt_ff2_h = bf16_copy(m->lt_ff2, (size_t)D * F);
    for (int c = 0; c < 8; ++c) m->lt_out_w_h[c] = bf16_copy(m->lt_out_w[c], (size_t)m->vocab_cb * D);
    m->half = 1;
    return 0;
}

void orc_free(orc_model *m) {
    if (!m) return;
    free_half(m);
    for (int i = 0; i < m->n_q8; ++i) { free(m->q8[i].q); free(m->q8[i].d); }
    free(m->q8);
    free(m->f16w);
    for (int i = 0; i < m->n_owned; ++i) free(m->owned[i]);
    free(m->owned);
    free(m->enc);
    free(m->dec);
    free(m);
}

// ------------------------------------------------------------------ encoder
// Causal multi-head self-attention over a block of rows (magpie.cpp:1477-1575 with
// the causal mask of 2343-2353; batched prefill magpie.cpp:3911-3988 uses
// ggml_diag_mask_inf, identical semantics). qkv: [M][3d] rows; writes attn [M][d].
static void causal_mha(const float *qkv, int M, int d, int heads, float *attn, int kv_offset_rows,
                       const float *Kc, const float *Vc) {
    // When Kc/Vc are given, keys/values for row m come from cache rows [0, kv_offset_rows + m].
    const int dh = d / heads;
    const double scale = 1.0 / sqrt((double)dh);
#pragma omp parallel
    {
        const int nk_max = kv_offset_rows + M;
        double *sb = malloc(sizeof(double) * (size_t)nk_max);
        double *pb = malloc(sizeof(double) * (size_t)nk_max);
#pragma omp for schedule(static) collapse(2)
        for (int m = 0; m < M; ++m)
            for (int h = 0; h < heads; ++h) {
                const float *q = qkv + (size_t)m * 3 * d + h * dh;
                if (Kc)
                    attend(q, Kc + h * dh, Vc + h * dh, kv_offset_rows + m + 1, d, dh, scale,
                           attn + (size_t)m * d + h * dh, sb, pb);
                else
                    attend(q, qkv + d + h * dh, qkv + 2 * d + h * dh, m + 1, 3 * d, dh, scale,
                           attn + (size_t)m * d + h * dh, sb, pb);
            }
        free(sb);
        free(pb);
    }
}

// magpie_build_conv_ffn kernel_size=3 branch (magpie.cpp:1806-1917): tap k of
// W[j][i][k] multiplies input row t-2+k (zero left padding).
static void conv_ffn_k(const orc_model *m, const float *W, const float *X0, float *Y, int M, int N, int K, int ks) {
    // F16 conv weights (weight mode 3): ggml's im2col takes the kernel's type, so the
    // input is rounded to f16 before the F16 mul_mat
    float *Xh = is_f16(m, W) ? f16_rows(X0, (size_t)M * K) : NULL;
    const float *X = Xh ? Xh : X0;
#pragma omp parallel for schedule(static)
    for (int n = 0; n < N; ++n) {
        const float *w = W + (size_t)n * K * ks;
        for (int t = 0; t < M; ++t) {
            double acc = 0.0;
            for (int k = 0; k < ks; ++k) {
                const int src = t - (ks - 1) + k;
                if (src < 0) continue;
                const float *x = X + (size_t)src * K;
                if (g_acc64) {
                    double a = 0.0;
                    for (int i = 0; i < K; ++i) a += (double)w[(size_t)i * ks + k] * (double)x[i];
                    acc += a;
                } else {
                    float a = 0.f;
                    for (int i = 0; i < K; ++i) a += w[(size_t)i * ks + k] * x[i];
                    acc = (float)acc + a;
                }
            }
            Y[(size_t)t * N + n] = (float)acc;
        }
    }
    free(Xh);
}

// magpie_encode_text (magpie.cpp:2284-2374) -> magpie_build_full_encoder (1960-1995)
int orc_encode(orc_model *m, const int32_t *tok, int T, float *enc_out) {
    const int d = m->d, dff = m->dff;
    float *x = malloc(sizeof(float) * (size_t)T * d);
    float *h = malloc(sizeof(float) * (size_t)T * d);
    float *qkv = malloc(sizeof(float) * (size_t)T * 3 * d);
    float *att = malloc(sizeof(float) * (size_t)T * d);
    float *o = malloc(sizeof(float) * (size_t)T * d);
    float *f = malloc(sizeof(float) * (size_t)T * dff);
    for (int t = 0; t < T; ++t) {
        if (tok[t] < 0 || tok[t] >= 2380) return -1;
        for (int i = 0; i < d; ++i)
            x[(size_t)t * d + i] = m->text_emb[(size_t)tok[t] * d + i] + m->enc_pos[(size_t)t * d + i];
    }
    for (int l = 0; l < m->enc_layers; ++l) {
        const enc_layer *L = &m->enc[l];
        layernorm_rows(x, L->norm_self, h, T, d, m->eps);
        mm(m, L->qkv, NULL, h, qkv, T, 3 * d, d);
        causal_mha(qkv, T, d, m->enc_heads, att, 0, NULL, NULL);
        mm(m, L->o, NULL, att, o, T, d, d);
        for (size_t i = 0; i < (size_t)T * d; ++i) x[i] = o[i] + x[i];
        layernorm_rows(x, L->norm_ff, h, T, d, m->eps);
        conv_ffn_k(m, L->ff1, h, f, T, dff, d, m->enc_kernel);
        gelu_inplace(f, (size_t)T * dff);
        conv_ffn_k(m, L->ff2, f, o, T, d, dff, m->enc_kernel);
        for (size_t i = 0; i < (size_t)T * d; ++i) x[i] = o[i] + x[i];
    }
    layernorm_rows(x, m->enc_norm_out, enc_out, T, d, m->eps);
    free(x); free(h); free(qkv); free(att); free(o); free(f);
    return 0;
}

// ------------------------------------------------------------------ decoder
typedef struct {
    int T, max_seq;
    float *xa_k, *xa_v;  // [L][T][128]
    float *kc, *vc;      // [L][max_seq][d]
} dstate;

// One decoder layer over M rows at positions [pos0, pos0+M) (M=110 for the
// batched prefill magpie.cpp:3991-4060, M=1 for a cached step magpie.cpp:3484-3528).
static void decoder_layer(const orc_model *m, dstate *s, int l, float *x, int M, int pos0) {
    const dec_layer *L = &m->dec[l];
    const int d = m->d, dff = m->dff, dxa = m->xa_heads * m->xa_dh;
    float *h = malloc(sizeof(float) * (size_t)M * d);
    float *qkv = malloc(sizeof(float) * (size_t)M * 3 * d);
    float *att = malloc(sizeof(float) * (size_t)M * d);
    float *o = malloc(sizeof(float) * (size_t)M * d);
    float *q = malloc(sizeof(float) * (size_t)M * dxa);
    float *f = malloc(sizeof(float) * (size_t)M * dff);
    float *Kc = s->kc + (size_t)l * s->max_seq * d, *Vc = s->vc + (size_t)l * s->max_seq * d;
    // self-attention: LN -> qkv -> cache append -> attention over [0, pos] -> o_net (3395-3480)
    const int hm = m->half && M == 1;  // decode steps only; the 110-frame prefill stays f32
    layernorm_rows(x, L->norm_self, h, M, d, m->eps);
    matmul_sel(m, L->qkv, hm ? L->qkv_h : NULL, NULL, h, qkv, M, 3 * d, d);
    for (int r = 0; r < M; ++r) {
        memcpy(Kc + (size_t)(pos0 + r) * d, qkv + (size_t)r * 3 * d + d, sizeof(float) * d);
        memcpy(Vc + (size_t)(pos0 + r) * d, qkv + (size_t)r * 3 * d + 2 * d, sizeof(float) * d);
        if (g_kv_bf16)
            for (int i = 0; i < d; ++i) {
                Kc[(size_t)(pos0 + r) * d + i] = round_bf16(Kc[(size_t)(pos0 + r) * d + i]);
                Vc[(size_t)(pos0 + r) * d + i] = round_bf16(Vc[(size_t)(pos0 + r) * d + i]);
            }
    }
    causal_mha(qkv, M, d, m->dec_heads, att, pos0, Kc, Vc);
    matmul_sel(m, L->o, hm ? L->o_h : NULL, NULL, att, o, M, d, d);
    for (size_t i = 0; i < (size_t)M * d; ++i) x[i] = o[i] + x[i];
    // cross-attention with cached K/V (1713-1767): 1 head x 128, no mask
    layernorm_rows(x, L->norm_xq, h, M, d, m->eps);
    mm(m, L->xq, NULL, h, q, M, dxa, d);
    {
        const int dh = m->xa_dh;
        const double scale = 1.0 / sqrt((double)dh);
        double *sb = malloc(sizeof(double) * (size_t)s->T), *pb = malloc(sizeof(double) * (size_t)s->T);
        float *ax = malloc(sizeof(float) * (size_t)M * dxa);
        const float *XK = s->xa_k + (size_t)l * s->T * dxa, *XV = s->xa_v + (size_t)l * s->T * dxa;
        for (int r = 0; r < M; ++r)
            for (int hh = 0; hh < m->xa_heads; ++hh)
                attend(q + (size_t)r * dxa + hh * dh, XK + hh * dh, XV + hh * dh, s->T, dxa, dh, scale,
                       ax + (size_t)r * dxa + hh * dh, sb, pb);
        mm(m, L->xo, NULL, ax, o, M, d, dxa);
        free(sb); free(pb); free(ax);
    }
    for (size_t i = 0; i < (size_t)M * d; ++i) x[i] = o[i] + x[i];
    // pointwise conv-FFN (1791-1805)
    layernorm_rows(x, L->norm_ff, h, M, d, m->eps);
    matmul_sel(m, L->ff1, hm ? L->ff1_h : NULL, NULL, h, f, M, dff, d);
    gelu_inplace(f, (size_t)M * dff);
    matmul_sel(m, L->ff2, hm ? L->ff2_h : NULL, NULL, f, o, M, d, dff);
    for (size_t i = 0; i < (size_t)M * d; ++i) x[i] = o[i] + x[i];
    free(h); free(qkv); free(att); free(o); free(q); free(f);
}

// compute_single_frame_audio_embedding (magpie.cpp:2746-2787): sum_cb emb[cb][c] * 1/8,
// then + dec_pos[pos] (4376-4379).
static void frame_embed(const orc_model *m, const int32_t *codes, int pos, float *x) {
    const int d = m->d;
    for (int i = 0; i < d; ++i) {
        float s = m->audio_emb[0][(size_t)codes[0] * d + i];
        for (int c = 1; c < 8; ++c) s = s + m->audio_emb[c][(size_t)codes[c] * d + i];
        x[i] = s * 0.125f + m->dec_pos[(size_t)pos * d + i];
    }
}

// Sampling stream (this repo's convention; the reference draws from an unseeded
// process-global mt19937, magpie.cpp:1129, so its draws are not reproducible):
// u(seed, stream, step, cb) = 24 high bits of splitmix64(splitmix64(seed ^ stream*C) ^ (step<<8 | cb)) / 2^24.
static uint64_t mix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
float orc_draw_u(uint64_t seed, int stream, int step, int cb) {
    uint64_t h = mix64(seed ^ ((uint64_t)(uint32_t)stream * 0xD1B54A32D192ED03ull));
    h = mix64(h ^ (((uint64_t)(uint32_t)step << 8) | (uint32_t)cb));
    return (float)(h >> 40) * (1.0f / 16777216.0f);
}

typedef struct { float v; int i; } scored_t;
static int scored_desc(const void *a, const void *b) {
    const scored_t *x = a, *y = b;
    if (x->v != y->v) return x->v > y->v ? -1 : 1;
    return x->i - y->i;  // ties: ascending index (std::partial_sort leaves them unspecified)
}

// sample_top_k (magpie.cpp:1072-1109): top-k by value, p_i = exp((l_i - l_0)/T)
// normalised by a sequential float sum, first i with u < cumsum_i, else the k-th.
// *margin = distance of u to the nearest boundary of the chosen interval.
int orc_sample_top_k(const float *logits, int n, float temperature, int top_k, float u, float *margin) {
    scored_t *sc = malloc(sizeof(scored_t) * (size_t)n);
    for (int i = 0; i < n; ++i) { sc[i].v = logits[i]; sc[i].i = i; }
    qsort(sc, (size_t)n, sizeof(scored_t), scored_desc);
    const int k = top_k < n ? top_k : n;
    float *pr = malloc(sizeof(float) * (size_t)k);
    const float mx = sc[0].v;
    float sum = 0.0f;
    for (int i = 0; i < k; ++i) { pr[i] = expf((sc[i].v - mx) / temperature); sum += pr[i]; }
    for (int i = 0; i < k; ++i) pr[i] /= sum;
    float cum = 0.0f, lo = 0.0f;
    int pick = sc[k - 1].i;
    float mg = INFINITY;
    for (int i = 0; i < k; ++i) {
        lo = cum;
        cum += pr[i];
        if (u < cum) { pick = sc[i].i; mg = fminf(u - lo, cum - u); break; }
    }
    if (margin) *margin = mg;
    free(pr); free(sc);
    return pick;
}

// magpie_local_transformer_sample_all (magpie.cpp:1113-1317), computed
// incrementally over positions (causal => identical to the reference's
// per-codebook recompute). temperature < 0.01 => argmax (1263-1264).
// *argeos is set when any codebook's argmax is EOS (the loop's EOS test, 4340-4346).
// force (nullable): teacher forcing; codes[] still receives this oracle's own
// decisions (and margins[] their margins), but codebook cb+1 is conditioned on
// force[cb] (the trajectory under test), so every decision can be checked.
static void lt_sample(const orc_model *m, const float *hidden, int forbid_eos, float temperature, int top_k,
                      uint64_t seed, int stream, int step, int32_t *codes, float *margins, int *argeos,
                      int32_t *argmax, const int32_t *force) {
    const int D = m->lt_dim, F = m->lt_ffn, V = m->vocab_cb, d = m->d;
    float s[9][256], X[256], h[256], qkv[768], kk[8][256], vv[8][256], a[256], Y[256], f[1024], y2[256];
    float *logits = malloc(sizeof(float) * (size_t)V);
    double sb[8], pb[8];
    mm(m, m->lt_in_w, m->lt_in_b, hidden, s[0], 1, D, d);
    for (int cb = 0; cb < 8; ++cb) {
        for (int i = 0; i < D; ++i) X[i] = s[cb][i] + m->lt_pos[(size_t)cb * D + i];
        layernorm(X, m->lt_norm_self, h, D, m->eps);
        matmul_sel(m, m->lt_qkv, m->lt_qkv_h, NULL, h, qkv, 1, 3 * D, D);
        memcpy(kk[cb], qkv + D, sizeof(float) * D);
        memcpy(vv[cb], qkv + 2 * D, sizeof(float) * D);
        attend(qkv, &kk[0][0], &vv[0][0], cb + 1, D, D, 1.0 / sqrt((double)D), a, sb, pb);
        matmul_sel(m, m->lt_o, m->lt_o_h, NULL, a, Y, 1, D, D);
        for (int i = 0; i < D; ++i) Y[i] = Y[i] + X[i];
        layernorm(Y, m->lt_norm_ff, h, D, m->eps);
        matmul_sel(m, m->lt_ff1, m->lt_ff1_h, NULL, h, f, 1, F, D);
        gelu_inplace(f, (size_t)F);
        matmul_sel(m, m->lt_ff2, m->lt_ff2_h, NULL, f, y2, 1, D, F);
        for (int i = 0; i < D; ++i) y2[i] = y2[i] + Y[i];
        matmul_sel(m, m->lt_out_w[cb], m->lt_out_w_h[cb], m->lt_out_b[cb], y2, logits, 1, V, D);
        // forbidden tokens (1133-1145) and first-max argmax (1250-1259)
        for (int t = m->audio_bos; t <= m->audio_bos + 7 && t < V; ++t)
            if (t != m->audio_eos || forbid_eos) logits[t] = -INFINITY;
        int am = 0;
        float mx = logits[0];
        for (int i = 1; i < V; ++i) if (logits[i] > mx) { mx = logits[i]; am = i; }
        float second = -INFINITY;
        for (int i = 0; i < V; ++i) if (i != am && logits[i] > second) second = logits[i];
        int code = am;
        if (argmax) argmax[cb] = am;
        float mg = mx - second;
        if (am == m->audio_eos && argeos) *argeos = 1;
        if (temperature >= 0.01f) {
            float sm;
            code = orc_sample_top_k(logits, V, temperature, top_k, orc_draw_u(seed, stream, step, cb), &sm);
            mg = fminf(mg, sm);
        }
        codes[cb] = code;
        if (margins) margins[cb] = mg;
        if (cb < 7) {
            const int next = force ? force[cb] : code;
            const float *e = m->audio_emb[cb] + (size_t)next * d;  // no 1/8 here (1284-1291)
            mm(m, m->lt_in_w, m->lt_in_b, e, s[cb + 1], 1, D, d);
        }
    }
    free(logits);
}

int orc_synthesize(orc_model *m, const int32_t *tokens, int T, int speaker, int max_steps, int ignore_eos,
                   int32_t *codes_out, float *margins_out, float *hidden_out, double *timing_out) {
    return orc_synthesize_ex(m, tokens, T, speaker, max_steps, ignore_eos, 0.0f, 80, 0, 0, 0, codes_out, margins_out,
                             hidden_out, timing_out);
}

int orc_lt_sample(orc_model *m, const float *hidden, float temperature, int top_k, int forbid_eos, uint64_t seed,
                  int stream, int step, int32_t *sampled, int32_t *argmax, float *margins) {
    if (!m || !hidden || !sampled || (temperature >= 0.01f && top_k < 1)) return -1;
    lt_sample(m, hidden, forbid_eos, temperature, top_k, seed, stream, step, sampled, margins, NULL, argmax, NULL);
    return 0;
}

static int synthesize(orc_model *m, const int32_t *tokens, int T, int speaker, int max_steps, int ignore_eos,
                      float temperature, int top_k, uint64_t seed, int stream, int emit_eos, const int32_t *force,
                      int32_t *codes_out, float *margins_out, float *hidden_out, double *timing_out) {
    if (temperature >= 0.01f && top_k < 1) return -1;
    if (!m || !tokens || T <= 0 || speaker < 0 || speaker >= m->n_spk) return -1;
    if (max_steps <= 0) max_steps = m->max_dec_steps;
    const int d = m->d, L = m->dec_layers, dxa = m->xa_heads * m->xa_dh;
    const int max_seq = m->ctx_frames + max_steps + 16;  // magpie.cpp:4077
    if (m->ctx_frames + max_steps > m->dec_pos_rows) return -2;
    double t0 = now_ms();
    dstate s = {T, max_seq, NULL, NULL, NULL, NULL};
    float *enc = malloc(sizeof(float) * (size_t)T * d);
    if (orc_encode(m, tokens, T, enc) != 0) { free(enc); return -3; }
    s.xa_k = malloc(sizeof(float) * (size_t)L * T * dxa);
    s.xa_v = malloc(sizeof(float) * (size_t)L * T * dxa);
    s.kc = calloc((size_t)L * max_seq * d, sizeof(float));
    s.vc = calloc((size_t)L * max_seq * d, sizeof(float));
    {   // magpie_precompute_cross_attention_kv (1663-1711) per layer (4098-4136)
        float *hn = malloc(sizeof(float) * (size_t)T * d), *kv = malloc(sizeof(float) * (size_t)T * 2 * dxa);
        for (int l = 0; l < L; ++l) {
            layernorm_rows(enc, m->dec[l].norm_xmem, hn, T, d, m->eps);
            mm(m, m->dec[l].xkv, NULL, hn, kv, T, 2 * dxa, d);
            for (int t = 0; t < T; ++t) {
                memcpy(s.xa_k + ((size_t)l * T + t) * dxa, kv + (size_t)t * 2 * dxa, sizeof(float) * dxa);
                memcpy(s.xa_v + ((size_t)l * T + t) * dxa, kv + (size_t)t * 2 * dxa + dxa, sizeof(float) * dxa);
            }
        }
        free(hn); free(kv);
    }
    {   // baked speaker context + batched 110-frame prefill (4138-4238)
        const int C = m->ctx_frames;
        float *x = malloc(sizeof(float) * (size_t)C * d);
        for (int t = 0; t < C; ++t)
            for (int i = 0; i < d; ++i)
                x[(size_t)t * d + i] = m->baked[(size_t)speaker * C * d + (size_t)t * d + i] + m->dec_pos[(size_t)t * d + i];
        for (int l = 0; l < L; ++l) decoder_layer(m, &s, l, x, C, 0);
        free(x);
    }
    double t1 = now_ms();
    // BOS step + autoregressive loop (4245-4407)
    float x[768], hid[768];
    int32_t prev[8];
    for (int c = 0; c < 8; ++c) prev[c] = m->audio_bos;
    int pos = m->ctx_frames, n_frames = 0;
    frame_embed(m, prev, pos, x);
    for (int l = 0; l < L; ++l) decoder_layer(m, &s, l, x, 1, pos);
    layernorm(x, m->dec_norm_out, hid, d, m->eps);
    if (hidden_out) memcpy(hidden_out, hid, sizeof hid);
    pos++;
    for (int step = 0; step < max_steps; ++step) {
        int32_t codes[8];
        const int forbid = ignore_eos || step < 4;  // min_generated_frames (4267,4325)
        int eos = 0;
        const int32_t *fc = force ? force + (size_t)step * 8 : NULL;
        lt_sample(m, hid, forbid, temperature, top_k, seed, stream, step, codes,
                  margins_out ? margins_out + (size_t)step * 8 : NULL, &eos, NULL, fc);
        for (int c = 0; c < 8; ++c) if (codes[c] == m->audio_eos) eos = 1;
        if (fc) {  // forced: the trajectory under test decides what comes next
            memcpy(codes_out + (size_t)step * 8, codes, sizeof codes);
            n_frames = step + 1;
            if (step + 1 >= max_steps) break;
            frame_embed(m, fc, pos, x);
            for (int l = 0; l < L; ++l) decoder_layer(m, &s, l, x, 1, pos);
            layernorm(x, m->dec_norm_out, hid, d, m->eps);
            if (hidden_out) memcpy(hidden_out + (size_t)(step + 1) * d, hid, sizeof hid);
            pos++;
            continue;
        }
        if (eos) {
            // the streaming loop emits the EOS frame too (magpie.cpp:4800-4806)
            if (emit_eos) { memcpy(codes_out + (size_t)step * 8, codes, sizeof codes); n_frames = step + 1; }
            break;
        }
        memcpy(codes_out + (size_t)step * 8, codes, sizeof codes);
        n_frames = step + 1;
        if (step + 1 >= max_steps) break;
        frame_embed(m, codes, pos, x);
        for (int l = 0; l < L; ++l) decoder_layer(m, &s, l, x, 1, pos);
        layernorm(x, m->dec_norm_out, hid, d, m->eps);
        if (hidden_out) memcpy(hidden_out + (size_t)(step + 1) * d, hid, sizeof hid);
        pos++;
    }
    double t2 = now_ms();
    if (timing_out) { timing_out[0] = t1 - t0; timing_out[1] = t2 - t1; }
    free(enc); free(s.xa_k); free(s.xa_v); free(s.kc); free(s.vc);
    return n_frames;
}

int orc_synthesize_ex(orc_model *m, const int32_t *tokens, int T, int speaker, int max_steps, int ignore_eos,
                      float temperature, int top_k, uint64_t seed, int stream, int emit_eos, int32_t *codes_out,
                      float *margins_out, float *hidden_out, double *timing_out) {
    return synthesize(m, tokens, T, speaker, max_steps, ignore_eos, temperature, top_k, seed, stream, emit_eos, NULL,
                      codes_out, margins_out, hidden_out, timing_out);
}

int orc_synthesize_forced(orc_model *m, const int32_t *tokens, int T, int speaker, int n_frames, int ignore_eos,
                          float temperature, int top_k, uint64_t seed, int stream, const int32_t *forced,
                          int32_t *codes_out, float *margins_out, float *hidden_out) {
    if (!forced || n_frames <= 0) return -1;
    return synthesize(m, tokens, T, speaker, n_frames, ignore_eos, temperature, top_k, seed, stream, 0, forced,
                      codes_out, margins_out, hidden_out, NULL);
}

// ------------------------------------------------------------------ codec
typedef struct {
    int cin, cout, k;
    float *w, *b;  // w: [cout][cin][k] (PyTorch order)
    float *wh;     // fp16-rounded copy of w (ggml F16 im2col operand, A.7)
} conv_t;
typedef struct { float *alpha; int n; } snake_t;
typedef struct { snake_t in_act, sk_act; conv_t in_conv, sk_conv; } rblock;

struct orc_codec {
    conv_t pre, post;
    snake_t up_act[5], post_act;
    float *up_w[5], *up_b[5];
    rblock rb[5][3][3];
    float **owned;
    int n_owned;
    int resinit;  // orc_codec_set_resinit
};
static const int k_chans[6] = {864, 432, 216, 108, 54, 27};
static const int k_rates[5] = {8, 8, 4, 2, 2};
static const int k_ks[3] = {3, 7, 11};
static const int k_dil[3] = {1, 3, 5};

static float *ctake(orc_codec *c, const orc_gguf *g, const char *name, int *ok) {
    float *p = orc_gguf_f32(g, name, NULL);
    if (!p) { fprintf(stderr, "oracle: missing codec tensor %s\n", name); *ok = 0; return NULL; }
    c->owned = realloc(c->owned, sizeof(float *) * (size_t)(c->n_owned + 1));
    c->owned[c->n_owned++] = p;
    return p;
}
static void load_conv(orc_codec *c, const orc_gguf *g, conv_t *cv, const char *wname, const char *bname,
                      int cout, int cin, int k, int *ok) {
    cv->cin = cin; cv->cout = cout; cv->k = k;
    cv->w = ctake(c, g, wname, ok);
    cv->b = ctake(c, g, bname, ok);
    if (!cv->w) return;
    cv->wh = malloc(sizeof(float) * (size_t)cout * cin * k);
    c->owned = realloc(c->owned, sizeof(float *) * (size_t)(c->n_owned + 1));
    c->owned[c->n_owned++] = cv->wh;
    for (size_t i = 0; i < (size_t)cout * cin * k; ++i) cv->wh[i] = orc_f16_to_f32(orc_f32_to_f16(cv->w[i]));
}

// magpie_codec_load tensor mapping (nano-codec.cpp:84-199, 205-333)
orc_codec *orc_codec_load(const char *path) {
    orc_gguf g;
    if (orc_gguf_open(&g, path) != 0) return NULL;
    orc_codec *c = calloc(1, sizeof *c);
    int ok = 1;
    char a[160], b[160];
    load_conv(c, &g, &c->pre, "dec.pre.weight", "dec.pre.bias", 864, 32, 7, &ok);
    load_conv(c, &g, &c->post, "dec.post.weight", "dec.post.bias", 1, 27, 3, &ok);
    c->post_act.alpha = ctake(c, &g, "dec.post_act.alpha", &ok);
    c->post_act.n = 13;
    for (int i = 0; i < 5; ++i) {
        snprintf(a, sizeof a, "dec.act.%d.activation.snake_act.alpha", i);
        c->up_act[i].alpha = ctake(c, &g, a, &ok);
        c->up_act[i].n = k_chans[i] / 2;
        snprintf(a, sizeof a, "dec.up.%d.c.weight", i);
        c->up_w[i] = ctake(c, &g, a, &ok);
        snprintf(a, sizeof a, "dec.up.%d.c.bias", i);
        c->up_b[i] = ctake(c, &g, a, &ok);
        const int C = k_chans[i + 1];
        for (int j = 0; j < 3; ++j)
            for (int k = 0; k < 3; ++k) {
                rblock *r = &c->rb[i][j][k];
                snprintf(a, sizeof a, "dec.rl.%d.rb.%d.rb.%d.in_act.alpha", i, j, k);
                r->in_act.alpha = ctake(c, &g, a, &ok); r->in_act.n = C / 2;
                snprintf(a, sizeof a, "dec.rl.%d.rb.%d.rb.%d.sk_act.alpha", i, j, k);
                r->sk_act.alpha = ctake(c, &g, a, &ok); r->sk_act.n = C / 2;
                snprintf(a, sizeof a, "dec.rl.%d.rb.%d.rb.%d.in_conv.weight", i, j, k);
                snprintf(b, sizeof b, "dec.rl.%d.rb.%d.rb.%d.in_conv.bias", i, j, k);
                load_conv(c, &g, &r->in_conv, a, b, C, C, k_ks[j], &ok);
                snprintf(a, sizeof a, "dec.rl.%d.rb.%d.rb.%d.sk_conv.weight", i, j, k);
                snprintf(b, sizeof b, "dec.rl.%d.rb.%d.rb.%d.sk_conv.bias", i, j, k);
                load_conv(c, &g, &r->sk_conv, a, b, C, C, k_ks[j], &ok);
            }
    }
    orc_gguf_close(&g);
    if (!ok) { orc_codec_free(c); return NULL; }
    return c;
}

void orc_codec_free(orc_codec *c) {
    if (!c) return;
    for (int i = 0; i < c->n_owned; ++i) free(c->owned[i]);
    free(c->owned);
    free(c);
}

void orc_fsq(const int32_t *codes, int F, float *latent) {
    static const int base[4] = {1, 8, 56, 336}, levels[4] = {8, 7, 6, 6};
    for (int cb = 0; cb < 8; ++cb)
        for (int t = 0; t < F; ++t) {
            const int idx = codes[cb * F + t];
            for (int dd = 0; dd < 4; ++dd) {
                const int nonneg = (idx / base[dd]) % levels[dd];
                const int half = levels[dd] / 2;
                latent[(size_t)(cb * 4 + dd) * F + t] = (float)(nonneg - half) / (float)half;
            }
        }
}

// magpie_codec_build_half_snake (nano-codec.cpp:376-426): channels c < n get
// x + sin^2(alpha x)/alpha (ggml op order mul, sin, sqr, div, add); the rest leaky 0.01.
static void half_snake(const snake_t *s, const float *x, float *y, int C, int T) {
#pragma omp parallel for schedule(static)
    for (int c = 0; c < C; ++c) {
        const float *xi = x + (size_t)c * T;
        float *yo = y + (size_t)c * T;
        if (c < s->n) {
            const float al = s->alpha[c];
            for (int t = 0; t < T; ++t) {
                if (g_acc64) {
                    const double sn = sin((double)xi[t] * al);
                    yo[t] = (float)((double)xi[t] + sn * sn / al);
                } else {
                    const float sn = sinf(xi[t] * al);
                    yo[t] = xi[t] + (sn * sn) / al;
                }
            }
        } else {
            for (int t = 0; t < T; ++t) yo[t] = xi[t] > 0.f ? xi[t] : 0.01f * xi[t];
        }
    }
}

// magpie_codec_build_causal_conv1d (nano-codec.cpp:429-466): left pad (k-1)*dil.
// f16=1: operands rounded to fp16 as ggml_conv_1d's F16 im2col does (A.7).
// resid (nullable): the accumulators start at resid[o][t] instead of 0, so y = (resid + sum)
// + b: the rounding order of this build's residual convs (MP_RESINIT, mp_codec.hip), the
// oracle's codec "resinit" mode; the reference's is (sum + b) + resid (nano-codec.cpp:454-462,
// 568-599), the default.
static void causal_conv_r(const conv_t *cv, const float *x, float *y, int T, int dil, int f16, const float *resid);
static void causal_conv(const conv_t *cv, const float *x, float *y, int T, int dil, int f16) {
    causal_conv_r(cv, x, y, T, dil, f16, NULL);
}
static void causal_conv_r(const conv_t *cv, const float *x, float *y, int T, int dil, int f16, const float *resid) {
    const int Ci = cv->cin, Co = cv->cout, K = cv->k, pad = (K - 1) * dil;
    const float *w = f16 ? cv->wh : cv->w;
    const float *xs = x;
    float *xr = NULL;
    if (f16) {
        xr = malloc(sizeof(float) * (size_t)Ci * T);
        for (size_t i = 0; i < (size_t)Ci * T; ++i) xr[i] = orc_f16_to_f32(orc_f32_to_f16(x[i]));
        xs = xr;
    }
#pragma omp parallel
    {
        double *acc = malloc(sizeof(double) * (size_t)T);
        float *accf = malloc(sizeof(float) * (size_t)T);
#pragma omp for schedule(static)
        for (int o = 0; o < Co; ++o) {
            if (resid) {
                const float *ro = resid + (size_t)o * T;
                for (int t = 0; t < T; ++t) { acc[t] = ro[t]; accf[t] = ro[t]; }
            } else if (g_acc64) memset(acc, 0, sizeof(double) * (size_t)T);
            else memset(accf, 0, sizeof(float) * (size_t)T);
            for (int i = 0; i < Ci; ++i) {
                const float *xi = xs + (size_t)i * T;
                for (int k = 0; k < K; ++k) {
                    const float wv = w[((size_t)o * Ci + i) * K + k];
                    const int sh = k * dil - pad;  // input index = t + sh
                    const int t0 = sh < 0 ? -sh : 0;
                    if (g_acc64) for (int t = t0; t < T; ++t) acc[t] += (double)wv * (double)xi[t + sh];
                    else for (int t = t0; t < T; ++t) accf[t] += wv * xi[t + sh];
                }
            }
            float *yo = y + (size_t)o * T;
            const float b = cv->b ? cv->b[o] : 0.f;
            for (int t = 0; t < T; ++t) yo[t] = (float)(g_acc64 ? acc[t] : accf[t]) + b;
        }
        free(acc);
        free(accf);
    }
    free(xr);
}

// magpie_codec_build_conv_transpose1d (nano-codec.cpp:481-565): groups=Cout,
// in = 2*Cout, kernel K = 2s, output trimmed to T*s.
static void conv_transpose(const float *w, const float *bias, const float *x, float *y, int Cout, int T, int s) {
    const int K = 2 * s, To = T * s;
#pragma omp parallel for schedule(static)
    for (int g = 0; g < Cout; ++g)
        for (int t = 0; t < To; ++t) {
            double acc = 0.0;
            for (int ci = 0; ci < 2; ++ci) {
                const int c = 2 * g + ci;
                for (int tau = t / s - 1; tau <= t / s; ++tau) {
                    if (tau < 0 || tau >= T) continue;
                    const int k = t - tau * s;
                    if (k < 0 || k >= K) continue;
                    acc += (double)x[(size_t)c * T + tau] * (double)w[(size_t)c * K + k];
                }
            }
            y[(size_t)g * To + t] = (float)acc + bias[g];
        }
}

void orc_codec_set_resinit(orc_codec *c, int on) {
    if (c) c->resinit = on != 0;
}

// magpie_codec_build_decoder (nano-codec.cpp:676-715) + magpie_codec_decode (758-845)
int orc_codec_decode(orc_codec *c, const int32_t *codes, int F, float *audio, int f16) {
    if (!c || F <= 0) return -1;
    int T = F, C = 864;
    size_t cap = (size_t)27 * F * 1024 + (size_t)864 * F * 8 + 4096;
    float *x = malloc(sizeof(float) * cap), *h = malloc(sizeof(float) * cap), *h2 = malloc(sizeof(float) * cap);
    float *acc = malloc(sizeof(float) * cap), *rb = malloc(sizeof(float) * cap);
    float *lat = malloc(sizeof(float) * 32 * (size_t)F);
    orc_fsq(codes, F, lat);
    causal_conv(&c->pre, lat, x, T, 1, f16);
    for (int i = 0; i < 5; ++i) {
        half_snake(&c->up_act[i], x, h, C, T);
        const int Co = k_chans[i + 1], s = k_rates[i];
        conv_transpose(c->up_w[i], c->up_b[i], h, x, Co, T, s);
        C = Co;
        T = T * s;
        // magpie_codec_build_reslayer (619-641): mean of 3 HiFiGAN blocks
        for (int j = 0; j < 3; ++j) {
            memcpy(rb, x, sizeof(float) * (size_t)C * T);
            for (int k = 0; k < 3; ++k) {  // magpie_codec_build_residual_block (568-599)
                const rblock *r = &c->rb[i][j][k];
                half_snake(&r->in_act, rb, h, C, T);
                causal_conv(&r->in_conv, h, h2, T, k_dil[k], f16);
                half_snake(&r->sk_act, h2, h, C, T);
                if (c->resinit) {  // (x + sum) + b, this build's order
                    causal_conv_r(&r->sk_conv, h, h2, T, 1, f16, rb);
                    memcpy(rb, h2, sizeof(float) * (size_t)C * T);
                } else {  // (sum + b) + x, the reference's
                    causal_conv(&r->sk_conv, h, h2, T, 1, f16);
                    for (size_t e = 0; e < (size_t)C * T; ++e) rb[e] = rb[e] + h2[e];
                }
            }
            if (j == 0) memcpy(acc, rb, sizeof(float) * (size_t)C * T);
            else for (size_t e = 0; e < (size_t)C * T; ++e) acc[e] = acc[e] + rb[e];
        }
        for (size_t e = 0; e < (size_t)C * T; ++e) x[e] = acc[e] * (1.0f / 3.0f);
    }
    half_snake(&c->post_act, x, h, C, T);
    causal_conv(&c->post, h, h2, T, 1, f16);
    for (int t = 0; t < T; ++t) audio[t] = tanhf(h2[t]);
    free(x); free(h); free(h2); free(acc); free(rb); free(lat);
    return T;
}

int orc_q8_quantize_row(const float *x, int K, int8_t *q, float *d) {
    if (!x || !q || !d || K <= 0 || K % 32) return -1;
    quant_row_q8(x, K, q, d);
    return 0;
}

int orc_qblock_dots(const uint8_t *blocks, int type, int N, int K, const int8_t *aq, int32_t *dots) {
    if (!blocks || !aq || !dots || N <= 0 || K <= 0 || K % 32 || (type != 8 && type != 2)) return -1;
    const int nb = K / 32;
    int8_t *wq = malloc((size_t)N * K);
    float *wd = malloc(sizeof(float) * (size_t)N * nb);
    unpack_qblocks(blocks, type, (int64_t)N * K, wq, wd);
    for (int n = 0; n < N; ++n)
        for (int b = 0; b < nb; ++b) dots[(size_t)n * nb + b] = block_dot_q8(wq + (size_t)n * K + b * 32, aq + b * 32);
    free(wq);
    free(wd);
    return 0;
}

// Unit-test entry: y[N] = ggml Q8_0 mul_mat of the raw GGUF Q8_0 blocks
// (34 bytes per 32 weights, row-major [N][K]) with the activation x[K].
int orc_q8_matvec(const uint8_t *blocks, int N, int K, const float *x, float *y) {
    if (!blocks || !x || !y || N <= 0 || K <= 0 || K % 32) return -1;
    q8w_t w = {NULL, malloc((size_t)N * K), malloc(sizeof(float) * (size_t)N * (K / 32))};
    for (int64_t b = 0; b < (int64_t)N * K / 32; ++b) {
        uint16_t h;
        memcpy(&h, blocks + b * 34, 2);
        w.d[b] = orc_f16_to_f32(h);
        memcpy(w.q + b * 32, blocks + b * 34 + 2, 32);
    }
    matmul_q8(&w, NULL, x, y, 1, N, K);
    free(w.q);
    free(w.d);
    return 0;
}
