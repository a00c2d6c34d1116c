// Kernel parameter blocks shared by the host runtime (mp_runtime.hip) and the
// kernels. Plain pointers only: every launch in a decode iteration reads its
// per-utterance state (positions, codes, done flags) from device memory, so one
// captured hipGraph replays unchanged for every frame.
#pragma once
#include <stdint.h>

namespace mp {

constexpr int D = 768;        // d_model                      (magpie.h:37)
constexpr int DFF = 3072;     // d_ffn                        (magpie.h:38)
constexpr int NH = 12;        // decoder SA heads             (magpie.h:48)
constexpr int DH = 64;        // SA head dim                  (magpie.h:39)
constexpr int DXA = 128;      // XA 1 head x 128              (magpie.h:49-50)
constexpr int LTD = 256;      // local transformer dim        (magpie.h:54)
constexpr int LTF = 1024;     // LT ffn dim                   (magpie.h:55)
constexpr int NCB = 8;        // codebooks                    (magpie.h:61)
constexpr int VCB = 2024;     // vocab per codebook           (magpie.h:63)
#ifndef MP_RW_LTE
#define MP_RW_LTE 2  // f32 LT head rows per wave at batch 1 (253 workgroups at 2)
#endif
constexpr int LT_HEAD_WGS = (VCB + 4 * MP_RW_LTE - 1) / (4 * MP_RW_LTE);  // its workgroups = candidates
constexpr int CTX = 110;      // baked context frames         (magpie.h:67)
constexpr int SA_CHUNK = 64;  // cache rows are allocated in whole 64-key chunks
constexpr int NCH_MAX = 16;   // -> max_seq <= 1024 (reference: 626, magpie.cpp:4077)
constexpr int TMAX_LIMIT = 1024;  // text tokens per utterance (LDS score buffer)
// split-K decode attention: partial softmax states, merged in the next op's prologue
constexpr int SA_SPLITS = 4;        // key splits of each SA head (sa_attn_kernel)
constexpr int SA_PART = 4 + DH;     // per (slot, head, split): m, l, -, -, O[64] (unnormalised)
#ifndef MP_XA_SPLITS
#define MP_XA_SPLITS 4
#endif
constexpr int XA_SPLITS = MP_XA_SPLITS;  // text-key splits of the fused cross-attention (xa_part_kernel)
constexpr int XA_PART = 4 + D;      // per (slot, split): m, l, -, -, O[768] (unnormalised)
#ifndef MP_LT_FFN_P
#define MP_LT_FFN_P 64
#endif
constexpr int LT_FFN_P = MP_LT_FFN_P;  // LT FFN (f32 / F16 modes): workgroups of lt_ffn(2)_kernel = partial FFN-down sums per slot
#ifndef MP_LTS_P
#define MP_LTS_P 32
#endif
constexpr int LTS_P = MP_LTS_P;           // bf16 mode LT step (lt_slot_kernel): workgroups per slot = partial FFN-down sums
constexpr int LTQ_P = 64;           // Q8_0 mode LT step (lt_slot_q8_kernel): workgroups per slot = partial FFN-down sums

// prologue / epilogue selectors of the fused GEMV family (mp_decode.hip)
enum Pro {
    PRO_PLAIN = 0,      // act = src
    PRO_LN = 1,         // act = LN(src) * lnw                          (magpie.cpp:2237-2259)
    // 2: retired (the frame embedding is written by lt_finalize_kernel, FinP::x)
    PRO_LTX_LN = 5,     // X = s_cb + lt_pos[cb]; act = LN(X)*lnw       (1015-1034, 946-958)
    PRO_LT_ATTN = 6,    // act = causal 1x256 attention over LT positions 0..cb (965-966)
    PRO_LTARG_ATTN = 8, // cb >= 1: code_{cb-1} = top-k draw / masked argmax of the logits; q|k|v of
                        // LT position cb = Q[cb-1][code], gathered; act = PRO_LT_ATTN's attention.
                        // Q[c][v] = qkv_net(LN(P[c][v] + lt_pos[c+1])) and P[c][v] =
                        // in_proj(audio_emb[c][v]) + b depend only on (c, v) (magpie.cpp:1274-1313,
                        // 946-958): both tables are built at load
    PRO_SA_MERGE = 9,   // act = SA output: the SA_SPLITS partial softmax states of each head merged
    PRO_XA_LN = 10,     // x2 = src + XA output (XA_SPLITS partial states merged), block 0 stores
                        // x2 to xres; act = LN(x2)*lnw              (3513-3525)
    PRO_PLAIN_B16 = 11, // bf16 kernels only: act = src_b16 (rows already bf16, EPI_GELU_B16 output)
    PRO_LTFFN_MERGE = 12, // act = (sum over p of the LT_FFN_P partial FFN-down sums, p ascending)
                          //       + addsrc: the LT FFN output (lt_ffn_kernel, 983-992)
    PRO_LTS_MERGE = 13,   // the same over the LTS_P partial sums of lt_slot_kernel (bf16 mode, small batches)
    PRO_LTQ_MERGE = 14,   // the same over the LTQ_P partial sums of lt_slot_q8_kernel (Q8_0 mode, batch 1)
};
// partial sums merged by the LT heads' merge prologues
template <int PRO>
constexpr int ltm_count() { return PRO == PRO_LTQ_MERGE ? LTQ_P : LT_FFN_P; }
enum Epi {
    EPI_STORE = 0,      // out = v
    EPI_BIAS = 1,       // out = v + bias
    EPI_GELU = 2,       // out = gelu(v)
    EPI_RESID = 3,      // resid += v
    EPI_QKV = 4,        // q -> out, k/v -> SA cache at pos       (3415-3442)
    EPI_LTQKV = 5,      // q -> lq, k/v -> LT position cb
    EPI_ADD_STORE = 6,  // out = v + addsrc
    EPI_GELU_B16 = 7,   // out_b16 = bf16(gelu(v)): the bf16 FFN-down operand, rounded once here
    EPI_LTX_ADD = 8,    // out = v + (P[cb-1][code] + lt_pos[cb]): LT residual of PRO_LTARG_ATTN's code
    EPI_LTKVO = 9,      // f32 LT position 0: rows [0,256) k_0 -> lk[b][0], rows [256,512) vo_0 -> lv[b][0]
    EPI_GELU_F16 = 11,  // out_b16 = f16(gelu(v)): EPI_GELU_B16 for the F16 weight mode
    EPI_RESID_XA = 10,  // resid += v, each new x1 value also published as a tagged granule; the
                        // launch's last XA_SPLITS x NB workgroups run the fused XA on it (below)
    EPI_QKV_SA = 12,    // EPI_QKV, each q|k|v value also published as a tagged granule qh[b][2304];
                        // the launch's last NH x SA_SPLITS x NB workgroups run the SA on it
    EPI_RESID_XQ8 = 13, // Q8_0 O-projection: EPI_RESID_XA's stores and granules; then XQG x NB
                        // workgroups compute the cross-attention's q = Q8(q_net) LN(x1) and hand it on
                        // as granules, and XQ8A x NB workgroups the attention + o_net: x2 (direct
                        // Q8_0 XA, xa_q8_kernel's arithmetic)
};

// Temperature / top-k sampling (sample_top_k, magpie.cpp:1072-1109). Off when
// temperature < 0.01 (greedy, 1263-1264). Every draw is keyed by
// (seed, slot, step, codebook) through mp_uniform(), so a decode is reproducible
// and graph replays need no RNG state.
struct SmpCfg {                // device-resident, so a captured graph serves any setting
    float temperature;
    int top_k;                 // 1..VCB
    unsigned long long seed;
    int stream_base;           // draw stream of slot b = stream_base + b
};
struct Sampling {
    int on;                    // temperature >= 0.01 (baked into the captured graph)
    const SmpCfg *cfg;
    int *argeos;               // [B] 1 once a codebook's argmax was EOS this frame (4343-4346)
    int *amax;                 // optional [B][8]: every codebook's argmax (magpie_sample_result.argmax_codes)
};

// LT FFN up + GELU + FFN down in one launch (lt_ffn_kernel): workgroup p owns
// hidden units [p*16, p*16+16) and writes its share of FFN down, part[b][p][256]
struct LtFfnP {
    const float *y;      // [B][256] LT residual stream after attention (ltY)
    const float *lnw;    // norm_pos_ff weight
    const float *w1;     // [1024][256] FFN up
    const float *w2;     // FFN down [256][1024] re-laid slice-major [LT_FFN_P][256][1024 / LT_FFN_P]
    float eps;
    float *part;         // [B][LT_FFN_P][256]
    float *out;          // lt_merge_kernel: [B][256] = ltY + merged FFN down
    unsigned long long *ts;  // profiling (nullable): [first wave start, last wave end], s_memrealtime ticks
};

// f32 weight mode: the LT's attention + o_net + residual folded into the FFN launch
// (lt_ffn2_kernel). Position j's o_net contribution is W_o v_j: for j >= 1 a
// load-time table row VO[j-1][code] = W_o V[j-1][code] (V = the v third of the q|k|v
// table), for j = 0 the per-frame vo_0 = (W_o W_v) LN(X_0) (lt_a's epilogue), so
// y = X_c + sum_j softmax_j(q_c k_j / 16) vo_j  (= X_c + o_net(attn), magpie.cpp:946-966,
// reassociated; o_net is linear).
struct LtFfn2P {
    LtFfnP f;             // y = ltY (written by block 0), FFN weights, partials
    int cb;
    const float *ltX;     // [B][256] X_0 (cb 0)
    float *ltk, *ltv;     // [B][8][256] k_j and vo_j rows of the frame's positions
    const float *qkvtab;  // [7][2024][768] q|k|v of codebook c's code at position c+1
    const float *votab;   // [7][2024][256] W_o v of the same rows
    const float *ptab;    // [8][2024][256] in_proj(audio_emb) + b
    const float *lt_pos;
    const float *logits;  // [B][2024] codebook cb-1's logits
    int *codes_cur;       // [B][8]
    const int *step;
    int ignore_eos, audio_bos, audio_eos;
    Sampling smp;
    // bf16 weight mode (lt_slot_kernel): the FFN weights rounded to bf16, W1 row-major
    // [1024][256], W2 slice-major [LTS_P][256][1024 / LTS_P]. The LTS_P partial sums per slot
    // go to f.part, merged by the head's prologue (PRO_LTS_MERGE; gh null, batch 1), or as
    // {tag, value} granules gh[B][LTS_P][256] of which every workgroup merges its 256 / LTS_P
    // outputs into f.out = y2 (tags iter[0] * 64 + 32 + cb; hx_err: hand-off timeout)
    const unsigned short *w1h, *w2h;
    unsigned long long *gh;
    const int *iter;
    int *hx_err;
    // f32 batch 1, greedy: the previous head's workgroup candidates (GemvP::cand), ncand of them
    const unsigned long long *cand;
    int ncand;
};

// f32 mode at batch 1: the LT's front in ONE launch (lt_front_kernel) instead of three
// (lt_in0, lt_kvo, lt_ffn2 of codebook 0): in_proj of LN(x) (rows 4p + w of workgroup p)
// and the rows of [W_k ; W_o W_v] LN(X_0) are handed between the 64 workgroups as
// {tag, value} granules gh[2][256] (tags iter[0] * 64 + 40, + 41), then codebook 0's FFN
// step as lt_ffn2_kernel computes it. Every row is computed with the same arithmetic as
// the three separate launches, so batch 1 equals the batched path bit for bit.
struct LtFrontP {
    LtFfn2P l;                 // the codebook-0 FFN step (cb = 0): FFN weights, partials, y, ltX, ltk, ltv
    const float *x;            // [768] decoder output (final LN input)
    const float *norm_out;     // final decoder LayerNorm weight
    const float *w_in, *b_in;  // LT in_proj [256][768] + bias
    float *lt_s;               // [9][256] in_proj output (row 0 written)
    float *hidden_out;         // [768] LN(x) (magpie_synthesize's hidden), nullable
    float *trace;              // [trace_steps][768] per-step LN(x) (nullable)
    int trace_steps;
    const float *lt_pos, *norm_self;
    const float *w_kvo;        // [512][256] = [W_k ; W_o W_v]
    unsigned long long *gh;    // [2][256] granules: in_proj output, vo_0
    const int *iter;
    int *hx_err;
};

// f32 mode at batch 1, greedy: the whole LT of a frame in ONE launch (lt_all_kernel, 64
// workgroups): the front as lt_front_kernel (k_0 handed over too), then per codebook the
// FFN-down partial sums as {tag, value} granules gp[64][256] (tag iter * 64 + 48 + cb), each
// workgroup merging 4 of the 256 outputs in partial order into y2 granules gy[256] (+ 56 + cb),
// every workgroup 32 head rows on the swept y2 and its masked first-max logit as one ordered
// key gc[wg] (EOS's own key in gc[64]; the low 21 bits a per-codebook tag), and every
// workgroup the next code from the 65 keys, that position's y and its 16 FFN units. Per row,
// output and step the arithmetic of lt_ffn2_kernel<1> and the batch-1 head (same bits).
struct LtAllP {
    LtFrontP f;                  // the front; f.l: tables, FFN weights, y, codes, step, logits (read)
    const float *w_out, *b_out;  // heads [8][2024][256], biases [8][2024]
    float *logits;               // [2024] each codebook's logits (codebook 7's: the finalize's pick)
    unsigned long long *gp;      // [LT_FFN_P][256]
    unsigned long long *gy;      // [256]
    unsigned long long *gc;      // [LT_FFN_P + 1]
};

// Frame embedding of every slot (layer 0's residual input, magpie.cpp:2746-2787,
// 4376-4379): x[b] = (sum_cb emb[cb][code_cb]) / 8 + pos_emb[pos[b]]
struct EmbP {
    const float *emb;      // [8][2024][768]
    const int *codes;      // [B][8] (codes_prev)
    const float *pos_emb;
    const int *pos;        // [B]
    float *x;              // [B][768]
};

// splitmix64 finaliser
__host__ __device__ inline unsigned long long mp_mix64(unsigned long long x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
// u in [0, 1) with 24 random bits, like uniform_real_distribution<float>(0, 1)
__host__ __device__ inline float mp_uniform(unsigned long long seed, int stream, int step, int cb) {
    unsigned long long h = mp_mix64(seed ^ ((unsigned long long)(unsigned)stream * 0xD1B54A32D192ED03ull));
    h = mp_mix64(h ^ (((unsigned long long)(unsigned)step << 8) | (unsigned)cb));
    return (float)(h >> 40) * (1.0f / 16777216.0f);
}

// Fused cross-attention for one decode step (replaces the xq GEMV + XA attention
// + xo GEMV). With K'_t = W_q^T K_t and V'_t = W_o V_t precomputed per utterance
// and layer:  x += sum_t softmax_t(K'_t . LN(x) / sqrt(128)) V'_t
// (= o_net(attn(q_net(LN(x)), K, V)), magpie.cpp:1713-1767, by associativity).
struct XaP {
    const float *x;        // [B][768] residual in
    float *part;           // [B][XA_SPLITS][XA_PART] partial softmax states over text-key splits
                           // (merged + added to x in the next op's PRO_XA_LN prologue)
    const float *lnw;      // norm_xattn_query
    float eps;
    const float *kp, *vp;  // K', V': [B][L][Tmax][768]
    const int *T;
    int Tmax, layer, nlayers;
    int q_f16;             // F16 weight mode: LN(x) rounded to f16, the q_net operand ggml multiplies
    unsigned long long *ts;  // profiling (nullable): [first wave start, last wave end], s_memrealtime ticks
    // x2 (nullable; the O-projection's XA tail at 16 slots): the split states published as
    // {tag, value} granules gh[b][split][XA_PART]; each of a slot's XA_SPLITS workgroups
    // merges 768 / XA_SPLITS outputs with x1 into x2[b][768] (FFN up then normalises
    // plain rows)
    float *x2;
    unsigned long long *gh;
};

// Cross-attention with Q8_0 q_net / o_net (weight mode MP_WEIGHTS_Q8) after the
// q GEMV: x2 = x + Q8(o_net) attn(q, K, V), the attention output quantised where
// ggml quantises it (magpie.cpp:1713-1767, 3513-3519).
constexpr int XQ8_QIN_NB = 2;      // Q8_0 XA in the O-projection launch: q in the attention workgroups up to this batch
struct XaQ8P {
    const float *x;                 // [B][768]
    float *x2;                      // [B][768]
    const float *q;                 // [B][128] = Q8(q_net) LN(x)
    const signed char *wo;          // o_net int8 [768][128]
    const unsigned short *wod;      //   fp16 block scales [768][4]
    const float *wof;               // or f32 o_net [768][128] (direct f32 XA, long texts)
    const float *xak, *xav;         // XA K, V [B][L][Tmax][128]
    const int *T;
    int Tmax, layer, nlayers;
    // EPI_RESID_XQ8 (the XA in the Q8_0 O-projection's launch): q = Q8(q_net) Q8(LN(x1) * lnw)
    // from the handed-off x1, handed to the attention workgroups as granules qg[B][128]
    const signed char *wq;          // q_net int8 [128][768] as stored
    const unsigned short *wqd;      //   fp16 block scales [128][24]
    const float *lnw;               // norm_xattn_query
    float eps;
    unsigned long long *qg;         // [B][128] {tag, value} granules of q
    int qin;                        // 1: q computed in the attention workgroups (no q granules)
};

struct AttnP {  // decode self-attention (one query per utterance)
    const float *q;
    const float *kc, *vc;    // bf16 elements when kv16
    int layer, nlayers, max_seq;
    const int *pos;
    int kv16;
    float *part;         // [B][NH][SA_SPLITS][SA_PART] partial softmax states over key splits
                         // (merged in the O-projection's PRO_SA_MERGE prologue)
    unsigned long long *ts;  // profiling (nullable): [first wave start, last wave end], s_memrealtime ticks
    // merged (nullable; sa_attn_kernel at 16 slots): the split states published as {tag,
    // value} granules gh[b][h][split][SA_PART] (tag iter[0] * 64 + layer + 1); each of a
    // head's SA_SPLITS workgroups merges 64 / SA_SPLITS of its dims into merged[b][768]
    // (the O-projection then reads plain rows)
    float *merged;
    unsigned long long *gh;
    const int *iter;
    int *hx_err;
};

struct GemvP {
    const float *W;
    const unsigned short *Wb;  // bf16 weights in MFMA fragment order (mp_decode_b16.hip), or null
    const signed char *Wq;     // Q8_0 weights as stored: int8 [N][K] (mp_decode_q8.hip), or null
    const unsigned short *Wd;  //   and their fp16 block scales [N][K/32]
    int q4;                    // Wq holds Q4_0 nibble fragments (pack_q4), not int8 ones
    int N;
    const float *bias;
    // prologue inputs
    const float *src;
    int src_ld;
    const unsigned short *src_b16;  // PRO_PLAIN in the bf16 kernels: rows already bf16 (EPI_GELU_B16 output)
    const float *lnw;
    float eps;
    float *hidden_out;   // PRO_LN: block 0 stores the normalised vector (decoder hidden)
    float *trace;        // optional [B][trace_steps][768] hidden trace
    int trace_steps;
    const int *pos;      // [B] decoder position
    float *xres;         // [B][768] residual stream
    int layer, nlayers;
    const float *lt_s;   // [B][9][256]
    const float *ptab;   // [8][2024][256] in_proj(audio_emb) + b
    const float *qkvtab; // [7][2024][768] LT q|k|v of codebook c's code v at position c+1
    int cb;
    const float *lt_pos;
    float *ltX;
    const float *ltq, *ltk, *ltv;
    const float *logits;  // [B][2024]
    int *codes_cur;       // [B][8]
    const int *step;      // [B]
    int ignore_eos, audio_bos, audio_eos;
    Sampling smp;
    // epilogue outputs
    float *out;
    int out_ld;
    unsigned short *out_b16;        // EPI_GELU_B16
    float *resid;
    const float *addsrc;
    float *kc, *vc;      // SA cache; bf16 elements when kv16 (mp_hip_set_kv_mode)
    int kv16;
    int max_seq;
    float *lq, *lk, *lv;
    // early exit once every slot is done (count >= nslots)
    const int *ndone;
    int nslots;
    const float *part;   // PRO_SA_MERGE: [B][NH][SA_SPLITS][SA_PART]; PRO_XA_LN: [B][XA_SPLITS][XA_PART]
    unsigned long long *ts;  // profiling (nullable): [first wave start, last wave end], s_memrealtime ticks
    // EPI_RESID_XA (O-projection + cross-attention in one launch): the O-projection's
    // workgroups publish x1 = x + W_o attn as 8-byte {tag, value} granules xh[B][768]
    // (relaxed agent-scope atomic stores: write-through, no fence); the last
    // XA_SPLITS x B workgroups prefetch their K'/V' rows, sweep the granules until
    // every tag equals this launch's (iteration counter * 64 + layer + 1, never 0;
    // xh is zeroed per batch) and run xa_part on x1. A sweep that never completes
    // gives up after a bound and raises *hx_err.
    XaP xa;
    unsigned long long *xh;
    // EPI_QKV_SA (QKV projection + self-attention in one launch): the QKV workgroups
    // publish q|k|v as {tag, value} granules qh[B][2304] (tag as for xh); the last
    // NH x SA_SPLITS x B workgroups prefetch their cached K/V rows (keys < pos), sweep
    // their head's granules and run the split's attention (the new key from the
    // granules, not from the cache row this launch writes)
    AttnP sa;
    XaQ8P xq8;           // EPI_RESID_XQ8: the q_net of the launch's tail
    unsigned long long *qh;
    // split-K 16-bit GEMMs (gemm_b16_kernel KS > 1): each of a row tile's KS workgroups
    // publishes its 16 x 16 partial tile as {tag, value} granules kgh[tile][KS][256] (tag
    // as for xh) and merges 16 / KS of the tile's rows from the KS partials in split order
    unsigned long long *kgh;
    const int *iter;
    int *hx_err;
    int nrow_blocks;     // set by the launcher: workgroups of the O-projection
    // diagnostics (MAGPIE_Q8DUMP, gemm_q8_kernel_dec only; nullable): this launch's f32
    // activation rows [NB][K], their Q8_0 blocks (int8 [NB][K], fp16 d as f32 [NB][K/32])
    // and every integer block dot [N][K/32][NB] (int32), as the kernel's operands give them
    void *q8dump;
    // f32 LT head at batch 1, greedy (nullable): every workgroup also publishes its masked
    // first-max logit as one ordered 64-bit key cand[blockIdx.x] (lt_cand_key), so the next
    // LT step picks the code from the head's ~253 workgroup candidates instead of its 2024 logits
    unsigned long long *cand;
};

// Q8_0 weight mode: the LT step of codebook cb as LTQ_P workgroups per slot
// (lt_slot_q8_kernel): pick, gathers and attention as lt_pick_kernel (g), the Q8_0 o_net
// of 256 / LTQ_P rows per workgroup (ggml's Q8_0 x Q8_0 dot: the attention output quantised per
// 32-block, per-block integer dots times d_w d_a, blocks in order) published as y
// granules, the F32 FFN (the Q8 file's FFN convs) for 1024 / LTQ_P hidden units per workgroup,
// partial sums merged through granules into y2 for the Q8_0 head.
struct LtSlotQ8P {
    GemvP g;                       // pick / gathers / attention fields (lt_pick_kernel's), cb
    const signed char *woq;        // o_net int8 [256][256] (Q4_0 blocks as q - 8)
    const signed char *wot;        // the same transposed by 16-byte chunks [16][256][16] (RED: every workgroup all rows)
    float *part;                   // DEFER (batch 1): plain partial sums [LTQ_P][256], merged by the head's prologue
    const unsigned short *wod;     // o_net fp16 block scales [256][8]
    const float *lnw;              // norm_pos_ff
    float eps;
    const float *w1;               // FFN up f32 [1024][256]
    const float *w2s;              // FFN down f32 slice-major [LTQ_P][256][1024 / LTQ_P]
    float *y, *y2;                 // [B][256] attention residual (ltY) and FFN output (the head's input)
    unsigned long long *gy, *gp;   // granules: y [B][256] (tag iter * 64 + 32 + cb), partials [B][LTQ_P][256] (+ 48 + cb)
    const int *iter;
    int *hx_err;
    unsigned long long *ts;
};

// error bits raised in *hx_err (ndone[2]) by an in-launch hand-off that gave up
constexpr int HX_ERR_XA = 1, HX_ERR_SA = 2, HX_ERR_LT = 4, HX_ERR_KS = 8;
constexpr int KGH_MAX_KS = 8;  // split-K granule buffers hold up to this many slices per tile

struct FinP {
    const float *logits;
    int *codes_cur, *codes_prev, *codes_out;
    int *step, *pos, *done, *nframes, *ndone;
    int max_steps, ignore_eos, audio_bos, audio_eos, nslots;
    Sampling smp;
    int emit_eos;   // streaming semantics: the EOS frame's codes are emitted too (magpie.cpp:4800-4806)
    int lt_only;    // magpie_local_transformer_sample_all: pick codebook 7, no loop bookkeeping
    int *iter;      // decode iteration counter (tags of the in-launch hand-offs), +1 per iteration
    unsigned long long *ts;  // profiling (nullable): [first wave start, last wave end], s_memrealtime ticks
    // the next frame's decoder input (magpie.cpp:2746-2787): for a slot that advances,
    // x[b] = (sum over codebooks of emb[cb][code]) / 8 + pos_emb[new pos] (null: not written)
    const float *emb, *pos_emb;
    float *x;
    int pos_rows;   // rows of pos_emb (the speculative read of the next position is clamped to it)
};



}  // namespace mp
