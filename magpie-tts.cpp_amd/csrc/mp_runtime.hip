// Host runtime of the MI355X decode path: weight residency, per-batch device
// state, the per-utterance preamble, and the hipGraph-captured frame loop.
// Exposes the C-ABI declared in include/magpie_hip.h.
//
// Design: one mp_dev per GPU. Weights are uploaded once (f32, one
// arena). A batch of B utterances (1..8 with f32 weights, 1..16 in the bf16 / F16 /
// Q8_0 / Q4_0 modes: mp_hip_max_batch) occupies NB = next_pow2(B) slots; every
// per-utterance quantity (residual stream, KV cache, XA K/V, codes, position,
// done flag) lives in HBM and is addressed by slot, so one decode iteration
// (12 decoder layers + 8-codebook local transformer + EOS bookkeeping, 65
// kernels at NB=1 in the f32 mode) is captured once as a hipGraph and replayed per frame with
// no host round trip; the host only polls the done counter every few frames.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <future>
#include <memory>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/magpie_hip.h"
#include "mp_gguf.hpp"
#include "mp_device.hpp"
#include "mp_params.hpp"


namespace mp {

// ---- launchers (mp_decode.hip / mp_prefill.hip)
using GemvFn = hipError_t (*)(const GemvP &, hipStream_t);
#define MP_DECL_OPS(NB)                                                                                     \
    hipError_t op_qkv_##NB(const GemvP &, hipStream_t);        \
    hipError_t op_oproj_##NB(const GemvP &, hipStream_t); hipError_t op_ff1_##NB(const GemvP &, hipStream_t);            \
    hipError_t op_ff1x_##NB(const GemvP &, hipStream_t); hipError_t op_oproj_xa_##NB(const GemvP &, hipStream_t);       \
    hipError_t op_qkv_sa_##NB(const GemvP &, hipStream_t); hipError_t op_xq_##NB(const GemvP &, hipStream_t); \
    hipError_t op_ff2_##NB(const GemvP &, hipStream_t); hipError_t op_lt_in0_##NB(const GemvP &, hipStream_t);           \
    hipError_t op_lt_a_##NB(const GemvP &, hipStream_t); hipError_t op_lt_b_##NB(const GemvP &, hipStream_t);            \
    hipError_t op_lt_bg_##NB(const GemvP &, hipStream_t);                                                              \
    hipError_t op_lt_c_##NB(const GemvP &, hipStream_t); hipError_t op_lt_d_##NB(const GemvP &, hipStream_t);            \
    hipError_t op_lt_e_##NB(const GemvP &, hipStream_t);
MP_DECL_OPS(1)
MP_DECL_OPS(2)
MP_DECL_OPS(4)
MP_DECL_OPS(8)
hipError_t op_lt_in0_16(const GemvP &, hipStream_t);
#define MP_DECL_B16(NB)                                                                                      \
    hipError_t b16_qkv_##NB(const GemvP &, hipStream_t);      \
    hipError_t b16_oproj_##NB(const GemvP &, hipStream_t); hipError_t b16_ff1_##NB(const GemvP &, hipStream_t);          \
    hipError_t b16_ff2_##NB(const GemvP &, hipStream_t); hipError_t b16_lt_a_##NB(const GemvP &, hipStream_t);           \
    hipError_t b16_lt_bg_##NB(const GemvP &, hipStream_t); hipError_t b16_lt_b_##NB(const GemvP &, hipStream_t);         \
    hipError_t b16_lt_c_##NB(const GemvP &, hipStream_t); hipError_t b16_lt_d_##NB(const GemvP &, hipStream_t);          \
    hipError_t b16_lt_e_##NB(const GemvP &, hipStream_t); hipError_t b16_oproj_xa_##NB(const GemvP &, hipStream_t); \
    hipError_t b16_qkv_sa_##NB(const GemvP &, hipStream_t); hipError_t b16_ff1p_##NB(const GemvP &, hipStream_t); \
    hipError_t b16_lt_es_##NB(const GemvP &, hipStream_t); hipError_t b16_lt_em_##NB(const GemvP &, hipStream_t);
MP_DECL_B16(1)
MP_DECL_B16(2)
MP_DECL_B16(4)
MP_DECL_B16(8)
MP_DECL_B16(16)
#define MP_DECL_F16(NB)                                                                                      \
    hipError_t f16_qkv_##NB(const GemvP &, hipStream_t);      \
    hipError_t f16_oproj_##NB(const GemvP &, hipStream_t); hipError_t f16_ff1_##NB(const GemvP &, hipStream_t);          \
    hipError_t f16_ff2_##NB(const GemvP &, hipStream_t); hipError_t f16_lt_a_##NB(const GemvP &, hipStream_t);           \
    hipError_t f16_lt_bg_##NB(const GemvP &, hipStream_t); hipError_t f16_lt_b_##NB(const GemvP &, hipStream_t);         \
    hipError_t f16_lt_c_##NB(const GemvP &, hipStream_t); hipError_t f16_lt_d_##NB(const GemvP &, hipStream_t);          \
    hipError_t f16_lt_e_##NB(const GemvP &, hipStream_t); hipError_t f16_lt_in0_##NB(const GemvP &, hipStream_t); \
    hipError_t f16_oproj_xa_##NB(const GemvP &, hipStream_t); hipError_t f16_qkv_sa_##NB(const GemvP &, hipStream_t);
MP_DECL_F16(1)
MP_DECL_F16(2)
MP_DECL_F16(4)
MP_DECL_F16(8)
MP_DECL_F16(16)
hipError_t f16_lt_inh_1(const GemvP &, hipStream_t);
hipError_t f16_lt_bo_8(const GemvP &, hipStream_t);
hipError_t f16_lt_bo_16(const GemvP &, hipStream_t);
hipError_t pack_b16(const float *, int, int, unsigned short *, hipStream_t, bool f16);
#define MP_DECL_Q8(NB)                                                                                       \
    hipError_t q8_qkv_##NB(const GemvP &, hipStream_t);        \
    hipError_t q8_oproj_##NB(const GemvP &, hipStream_t); hipError_t q8_xq_##NB(const GemvP &, hipStream_t);             \
    hipError_t q8_lt_in0_##NB(const GemvP &, hipStream_t);                                                             \
    hipError_t q8_lt_a_##NB(const GemvP &, hipStream_t); hipError_t q8_lt_bg_##NB(const GemvP &, hipStream_t);           \
    hipError_t q8_lt_b_##NB(const GemvP &, hipStream_t); hipError_t q8_lt_e_##NB(const GemvP &, hipStream_t);           \
    hipError_t q8_qkv_sa_##NB(const GemvP &, hipStream_t); hipError_t q8_oproj_xq_##NB(const GemvP &, hipStream_t);
MP_DECL_Q8(1)
MP_DECL_Q8(2)
MP_DECL_Q8(4)
MP_DECL_Q8(8)
MP_DECL_Q8(16)
hipError_t q8_lt_bo_16(const GemvP &, hipStream_t);
hipError_t op_ff1_16(const GemvP &, hipStream_t);
hipError_t op_ff2_16(const GemvP &, hipStream_t);
hipError_t op_xq_16(const GemvP &, hipStream_t);
hipError_t op_lt_in0_16(const GemvP &, hipStream_t);
hipError_t pack_q8(const signed char *, const unsigned short *, int, int, unsigned char *, unsigned short *, hipStream_t);
hipError_t pack_q4(const signed char *, int, int, unsigned char *, hipStream_t);
hipError_t q8_lt_inh_1(const GemvP &, hipStream_t);
hipError_t q8_lt_em_1(const GemvP &, hipStream_t);
hipError_t q8_lt_emf_1(const GemvP &, hipStream_t);
hipError_t op_lt_pick(const GemvP &, int, hipStream_t);
hipError_t op_embed(const EmbP &, int, hipStream_t);
hipError_t op_lt_bo_8(const GemvP &, hipStream_t);
hipError_t b16_lt_bo_8(const GemvP &, hipStream_t);
hipError_t b16_lt_bo_16(const GemvP &, hipStream_t);
hipError_t q8_lt_bo_8(const GemvP &, hipStream_t);
hipError_t op_lt_em_1(const GemvP &, hipStream_t);
int b16_oproj_ks();
hipError_t op_lt_ffn(const LtFfnP &, int, hipStream_t);
hipError_t op_lt_merge(const LtFfnP &, int, hipStream_t);
hipError_t op_lt_ffn2(const LtFfn2P &, int, hipStream_t);
hipError_t op_lt_slot(const LtFfn2P &, int, hipStream_t);
hipError_t op_lt_front(const LtFrontP &, hipStream_t);
hipError_t op_lt_all(const LtAllP &, hipStream_t);
hipError_t op_lt_slot_q8(const LtSlotQ8P &, int, hipStream_t);
hipError_t op_lt_kvo(const GemvP &, int, hipStream_t);
hipError_t op_sa_attn(const AttnP &, int, hipStream_t);
hipError_t b16_oproj_xa_pm_16(const GemvP &, hipStream_t);
hipError_t b16_oproj_xa_pm_8(const GemvP &, hipStream_t);
hipError_t op_xa(const XaP &, int, hipStream_t);
hipError_t op_xa_q8(const XaQ8P &, int, hipStream_t);
hipError_t op_finalize(const FinP &, int, hipStream_t);

}  // namespace mp

#include "mp_prefill_api.hpp"

namespace mp {

// ff1: LN(x2) prologue (x2 materialised: Q8 unfused XA); ff1x: the fused XA's split states merged into x2 first
// oproj_xa: O-projection + the fused XA in one launch (EPI_RESID_XA)
// qkv_sa: the QKV projection + the SA in one launch (EPI_QKV_SA)
// xq: the direct XA's f32 q_net GEMV (f32 and bf16 modes); ff1: FFN up from a materialised x2
struct OpTable { GemvFn qkv, oproj, ff1, ff1x, ff2, lt_in0, lt_a, lt_bg, lt_b, lt_c, lt_d, lt_e, oproj_xa,
                 qkv_sa, xq, lt_es, lt_em; };
#define MP_TABLE(NB) { op_qkv_##NB, op_oproj_##NB, op_ff1_##NB, op_ff1x_##NB, op_ff2_##NB, \
                       op_lt_in0_##NB, op_lt_a_##NB, op_lt_bg_##NB, op_lt_b_##NB, op_lt_c_##NB, op_lt_d_##NB, op_lt_e_##NB, \
                       op_oproj_xa_##NB, op_qkv_sa_##NB, op_xq_##NB }
// 16 slots in the f32 family only for a Q8_0 file's F32 tensors: its FFN convs and LT in_proj
static const OpTable kTables[5] = {MP_TABLE(1), MP_TABLE(2), MP_TABLE(4), MP_TABLE(8),
                                   {nullptr, nullptr, op_ff1_16, nullptr, op_ff2_16, op_lt_in0_16, nullptr,
                                    nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, op_xq_16}};
// bf16 weight mode: every projection on MFMA except the f32 LT in_proj
#define MP_TABLE_B16(NB) { b16_qkv_##NB, b16_oproj_##NB, b16_ff1p_##NB, b16_ff1_##NB, b16_ff2_##NB, \
                           op_lt_in0_##NB, b16_lt_a_##NB, b16_lt_bg_##NB, b16_lt_b_##NB, b16_lt_c_##NB,  \
                           b16_lt_d_##NB, b16_lt_e_##NB, b16_oproj_xa_##NB, b16_qkv_sa_##NB, op_xq_##NB, b16_lt_es_##NB, b16_lt_em_##NB }
static const OpTable kTablesB16[5] = {MP_TABLE_B16(1), MP_TABLE_B16(2), MP_TABLE_B16(4), MP_TABLE_B16(8),
                                      MP_TABLE_B16(16)};
// F16 weight mode (an F16 GGUF): the same MFMA family on f16, the LT in_proj included
#define MP_TABLE_F16(NB) { f16_qkv_##NB, f16_oproj_##NB, nullptr, f16_ff1_##NB, f16_ff2_##NB, \
                           f16_lt_in0_##NB, f16_lt_a_##NB, f16_lt_bg_##NB, f16_lt_b_##NB, f16_lt_c_##NB,  \
                           f16_lt_d_##NB, f16_lt_e_##NB, f16_oproj_xa_##NB, f16_qkv_sa_##NB }
static const OpTable kTablesF16[5] = {MP_TABLE_F16(1), MP_TABLE_F16(2), MP_TABLE_F16(4), MP_TABLE_F16(8),
                                      MP_TABLE_F16(16)};
// Q8_0 weight mode: the projections whose tensors are Q8_0 in the file (mp_decode_q8.hip)
struct OpTableQ8 { GemvFn qkv, oproj, xq, lt_in0, lt_a, lt_bg, lt_b, lt_e, qkv_sa, oproj_xq; };
#define MP_TABLE_Q8(NB) { q8_qkv_##NB, q8_oproj_##NB, q8_xq_##NB, q8_lt_in0_##NB, \
                          q8_lt_a_##NB, q8_lt_bg_##NB, q8_lt_b_##NB, q8_lt_e_##NB, q8_qkv_sa_##NB, q8_oproj_xq_##NB }
static const OpTableQ8 kTablesQ8[5] = {MP_TABLE_Q8(1), MP_TABLE_Q8(2), MP_TABLE_Q8(4), MP_TABLE_Q8(8),
                                        MP_TABLE_Q8(16)};
static int nb_index(int NB) { return NB == 1 ? 0 : NB == 2 ? 1 : NB == 4 ? 2 : NB == 8 ? 3 : 4; }
// the 16-bit MFMA family serves the bf16 and F16 weight modes
static bool h16_mode(int weight_mode) { return weight_mode == MP_WEIGHTS_BF16 || weight_mode == MP_WEIGHTS_F16; }
static const OpTable &table_for(int NB, int weight_mode) {
    return weight_mode == MP_WEIGHTS_F16 ? kTablesF16[nb_index(NB)]
           : weight_mode == MP_WEIGHTS_BF16 ? kTablesB16[nb_index(NB)]
                                            : kTables[nb_index(NB)];
}
static const OpTableQ8 &table_q8(int NB) { return kTablesQ8[nb_index(NB)]; }

// A Q8_0 tensor (weight mode MP_WEIGHTS_Q8): as stored, int8 [N][K] + fp16 scales
// [N][K/32] (the preamble GEMMs), and for the decode projections also in int8 MFMA
// fragment order (pq, pd: mp_decode_q8.hip)
struct QW {
    const signed char *q = nullptr;
    const unsigned short *d = nullptr;
    const signed char *pq = nullptr;
    const unsigned short *pd = nullptr;
    int nib = 0;        // a Q4_0 tensor: pq holds nibble fragments (pack_q4, 18 B per 32 weights)
    size_t head_q = 0;  // bytes between consecutive heads' fragments (the 8 LT output heads)
    explicit operator bool() const { return q != nullptr; }
};
// bytes of a packed Q8_0 tensor: fragments and scales (Q4_0: half the fragment bytes)
static size_t q8p_qbytes(int N, int K) { return (size_t)((N + 15) / 16) * (K / 64) * 1024; }
static size_t q4p_qbytes(int N, int K) { return (size_t)((N + 15) / 16) * (K / 64) * 512; }
static size_t q8p_dbytes(int N, int K) { return (size_t)((N + 15) / 16) * (K / 64) * 64; }

struct EncLayerW { const float *norm_self, *qkv, *o, *norm_ff, *ff1, *ff2; QW qkv8, o8; };
struct DecLayerW {
    const float *norm_self, *qkv, *o, *norm_xq, *xq, *xkv, *xo, *norm_xmem, *norm_ff, *ff1, *ff2;
    QW qkv8, o8, xq8, xkv8, xo8;
};

struct Model {
    int enc_layers = 6, dec_layers = 12, n_spk = 5, dec_pos_rows = 0, text_vocab = 2380;
    int audio_bos = 2016, audio_eos = 2017, max_dec_steps = 500;
    float eps = 1e-5f;
    const float *text_emb = nullptr, *enc_pos = nullptr, *enc_norm_out = nullptr, *dec_pos = nullptr;
    const float *dec_norm_out = nullptr, *baked = nullptr, *audio_emb = nullptr;
    std::vector<EncLayerW> enc;
    std::vector<DecLayerW> dec;
    const float *lt_in_w, *lt_in_b, *lt_pos, *lt_norm_self, *lt_qkv, *lt_o, *lt_norm_ff, *lt_ff1, *lt_ff2, *lt_out_w,
        *lt_out_b;
    float *lt_ptab = nullptr;  // [8][2024][256] = in_proj(audio_emb[c][v]) + b, built at load
    float *lt_qkvtab = nullptr;  // [7][2024][768] = qkv_net(LN(ptab[c][v] + lt_pos[c+1])), built at load
    // f32 weight mode (lt_ffn2_kernel): [7][2024][256] = o_net(v third of lt_qkvtab), and
    // [512][256] = [W_k ; W_o W_v] for position 0 (W_o W_v formed in double on the host)
    float *lt_votab = nullptr, *lt_kvo = nullptr;
    // the LT FFN-down weights [256][1024] re-laid slice-major [LT_FFN_P][256][16]: the FFN
    // workgroup that owns hidden units [16p, 16p+16) reads one contiguous 16 KiB block
    // instead of 256 half cache lines (whose other halves sit with workgroup p +- 1 on
    // another XCD: every line was fetched twice)
    float *lt_ff2s = nullptr;
    // bf16 weight mode (lt_slot_kernel): the LT FFN weights rounded to bf16, W1 row-major
    // [1024][256] and W2 slice-major [LTS_P][256][1024 / LTS_P]
    unsigned short *lt_ff1h = nullptr, *lt_ff2h = nullptr;
    // Q8_0 weight mode (lt_slot_q8_kernel): the F32 FFN-down weights slice-major [LTQ_P][256][1024 / LTQ_P]
    float *lt_ff2q = nullptr;
    std::vector<float *> xq_t;  // per layer W_q^T [768][128] (for K' = K W_q)
    // weight mode MP_WEIGHTS_BF16: decode projections repacked as bf16 MFMA fragments
    int weight_mode = 0;
    unsigned short *pk_arena = nullptr;
    std::vector<const unsigned short *> pk_qkv, pk_o, pk_ff1, pk_ff2;
    const unsigned short *pk_lt_qkv = nullptr, *pk_lt_o = nullptr, *pk_lt_ff1 = nullptr, *pk_lt_ff2 = nullptr,
                         *pk_lt_out = nullptr,  // lt_out: [8][127 tiles][8][64][8]
                         *pk_lt_in = nullptr;   // F16 mode only: the LT in_proj [256][768]
    // weight mode MP_WEIGHTS_Q8: the file's Q8_0 tensors as stored (ggml's quantised mul_mat)
    void *q8_arena = nullptr, *q8p_arena = nullptr;
    size_t q8_bytes = 0;
    bool q8_all = false;  // every decode projection is Q8_0 / Q4_0: batches up to 16
    QW lt_in8, lt_qkv8, lt_o8, lt_out8;  // lt_out8: [8][2024][256] (+ [8][2024][8] scales)
    const signed char *lt_o8t = nullptr;  // lt_o8's int8 transposed by 16-byte chunks [16][256][16] (lt_slot_q8_kernel)
    float *arena = nullptr;
    size_t arena_bytes = 0;
};

enum OpKind { K_GEMV = 0, K_ATTN = 1, K_FIN = 2, K_XA = 3, K_XAQ8 = 5, K_LTFFN = 6, K_LTMERGE = 7, K_LTPICK = 8, K_EMBED = 9,
              K_LTFFN2 = 10, K_LTKVO = 11, K_LTSLOT = 12, K_LTFRONT = 13, K_LTSLOTQ8 = 14, K_LTALL = 15 };
// the f32 batch-1 LT's granules (one zeroed buffer): the front's in_proj / vo_0 / k_0, then
// lt_all_kernel's FFN-down partials, y2 and workgroup keys
constexpr size_t LTFG_GP = 3 * 256, LTFG_GY = LTFG_GP + (size_t)LT_FFN_P * 256, LTFG_GC = LTFG_GY + 256,
                 LTFG_TOTAL = LTFG_GC + 128;
struct OpRec {
    std::string name;
    int kind;
    GemvFn fn;
    GemvP g;
    AttnP a;
    FinP f;
    XaP x;
    XaQ8P xq;
    LtFfnP lf;
    LtFfn2P l2;
    LtFrontP lf3;
    LtAllP la;
    LtSlotQ8P lq8;
    EmbP e;
    int B;
    double bytes;
    bool add_sa = false;  // the launch also runs the SA (EPI_QKV_SA): its live-cache bytes are added
};

// Buffers of the local-transformer + bookkeeping part of an iteration
struct LtIo {
    float *x, *hidden, *trace;
    int trace_steps;
    float *lt_s, *ltX, *ltY, *lty2, *ltq, *ltk, *ltv, *ltf, *logits;
    float *ltp;  // [NB][LT_FFN_P][256] partial FFN-down sums (lt_ffn_kernel; lt_slot_kernel: [NB][LTS_P][256])
    unsigned long long *ltgh;  // [NB][LTS_P or LTQ_P][256] lt_slot(_q8)_kernel's partial-sum granules
    unsigned long long *ltfg;  // lt_front / lt_all_kernel's hand-off granules (f32, batch 1; LTFG_* below)
    unsigned long long *ltcand;  // [256] the f32 batch-1 head's workgroup candidates (GemvP::cand; null: off)
    unsigned long long *ltyg;  // [NB][256] lt_slot_q8_kernel's y granules (Q8_0 mode)
    int *iter, *hx_err;        // decode iteration counter (hand-off tags), hand-off error bits
    int *codes_cur, *codes_prev, *codes_out, *step, *pos, *done, *nframes, *ndone, *argeos, *amax;
    SmpCfg *cfg;
    int sampling, ignore_eos, emit_eos, max_steps, lt_only;
};
hipError_t op_lt_inh_1(const GemvP &, hipStream_t);

}  // namespace mp

struct mp_dev {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    mp::Model m;
    bool loaded = false;
    // batch configuration
    int B = 0, NB = 0, Tmax = 0, max_steps = 0, max_seq = 0, nch = 0;
    mp_params params{};
    int kv_mode = MP_KV_F32;  // mp_hip_set_kv_mode: applies from the next mp_hip_begin_batch
    int xa_mode = MP_XA_AUTO;  // mp_hip_set_xa_mode: likewise
    bool xa_direct = false;    // this batch runs the direct XA form (f32 / bf16 modes)
    int kv16 = 0;             // the current batch's SA cache holds bf16
    // device state (one allocation per buffer, sized for the configuration)
    std::vector<void *> allocs;
    float *x = nullptr, *x2 = nullptr, *kp = nullptr, *vp = nullptr, *q = nullptr, *sa_out = nullptr,
          *h = nullptr, *hidden = nullptr;
    float *xqb = nullptr;  // Q8 mode: q_net output [NB][128]
    unsigned short *h_b16 = nullptr;  // bf16 mode: GELU(FFN up) as the bf16 FFN-down operand [NB][3072]
    float *gpart = nullptr;            // preamble split-K partial sums (mp::gemm_splits)
    hipEvent_t sev[2] = {nullptr, nullptr};  // streaming: the two chunk snapshots landed
    int32_t *h_codes = nullptr;              // streaming: pinned host mirror of codes_out [NB][S][8] + snapshots
    size_t h_codes_n = 0;
    float *sa_part = nullptr, *xa_part = nullptr;  // split-K attention states [NB][12][4][68], [NB][4][772]
    unsigned long long *sagh = nullptr, *xagh = nullptr;  // 16-slot merges: split-state granules
    unsigned long long *kgh = nullptr;  // split-K FFN-down partial tiles (16-bit modes): [48][KS][256]
    unsigned long long *xh = nullptr;  // O-projection -> XA hand-off granules [NB][768] (EPI_RESID_XA)
    unsigned long long *qh = nullptr;  // QKV -> SA hand-off granules [NB][2304] (EPI_QKV_SA)
    unsigned long long *xqh = nullptr; // Q8_0 XA q_net -> attention hand-off granules [NB][128] (EPI_RESID_XQ8)
    float *kc = nullptr, *vc = nullptr, *xak = nullptr, *xav = nullptr;
    float *lt_s = nullptr, *ltX = nullptr, *ltY = nullptr, *lty2 = nullptr, *ltq = nullptr, *ltk = nullptr,
          *ltv = nullptr, *ltf = nullptr, *logits = nullptr, *trace = nullptr, *ltp = nullptr;
    unsigned long long *ltgh = nullptr, *ltfg = nullptr, *ltyg = nullptr, *ltcand = nullptr;
    int *T = nullptr, *spk = nullptr, *pos = nullptr, *step = nullptr, *done = nullptr, *nframes = nullptr,
        *ndone = nullptr, *codes_cur = nullptr, *codes_prev = nullptr, *codes_out = nullptr, *tok = nullptr,
        *argeos = nullptr, *amax = nullptr;
    mp::SmpCfg *smpcfg = nullptr;
    int lt_calls = 0;
    // magpie_local_transformer_sample_all scratch (batch 1, independent of any batch)
    std::vector<void *> lt_allocs;
    mp::LtIo lt_io{};
    // preamble scratch
    float *pX = nullptr, *pH = nullptr, *pQKV = nullptr, *pATT = nullptr, *pF = nullptr, *pXQ = nullptr,
          *pXAO = nullptr, *enc_out = nullptr;
    // graph
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    std::vector<mp::OpRec> ops;
    bool batch_ready = false;
    mp_timing timing{};
    int *h_ndone = nullptr;  // pinned
    // mp_hip_encode_text's private workspace: grows on demand, freed by mp_hip_free (a
    // per-call hipFree would synchronise the whole device, stalling other streams' work)
    char *enc_ws = nullptr;
    size_t enc_ws_bytes = 0;
    // streaming rounds overlapped with a background codec: the frame loop on the CUs the
    // codec's background stream leaves (cu_share_mask complement), created on first use
    hipStream_t stream_fg = nullptr;
    int stream_fg_cus = 0;
    // diagnostics (MAGPIE_Q8DUMP=1 at mp_hip_begin_batch, Q8_0 weights): one dump slot per
    // int8-MFMA decode GEMM launch of the iteration (GemvP::q8dump), records in q8dump_index
    char *q8dump = nullptr;
    size_t q8dump_slot = 0;
    int q8dump_cap = 0, q8dump_n = 0;
    bool q8dump_live = false;  // set while enqueue_iteration runs (not for mp_hip_lt_sample)
    std::vector<int> q8dump_index;
};

namespace {

#define HIPCHK(expr)                                                                           \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess) {                                                                \
            dev->err = std::string(#expr) + " failed: " + hipGetErrorString(e_);               \
            return MP_ERR_HIP;                                                                 \
        }                                                                                      \
    } while (0)

int fail(mp_dev *dev, int code, const std::string &msg) {
    dev->err = msg;
    return code;
}

template <class T> int dalloc(mp_dev *dev, T **p, size_t count) {
    void *v = nullptr;
    HIPCHK(hipMalloc(&v, count * sizeof(T) + 256));
    HIPCHK(hipMemsetAsync(v, 0, count * sizeof(T) + 256, dev->stream));
    dev->allocs.push_back(v);
    *p = (T *)v;
    return MP_OK;
}

void free_batch(mp_dev *dev) {
    if (dev->exec) hipGraphExecDestroy(dev->exec);
    if (dev->graph) hipGraphDestroy(dev->graph);
    dev->exec = nullptr;
    dev->graph = nullptr;
    for (void *p : dev->allocs) hipFree(p);
    dev->allocs.clear();
    dev->ops.clear();
    dev->batch_ready = false;
    dev->B = dev->NB = dev->Tmax = dev->max_steps = 0;
    dev->xa_direct = false;
    dev->kp = dev->vp = nullptr;
    dev->q8dump = nullptr;  // (one of allocs)
    dev->q8dump_cap = dev->q8dump_n = 0;
    dev->q8dump_index.clear();
}

// MAGPIE_Q8DUMP: give a Q8_0 decode GEMM launch its dump slot and index record
// [N, K, NB, layer, cb, byte offset, name (40 bytes)] (16 ints)
constexpr int Q8DUMP_REC = 16;
void q8dump_assign(mp_dev *dev, const char *name, mp::GemvP &g) {
    g.q8dump = nullptr;
    if (!dev->q8dump || !dev->q8dump_live || !g.Wq || dev->q8dump_n >= dev->q8dump_cap) return;
    const int n = dev->q8dump_n++;
    g.q8dump = dev->q8dump + (size_t)n * dev->q8dump_slot;
    const int K = strncmp(name, "lt_in", 5) == 0 ? 768 : (strncmp(name, "lt_", 3) == 0 ? 256 : 768);
    int rec[Q8DUMP_REC] = {g.N, K, dev->NB, g.layer, g.cb, (int)((size_t)n * dev->q8dump_slot)};
    strncpy((char *)&rec[6], name, 39);
    dev->q8dump_index.insert(dev->q8dump_index.end(), rec, rec + Q8DUMP_REC);
}

double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// ------------------------------------------------------------------ weights
// Tensor names and mapping: create_tensors (magpie.cpp:572-672).
// Size (elements) of one packed [N][K] matrix: [ceil(N/16)][K/32][64][8].
size_t pk_elems(int N, int K) { return (size_t)((N + 15) / 16) * 16 * K; }

// bf16 weight mode: the f32 weights rounded to bf16 fragments; F16 mode (an F16
// file): its f16 values (widened exactly at load) repacked as f16 fragments.
int pack_weights(mp_dev *dev, bool f16) {
    mp::Model &m = dev->m;
    if (m.pk_arena) { hipFree(m.pk_arena); m.pk_arena = nullptr; }
    const int L = m.dec_layers;
    const size_t per_layer = pk_elems(2304, 768) + pk_elems(768, 768) + pk_elems(3072, 768) + pk_elems(768, 3072);
    const size_t lt = pk_elems(768, 256) + pk_elems(256, 256) + pk_elems(1024, 256) + pk_elems(256, 1024) +
                      8 * pk_elems(2024, 256) + (f16 ? pk_elems(256, 768) : 0);
    HIPCHK(hipMalloc(&m.pk_arena, (per_layer * L + lt) * 2));
    unsigned short *cur = m.pk_arena;
    auto pack = [&](const float *W, int N, int K) -> const unsigned short * {
        unsigned short *dst = cur;
        cur += pk_elems(N, K);
        return mp::pack_b16(W, N, K, dst, dev->stream, f16) == hipSuccess ? dst : nullptr;
    };
    m.pk_qkv.assign(L, nullptr); m.pk_o.assign(L, nullptr); m.pk_ff1.assign(L, nullptr); m.pk_ff2.assign(L, nullptr);
    for (int l = 0; l < L; ++l) {
        m.pk_qkv[l] = pack(m.dec[l].qkv, 2304, 768);
        m.pk_o[l] = pack(m.dec[l].o, 768, 768);
        m.pk_ff1[l] = pack(m.dec[l].ff1, 3072, 768);
        m.pk_ff2[l] = pack(m.dec[l].ff2, 768, 3072);
        if (!m.pk_qkv[l] || !m.pk_o[l] || !m.pk_ff1[l] || !m.pk_ff2[l]) return fail(dev, MP_ERR_HIP, "bf16 pack failed");
    }
    m.pk_lt_qkv = pack(m.lt_qkv, 768, 256);
    m.pk_lt_o = pack(m.lt_o, 256, 256);
    m.pk_lt_ff1 = pack(m.lt_ff1, 1024, 256);
    m.pk_lt_ff2 = pack(m.lt_ff2, 256, 1024);
    m.pk_lt_out = cur;
    for (int c = 0; c < 8; ++c)
        if (!pack(m.lt_out_w + (size_t)c * 2024 * 256, 2024, 256)) return fail(dev, MP_ERR_HIP, "bf16 pack failed");
    if (!m.pk_lt_qkv || !m.pk_lt_o || !m.pk_lt_ff1 || !m.pk_lt_ff2) return fail(dev, MP_ERR_HIP, "bf16 pack failed");
    m.pk_lt_in = f16 ? pack(m.lt_in_w, 256, 768) : nullptr;
    if (f16 && !m.pk_lt_in) return fail(dev, MP_ERR_HIP, "f16 pack failed");
    HIPCHK(hipStreamSynchronize(dev->stream));
    return MP_OK;
}

int load_model(mp_dev *dev, const char *path) {
    mp::Gguf g;
    std::string err;
    if (!g.open(path, err)) return fail(dev, MP_ERR_IO, err);
    mp::Model &m = dev->m;
    // read_hparams (magpie.cpp:73-121): the reader's keys, struct defaults otherwise
    if (g.get_u32("magpie.d_model", 768) != 768 || g.get_u32("magpie.d_ffn", 3072) != 3072 ||
        g.get_u32("magpie.d_head", 64) != 64 || g.get_u32("magpie.dec_sa_heads", 12) != 12 ||
        g.get_u32("magpie.dec_xa_heads", 1) != 1 || g.get_u32("magpie.dec_xa_d_head", 128) != 128 ||
        g.get_u32("magpie.lt_dim", 256) != 256 || g.get_u32("magpie.lt_ffn_dim", 1024) != 1024 ||
        g.get_u32("magpie.num_codebooks", 8) != 8 || g.get_u32("magpie.vocab_per_cb", 2024) != 2024 ||
        g.get_u32("magpie.context_frames", 110) != 110 || g.get_u32("magpie.enc_heads", 12) != 12 ||
        g.get_u32("magpie.enc_kernel", 3) != 3 || g.get_u32("magpie.dec_kernel", 1) != 1 ||
        g.get_u32("magpie.lt_layers", 1) != 1 || g.get_u32("magpie.lt_heads", 1) != 1)
        return fail(dev, MP_ERR_UNSUPPORTED, "model dimensions differ from Magpie-357M (kernels are specialised)");
    m.enc_layers = (int)g.get_u32("magpie.enc_layers", 6);
    m.dec_layers = (int)g.get_u32("magpie.dec_layers", 12);
    m.n_spk = (int)g.get_u32("magpie.num_speakers", 5);
    m.text_vocab = (int)g.get_u32("magpie.text_vocab_size", 2380);
    m.audio_bos = (int)g.get_u32("magpie.audio_bos_id", 2016);
    m.audio_eos = (int)g.get_u32("magpie.audio_eos_id", 2017);
    // the kernels' forbidden-token mask is the range [bos, bos + 7] minus eos, which is
    // the reference's explicit list (magpie.cpp:1133-1145) only when eos == bos + 1
    if (m.audio_eos != m.audio_bos + 1 || m.audio_bos < 0 || m.audio_bos + 8 > mp::VCB)
        return fail(dev, MP_ERR_UNSUPPORTED, "audio_eos_id must be audio_bos_id + 1 (forbidden-token layout)");
    m.max_dec_steps = (int)g.get_u32("magpie.max_dec_steps", 500);
    m.eps = (float)g.get_f32("magpie.eps", 1e-5);
    if (m.enc_layers < 1 || m.dec_layers < 1 || m.enc_layers > 64 || m.dec_layers > 64)
        return fail(dev, MP_ERR_FORMAT, "bad layer counts");

    struct Want { std::string name; int64_t n; const float **dst; };
    std::vector<Want> want;
    auto need = [&](const std::string &name, int64_t n, const float **dst) { want.push_back({name, n, dst}); };
    const int64_t D = 768;
    need("text_embedding.weight", (int64_t)m.text_vocab * D, &m.text_emb);
    need("encoder.position_embeddings.weight", -1, &m.enc_pos);
    m.enc.assign(m.enc_layers, mp::EncLayerW{});
    for (int l = 0; l < m.enc_layers; ++l) {
        const std::string p = "encoder.layers." + std::to_string(l) + ".";
        mp::EncLayerW &L = m.enc[l];
        need(p + "norm_self.weight", D, &L.norm_self);
        need(p + "self_attention.qkv_net.weight", 3 * D * D, &L.qkv);
        need(p + "self_attention.o_net.weight", D * D, &L.o);
        need(p + "norm_pos_ff.weight", D, &L.norm_ff);
        need(p + "pos_ff.proj.conv.weight", 3072 * D * 3, &L.ff1);
        need(p + "pos_ff.o_net.conv.weight", 3072 * D * 3, &L.ff2);
    }
    need("encoder.norm_out.weight", D, &m.enc_norm_out);
    need("decoder.position_embeddings.weight", -1, &m.dec_pos);
    m.dec.assign(m.dec_layers, mp::DecLayerW{});
    for (int l = 0; l < m.dec_layers; ++l) {
        const std::string p = "decoder.layers." + std::to_string(l) + ".";
        mp::DecLayerW &L = m.dec[l];
        need(p + "norm_self.weight", D, &L.norm_self);
        need(p + "self_attention.qkv_net.weight", 3 * D * D, &L.qkv);
        need(p + "self_attention.o_net.weight", D * D, &L.o);
        need(p + "norm_xattn_query.weight", D, &L.norm_xq);
        need(p + "cross_attention.q_net.weight", 128 * D, &L.xq);
        need(p + "cross_attention.kv_net.weight", 256 * D, &L.xkv);
        need(p + "cross_attention.o_net.weight", D * 128, &L.xo);
        need(p + "norm_xattn_memory.weight", D, &L.norm_xmem);
        need(p + "norm_pos_ff.weight", D, &L.norm_ff);
        need(p + "pos_ff.proj.conv.weight", 3072 * D, &L.ff1);
        need(p + "pos_ff.o_net.conv.weight", 3072 * D, &L.ff2);
    }
    need("decoder.norm_out.weight", D, &m.dec_norm_out);
    need("baked_context_embedding.weight", -1, &m.baked);
    need("local_transformer_in_projection.weight", 256 * D, &m.lt_in_w);
    need("local_transformer_in_projection.bias", 256, &m.lt_in_b);
    need("local_transformer.position_embeddings.weight", -1, &m.lt_pos);
    need("local_transformer.layers.0.norm_self.weight", 256, &m.lt_norm_self);
    need("local_transformer.layers.0.self_attention.qkv_net.weight", 768 * 256, &m.lt_qkv);
    need("local_transformer.layers.0.self_attention.o_net.weight", 256 * 256, &m.lt_o);
    need("local_transformer.layers.0.norm_pos_ff.weight", 256, &m.lt_norm_ff);
    need("local_transformer.layers.0.pos_ff.proj.conv.weight", 1024 * 256, &m.lt_ff1);
    need("local_transformer.layers.0.pos_ff.o_net.conv.weight", 1024 * 256, &m.lt_ff2);
    // per-codebook tensors become one contiguous [8][...] array each so a kernel
    // can index them by a codebook read from device memory
    std::vector<std::string> grouped[3];
    for (int c = 0; c < 8; ++c) {
        grouped[0].push_back("audio_embeddings." + std::to_string(c) + ".weight");
        grouped[1].push_back("local_transformer_out_projections." + std::to_string(c) + ".weight");
        grouped[2].push_back("local_transformer_out_projections." + std::to_string(c) + ".bias");
    }
    const int64_t gsize[3] = {2024 * D, 2024 * 256, 2024};
    const float **gdst[3] = {&m.audio_emb, &m.lt_out_w, &m.lt_out_b};

    // size the arena
    auto align_up = [](size_t v) { return (v + 255) & ~(size_t)255; };
    size_t total = 0;
    for (auto &w : want) {
        const mp::GgufTensor *t = g.find(w.name);
        if (!t) return fail(dev, MP_ERR_FORMAT, "missing tensor " + w.name);
        if (w.n >= 0 && t->nelements() != w.n) return fail(dev, MP_ERR_FORMAT, "unexpected shape for " + w.name);
        total += align_up((size_t)t->nelements() * 4);
    }
    for (int k = 0; k < 3; ++k)
        for (auto &nm : grouped[k]) {
            const mp::GgufTensor *t = g.find(nm);
            if (!t) return fail(dev, MP_ERR_FORMAT, "missing tensor " + nm);
            if (t->nelements() != gsize[k]) return fail(dev, MP_ERR_FORMAT, "unexpected shape for " + nm);
        }
    for (int k = 0; k < 3; ++k) total += align_up((size_t)gsize[k] * 8 * 4);
    {
        const mp::GgufTensor *dp = g.find("decoder.position_embeddings.weight");
        const mp::GgufTensor *bk = g.find("baked_context_embedding.weight");
        const mp::GgufTensor *ep = g.find("encoder.position_embeddings.weight");
        const mp::GgufTensor *lp = g.find("local_transformer.position_embeddings.weight");
        if (dp->ne[0] != D || bk->ne[0] != 110 * D || ep->ne[0] != D || lp->ne[0] != 256 || lp->ne[1] < 8)
            return fail(dev, MP_ERR_FORMAT, "unexpected embedding table shapes");
        m.dec_pos_rows = (int)dp->ne[1];
        m.n_spk = (int)std::min<int64_t>(m.n_spk, bk->ne[1]);
    }
    if (m.arena) { hipFree(m.arena); m.arena = nullptr; }
    HIPCHK(hipMalloc(&m.arena, total));
    m.arena_bytes = total;
    std::vector<float> host;
    size_t off = 0;
    std::vector<float> tmp;
    auto upload = [&](const mp::GgufTensor *t, float *dst) -> int {
        host.resize((size_t)t->nelements());
        if (!g.to_f32(*t, host.data())) return fail(dev, MP_ERR_FORMAT, "unsupported tensor type in " + t->name);
        if (t->n_dims == 3 && t->ne[0] == 3 && t->name.rfind("encoder.layers.", 0) == 0) {
            // causal k=3 conv weight [out][in][k] -> tap-major [out][k][in] (mp_prefill.hip loader)
            const int64_t K = 3, Cin = t->ne[1], Co = t->ne[2];
            tmp.resize(host.size());
            for (int64_t o = 0; o < Co; ++o)
                for (int64_t i = 0; i < Cin; ++i)
                    for (int64_t k = 0; k < K; ++k) tmp[(o * K + k) * Cin + i] = host[(o * Cin + i) * K + k];
            host.swap(tmp);
        }
        HIPCHK(hipMemcpy(dst, host.data(), host.size() * 4, hipMemcpyHostToDevice));
        return MP_OK;
    };
    for (auto &w : want) {
        const mp::GgufTensor *t = g.find(w.name);
        float *dst = (float *)((char *)m.arena + off);
        if (int rc = upload(t, dst)) return rc;
        *w.dst = dst;
        off += align_up((size_t)t->nelements() * 4);
    }
    for (int k = 0; k < 3; ++k) {
        float *base = (float *)((char *)m.arena + off);
        for (int c = 0; c < 8; ++c)
            if (int rc = upload(g.find(grouped[k][c]), base + (size_t)c * gsize[k])) return rc;
        *gdst[k] = base;
        off += align_up((size_t)gsize[k] * 8 * 4);
    }
    // W_q^T per decoder layer (for the per-utterance K' = K W_q of the fused XA), one
    // allocation, layer l at l * 768 * 128 (the batched K' GEMM strides over it)
    if (!m.xq_t.empty() && m.xq_t[0]) hipFree(m.xq_t[0]);
    m.xq_t.assign(m.dec_layers, nullptr);
    {
        std::vector<float> wq((size_t)128 * 768), wt((size_t)768 * 128);
        float *all = nullptr;
        HIPCHK(hipMalloc(&all, wt.size() * 4 * m.dec_layers));
        for (int l = 0; l < m.dec_layers; ++l) {
            HIPCHK(hipMemcpy(wq.data(), m.dec[l].xq, wq.size() * 4, hipMemcpyDeviceToHost));
            for (int j = 0; j < 128; ++j)
                for (int n = 0; n < 768; ++n) wt[(size_t)n * 128 + j] = wq[(size_t)j * 768 + n];
            m.xq_t[l] = all + (size_t)l * wt.size();
            HIPCHK(hipMemcpy(m.xq_t[l], wt.data(), wt.size() * 4, hipMemcpyHostToDevice));
        }
    }
    dev->loaded = true;
    return MP_OK;
}

// f32 -> bf16 bits, round to nearest even (ggml_compute_fp32_to_bf16; finite weights)
static unsigned short bf16_bits(float x) {
    unsigned u;
    memcpy(&u, &x, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (unsigned short)((u >> 16) | 64);
    return (unsigned short)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

// f32 mode's LT (lt_ffn2_kernel) needs o_net applied to v rows ahead of time:
// VO[c][v] = W_o V[c][v] for every table row, and [W_k ; W_o W_v] for position 0.
bool f32_lt_mode(const mp::Model &m) { return m.weight_mode == MP_WEIGHTS_AS_STORED; }
// MAGPIE_LT_ALL=1: the whole f32 batch-1 greedy LT of a frame in one launch (lt_all_kernel)
// instead of the front + 7 x {lt_ffn2, lt_e} + lt_e launches (the same bits). Off by default:
// its three granule edges per codebook (FFN-down partials -> 4-output merges -> y2 -> head
// keys -> pick) cost ~9 us per codebook against 2 launches' ~9.2: 73.5 vs 76.7 us per frame
// in the per-op timing, 2,967 vs 3,070 frames/s graph-replayed (gpurun_out/r06t_ops_f32_b1*)
bool lt_all_mode() {
    const char *e = getenv("MAGPIE_LT_ALL");
    return e && atoi(e) != 0;
}
// the LT attention through the load-time q|k|vo tables in f32: the f32 mode, and the bf16
// mode (whose LT FFN and heads are bf16: lt_slot_kernel + the bf16 head)
bool lt_table_attn(const mp::Model &m) { return m.weight_mode == MP_WEIGHTS_AS_STORED || m.weight_mode == MP_WEIGHTS_BF16; }

int build_vo_tables(mp_dev *dev) {
    mp::Model &m = dev->m;
    if (m.lt_votab) { hipFree(m.lt_votab); m.lt_votab = nullptr; }
    if (m.lt_kvo) { hipFree(m.lt_kvo); m.lt_kvo = nullptr; }
    const size_t R = (size_t)7 * 2024;
    HIPCHK(hipMalloc(&m.lt_votab, R * 256 * 4));
    mp::GemmP gp{};
    gp.A = m.lt_qkvtab + 512; gp.lda = 768; gp.W = m.lt_o; gp.C = m.lt_votab; gp.ldc = 256;
    gp.M = (int)R; gp.N = 256; gp.K = 256; gp.rows_per_utt = (int)R;
    HIPCHK(mp::pre_gemm(gp, mp::GE_STORE, dev->stream));
    std::vector<float> qkv((size_t)768 * 256), o((size_t)256 * 256), kvo((size_t)512 * 256);
    HIPCHK(hipMemcpy(qkv.data(), m.lt_qkv, qkv.size() * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(o.data(), m.lt_o, o.size() * 4, hipMemcpyDeviceToHost));
    memcpy(kvo.data(), qkv.data() + (size_t)256 * 256, (size_t)256 * 256 * 4);  // W_k rows
    for (int n = 0; n < 256; ++n)
        for (int k = 0; k < 256; ++k) {
            double acc = 0.0;
            for (int j = 0; j < 256; ++j) acc += (double)o[(size_t)n * 256 + j] * qkv[(size_t)(512 + j) * 256 + k];
            kvo[(size_t)(256 + n) * 256 + k] = (float)acc;
        }
    HIPCHK(hipMalloc(&m.lt_kvo, kvo.size() * 4));
    HIPCHK(hipMemcpy(m.lt_kvo, kvo.data(), kvo.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(hipStreamSynchronize(dev->stream));
    return MP_OK;
}

// P[c][v] = in_proj(audio_emb[c][v]) + b: the LT's per-codebook re-embedding
// (magpie.cpp:1274-1313) depends only on (c, v) -> one GEMM at load time (with
// ggml's Q8_0 arithmetic when in_proj is a Q8_0 tensor in Q8 mode).
int build_ptab(mp_dev *dev, int weight_mode) {
    mp::Model &m = dev->m;
    if (m.lt_ptab) { hipFree(m.lt_ptab); m.lt_ptab = nullptr; }
    HIPCHK(hipMalloc(&m.lt_ptab, (size_t)8 * 2024 * 256 * 4));
    mp::GemmP gp{};
    gp.A = m.audio_emb; gp.lda = 768; gp.W = m.lt_in_w; gp.Wq = m.lt_in8.q; gp.Wd = m.lt_in8.d; gp.bias = m.lt_in_b;
    gp.C = m.lt_ptab; gp.ldc = 256; gp.M = 8 * 2024; gp.N = 256; gp.K = 768; gp.rows_per_utt = 8 * 2024;
    gp.xround = weight_mode == MP_WEIGHTS_F16 ? 2 : 0;  // F16 in_proj: the embedding row rounded to f16
    HIPCHK(mp::pre_gemm(gp, mp::GE_STORE, dev->stream));
    // LT q|k|v of position c+1 for every code v of codebook c < 7: the rows PRO_LTARG_ATTN
    // gathers instead of running the q|k|v GEMV per codebook. The projection uses the
    // weights the decode-time GEMV would (f32, Q8_0 with activations quantised per
    // block, or bf16 / f16 weights and activations, f32 accumulation).
    if (m.lt_qkvtab) { hipFree(m.lt_qkvtab); m.lt_qkvtab = nullptr; }
    const size_t R = (size_t)7 * 2024;
    HIPCHK(hipMalloc(&m.lt_qkvtab, R * 768 * 4));
    float *rows = nullptr, *wq = nullptr;
    HIPCHK(hipMalloc(&rows, R * 256 * 4));
    // the bf16 mode's LT attention is f32 (lt_table_attn); F16: the file's weights are already f16 values
    const bool b16 = false;
    HIPCHK(mp::pre_lt_tab_rows(m.lt_ptab, m.lt_pos, m.lt_norm_self, m.eps, rows,
                               weight_mode == MP_WEIGHTS_F16 ? 2 : 0, dev->stream));
    if (b16) {
        HIPCHK(hipMalloc(&wq, (size_t)768 * 256 * 4));
        HIPCHK(mp::pre_round_bf16(m.lt_qkv, wq, (size_t)768 * 256, dev->stream));
    }
    gp = mp::GemmP{};
    gp.A = rows; gp.lda = 256; gp.W = b16 ? wq : m.lt_qkv; gp.Wq = m.lt_qkv8.q; gp.Wd = m.lt_qkv8.d;
    gp.C = m.lt_qkvtab; gp.ldc = 768; gp.M = (int)R; gp.N = 768; gp.K = 256; gp.rows_per_utt = (int)R;
    const hipError_t ge = mp::pre_gemm(gp, mp::GE_STORE, dev->stream);
    const hipError_t se = hipStreamSynchronize(dev->stream);
    hipFree(rows);
    if (wq) hipFree(wq);
    HIPCHK(ge);
    HIPCHK(se);
    if (!m.lt_ff2s) {
        constexpr int U = 1024 / mp::LT_FFN_P;
        std::vector<float> w2((size_t)256 * 1024), w2s(w2.size());
        HIPCHK(hipMemcpy(w2.data(), m.lt_ff2, w2.size() * 4, hipMemcpyDeviceToHost));
        for (int p = 0; p < mp::LT_FFN_P; ++p)
            for (int n = 0; n < 256; ++n)
                memcpy(&w2s[((size_t)p * 256 + n) * U], &w2[(size_t)n * 1024 + p * U], U * 4);
        HIPCHK(hipMalloc(&m.lt_ff2s, w2s.size() * 4));
        HIPCHK(hipMemcpy(m.lt_ff2s, w2s.data(), w2s.size() * 4, hipMemcpyHostToDevice));
    }
    if (weight_mode == MP_WEIGHTS_BF16 && !m.lt_ff1h) {
        std::vector<float> w1((size_t)1024 * 256), w2((size_t)256 * 1024);
        HIPCHK(hipMemcpy(w1.data(), m.lt_ff1, w1.size() * 4, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(w2.data(), m.lt_ff2, w2.size() * 4, hipMemcpyDeviceToHost));
        constexpr int U = 1024 / mp::LTS_P;
        std::vector<unsigned short> h1(w1.size()), h2(w2.size());
        for (size_t i = 0; i < w1.size(); ++i) h1[i] = bf16_bits(w1[i]);
        for (int q = 0; q < mp::LTS_P; ++q)
            for (int n = 0; n < 256; ++n)
                for (int u = 0; u < U; ++u) h2[((size_t)q * 256 + n) * U + u] = bf16_bits(w2[(size_t)n * 1024 + q * U + u]);
        HIPCHK(hipMalloc(&m.lt_ff1h, h1.size() * 2));
        HIPCHK(hipMemcpy(m.lt_ff1h, h1.data(), h1.size() * 2, hipMemcpyHostToDevice));
        HIPCHK(hipMalloc(&m.lt_ff2h, h2.size() * 2));
        HIPCHK(hipMemcpy(m.lt_ff2h, h2.data(), h2.size() * 2, hipMemcpyHostToDevice));
    }
    if (weight_mode == MP_WEIGHTS_Q8 && !m.lt_ff2q) {
        constexpr int U = 1024 / mp::LTQ_P;
        std::vector<float> w2((size_t)256 * 1024), w2q(w2.size());
        HIPCHK(hipMemcpy(w2.data(), m.lt_ff2, w2.size() * 4, hipMemcpyDeviceToHost));
        for (int q = 0; q < mp::LTQ_P; ++q)
            for (int n = 0; n < 256; ++n)
                memcpy(&w2q[((size_t)q * 256 + n) * U], &w2[(size_t)n * 1024 + q * U], U * 4);
        HIPCHK(hipMalloc(&m.lt_ff2q, w2q.size() * 4));
        HIPCHK(hipMemcpy(m.lt_ff2q, w2q.data(), w2q.size() * 4, hipMemcpyHostToDevice));
    }
    return lt_table_attn(m) ? build_vo_tables(dev) : MP_OK;
}

// Weight mode MP_WEIGHTS_Q8: upload every block-quantised tensor the decode path
// uses (scripts/convert_magpie_to_gguf.py:155-176 decides which: attention,
// cross-attention and LT projections), repacked to int8 [N][K] + fp16 scales
// [N][K/32] (34 B per 32 weights). Q8_0 blocks are copied; Q4_0 blocks
// (convert_magpie_to_gguf.py:107-138: q in 0..15, byte j = q_j | q_{j+16} << 4) become
// the int8 values q - 8 with the same scale, so the Q8_0 kernels compute exactly
// ggml's vec_dot_q4_0_q8_0: the integer dot of (q - 8) with the Q8_0-quantised
// activation times d_w * d_a. F32 tensors keep the f32 path.
int load_q8(mp_dev *dev, const char *path) {
    mp::Gguf g;
    std::string err;
    if (!g.open(path, err)) return fail(dev, MP_ERR_IO, err);
    mp::Model &m = dev->m;
    struct Item { const mp::GgufTensor *t; mp::QW *dst; int group; };
    // a Q4_0 tensor's decode fragments stream its nibbles (MAGPIE_Q4_AS_Q8=1: as int8 q - 8,
    // the same integers at 34 B per 32 weights; both compute the same bits)
    const char *q4e = getenv("MAGPIE_Q4_AS_Q8");
    const bool q4_nib = !(q4e && atoi(q4e) != 0);
    std::vector<Item> items;
    auto want = [&](const std::string &name, mp::QW *dst) {
        const mp::GgufTensor *t = g.find(name);
        if (t && (t->type == 8 || t->type == 2) && t->ne[0] % 32 == 0) items.push_back({t, dst, -1});
    };
    for (int l = 0; l < m.enc_layers; ++l) {
        const std::string p = "encoder.layers." + std::to_string(l) + ".self_attention.";
        want(p + "qkv_net.weight", &m.enc[l].qkv8);
        want(p + "o_net.weight", &m.enc[l].o8);
    }
    for (int l = 0; l < m.dec_layers; ++l) {
        const std::string p = "decoder.layers." + std::to_string(l) + ".";
        want(p + "self_attention.qkv_net.weight", &m.dec[l].qkv8);
        want(p + "self_attention.o_net.weight", &m.dec[l].o8);
        want(p + "cross_attention.q_net.weight", &m.dec[l].xq8);
        want(p + "cross_attention.kv_net.weight", &m.dec[l].xkv8);
        want(p + "cross_attention.o_net.weight", &m.dec[l].xo8);
    }
    want("local_transformer_in_projection.weight", &m.lt_in8);
    want("local_transformer.layers.0.self_attention.qkv_net.weight", &m.lt_qkv8);
    want("local_transformer.layers.0.self_attention.o_net.weight", &m.lt_o8);
    int nout = 0;
    for (int c = 0; c < 8; ++c) {
        const mp::GgufTensor *t = g.find("local_transformer_out_projections." + std::to_string(c) + ".weight");
        if (t && (t->type == 8 || t->type == 2)) { items.push_back({t, &m.lt_out8, c}); ++nout; }
    }
    if (nout != 0 && nout != 8) return fail(dev, MP_ERR_UNSUPPORTED, "mixed quantised/F32 LT output projections");
    if (items.empty()) return fail(dev, MP_ERR_UNSUPPORTED, "Q8 weight mode needs a GGUF with Q8_0 or Q4_0 tensors");
    // the reassociated XA (K' = K W_q, V' = W_o V) is an f32 identity: with Q8_0
    // q_net / o_net the activations must be quantised where ggml quantises them
    for (int l = 0; l < m.dec_layers; ++l)
        if ((bool)m.dec[l].xq8 != (bool)m.dec[l].xo8)
            return fail(dev, MP_ERR_UNSUPPORTED, "cross-attention q_net / o_net must both be Q8_0 or both F32");
    auto align_up = [](size_t v) { return (v + 255) & ~(size_t)255; };
    size_t total = 0;
    for (auto &it : items) {
        const size_t n = (size_t)it.t->nelements();
        total += align_up(n) + align_up(n / 32 * 2);
        if (it.dst == &m.lt_o8) total += align_up(n);  // the transposed copy
    }
    if (m.q8_arena) { hipFree(m.q8_arena); m.q8_arena = nullptr; }
    HIPCHK(hipMalloc(&m.q8_arena, total));
    m.q8_bytes = total;
    char *cur = (char *)m.q8_arena;
    std::vector<signed char> hq;
    std::vector<unsigned short> hd;
    signed char *out_q = nullptr;
    unsigned short *out_d = nullptr;
    const size_t out_n = (size_t)2024 * 256;
    for (auto &it : items) {
        const size_t n = (size_t)it.t->nelements();
        const uint8_t *src = g.data(*it.t);
        hq.resize(n);
        hd.resize(n / 32);
        for (size_t b = 0; b < n / 32; ++b) {
            if (it.t->type == 8) {
                memcpy(&hd[b], src + b * 34, 2);
                memcpy(&hq[b * 32], src + b * 34 + 2, 32);
            } else {  // Q4_0
                const uint8_t *blk = src + b * 18;
                memcpy(&hd[b], blk, 2);
                for (int j = 0; j < 16; ++j) {
                    hq[b * 32 + j] = (signed char)((blk[2 + j] & 0x0F) - 8);
                    hq[b * 32 + j + 16] = (signed char)((blk[2 + j] >> 4) - 8);
                }
            }
        }
        signed char *dq;
        unsigned short *dd;
        if (it.group < 0) {
            dq = (signed char *)cur; cur += align_up(n);
            dd = (unsigned short *)cur; cur += align_up(n / 32 * 2);
            it.dst->q = dq; it.dst->d = dd;
            it.dst->nib = q4_nib && it.t->type == 2;
        } else {  // the 8 LT heads as one [8][2024][256] array (indexed by a device codebook)
            if (n != out_n) return fail(dev, MP_ERR_FORMAT, "unexpected LT output projection shape");
            if (!out_q) {
                out_q = (signed char *)cur; cur += align_up(8 * n);
                out_d = (unsigned short *)cur; cur += align_up(8 * (n / 32) * 2);
            }
            dq = out_q + (size_t)it.group * n;
            dd = out_d + (size_t)it.group * (n / 32);
            it.dst->q = out_q; it.dst->d = out_d;
            if (it.group == 0) it.dst->nib = q4_nib && it.t->type == 2;
            else if (it.dst->nib != (int)(q4_nib && it.t->type == 2))
                return fail(dev, MP_ERR_UNSUPPORTED, "mixed Q4_0 / Q8_0 LT output projections");
        }
        HIPCHK(hipMemcpy(dq, hq.data(), n, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(dd, hd.data(), n / 32 * 2, hipMemcpyHostToDevice));
        if (it.dst == &m.lt_o8) {  // chunk i of row r at [i][r]: thread r's 16 loads coalesce across the wave
            if (n != (size_t)256 * 256) return fail(dev, MP_ERR_FORMAT, "unexpected LT o_net shape");
            std::vector<signed char> ht(n);
            for (int r = 0; r < 256; ++r)
                for (int i = 0; i < 16; ++i) memcpy(&ht[((size_t)i * 256 + r) * 16], &hq[(size_t)r * 256 + i * 16], 16);
            signed char *dt = (signed char *)cur;
            cur += align_up(n);
            HIPCHK(hipMemcpy(dt, ht.data(), n, hipMemcpyHostToDevice));
            m.lt_o8t = dt;
        }
    }
    // the decode projections once more in int8 MFMA fragment order
    struct Dec { mp::QW *w; int N, K, heads; };
    std::vector<Dec> dec;
    bool all = true;
    auto add = [&](mp::QW &w, int N, int K, int heads) {
        if (w) dec.push_back({&w, N, K, heads});
        else all = false;
    };
    for (int l = 0; l < m.dec_layers; ++l) {
        add(m.dec[l].qkv8, 2304, 768, 1);
        add(m.dec[l].o8, 768, 768, 1);
        add(m.dec[l].xq8, 128, 768, 1);
        if (!m.dec[l].xo8) all = false;
    }
    add(m.lt_in8, 256, 768, 1);
    add(m.lt_qkv8, 768, 256, 1);
    add(m.lt_o8, 256, 256, 1);
    add(m.lt_out8, 2024, 256, 8);
    size_t ptotal = 0;
    auto frag_bytes = [&](const Dec &d) {
        return align_up(d.w->nib ? mp::q4p_qbytes(d.N, d.K) : mp::q8p_qbytes(d.N, d.K));
    };
    for (auto &d : dec) ptotal += d.heads * (frag_bytes(d) + align_up(mp::q8p_dbytes(d.N, d.K)));
    if (m.q8p_arena) { hipFree(m.q8p_arena); m.q8p_arena = nullptr; }
    if (ptotal) HIPCHK(hipMalloc(&m.q8p_arena, ptotal));
    char *pc = (char *)m.q8p_arena;
    for (auto &d : dec) {
        const size_t qb = frag_bytes(d), db = align_up(mp::q8p_dbytes(d.N, d.K));
        signed char *oq = (signed char *)pc;
        pc += d.heads * qb;
        unsigned short *od = (unsigned short *)pc;
        pc += d.heads * db;
        for (int h = 0; h < d.heads; ++h) {
            const signed char *hq = d.w->q + (size_t)h * d.N * d.K;
            // the scales (and, for Q8_0, the int8 fragments) in fragment order
            HIPCHK(mp::pack_q8(hq, d.w->d + (size_t)h * d.N * (d.K / 32), d.N, d.K,
                               d.w->nib ? nullptr : (unsigned char *)oq + h * qb,
                               (unsigned short *)((char *)od + h * db), nullptr));
            if (d.w->nib) HIPCHK(mp::pack_q4(hq, d.N, d.K, (unsigned char *)oq + h * qb, nullptr));
        }
        d.w->pq = oq;
        d.w->pd = od;
        d.w->head_q = qb;
    }
    HIPCHK(hipDeviceSynchronize());
    m.q8_all = all;
    return MP_OK;
}
// stride between the 8 packed LT heads' scales, as laid out above (fragments: QW::head_q)
static size_t q8p_head_d() { return (mp::q8p_dbytes(2024, 256) + 255) & ~(size_t)255; }

// ------------------------------------------------------------------ batch state
// the cross-attention form of a batch (mp_hip_set_xa_mode): direct where it reads fewer
// bytes (Tmax > MP_XA_DIRECT_T); F16 keeps the reassociated form, Q8_0 has its own
bool want_xa_direct(const mp_dev *dev, int Tmax) {
    const int wm = dev->m.weight_mode;
    if (wm != MP_WEIGHTS_AS_STORED && wm != MP_WEIGHTS_BF16) return false;
    return dev->xa_mode == MP_XA_DIRECT || (dev->xa_mode == MP_XA_AUTO && Tmax > MP_XA_DIRECT_T);
}

static size_t enc_gpart_elems(size_t Me);
int alloc_batch(mp_dev *dev, int B, int Tmax, int max_steps, bool trace) {
    free_batch(dev);
    const int NB = B <= 1 ? 1 : B <= 2 ? 2 : B <= 4 ? 4 : B <= 8 ? 8 : 16;
    const int L = dev->m.dec_layers;
    dev->B = B;
    dev->NB = NB;
    dev->Tmax = Tmax;
    dev->max_steps = max_steps;
    dev->max_seq = mp::CTX + max_steps + 16;  // magpie.cpp:4077
    dev->nch = (dev->max_seq + mp::SA_CHUNK - 1) / mp::SA_CHUNK;
    dev->max_seq = dev->nch * mp::SA_CHUNK;  // whole chunks: attention loads never leave the cache slab
    const size_t D = 768;
    int rc = MP_OK;
#define A(ptr, n) if ((rc = dalloc(dev, &dev->ptr, (size_t)(n))) != MP_OK) return rc
    // this batch's KV width and XA form first: the allocations below depend on them
    // (a batch must never inherit the previous batch's form)
    dev->kv16 = dev->kv_mode == MP_KV_BF16;
    dev->xa_direct = want_xa_direct(dev, Tmax);
    A(x, NB * D); A(x2, NB * D); A(q, NB * D);
    if (!dev->xa_direct) { A(kp, (size_t)NB * L * Tmax * D); A(vp, (size_t)NB * L * Tmax * D); }
    else dev->kp = dev->vp = nullptr;
    A(sa_out, NB * 768);
    A(h, NB * 3072); A(hidden, NB * D); A(xqb, NB * 128); A(h_b16, NB * 3072);
    A(sa_part, (size_t)NB * mp::NH * mp::SA_SPLITS * mp::SA_PART); A(xa_part, (size_t)NB * mp::XA_SPLITS * mp::XA_PART);
    A(sagh, (size_t)NB * mp::NH * mp::SA_SPLITS * mp::SA_PART); A(xagh, (size_t)NB * mp::XA_SPLITS * mp::XA_PART);
    A(kgh, (size_t)2 * (768 / 16) * mp::KGH_MAX_KS * 256);  // [O-projection | FFN down]
    A(xh, (size_t)NB * D); A(qh, (size_t)NB * 3 * D); A(xqh, (size_t)NB * 128);
    const size_t kvn = (size_t)NB * L * dev->max_seq * D;  // elements; bf16 mode: 2 per float slot
    A(kc, dev->kv16 ? kvn / 2 : kvn); A(vc, dev->kv16 ? kvn / 2 : kvn);
    A(xak, (size_t)NB * L * Tmax * 128); A(xav, (size_t)NB * L * Tmax * 128);
    A(lt_s, NB * 9 * 256); A(ltX, NB * 256); A(ltY, NB * 256); A(lty2, NB * 256); A(ltq, NB * 256);
    A(ltk, NB * 8 * 256); A(ltv, NB * 8 * 256); A(ltf, NB * 1024); A(logits, NB * 2024);
    A(ltp, (size_t)NB * std::max({mp::LT_FFN_P, mp::LTS_P, mp::LTQ_P}) * 256); A(ltgh, (size_t)NB * std::max(mp::LTS_P, mp::LTQ_P) * 256); A(ltfg, mp::LTFG_TOTAL); A(ltyg, (size_t)NB * 256);
    A(ltcand, 256);  // zeroed: slots past the head's workgroups + EOS slot stay 0
    if (trace) A(trace, (size_t)NB * (max_steps + 1) * D);
    A(T, NB); A(spk, NB); A(pos, NB); A(step, NB); A(done, NB); A(nframes, NB); A(ndone, 4);  // ndone: [done count, iteration, hand-off timeout, -]
    A(argeos, NB); A(amax, NB * 8); A(smpcfg, 1);
    A(codes_cur, NB * 8); A(codes_prev, NB * 8); A(codes_out, (size_t)NB * max_steps * 8); A(tok, (size_t)NB * Tmax);
    const size_t rows = (size_t)NB * std::max(Tmax, mp::CTX);
    A(pX, rows * D); A(pH, rows * D); A(pQKV, rows * 3 * D); A(pATT, rows * D); A(pF, rows * 3072);
    A(pXQ, rows * 128); A(pXAO, rows * 128); A(enc_out, (size_t)NB * Tmax * D);
    {   // largest S x M x N of the preamble GEMMs (encoder FFN up/down, prefill FFN)
        const size_t Me = (size_t)NB * Tmax, Mc = (size_t)NB * mp::CTX;
        size_t cap = enc_gpart_elems(Me);
        auto need = [&](size_t M, int N, int K) { cap = std::max(cap, (size_t)mp::gemm_splits_max(K) * M * N); };
        need(Mc, 2304, 768); need(Mc, 3072, 768); need(Mc, 768, 3072); need(Mc, 768, 768);
        need(Me, 256 * L, 768);  // the XA K/V GEMMs batched over layers
        A(gpart, cap);
    }
    if (const char *qd = getenv("MAGPIE_Q8DUMP"); qd && atoi(qd) != 0 && dev->m.weight_mode == MP_WEIGHTS_Q8) {
        // the largest launch: K = 768, N = 2304 (QKV): rows, blocks, d, dots
        const size_t slot = ((size_t)NB * 768 * 5 + (size_t)NB * 24 * 4 + (size_t)2304 * 24 * NB * 4 + 255) / 256 * 256;
        dev->q8dump_cap = 4 * L + 16;
        dev->q8dump_slot = slot;
        if ((rc = dalloc(dev, &dev->q8dump, slot * dev->q8dump_cap)) != MP_OK) return rc;
    }
#undef A
    return MP_OK;
}

mp::GemvP gemv_base(mp_dev *dev) {
    mp::GemvP g;
    memset(&g, 0, sizeof g);
    g.eps = dev->m.eps;
    g.nlayers = dev->m.dec_layers;
    g.max_seq = dev->max_seq;
    g.pos = dev->pos;
    g.step = dev->step;
    g.ndone = dev->ndone;
    g.smp = mp::Sampling{dev->params.temperature >= 0.01f, dev->smpcfg, dev->argeos};
    g.nslots = dev->NB;
    g.ignore_eos = dev->params.ignore_eos;
    g.audio_bos = dev->m.audio_bos;
    g.audio_eos = dev->m.audio_eos;
    return g;
}

int enqueue_lt(mp_dev *dev, const mp::LtIo &io, int NB, hipStream_t s, std::vector<mp::OpRec> *ops);
bool q8_unfused();
bool lt_cand_mode();
bool sa16_fused(int weight_mode);
int split_merge8();

// Enqueue one decode iteration: decoder step at pos (embedding codes_prev), LT
// over 8 codebooks, finalize. When `record` is set, the op list is rebuilt for
// measurement (mp_hip_time_op).
int enqueue_iteration_body(mp_dev *dev, hipStream_t s, bool record);
int enqueue_iteration(mp_dev *dev, hipStream_t s, bool record) {
    dev->q8dump_n = 0;
    dev->q8dump_index.clear();
    dev->q8dump_live = true;
    const int rc = enqueue_iteration_body(dev, s, record);
    dev->q8dump_live = false;
    return rc;
}
int enqueue_iteration_body(mp_dev *dev, hipStream_t s, bool record) {
    const mp::Model &m = dev->m;
    const int NB = dev->NB, L = m.dec_layers;
    const bool b16 = mp::h16_mode(m.weight_mode);  // 16-bit MFMA family (bf16 or F16 weights)
    const mp::OpTable &tb = mp::table_for(NB, m.weight_mode);
    const mp::OpTableQ8 &tq = mp::table_q8(NB);
    // algorithmic bytes: weights at their stored width (Q8_0: 34 B per 32), activations f32
    const double F = b16 ? 2.0 : 4.0, A = 4.0, act = (double)NB;
    // a quantised tensor's decode bytes per weight: Q8_0 34/32, Q4_0 nibble fragments 18/32
    auto Fq = [](const mp::QW &w) { return w.nib ? 18.0 / 32.0 : 34.0 / 32.0; };
    if (record) dev->ops.clear();
    auto run = [&](const char *name, mp::GemvFn fn, const mp::GemvP &g0, double bytes) -> int {
        mp::GemvP g = g0;
        q8dump_assign(dev, name, g);
        if (record) {
            mp::OpRec r{};
            r.name = name; r.kind = mp::K_GEMV; r.fn = fn; r.g = g; r.B = NB; r.bytes = bytes;
            dev->ops.push_back(r);
        }
        if (!fn) return fail(dev, MP_ERR_UNSUPPORTED, std::string(name) + ": no kernel for this batch size / weight mode");
        HIPCHK(fn(g, s));
        return MP_OK;
    };
    int rc;
    for (int l = 0; l < L; ++l) {
        const mp::DecLayerW &W = m.dec[l];
        mp::GemvP g = gemv_base(dev);
        g.layer = l;
        // LN + QKV (+ frame embedding on layer 0) + KV append   (3415-3442)
        g.W = W.qkv; g.Wb = b16 ? m.pk_qkv[l] : nullptr; g.N = 2304; g.lnw = W.norm_self; g.src = dev->x; g.src_ld = 768; g.out = dev->q;
        g.Wq = W.qkv8.pq; g.Wd = W.qkv8.pd; g.q4 = W.qkv8.nib;
        g.kc = dev->kc; g.vc = dev->vc; g.kv16 = dev->kv16;
        // the frame embedding (2746-2787) is in x already: written by the previous
        // iteration's finalize (lt_finalize_kernel), for the first frame by reset_decode_state
        // self-attention over the cache, split over keys (3457-3476); the f32 family runs
        // it in the QKV launch on a hand-off of q|k|v (EPI_QKV_SA), the others separately
        mp::AttnP a{dev->q, dev->kc, dev->vc, l, L, dev->max_seq, dev->pos, dev->kv16, dev->sa_part};
        // bf16 mode at 8 and 16 slots: the SA and XA split states are merged once, by the split
        // workgroups themselves through granules (sa_merge_split, xa_merge_split: each merges
        // 1 / SPLITS of its head's / slot's outputs), not by every O-projection / FFN-up
        // workgroup's prologue (196 / 245 KiB each at 16 slots); the same arithmetic, so
        // batches still reproduce single runs (at 8 slots the SA merge runs in the QKV launch)
        const bool mb16 = m.weight_mode == MP_WEIGHTS_BF16 && !dev->xa_direct;
        const bool merge_sa = mb16 && (NB >= 16 || (NB == 8 && (split_merge8() & 1)));
        const bool merge_xa = mb16 && (NB >= 16 || (NB == 8 && (split_merge8() & 2)));
        if (merge_sa) { a.merged = dev->sa_out; a.gh = dev->sagh; a.iter = dev->ndone + 1; a.hx_err = dev->ndone + 2; }
        // (at 16 slots too unless MAGPIE_SA16=0, sa16_fused; both forms compute the same bits)
        // (Q8_0: the same hand-off in the int8 MFMA launch, mp_decode_q8.hip; MAGPIE_Q8_UNFUSED=1
        // keeps the separate launches, which compute the same bits)
        const bool q8_fuse = !q8_unfused();
        const bool sa_in_qkv = (W.qkv8 ? q8_fuse && tq.qkv_sa : tb.qkv_sa != nullptr) && (NB < 16 || sa16_fused(m.weight_mode));
        {
            mp::GemvFn fn = W.qkv8 ? tq.qkv : tb.qkv;
            if (sa_in_qkv) {
                fn = W.qkv8 ? tq.qkv_sa : tb.qkv_sa;
                g.sa = a; g.qh = dev->qh; g.iter = dev->ndone + 1; g.hx_err = dev->ndone + 2;
            }
            if ((rc = run(sa_in_qkv ? "qkv_sa" : "qkv", fn, g,
                          (W.qkv8 ? Fq(W.qkv8) : F) * (2304.0 * 768) + A * act * ((768 + 2304)))) != MP_OK) return rc;
            if (sa_in_qkv && record) dev->ops.back().add_sa = true;
        }
        if (!sa_in_qkv) {
        if (record) {
            mp::OpRec r{};
            r.name = "sa_attn"; r.kind = mp::K_ATTN; r.a = a; r.B = NB;
            r.bytes = -1;  // depends on the live cache length; computed at timing time
            dev->ops.push_back(r);
        }
        HIPCHK(mp::op_sa_attn(a, NB, s));
        }
        // O-proj + residual (3479, 3509)
        g = gemv_base(dev); g.layer = l;
        g.W = W.o; g.Wb = b16 ? m.pk_o[l] : nullptr; g.N = 768; g.resid = dev->x; g.part = dev->sa_part;
        g.Wq = W.o8.pq; g.Wd = W.o8.pd; g.q4 = W.o8.nib;
        // split-K partial tiles (MP_OPROJ_KS > 1 builds only): the plain O-projection then
        // carries a hand-off; with one slice it has none and stays timeable standalone
        if (b16 && mp::b16_oproj_ks() > 1) { g.kgh = dev->kgh; g.iter = dev->ndone + 1; g.hx_err = dev->ndone + 2; }
        mp::XaP xp{dev->x, dev->xa_part, W.norm_xq, m.eps, dev->kp, dev->vp, dev->T, dev->Tmax, l, L};
        xp.q_f16 = m.weight_mode == MP_WEIGHTS_F16;
        const double xa_bytes = A * act * (768.0 + 2.0 * 768 * dev->Tmax + mp::XA_SPLITS * mp::XA_PART);
        // direct XA (Q8_0 q_net / o_net, or long texts: mp_hip_set_xa_mode): x2 materialised
        const bool xa_dir = W.xq8 || dev->xa_direct;
        const bool xa_in_oproj = tb.oproj_xa && !W.o8 && !xa_dir;
        // Q8_0 file: the whole direct Q8_0 cross-attention rides in the Q8_0 O-projection's
        // launch (EPI_RESID_XQ8): q_net workgroups on a hand-off of x1, then attention +
        // o_net workgroups on a hand-off of q (up to XQ8_QIN_NB slots: the attention
        // workgroups compute q on the hand-off of x1 themselves); x2 materialised
        // (up to 8 slots: its 48 + 20 NB workgroups are then co-resident even at one per CU,
        // so no hand-off waits on a workgroup that has not been dispatched)
        const bool xq8_in_oproj = q8_fuse && W.o8 && W.xq8 && W.xo8 && tq.oproj_xq && NB <= 8;
        if (xq8_in_oproj) {
            mp::XaQ8P xq{};
            xq.x2 = dev->x2; xq.xak = dev->xak; xq.xav = dev->xav; xq.T = dev->T; xq.Tmax = dev->Tmax;
            xq.layer = l; xq.nlayers = L; xq.wo = W.xo8.q; xq.wod = W.xo8.d;
            xq.wq = W.xq8.q; xq.wqd = W.xq8.d; xq.lnw = W.norm_xq; xq.eps = m.eps; xq.qg = dev->xqh;
            xq.qin = NB <= mp::XQ8_QIN_NB;  // small batches: q in the attention workgroups (one hand-off)
            g.xq8 = xq; g.xh = dev->xh; g.iter = dev->ndone + 1; g.hx_err = dev->ndone + 2;
            if ((rc = run("oproj_xa_q8", tq.oproj_xq, g,
                          Fq(W.o8) * (768.0 * 768) + A * act * (768 * 3) + (34.0 / 32.0) * (2.0 * 128 * 768) +
                              A * act * (768 + 2.0 * 128 * dev->Tmax))) != MP_OK)
                return rc;
        } else if (xa_in_oproj) {
            // f32: the fused XA rides in the O-projection's launch on a hand-off of x1
            mp::GemvFn fn = tb.oproj_xa;
            if (merge_sa) {  // the SA output merged by its split workgroups: plain rows
                g.part = nullptr; g.src = dev->sa_out; g.src_ld = 768;
                fn = NB == 16 ? mp::b16_oproj_xa_pm_16 : mp::b16_oproj_xa_pm_8;
            }
            if (merge_xa) { xp.x2 = dev->x2; xp.gh = dev->xagh; }  // x2 merged by the XA workgroups
            g.xa = xp; g.xh = dev->xh; g.iter = dev->ndone + 1; g.hx_err = dev->ndone + 2;
            if ((rc = run("oproj_xa", fn, g, F * (768.0 * 768) + A * act * (768 * 3) + xa_bytes)) != MP_OK)
                return rc;
        } else if ((rc = run("oproj", W.o8 ? tq.oproj : tb.oproj, g,
                             (W.o8 ? Fq(W.o8) : F) * (768.0 * 768) + A * act * (768 * 3))) != MP_OK) {
            return rc;
        }
        if (xa_dir && !xq8_in_oproj) {
            // cross-attention as ggml computes it (1713-1767): q = q_net LN(x) (GEMV), then
            // x2 = x + o_net attn(q, K, V) (xa_q8_kernel / xa_f32_kernel); Q8_0 q_net / o_net
            // quantise their activations, else f32 (the bf16 mode keeps XA f32)
            g = gemv_base(dev); g.layer = l;
            g.W = W.xq; g.Wq = W.xq8.pq; g.Wd = W.xq8.pd; g.q4 = W.xq8.nib; g.N = 128; g.lnw = W.norm_xq; g.src = dev->x; g.src_ld = 768;
            g.out = dev->xqb; g.out_ld = 128;
            const double Fx = W.xq8 ? Fq(W.xq8) : A;
            if ((rc = run("xq", W.xq8 ? tq.xq : tb.xq, g, Fx * (128.0 * 768) + A * act * (768 + 128))) != MP_OK)
                return rc;
            mp::XaQ8P xq{};
            xq.x = dev->x; xq.x2 = dev->x2; xq.q = dev->xqb; xq.xak = dev->xak; xq.xav = dev->xav; xq.T = dev->T;
            xq.Tmax = dev->Tmax; xq.layer = l; xq.nlayers = L;
            if (W.xq8) { xq.wo = W.xo8.q; xq.wod = W.xo8.d; }
            else xq.wof = W.xo;
            if (record) {
                mp::OpRec r{};
                r.name = W.xq8 ? "xa_q8" : "xa_dir"; r.kind = mp::K_XAQ8; r.xq = xq; r.B = NB;
                r.bytes = Fx * (768.0 * 128) + A * act * (128.0 + 768 * 2 + 2.0 * 128 * dev->Tmax);
                dev->ops.push_back(r);
            }
            HIPCHK(mp::op_xa_q8(xq, NB, s));
        } else if (!xa_in_oproj && !xq8_in_oproj) {
            // cross-attention, fused (1713-1767, 3513-3519): x2 = x + o_net(attn(q_net(LN(x))))
            if (record) {
                mp::OpRec r{};
                r.name = "xa"; r.kind = mp::K_XA; r.x = xp; r.B = NB;
                r.bytes = xa_bytes;
                dev->ops.push_back(r);
            }
            HIPCHK(mp::op_xa(xp, NB, s));
        }
        // LN + FFN up + GELU (1796-1799)
        g = gemv_base(dev); g.layer = l;
        g.W = W.ff1; g.Wb = b16 ? m.pk_ff1[l] : nullptr; g.N = 3072; g.lnw = W.norm_ff; g.out = dev->h; g.out_ld = 3072;
        if (xa_dir || merge_xa) {  // x2 materialised by the direct XA / the XA tail's merge
            g.src = dev->x2; g.src_ld = 768;
            if (b16) g.out_b16 = dev->h_b16;
            if ((rc = run("ff1", tb.ff1, g, F * (3072.0 * 768) + A * act * ((768 + 3072)))) != MP_OK) return rc;
        } else {      // x2 = x + merged XA split states, stored by block 0 for the FFN residual
            g.src = dev->x; g.src_ld = 768; g.part = dev->xa_part; g.xres = dev->x2;
            if (b16) g.out_b16 = dev->h_b16;  // GELU output stored bf16 / f16 (what FFN down rounds it to)
            if ((rc = run("ff1", tb.ff1x, g,
                          F * (3072.0 * 768) + A * act * (768 * 2 + 3072 + mp::XA_SPLITS * mp::XA_PART))) != MP_OK)
                return rc;
        }
        // FFN down + residual (1805, 3525): x = x2 + W2 h
        g = gemv_base(dev); g.layer = l;
        g.W = W.ff2; g.Wb = b16 ? m.pk_ff2[l] : nullptr; g.N = 768; g.src = dev->h; g.src_ld = 3072; g.out = dev->x; g.out_ld = 768; g.addsrc = dev->x2;
        if (b16) {
            g.src = nullptr; g.src_b16 = dev->h_b16;
            // split-K partial tiles (the FFN-down half of kgh: each op its own granules)
            g.kgh = dev->kgh + (size_t)(768 / 16) * mp::KGH_MAX_KS * 256; g.iter = dev->ndone + 1; g.hx_err = dev->ndone + 2;
        }
        if ((rc = run("ff2", tb.ff2, g, F * (768.0 * 3072) + A * act * ((3072 + 2 * 768)))) != MP_OK) return rc;
    }
    mp::LtIo io{};
    io.x = dev->x; io.hidden = dev->hidden; io.trace = dev->trace; io.trace_steps = dev->max_steps + 1;
    io.lt_s = dev->lt_s; io.ltX = dev->ltX; io.ltY = dev->ltY; io.lty2 = dev->lty2; io.ltq = dev->ltq;
    io.ltk = dev->ltk; io.ltv = dev->ltv; io.ltf = dev->ltf; io.logits = dev->logits; io.ltp = dev->ltp;
    io.ltgh = dev->ltgh; io.ltfg = dev->ltfg; io.ltyg = dev->ltyg; io.iter = dev->ndone + 1; io.hx_err = dev->ndone + 2;
    io.ltcand = lt_cand_mode() ? dev->ltcand : nullptr;
    io.codes_cur = dev->codes_cur; io.codes_prev = dev->codes_prev; io.codes_out = dev->codes_out; io.step = dev->step;
    io.pos = dev->pos; io.done = dev->done; io.nframes = dev->nframes; io.ndone = dev->ndone; io.argeos = dev->argeos;
    io.amax = dev->amax; io.cfg = dev->smpcfg;
    io.sampling = dev->params.temperature >= 0.01f; io.ignore_eos = dev->params.ignore_eos;
    io.emit_eos = dev->params.emit_eos_frame; io.max_steps = dev->max_steps; io.lt_only = false;
    return enqueue_lt(dev, io, NB, s, record ? &dev->ops : nullptr);
}

// The local transformer over one frame (magpie_local_transformer_sample_all,
// magpie.cpp:1113-1317) + the frame bookkeeping (4320-4358), for NB slots whose
// buffers `io` names. lt_only: in_proj of a given normalised hidden, codes only.
// MAGPIE_EAGER=1: launch the iteration's kernels directly instead of replaying
// the captured graph (identical kernels and arguments; used under rocprofv3,
// whose kernel tracer crashes on graph replays on this image).
bool eager_mode() {
    const char *e = getenv("MAGPIE_EAGER");
    return e && atoi(e) != 0;
}
// MAGPIE_Q8_UNFUSED=1: the Q8_0 mode's SA and XA as separate launches (the fused forms
// compute the same bits; tests/test_q8_fused_gpu.py compares them)
// MAGPIE_LT_CAND=1 (f32 batch 1, greedy): the LT head publishes a masked first-max
// candidate per workgroup and the next LT step picks from those (GemvP::cand) instead of
// scanning the head's 2024 logits. Both pick the same code (same bits). Off by default:
// measured 1.6 % slower at f32 B=1 (2,985 vs 3,034 frames/s, three alternating pairs on one
// box, profiles/r06b_ab_lt_cand.txt): the head's workgroup barrier and 64-bit reduction cost
// more than the step saves, whose pick waits on the logits' memory round trip either way.
bool lt_cand_mode() {
    const char *e = getenv("MAGPIE_LT_CAND");
    return e && atoi(e) != 0;
}
// The SA in the QKV launch at 16 slots: MAGPIE_SA16 unset = the bf16 mode's, 1 = every
// mode's, 0 = none (A/B; both forms compute the same bits). Round 3 kept it separate (bf16
// B=16 20.1k vs 21.5k frames/s then); since round 4's single pollers the fused form is
// faster: 31,891 -> 32,620 / 32,893 frames/s (qkv 4.54 + sa_attn 7.34 -> qkv_sa 11.05 us
// per layer; gpurun_out/r06l_ops_bf16_b16*)
bool sa16_fused(int weight_mode) {
    const char *e = getenv("MAGPIE_SA16");
    return e ? atoi(e) != 0 : weight_mode == MP_WEIGHTS_BF16;
}
// At 8 bf16 slots, which split states the split workgroups merge themselves (bit 0: SA, in
// the QKV launch; bit 1: XA, in the O-projection's) rather than the consumers' prologues
// (PRO_SA_MERGE, PRO_XA_LN): MAGPIE_MERGE8, default 3 (A/B; every setting the same bits)
int split_merge8() {
    const char *e = getenv("MAGPIE_MERGE8");
    return e ? atoi(e) : 3;
}
bool q8_unfused() {
    const char *e = getenv("MAGPIE_Q8_UNFUSED");
    return e && atoi(e) != 0;
}
// MAGPIE_LTQ8 (Q8_0 LT step, lt_slot_q8_kernel): 0 = o_net rows split over the workgroups
// (y hand-off) and the FFN merge in the launch; 1 = every workgroup all o_net rows (no y
// hand-off); 2 (default) = that up to 4 slots, and at batch 1 the FFN merge deferred to
// the head's prologue. Every setting computes the same bits (tests/test_q8_fused_gpu.py).
int ltq8_mode() {
    const char *e = getenv("MAGPIE_LTQ8");
    return e ? atoi(e) : 2;
}

// Diagnostics (MAGPIE_EAGER=1 and MAGPIE_DUMP_LT=file): after every launch of
// the local transformer, slot 0's LT state is appended to the file as f32
// records [logits 2024 | codes_cur 8 (int bits) | ltX | ltY | lty2 | ltq 256 each].
void dump_lt(const mp::LtIo &io, hipStream_t s) {
    const char *path = getenv("MAGPIE_DUMP_LT");
    if (!path || !eager_mode() || hipStreamSynchronize(s) != hipSuccess) return;
    std::vector<float> rec(2024 + 8 + 4 * 256);
    float *p = rec.data();
    auto get = [&](const void *src, size_t n) {
        if (hipMemcpy(p, src, n * 4, hipMemcpyDeviceToHost) != hipSuccess) return;
        p += n;
    };
    get(io.logits, 2024); get(io.codes_cur, 8); get(io.ltX, 256); get(io.ltY, 256); get(io.lty2, 256); get(io.ltq, 256);
    if (FILE *fp = fopen(path, "ab")) { fwrite(rec.data(), 4, rec.size(), fp); fclose(fp); }
}

int enqueue_lt(mp_dev *dev, const mp::LtIo &io, int NB, hipStream_t s, std::vector<mp::OpRec> *ops) {
    const mp::Model &m = dev->m;
    const bool b16 = mp::h16_mode(m.weight_mode);
    const mp::OpTable &tb = mp::table_for(NB, m.weight_mode);
    const mp::OpTableQ8 &tq = mp::table_q8(NB);
    const double F = b16 ? 2.0 : 4.0, A = 4.0, act = (double)NB;
    // a quantised tensor's decode bytes per weight: Q8_0 34/32, Q4_0 nibble fragments 18/32
    auto Fq = [](const mp::QW &w) { return w.nib ? 18.0 / 32.0 : 34.0 / 32.0; };
    auto run = [&](const char *name, mp::GemvFn fn, const mp::GemvP &g0, double bytes) -> int {
        mp::GemvP g = g0;
        q8dump_assign(dev, name, g);
        if (ops) {
            mp::OpRec r{};
            r.name = name; r.kind = mp::K_GEMV; r.fn = fn; r.g = g; r.B = NB; r.bytes = bytes;
            ops->push_back(r);
        }
        if (!fn) return fail(dev, MP_ERR_UNSUPPORTED, std::string(name) + ": no kernel for this batch size / weight mode");
        HIPCHK(fn(g, s));
        dump_lt(io, s);
        return MP_OK;
    };
    auto base = [&]() {
        mp::GemvP g;
        memset(&g, 0, sizeof g);
        g.eps = m.eps;
        g.step = io.step;
        g.smp = mp::Sampling{io.sampling, io.cfg, io.argeos, io.amax};
        g.nslots = NB;
        g.ignore_eos = io.ignore_eos;
        g.audio_bos = m.audio_bos;
        g.audio_eos = m.audio_eos;
        return g;
    };
    int rc;
    // f32 mode at batch 1: final LN + in_proj + position 0 + codebook 0's FFN step in one
    // launch (lt_front_kernel: the same rows, the same arithmetic; 2 in-launch granule edges)
    const bool front = f32_lt_mode(m) && NB == 1 && !io.lt_only && io.ltfg && io.iter;
    {
        mp::GemvP g = base();
        g.W = m.lt_in_w; g.N = 256; g.bias = m.lt_in_b; g.out = io.lt_s; g.out_ld = 9 * 256;
        g.Wq = m.lt_in8.pq; g.Wd = m.lt_in8.pd; g.q4 = m.lt_in8.nib; g.Wb = m.pk_lt_in;  // pk_lt_in: F16 mode only
        const double Fi = m.lt_in8 ? Fq(m.lt_in8) : m.pk_lt_in ? 2.0 : A;
        if (io.lt_only) {
            // in_proj of the caller's (already normalised) hidden (1161-1163)
            g.src = io.hidden; g.src_ld = 768;
            if ((rc = run("lt_inh", m.lt_in8 ? mp::q8_lt_inh_1 : m.pk_lt_in ? mp::f16_lt_inh_1 : mp::op_lt_inh_1, g,
                          Fi * 256.0 * 768 + A * 256 + A * (768 + 256))) != MP_OK)
                return rc;
        } else if (front) {
            // f32, batch 1: lt_front_kernel below runs the final LN, in_proj, position 0 and
            // codebook 0's FFN step in one launch
        } else {
            // final LN -> hidden (4394) fused into LT in_proj (1162-1163)
            g.lnw = m.dec_norm_out; g.src = io.x; g.src_ld = 768; g.hidden_out = io.hidden;
            if (io.trace) { g.trace = io.trace; g.trace_steps = io.trace_steps; g.step = io.step; }
            if ((rc = run("lt_in0", m.lt_in8 ? tq.lt_in0 : tb.lt_in0, g,
                          Fi * 256.0 * 768 + A * 256 + A * act * ((768 + 768 + 256)))) != MP_OK)
                return rc;
        }
    }
    if (m.weight_mode == MP_WEIGHTS_BF16) {
        // bf16 mode: the f32 mode's position 0 (LN + [k_0 | vo_0]), then per codebook the
        // LT step as LTS_P workgroups per slot (lt_slot_kernel: pick, f32 attention
        // through the tables, bf16 FFN, partial sums merged by the slot's last
        // workgroup) and the bf16 head: 2 launches per codebook at every batch size
        mp::GemvP g = base(); g.cb = 0;
        g.W = m.lt_kvo; g.N = 512; g.lt_s = io.lt_s; g.lt_pos = m.lt_pos; g.ltX = io.ltX; g.lnw = m.lt_norm_self;
        g.lk = io.ltk; g.lv = io.ltv;
        if (ops) {
            mp::OpRec r{};
            r.name = "lt_kvo"; r.kind = mp::K_LTKVO; r.g = g; r.B = NB;
            r.bytes = A * (512.0 * 256) + A * act * (256 * 4);
            ops->push_back(r);
        }
        HIPCHK(mp::op_lt_kvo(g, NB, s));
        dump_lt(io, s);
        for (int cb = 0; cb < 8; ++cb) {
            mp::LtFfn2P l2{};
            l2.f = mp::LtFfnP{io.ltY, m.lt_norm_ff, nullptr, nullptr, m.eps, io.ltp, io.lty2};
            // the partial sums merged by the head's prologue at batch 1 (32 KiB per head
            // workgroup; 4 slots' 128 KiB took 11.5 us), through granules by the LT step
            // itself above (the standalone LT API is batch 1: no iteration counter needed)
            const bool head_merge = NB == 1;
            l2.w1h = m.lt_ff1h; l2.w2h = m.lt_ff2h;
            if (!head_merge) { l2.gh = io.ltgh; l2.iter = io.iter; l2.hx_err = io.hx_err; }
            l2.cb = cb; l2.ltX = io.ltX; l2.ltk = io.ltk; l2.ltv = io.ltv; l2.qkvtab = m.lt_qkvtab;
            l2.votab = m.lt_votab; l2.ptab = m.lt_ptab; l2.lt_pos = m.lt_pos; l2.logits = io.logits;
            l2.codes_cur = io.codes_cur; l2.step = io.step; l2.ignore_eos = io.ignore_eos;
            l2.audio_bos = m.audio_bos; l2.audio_eos = m.audio_eos;
            l2.smp = mp::Sampling{io.sampling, io.cfg, io.argeos, io.amax};
            if (ops) {
                mp::OpRec r{};
                r.name = "lt_slot"; r.kind = mp::K_LTSLOT; r.l2 = l2; r.B = NB;
                r.bytes = F * (1024.0 * 256 * 2) + A * act * (cb ? 2024 + 4 * 256 + 2 * 256 * cb : 512) +
                          A * act * (mp::LTS_P * 256 + 256);
                ops->push_back(r);
            }
            HIPCHK(mp::op_lt_slot(l2, NB, s));
            dump_lt(io, s);
            g = base(); g.cb = cb;
            g.W = m.lt_out_w + (size_t)cb * 2024 * 256; g.N = 2024; g.bias = m.lt_out_b + (size_t)cb * 2024;
            g.Wb = m.pk_lt_out + (size_t)cb * pk_elems(2024, 256);
            g.src = io.lty2; g.src_ld = 256; g.out = io.logits; g.out_ld = 2024;
            if (head_merge) { g.part = io.ltp; g.addsrc = io.ltY; }
            if ((rc = run("lt_e", head_merge ? tb.lt_em : tb.lt_es, g,
                          F * (2024.0 * 256) + A * 2024 + A * act * ((head_merge ? mp::LTS_P * 256 : 256) + 2024))) != MP_OK)
                return rc;
        }
    } else if (f32_lt_mode(m)) {
        // f32 mode: LN + [k_0 | vo_0] for position 0, then per codebook ONE launch for
        // pick + attention + o_net + residual + FFN (lt_ffn2_kernel) and the head
        mp::GemvP g = base(); g.cb = 0;
        g.W = m.lt_kvo; g.N = 512; g.lt_s = io.lt_s; g.lt_pos = m.lt_pos; g.ltX = io.ltX; g.lnw = m.lt_norm_self;
        g.lk = io.ltk; g.lv = io.ltv;
        if (!front) {
            if (ops) {
                mp::OpRec r{};
                r.name = "lt_kvo"; r.kind = mp::K_LTKVO; r.g = g; r.B = NB;
                r.bytes = A * (512.0 * 256) + A * act * (256 * 4);
                ops->push_back(r);
            }
            HIPCHK(mp::op_lt_kvo(g, NB, s));
            dump_lt(io, s);
        }
        for (int cb = 0; cb < 8; ++cb) {
            mp::LtFfn2P l2{};
            l2.f = mp::LtFfnP{io.ltY, m.lt_norm_ff, m.lt_ff1, m.lt_ff2s, m.eps, io.ltp, io.lty2};
            l2.cb = cb; l2.ltX = io.ltX; l2.ltk = io.ltk; l2.ltv = io.ltv; l2.qkvtab = m.lt_qkvtab;
            l2.votab = m.lt_votab; l2.ptab = m.lt_ptab; l2.lt_pos = m.lt_pos; l2.logits = io.logits;
            l2.codes_cur = io.codes_cur; l2.step = io.step; l2.ignore_eos = io.ignore_eos;
            l2.audio_bos = m.audio_bos; l2.audio_eos = m.audio_eos;
            l2.smp = mp::Sampling{io.sampling, io.cfg, io.argeos, io.amax};
            // greedy batch 1: the pick from the previous head's workgroup candidates
            const bool cand = NB == 1 && !io.sampling && io.ltcand && !io.lt_only;
            if (cand && cb > 0) { l2.cand = io.ltcand; l2.ncand = (2024 + 4 * MP_RW_LTE - 1) / (4 * MP_RW_LTE); }
            if (front && cb == 0) {
                mp::LtFrontP fp{};
                fp.l = l2; fp.x = io.x; fp.norm_out = m.dec_norm_out; fp.w_in = m.lt_in_w; fp.b_in = m.lt_in_b;
                fp.lt_s = io.lt_s; fp.hidden_out = io.hidden; fp.lt_pos = m.lt_pos; fp.norm_self = m.lt_norm_self;
                fp.w_kvo = m.lt_kvo; fp.gh = io.ltfg; fp.iter = io.iter; fp.hx_err = io.hx_err;
                if (io.trace) { fp.trace = io.trace; fp.trace_steps = io.trace_steps; }
                if (!io.sampling && lt_all_mode()) {
                    // the whole LT in one launch (lt_all_kernel): the front, then every codebook's
                    // FFN merge, head and greedy pick through granules; codebook 7's pick is the finalize's
                    mp::LtAllP la{};
                    la.f = fp; la.w_out = m.lt_out_w; la.b_out = m.lt_out_b; la.logits = io.logits;
                    la.gp = io.ltfg + mp::LTFG_GP; la.gy = io.ltfg + mp::LTFG_GY; la.gc = io.ltfg + mp::LTFG_GC;
                    if (ops) {
                        mp::OpRec r{};
                        r.name = "lt_all"; r.kind = mp::K_LTALL; r.la = la; r.B = NB;
                        r.bytes = A * (256.0 * 768 + 512.0 * 256 + 1024.0 * 256 * 2 + 8.0 * 2024 * 256 + 8.0 * 2024) +
                                  A * (768 * 2 + 256 * 4) + A * 7.0 * (3 * 256 + 2 * 256);
                        ops->push_back(r);
                    }
                    HIPCHK(mp::op_lt_all(la, s));
                    dump_lt(io, s);
                    break;
                }
                if (ops) {
                    mp::OpRec r{};
                    r.name = "lt_front"; r.kind = mp::K_LTFRONT; r.lf3 = fp; r.B = NB;
                    r.bytes = A * (256.0 * 768 + 512.0 * 256 + 1024.0 * 256 * 2) + A * (768 * 2 + 256 * 4) +
                              A * (mp::LT_FFN_P * 256);
                    ops->push_back(r);
                }
                HIPCHK(mp::op_lt_front(fp, s));
                dump_lt(io, s);
            } else {
                if (ops) {
                    mp::OpRec r{};
                    r.name = "lt_ffn2"; r.kind = mp::K_LTFFN2; r.l2 = l2; r.B = NB;
                    r.bytes = A * (1024.0 * 256 * 2) + A * act * (cb ? 2024 + 4 * 256 + 2 * 256 * cb : 512) +
                              A * act * (mp::LT_FFN_P * 256 + 256);
                    ops->push_back(r);
                }
                HIPCHK(mp::op_lt_ffn2(l2, NB, s));
                dump_lt(io, s);
            }
            if (NB > 1) {
                if (ops) {
                    mp::OpRec r{};
                    r.name = "lt_merge"; r.kind = mp::K_LTMERGE; r.lf = l2.f; r.B = NB;
                    r.bytes = A * act * (mp::LT_FFN_P * 256 + 512);
                    ops->push_back(r);
                }
                HIPCHK(mp::op_lt_merge(l2.f, NB, s));
            }
            g = base(); g.cb = cb;
            g.W = m.lt_out_w + (size_t)cb * 2024 * 256; g.N = 2024; g.bias = m.lt_out_b + (size_t)cb * 2024;
            g.src = io.lty2; g.src_ld = 256; g.out = io.logits; g.out_ld = 2024;
            mp::GemvFn efn = tb.lt_e;
            if (NB == 1) {  // the FFN merge is the head's prologue
                g.part = io.ltp; g.addsrc = io.ltY;
                efn = mp::op_lt_em_1;
                if (cand && cb < 7) g.cand = io.ltcand;  // (codebook 7's code is the finalize's pick)
            }
            if ((rc = run("lt_e", efn, g, A * (2024.0 * 256) + A * 2024 + A * act * ((256 + 2024)))) != MP_OK)
                return rc;
        }
    } else if (m.weight_mode == MP_WEIGHTS_Q8 && m.lt_o8 && m.lt_out8 && m.lt_ff2q && !io.lt_only && io.ltyg) {
        // Q8_0 mode: position 0's q|k|v (the Q8_0 GEMV), then per codebook the LT step as
        // LTQ_P workgroups per slot (lt_slot_q8_kernel: pick, attention, Q8_0 o_net, F32
        // FFN, partial sums merged through granules) and the Q8_0 head on its output
        mp::GemvP g = base(); g.cb = 0;
        g.W = m.lt_qkv; g.N = 768; g.lt_s = io.lt_s; g.lt_pos = m.lt_pos; g.ltX = io.ltX;
        g.Wq = m.lt_qkv8.pq; g.Wd = m.lt_qkv8.pd; g.q4 = m.lt_qkv8.nib;
        g.lnw = m.lt_norm_self; g.lq = io.ltq; g.lk = io.ltk; g.lv = io.ltv;
        if ((rc = run("lt_a", tq.lt_a, g, Fq(m.lt_qkv8) * (768.0 * 256) + A * act * (256 * 3 + 768 + 256))) != MP_OK)
            return rc;
        for (int cb = 0; cb < 8; ++cb) {
            mp::LtSlotQ8P sp{};
            sp.g = base(); sp.g.cb = cb;
            sp.g.logits = io.logits; sp.g.codes_cur = io.codes_cur; sp.g.qkvtab = m.lt_qkvtab; sp.g.ptab = m.lt_ptab;
            sp.g.lt_pos = m.lt_pos; sp.g.ltk = io.ltk; sp.g.ltv = io.ltv; sp.g.lk = io.ltk; sp.g.lv = io.ltv;
            sp.g.ltX = io.ltX;
            sp.woq = m.lt_o8.q; sp.wod = m.lt_o8.d; sp.lnw = m.lt_norm_ff; sp.eps = m.eps; sp.w1 = m.lt_ff1;
            sp.w2s = m.lt_ff2q; sp.y = io.ltY; sp.y2 = io.lty2; sp.gy = io.ltyg; sp.gp = io.ltgh;
            sp.iter = io.iter; sp.hx_err = io.hx_err;
            const int lm = ltq8_mode();
            if (lm == 1 || (lm >= 2 && NB <= 4)) sp.wot = m.lt_o8t;  // (8+ slots: 512+ workgroups, the split rows)
            if (lm >= 2 && NB == 1 && sp.wot) sp.part = io.ltp;
            if (ops) {
                mp::OpRec r{};
                r.name = "lt_slot_q8"; r.kind = mp::K_LTSLOTQ8; r.lq8 = sp; r.B = NB;
                r.bytes = (34.0 / 32.0) * (256.0 * 256) + A * (1024.0 * 256 * 2) +
                          A * act * (cb ? 2024 + 4 * 256 + 2 * 256 * cb : 512) + A * act * (mp::LTQ_P * 256 + 512);
                ops->push_back(r);
            }
            HIPCHK(mp::op_lt_slot_q8(sp, NB, s));
            dump_lt(io, s);
            g = base(); g.cb = cb;
            g.W = m.lt_out_w + (size_t)cb * 2024 * 256; g.N = 2024; g.bias = m.lt_out_b + (size_t)cb * 2024;
            g.src = io.lty2; g.src_ld = 256; g.out = io.logits; g.out_ld = 2024;
            g.Wq = m.lt_out8.pq + (size_t)cb * m.lt_out8.head_q; g.q4 = m.lt_out8.nib;
            g.Wd = (const unsigned short *)((const char *)m.lt_out8.pd + (size_t)cb * q8p_head_d());
            mp::GemvFn efn = tq.lt_e;
            if (sp.part) {  // the FFN merge is the head's prologue
                g.part = io.ltp; g.addsrc = io.ltY;
                efn = mp::q8_lt_em_1;
            }
            if ((rc = run("lt_e", efn, g, Fq(m.lt_out8) * (2024.0 * 256) + A * 2024 + A * act * ((256 + 2024)))) != MP_OK)
                return rc;
        }
    } else
    for (int cb = 0; cb < 8; ++cb) {
        mp::GemvP g;
        if (cb == 0) {
            // position 0 (the hidden's in_proj): LN + q|k|v GEMV, then attention + o_net
            g = base(); g.cb = 0;
            g.W = m.lt_qkv; g.Wb = m.pk_lt_qkv; g.N = 768; g.lt_s = io.lt_s; g.lt_pos = m.lt_pos; g.ltX = io.ltX;
            g.Wq = m.lt_qkv8.pq; g.Wd = m.lt_qkv8.pd; g.q4 = m.lt_qkv8.nib;
            g.lnw = m.lt_norm_self; g.lq = io.ltq; g.lk = io.ltk; g.lv = io.ltv;
            if ((rc = run("lt_a", m.lt_qkv8 ? tq.lt_a : tb.lt_a, g,
                          (m.lt_qkv8 ? Fq(m.lt_qkv8) : F) * (768.0 * 256) + A * act * (256 * 3 + 768 + 256))) != MP_OK)
                return rc;
            g = base(); g.cb = 0;
            g.W = m.lt_o; g.Wb = m.pk_lt_o; g.N = 256; g.ltq = io.ltq; g.ltk = io.ltk; g.ltv = io.ltv; g.out = io.ltY;
            g.Wq = m.lt_o8.pq; g.Wd = m.lt_o8.pd; g.q4 = m.lt_o8.nib;
            g.out_ld = 256; g.addsrc = io.ltX;
            if ((rc = run("lt_b", m.lt_o8 ? tq.lt_b : tb.lt_b, g,
                          (m.lt_o8 ? Fq(m.lt_o8) : F) * (256.0 * 256) + A * act * (256 * 5))) != MP_OK)
                return rc;
        } else if (NB >= 8) {
            // large batches: the per-slot pick + gathers + attention as one wave per slot
            // (lt_pick_kernel), then o_net + residual; the same arithmetic as lt_bg
            g = base(); g.cb = cb;
            g.logits = io.logits; g.codes_cur = io.codes_cur; g.qkvtab = m.lt_qkvtab; g.ptab = m.lt_ptab;
            g.lt_pos = m.lt_pos; g.ltk = io.ltk; g.ltv = io.ltv; g.lk = io.ltk; g.lv = io.ltv; g.ltX = io.ltX;
            g.out = io.ltq;
            if (ops) {
                mp::OpRec r{};
                r.name = "lt_pick"; r.kind = mp::K_LTPICK; r.g = g; r.B = NB;
                r.bytes = A * act * (2024 + 4 * 256 + 2 * 256 * cb + 4 * 256);
                ops->push_back(r);
            }
            HIPCHK(mp::op_lt_pick(g, NB, s));
            dump_lt(io, s);
            g = base(); g.cb = cb;
            g.W = m.lt_o; g.Wb = m.pk_lt_o; g.N = 256; g.src = io.ltq; g.src_ld = 256; g.out = io.ltY; g.out_ld = 256;
            g.addsrc = io.ltX; g.Wq = m.lt_o8.pq; g.Wd = m.lt_o8.pd; g.q4 = m.lt_o8.nib;
            const bool f16 = m.weight_mode == MP_WEIGHTS_F16;
            const mp::GemvFn bo = m.lt_o8 ? (NB == 16 ? mp::q8_lt_bo_16 : mp::q8_lt_bo_8)
                                  : f16   ? (NB == 16 ? mp::f16_lt_bo_16 : mp::f16_lt_bo_8)
                                  : b16   ? (NB == 16 ? mp::b16_lt_bo_16 : mp::b16_lt_bo_8)
                                          : mp::op_lt_bo_8;
            if ((rc = run("lt_bo", bo, g, (m.lt_o8 ? Fq(m.lt_o8) : F) * (256.0 * 256) + A * act * (256 * 3))) != MP_OK) return rc;
        } else {
            // position cb: codebook cb-1's pick, its q|k|v row gathered from the load-time
            // table (no q|k|v GEMV), attention + o_net + residual, one launch
            g = base(); g.cb = cb;
            g.W = m.lt_o; g.Wb = m.pk_lt_o; g.N = 256; g.out = io.ltY; g.out_ld = 256;
            g.Wq = m.lt_o8.pq; g.Wd = m.lt_o8.pd; g.q4 = m.lt_o8.nib;
            g.logits = io.logits; g.codes_cur = io.codes_cur; g.qkvtab = m.lt_qkvtab; g.ptab = m.lt_ptab;
            g.lt_pos = m.lt_pos; g.ltk = io.ltk; g.ltv = io.ltv; g.lk = io.ltk; g.lv = io.ltv;
            if ((rc = run("lt_bg", m.lt_o8 ? tq.lt_bg : tb.lt_bg, g,
                          (m.lt_o8 ? Fq(m.lt_o8) : F) * (256.0 * 256) +
                              A * act * (2024 + 3 * 256 + 2 * 256 * cb + 2 * 256 + 256))) != MP_OK)
                return rc;
        }
        // FFN up + GELU + FFN down: one launch of partial sums (f32 FFN weights), merged by
        // the head's prologue at batch 1 or by a one-workgroup merge; bf16 mode: two GEMVs
        const bool ffn1 = !b16;
        if (ffn1) {
            mp::LtFfnP lf{io.ltY, m.lt_norm_ff, m.lt_ff1, m.lt_ff2s, m.eps, io.ltp, io.lty2};
            if (ops) {
                mp::OpRec r{};
                r.name = "lt_ffn"; r.kind = mp::K_LTFFN; r.lf = lf; r.B = NB;
                r.bytes = A * (1024.0 * 256 * 2) + A * act * (256 + mp::LT_FFN_P * 256);
                ops->push_back(r);
            }
            HIPCHK(mp::op_lt_ffn(lf, NB, s));
            if (NB > 1) {
                if (ops) {
                    mp::OpRec r{};
                    r.name = "lt_merge"; r.kind = mp::K_LTMERGE; r.lf = lf; r.B = NB;
                    r.bytes = A * act * (mp::LT_FFN_P * 256 + 512);
                    ops->push_back(r);
                }
                HIPCHK(mp::op_lt_merge(lf, NB, s));
            }
        } else {
            g = base(); g.cb = cb;
            g.W = m.lt_ff1; g.Wb = m.pk_lt_ff1; g.N = 1024; g.lnw = m.lt_norm_ff; g.src = io.ltY; g.src_ld = 256;
            g.out = io.ltf; g.out_ld = 1024;
            if ((rc = run("lt_c", tb.lt_c, g, F * (1024.0 * 256) + A * act * ((256 + 1024)))) != MP_OK) return rc;
            g = base(); g.cb = cb;
            g.W = m.lt_ff2; g.Wb = m.pk_lt_ff2; g.N = 256; g.src = io.ltf; g.src_ld = 1024; g.out = io.lty2;
            g.out_ld = 256; g.addsrc = io.ltY;
            if ((rc = run("lt_d", tb.lt_d, g, F * (256.0 * 1024) + A * act * ((1024 + 512)))) != MP_OK) return rc;
        }
        g = base(); g.cb = cb;
        g.W = m.lt_out_w + (size_t)cb * 2024 * 256; g.N = 2024;
        g.Wb = b16 ? m.pk_lt_out + (size_t)cb * pk_elems(2024, 256) : nullptr; g.bias = m.lt_out_b + (size_t)cb * 2024;
        g.src = io.lty2; g.src_ld = 256; g.out = io.logits; g.out_ld = 2024;
        if (m.lt_out8) {
            g.Wq = m.lt_out8.pq + (size_t)cb * m.lt_out8.head_q; g.q4 = m.lt_out8.nib;
            g.Wd = (const unsigned short *)((const char *)m.lt_out8.pd + (size_t)cb * q8p_head_d());
        }
        mp::GemvFn efn = m.lt_out8 ? tq.lt_e : tb.lt_e;
        if (ffn1 && NB == 1) {  // the FFN merge (lt_ffn_kernel's interleaved partials) is the head's prologue
            g.part = io.ltp; g.addsrc = io.ltY;
            efn = m.lt_out8 ? mp::q8_lt_emf_1 : mp::op_lt_em_1;
        }
        if ((rc = run("lt_e", efn, g,
                      (m.lt_out8 ? Fq(m.lt_out8) : F) * (2024.0 * 256) + A * 2024 + A * act * ((256 + 2024)))) != MP_OK)
            return rc;
    }
    mp::FinP f{io.logits, io.codes_cur, io.codes_prev, io.codes_out, io.step, io.pos, io.done, io.nframes, io.ndone,
               io.max_steps, io.ignore_eos, m.audio_bos, m.audio_eos, NB,
               mp::Sampling{io.sampling, io.cfg, io.argeos, io.amax}, io.emit_eos, io.lt_only,
               io.lt_only ? nullptr : io.ndone + 1};
    if (!io.lt_only) { f.emb = m.audio_emb; f.pos_emb = m.dec_pos; f.x = io.x; f.pos_rows = m.dec_pos_rows; }  // the next frame's input
    if (ops) {
        mp::OpRec r{};
        r.name = "finalize"; r.kind = mp::K_FIN; r.f = f; r.B = NB; r.bytes = A * act * 2024;
        ops->push_back(r);
    }
    HIPCHK(mp::op_finalize(f, NB, s));
    return MP_OK;
}

// ------------------------------------------------------------------ preamble
// The text encoder's buffers: the batch's preamble scratch (run_preamble) or a private
// workspace (mp_hip_encode_text, which must not touch a batch in progress).
struct EncWs {
    const int32_t *tok, *T;  // device [NB][Tmax] token ids, [NB] lengths
    int NB, Tmax;
    float *pX, *pH, *pQKV, *pATT, *pF, *gpart, *enc_out;
};
static size_t enc_gpart_elems(size_t Me) {
    size_t cap = 0;
    auto need = [&](size_t M, int N, int K) { cap = std::max(cap, (size_t)mp::gemm_splits_max(K) * M * N); };
    need(Me, 2304, 768); need(Me, 3072, 768 * 3); need(Me, 768, 3072 * 3); need(Me, 256, 768);
    return cap;
}
// every preamble GEMM runs split-K over K (deterministic, batch-invariant)
// F16 file: every projection's operand rounded to f16 as ggml's F16 mul_mat does
// (the K'/V' precompute is weight algebra, not a mul_mat of the file)
static hipError_t preamble_gemm(const mp::Model &m, float *gpart, mp::GemmP gp, int epi, hipStream_t st) {
    gp.part = gpart;
    if (gp.ln_w) gp.ln_eps = m.eps;
    gp.xround = gp.xround < 0 ? 0 : (m.weight_mode == MP_WEIGHTS_F16 ? 2 : 0);  // -1: opted out
    return mp::pre_gemm(gp, epi, st);
}
// --- text encoder (magpie_build_full_encoder, 1960-1995) into w.enc_out [NB][Tmax][768]
static int run_encoder(mp_dev *dev, const EncWs &w, hipStream_t s) {
    using namespace mp;
    const Model &m = dev->m;
    const int Tmax = w.Tmax, Me = w.NB * Tmax;
    auto pre_gemm = [&](GemmP gp, int epi, hipStream_t st) { return preamble_gemm(m, w.gpart, gp, epi, st); };
    HIPCHK(pre_embed_text(w.tok, w.T, w.NB, Tmax, m.text_emb, m.enc_pos, w.pX, s));
    // the residual GEMMs (O-projection, FFN down) normalise the rows they complete for the
    // next LayerNorm (GemmP::ln_w: fused into their split reduction)
    HIPCHK(pre_ln_rows(w.pX, 768, m.enc[0].norm_self, w.pH, 768, Me, m.eps, s));
    for (int l = 0; l < m.enc_layers; ++l) {
        const EncLayerW &W = m.enc[l];
        GemmP gp{};
        gp.A = w.pH; gp.lda = 768; gp.W = W.qkv; gp.Wq = W.qkv8.q; gp.Wd = W.qkv8.d; gp.C = w.pQKV; gp.ldc = 2304; gp.M = Me; gp.N = 2304; gp.K = 768;
        gp.rows_per_utt = Tmax; gp.T = w.T;
        HIPCHK(pre_gemm(gp, GE_STORE, s));
        RowAttnP ra{};
        ra.Q = w.pQKV; ra.ldq = 2304; ra.Kb = w.pQKV + 768; ra.Vb = w.pQKV + 1536;
        ra.utt_stride = (size_t)Tmax * 2304; ra.row_stride = 2304; ra.O = w.pATT; ra.M = Me; ra.rows_per_utt = Tmax;
        ra.heads = 12; ra.T = w.T;
        HIPCHK(pre_row_attn(ra, s));
        gp = GemmP{};
        gp.A = w.pATT; gp.lda = 768; gp.W = W.o; gp.Wq = W.o8.q; gp.Wd = W.o8.d; gp.C = w.pX; gp.ldc = 768; gp.M = Me; gp.N = 768; gp.K = 768;
        gp.rows_per_utt = Tmax; gp.T = w.T;
        gp.ln_w = W.norm_ff; gp.ln_out = w.pH; gp.ln_ld = 768;
        HIPCHK(pre_gemm(gp, GE_RESID, s));
        gp = GemmP{};  // causal conv k=3 d_model -> d_ffn + GELU (1816-1869)
        gp.A = w.pH; gp.lda = 768; gp.W = W.ff1; gp.C = w.pF; gp.ldc = 3072; gp.M = Me; gp.N = 3072;
        gp.K = 768 * 3; gp.conv_taps = 3; gp.rows_per_utt = Tmax; gp.T = w.T;
        HIPCHK(pre_gemm(gp, GE_GELU, s));
        gp = GemmP{};  // causal conv k=3 d_ffn -> d_model + residual (1875-1916)
        gp.A = w.pF; gp.lda = 3072; gp.W = W.ff2; gp.C = w.pX; gp.ldc = 768; gp.M = Me; gp.N = 768;
        gp.K = 3072 * 3; gp.conv_taps = 3; gp.rows_per_utt = Tmax; gp.T = w.T;
        if (l + 1 < m.enc_layers) { gp.ln_w = m.enc[l + 1].norm_self; gp.ln_out = w.pH; }
        else { gp.ln_w = m.enc_norm_out; gp.ln_out = w.enc_out; }  // the encoder's final norm
        gp.ln_ld = 768;
        HIPCHK(pre_gemm(gp, GE_RESID, s));
    }
    return MP_OK;
}

int run_preamble(mp_dev *dev) {
    using namespace mp;
    const Model &m = dev->m;
    const int NB = dev->NB, Tmax = dev->Tmax, L = m.dec_layers;
    hipStream_t s = dev->stream;
    const int Me = NB * Tmax;
    auto pre_gemm = [&](GemmP gp, int epi, hipStream_t st) { return preamble_gemm(m, dev->gpart, gp, epi, st); };
    {
        const EncWs w{dev->tok, dev->T, NB, Tmax, dev->pX, dev->pH, dev->pQKV, dev->pATT, dev->pF, dev->gpart, dev->enc_out};
        if (int rc = run_encoder(dev, w, s)) return rc;
    }
    // --- cross-attention K/V per layer (1663-1711): LN(encoder output) with each layer's
    //     norm_xmem, then kv_net. Layers whose tensors sit at one stride in the arena (the
    //     loader places every layer's tensors alike) run G at a time: one LN launch for G
    //     weight vectors, one batched GEMM (grid.z = G x splits) and its reduce, instead of
    //     3 launches per layer; each layer's arithmetic is its own GEMM's
    auto stride_of = [&](auto get) -> long long {  // elements between layers' tensors, or -1
        if (L == 1) return 0;
        const long long st = (long long)(get(1) - get(0));
        for (int l = 2; l < L; ++l)
            if ((long long)(get(l) - get(0)) != st * l) return -1;
        return st;
    };
    const long long s_norm = stride_of([&](int l) { return m.dec[l].norm_xmem; });
    const long long s_xkv = stride_of([&](int l) { return m.dec[l].xkv; });
    const bool q8kv = (bool)m.dec[0].xkv8;
    const long long s_xkvq = q8kv ? stride_of([&](int l) { return m.dec[l].xkv8.q; }) : 0;
    const long long s_xkvd = q8kv ? stride_of([&](int l) { return m.dec[l].xkv8.d; }) : 0;
    const size_t pf_rows = (size_t)NB * std::max(Tmax, (int)CTX);
    const int G = (s_norm >= 0 && s_xkv >= 0 && s_xkvq >= 0 && s_xkvd >= 0)
                      ? (int)std::max<size_t>(1, std::min<size_t>(L, pf_rows * 3072 / ((size_t)Me * 768)))
                      : 1;
    for (int l0 = 0; l0 < L; l0 += G) {
        const int g = std::min(G, L - l0);
        HIPCHK(pre_ln_rows_multi(dev->enc_out, 768, m.dec[l0].norm_xmem, s_norm, dev->pF, 768, (long long)Me * 768, Me, g,
                                 m.eps, s));
        GemmP gp{};
        gp.A = dev->pF; gp.lda = 768; gp.W = m.dec[l0].xkv; gp.Wq = m.dec[l0].xkv8.q; gp.Wd = m.dec[l0].xkv8.d; gp.M = Me; gp.N = 256; gp.K = 768; gp.rows_per_utt = Tmax;
        gp.T = dev->T; gp.xak = dev->xak; gp.xav = dev->xav; gp.layer = l0; gp.nlayers = L; gp.Tmax = Tmax;
        gp.nbatch = g; gp.wmod = g; gp.sA = (long long)Me * 768; gp.sW = s_xkv; gp.sWq = s_xkvq; gp.sWd = s_xkvd;
        HIPCHK(pre_gemm(gp, GE_XAKV, s));
    }
    // --- K'_t = W_q^T K_t, V'_t = W_o V_t per utterance and layer (decode-time fused XA;
    //     not with Q8_0 q_net / o_net, whose activations ggml quantises: unfused XA there).
    //     Every (utterance, layer) pair in one batched GEMM each (K = 128: no split): A rows
    //     at stride Tmax x 128, weights of layer (pair % L), outputs at stride Tmax x 768
    bool any_xq8 = false;
    for (int l = 0; l < L; ++l) any_xq8 |= (bool)m.dec[l].xq8;
    const long long s_xo = stride_of([&](int l) { return m.dec[l].xo; });
    if (!dev->xa_direct && !any_xq8 && s_xo >= 0) {
        GemmP gp{};
        gp.A = dev->xak; gp.lda = 128; gp.W = m.xq_t[0]; gp.C = dev->kp; gp.ldc = 768;
        gp.M = Tmax; gp.N = 768; gp.K = 128; gp.rows_per_utt = Tmax;
        gp.xround = -1;
        gp.nbatch = NB * L; gp.wmod = L; gp.sA = (long long)Tmax * 128; gp.sW = 768 * 128; gp.sC = (long long)Tmax * 768;
        HIPCHK(pre_gemm(gp, GE_STORE, s));
        gp.A = dev->xav; gp.W = m.dec[0].xo; gp.C = dev->vp; gp.sW = s_xo;
        HIPCHK(pre_gemm(gp, GE_STORE, s));
    } else {
        for (int b = 0; b < NB; ++b)
            for (int l = 0; l < L; ++l) {
                if (m.dec[l].xq8 || dev->xa_direct) continue;
                const size_t xo = ((size_t)(b * L + l) * Tmax) * 128, po = ((size_t)(b * L + l) * Tmax) * 768;
                GemmP gp{};
                gp.A = dev->xak + xo; gp.lda = 128; gp.W = m.xq_t[l]; gp.C = dev->kp + po; gp.ldc = 768;
                gp.M = Tmax; gp.N = 768; gp.K = 128; gp.rows_per_utt = Tmax;
                gp.xround = -1;
                HIPCHK(pre_gemm(gp, GE_STORE, s));
                gp.A = dev->xav + xo; gp.W = m.dec[l].xo; gp.C = dev->vp + po;
                HIPCHK(pre_gemm(gp, GE_STORE, s));
            }
    }
    // --- baked context + 110-frame causal prefill (3991-4060, 4167-4238)
    const int Mc = NB * CTX;
    HIPCHK(pre_embed_context(dev->spk, NB, m.baked, m.dec_pos, dev->pX, s));
    HIPCHK(pre_ln_rows(dev->pX, 768, m.dec[0].norm_self, dev->pH, 768, Mc, m.eps, s));
    for (int l = 0; l < L; ++l) {
        const DecLayerW &W = m.dec[l];
        GemmP gp{};
        gp.A = dev->pH; gp.lda = 768; gp.W = W.qkv; gp.Wq = W.qkv8.q; gp.Wd = W.qkv8.d; gp.C = dev->pQKV; gp.ldc = 2304; gp.M = Mc; gp.N = 2304; gp.K = 768;
        gp.rows_per_utt = CTX; gp.kc = dev->kc; gp.vc = dev->vc; gp.kv16 = dev->kv16; gp.layer = l; gp.nlayers = L;
        gp.max_seq = dev->max_seq;
        HIPCHK(pre_gemm(gp, GE_QKV_CACHE, s));
        RowAttnP ra{};
        ra.Q = dev->pQKV; ra.ldq = 2304;
        {   // layer l's rows, offset in cache elements (bf16 elements in MP_KV_BF16 mode)
            const size_t off = (size_t)l * dev->max_seq * 768;
            ra.Kb = dev->kv16 ? (const float *)((const unsigned short *)dev->kc + off) : dev->kc + off;
            ra.Vb = dev->kv16 ? (const float *)((const unsigned short *)dev->vc + off) : dev->vc + off;
        }
        ra.utt_stride = (size_t)L * dev->max_seq * 768; ra.row_stride = 768; ra.O = dev->pATT; ra.M = Mc;
        ra.rows_per_utt = CTX; ra.heads = 12; ra.T = dev->T; ra.kv16 = dev->kv16;
        HIPCHK(pre_row_attn(ra, s));
        gp = GemmP{};
        gp.A = dev->pATT; gp.lda = 768; gp.W = W.o; gp.Wq = W.o8.q; gp.Wd = W.o8.d; gp.C = dev->pX; gp.ldc = 768; gp.M = Mc; gp.N = 768; gp.K = 768;
        gp.rows_per_utt = CTX;
        gp.ln_w = W.norm_xq; gp.ln_out = dev->pH; gp.ln_ld = 768;
        HIPCHK(pre_gemm(gp, GE_RESID, s));
        gp = GemmP{};
        gp.A = dev->pH; gp.lda = 768; gp.W = W.xq; gp.Wq = W.xq8.q; gp.Wd = W.xq8.d; gp.C = dev->pXQ; gp.ldc = 128; gp.M = Mc; gp.N = 128; gp.K = 768;
        gp.rows_per_utt = CTX;
        HIPCHK(pre_gemm(gp, GE_STORE, s));
        RowXaP rx{dev->pXQ, dev->xak, dev->xav, l, L, Tmax, CTX, Mc, dev->T, dev->pXAO};
        HIPCHK(pre_row_xa(rx, s));
        gp = GemmP{};
        gp.A = dev->pXAO; gp.lda = 128; gp.W = W.xo; gp.Wq = W.xo8.q; gp.Wd = W.xo8.d; gp.C = dev->pX; gp.ldc = 768; gp.M = Mc; gp.N = 768; gp.K = 128;
        gp.rows_per_utt = CTX;
        gp.ln_w = W.norm_ff; gp.ln_out = dev->pH; gp.ln_ld = 768;
        HIPCHK(pre_gemm(gp, GE_RESID, s));
        gp = GemmP{};
        gp.A = dev->pH; gp.lda = 768; gp.W = W.ff1; gp.C = dev->pF; gp.ldc = 3072; gp.M = Mc; gp.N = 3072; gp.K = 768;
        gp.rows_per_utt = CTX;
        HIPCHK(pre_gemm(gp, GE_GELU, s));
        gp = GemmP{};
        gp.A = dev->pF; gp.lda = 3072; gp.W = W.ff2; gp.C = dev->pX; gp.ldc = 768; gp.M = Mc; gp.N = 768; gp.K = 3072;
        gp.rows_per_utt = CTX;
        if (l + 1 < L) { gp.ln_w = m.dec[l + 1].norm_self; gp.ln_out = dev->pH; gp.ln_ld = 768; }
        HIPCHK(pre_gemm(gp, GE_RESID, s));
    }
    return MP_OK;
}

}  // namespace

// ====================================================================== C-ABI
extern "C" {

int mp_hip_device_count(int *n) {
    if (!n) return MP_ERR_ARG;
    if (hipGetDeviceCount(n) != hipSuccess) { *n = 0; return MP_ERR_HIP; }
    return MP_OK;
}

const char *mp_hip_runtime_path(void) {
    Dl_info info;
    if (dladdr((void *)&hipGetDeviceCount, &info) && info.dli_fname) return info.dli_fname;
    return "";
}

int mp_hip_init(int device, mp_dev **out) {
    if (!out) return MP_ERR_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return MP_ERR_HIP;
    mp_dev *dev = new mp_dev();
    dev->device = device;
    // the decode stream at the device's greatest priority: when the codec runs beside it (the
    // streaming loop, configs[2]'s overlapped chunks) the dispatcher serves the latency-bound
    // frame loop's workgroups first and the codec (least priority, mp_hip_codec_init) fills in
    // (MAGPIE_STREAM_PRIO=0: the default priority, A/B)
    int least = 0, greatest = 0;
    const char *pe = getenv("MAGPIE_STREAM_PRIO");
    const bool prio = !pe || atoi(pe) != 0;
    if (hipSetDevice(device) != hipSuccess || hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess ||
        hipStreamCreateWithPriority(&dev->stream, hipStreamNonBlocking, prio ? greatest : 0) != hipSuccess ||
        hipHostMalloc((void **)&dev->h_ndone, 64, 0) != hipSuccess) {
        delete dev;
        return MP_ERR_HIP;
    }
    *out = dev;
    return MP_OK;
}

int mp_hip_load_model_ex(mp_dev *dev, const char *path, int weight_mode) {
    if (!dev || !path) return MP_ERR_ARG;
    if (weight_mode != MP_WEIGHTS_AS_STORED && weight_mode != MP_WEIGHTS_BF16 && weight_mode != MP_WEIGHTS_Q8 &&
        weight_mode != MP_WEIGHTS_F16)
        return fail(dev, MP_ERR_ARG, "unknown weight mode");
    HIPCHK(hipSetDevice(dev->device));
    free_batch(dev);
    dev->loaded = false;
    dev->m.weight_mode = MP_WEIGHTS_AS_STORED;
    // drop the Q8_0 views of a previous model
    if (dev->m.q8_arena) { hipFree(dev->m.q8_arena); dev->m.q8_arena = nullptr; dev->m.q8_bytes = 0; }
    if (dev->m.q8p_arena) { hipFree(dev->m.q8p_arena); dev->m.q8p_arena = nullptr; }
    dev->m.q8_all = false;
    dev->m.lt_in8 = dev->m.lt_qkv8 = dev->m.lt_o8 = dev->m.lt_out8 = mp::QW{};
    dev->m.lt_o8t = nullptr;
    dev->m.pk_lt_in = nullptr;  // set again by an F16 load
    // derived LT weight layouts of a previous model (rebuilt by build_ptab)
    for (void **pp : {(void **)&dev->m.lt_ff2s, (void **)&dev->m.lt_ff1h, (void **)&dev->m.lt_ff2h, (void **)&dev->m.lt_ff2q})
        if (*pp) { hipFree(*pp); *pp = nullptr; }
    if (weight_mode == MP_WEIGHTS_Q8 || weight_mode == MP_WEIGHTS_F16) {  // cheap header check before any upload
        mp::Gguf g;
        std::string err;
        if (!g.open(path, err)) return fail(dev, MP_ERR_IO, err);
        const mp::GgufTensor *t = g.find("decoder.layers.0.self_attention.qkv_net.weight");
        if (weight_mode == MP_WEIGHTS_Q8 && (!t || (t->type != 8 && t->type != 2)))
            return fail(dev, MP_ERR_UNSUPPORTED, "Q8 weight mode needs a GGUF with Q8_0 or Q4_0 tensors");
        // every tensor the F16 mode streams as f16 must be stored F16 (the converter's
        // pattern set, convert_magpie_to_gguf.py:155-176, 311-327)
        if (weight_mode == MP_WEIGHTS_F16)
            for (const auto &kv : g.tensors()) {
                const std::string &n = kv.first;
                const bool proj = n.find(".self_attention.") != std::string::npos ||
                                  n.find(".pos_ff.") != std::string::npos ||
                                  n.find("local_transformer_out_projections.") == 0 ||
                                  n == "local_transformer_in_projection.weight";
                if (proj && n.size() > 7 && n.compare(n.size() - 7, 7, ".weight") == 0 && kv.second.type != 1)
                    return fail(dev, MP_ERR_UNSUPPORTED, "F16 weight mode needs a GGUF with F16 projections (" + n + ")");
            }
    }
    if (int rc = load_model(dev, path)) return rc;
    dev->loaded = false;
    if (weight_mode == MP_WEIGHTS_BF16 || weight_mode == MP_WEIGHTS_F16) {
        if (int rc = pack_weights(dev, weight_mode == MP_WEIGHTS_F16)) return rc;
    } else if (weight_mode == MP_WEIGHTS_Q8) {
        if (int rc = load_q8(dev, path)) return rc;
    }
    dev->m.weight_mode = weight_mode;  // the load-time LT tables depend on it
    if (int rc = build_ptab(dev, weight_mode)) return rc;
    dev->loaded = true;
    return MP_OK;
}

int mp_hip_load_model(mp_dev *dev, const char *path) { return mp_hip_load_model_ex(dev, path, MP_WEIGHTS_AS_STORED); }

int mp_hip_model_info(mp_dev *dev, int *dec_layers, int *enc_layers, size_t *weight_bytes) {
    if (!dev || !dev->loaded) return MP_ERR_STATE;
    if (dec_layers) *dec_layers = dev->m.dec_layers;
    if (enc_layers) *enc_layers = dev->m.enc_layers;
    if (weight_bytes) *weight_bytes = dev->m.arena_bytes;
    return MP_OK;
}

int mp_hip_weight_mode(mp_dev *dev) { return dev && dev->loaded ? dev->m.weight_mode : MP_ERR_STATE; }
int mp_hip_max_batch(mp_dev *dev) {
    if (!dev || !dev->loaded) return MP_ERR_STATE;
    return mp::h16_mode(dev->m.weight_mode) || (dev->m.weight_mode == MP_WEIGHTS_Q8 && dev->m.q8_all) ? 16 : 8;
}

int mp_hip_set_xa_mode(mp_dev *dev, int xa_mode) {
    if (!dev || xa_mode < MP_XA_AUTO || xa_mode > MP_XA_DIRECT) return MP_ERR_ARG;
    dev->xa_mode = xa_mode;
    return MP_OK;
}

int mp_hip_set_kv_mode(mp_dev *dev, int kv_mode) {
    if (!dev || (kv_mode != MP_KV_F32 && kv_mode != MP_KV_BF16)) return MP_ERR_ARG;
    dev->kv_mode = kv_mode;
    return MP_OK;
}

void mp_hip_free(mp_dev *dev) {
    if (!dev) return;
    hipSetDevice(dev->device);
    if (dev->stream) hipStreamSynchronize(dev->stream);
    free_batch(dev);
    if (dev->m.arena) hipFree(dev->m.arena);
    if (dev->m.lt_ptab) hipFree(dev->m.lt_ptab);
    if (dev->m.lt_qkvtab) hipFree(dev->m.lt_qkvtab);
    if (dev->m.lt_votab) hipFree(dev->m.lt_votab);
    if (dev->m.lt_kvo) hipFree(dev->m.lt_kvo);
    if (dev->m.lt_ff2s) hipFree(dev->m.lt_ff2s);
    if (dev->m.lt_ff1h) hipFree(dev->m.lt_ff1h);
    if (dev->m.lt_ff2h) hipFree(dev->m.lt_ff2h);
    if (dev->m.lt_ff2q) hipFree(dev->m.lt_ff2q);
    if (dev->m.pk_arena) hipFree(dev->m.pk_arena);
    if (dev->m.q8_arena) hipFree(dev->m.q8_arena);
    if (dev->m.q8p_arena) hipFree(dev->m.q8p_arena);
    for (void *p : dev->lt_allocs) hipFree(p);
    if (!dev->m.xq_t.empty() && dev->m.xq_t[0]) hipFree(dev->m.xq_t[0]);  // one allocation (load_model)
    if (dev->h_ndone) hipHostFree(dev->h_ndone);
    for (hipEvent_t e : dev->sev)
        if (e) hipEventDestroy(e);
    if (dev->h_codes) hipHostFree(dev->h_codes);
    if (dev->enc_ws) hipFree(dev->enc_ws);
    if (dev->stream_fg) { hipStreamSynchronize(dev->stream_fg); hipStreamDestroy(dev->stream_fg); }
    if (dev->stream) hipStreamDestroy(dev->stream);
    delete dev;
}

const char *mp_hip_error(mp_dev *dev) { return dev ? dev->err.c_str() : "null mp_dev"; }

int mp_hip_begin_batch(mp_dev *dev, const int32_t *tokens, const int32_t *n_tokens, const int32_t *speaker, int B,
                       int tmax, const mp_params *params) {
    if (!dev) return MP_ERR_ARG;
    if (!dev->loaded) return fail(dev, MP_ERR_STATE, "no model loaded");
    const int bmax = mp_hip_max_batch(dev);
    if (!tokens || !n_tokens || !speaker || B < 1 || B > bmax || tmax < 1 || !params)
        return fail(dev, MP_ERR_ARG, "invalid arguments (B must be 1..mp_hip_max_batch: 8 with f32 weights, 16 in the bf16 / F16 / Q8_0 / Q4_0 modes)");
    if (params->temperature >= 0.01f && (params->top_k < 1 || params->top_k > mp::VCB))
        return fail(dev, MP_ERR_ARG, "top_k must be in 1..2024 when sampling");
    int Tmax = 0;
    for (int b = 0; b < B; ++b) {
        if (n_tokens[b] < 1 || n_tokens[b] > tmax) return fail(dev, MP_ERR_ARG, "n_tokens out of range");
        if (speaker[b] < 0 || speaker[b] >= dev->m.n_spk) return fail(dev, MP_ERR_ARG, "speaker id out of range");
        for (int t = 0; t < n_tokens[b]; ++t)
            if (tokens[(size_t)b * tmax + t] < 0 || tokens[(size_t)b * tmax + t] >= dev->m.text_vocab)
                return fail(dev, MP_ERR_ARG, "token id out of range");
        Tmax = std::max(Tmax, (int)n_tokens[b]);
    }
    if (Tmax > mp::TMAX_LIMIT || Tmax > 4096) return fail(dev, MP_ERR_ARG, "too many text tokens");
    const int max_steps = params->max_dec_steps > 0 ? params->max_dec_steps : dev->m.max_dec_steps;
    if (mp::CTX + max_steps + 16 > mp::NCH_MAX * mp::SA_CHUNK)
        return fail(dev, MP_ERR_ARG, "max_dec_steps too large (cache limited to 1024 positions)");
    if (mp::CTX + max_steps > dev->m.dec_pos_rows)
        return fail(dev, MP_ERR_ARG, "max_dec_steps exceeds the decoder position table");
    HIPCHK(hipSetDevice(dev->device));
    const bool trace = params->trace_hidden != 0;
    const bool same = dev->NB > 0 && dev->B == B && dev->Tmax == Tmax && dev->max_steps == max_steps &&
                      (dev->trace != nullptr) == trace && dev->params.ignore_eos == params->ignore_eos &&
                      (dev->params.temperature >= 0.01f) == (params->temperature >= 0.01f) &&
                      dev->params.emit_eos_frame == params->emit_eos_frame &&
                      dev->kv16 == (dev->kv_mode == MP_KV_BF16) && dev->xa_direct == want_xa_direct(dev, Tmax);
    dev->params = *params;
    if (!same) {
        if (int rc = alloc_batch(dev, B, Tmax, max_steps, trace)) return rc;
    }
    const int NB = dev->NB;
    auto t0 = std::chrono::steady_clock::now();
    std::vector<int> h_tok((size_t)NB * Tmax, 0), h_T(NB, 1), h_spk(NB, 0);
    for (int b = 0; b < B; ++b) {
        h_T[b] = n_tokens[b];
        h_spk[b] = speaker[b];
        for (int t = 0; t < n_tokens[b]; ++t) h_tok[(size_t)b * Tmax + t] = tokens[(size_t)b * tmax + t];
    }
    for (int b = B; b < NB; ++b) { h_T[b] = h_T[0]; h_spk[b] = h_spk[0]; }
    HIPCHK(hipMemcpyAsync(dev->tok, h_tok.data(), h_tok.size() * 4, hipMemcpyHostToDevice, dev->stream));
    HIPCHK(hipMemcpyAsync(dev->T, h_T.data(), NB * 4, hipMemcpyHostToDevice, dev->stream));
    HIPCHK(hipMemcpyAsync(dev->spk, h_spk.data(), NB * 4, hipMemcpyHostToDevice, dev->stream));
    {   // sampling settings live on the device: the captured graph serves any of them
        mp::SmpCfg cfg{params->temperature, params->top_k, (unsigned long long)params->seed, params->stream_base};
        HIPCHK(hipMemcpyAsync(dev->smpcfg, &cfg, sizeof cfg, hipMemcpyHostToDevice, dev->stream));
        HIPCHK(hipMemsetAsync(dev->argeos, 0, NB * 4, dev->stream));
    }
    if (int rc = run_preamble(dev)) return rc;
    HIPCHK(hipStreamSynchronize(dev->stream));
    dev->timing = mp_timing{};
    dev->timing.preamble_ms = ms_since(t0);
    dev->batch_ready = true;
    return MP_OK;
}

// magpie_encode_text (magpie.cpp:2284-2374) on its own: the text encoder of one
// utterance into a private device workspace (kept on the mp_dev, grown on demand), the
// output copied to enc_out [n_tokens][768]. A batch in progress is not touched.
int mp_hip_encode_text(mp_dev *dev, const int32_t *tokens, int n_tokens, float *enc_out) {
    if (!dev) return MP_ERR_ARG;
    if (!dev->loaded) return fail(dev, MP_ERR_STATE, "no model loaded");
    if (!tokens || !enc_out || n_tokens < 1) return fail(dev, MP_ERR_ARG, "invalid arguments");
    if (n_tokens > mp::TMAX_LIMIT || n_tokens > 4096) return fail(dev, MP_ERR_ARG, "too many text tokens");
    for (int t = 0; t < n_tokens; ++t)
        if (tokens[t] < 0 || tokens[t] >= dev->m.text_vocab) return fail(dev, MP_ERR_ARG, "token id out of range");
    HIPCHK(hipSetDevice(dev->device));
    const size_t M = (size_t)n_tokens, D = 768;
    const size_t nf = M * D * 4 + M * 3 * D + M * 3072 + enc_gpart_elems(M) + M * D;  // pX pH pATT enc_out | pQKV | pF | gpart
    const size_t need = nf * 4 + 64 + M * 4;  // floats | T (64 B slot) | token ids
    if (dev->enc_ws_bytes < need) {
        // the old workspace may still be read by this stream's earlier encode: wait for it
        // (the stream only, not the device) before it goes
        HIPCHK(hipStreamSynchronize(dev->stream));
        if (dev->enc_ws) hipFree(dev->enc_ws);
        dev->enc_ws = nullptr;
        dev->enc_ws_bytes = 0;
        HIPCHK(hipMalloc(&dev->enc_ws, need));
        dev->enc_ws_bytes = need;
    }
    char *ws = dev->enc_ws;
    float *f = (float *)ws;
    EncWs w{};
    w.NB = 1; w.Tmax = n_tokens;
    w.pX = f; f += M * D; w.pH = f; f += M * D; w.pATT = f; f += M * D; w.enc_out = f; f += M * D;
    w.pQKV = f; f += M * 3 * D; w.pF = f; f += M * 3072; w.gpart = f; f += enc_gpart_elems(M);
    int32_t *ti = (int32_t *)(ws + nf * 4 + 64);
    int32_t *Ti = (int32_t *)(ws + nf * 4);
    w.tok = ti; w.T = Ti;
    HIPCHK(hipMemcpyAsync(ti, tokens, M * 4, hipMemcpyHostToDevice, dev->stream));
    HIPCHK(hipMemcpyAsync(Ti, &n_tokens, 4, hipMemcpyHostToDevice, dev->stream));
    if (int rc = run_encoder(dev, w, dev->stream)) {
        hipStreamSynchronize(dev->stream);  // the host token copies above must land first
        return rc;
    }
    HIPCHK(hipMemcpyAsync(enc_out, w.enc_out, M * D * 4, hipMemcpyDeviceToHost, dev->stream));
    HIPCHK(hipStreamSynchronize(dev->stream));
    return MP_OK;
}

// Per-decode device state: BOS frame at position 110 (magpie.cpp:4243-4318).
int reset_decode_state(mp_dev *dev) {
    const int NB = dev->NB, B = dev->B;
    std::vector<int> h_pos(NB, mp::CTX), h_zero(NB, 0), h_done(NB, 0), h_prev((size_t)NB * 8, dev->m.audio_bos);
    for (int b = B; b < NB; ++b) h_done[b] = 1;
    int h_nd[4] = {NB - B, 0, 0, 0};
    HIPCHK(hipMemcpyAsync(dev->pos, h_pos.data(), NB * 4, hipMemcpyHostToDevice, dev->stream));
    HIPCHK(hipMemcpyAsync(dev->step, h_zero.data(), NB * 4, hipMemcpyHostToDevice, dev->stream));
    HIPCHK(hipMemcpyAsync(dev->nframes, h_zero.data(), NB * 4, hipMemcpyHostToDevice, dev->stream));
    HIPCHK(hipMemcpyAsync(dev->done, h_done.data(), NB * 4, hipMemcpyHostToDevice, dev->stream));
    HIPCHK(hipMemcpyAsync(dev->ndone, h_nd, 16, hipMemcpyHostToDevice, dev->stream));
    HIPCHK(hipMemcpyAsync(dev->codes_prev, h_prev.data(), h_prev.size() * 4, hipMemcpyHostToDevice, dev->stream));
    HIPCHK(hipMemsetAsync(dev->codes_out, 0, (size_t)NB * dev->max_steps * 8 * 4, dev->stream));
    HIPCHK(hipMemsetAsync(dev->argeos, 0, NB * 4, dev->stream));
    // hand-off tags restart with the iteration counter (ndone[1]): no stale tag may match
    HIPCHK(hipMemsetAsync(dev->xh, 0, (size_t)NB * 768 * 8, dev->stream));
    HIPCHK(hipMemsetAsync(dev->qh, 0, (size_t)NB * 3 * 768 * 8, dev->stream));
    HIPCHK(hipMemsetAsync(dev->xqh, 0, (size_t)NB * 128 * 8, dev->stream));
    HIPCHK(hipMemsetAsync(dev->ltgh, 0, (size_t)NB * std::max(mp::LTS_P, mp::LTQ_P) * 256 * 8, dev->stream));
    HIPCHK(hipMemsetAsync(dev->ltfg, 0, mp::LTFG_TOTAL * 8, dev->stream));
    HIPCHK(hipMemsetAsync(dev->ltyg, 0, (size_t)NB * 256 * 8, dev->stream));
    HIPCHK(hipMemsetAsync(dev->sagh, 0, (size_t)NB * mp::NH * mp::SA_SPLITS * mp::SA_PART * 8, dev->stream));
    HIPCHK(hipMemsetAsync(dev->xagh, 0, (size_t)NB * mp::XA_SPLITS * mp::XA_PART * 8, dev->stream));
    HIPCHK(hipMemsetAsync(dev->kgh, 0, (size_t)2 * (768 / 16) * mp::KGH_MAX_KS * 256 * 8, dev->stream));
    // the first frame's decoder input (the BOS codes); later frames' by lt_finalize_kernel
    HIPCHK(mp::op_embed(mp::EmbP{dev->m.audio_emb, dev->codes_prev, dev->m.dec_pos, dev->pos, dev->x}, NB, dev->stream));
    // the host copies are stack/heap temporaries: finish the uploads before they go
    HIPCHK(hipStreamSynchronize(dev->stream));
    return MP_OK;
}


// Capture the iteration graph (or, eager, record the op list) once per batch
// configuration; leaves the decode state reset.
int prepare_iteration(mp_dev *dev) {
    if (eager_mode()) {
        if (dev->ops.empty()) {
            if (int rc = enqueue_iteration(dev, dev->stream, true)) return rc;  // a real first iteration
            HIPCHK(hipStreamSynchronize(dev->stream));
        }
    } else if (!dev->exec) {
        HIPCHK(hipStreamBeginCapture(dev->stream, hipStreamCaptureModeThreadLocal));
        int rc = enqueue_iteration(dev, dev->stream, true);
        hipGraph_t g = nullptr;
        hipError_t e = hipStreamEndCapture(dev->stream, &g);
        if (rc != MP_OK) { if (g) hipGraphDestroy(g); return rc; }
        if (e != hipSuccess) return fail(dev, MP_ERR_HIP, std::string("graph capture failed: ") + hipGetErrorString(e));
        dev->graph = g;
        HIPCHK(hipGraphInstantiate(&dev->exec, dev->graph, nullptr, nullptr, 0));
    }
    return reset_decode_state(dev);
}

int launch_iteration(mp_dev *dev, hipStream_t s = nullptr) {
    if (!s) s = dev->stream;
    if (eager_mode()) return enqueue_iteration(dev, s, false);
    HIPCHK(hipGraphLaunch(dev->exec, s));
    return MP_OK;
}

// An in-launch hand-off that gave up (EPI_RESID_XA's bounded sweep) poisons its
// output and raises ndone[2]: report it instead of returning those codes.
static int check_handoff(mp_dev *dev) {
    int nd[4] = {0, 0, 0, 0};
    HIPCHK(hipMemcpy(nd, dev->ndone, sizeof nd, hipMemcpyDeviceToHost));
    if (nd[2]) {
        std::string what;
        if (nd[2] & mp::HX_ERR_XA) what += " O-projection -> cross-attention";
        if (nd[2] & mp::HX_ERR_SA) what += std::string(what.empty() ? "" : ",") + " QKV -> self-attention";
        if (nd[2] & mp::HX_ERR_LT) what += std::string(what.empty() ? "" : ",") + " LT FFN partial sums";
        if (nd[2] & mp::HX_ERR_KS) what += std::string(what.empty() ? "" : ",") + " split-K partial tiles";
        return fail(dev, MP_ERR_HIP, "in-launch hand-off timed out:" + what);
    }
    return MP_OK;
}

int mp_hip_decode(mp_dev *dev, int32_t *codes_out, int32_t *n_frames) {
    if (!dev) return MP_ERR_ARG;
    if (!dev->batch_ready) return fail(dev, MP_ERR_STATE, "mp_hip_begin_batch must precede mp_hip_decode");
    HIPCHK(hipSetDevice(dev->device));
    const int NB = dev->NB, B = dev->B;
    if (int rc = prepare_iteration(dev)) return rc;
    hipEvent_t e0, e1;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    HIPCHK(hipEventRecord(e0, dev->stream));
    // one graph replay per frame: capturing 4 to 64 iterations per graph measured the same
    // frames/s (2619 vs 2617-2626, tools_dev/graph_iters_ab.py), replay boundaries cost nothing
    const int poll = 8;  // the host checks the done counter every `poll` iterations
    int it = 0;
    while (it < dev->max_steps) {
        if (int rc = launch_iteration(dev)) return rc;
        ++it;
        if (!dev->params.ignore_eos && it % poll == 0 && it < dev->max_steps) {
            HIPCHK(hipMemcpyAsync(dev->h_ndone, dev->ndone, 4, hipMemcpyDeviceToHost, dev->stream));
            HIPCHK(hipStreamSynchronize(dev->stream));
            if (*dev->h_ndone >= NB) break;
        }
    }
    HIPCHK(hipEventRecord(e1, dev->stream));
    HIPCHK(hipEventSynchronize(e1));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1));
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    if (int rc = check_handoff(dev)) return rc;
    std::vector<int> h_nf(NB);
    HIPCHK(hipMemcpy(h_nf.data(), dev->nframes, NB * 4, hipMemcpyDeviceToHost));
    std::vector<int> h_codes((size_t)NB * dev->max_steps * 8);
    HIPCHK(hipMemcpy(h_codes.data(), dev->codes_out, h_codes.size() * 4, hipMemcpyDeviceToHost));
    int total = 0;
    for (int b = 0; b < B; ++b) {
        if (n_frames) n_frames[b] = h_nf[b];
        total += h_nf[b];
    }
    if (codes_out) memcpy(codes_out, h_codes.data(), (size_t)B * dev->max_steps * 8 * 4);
    dev->timing.decode_ms = ms;
    dev->timing.frames_total = total;
    dev->timing.iterations = it;
    return MP_OK;
}

// Streaming frame loop (magpie_synthesize_sentence_streaming's loop,
// magpie.cpp:4762-4838) for every utterance of the batch: after each
// frames_per_chunk iterations the new frames of every utterance are decoded by
// the codec in chunks of frames_per_chunk (the last chunk of an utterance may
// be shorter: EOS or max_dec_steps) and handed to `on_audio` in order.
// Every full chunk of a round goes through the codec in one launch sequence
// (chunks are independent, magpie.cpp:4739-4742: the audio is the same); the
// frames reach the host through a pinned mirror filled on the decode stream.
extern "C" int mp_codec_set_background(mp_codec *c, int cus);  // mp_codec.hip (internal)
// MAGPIE_STREAM_ASYNC=0: queue each chunk from the calling thread (default 1: a helper thread)
static bool stream_async() {
    const char *e = getenv("MAGPIE_STREAM_ASYNC");
    return !(e && atoi(e) == 0);
}
// MAGPIE_STREAM_TRACE=1: host-side timeline of the streaming loop on stderr (diagnostics)
static bool stream_trace() {
    const char *e = getenv("MAGPIE_STREAM_TRACE");
    return e && atoi(e) != 0;
}
// MAGPIE_CODEC_BG_CUS: CUs of the codec's background stream while a decode is in flight
// (default 64 of 256; 0 = the codec's own stream, the whole chip, for every round)
static int codec_bg_cus() {
    const char *e = getenv("MAGPIE_CODEC_BG_CUS");
    return e ? atoi(e) : 0;
}
// codec rounds of at least this many frames go to the background stream while the decode
// continues (throughput: configs[2]'s 16 slots x 32-frame chunks); smaller rounds (a stream's
// 4-frame chunks, whose first chunk is the time to first audio) keep the whole chip
constexpr int CODEC_BG_MIN_FRAMES = 256;

int mp_hip_decode_stream(mp_dev *dev, mp_codec *codec, int frames_per_chunk, mp_audio_cb on_audio, void *user,
                         int32_t *codes_out, int32_t *n_frames, int64_t *total_samples) {
    if (!dev) return MP_ERR_ARG;
    if (!dev->batch_ready) return fail(dev, MP_ERR_STATE, "mp_hip_begin_batch must precede mp_hip_decode_stream");
    if (!codec) return fail(dev, MP_ERR_ARG, "codec is required");
    const int fpc = frames_per_chunk > 0 ? frames_per_chunk : 4;  // default 4 (magpie.h:621)
    HIPCHK(hipSetDevice(dev->device));
    const int NB = dev->NB, B = dev->B, S = dev->max_steps;
    if (int rc = prepare_iteration(dev)) return rc;
    if (!dev->sev[0]) {
        HIPCHK(hipEventCreateWithFlags(&dev->sev[0], hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&dev->sev[1], hipEventDisableTiming));
    }
    // pinned: a copy into pageable memory would block the host until the chunk's kernels finish
    if (dev->h_codes_n < (size_t)NB * S * 8 + 6 * NB) {
        if (dev->h_codes) hipHostFree(dev->h_codes);
        dev->h_codes = nullptr;
        dev->h_codes_n = 0;
        HIPCHK(hipHostMalloc((void **)&dev->h_codes, ((size_t)NB * S * 8 + 6 * NB) * 4, hipHostMallocDefault));
        dev->h_codes_n = (size_t)NB * S * 8 + 6 * NB;
    }
    int *const snap = dev->h_codes + (size_t)NB * S * 8;  // two snapshots of (step, done, nframes)
    auto t0 = std::chrono::steady_clock::now();
    // two snapshots of (step, done, nframes): the host reads one while the next chunk's land in the other
    std::vector<int> delivered(B, 0), stopped(B, 0), ended(B, 0);
    std::vector<int32_t> cbm;
    std::vector<float> audio;
    int64_t samples = 0;
    int it = 0;
    bool first = true;
    dev->timing = mp_timing{dev->timing.preamble_ms, 0.0, 0, 0, 0.0};
    // the stream the last chunk was queued on (the stop writes below follow it)
    hipStream_t cur = dev->stream;
    auto enqueue_chunk = [&](int slot, hipStream_t st) -> int {
        const int n_it = std::min(fpc, S - it);
        for (int i = 0; i < n_it; ++i)
            if (int rc = launch_iteration(dev, st)) return rc;
        // the frames these iterations wrote (columns it..it+n_it of every slot) to the
        // pinned mirror, on the decode stream: no host copy waits on the GPU later
        HIPCHK(hipMemcpy2DAsync(dev->h_codes + (size_t)it * 8, (size_t)S * 32, dev->codes_out + (size_t)it * 8,
                                (size_t)S * 32, (size_t)n_it * 32, NB, hipMemcpyDeviceToHost, st));
        it += n_it;
        int *h = snap + (size_t)slot * 3 * NB;
        HIPCHK(hipMemcpyAsync(h, dev->step, NB * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipMemcpyAsync(h + NB, dev->done, NB * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipMemcpyAsync(h + 2 * NB, dev->nframes, NB * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipEventRecord(dev->sev[slot], st));
        return MP_OK;
    };
    // rounds whose codec runs in the background: the decode on the complementary CUs. Every
    // chunk is queued after the previous one landed (the host waited for its event), so
    // moving between the two streams needs no other ordering.
    const int bg_cus = codec_bg_cus();
    const bool split_cus = B * fpc >= CODEC_BG_MIN_FRAMES && bg_cus > 0 && stream_async();
    if (split_cus && (!dev->stream_fg || dev->stream_fg_cus != bg_cus)) {
        if (dev->stream_fg) { HIPCHK(hipStreamSynchronize(dev->stream_fg)); hipStreamDestroy(dev->stream_fg); dev->stream_fg = nullptr; }
        int ncu = 0, least = 0, greatest = 0;
        HIPCHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev->device));
        HIPCHK(hipDeviceGetStreamPriorityRange(&least, &greatest));
        const std::vector<uint32_t> mask = mp::cu_share_mask(ncu, bg_cus, true);
        HIPCHK(hipExtStreamCreateWithCUMask(&dev->stream_fg, (uint32_t)mask.size(), mask.data()));
        dev->stream_fg_cus = bg_cus;
    }
    struct Job { int b, f0, n; };
    std::vector<Job> jobs;
    int slot = 0;
    if (int rc = enqueue_chunk(0, dev->stream)) return rc;
    for (;;) {
        HIPCHK(hipEventSynchronize(dev->sev[slot]));
        const int *h_step = snap + (size_t)slot * 3 * NB, *h_done = h_step + NB, *h_nf = h_step + 2 * NB;
        bool more = false;
        for (int b = 0; b < B; ++b) more |= !(h_done[b] != 0 || stopped[b]);
        more &= it < S;
        // the next chunk's iterations are queued before this round's codec work, so
        // the decode runs on its stream while the codec runs on the codec's (bit-exact
        // beside it: tests/test_concurrency_gpu.py); a stop requested by a callback
        // below takes effect after that chunk, whose frames are then not delivered.
        // Queuing a chunk's graph replays can block the host (the queue's packet slots fill
        // up: 32 iterations of 65 launches), which left the codec waiting behind the next
        // chunk's decode, serialising the two (configs[2]: 27.2k vs 27.5k frames/s serial,
        // r06d): a round with codec work large enough to matter queues the chunk from a
        // helper thread while this thread runs the codec (HIP calls are thread-safe; the
        // helper touches only the decode stream and its pinned snapshot)
        const double t_wait = ms_since(t0);
        std::future<int> queued;
        const bool async_q = more && stream_async() && B * fpc >= CODEC_BG_MIN_FRAMES;  // (a thread per round)
        if (more) {
            cur = async_q && split_cus ? dev->stream_fg : dev->stream;
            if (async_q) queued = std::async(std::launch::async, [&, sl = slot ^ 1, st = cur]() { return enqueue_chunk(sl, st); });
            else if (int rc = enqueue_chunk(slot ^ 1, cur)) return rc;
        }
        if (stream_trace()) fprintf(stderr, "[stream] round at %.3f ms: chunk landed, next queued %s at %.3f ms\n", t_wait,
                                    async_q ? "(async)" : "", ms_since(t0));
        // this round's chunks, utterance by utterance, in delivery order
        jobs.clear();
        for (int b = 0; b < B; ++b) {
            if (stopped[b]) continue;
            const bool done = h_done[b] != 0;
            const int produced = done ? h_nf[b] : h_step[b];
            for (int d = delivered[b]; produced - d >= (done ? 1 : fpc);) {
                const int n = std::min(fpc, produced - d);
                jobs.push_back({b, d, n});
                d += n;
            }
        }
        // full chunks through the codec together, a shorter final chunk on its own
        size_t nfull = 0;
        for (const Job &j : jobs) nfull += j.n == fpc;
        cbm.assign(jobs.size() * 8 * fpc, 0);
        audio.resize(jobs.size() * fpc * 1024);
        std::vector<size_t> at(jobs.size());
        {
            size_t kf = 0, ks = nfull;
            for (size_t q = 0; q < jobs.size(); ++q) at[q] = jobs[q].n == fpc ? kf++ : ks++;
        }
        for (size_t q = 0; q < jobs.size(); ++q) {
            const Job &j = jobs[q];
            const int32_t *fm = dev->h_codes + ((size_t)j.b * S + j.f0) * 8;
            int32_t *dst = cbm.data() + at[q] * 8 * fpc;
            for (int t = 0; t < j.n; ++t)  // frame-major -> codebook-major (decode_frames_to_audio, 4468-4473)
                for (int c = 0; c < 8; ++c) dst[(size_t)c * j.n + t] = fm[(size_t)t * 8 + c];
        }
        if (nfull) {
            // beside a decode still in flight, large rounds run on the codec's CU-masked
            // background stream: the frame loop keeps most of the chip (with the whole chip the
            // codec's long workgroups held the CUs the decode's next launches waited for, and
            // overlapping bought nothing: 27.2k vs 27.5k frames/s serial, round 6 r06c)
            const int bg = more && (int)nfull * fpc >= CODEC_BG_MIN_FRAMES ? codec_bg_cus() : 0;
            if (int rc = mp_codec_set_background(codec, bg)) return fail(dev, rc, "codec background stream");
            const int rc = mp_hip_codec_decode_chunks(codec, cbm.data(), (int)nfull, fpc, audio.data());
            mp_codec_set_background(codec, 0);
            if (rc) return fail(dev, rc, std::string("codec: ") + mp_hip_codec_error(codec));
        }
        for (size_t q = 0; q < jobs.size(); ++q)
            if (jobs[q].n != fpc)
                if (int rc = mp_hip_codec_decode(codec, cbm.data() + at[q] * 8 * fpc, jobs[q].n,
                                                 audio.data() + at[q] * fpc * 1024))
                    return fail(dev, rc, std::string("codec: ") + mp_hip_codec_error(codec));
        if (stream_trace()) fprintf(stderr, "[stream]   codec of %zu chunks done at %.3f ms\n", jobs.size(), ms_since(t0));
        if (queued.valid())
            if (int rc = queued.get()) return rc;
        for (size_t q = 0, b = 0; b < (size_t)B; ++b) {
            for (; q < jobs.size() && jobs[q].b == (int)b; ++q) {
                const Job &j = jobs[q];
                if (stopped[b]) continue;  // a callback of this round stopped the utterance
                delivered[b] += j.n;
                samples += (int64_t)j.n * 1024;
                if (first) {
                    dev->timing.first_audio_ms = ms_since(t0);
                    first = false;
                }
                if (on_audio && !on_audio((int)b, audio.data() + at[q] * fpc * 1024, j.n * 1024, user)) {
                    // the callback asked to stop (4820-4824): the utterance ends here
                    stopped[b] = 1;
                    const int one = 1;
                    HIPCHK(hipMemcpyAsync(dev->done + b, &one, 4, hipMemcpyHostToDevice, cur));
                    HIPCHK(hipStreamSynchronize(cur));
                }
            }
            if ((h_done[b] != 0 || stopped[b]) && !ended[b]) {  // end-of-utterance notice: (utt, NULL, 0)
                ended[b] = 1;
                if (on_audio) on_audio((int)b, nullptr, 0, user);
            }
        }
        if (!more) break;
        slot ^= 1;
    }
    HIPCHK(hipStreamSynchronize(dev->stream));
    if (dev->stream_fg) HIPCHK(hipStreamSynchronize(dev->stream_fg));
    if (int rc = check_handoff(dev)) return rc;
    dev->timing.decode_ms = ms_since(t0);
    dev->timing.iterations = it;
    int total = 0;
    for (int b = 0; b < B; ++b) {
        if (n_frames) n_frames[b] = delivered[b];
        total += delivered[b];
    }
    dev->timing.frames_total = total;
    if (codes_out) HIPCHK(hipMemcpy(codes_out, dev->codes_out, (size_t)B * S * 8 * 4, hipMemcpyDeviceToHost));
    if (total_samples) *total_samples = samples;
    return MP_OK;
}

int mp_hip_lt_sample(mp_dev *dev, const float *hidden, float temperature, int top_k, int forbid_eos, uint64_t seed,
                     int32_t *sampled, int32_t *argmax) {
    if (!dev || !hidden || !sampled || !argmax) return MP_ERR_ARG;
    if (!dev->loaded) return fail(dev, MP_ERR_STATE, "no model loaded");
    if (temperature >= 0.01f && (top_k < 1 || top_k > mp::VCB)) return fail(dev, MP_ERR_ARG, "top_k must be in 1..2024");
    HIPCHK(hipSetDevice(dev->device));
    mp::LtIo &io = dev->lt_io;
    if (dev->lt_allocs.empty()) {
        auto al = [&](auto **p, size_t n) -> int {
            void *v = nullptr;
            HIPCHK(hipMalloc(&v, n * 4 + 256));
            HIPCHK(hipMemset(v, 0, n * 4 + 256));
            dev->lt_allocs.push_back(v);
            *p = (std::remove_reference_t<decltype(**p)> *)v;
            return MP_OK;
        };
        int rc = MP_OK;
        if ((rc = al(&io.hidden, 768)) || (rc = al(&io.lt_s, 9 * 256)) || (rc = al(&io.ltX, 256)) ||
            (rc = al(&io.ltY, 256)) || (rc = al(&io.lty2, 256)) || (rc = al(&io.ltq, 256)) ||
            (rc = al(&io.ltk, 8 * 256)) || (rc = al(&io.ltv, 8 * 256)) || (rc = al(&io.ltf, 1024)) || (rc = al(&io.ltp, std::max({mp::LT_FFN_P, mp::LTS_P, mp::LTQ_P}) * 256)) ||

            (rc = al(&io.logits, 2024)) || (rc = al(&io.codes_cur, 8)) || (rc = al(&io.step, 1)) ||
            (rc = al(&io.done, 1)) || (rc = al(&io.argeos, 1)) || (rc = al(&io.amax, 8)) || (rc = al(&io.cfg, 8)))
            return rc;
        io.lt_only = 1;
        io.max_steps = 1;
    }
    io.sampling = temperature >= 0.01f;
    io.ignore_eos = forbid_eos != 0;
    // step: a call counter >= 4 (so only forbid_eos masks EOS), also the draw's step index
    const int step = 4 + dev->lt_calls++;
    mp::SmpCfg cfg{temperature, top_k, (unsigned long long)seed, -1};
    HIPCHK(hipMemcpyAsync(io.hidden, hidden, 768 * 4, hipMemcpyHostToDevice, dev->stream));
    HIPCHK(hipMemcpyAsync(io.step, &step, 4, hipMemcpyHostToDevice, dev->stream));
    HIPCHK(hipMemcpyAsync(io.cfg, &cfg, sizeof cfg, hipMemcpyHostToDevice, dev->stream));
    HIPCHK(hipMemsetAsync(io.argeos, 0, 4, dev->stream));
    if (int rc = enqueue_lt(dev, io, 1, dev->stream, nullptr)) return rc;
    HIPCHK(hipMemcpyAsync(sampled, io.codes_cur, 32, hipMemcpyDeviceToHost, dev->stream));
    HIPCHK(hipMemcpyAsync(argmax, io.amax, 32, hipMemcpyDeviceToHost, dev->stream));
    HIPCHK(hipStreamSynchronize(dev->stream));
    return MP_OK;
}

int mp_hip_get_trace(mp_dev *dev, float *hidden) {
    if (!dev || !hidden) return MP_ERR_ARG;
    if (!dev->trace) return fail(dev, MP_ERR_STATE, "trace_hidden was not enabled");
    HIPCHK(hipMemcpy(hidden, dev->trace, (size_t)dev->B * (dev->max_steps + 1) * 768 * 4, hipMemcpyDeviceToHost));
    return MP_OK;
}

int64_t mp_hip_debug_buffer(mp_dev *dev, const char *name, void *host, int64_t bytes) {
    if (!dev || !name || bytes < 0) return MP_ERR_ARG;
    if (!dev->batch_ready) return fail(dev, MP_ERR_STATE, "no batch");
    const size_t NB = dev->NB, L = dev->m.dec_layers, T = dev->Tmax, S = dev->max_seq;
    const std::string n(name);
    const void *src = nullptr;
    size_t sz = 0;
    if (n == "enc_out") { src = dev->enc_out; sz = NB * T * 768 * 4; }
    else if (n == "xak") { src = dev->xak; sz = NB * L * T * 128 * 4; }
    else if (n == "xav") { src = dev->xav; sz = NB * L * T * 128 * 4; }
    else if (n == "kc") { src = dev->kc; sz = NB * L * S * 768 * (dev->kv16 ? 2 : 4); }
    else if (n == "vc") { src = dev->vc; sz = NB * L * S * 768 * (dev->kv16 ? 2 : 4); }
    else if (n == "x") { src = dev->x; sz = NB * 768 * 4; }
    else if (n == "q8dump" && dev->q8dump) { src = dev->q8dump; sz = dev->q8dump_slot * dev->q8dump_n; }
    else if (n == "q8dump_index" && dev->q8dump) {
        sz = dev->q8dump_index.size() * 4;
        if (host) memcpy(host, dev->q8dump_index.data(), std::min<size_t>(sz, (size_t)bytes));
        return (int64_t)sz;
    }
    else return fail(dev, MP_ERR_ARG, "unknown buffer " + n);
    if (host) {
        HIPCHK(hipSetDevice(dev->device));
        HIPCHK(hipStreamSynchronize(dev->stream));
        HIPCHK(hipMemcpy(host, src, std::min<size_t>(sz, (size_t)bytes), hipMemcpyDeviceToHost));
    }
    return (int64_t)sz;
}

int mp_hip_get_timing(mp_dev *dev, mp_timing *t) {
    if (!dev || !t) return MP_ERR_ARG;
    *t = dev->timing;
    return MP_OK;
}

int mp_hip_num_ops(mp_dev *dev) { return dev ? (int)dev->ops.size() : 0; }

const char *mp_hip_op_name(mp_dev *dev, int op) {
    if (!dev || op < 0 || op >= (int)dev->ops.size()) return "";
    return dev->ops[op].name.c_str();
}

double mp_hip_op_bytes(mp_dev *dev, int op) {
    if (!dev || op < 0 || op >= (int)dev->ops.size()) return -1.0;
    const mp::OpRec &r = dev->ops[op];
    if (r.kind == mp::K_ATTN || r.add_sa) {
        // live cache length of slot 0 after the run: keys 0..pos
        int pos = 0;
        hipMemcpy(&pos, dev->pos, 4, hipMemcpyDeviceToHost);
        // K, V rows (+ q in, unless handed over in-launch) + the split states out
        const double kvb = dev->kv16 ? 2.0 : 4.0;
        return (r.add_sa ? r.bytes : 4.0 * dev->NB * 768) +
               dev->NB * ((double)(pos + 1) * 768 * 2 * kvb + 4.0 * mp::NH * mp::SA_SPLITS * mp::SA_PART);
    }
    return r.bytes;
}

// one recorded op, launched on s (profiling and standalone timing)
static hipError_t launch_rec(const mp::OpRec &r, hipStream_t s) {
    switch (r.kind) {
    case mp::K_GEMV: return r.fn(r.g, s);
    case mp::K_ATTN: return mp::op_sa_attn(r.a, r.B, s);
    case mp::K_XA: return mp::op_xa(r.x, r.B, s);
    case mp::K_XAQ8: return mp::op_xa_q8(r.xq, r.B, s);
    case mp::K_LTFFN: return mp::op_lt_ffn(r.lf, r.B, s);
    case mp::K_LTMERGE: return mp::op_lt_merge(r.lf, r.B, s);
    case mp::K_LTPICK: return mp::op_lt_pick(r.g, r.B, s);
    case mp::K_LTFFN2: return mp::op_lt_ffn2(r.l2, r.B, s);
    case mp::K_LTSLOT: return mp::op_lt_slot(r.l2, r.B, s);
    case mp::K_LTFRONT: return mp::op_lt_front(r.lf3, s);
    case mp::K_LTALL: return mp::op_lt_all(r.la, s);
    case mp::K_LTSLOTQ8: return mp::op_lt_slot_q8(r.lq8, r.B, s);
    case mp::K_LTKVO: return mp::op_lt_kvo(r.g, r.B, s);
    case mp::K_EMBED: return mp::op_embed(r.e, r.B, s);
    case mp::K_FIN: return mp::op_finalize(r.f, r.B, s);
    }
    return hipErrorInvalidValue;
}

int mp_hip_profile_ops(mp_dev *dev, int iters, float *avg_us) { return mp_hip_profile_ops_ex(dev, iters, avg_us, nullptr); }

int mp_hip_profile_ops_ex(mp_dev *dev, int iters, float *avg_us, float *pair_us) {
    if (!dev || !avg_us || iters < 1) return MP_ERR_ARG;
    if (!dev->batch_ready || dev->ops.empty())
        return fail(dev, MP_ERR_STATE, "mp_hip_profile_ops needs a decoded batch (mp_hip_decode first)");
    HIPCHK(hipSetDevice(dev->device));
    const int n = (int)dev->ops.size();
    std::vector<hipEvent_t> ev(3 * (size_t)n);  // [before, after, after + an empty pair's second event]
    for (auto &e : ev) HIPCHK(hipEventCreate(&e));
    std::vector<double> sum(n, 0.0), psum(n, 0.0);
    int rc = MP_OK;
    for (int it = 0; it < iters && rc == MP_OK; ++it) {
        for (int i = 0; i < n; ++i) {
            const mp::OpRec &r = dev->ops[i];
            HIPCHK(hipEventRecord(ev[3 * i], dev->stream));
            const hipError_t e = launch_rec(r, dev->stream);
            HIPCHK(e);
            HIPCHK(hipEventRecord(ev[3 * i + 1], dev->stream));
            if (pair_us) HIPCHK(hipEventRecord(ev[3 * i + 2], dev->stream));
        }
        HIPCHK(hipStreamSynchronize(dev->stream));
        for (int i = 0; i < n; ++i) {
            float ms = 0.f;
            HIPCHK(hipEventElapsedTime(&ms, ev[3 * i], ev[3 * i + 1]));
            sum[i] += ms;
            if (pair_us) {
                HIPCHK(hipEventElapsedTime(&ms, ev[3 * i + 1], ev[3 * i + 2]));
                psum[i] += ms;
            }
        }
    }
    for (auto &e : ev) hipEventDestroy(e);
    for (int i = 0; i < n; ++i) avg_us[i] = (float)(sum[i] * 1000.0 / iters);
    if (pair_us)
        for (int i = 0; i < n; ++i) pair_us[i] = (float)(psum[i] * 1000.0 / iters);
    return rc;
}

int mp_hip_profile_ops_ts(mp_dev *dev, int iters, float *avg_us) {
    if (!dev || !avg_us || iters < 1) return MP_ERR_ARG;
    if (!dev->batch_ready || dev->ops.empty())
        return fail(dev, MP_ERR_STATE, "mp_hip_profile_ops_ts needs a decoded batch (mp_hip_decode first)");
    HIPCHK(hipSetDevice(dev->device));
    const int n = (int)dev->ops.size();
    const size_t per = (size_t)2 * TS_BLOCKS * TS_WAVES;  // u64 per op
    unsigned long long *ts = nullptr;
    HIPCHK(hipMalloc(&ts, (size_t)n * per * 8));
    std::vector<unsigned long long> h((size_t)n * per);
    std::vector<double> sum(n, 0.0);
    std::vector<int> cnt(n, 0);
    int rc = MP_OK;
    for (int it = 0; it < iters && rc == MP_OK; ++it) {
        HIPCHK(hipMemsetAsync(ts, 0, (size_t)n * per * 8, dev->stream));
        for (int i = 0; i < n; ++i) {
            mp::OpRec r = dev->ops[i];
            unsigned long long *t = ts + (size_t)i * per;
            r.g.ts = t; r.a.ts = t; r.x.ts = t; r.f.ts = t; r.lf.ts = t; r.l2.f.ts = t; r.lf3.l.f.ts = t; r.lq8.ts = t;
            const hipError_t e = launch_rec(r, dev->stream);
            if (e != hipSuccess) { rc = fail(dev, MP_ERR_HIP, std::string("profile launch: ") + hipGetErrorString(e)); break; }
        }
        if (rc != MP_OK) break;
        HIPCHK(hipMemcpyAsync(h.data(), ts, (size_t)n * per * 8, hipMemcpyDeviceToHost, dev->stream));
        HIPCHK(hipStreamSynchronize(dev->stream));
        if (const char *dump = getenv("MAGPIE_TS_DUMP")) {  // raw stamps of the last iteration (diagnostics)
            if (FILE *fp = fopen(dump, "wb")) { fwrite(h.data(), 8, h.size(), fp); fclose(fp); }
        }
        for (int i = 0; i < n; ++i) {
            unsigned long long t0 = ~0ull, t1 = 0;
            for (size_t k = 0; k < per / 2; ++k) {
                const unsigned long long a = h[(size_t)i * per + 2 * k], b = h[(size_t)i * per + 2 * k + 1];
                if (b == 0) continue;  // slot not written
                t0 = std::min(t0, a);
                t1 = std::max(t1, b);
            }
            if (t1 > t0 && t0 != ~0ull) { sum[i] += (double)(t1 - t0); ++cnt[i]; }
        }
    }
    hipFree(ts);
    // s_memrealtime counts at 100 MHz: 10 ns per tick; -1 for ops without timestamps
    for (int i = 0; i < n; ++i) avg_us[i] = cnt[i] ? (float)(sum[i] / cnt[i] * 0.01) : -1.f;
    return rc;
}

// Empty dispatches bracketing mp_hip_profile_ops_kev's launches, so that a
// rocprofv3 kernel trace of the same command can be cut to exactly those launches
// (tools_dev/prof_phase.py) and compared with the events' figures.
__global__ void profile_mark_kernel() {}

int mp_hip_profile_ops_kev(mp_dev *dev, int iters, float *avg_us) {
    if (!dev || !avg_us || iters < 1) return MP_ERR_ARG;
    if (!dev->batch_ready || dev->ops.empty())
        return fail(dev, MP_ERR_STATE, "mp_hip_profile_ops_kev needs a decoded batch (mp_hip_decode first)");
    HIPCHK(hipSetDevice(dev->device));
    const int n = (int)dev->ops.size();
    std::vector<hipEvent_t> ev(2 * (size_t)n);
    for (auto &e : ev) HIPCHK(hipEventCreate(&e));
    std::vector<double> sum(n, 0.0);
    int rc = MP_OK;
    hipLaunchKernelGGL(profile_mark_kernel, dim3(1), dim3(64), 0, dev->stream);
    for (int it = 0; it < iters && rc == MP_OK; ++it) {
        for (int i = 0; i < n && rc == MP_OK; ++i) {
            mp::g_kev[0] = ev[2 * i];
            mp::g_kev[1] = ev[2 * i + 1];
            const hipError_t e = launch_rec(dev->ops[i], dev->stream);
            mp::g_kev[0] = mp::g_kev[1] = nullptr;
            if (e != hipSuccess) rc = fail(dev, MP_ERR_HIP, std::string("profile launch: ") + hipGetErrorString(e));
        }
        if (rc != MP_OK) break;
        HIPCHK(hipStreamSynchronize(dev->stream));
        for (int i = 0; i < n; ++i) {
            float ms = 0.f;
            HIPCHK(hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]));
            sum[i] += ms;
        }
    }
    hipLaunchKernelGGL(profile_mark_kernel, dim3(1), dim3(64), 0, dev->stream);
    HIPCHK(hipStreamSynchronize(dev->stream));
    for (auto &e : ev) hipEventDestroy(e);
    for (int i = 0; i < n; ++i) avg_us[i] = (float)(sum[i] * 1000.0 / iters);
    return rc;
}

int mp_hip_time_op(mp_dev *dev, int op, int reps, float *avg_us) {
    if (!dev || !avg_us || reps < 1 || op < 0 || op >= (int)dev->ops.size()) return MP_ERR_ARG;
    HIPCHK(hipSetDevice(dev->device));
    mp::OpRec r = dev->ops[op];
    r.g.ndone = nullptr;
    r.g.trace = nullptr;
    // XA rewrites this layer's split states only; XA-Q8 rewrites x2 with the same values
    auto launch = [&]() -> hipError_t { return launch_rec(r, dev->stream); };
    if (r.kind == mp::K_FIN) return fail(dev, MP_ERR_ARG, "op cannot be timed standalone");
    // an op carrying an in-launch hand-off (QKV -> SA, O-projection -> XA) tags it with the
    // iteration counter: relaunched with the same tag, its consumers would find the previous
    // launch's granules and not wait for their producers (a different, shorter critical path)
    const bool handoff = (r.kind == mp::K_GEMV && r.g.iter) || (r.kind == mp::K_LTSLOT && r.l2.gh) ||
                         r.kind == mp::K_LTFRONT || r.kind == mp::K_LTALL || r.kind == mp::K_LTSLOTQ8 ||
                         (r.kind == mp::K_ATTN && r.a.gh);
    if (handoff)
        return fail(dev, MP_ERR_ARG, "op carries an in-launch hand-off: back-to-back timing would not wait for it");
    HIPCHK(launch());  // warm
    hipEvent_t e0, e1;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    HIPCHK(hipEventRecord(e0, dev->stream));
    for (int i = 0; i < reps; ++i) HIPCHK(launch());
    HIPCHK(hipEventRecord(e1, dev->stream));
    HIPCHK(hipEventSynchronize(e1));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1));
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    *avg_us = ms * 1000.f / reps;
    return MP_OK;
}

}  // extern "C"
