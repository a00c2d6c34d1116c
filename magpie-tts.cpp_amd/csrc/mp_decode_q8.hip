// Q8_0 weight mode of the decode projections (gfx950) on int8 MFMA, batch NB <= 16.
//
// The reference's Q8 GGUF stores the attention / cross-attention / LT
// projections as Q8_0 blocks (scripts/convert_magpie_to_gguf.py:155-176: per 32
// weights an fp16 scale d and 32 int8 q) and ggml multiplies them with its
// quantised mul_mat: the activation row is itself quantised to Q8_0
// (quantize_row_q8_0_ref: d = amax/127, id = 1/d, q = roundf(x*id), d kept as
// fp16) and every block contributes its exact integer dot times d_w * d_a
// (ggml_vec_dot_q8_0_q8_0). This file computes exactly that per
// decode step as a skinny GEMM on v_mfma_i32_16x16x32_i8:
//
//  * one MFMA = one Q8_0 block: A = 16 weight rows x 32 int8 (the block), B =
//    32 int8 x 16 utterance columns (columns >= NB read a zero row), D = the 256
//    exact int32 block dots; the block scales are applied in f32 as the
//    accumulator is updated (acc += (float)sumi * (d_w * d_a)), so the int8 ->
//    real dequantisation is fused into the MFMA loop and no weight is ever
//    widened in memory;
//  * weights stay int8 in HBM (34/32 B per param as in the file), repacked once
//    at load into fragment order [N/16][K/64][64 lanes][16 B] (lane l: row l&15,
//    8 bytes of block 2j and 8 of block 2j+1 at k-offset 8(l>>4)): every
//    wave-instruction of the weight stream is one contiguous 1 KiB
//    global_load_dwordx4; the scales likewise [N/16][K/64][4][2 blocks x 4 rows]
//    fp16, one 16-byte load per lane per two blocks;
//  * the prologue (LN / frame embedding / LT pick + gather / LT attention,
//    shared with the f32 and 16-bit families, mp_fused.hpp) builds the f32
//    activation rows in LDS, then 4 lanes per block quantise them to Q8_0 in LDS;
//  * a workgroup owns one 16-row tile, its 4 waves split K and reduce in LDS in a
//    fixed order: every output's arithmetic is independent of NB, so a batch
//    reproduces its utterances run alone bit for bit.
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <math.h>

#include <type_traits>

#include "mp_device.hpp"
#include "mp_fused.hpp"
#include "mp_params.hpp"
#include "mp_sa.hpp"
#include "mp_xa.hpp"

namespace mp {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef int intx4 __attribute__((ext_vector_type(4)));

// max over the 4 lanes of a DPP quad
__device__ __forceinline__ float quad_max(float v) {
    v = fmaxf(v, dpp_mov<0xB1>(v));
    return fmaxf(v, dpp_mov<0x4E>(v));
}

__device__ __forceinline__ void xq8_tail(const GemvP &p, float *act, signed char *actq, float *actd, unsigned long long t_start);
__device__ __forceinline__ void xq8a_tail(const GemvP &p, unsigned long long t_start);
__device__ __forceinline__ void xq8qa_tail(const GemvP &p, float *act, signed char *actq, float *actd,
                                           unsigned long long t_start);
constexpr int XQG = 8;  // q_net workgroups per slot in EPI_RESID_XQ8 (16 rows each)

template <int NB, int K, int PRO, int EPI, bool Q4>
__global__ __launch_bounds__(MP_BLOCK) void gemm_q8_kernel_dec(GemvP p) {
    const unsigned long long t_start = ts_begin(p.ts);
    static_assert(NB >= 1 && NB <= 16, "one 16-column MFMA tile of utterances");
    static_assert(K % 256 == 0, "K splits into 4 waves x 64-wide block pairs");
    constexpr int KP = K / 64, KW = KP / MP_NWAVES, NBLK = K / 32;
    constexpr int QS = K + 16;  // padded int8 row: the 16 column rows spread over the banks
    constexpr int SC = pro_scratch<NB, PRO>();
    __shared__ __attribute__((aligned(16))) float act[NB * K];
    __shared__ __attribute__((aligned(16))) signed char actq[(NB + 1) * QS];
    __shared__ float actd[(NB + 1) * NBLK];
    __shared__ int actsum[Q4 ? (NB + 1) * NBLK : 1];  // Q4: each activation block's integer sum
    __shared__ __attribute__((aligned(16))) floatx4 part[MP_NWAVES][64];
    __shared__ float red[8];
    __shared__ float sc[SC];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, rt = blockIdx.x;
    if constexpr (EPI == EPI_QKV_SA) {
        // the launch's last NH x SA_SPLITS x NB workgroups: self-attention on this launch's q|k|v
        if (rt >= p.nrow_blocks) {
            sa_tail(p, t_start);
            return;
        }
    }
    if constexpr (EPI == EPI_RESID_XQ8) {
        // then XQG x NB workgroups: the XA's q_net on this launch's x1; then XQ8A x NB:
        // the XA's attention + o_net on that q
        if (NB <= XQ8_QIN_NB && rt >= p.nrow_blocks && p.xq8.qin) {
            xq8qa_tail(p, act, actq, actd, t_start);
            return;
        }
        if (rt >= p.nrow_blocks + XQG * NB) {
            xq8a_tail(p, t_start);
            return;
        }
        if (rt >= p.nrow_blocks) {
            xq8_tail(p, act, actq, actd, t_start);
            return;
        }
    }

    // this wave's weight fragments and their scales, issued before the prologue
    // (Q4: 8 nibbles per block and lane, half the bytes: the Q4_0 file's 18 per 32)
    // (the PreRows prologues' loads go first: vector loads complete in issue order)
    constexpr bool PRE = PreRows<NB, K, PRO>::ON;
    PreRows<NB, K, PRO> pre;
    if constexpr (PRE) {
        pre_load<NB, K, PRO>(p, pre);
        __builtin_amdgcn_sched_barrier(0);
    }
    using AT = typename std::conditional<Q4, uint2, uint4>::type;
    const AT *wf = (const AT *)p.Wq + ((size_t)rt * KP + w * KW) * 64 + lane + ts_dep(t_start);
    const uint4 *sf = (const uint4 *)p.Wd + ((size_t)rt * KP + w * KW) * 4 + (lane >> 4);
    AT a[KW];
    uint4 sd[KW];
#pragma unroll
    for (int i = 0; i < KW; ++i) { a[i] = ld_weight(wf + (size_t)i * 64); sd[i] = ld_weight(sf + (size_t)i * 4); }
    // the epilogue's operand of this thread's output (row tid/16, column tid%16), behind the weights
    constexpr int EOP = EPI == EPI_RESID_XQ8 ? EPI_RESID_XA : EPI;
    float eop = 0.f;
    if constexpr (epi_has_operand<EOP>()) {
        const int cq = tid & 15, nq = rt * 16 + (tid >> 4);
        if (cq < NB && nq < p.N) eop = epi_operand<EOP>(p, nq, cq);
    }
    if constexpr (PRE) {
        __builtin_amdgcn_sched_barrier(0);
        pre_finish<NB, K, PRO>(p, pre, act, sc);
    } else {
        if constexpr (epi_has_operand<EOP>()) __builtin_amdgcn_sched_barrier(0);
        prologue<NB, K, PRO>(p, act, red, sc);
    }

    // activation rows -> Q8_0 (quantize_row_q8_0_ref), 4 lanes x 8 elements per block;
    // row NB is zero (q = 0, d = 0) and feeds MFMA columns NB..15
    for (int e = tid; e < (QS + 4 * NBLK) / 4; e += MP_BLOCK) {
        if (e < QS / 4) ((int *)(actq + NB * QS))[e] = 0;
        else actd[NB * NBLK + (e - QS / 4)] = 0.f;
    }
    if constexpr (Q4)
        for (int e = tid; e < NBLK; e += MP_BLOCK) actsum[NB * NBLK + e] = 0;
    for (int blk = (tid >> 2); blk < NB * NBLK; blk += MP_BLOCK / 4) {
        const int b = blk / NBLK, kb = blk % NBLK, e8 = 8 * (lane & 3);
        const float4 x0 = *(const float4 *)(act + b * K + kb * 32 + e8);
        const float4 x1 = *(const float4 *)(act + b * K + kb * 32 + e8 + 4);
        float am = fmaxf(fmaxf(fmaxf(fabsf(x0.x), fabsf(x0.y)), fmaxf(fabsf(x0.z), fabsf(x0.w))),
                         fmaxf(fmaxf(fabsf(x1.x), fabsf(x1.y)), fmaxf(fabsf(x1.z), fabsf(x1.w))));
        am = quad_max(am);
        const float dd = am / 127.0f;
        const float id = dd != 0.f ? 1.0f / dd : 0.0f;
        const float xs[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
        unsigned qw[2] = {0u, 0u};
        int qs = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int qj = (int)roundf(xs[j] * id);
            qs += qj;
            qw[j >> 2] |= ((unsigned)qj & 0xFFu) << (8 * (j & 3));
        }
        *(uint2 *)(actq + b * QS + kb * 32 + e8) = make_uint2(qw[0], qw[1]);
        if ((lane & 3) == 0) actd[blk] = __half2float(__float2half(dd));
        if constexpr (Q4) {  // the block's sum over its 4 lanes (a DPP quad)
            qs += __builtin_amdgcn_update_dpp(0, qs, 0xB1, 0xF, 0xF, false);
            qs += __builtin_amdgcn_update_dpp(0, qs, 0x4E, 0xF, 0xF, false);
            if ((lane & 3) == 0) actsum[blk] = qs;
        }
    }
    lds_sync();
    ts_mark(p.ts, t_start);  // profiling: activation tile quantised

    const int c = min(lane & 15, NB);
    const signed char *bq = actq + c * QS + 8 * (lane >> 4);
    const float *bd = actd + c * NBLK;
    const int *bs = actsum + (Q4 ? c * NBLK : 0);
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < KW; ++i) {
        const int kp = w * KW + i;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int kc = 2 * kp + h;
            long av;
            if constexpr (Q4) {
                // nibbles u = q + 8 (byte i of the word: u_i | u_{i+4} << 4) as int8 0..15
                const unsigned wn = h ? a[i].y : a[i].x;
                av = (long)(((unsigned long)((wn >> 4) & 0x0F0F0F0Fu) << 32) | (wn & 0x0F0F0F0Fu));
            } else {
                av = h ? (long)(((unsigned long)a[i].w << 32) | a[i].z) : (long)(((unsigned long)a[i].y << 32) | a[i].x);
            }
            const long bv = *(const long *)(bq + kc * 32);
            const intx4 zero = {0, 0, 0, 0};
            intx4 s = __builtin_amdgcn_mfma_i32_16x16x32_i8(av, bv, zero, 0, 0, 0);
            if constexpr (Q4) {  // sum (u - 8) a = sum u a - 8 sum a: the exact integer dot of ggml's q - 8
                const int corr = 8 * bs[kc];
                s[0] -= corr; s[1] -= corr; s[2] -= corr; s[3] -= corr;
            }
            const float da = bd[kc];
            const unsigned dlo = h ? sd[i].z : sd[i].x, dhi = h ? sd[i].w : sd[i].y;  // rows 4g..4g+3
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const unsigned wd = r < 2 ? dlo : dhi;
                const float dw = __half2float(__ushort_as_half((unsigned short)((r & 1) ? wd >> 16 : wd & 0xFFFFu)));
                acc[r] = fmaf((float)s[r], dw * da, acc[r]);  // ggml's per-block update (the fused XA repeats it)
            }
        }
    }
    if (p.q8dump) {
        // diagnostics (MAGPIE_Q8DUMP): the operands this launch quantised and the integer
        // block dots its MFMAs form from them (the same fragments and instructions as the
        // loop above, without the scales), for an exact comparison with ggml's
        // quantize_row_q8_0 / vec_dot_q8_0_q8_0 fed the same f32 rows (tests/test_q8_exact_gpu.py)
        char *db = (char *)p.q8dump;
        if (rt == 0) {
            float *da = (float *)db;
            signed char *dq = (signed char *)(db + (size_t)NB * K * 4);
            float *dd = (float *)(db + (size_t)NB * K * 5);
            for (int e = tid; e < NB * K; e += MP_BLOCK) {
                da[e] = act[e];
                dq[e] = actq[(e / K) * QS + e % K];
            }
            for (int e = tid; e < NB * NBLK; e += MP_BLOCK) dd[e] = actd[e];
        }
        int *ds = (int *)(db + (size_t)NB * K * 5 + (size_t)NB * NBLK * 4);
#pragma unroll
        for (int i = 0; i < KW; ++i) {
            const int kp = w * KW + i;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int kc = 2 * kp + h;
                long av;
                if constexpr (Q4) {
                    const unsigned wn = h ? a[i].y : a[i].x;
                    av = (long)(((unsigned long)((wn >> 4) & 0x0F0F0F0Fu) << 32) | (wn & 0x0F0F0F0Fu));
                } else {
                    av = h ? (long)(((unsigned long)a[i].w << 32) | a[i].z) : (long)(((unsigned long)a[i].y << 32) | a[i].x);
                }
                const long bv = *(const long *)(bq + kc * 32);
                const intx4 zero = {0, 0, 0, 0};
                intx4 sv = __builtin_amdgcn_mfma_i32_16x16x32_i8(av, bv, zero, 0, 0, 0);
                if constexpr (Q4) {
                    const int corr = 8 * bs[kc];
                    sv[0] -= corr; sv[1] -= corr; sv[2] -= corr; sv[3] -= corr;
                }
                const int col = lane & 15;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int n = rt * 16 + 4 * (lane >> 4) + r;
                    if (col < NB && n < p.N) ds[((size_t)n * NBLK + kc) * NB + col] = sv[r];
                }
            }
        }
    }
    part[w][lane] = acc;
    lds_sync();
    // thread t -> (row t/16, column t%16); D[row][col] sits in lane (row/4)*16 + col, register row%4
    const int row = tid >> 4, col = tid & 15;
    if (col >= NB) return;
    const int ls = (row >> 2) * 16 + col, rg = row & 3;
    const float v = ((part[0][ls][rg] + part[1][ls][rg]) + part[2][ls][rg]) + part[3][ls][rg];
    const int n = rt * 16 + row;
    if (n >= p.N) return;
    if constexpr (EPI == EPI_QKV_SA) publish_qkv(p, v, n, col);
    else if constexpr (EPI == EPI_RESID_XQ8) publish_x1_op(p, v, n, col, eop);
    else if constexpr (EPI == EPI_BIAS || EPI == EPI_RESID || EPI == EPI_ADD_STORE) epi_store_op<EPI>(p, v, n, col, eop);
    else epi_store<EPI>(p, v, n, col, EPI == EPI_LTX_ADD ? sc[col * LTD + n] : 0.f);
    ts_end(p.ts, t_start);
}

// ---------------------------------------------------------------- LT step, Q8_0 mode
// LtSlotQ8P (mp_params.hpp). Workgroup (q, b), WP per slot (below).
// RED (p.wot set): every workgroup computes all 256 o_net rows itself (thread t row t,
// from the transposed copy: 16 coalesced 16-byte loads, L2-resident after the first
// workgroup), so y needs no hand-off. DEFER (p.part set, batch 1): the partial FFN-down
// sums are plain stores and the Q8_0 head's prologue merges them (PRO_LTQ_MERGE: the
// same p-ascending sum, then + y), so the launch has no hand-off at all. Every variant
// computes the same bits: the o_net row is the block-ordered sum of (int dot) x (d_w d_a)
// from 0, the merge sums the LTQ_P partials in ascending p, then adds y.
// WP workgroups per slot (64, or 32 from 8 slots: 512 instead of 1024 workgroups at 16),
// each computing LTQ_P / WP of the LTQ_P partial sums (16 hidden units each), so the
// partials, their order and the merge are the same for every WP.
constexpr int LTQ_U = LTF / LTQ_P;  // hidden units per partial sum
// (the deferred merge at batch 1 is the Q8_0 head's PRO_LTQ_MERGE prologue: LTQ_P partials)
template <bool RED, bool DEFER, int WP>
__global__ __launch_bounds__(MP_BLOCK) void lt_slot_q8_kernel(LtSlotQ8P p) {
#pragma clang fp contract(off)
    const unsigned long long t_start = ts_begin(p.ts);
    constexpr int PPW = LTQ_P / WP, UW = LTF / WP, UWW = UW / MP_NWAVES, RWG = LTD / WP, RWW = RWG / MP_NWAVES;
    constexpr int NPT = LTQ_P * RWG / MP_BLOCK;  // merge: partial granules per thread
    static_assert(LTD == MP_BLOCK && RWW >= 1 && RWW * MP_NWAVES * WP == LTD && PPW * WP == LTQ_P && LTQ_U % 4 == 0 &&
                      NPT * MP_BLOCK == LTQ_P * RWG, "split");
    static_assert(RED || !DEFER, "the deferred merge needs y in every workgroup");
    __shared__ __attribute__((aligned(16))) float xs[LTD];   // X (the attention residual), then LN(y)
    __shared__ __attribute__((aligned(16))) float ys[LTD];
    __shared__ __attribute__((aligned(16))) int aq[LTD / 4];  // the attention output as Q8_0 (4 int8 per lane)
    __shared__ float ad[LTD / 32];
    __shared__ __attribute__((aligned(16))) float fs[UW];
    __shared__ float mv[LTQ_P][RWG];
    __shared__ __attribute__((aligned(16))) float wsc[2 * VCB];
    const GemvP &g = p.g;
    const int q = blockIdx.x, b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6, cb = g.cb;
    const int dep = ts_dep(t_start);
    // wave 0 first issues what its pick waits on (the logits, earlier positions' k / v;
    // position 0's v and X), then every wave its weights: o_net rows (4 int8 per lane,
    // the lane's block scale), FFN rows / slice
    const size_t rowb = (size_t)b * NCB * LTD + 4 * lane;
    float4 kr[NCB], vr[NCB], pos4, a4, x4;
    float lv[PICK_R];
    // greedy: the pick split over the 4 waves (lt_pick_split's scheme, mp_decode.hip): every
    // wave loads its logit rows and what y needs; the wave holding the code continues
    float lq[QPR];
    int stq = 0;
    const bool quad = cb > 0 && !g.smp.on;
    if (quad) {
        const float *lg = g.logits + (size_t)b * VCB;
#pragma unroll
        for (int r = 0; r < QPR; ++r) {
            const int i = lane + 64 * (w * QPR + r);
            lq[r] = i < VCB ? lg[i] : -INFINITY;
        }
#pragma unroll
        for (int j = 0; j < NCB - 1; ++j)
            if (j < cb) { kr[j] = *(const float4 *)(g.ltk + rowb + j * LTD); vr[j] = *(const float4 *)(g.ltv + rowb + j * LTD); }
        pos4 = *(const float4 *)(g.lt_pos + (size_t)cb * LTD + 4 * lane);
        stq = g.step[b];
    } else if (w == 0) {
        if (cb > 0) {
            load_logits(g.logits + (size_t)b * VCB, lv);
#pragma unroll
            for (int j = 0; j < NCB - 1; ++j)
                if (j < cb) { kr[j] = *(const float4 *)(g.ltk + rowb + j * LTD); vr[j] = *(const float4 *)(g.ltv + rowb + j * LTD); }
            pos4 = *(const float4 *)(g.lt_pos + (size_t)cb * LTD + 4 * lane);
        } else {  // one position: softmax weight 1, a = v_0 (lt_attend computes exactly that)
            a4 = *(const float4 *)(g.ltv + rowb);
            x4 = *(const float4 *)(g.ltX + (size_t)b * LTD + 4 * lane);
        }
    }
    const int r0 = q * RWG + RWW * w + dep;
    int wq[RWW];
    float wd[RWW];
    intx4 wr[RED ? LTD / 16 : 1];  // RED: row tid's 256 int8 (16 B per load, wot[i][tid])
    intx4 wrd;                     // RED: row tid's 8 fp16 block scales
    if constexpr (RED) {
#pragma unroll
        for (int i = 0; i < LTD / 16; ++i) wr[i] = *(const intx4 *)(p.wot + ((size_t)i * LTD + tid + dep) * 16);
        wrd = *(const intx4 *)(p.wod + (size_t)tid * (LTD / 32));
    } else {
#pragma unroll
        for (int r = 0; r < RWW; ++r) {
            wq[r] = *(const int *)(p.woq + (size_t)(r0 + r) * LTD + 4 * lane);
            wd[r] = __half2float(__ushort_as_half(p.wod[(size_t)(r0 + r) * (LTD / 32) + (lane >> 3)]));
        }
    }
    const int u0 = q * UW;
    float4 a1[UWW], a2[PPW][LTQ_U / 4];
#pragma unroll
    for (int r = 0; r < UWW; ++r) a1[r] = *(const float4 *)(p.w1 + (size_t)(u0 + w * UWW + r) * LTD + 4 * lane);
#pragma unroll
    for (int k = 0; k < PPW; ++k)
#pragma unroll
        for (int i = 0; i < LTQ_U / 4; ++i)
            a2[k][i] = *(const float4 *)(p.w2s + ((size_t)(q * PPW + k) * LTD + tid) * LTQ_U + 4 * i);
    // per codebook step its own tags (8 steps share the buffers within one frame)
    const unsigned tag_y = (unsigned)p.iter[0] * 64u + 32u + (unsigned)cb, tag_p = tag_y + 16u;
    int yw = 0;  // the wave computing the attention output
    int code = 0, amax = 0;
    float4 q4, k4, v4, xp;
    auto gather = [&](int c) {
        const size_t rr = (size_t)(cb - 1) * VCB + c;
        const float *row = g.qkvtab + rr * (3 * LTD) + 4 * lane;
        q4 = *(const float4 *)row; k4 = *(const float4 *)(row + LTD); v4 = *(const float4 *)(row + 2 * LTD);
        xp = *(const float4 *)(g.ptab + rr * LTD + 4 * lane);
    };
    if (quad) {
        float bv;
        int bi = wave_pick_rows(lq, w, g.ignore_eos || stq < 4, g.audio_bos, g.audio_eos, bv);
        if (bi < 0 || bi >= VCB) bi = 0;
        gather(bi);  // this wave's candidate, in flight during the exchange
        yw = pick_exchange(bv, bi, code);
        amax = code;
    }
    if (w == yw) {
        // the attention output a of position cb and its residual X (lt_pick_kernel's steps)
        if (cb > 0) {
            if (!quad) {
                const int stp = g.step[b];
                code = wave_pick_v(lv, g.ignore_eos || stp < 4, g.audio_bos, g.audio_eos, g.smp, b, stp, cb - 1, wsc, amax);
                gather(code);
            }
            if (q == 0) {
                if (lane == 0) {
                    g.codes_cur[b * NCB + cb - 1] = code;
                    if (amax == g.audio_eos) g.smp.argeos[b] = 1;
                    if (g.smp.amax) g.smp.amax[b * NCB + cb - 1] = amax;
                }
                *(float4 *)(g.lk + ((size_t)b * NCB + cb) * LTD + 4 * lane) = k4;
                *(float4 *)(g.lv + ((size_t)b * NCB + cb) * LTD + 4 * lane) = v4;
            }
            x4 = make_float4(xp.x + pos4.x, xp.y + pos4.y, xp.z + pos4.z, xp.w + pos4.w);
            a4 = lt_attend<true, true>(g, b, q4, k4, v4, kr, vr);
        }
        *(float4 *)&xs[4 * lane] = x4;
        // a -> Q8_0 (quantize_row_q8_0_ref): block = 8 lanes x 4 elements
        float am = fmaxf(fmaxf(fabsf(a4.x), fabsf(a4.y)), fmaxf(fabsf(a4.z), fabsf(a4.w)));
        am = quad_max(am);
        am = fmaxf(am, dpp_mov<0x141>(am));  // the other quad of the 8-lane block (row half mirror)
        const float dd = am / 127.0f;
        const float id = dd != 0.f ? 1.0f / dd : 0.0f;
        const float av[4] = {a4.x, a4.y, a4.z, a4.w};
        unsigned qw = 0u;
#pragma unroll
        for (int j = 0; j < 4; ++j) qw |= ((unsigned)(int)roundf(av[j] * id) & 0xFFu) << (8 * j);
        aq[lane] = (int)qw;
        if ((lane & 7) == 0) ad[lane >> 3] = __half2float(__float2half(dd));
    }
    lds_sync();
    // o_net: per block the exact integer dot, then sum_blocks isum * (d_w d_a) in block order
    if constexpr (RED) {
        float acc = 0.f;
#pragma unroll
        for (int kb = 0; kb < LTD / 32; ++kb) {
            const intx4 x0 = *(const intx4 *)&aq[8 * kb], x1 = *(const intx4 *)&aq[8 * kb + 4];
            const intx4 w0 = wr[2 * kb], w1 = wr[2 * kb + 1];
            int is = __builtin_amdgcn_sdot4(w0.x, x0.x, 0, false);
            is = __builtin_amdgcn_sdot4(w0.y, x0.y, is, false);
            is = __builtin_amdgcn_sdot4(w0.z, x0.z, is, false);
            is = __builtin_amdgcn_sdot4(w0.w, x0.w, is, false);
            is = __builtin_amdgcn_sdot4(w1.x, x1.x, is, false);
            is = __builtin_amdgcn_sdot4(w1.y, x1.y, is, false);
            is = __builtin_amdgcn_sdot4(w1.z, x1.z, is, false);
            is = __builtin_amdgcn_sdot4(w1.w, x1.w, is, false);
            const unsigned dw2 = (unsigned)wrd[kb >> 1];
            const float dwk = __half2float(__ushort_as_half((unsigned short)((kb & 1) ? dw2 >> 16 : dw2 & 0xFFFFu)));
            const float fb = (float)is * (dwk * ad[kb]);
            acc += fb;
        }
        const float yv = acc + xs[tid];
        ys[tid] = yv;
        if (q == 0) p.y[(size_t)b * LTD + tid] = yv;
        lds_sync();
    } else {
        const int av = aq[lane];
        float o[RWW];
#pragma unroll
        for (int r = 0; r < RWW; ++r) {
            int is = __builtin_amdgcn_sdot4(wq[r], av, 0, false);
            // the 8-lane block's integer sum (exact in any order) by DPP: quad, then half-row mirror
            is += __builtin_amdgcn_update_dpp(0, is, 0xB1, 0xF, 0xF, false);
            is += __builtin_amdgcn_update_dpp(0, is, 0x4E, 0xF, 0xF, false);
            is += __builtin_amdgcn_update_dpp(0, is, 0x141, 0xF, 0xF, false);
            const float fb = (float)is * (wd[r] * ad[lane >> 3]);  // lanes 8kb .. 8kb+7: block kb's term
            float acc = 0.f;
#pragma unroll
            for (int kb = 0; kb < LTD / 32; ++kb) acc += __shfl(fb, 8 * kb, 64);
            o[r] = acc;
        }
        if (lane < RWW) {
            const int n = r0 + lane;
            float ov = o[0];
#pragma unroll
            for (int r = 1; r < RWW; ++r) ov = lane == r ? o[r] : ov;
            const float yv = ov + xs[n];
            __hip_atomic_store((gu64 *)p.gy + (size_t)b * LTD + n, ((unsigned long long)tag_y << 32) | __float_as_uint(yv),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            p.y[(size_t)b * LTD + n] = yv;
        }
    }
    // y (all 256) from the slot's granules, LN -> xs (wave 0; the other waves wait)
    if (w == 0) {
        float yv[4];
        if constexpr (RED) {
            const float4 y4 = *(const float4 *)&ys[4 * lane];
            yv[0] = y4.x; yv[1] = y4.y; yv[2] = y4.z; yv[3] = y4.w;
        } else {
            gh_wait_n<4, 1>(p.gy + (size_t)b * LTD + 4 * lane, tag_y, yv, p.hx_err);
            *(float4 *)&ys[4 * lane] = make_float4(yv[0], yv[1], yv[2], yv[3]);
        }
        ts_mark(p.ts, t_start);  // profiling: y seen
        float mean, var;
        wave_meanvar<4>(yv, mean, var);
        const float rstd = 1.0f / sqrtf(var + p.eps);
        const float4 gl = *(const float4 *)(p.lnw + 4 * lane);
        *(float4 *)&xs[4 * lane] = make_float4(((yv[0] - mean) * rstd) * gl.x, ((yv[1] - mean) * rstd) * gl.y,
                                               ((yv[2] - mean) * rstd) * gl.z, ((yv[3] - mean) * rstd) * gl.w);
    }
    lds_sync();
    {
        const float4 xv = *(const float4 *)&xs[4 * lane];
        float v[UWW];
#pragma unroll
        for (int r = 0; r < UWW; ++r) v[r] = dotv(a1[r], xv);
        ffn_units_store<UWW>(v, &fs[w * UWW], [](float g) { return g; });
    }
    lds_sync();
    float acc[PPW];
#pragma unroll
    for (int k = 0; k < PPW; ++k) {
        acc[k] = 0.f;
#pragma unroll
        for (int i = 0; i < LTQ_U / 4; ++i) {
            const float4 f4 = *(const float4 *)&fs[k * LTQ_U + 4 * i];
            acc[k] = fmaf(a2[k][i].x, f4.x, acc[k]);
            acc[k] = fmaf(a2[k][i].y, f4.y, acc[k]);
            acc[k] = fmaf(a2[k][i].z, f4.z, acc[k]);
            acc[k] = fmaf(a2[k][i].w, f4.w, acc[k]);
        }
    }
    if constexpr (DEFER) {  // the head's prologue merges (PRO_LTQ_MERGE)
#pragma unroll
        for (int k = 0; k < PPW; ++k) p.part[((size_t)b * LTQ_P + q * PPW + k) * LTD + tid] = acc[k];
        ts_end(p.ts, t_start);
        return;
    }
    // partial sums through granules; this workgroup merges its RWG outputs in partial order
    gu64 *gp = (gu64 *)p.gp + (size_t)b * LTQ_P * LTD;
#pragma unroll
    for (int k = 0; k < PPW; ++k)
        __hip_atomic_store(gp + (size_t)(q * PPW + k) * LTD + tid, ((unsigned long long)tag_p << 32) | __float_as_uint(acc[k]),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    {   // thread t: partials t / RWG + (256 / RWG) i of output RWG q + t % RWG, one round trip per poll
        float mvv[NPT];
        gh_wait_n<NPT, (MP_BLOCK / RWG) * LTD>(p.gp + (size_t)b * LTQ_P * LTD + (size_t)(tid / RWG) * LTD + RWG * q + tid % RWG,
                                               tag_p, mvv, p.hx_err);
#pragma unroll
        for (int i = 0; i < NPT; ++i) mv[tid / RWG + (MP_BLOCK / RWG) * i][tid % RWG] = mvv[i];
    }
    lds_sync();
    if (tid < RWG) {
        float s = mv[0][tid];
#pragma unroll 8
        for (int k = 1; k < LTQ_P; ++k) s += mv[k][tid];
        p.y2[(size_t)b * LTD + RWG * q + tid] = s + ys[RWG * q + tid];
    }
    ts_end(p.ts, t_start);
}
hipError_t op_lt_slot_q8(const LtSlotQ8P &p, int NB, hipStream_t s) {
    const GemvP &g = p.g;
    if (!(p.woq || p.wot) || !p.wod || !p.lnw || !p.w1 || !p.w2s || !p.y || (!p.part && (!p.y2 || !p.gp)) ||
        (!p.wot && !p.gy) || (p.part && (!p.wot || NB != 1)) || !p.iter || !p.hx_err ||
        !g.ltX || !g.ltk || !g.ltv || !g.lk || !g.lv || g.cb < 0 || g.cb >= NCB || NB < 1 || NB > 16 ||
        (g.cb > 0 && (!g.logits || !g.codes_cur || !g.qkvtab || !g.ptab || !g.lt_pos || !g.step || !g.smp.cfg ||
                      !g.smp.argeos)))
        return hipErrorInvalidValue;
    if (p.part) mp::launch(lt_slot_q8_kernel<true, true, 64>, dim3(64, NB), dim3(MP_BLOCK), 0, s, p);
    else if (p.wot) mp::launch(lt_slot_q8_kernel<true, false, 64>, dim3(64, NB), dim3(MP_BLOCK), 0, s, p);
    else if (NB >= 8) mp::launch(lt_slot_q8_kernel<false, false, 32>, dim3(32, NB), dim3(MP_BLOCK), 0, s, p);
    else mp::launch(lt_slot_q8_kernel<false, false, 64>, dim3(64, NB), dim3(MP_BLOCK), 0, s, p);
    return hipGetLastError();
}

// int8 [N][K] + fp16 scales [N][K/32] (the file's blocks) -> fragment order:
// q [ceil(N/16)][K/64][64][16 B], d [ceil(N/16)][K/64][4][8 fp16]; rows >= N zero
__global__ void pack_q8_kernel(const signed char *q, const unsigned short *d, int N, int K, unsigned char *oq,
                               unsigned short *od) {
    const int KP = K / 64;
    const size_t total = (size_t)((N + 15) / 16) * KP * 64;
    for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
        const int lane = (int)(e % 64), g = lane >> 4;
        const size_t frag = e / 64;
        const int kp = (int)(frag % KP), rt = (int)(frag / KP);
        const int n = rt * 16 + (lane & 15);
        if (oq)  // (null: the scales only, a Q4_0 tensor's nibbles come from pack_q4)
            for (int j = 0; j < 16; ++j) {
                const int k = kp * 64 + (j >> 3) * 32 + 8 * g + (j & 7);
                oq[e * 16 + j] = n < N ? (unsigned char)q[(size_t)n * K + k] : 0;
            }
        if ((lane & 15) == 0)
            for (int j = 0; j < 8; ++j) {
                const int r = rt * 16 + 4 * g + (j & 3), blk = 2 * kp + (j >> 2);
                od[(frag * 4 + g) * 8 + j] = r < N ? d[(size_t)r * (K / 32) + blk] : 0;
            }
    }
}
hipError_t pack_q8(const signed char *q, const unsigned short *d, int N, int K, unsigned char *oq,
                   unsigned short *od, hipStream_t s) {
    if (!q || !d || !od || N <= 0 || K % 256) return hipErrorInvalidValue;
    mp::launch(pack_q8_kernel, dim3(1024), dim3(256), 0, s, q, d, N, K, oq, od);
    return hipGetLastError();
}

// Q4_0 decode fragments from the int8 q - 8 values: [ceil(N/16)][K/64][64 lanes][2 x u32],
// word h of lane l = the 8 values of block 2j+h at k-offset 8(l>>4) as nibbles u = q + 8,
// byte i holding u_i | u_{i+4} << 4 (two masks give the MFMA operand's 8 int8 bytes);
// the scales as pack_q8 lays them out (pass od = null to keep those of a pack_q8 call)
__global__ void pack_q4_kernel(const signed char *q, int N, int K, unsigned *oq) {
    const int KP = K / 64;
    const size_t total = (size_t)((N + 15) / 16) * KP * 64;
    for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
        const int lane = (int)(e % 64), g = lane >> 4;
        const size_t frag = e / 64;
        const int kp = (int)(frag % KP), rt = (int)(frag / KP);
        const int n = rt * 16 + (lane & 15);
        for (int h = 0; h < 2; ++h) {
            unsigned wd = 0u;
            for (int i = 0; i < 8; ++i) {
                const int k = kp * 64 + h * 32 + 8 * g + i;
                const unsigned u = (unsigned)((n < N ? (int)q[(size_t)n * K + k] : 0) + 8) & 15u;
                wd |= u << (i < 4 ? 8 * i : 8 * (i - 4) + 4);
            }
            oq[e * 2 + h] = wd;
        }
    }
}
hipError_t pack_q4(const signed char *q, int N, int K, unsigned char *oq, hipStream_t s) {
    if (!q || !oq || N <= 0 || K % 256) return hipErrorInvalidValue;
    mp::launch(pack_q4_kernel, dim3(1024), dim3(256), 0, s, q, N, K, (unsigned *)oq);
    return hipGetLastError();
}

// ---------------------------------------------------------------- XA, direct form
// Cross-attention as ggml computes it (magpie.cpp:1713-1767): q = q_net LN(x) is
// one GEMV launch (8 workgroups: q_net's 128 rows spread over CUs); xa_dir_kernel
// then does attention + o_net + residual: grid (768/64, B), a workgroup owns 64 rows
// of o_net, issues them first, recomputes the slot's attention over the text (K, V:
// 2 x T x 128 f32, coalesced: half a wave per key row; xa_text_attention) and
// finishes x2 = x + o_net a for its rows.
//  * Q8_0 q_net / o_net (xa_q8_kernel): a is quantised to Q8_0 and dotted with
//    v_dot4 per half block (the exact int32 block dots, times d_w * d_a);
//  * f32 (xa_f32_kernel; long texts, where the reassociated K'/V' form of mp_xa.hpp
//    would read 6 KB per text token and layer against 1 KB here).
constexpr int XQ8_ROWS = 64;  // o_net rows per workgroup

// xa_text_attention_q / xa_text_attention (the text attention itself): mp_xa.hpp, shared
// with the preamble's cross-attention rows (mp_prefill.hip row_xa_kernel).

// a (LDS, [128]) -> Q8_0 blocks aq / ad (ggml quantises the o_net operand), wave 0
__device__ __forceinline__ void xa_quantize_a(const float *a_s, signed char *aq, float *ad) {
    const int lane = threadIdx.x & 63;
    if ((threadIdx.x >> 6) == 0) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {  // element lane + 64 i; its Q8_0 block = this half-wave
            const float av = a_s[lane + 64 * i];
            float a = row_max16(fabsf(av));
            // the block = 2 rows of 16: their maxima from the rows' last lanes (readlane)
            const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, a), 15));
            const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, a), 31));
            const float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, a), 47));
            const float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, a), 63));
            a = lane < 32 ? fmaxf(r0, r1) : fmaxf(r2, r3);
            const float dd = a / 127.0f;
            const float id = dd != 0.f ? 1.0f / dd : 0.0f;
            aq[lane + 64 * i] = (signed char)(int)roundf(av * id);
            if ((lane & 31) == 0) ad[(lane + 64 * i) / 32] = __half2float(__float2half(dd));
        }
    }
    lds_sync();
}

// o_net rows of one wave: G groups of 8 rows (8 lanes x 16 B per row), the Q8_0 block
// dots on v_dot4 times d_w * d_a, summed over the row's 4 blocks; x2 = v + x1
constexpr int XQ8_OR = 8, XQ8_OCPR = DXA / 16;
template <int G>
__device__ __forceinline__ void xa_q8_onet(const uint4 (&wo)[G], const float (&wos)[G], int row0, const signed char *aq,
                                           const float *ad, const float *x1, float *x2) {
#pragma clang fp contract(off)
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int r = lane / XQ8_OCPR, kc = lane % XQ8_OCPR;
        const int4 a4 = *(const int4 *)(aq + kc * 16);
        int s = __builtin_amdgcn_sdot4((int)wo[g].x, a4.x, 0, false);
        s = __builtin_amdgcn_sdot4((int)wo[g].y, a4.y, s, false);
        s = __builtin_amdgcn_sdot4((int)wo[g].z, a4.z, s, false);
        s = __builtin_amdgcn_sdot4((int)wo[g].w, a4.w, s, false);
        s += __builtin_amdgcn_update_dpp(0, s, 0xB1, 0xF, 0xF, false);
        const float f = (lane & 1) ? 0.f : (float)s * (wos[g] * ad[kc >> 1]);
        // the row's 4 block terms (lanes 8r + 0, 2, 4, 6) as (f0 + f2) + (f4 + f6) in all 8 of
        // its lanes, every row at once: the same bits as a full-wave tree sum of the row's
        // lanes alone (whose remaining steps add +0, hence the final + 0)
        float v = f + dpp_mov<0xB1>(f);
        v += dpp_mov<0x4E>(v);
        v += dpp_mov<0x141>(v);
        v += 0.f;
        if ((lane & 7) == 0) {
            const int row = row0 + g * XQ8_OR + r;
            x2[row] = v + x1[row];
        }
    }
}

__global__ __launch_bounds__(MP_BLOCK) void xa_q8_kernel(XaQ8P p) {
    constexpr int OG = XQ8_ROWS / MP_NWAVES / XQ8_OR;  // 2 groups of 8 rows per wave
    __shared__ float pr[TMAX_LIMIT];
    __shared__ __attribute__((aligned(16))) float a_s[DXA];
    __shared__ __attribute__((aligned(16))) signed char aq[DXA];
    __shared__ float ad[DXA / 32];
    const int b = blockIdx.y, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r0 = blockIdx.x * XQ8_ROWS + w * OG * XQ8_OR;
    uint4 wo[OG];
    float wos[OG];
#pragma unroll
    for (int g = 0; g < OG; ++g) {
        const int row = r0 + g * XQ8_OR + lane / XQ8_OCPR, kc = lane % XQ8_OCPR;
        wo[g] = *(const uint4 *)(p.wo + (size_t)row * DXA + kc * 16);
        wos[g] = __half2float(__ushort_as_half(p.wod[(size_t)row * (DXA / 32) + kc / 2]));
    }
    const size_t kv = ((size_t)(b * p.nlayers + p.layer) * p.Tmax) * DXA;
    xa_text_attention(p.q + (size_t)b * DXA, p.xak + kv, p.xav + kv, p.T[b], pr, a_s);
    xa_quantize_a(a_s, aq, ad);
    // ---- x2 = x + Q8(o_net) a for this workgroup's 64 rows (8 per group)
    xa_q8_onet<OG>(wo, wos, r0, aq, ad, p.x + (size_t)b * D, p.x2 + (size_t)b * D);
}

// ---------------------------------------------------------------- XA q_net, fused (EPI_RESID_XQ8)
constexpr int XQ_ROWS = DXA / XQG, XQ_QB = D / 32 / 4;  // 8 workgroups x 16 rows; 6 blocks per quarter
// q_net row qr, quarter qa (6 blocks of int8 + their scales): issued before x1 exists
__device__ __forceinline__ void xq8_load_rows(const XaQ8P &x, int qr, int qa, int dep, uint4 (&wq)[2 * XQ_QB],
                                              unsigned short (&wqs)[XQ_QB]) {
    const uint4 *src = (const uint4 *)(x.wq + (size_t)qr * D + qa * XQ_QB * 32 + dep);
#pragma unroll
    for (int i = 0; i < 2 * XQ_QB; ++i) wq[i] = src[i];
#pragma unroll
    for (int j = 0; j < XQ_QB; ++j) wqs[j] = x.wqd[(size_t)qr * (D / 32) + qa * XQ_QB + j];
}
// x1 of slot b into dst[768] (LDS), wave w sweeping its quarter (3 granules per lane) and
// storing it; the caller's barrier publishes the row. One poller per granule: when every
// wave polled the whole row, the barrier after it waited for the unluckiest wave's next
// round trip (~1 us) after the row was complete.
__device__ __forceinline__ void xq8_sweep_x1_quarter(const GemvP &p, int b, float *dst) {
    constexpr int PQ = D / 64 / MP_NWAVES;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned tag = (unsigned)p.iter[0] * 64u + p.layer + 1u;
    gu64 *gr = (gu64 *)(p.xh + (size_t)b * D) + w * PQ * 64;
    float v[PQ];
    for (unsigned spins = 0;; ++spins) {
        bool ok = true;
#pragma unroll
        for (int j = 0; j < PQ; ++j) {
            const unsigned long long u = __hip_atomic_load(gr + lane + 64 * j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            v[j] = __uint_as_float((unsigned)u);
            ok &= (unsigned)(u >> 32) == tag;
        }
        if (__all(ok)) break;
        if (spins >= HX_SPIN_LIMIT) {  // never seen: poison the output and say so
            if (lane == 0) __hip_atomic_fetch_or((gi32 *)p.hx_err, HX_ERR_XA, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
            for (int j = 0; j < PQ; ++j) v[j] = __builtin_nanf("");
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
#pragma unroll
    for (int j = 0; j < PQ; ++j) dst[w * PQ * 64 + lane + 64 * j] = v[j];
}
// LN(x1) * lnw (PRO_LN at batch 1: every wave the whole row, wave w stores its quarter),
// then the row's Q8_0 blocks (gemm_q8_kernel_dec's quantiser) into actq / actd
__device__ __forceinline__ void xq8_ln_quant(const XaQ8P &x, const float (&v)[D / 64], const float (&g)[D / 64],
                                             float *act, signed char *actq, float *actd) {
#pragma clang fp contract(off)
    constexpr int PER = D / 64, Q = PER / MP_NWAVES, NBLK = D / 32;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    {
        float mean, var;
        wave_meanvar<PER>(v, mean, var);
        const float rstd = 1.0f / sqrtf(var + x.eps);
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            if (i / Q != w) continue;
            act[lane + 64 * i] = ((v[i] - mean) * rstd) * g[i];
        }
    }
    lds_sync();
    if (tid < 4 * NBLK) {
        const int kb = tid >> 2, e8 = 8 * (lane & 3);
        const float4 x0 = *(const float4 *)(act + kb * 32 + e8);
        const float4 xx = *(const float4 *)(act + kb * 32 + e8 + 4);
        float am = fmaxf(fmaxf(fmaxf(fabsf(x0.x), fabsf(x0.y)), fmaxf(fabsf(x0.z), fabsf(x0.w))),
                         fmaxf(fmaxf(fabsf(xx.x), fabsf(xx.y)), fmaxf(fabsf(xx.z), fabsf(xx.w))));
        am = quad_max(am);
        const float dd = am / 127.0f;
        const float id = dd != 0.f ? 1.0f / dd : 0.0f;
        const float xs[8] = {x0.x, x0.y, x0.z, x0.w, xx.x, xx.y, xx.z, xx.w};
        unsigned qw[2] = {0u, 0u};
#pragma unroll
        for (int j = 0; j < 8; ++j) qw[j >> 2] |= ((unsigned)(int)roundf(xs[j] * id) & 0xFFu) << (8 * (j & 3));
        *(uint2 *)(actq + kb * 32 + e8) = make_uint2(qw[0], qw[1]);
        if ((lane & 3) == 0) actd[kb] = __half2float(__float2half(dd));
    }
    lds_sync();
}
// this lane's quarter: its blocks in order (fmaf, as gemm_q8_kernel_dec), then the row's
// 4 quarters summed in order (valid in the quarter-0 lane)
__device__ __forceinline__ float xq8_dot(const uint4 (&wq)[2 * XQ_QB], const unsigned short (&wqs)[XQ_QB], int qa,
                                         const signed char *actq, const float *actd) {
#pragma clang fp contract(off)
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < XQ_QB; ++j) {
        const int blk = qa * XQ_QB + j;
        const int4 x0 = *(const int4 *)(actq + blk * 32), xx = *(const int4 *)(actq + blk * 32 + 16);
        const uint4 w0 = wq[2 * j], w1 = wq[2 * j + 1];
        int sd = __builtin_amdgcn_sdot4((int)w0.x, x0.x, 0, false);
        sd = __builtin_amdgcn_sdot4((int)w0.y, x0.y, sd, false);
        sd = __builtin_amdgcn_sdot4((int)w0.z, x0.z, sd, false);
        sd = __builtin_amdgcn_sdot4((int)w0.w, x0.w, sd, false);
        sd = __builtin_amdgcn_sdot4((int)w1.x, xx.x, sd, false);
        sd = __builtin_amdgcn_sdot4((int)w1.y, xx.y, sd, false);
        sd = __builtin_amdgcn_sdot4((int)w1.z, xx.z, sd, false);
        sd = __builtin_amdgcn_sdot4((int)w1.w, xx.w, sd, false);
        const float dw = __half2float(__ushort_as_half(wqs[j]));
        acc = fmaf((float)sd, dw * actd[blk], acc);
    }
    // lanes 1..3 of the quad into lane 0 by DPP quad permutes (no LDS round trip)
    const float p1 = dpp_mov<0xE5>(acc), p2 = dpp_mov<0xE6>(acc), p3 = dpp_mov<0xE7>(acc);
    return ((acc + p1) + p2) + p3;
}

// The cross-attention's Q8_0 q_net riding in the Q8_0 O-projection's launch: the
// launch's last XQG x NB workgroups, XQ_ROWS rows of q each. A workgroup issues its
// q_net rows (wave 0, lane = (row, quarter): 6 blocks of int8 + their scales, the
// MFMA kernel's K split) before x1 exists, sweeps the x1 granules (publish_x1), and
// computes exactly what the separate q GEMV does: LN(x1) * lnw (PRO_LN's wave
// statistics), the Q8_0 activation blocks (gemm_q8_kernel_dec's quantiser), each
// quarter's block dots accumulated in block order and the quarters summed in order,
// stored to q. xa_q8_kernel (the next launch) does the attention and o_net. Same bits
// as the q GEMV (tests/test_q8_fused_gpu.py).
__device__ __forceinline__ void xq8_tail(const GemvP &p, float *act, signed char *actq, float *actd,
                                         unsigned long long t_start) {
    const XaQ8P &x = p.xq8;
    const int k = blockIdx.x - p.nrow_blocks, b = k / XQG, r0 = (k % XQG) * XQ_ROWS;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int qr = r0 + (lane >> 2), qa = lane & 3;  // wave 0: (row, quarter) per lane
    uint4 wq[2 * XQ_QB];
    unsigned short wqs[XQ_QB];
    if (w == 0) xq8_load_rows(x, qr, qa, ts_dep(t_start), wq, wqs);
    constexpr int PER = D / 64;
    float g[PER];
    load_lnw<PER>(x.lnw, g);
    __shared__ float x1row[D];
    xq8_sweep_x1_quarter(p, b, x1row);
    lds_sync();
    float v[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) v[j] = x1row[lane + 64 * j];
    ts_mark(p.ts, t_start);  // profiling: x1 seen
    xq8_ln_quant(x, v, g, act, actq, actd);
    if (w != 0) return;
    const float qv = xq8_dot(wq, wqs, qa, actq, actd);
    if (qa == 0) {  // q to the launch's attention workgroups as a {tag, value} granule
        const unsigned tag = (unsigned)p.iter[0] * 64u + p.layer + 1u;
        __hip_atomic_store((gu64 *)(x.qg + (size_t)b * DXA + qr), ((unsigned long long)tag << 32) | __float_as_uint(qv),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    ts_end(p.ts, t_start);
}

// The attention + o_net stage of the same launch (the launch's last XQ8A x NB
// workgroups, XQ8_ROWS o_net rows each): o_net rows and the first 64 text keys and
// values issued at entry, q swept from the q_net tail's granules (waves 0 and 1 a half
// each, into one LDS row), then xa_q8_kernel's arithmetic:
// the attention, a quantised to Q8_0, x2 = x1 + o_net a for its rows (x1 from the
// O-projection's granules).
constexpr int XQ8A = D / XQ8_ROWS;
__device__ __forceinline__ void xq8a_tail(const GemvP &p, unsigned long long t_start) {
    constexpr int OG = XQ8_ROWS / MP_NWAVES / XQ8_OR;
    const XaQ8P &x = p.xq8;
    __shared__ float pr[TMAX_LIMIT];
    __shared__ __attribute__((aligned(16))) float a_s[DXA];
    __shared__ __attribute__((aligned(16))) signed char aq[DXA];
    __shared__ float ad[DXA / 32];
    __shared__ __attribute__((aligned(16))) float qrow[DXA];
    __shared__ float x1s[XQ8_ROWS];
    const int k = blockIdx.x - p.nrow_blocks - XQG * p.nslots, b = k / XQ8A, rb = k % XQ8A;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r0 = rb * XQ8_ROWS + w * OG * XQ8_OR;
    uint4 wo[OG];
    float wos[OG];
#pragma unroll
    for (int g = 0; g < OG; ++g) {
        const int row = r0 + g * XQ8_OR + lane / XQ8_OCPR, kc = lane % XQ8_OCPR;
        wo[g] = *(const uint4 *)(x.wo + (size_t)row * DXA + kc * 16 + ts_dep(t_start));
        wos[g] = __half2float(__ushort_as_half(x.wod[(size_t)row * (DXA / 32) + kc / 2]));
    }
    const unsigned tag = (unsigned)p.iter[0] * 64u + p.layer + 1u;
    auto sweep = [&](gu64 *gr, float *dst, int n) {  // n = 64 or 128 granules, every lane its share
        float v[2];
        for (unsigned spins = 0;; ++spins) {
            bool ok = true;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                if (lane + 64 * j >= n) continue;
                const unsigned long long u = __hip_atomic_load(gr + lane + 64 * j, __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_AGENT);
                v[j] = __uint_as_float((unsigned)u);
                ok &= (unsigned)(u >> 32) == tag;
            }
            if (__all(ok)) break;
            if (spins >= HX_SPIN_LIMIT) {  // never seen: poison the output and say so
                if (lane == 0)
                    __hip_atomic_fetch_or((gi32 *)p.hx_err, HX_ERR_XA, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                v[0] = v[1] = __builtin_nanf("");
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j)
            if (lane + 64 * j < n) dst[lane + 64 * j] = v[j];
    };
    const size_t kv = ((size_t)(b * x.nlayers + x.layer) * x.Tmax) * DXA;
    unsigned long long x1u = 0;
    xa_text_attention_q(
        [&]() {  // waves 0 and 1 sweep a half of q each (one poller per granule)
            if (w < 2) sweep((gu64 *)(x.qg + (size_t)b * DXA) + 64 * w, qrow + 64 * w, 64);
            lds_sync();
            // q is complete, so x1 is (q_net read all of it): wave 0's residual rows issued
            // now, used after the attention
            if (w == 0) x1u = __hip_atomic_load((gu64 *)(p.xh + (size_t)b * D + rb * XQ8_ROWS) + lane, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
            return (const float *)qrow;
        },
        x.xak + kv, x.xav + kv, x.T[b], pr, a_s);
    ts_mark(p.ts, t_start);  // profiling: attention done
    if (w == 0) {
        if (__all((unsigned)(x1u >> 32) == tag)) x1s[lane] = __uint_as_float((unsigned)x1u);
        else sweep((gu64 *)(p.xh + (size_t)b * D + rb * XQ8_ROWS), x1s, XQ8_ROWS);  // (never taken)
    }
    xa_quantize_a(a_s, aq, ad);  // (its barrier also publishes x1s)
    xa_q8_onet<OG>(wo, wos, r0, aq, ad, x1s - rb * XQ8_ROWS, x.x2 + (size_t)b * D);
    ts_end(p.ts, t_start);
}

// Small batches (XaQ8P::qin): the attention + o_net workgroups (XQ8A x NB, no q_net
// workgroups) compute q themselves, so the launch has one hand-off (x1) instead of two.
// A workgroup issues its o_net rows, all 128 q_net rows (lane = (row, quarter) as
// xq8_tail, 2 rows per lane) and the first text keys / values at entry, sweeps x1,
// and computes q with xq8_tail's arithmetic (same bits: LN, quantiser, block order,
// quarter order) into LDS, then xq8a_tail's attention and o_net.
__device__ __forceinline__ void xq8qa_tail(const GemvP &p, float *act, signed char *actq, float *actd,
                                           unsigned long long t_start) {
    constexpr int OG = XQ8_ROWS / MP_NWAVES / XQ8_OR, PER = D / 64, QR = DXA / 64;  // q rows per lane
    const XaQ8P &x = p.xq8;
    __shared__ float pr[TMAX_LIMIT];
    __shared__ __attribute__((aligned(16))) float a_s[DXA];
    __shared__ __attribute__((aligned(16))) signed char aq[DXA];
    __shared__ float ad[DXA / 32];
    __shared__ __attribute__((aligned(16))) float qs[DXA];
    __shared__ float x1s[XQ8_ROWS];
    const int k = blockIdx.x - p.nrow_blocks, b = k / XQ8A, rb = k % XQ8A;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r0 = rb * XQ8_ROWS + w * OG * XQ8_OR, dep = ts_dep(t_start);
    uint4 wo[OG];
    float wos[OG];
#pragma unroll
    for (int g = 0; g < OG; ++g) {
        const int row = r0 + g * XQ8_OR + lane / XQ8_OCPR, kc = lane % XQ8_OCPR;
        wo[g] = *(const uint4 *)(x.wo + (size_t)row * DXA + kc * 16 + dep);
        wos[g] = __half2float(__ushort_as_half(x.wod[(size_t)row * (DXA / 32) + kc / 2]));
    }
    const int qa = lane & 3;
    uint4 wq[QR][2 * XQ_QB];
    unsigned short wqs[QR][XQ_QB];
#pragma unroll
    for (int j = 0; j < QR; ++j) xq8_load_rows(x, 16 * w + 64 * j + (lane >> 2), qa, dep, wq[j], wqs[j]);
    float g[PER];
    load_lnw<PER>(x.lnw, g);
    const size_t kv = ((size_t)(b * x.nlayers + x.layer) * x.Tmax) * DXA;
    xa_text_attention_q(
        [&]() {
            float v[PER];
            xq8_sweep_x1_quarter(p, b, pr);  // (pr is free until the scores)
            lds_sync();
#pragma unroll
            for (int j = 0; j < PER; ++j) v[j] = pr[lane + 64 * j];
            ts_phase<0>(p.ts, t_start);  // profiling: x1 seen
            if (w == 0) {  // the residual rows of this workgroup's o_net
                float xr = v[0];
#pragma unroll
                for (int j = 1; j < PER; ++j) xr = j == rb ? v[j] : xr;
                x1s[lane] = xr;
            }
            xq8_ln_quant(x, v, g, act, actq, actd);
            ts_phase<1>(p.ts, t_start);  // profiling: LN + quantised
#pragma unroll
            for (int j = 0; j < QR; ++j) {
                const float qv = xq8_dot(wq[j], wqs[j], qa, actq, actd);
                if (qa == 0) qs[16 * w + 64 * j + (lane >> 2)] = qv;
            }
            lds_sync();
            ts_phase<2>(p.ts, t_start);  // profiling: q done
            return (const float *)qs;
        },
        x.xak + kv, x.xav + kv, x.T[b], pr, a_s);
    ts_phase<3>(p.ts, t_start);  // profiling: attention done
    xa_quantize_a(a_s, aq, ad);
    xa_q8_onet<OG>(wo, wos, r0, aq, ad, x1s - rb * XQ8_ROWS, x.x2 + (size_t)b * D);
    ts_end(p.ts, t_start);
}

// f32 o_net: lane l holds elements 4l..4l+3 of half a row, a wave covers 2 rows
// per instruction; 64 rows = 4 waves x 8 pairs
__global__ __launch_bounds__(MP_BLOCK) void xa_f32_kernel(XaQ8P p) {
    constexpr int RP = XQ8_ROWS / MP_NWAVES / 2;  // row pairs per wave
    __shared__ float pr[TMAX_LIMIT];
    __shared__ __attribute__((aligned(16))) float a_s[DXA];
    const int b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r0 = blockIdx.x * XQ8_ROWS + w * 2 * RP, hr = lane >> 5, d4 = 4 * (lane & 31);
    float4 wo[RP];
#pragma unroll
    for (int i = 0; i < RP; ++i) wo[i] = *(const float4 *)(p.wof + (size_t)(r0 + 2 * i + hr) * DXA + d4);
    const size_t kv = ((size_t)(b * p.nlayers + p.layer) * p.Tmax) * DXA;
    xa_text_attention(p.q + (size_t)b * DXA, p.xak + kv, p.xav + kv, p.T[b], pr, a_s);
    const float4 a4 = *(const float4 *)&a_s[d4];
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < RP; ++i) {
        const float t = group_sum<32>(dotv(wo[i], a4));
        if ((lane & 31) == i) v = t;  // row r0 + 2 i + hr lands in lane i (+32)
    }
    if ((lane & 31) < RP) {
        const int row = r0 + 2 * (lane & 31) + hr;
        p.x2[(size_t)b * D + row] = v + p.x[(size_t)b * D + row];
    }
}

hipError_t op_xa_q8(const XaQ8P &p, int B, hipStream_t s) {
    if (!p.x || !p.x2 || !p.q || !p.xak || !p.xav || !p.T || p.Tmax < 1 || p.Tmax > TMAX_LIMIT) return hipErrorInvalidValue;
    if (p.wof) mp::launch(xa_f32_kernel, dim3(D / XQ8_ROWS, B), dim3(MP_BLOCK), 0, s, p);
    else if (p.wo && p.wod) mp::launch(xa_q8_kernel, dim3(D / XQ8_ROWS, B), dim3(MP_BLOCK), 0, s, p);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}

template <int PRO, int EPI>
static bool q8_args_ok(const GemvP &p) {
    if (!p.Wq || !p.Wd || p.N <= 0) return false;
    bool ok = true;
    if constexpr (PRO == PRO_PLAIN) ok &= p.src != nullptr;
    if constexpr (PRO == PRO_SA_MERGE) ok &= p.part != nullptr;
    if constexpr (PRO == PRO_LTFFN_MERGE || PRO == PRO_LTQ_MERGE) ok &= p.part && p.addsrc;
    if constexpr (PRO == PRO_XA_LN) ok &= p.part && p.src && p.lnw && p.xres;
    if constexpr (PRO == PRO_LN) ok &= p.src && p.lnw;
    if constexpr (PRO == PRO_LTX_LN) ok &= p.lt_s && p.lt_pos && p.ltX && p.lnw;
    if constexpr (PRO == PRO_LT_ATTN) ok &= p.ltq && p.ltk && p.ltv;
    if constexpr (PRO == PRO_LTARG_ATTN)
        ok &= p.logits && p.codes_cur && p.qkvtab && p.lk && p.lv && p.ltk && p.ltv && p.step && p.smp.cfg && p.smp.argeos;
    if constexpr (EPI == EPI_STORE || EPI == EPI_GELU) ok &= p.out != nullptr;
    if constexpr (EPI == EPI_BIAS) ok &= p.out && p.bias;
    if constexpr (EPI == EPI_RESID) ok &= p.resid != nullptr;
    if constexpr (EPI == EPI_ADD_STORE) ok &= p.out && p.addsrc;
    if constexpr (EPI == EPI_LTX_ADD) ok &= p.out && p.ptab && p.lt_pos && p.cb >= 1;
    if constexpr (EPI == EPI_QKV || EPI == EPI_QKV_SA) ok &= p.out && p.kc && p.vc && p.pos;
    if constexpr (EPI == EPI_QKV_SA) ok &= qkv_sa_args_ok(p);
    if constexpr (EPI == EPI_LTQKV) ok &= p.lq && p.lk && p.lv;
    if constexpr (EPI == EPI_RESID_XQ8) {
        const XaQ8P &x = p.xq8;
        ok &= p.resid && p.xh && p.iter && p.hx_err && p.N == D && x.qg && x.wq && x.wqd && x.lnw && x.x2 && x.wo &&
              x.wod && x.xak && x.xav && x.T && x.Tmax >= 1 && x.Tmax <= TMAX_LIMIT && x.layer == p.layer;
    }
    return ok;
}

template <int NB, int K, int PRO, int EPI>
static hipError_t launch_q8(const GemvP &p, hipStream_t s) {
    if (!q8_args_ok<PRO, EPI>(p)) return hipErrorInvalidValue;
    GemvP q = p;
    q.nrow_blocks = (p.N + 15) / 16;
    const int grid = q.nrow_blocks + (EPI == EPI_QKV_SA ? NH * SA_SPLITS * NB : EPI == EPI_RESID_XQ8 ? (NB <= XQ8_QIN_NB && p.xq8.qin ? XQ8A : XQG + XQ8A) * NB : 0);
    if (p.q4) mp::launch((gemm_q8_kernel_dec<NB, K, PRO, EPI, true>), dim3(grid), dim3(MP_BLOCK), 0, s, q);
    else mp::launch((gemm_q8_kernel_dec<NB, K, PRO, EPI, false>), dim3(grid), dim3(MP_BLOCK), 0, s, q);
    return hipGetLastError();
}

// Named entry points of the Q8_0 projections of one decode iteration (the
// pos_ff conv weights stay F32 in the reference's Q8 file and run on the f32
// GEMV family), instantiated for NB in {1, 2, 4, 8, 16}.
#define MP_Q8_OPS(NB)                                                                                                  \
    hipError_t q8_qkv_##NB(const GemvP &p, hipStream_t s) { return launch_q8<NB, D, PRO_LN, EPI_QKV>(p, s); }             \
    hipError_t q8_oproj_##NB(const GemvP &p, hipStream_t s) { return launch_q8<NB, D, PRO_SA_MERGE, EPI_RESID>(p, s); }      \
    hipError_t q8_xq_##NB(const GemvP &p, hipStream_t s) { return launch_q8<NB, D, PRO_LN, EPI_STORE>(p, s); }            \
    hipError_t q8_lt_in0_##NB(const GemvP &p, hipStream_t s) { return launch_q8<NB, D, PRO_LN, EPI_BIAS>(p, s); }         \
    hipError_t q8_lt_a_##NB(const GemvP &p, hipStream_t s) { return launch_q8<NB, LTD, PRO_LTX_LN, EPI_LTQKV>(p, s); }    \
    hipError_t q8_lt_bg_##NB(const GemvP &p, hipStream_t s) { return launch_q8<NB, LTD, PRO_LTARG_ATTN, EPI_LTX_ADD>(p, s); } \
    hipError_t q8_lt_b_##NB(const GemvP &p, hipStream_t s) { return launch_q8<NB, LTD, PRO_LT_ATTN, EPI_ADD_STORE>(p, s); } \
    hipError_t q8_lt_e_##NB(const GemvP &p, hipStream_t s) { return launch_q8<NB, LTD, PRO_PLAIN, EPI_BIAS>(p, s); } \
    hipError_t q8_qkv_sa_##NB(const GemvP &p, hipStream_t s) { return launch_q8<NB, D, PRO_LN, EPI_QKV_SA>(p, s); }   \
    hipError_t q8_oproj_xq_##NB(const GemvP &p, hipStream_t s) {                                                    \
        return launch_q8<NB, D, PRO_SA_MERGE, EPI_RESID_XQ8>(p, s);                                                  \
    }

MP_Q8_OPS(1)
MP_Q8_OPS(2)
MP_Q8_OPS(4)
MP_Q8_OPS(8)
MP_Q8_OPS(16)
// LT in_proj of a caller-supplied normalised hidden (magpie_local_transformer_sample_all)
hipError_t q8_lt_inh_1(const GemvP &p, hipStream_t s) { return launch_q8<1, D, PRO_PLAIN, EPI_BIAS>(p, s); }
// o_net + residual after lt_pick_kernel (large batches)
hipError_t q8_lt_bo_8(const GemvP &p, hipStream_t s) { return launch_q8<8, LTD, PRO_PLAIN, EPI_ADD_STORE>(p, s); }
hipError_t q8_lt_bo_16(const GemvP &p, hipStream_t s) { return launch_q8<16, LTD, PRO_PLAIN, EPI_ADD_STORE>(p, s); }
// the LT head at batch 1 with the LT FFN merge as its prologue (lt_ffn_kernel)
hipError_t q8_lt_em_1(const GemvP &p, hipStream_t s) { return launch_q8<1, LTD, PRO_LTQ_MERGE, EPI_BIAS>(p, s); }
// the same head after lt_ffn_kernel (the standalone LT sample of a Q8_0 file): its LT_FFN_P
// partials are interleaved (ltp_idx)
hipError_t q8_lt_emf_1(const GemvP &p, hipStream_t s) { return launch_q8<1, LTD, PRO_LTFFN_MERGE, EPI_BIAS>(p, s); }

}  // namespace mp
