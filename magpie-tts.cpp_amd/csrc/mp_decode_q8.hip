// Q8_0 weight mode of the decode projections (gfx950), batch NB <= 8.
//
// The reference's Q8 GGUF stores the attention / cross-attention / LT
// projections as Q8_0 blocks (scripts/convert_magpie_to_gguf.py:155-176: per 32
// weights an fp16 scale d and 32 int8 q) and ggml multiplies them with its
// quantised mul_mat: the activation row is itself quantised to Q8_0
// (quantize_row_q8_0_ref: d = amax/127, id = 1/d, q = roundf(x*id), d kept as
// fp16) and every block contributes its exact integer dot times d_w * d_a
// (ggml_vec_dot_q8_0_q8_0). This file computes exactly that, per
// decode step, as a weight-streaming GEMV:
//
//  * weights stay int8 in HBM (1 B/param + 2 B per 32: 34/32 B/param as in the
//    file, 26 % of f32), repacked once at load into int8 [N][K] + fp16 scales
//    [N][K/32] so each lane streams a 16-byte half block (one 1 KiB coalesced
//    wave-instruction over rows that are contiguous in memory);
//  * the prologue (LN / frame embedding / LT pick + gather / LT attention,
//    shared with the f32 and bf16 families, mp_fused.hpp) builds the f32
//    activation rows in LDS, then 32 lanes per block quantise them to Q8_0 in
//    LDS (amax by DPP);
//  * the two halves of a block (adjacent lanes) are dotted with v_dot4c_i32_i8
//    and summed exactly by one DPP swap, scaled by d_w * d_a, and accumulated
//    per output row; rows are then reduced across the wave by DPP.
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <math.h>

#include "mp_device.hpp"
#include "mp_fused.hpp"
#include "mp_params.hpp"

namespace mp {

// Rows [row0, row0 + R) of W are R*K contiguous bytes: 16-byte chunk c = lane +
// 64 j of the wave belongs to row c / (K/16), half block (c % (K/16)) of it.
template <int NB, int K, int R, int PRO, int EPI>
__global__ __launch_bounds__(MP_BLOCK) void gemv_q8_kernel(GemvP p) {
    constexpr int CPR = K / 16;    // 16-byte chunks per row
    constexpr int NBLK = K / 32;   // Q8_0 blocks per row
    constexpr int J = R * CPR / 64;
    static_assert(R * CPR % 64 == 0, "a wave's rows must fill whole wave-instructions");
    static_assert(R * NB <= 64, "one lane per output");
    constexpr int SC = pro_scratch<NB, PRO>();
    __shared__ __attribute__((aligned(16))) float act[NB * K];
    __shared__ __attribute__((aligned(16))) signed char actq[NB * K];
    __shared__ float actd[NB * NBLK];
    __shared__ float red[8];
    __shared__ float sc[SC];

    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int row0 = (blockIdx.x * MP_NWAVES + w) * R;
    // the weight stream (and its scales) does not depend on the prologue: issue it first
    uint4 wv[J];
    float ws[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int c = lane + 64 * j;
        const int n = min(row0 + c / CPR, p.N - 1);
        wv[j] = *(const uint4 *)(p.Wq + (size_t)n * K + (c % CPR) * 16);
        ws[j] = __half2float(__ushort_as_half(p.Wd[(size_t)n * NBLK + (c % CPR) / 2]));
    }
    prologue<NB, K, PRO>(p, act, red, sc);

    // activation rows -> Q8_0 (quantize_row_q8_0_ref), 32 lanes per block
    {
        const int e = lane & 31;
        for (int blk = 2 * w + (lane >> 5); blk < NB * NBLK; blk += 2 * MP_NWAVES) {
            const float x = act[blk * 32 + e];
            float a = row_max16(fabsf(x));
            a = fmaxf(a, __shfl_xor(a, 16, 64));
            const float dd = a / 127.0f;
            const float id = dd != 0.f ? 1.0f / dd : 0.0f;
            actq[blk * 32 + e] = (signed char)(int)roundf(x * id);
            if (e == 0) actd[blk] = __half2float(__float2half(dd));
        }
        lds_sync();
    }

    float acc[R][NB];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int b = 0; b < NB; ++b) acc[r][b] = 0.f;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int c = lane + 64 * j;
        const int r = c / CPR, kc = c % CPR;
        const int r_lo = (64 * j) / CPR, r_hi = (64 * j + 63) / CPR;  // rows this wave-instruction touches
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            const int4 a4 = *(const int4 *)(actq + b * K + kc * 16);
            int s = __builtin_amdgcn_sdot4((int)wv[j].x, a4.x, 0, false);
            s = __builtin_amdgcn_sdot4((int)wv[j].y, a4.y, s, false);
            s = __builtin_amdgcn_sdot4((int)wv[j].z, a4.z, s, false);
            s = __builtin_amdgcn_sdot4((int)wv[j].w, a4.w, s, false);
            s += __builtin_amdgcn_update_dpp(0, s, 0xB1, 0xF, 0xF, false);  // + the other half of the block
            const float f = (lane & 1) ? 0.f : (float)s * (ws[j] * actd[b * NBLK + (kc >> 1)]);
#pragma unroll
            for (int rr = r_lo; rr <= r_hi; ++rr) acc[rr][b] += (r == rr) ? f : 0.f;
        }
    }
    float v = 0.f;
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            const float t = wave_sum(acc[r][b]);
            if (lane == r * NB + b) v = t;
        }
    if (lane >= R * NB) return;
    const int b = lane % NB, n = row0 + lane / NB;
    if (n >= p.N) return;
    epi_store<EPI>(p, v, n, b, EPI == EPI_LTX_ADD ? sc[b * LTD + n] : 0.f);
}

// ---------------------------------------------------------------- fused Q8 XA tail
// Cross-attention with Q8_0 q_net / o_net: q = Q8(q_net) LN(x) is one GEMV
// launch (q8_xq, 8 workgroups: q_net's 98 KB spread over CUs); this kernel then
// does attention + o_net + residual: grid (768/64, B), a workgroup owns 64 rows
// of o_net and recomputes the slot's attention over the text (K, V: 2 x T x 128
// f32, coalesced: half a wave per key row), quantises it to Q8_0 and finishes
// x2 = x + Q8(o_net) a for its rows with gemv_q8<.., 128, 8, PRO_PLAIN,
// EPI_ADD_STORE>'s arithmetic. The o_net rows are issued first.
constexpr int XQ8_ROWS = 64;  // o_net rows per workgroup
__global__ __launch_bounds__(MP_BLOCK) void xa_q8_kernel(XaQ8P p) {
    constexpr int OR = 8, OCPR = DXA / 16;                 // o_net: groups of 8 rows
    constexpr int OG = XQ8_ROWS / MP_NWAVES / OR;          // 2 groups per wave
    __shared__ float pr[TMAX_LIMIT];
    __shared__ __attribute__((aligned(16))) signed char aq[DXA];
    __shared__ float ad[DXA / 32];
    const int b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r0 = blockIdx.x * XQ8_ROWS;
    uint4 wo[OG];
    float wos[OG];
#pragma unroll
    for (int g = 0; g < OG; ++g) {
        const int row = r0 + (w * OG + g) * OR + lane / OCPR, kc = lane % OCPR;
        wo[g] = *(const uint4 *)(p.wo + (size_t)row * DXA + kc * 16);
        wos[g] = __half2float(__ushort_as_half(p.wod[(size_t)row * (DXA / 32) + kc / 2]));
    }
    // ---- attention over the utterance's text, coalesced: a half-wave (32 lanes x
    //      float4) covers one 128-dim key row; wave w scores keys t = w + 4 u
    __shared__ __attribute__((aligned(16))) float pv[MP_NWAVES][DXA];
    __shared__ float wred[2 * MP_NWAVES];
    {
        const int Tb = p.T[b];
        const int h = lane >> 5, d4 = 4 * (lane & 31);
        const float4 q4 = *(const float4 *)(p.q + (size_t)b * DXA + d4);
        const float *Kb = p.xak + ((size_t)(b * p.nlayers + p.layer) * p.Tmax) * DXA;
        const float *Vb = p.xav + ((size_t)(b * p.nlayers + p.layer) * p.Tmax) * DXA;
        const float scale = 1.0f / sqrtf((float)DXA);
        float mx = -INFINITY;
        for (int t0 = 2 * w; t0 < Tb; t0 += 2 * MP_NWAVES * 4) {  // 4 key pairs in flight per wave
            float4 k4[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int t = min(t0 + 2 * MP_NWAVES * u + h, Tb - 1);
                k4[u] = *(const float4 *)(Kb + (size_t)t * DXA + d4);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int t = t0 + 2 * MP_NWAVES * u + h;
                const float sv = group_sum<32>(dotv(q4, k4[u])) * scale;
                if (t < Tb) {
                    if ((lane & 31) == 0) pr[t] = sv;
                    mx = fmaxf(mx, sv);
                }
            }
        }
        mx = wave_max(mx);
        if (lane == 0) wred[w] = mx;
        lds_sync();
        const float M = fmaxf(fmaxf(wred[0], wred[1]), fmaxf(wred[2], wred[3]));
        // o[d] = sum_t e_t V_t[d]: wave w takes keys t = w + 4 u, lane owns dims lane, 64 + lane
        float l = 0.f, o0 = 0.f, o1 = 0.f;
        for (int t0 = w; t0 < Tb; t0 += MP_NWAVES * 4) {
            float v0[4], v1[4], e[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int t = min(t0 + MP_NWAVES * u, Tb - 1);
                v0[u] = Vb[(size_t)t * DXA + lane];
                v1[u] = Vb[(size_t)t * DXA + 64 + lane];
                e[u] = t0 + MP_NWAVES * u < Tb ? expf(pr[t] - M) : 0.f;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) { l += e[u]; o0 += e[u] * v0[u]; o1 += e[u] * v1[u]; }
        }
        pv[w][lane] = o0;
        pv[w][64 + lane] = o1;
        if (lane == 0) wred[MP_NWAVES + w] = l;
        lds_sync();
        if (w == 0) {
            const float den = ((wred[4] + wred[5]) + wred[6]) + wred[7];
            float av[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int d = lane + 64 * i;
                av[i] = (((pv[0][d] + pv[1][d]) + pv[2][d]) + pv[3][d]) / den;
            }
#pragma unroll
            for (int i = 0; i < 2; ++i) {  // element lane + 64 i; its Q8_0 block = this half-wave
                float a = row_max16(fabsf(av[i]));
                a = fmaxf(a, __shfl_xor(a, 16, 64));
                const float dd = a / 127.0f;
                const float id = dd != 0.f ? 1.0f / dd : 0.0f;
                aq[lane + 64 * i] = (signed char)(int)roundf(av[i] * id);
                if ((lane & 31) == 0) ad[(lane + 64 * i) / 32] = __half2float(__float2half(dd));
            }
        }
    }
    lds_sync();
    // ---- x2 = x + Q8(o_net) a for this workgroup's 64 rows (8 per group)
#pragma unroll
    for (int g = 0; g < OG; ++g) {
        const int r = lane / OCPR, kc = lane % OCPR;
        const int4 a4 = *(const int4 *)(aq + kc * 16);
        int s = __builtin_amdgcn_sdot4((int)wo[g].x, a4.x, 0, false);
        s = __builtin_amdgcn_sdot4((int)wo[g].y, a4.y, s, false);
        s = __builtin_amdgcn_sdot4((int)wo[g].z, a4.z, s, false);
        s = __builtin_amdgcn_sdot4((int)wo[g].w, a4.w, s, false);
        s += __builtin_amdgcn_update_dpp(0, s, 0xB1, 0xF, 0xF, false);
        const float f = (lane & 1) ? 0.f : (float)s * (wos[g] * ad[kc >> 1]);
        float v = 0.f;
#pragma unroll
        for (int rr = 0; rr < OR; ++rr) {
            const float t = wave_sum((r == rr) ? f : 0.f);
            if (lane == rr) v = t;
        }
        if (lane < OR) {
            const int row = r0 + (w * OG + g) * OR + lane;
            p.x2[(size_t)b * D + row] = v + p.x[(size_t)b * D + row];
        }
    }
}

hipError_t op_xa_q8(const XaQ8P &p, int B, hipStream_t s) {
    if (!p.x || !p.x2 || !p.q || !p.wo || !p.wod || !p.xak || !p.xav || !p.T || p.Tmax < 1 ||
        p.Tmax > TMAX_LIMIT)
        return hipErrorInvalidValue;
    mp::launch(xa_q8_kernel, dim3(D / XQ8_ROWS, B), dim3(MP_BLOCK), 0, s, p);
    return hipGetLastError();
}

template <int PRO, int EPI>
static bool q8_args_ok(const GemvP &p) {
    if (!p.Wq || !p.Wd || p.N <= 0) return false;
    bool ok = true;
    if constexpr (PRO == PRO_PLAIN) ok &= p.src != nullptr;
    if constexpr (PRO == PRO_SA_MERGE) ok &= p.part != nullptr;
    if constexpr (PRO == PRO_LTFFN_MERGE) ok &= p.part && p.addsrc;
    if constexpr (PRO == PRO_XA_LN) ok &= p.part && p.src && p.lnw && p.xres;
    if constexpr (PRO == PRO_LN) ok &= p.src && p.lnw;
    if constexpr (PRO == PRO_EMBED_LN) ok &= p.emb && p.codes && p.pos_emb && p.pos && p.xres && p.lnw;
    if constexpr (PRO == PRO_LTX_LN) ok &= p.lt_s && p.lt_pos && p.ltX && p.lnw;
    if constexpr (PRO == PRO_LT_ATTN) ok &= p.ltq && p.ltk && p.ltv;
    if constexpr (PRO == PRO_LTARG_ATTN)
        ok &= p.logits && p.codes_cur && p.qkvtab && p.lk && p.lv && p.ltk && p.ltv && p.step && p.smp.cfg && p.smp.argeos;
    if constexpr (EPI == EPI_STORE || EPI == EPI_GELU) ok &= p.out != nullptr;
    if constexpr (EPI == EPI_BIAS) ok &= p.out && p.bias;
    if constexpr (EPI == EPI_RESID) ok &= p.resid != nullptr;
    if constexpr (EPI == EPI_ADD_STORE) ok &= p.out && p.addsrc;
    if constexpr (EPI == EPI_LTX_ADD) ok &= p.out && p.ptab && p.lt_pos && p.cb >= 1;
    if constexpr (EPI == EPI_QKV) ok &= p.out && p.kc && p.vc && p.pos;
    if constexpr (EPI == EPI_LTQKV) ok &= p.lq && p.lk && p.lv;
    return ok;
}

template <int NB, int K, int R, int PRO, int EPI>
static hipError_t launch_q8(const GemvP &p, hipStream_t s) {
    if (!q8_args_ok<PRO, EPI>(p)) return hipErrorInvalidValue;
    const int rows = MP_NWAVES * R;
    mp::launch((gemv_q8_kernel<NB, K, R, PRO, EPI>), dim3((p.N + rows - 1) / rows), dim3(MP_BLOCK), 0, s, p);
    return hipGetLastError();
}

// Named entry points of the Q8_0 projections of one decode iteration (the
// pos_ff conv weights stay F32 in the reference's Q8 file and run on the f32
// GEMV family), instantiated for NB in {1, 2, 4, 8}.
#define MP_Q8_OPS(NB)                                                                                                  \
    hipError_t q8_qkv_embed_##NB(const GemvP &p, hipStream_t s) { return launch_q8<NB, D, 4, PRO_EMBED_LN, EPI_QKV>(p, s); } \
    hipError_t q8_qkv_##NB(const GemvP &p, hipStream_t s) { return launch_q8<NB, D, 4, PRO_LN, EPI_QKV>(p, s); }             \
    hipError_t q8_oproj_##NB(const GemvP &p, hipStream_t s) { return launch_q8<NB, D, 4, PRO_SA_MERGE, EPI_RESID>(p, s); }      \
    hipError_t q8_xq_##NB(const GemvP &p, hipStream_t s) { return launch_q8<NB, D, 4, PRO_LN, EPI_STORE>(p, s); }            \
    hipError_t q8_lt_in0_##NB(const GemvP &p, hipStream_t s) { return launch_q8<NB, D, 4, PRO_LN, EPI_BIAS>(p, s); }         \
    hipError_t q8_lt_a_##NB(const GemvP &p, hipStream_t s) { return launch_q8<NB, LTD, 4, PRO_LTX_LN, EPI_LTQKV>(p, s); }    \
    hipError_t q8_lt_bg_##NB(const GemvP &p, hipStream_t s) { return launch_q8<NB, LTD, 4, PRO_LTARG_ATTN, EPI_LTX_ADD>(p, s); } \
    hipError_t q8_lt_b_##NB(const GemvP &p, hipStream_t s) { return launch_q8<NB, LTD, 4, PRO_LT_ATTN, EPI_ADD_STORE>(p, s); } \
    hipError_t q8_lt_e_##NB(const GemvP &p, hipStream_t s) { return launch_q8<NB, LTD, 4, PRO_PLAIN, EPI_BIAS>(p, s); }

MP_Q8_OPS(1)
MP_Q8_OPS(2)
MP_Q8_OPS(4)
MP_Q8_OPS(8)
// LT in_proj of a caller-supplied normalised hidden (magpie_local_transformer_sample_all)
hipError_t q8_lt_inh_1(const GemvP &p, hipStream_t s) { return launch_q8<1, D, 4, PRO_PLAIN, EPI_BIAS>(p, s); }
// o_net + residual after lt_pick_kernel (large batches)
hipError_t q8_lt_bo_8(const GemvP &p, hipStream_t s) { return launch_q8<8, LTD, 4, PRO_PLAIN, EPI_ADD_STORE>(p, s); }
// the LT head at batch 1 with the LT FFN merge as its prologue (lt_ffn_kernel)
hipError_t q8_lt_em_1(const GemvP &p, hipStream_t s) { return launch_q8<1, LTD, 4, PRO_LTFFN_MERGE, EPI_BIAS>(p, s); }

}  // namespace mp
