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

#include "mp_device.hpp"
#include "mp_fused.hpp"
#include "mp_params.hpp"

namespace mp {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef int intx4 __attribute__((ext_vector_type(4)));

// max over the 4 lanes of a DPP quad
__device__ __forceinline__ float quad_max(float v) {
    v = fmaxf(v, dpp_mov<0xB1>(v));
    return fmaxf(v, dpp_mov<0x4E>(v));
}

template <int NB, int K, int PRO, int EPI>
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
    __shared__ __attribute__((aligned(16))) floatx4 part[MP_NWAVES][64];
    __shared__ float red[8];
    __shared__ float sc[SC];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, rt = blockIdx.x;

    // this wave's weight fragments and their scales, issued before the prologue
    const uint4 *wf = (const uint4 *)p.Wq + ((size_t)rt * KP + w * KW) * 64 + lane + ts_dep(t_start);
    const uint4 *sf = (const uint4 *)p.Wd + ((size_t)rt * KP + w * KW) * 4 + (lane >> 4);
    uint4 a[KW], sd[KW];
#pragma unroll
    for (int i = 0; i < KW; ++i) { a[i] = wf[(size_t)i * 64]; sd[i] = sf[(size_t)i * 4]; }

    prologue<NB, K, PRO>(p, act, red, sc);

    // activation rows -> Q8_0 (quantize_row_q8_0_ref), 4 lanes x 8 elements per block;
    // row NB is zero (q = 0, d = 0) and feeds MFMA columns NB..15
    for (int e = tid; e < (QS + 4 * NBLK) / 4; e += MP_BLOCK) {
        if (e < QS / 4) ((int *)(actq + NB * QS))[e] = 0;
        else actd[NB * NBLK + (e - QS / 4)] = 0.f;
    }
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
#pragma unroll
        for (int j = 0; j < 8; ++j) qw[j >> 2] |= ((unsigned)(int)roundf(xs[j] * id) & 0xFFu) << (8 * (j & 3));
        *(uint2 *)(actq + b * QS + kb * 32 + e8) = make_uint2(qw[0], qw[1]);
        if ((lane & 3) == 0) actd[blk] = __half2float(__float2half(dd));
    }
    lds_sync();
    ts_mark(p.ts, t_start);  // profiling: activation tile quantised

    const int c = min(lane & 15, NB);
    const signed char *bq = actq + c * QS + 8 * (lane >> 4);
    const float *bd = actd + c * NBLK;
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < KW; ++i) {
        const int kp = w * KW + i;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int kc = 2 * kp + h;
            const long av = h ? (long)(((unsigned long)a[i].w << 32) | a[i].z)
                              : (long)(((unsigned long)a[i].y << 32) | a[i].x);
            const long bv = *(const long *)(bq + kc * 32);
            const intx4 zero = {0, 0, 0, 0};
            const intx4 s = __builtin_amdgcn_mfma_i32_16x16x32_i8(av, bv, zero, 0, 0, 0);
            const float da = bd[kc];
            const unsigned dlo = h ? sd[i].z : sd[i].x, dhi = h ? sd[i].w : sd[i].y;  // rows 4g..4g+3
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const unsigned wd = r < 2 ? dlo : dhi;
                const float dw = __half2float(__ushort_as_half((unsigned short)((r & 1) ? wd >> 16 : wd & 0xFFFFu)));
                acc[r] += (float)s[r] * (dw * da);
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
    epi_store<EPI>(p, v, n, col, EPI == EPI_LTX_ADD ? sc[col * LTD + n] : 0.f);
    ts_end(p.ts, t_start);
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
    if (!q || !d || !oq || !od || N <= 0 || K % 256) return hipErrorInvalidValue;
    mp::launch(pack_q8_kernel, dim3(1024), dim3(256), 0, s, q, d, N, K, oq, od);
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

// a = softmax_t(q . K_t / sqrt(128)) V  of slot b into a_s[128] (every thread
// returns after a barrier); pr: per-key scores [TMAX_LIMIT]
__device__ __forceinline__ void xa_text_attention(const float *q, const float *Kb, const float *Vb, int Tb,
                                                  float *pr, float *a_s) {
    __shared__ __attribute__((aligned(16))) float pv[MP_NWAVES][DXA];
    __shared__ float wred[2 * MP_NWAVES];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int h = lane >> 5, d4 = 4 * (lane & 31);
    const float4 q4 = *(const float4 *)(q + d4);
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
    if (tid < DXA) {
        const float den = ((wred[4] + wred[5]) + wred[6]) + wred[7];
        a_s[tid] = (((pv[0][tid] + pv[1][tid]) + pv[2][tid]) + pv[3][tid]) / den;
    }
    lds_sync();
}

__global__ __launch_bounds__(MP_BLOCK) void xa_q8_kernel(XaQ8P p) {
    constexpr int OR = 8, OCPR = DXA / 16;                 // o_net: groups of 8 rows
    constexpr int OG = XQ8_ROWS / MP_NWAVES / OR;          // 2 groups per wave
    __shared__ float pr[TMAX_LIMIT];
    __shared__ __attribute__((aligned(16))) float a_s[DXA];
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
    const size_t kv = ((size_t)(b * p.nlayers + p.layer) * p.Tmax) * DXA;
    xa_text_attention(p.q + (size_t)b * DXA, p.xak + kv, p.xav + kv, p.T[b], pr, a_s);
    if (w == 0) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {  // element lane + 64 i; its Q8_0 block = this half-wave
            const float av = a_s[lane + 64 * i];
            float a = row_max16(fabsf(av));
            a = fmaxf(a, __shfl_xor(a, 16, 64));
            const float dd = a / 127.0f;
            const float id = dd != 0.f ? 1.0f / dd : 0.0f;
            aq[lane + 64 * i] = (signed char)(int)roundf(av * id);
            if ((lane & 31) == 0) ad[(lane + 64 * i) / 32] = __half2float(__float2half(dd));
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
    if constexpr (PRO == PRO_LTFFN_MERGE) ok &= p.part && p.addsrc;
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
    if constexpr (EPI == EPI_QKV) ok &= p.out && p.kc && p.vc && p.pos;
    if constexpr (EPI == EPI_LTQKV) ok &= p.lq && p.lk && p.lv;
    return ok;
}

template <int NB, int K, int PRO, int EPI>
static hipError_t launch_q8(const GemvP &p, hipStream_t s) {
    if (!q8_args_ok<PRO, EPI>(p)) return hipErrorInvalidValue;
    mp::launch((gemm_q8_kernel_dec<NB, K, PRO, EPI>), dim3((p.N + 15) / 16), dim3(MP_BLOCK), 0, s, p);
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
    hipError_t q8_lt_e_##NB(const GemvP &p, hipStream_t s) { return launch_q8<NB, LTD, PRO_PLAIN, EPI_BIAS>(p, s); }

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
hipError_t q8_lt_em_1(const GemvP &p, hipStream_t s) { return launch_q8<1, LTD, PRO_LTFFN_MERGE, EPI_BIAS>(p, s); }

}  // namespace mp
