// Fused-projection building blocks shared by the f32 GEMV kernels
// (mp_decode.hip) and the bf16 MFMA kernels (mp_decode_b16.hip): the prologues
// that build the activation rows in LDS, the code pick (argmax / top-k draw) of
// the local transformer, and the epilogues.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

#include <type_traits>

#include "mp_device.hpp"
#include "mp_params.hpp"

namespace mp {

// ---------------------------------------------------------------- prologues
// Each prologue fills act[NB][K] (LDS) with the activation vector of every slot.


// One wave picks slot b's code for codebook `cb` of this frame: masked first-max
// argmax (always, for EOS detection, magpie.cpp:1250-1259), and at temperature
// >= 0.01 a top-k draw with the reference's sample_top_k arithmetic
// (magpie.cpp:1072-1109): the k largest masked logits in descending order (ties by
// ascending index), p_i = exp((l_i - l_max) / T) summed sequentially, normalised,
// and the first i with u < cumsum_i (fallback: the k-th). Radix-select finds the
// k-th key, a ballot compaction gathers the k candidates into LDS, a counting rank
// orders them, lane 0 runs the two sequential float loops. scratch: 2*VCB floats.
// `stream` is the batch slot; the draw stream is cfg->stream_base + slot.
constexpr int PICK_R = (VCB + 63) / 64;  // logits per lane
__device__ __forceinline__ void load_logits(const float *lg, float (&lv)[PICK_R]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int r = 0; r < PICK_R; ++r) {
        const int i = lane + 64 * r;
        lv[r] = i < VCB ? lg[i] : -INFINITY;
    }
}
// wave_pick on logits already loaded by load_logits (lv is modified)
__device__ inline int wave_pick_v(float (&lv)[PICK_R], bool forbid_eos, int audio_bos, int audio_eos,
                                  const Sampling &smp, int stream, int step, int cb, float *scratch, int &amax) {
    const int lane = threadIdx.x & 63;
    constexpr int R = PICK_R;
    // masked first-max argmax. The forbidden ids (audio_bos .. audio_bos + 7 but EOS, and
    // the padding past VCB) lie in the rows r whose 64 ids reach audio_bos or VCB: a
    // uniform (scalar) test per row skips the per-lane mask everywhere else. Then the
    // wave's max by DPP, and the first index holding it as the wave's minimum of each
    // lane's first matching index (VALU compares and one DPP min: no ballot / scalar
    // round trip per row). Same value and index as a scan of i = 0, 1, ... with '>'.
    // The reference's ids (magpie.h: audio_bos = 2016 = VCB - 8) put every forbidden id
    // in the last row, lanes (VCB - 8) % 64 .. 63: that row alone is masked, with lane
    // arithmetic only (a per-row mask mixing VALU compares and scalar logic cost ~0.8 us).
    // Any other audio_bos takes the general per-row mask (uniform branch).
    constexpr int RL = (VCB - 8) / 64, LL = (VCB - 8) % 64;
    static_assert(RL == R - 1 && (VCB - 1) / 64 == RL, "the 8 special ids and the padding share the last row");
    if (audio_bos == VCB - 8) {
        const int i = lane + 64 * RL;
        if (lane >= LL && (i >= VCB || i != audio_eos || forbid_eos)) lv[RL] = -INFINITY;
    } else {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int i = lane + 64 * r;
            if (i >= VCB || ((unsigned)(i - audio_bos) <= 7u && (i != audio_eos || forbid_eos))) lv[r] = -INFINITY;
        }
    }
    float bv = -INFINITY;
#pragma unroll
    for (int r = 0; r < R; ++r) bv = fmaxf(bv, lv[r]);
    bv = wave_max(bv);
    int first = 1 << 30;
#pragma unroll
    for (int r = R - 1; r >= 0; --r)
        if (lv[r] == bv) first = lane + 64 * r;
    int bi = wave_min_u(first);
    if (bi < 0 || bi >= VCB) bi = 0;
    amax = bi;
    if (!smp.on) return bi;
    const float temp = smp.cfg->temperature;
    const float M = bv;
    const int k = min(max(smp.cfg->top_k, 1), VCB);
    // order-preserving keys; padding lanes get 0 (below every real key)
    unsigned key[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const unsigned u = __float_as_uint(lv[r]);
        key[r] = (lane + 64 * r) < VCB ? ((u & 0x80000000u) ? ~u : (u | 0x80000000u)) : 0u;
    }
    unsigned t = 0;
    for (int bit = 31; bit >= 0; --bit) {
        const unsigned cand = t | (1u << bit);
        int c = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) c += key[r] >= cand;
        if ((int)wave_sum((float)c) >= k) t = cand;
    }
    int cgt = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) cgt += key[r] > t;
    const int need = k - (int)wave_sum((float)cgt);
    float *sv = scratch;
    int *si = (int *)(scratch + VCB);
    const unsigned long long below = (1ull << lane) - 1ull;
    int ties = 0, base = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const bool tie = key[r] == t;
        const unsigned long long bt = __ballot(tie);
        const bool sel = key[r] > t || (tie && ties + __popcll(bt & below) < need);
        ties += __popcll(bt);
        const unsigned long long bs = __ballot(sel);
        if (sel) {
            const int q = base + __popcll(bs & below);
            sv[q] = lv[r];
            si[q] = lane + 64 * r;
        }
        base += __popcll(bs);
    }
    wave_lds_sync();
    // counting rank (descending value, ascending index), then scatter in place
    constexpr int RK = (VCB + 63) / 64;
    float ev[RK];
    int ei[RK], rk[RK];
    for (int j = 0; j < RK; ++j) {
        const int e = lane + 64 * j;
        if (j * 64 >= k) break;
        if (e < k) {
            const float v = sv[e];
            const int i = si[e];
            int rank = 0;
            for (int e2 = 0; e2 < k; ++e2) {
                const float v2 = sv[e2];
                rank += (v2 > v) || (v2 == v && si[e2] < i);
            }
            rk[j] = rank;
            ev[j] = expf((v - M) / temp);
            ei[j] = i;
        }
    }
    wave_lds_sync();
    for (int j = 0; j < RK; ++j) {
        if (j * 64 >= k) break;
        if (lane + 64 * j < k) { sv[rk[j]] = ev[j]; si[rk[j]] = ei[j]; }
    }
    wave_lds_sync();
    int code = 0;
    if (lane == 0) {
        float sum = 0.f;
        for (int i = 0; i < k; ++i) sum += sv[i];
        const float u = mp_uniform(smp.cfg->seed, smp.cfg->stream_base + stream, step, cb);
        float cum = 0.f;
        code = si[k - 1];
        for (int i = 0; i < k; ++i) {
            cum += sv[i] / sum;
            if (u < cum) { code = si[i]; break; }
        }
    }
    code = __shfl(code, 0, 64);
    wave_lds_sync();
    return code;
}
__device__ inline int wave_pick(const float *lg, bool forbid_eos, int audio_bos, int audio_eos, const Sampling &smp,
                                int stream, int step, int cb, float *scratch, int &amax) {
    float lv[PICK_R];
    load_logits(lg, lv);
    return wave_pick_v(lv, forbid_eos, audio_bos, audio_eos, smp, stream, step, cb, scratch, amax);
}

// The greedy pick split over a workgroup's MP_NWAVES waves (batch-1 LT step, finalize):
// wave w scans logit rows [w QPR, (w + 1) QPR).
constexpr int QPR = PICK_R / MP_NWAVES;
static_assert(PICK_R % MP_NWAVES == 0 && (PICK_R - 1) / QPR == MP_NWAVES - 1, "logit rows split over the waves");
// this wave's masked (max, first index) over its rows; the same mask as wave_pick_v
__device__ __forceinline__ int wave_pick_rows(float (&lv)[QPR], int w, bool forbid_eos, int audio_bos, int audio_eos,
                                              float &bv) {
    const int lane = threadIdx.x & 63;
    constexpr int RL = (VCB - 8) / 64, LL = (VCB - 8) % 64;
    if (audio_bos == VCB - 8) {
        if (w == RL / QPR) {
            const int i = lane + 64 * RL;
            if (lane >= LL && (i >= VCB || i != audio_eos || forbid_eos)) lv[RL % QPR] = -INFINITY;
        }
    } else {
#pragma unroll
        for (int q = 0; q < QPR; ++q) {
            const int i = lane + 64 * (w * QPR + q);
            if (i >= VCB || ((unsigned)(i - audio_bos) <= 7u && (i != audio_eos || forbid_eos))) lv[q] = -INFINITY;
        }
    }
    bv = -INFINITY;
#pragma unroll
    for (int q = 0; q < QPR; ++q) bv = fmaxf(bv, lv[q]);
    bv = wave_max(bv);
    int first = 1 << 30;
#pragma unroll
    for (int q = QPR - 1; q >= 0; --q)
        if (lv[q] == bv) first = lane + 64 * (w * QPR + q);
    return wave_min_u(first);
}

// A logit as an ordered 64-bit key: the float's bits mapped to an unsigned order (high word)
// and 0xFFFFFFFF - index (low word), so the largest key is the largest value at the lowest
// index: the masked first-max argmax of wave_pick_rows / sample_top_k's greedy branch. 0 is
// below every real key (a forbidden id).
__device__ __forceinline__ unsigned long long lt_cand_key(float v, int i) {
    const unsigned u = __float_as_uint(v);
    const unsigned o = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    return ((unsigned long long)o << 32) | (0xFFFFFFFFu - (unsigned)i);
}
__device__ __forceinline__ float lt_cand_value(unsigned long long k) {
    const unsigned o = (unsigned)(k >> 32);
    return __uint_as_float((o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o);
}
__device__ __forceinline__ int lt_cand_index(unsigned long long k) { return (int)(0xFFFFFFFFu - (unsigned)k); }
__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long k) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const unsigned lo = __shfl_xor((unsigned)k, off), hi = __shfl_xor((unsigned)(k >> 32), off);
        const unsigned long long o = ((unsigned long long)hi << 32) | lo;
        k = o > k ? o : k;
    }
    return k;
}
// Whether logit i is forbidden (sample_top_k's mask, magpie.cpp:1237-1248): the 8 special
// audio ids except EOS, and EOS too while forbid_eos.
__device__ __forceinline__ bool lt_forbidden(int i, bool forbid_eos, int audio_bos, int audio_eos) {
    return i >= VCB || ((unsigned)(i - audio_bos) <= 7u && (i != audio_eos || forbid_eos));
}

// The split pick's exchange: every wave's (max, first index) pair through LDS; returns the
// first wave holding the workgroup-wide maximum (its first index is the global first
// index: its ids are the lowest among the waves at that value) and its index in `code`.
// Every wave of the workgroup calls it (one barrier).
__device__ __forceinline__ int pick_exchange(float bv, int bi, int &code) {
    __shared__ float qv[MP_NWAVES];
    __shared__ int qi[MP_NWAVES];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { qv[w] = bv; qi[w] = bi; }
    lds_sync();
    float gm = qv[0];
    int win = 0;
#pragma unroll
    for (int u = 1; u < MP_NWAVES; ++u)
        if (qv[u] > gm) { gm = qv[u]; win = u; }
    code = qi[win];
    return win;
}

// PRO_LTARG_ATTN keeps each slot's residual row X = P[cb-1][code] + lt_pos[cb] in
// sc[b*LTD ..] (the EPI_LTX_ADD epilogue adds it); the wave pick scratch follows.
template <int NB>
constexpr int ltc_off() { return NB * LTD; }

// Causal 1-head attention of LT position cb over positions 0..cb for slot b,
// one wave: lane l owns elements 4l..4l+3; scores are wave-wide DPP sums
// (softmax(K q / 16) V, magpie.cpp:965-966). Position cb's k/v are kc4/vc4
// (gathered this launch) when CUR, else row cb of ltk/ltv; earlier positions come
// from kr/vr when PRE (loaded ahead by the caller), else from ltk/ltv. The
// arithmetic is the same either way, at every batch size.
// Inlined (a __noinline__ copy took its arrays through scratch memory); the rounding is
// pinned instead (contraction off, explicit fmaf), so every caller computes the same bits.
__device__ __forceinline__ float dot4_pinned(float4 a, float4 b) { return dotv(a, b); }
template <bool CUR, bool PRE>
__device__ __forceinline__ float4 lt_attend(const GemvP &p, int b, float4 q4, float4 kc4, float4 vc4,
                                            const float4 (&kr)[NCB], const float4 (&vr)[NCB]) {
#pragma clang fp contract(off)
    const int lane = threadIdx.x & 63;
    const int nk = p.cb + 1;
    const float *kb = p.ltk + (size_t)b * NCB * LTD + 4 * lane, *vb = p.ltv + (size_t)b * NCB * LTD + 4 * lane;
    float sj[NCB];
#pragma unroll
    for (int j = 0; j < NCB; ++j) {
        if (j < nk) {
            const float4 k4 = (CUR && j == p.cb) ? kc4 : PRE ? kr[j] : *(const float4 *)(kb + j * LTD);
            sj[j] = wave_sum(dot4_pinned(q4, k4)) * (1.0f / 16.0f);
        } else {
            sj[j] = -INFINITY;
        }
    }
    float m = -INFINITY;
#pragma unroll
    for (int j = 0; j < NCB; ++j) m = fmaxf(m, sj[j]);
    float l = 0.f;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int j = 0; j < NCB; ++j) {
        if (j < nk) {
            const float e = expf(sj[j] - m);
            l += e;
            const float4 v4 = (CUR && j == p.cb) ? vc4 : PRE ? vr[j] : *(const float4 *)(vb + j * LTD);
            a.x = fmaf(e, v4.x, a.x); a.y = fmaf(e, v4.y, a.y); a.z = fmaf(e, v4.z, a.z); a.w = fmaf(e, v4.w, a.w);
        }
    }
    return make_float4(a.x / l, a.y / l, a.z / l, a.w / l);
}

// LT FFN output element k of slot b: the LT_FFN_P partial FFN-down sums added in
// ascending order, then the residual (the same arithmetic in the head's prologue
// at batch 1 and in lt_merge_kernel otherwise)
// The LT_FFN_P partial FFN-down sums of the f32 / F16 LT are stored 4 partials interleaved
// per output, [b][p / 4][k][p % 4]: a merge loads 4 consecutive partials of output k as one
// float4 (16 loads per thread at batch 1 instead of 64; the sum order is unchanged).
__device__ __forceinline__ size_t ltp_idx(int b, int p, int k) {
    static_assert(LT_FFN_P % 4 == 0, "4 interleaved partials");
    return (((size_t)b * (LT_FFN_P / 4) + p / 4) * LTD + k) * 4 + (p & 3);
}
// ILV: the interleaved layout above (LT_FFN_P partials); else [b][p][k] (the Q8_0 step's LTQ_P)
template <int NP = LT_FFN_P, bool ILV = true>
__device__ __forceinline__ float lt_ffn_merge(const float *part, const float *y, int b, int k) {
    float s;
    if constexpr (ILV) {
        static_assert(NP == LT_FFN_P, "interleaved layout");
        s = part[ltp_idx(b, 0, k)];
#pragma unroll
        for (int q = 1; q < NP; ++q) s += part[ltp_idx(b, q, k)];
    } else {
        const float *pp = part + (size_t)b * NP * LTD + k;
        s = pp[0];
#pragma unroll
        for (int q = 1; q < NP; ++q) s += pp[(size_t)q * LTD];
    }
    return s + y[(size_t)b * LTD + k];
}

// The same for the LTS_P partial sums of lt_slot_kernel (bf16 weight mode); the slot's
// last workgroup merges them with this arithmetic when the head does not
__device__ __forceinline__ float lts_merge(const float *part, const float *y, int b, int k) {
    const float *pp = part + (size_t)b * LTS_P * LTD + k;
    float s = pp[0];
#pragma unroll 8
    for (int q = 1; q < LTS_P; ++q) s += pp[(size_t)q * LTD];
    return s + y[(size_t)b * LTD + k];
}

// LayerNorm weights of this lane's elements lane + 64 i, loaded before the
// prologue's first global store (a load behind a store that may alias it waits
// for the store: one memory round trip per element otherwise)
template <int PER>
__device__ __forceinline__ void load_lnw(const float *lnw, float (&g)[PER]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int i = 0; i < PER; ++i) g[i] = lnw[lane + 64 * i];
}

// LDS scratch (floats) a prologue needs besides the activation rows
template <int NB, int PRO>
constexpr int pro_scratch() {
    return PRO == PRO_LT_ATTN ? 16
           : PRO == PRO_LTARG_ATTN ? ltc_off<NB>() + (NB < MP_NWAVES ? NB : MP_NWAVES) * 2 * VCB
           : PRO == PRO_SA_MERGE ? NB * NH * (SA_SPLITS + 1)
           : PRO == PRO_XA_LN ? NB * (XA_SPLITS + 1)
           : 1;
}

// Weights of NS partial softmax states (m_s, l_s, O_s relative to m_s) of `nq`
// groups (group q's split s at pp + (q*NS + s)*stride): e_s = exp(m_s - M),
// M = max_s m_s, den = sum_s e_s l_s (an empty split has m = -inf, l = 0, O = 0);
// sc[q*(NS+1) + s] = e_s, sc[q*(NS+1) + NS] = 1/den. The merged output is
// (sum_s e_s O_s) * (1/den). Computed once per group, not per element.
// x2 = merged XA output + x, unfused (shared by PRO_XA_LN and the XA tail's merge)
__device__ __forceinline__ float4 xa_x2(float4 a, float4 x) {
#pragma clang fp contract(off)
    return make_float4(a.x + x.x, a.y + x.y, a.z + x.z, a.w + x.w);
}

// The arithmetic is spelled out (contraction off, explicit fmaf) and shared by the
// merging prologues and the attention kernels' own last-arriver merges (16 slots),
// so a state merged by either computes the same bits.
template <int NS>
__device__ __forceinline__ void split_weights(const float (&ms)[NS], const float (&ls)[NS], float (&e)[NS], float &rd) {
#pragma clang fp contract(off)
    float M = -INFINITY;
#pragma unroll
    for (int s = 0; s < NS; ++s) M = fmaxf(M, ms[s]);
    float den = 0.f;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        e[s] = ms[s] == -INFINITY ? 0.f : expf(ms[s] - M);
        den = fmaf(e[s], ls[s], den);
    }
    rd = 1.0f / den;
}
// one merged output element: (sum_s e_s O_s) * rd
template <int NS>
__device__ __forceinline__ float split_merge(const float *e, const float (&o)[NS], float rd) {
#pragma clang fp contract(off)
    float num = 0.f;
#pragma unroll
    for (int s = 0; s < NS; ++s) num = fmaf(e[s], o[s], num);
    return num * rd;
}
template <int NS>
__device__ __forceinline__ float4 split_merge4(const float *e, const float4 (&o)[NS], float rd) {
    float ox[NS], oy[NS], oz[NS], ow[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) { ox[s] = o[s].x; oy[s] = o[s].y; oz[s] = o[s].z; ow[s] = o[s].w; }
    return make_float4(split_merge<NS>(e, ox, rd), split_merge<NS>(e, oy, rd), split_merge<NS>(e, oz, rd),
                       split_merge<NS>(e, ow, rd));
}
template <int NS>
__device__ __forceinline__ void merge_weights(const float *pp, int stride, int nq, float *sc) {
    for (int q = threadIdx.x; q < nq; q += MP_BLOCK) {
        float ms[NS], ls[NS], e[NS], rd;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            ms[s] = pp[((size_t)q * NS + s) * stride];
            ls[s] = pp[((size_t)q * NS + s) * stride + 1];
        }
        split_weights<NS>(ms, ls, e, rd);
#pragma unroll
        for (int s = 0; s < NS; ++s) sc[q * (NS + 1) + s] = e[s];
        sc[q * (NS + 1) + NS] = rd;
    }
}

// Batched LayerNorm rows: wave w owns slots w, w+4, ...; the statistics are one
// wave's DPP tree over the row (wave_meanvar), exactly as every wave computes them
// at batch 1, so a batch reproduces its slots run alone. Every slot's row is loaded,
// then every slot's statistics computed (independent DPP chains the scheduler can
// interleave), then y = ((x - mean) * rstd) * lnw handed to put(b, k, y) for every
// element (k = lane + 64 i). Block 0 stores the decoder hidden / trace rows after
// that: a store in the middle would order the later loads and waits behind it.
template <int NB, int K>
struct LnRows {
    static constexpr int PER = K / 64, SPW = (NB + MP_NWAVES - 1) / MP_NWAVES;
    float g[PER];
    float vs[SPW][PER];
};
// the loads of ln_slots (LN weights, this wave's rows): issued apart from the
// arithmetic so a caller can put them ahead of its weight stream (vector-memory
// loads complete in issue order: a row load issued behind the weights is only
// usable once every weight load before it has landed)
template <int NB, int K>
__device__ __forceinline__ void ln_load(const GemvP &p, LnRows<NB, K> &r) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    constexpr int PER = LnRows<NB, K>::PER, SPW = LnRows<NB, K>::SPW;
#pragma unroll
    for (int j = 0; j < SPW; ++j) {
        const int b = w + MP_NWAVES * j;
        if (b < NB)
#pragma unroll
            for (int i = 0; i < PER; ++i) r.vs[j][i] = p.src[(size_t)b * p.src_ld + lane + 64 * i];
    }
    load_lnw<PER>(p.lnw, r.g);
}
template <int NB, int K, typename Put>
__device__ __forceinline__ void ln_finish(const GemvP &p, LnRows<NB, K> &r, Put put) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    constexpr int PER = LnRows<NB, K>::PER, SPW = LnRows<NB, K>::SPW;
    float(&g)[PER] = r.g;
    float(&vs)[SPW][PER] = r.vs;
#ifdef MP_TS_PROBE  // diagnostics build: (loads landed, stats done) / (stats done, rows put)
    unsigned long long tA = 0, tB = 0;
    if (p.ts) { __builtin_amdgcn_s_waitcnt(0); tA = __builtin_amdgcn_s_memrealtime(); }
#endif
    float mean[SPW], var[SPW], rstd[SPW];
    if constexpr (SPW * MP_NWAVES == NB) {  // every wave owns SPW rows: one interleaved pass
        wave_meanvar_n<PER, SPW>(vs, mean, var);
    } else {
#pragma unroll
        for (int j = 0; j < SPW; ++j) {
            mean[j] = var[j] = 0.f;
            if (w + MP_NWAVES * j < NB) wave_meanvar<PER>(vs[j], mean[j], var[j]);
        }
    }
#pragma unroll
    for (int j = 0; j < SPW; ++j) rstd[j] = 1.0f / sqrtf(var[j] + p.eps);
#ifdef MP_TS_PROBE
    if (p.ts) asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(tB) : "v"(rstd[SPW - 1]), "v"(rstd[0]));
#endif
#pragma unroll
    for (int j = 0; j < SPW; ++j) {
        const int b = w + MP_NWAVES * j;
        if (b >= NB) break;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            vs[j][i] = ((vs[j][i] - mean[j]) * rstd[j]) * g[i];
            put(b, lane + 64 * i, vs[j][i]);
        }
    }
#ifdef MP_TS_PROBE
    if (p.ts) {
        __builtin_amdgcn_s_waitcnt(0);
        const unsigned long long tC = __builtin_amdgcn_s_memrealtime();
        if (lane == 0 && blockIdx.x < TS_BLOCKS)
            *(ulonglong2 *)(p.ts + 2 * ((size_t)blockIdx.x * TS_WAVES + TS_WAVES / 2 + w)) =
                w < 2 ? make_ulonglong2(tA, tB) : make_ulonglong2(tB, tC);
    }
#endif
    if (blockIdx.x == 0 && (p.hidden_out || p.trace)) {
#pragma unroll
        for (int j = 0; j < SPW; ++j) {
            const int b = w + MP_NWAVES * j;
            if (b >= NB) break;
            const int s = p.trace ? p.step[b] : 0;
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int k = lane + 64 * i;
                if (p.hidden_out) p.hidden_out[(size_t)b * K + k] = vs[j][i];
                if (p.trace && s < p.trace_steps) p.trace[((size_t)b * p.trace_steps + s) * K + k] = vs[j][i];
            }
        }
    }
}
template <int NB, int K, typename Put>
__device__ __forceinline__ void ln_slots(const GemvP &p, Put put) {
    LnRows<NB, K> r;
    ln_load<NB, K>(p, r);
    ln_finish<NB, K>(p, r, put);
}

// PRO_XA_LN's LayerNorm of the x2 rows in act (LN weights g already in registers):
// block 0 stores x2 (the FFN residual input); act = LN(x2) * lnw with the same
// one-wave DPP statistics as PRO_LN, so batch 1 and batched prologues agree bit for bit
template <int NB, int K>
__device__ __forceinline__ void xa_ln_rows(const GemvP &p, float *act, const float (&g)[K / 64]) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    constexpr int PER = K / 64;
    if constexpr (NB == 1) {
            constexpr int Q = PER / MP_NWAVES;
            float v[PER];
#pragma unroll
            for (int i = 0; i < PER; ++i) v[i] = act[lane + 64 * i];
            // x2 to HBM (block 0) after every global load of the prologue: a store
            // earlier would order the later loads behind it
            if (blockIdx.x == 0 && w == 0)
#pragma unroll
                for (int i = 0; i < PER; ++i) p.xres[lane + 64 * i] = v[i];
            float mean, var;
            wave_meanvar<PER>(v, mean, var);
            const float rstd = 1.0f / sqrtf(var + p.eps);
            lds_sync();  // every wave has read the row before any overwrites its quarter
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                if (i / Q != w) continue;
                const int k = lane + 64 * i;
                act[k] = ((v[i] - mean) * rstd) * g[i];
            }
        } else {
            for (int b = w; b < NB; b += MP_NWAVES) {  // a wave owns its slots' rows
                float v[PER];
#pragma unroll
                for (int i = 0; i < PER; ++i) v[i] = act[b * K + lane + 64 * i];
                if (blockIdx.x == 0)
#pragma unroll
                    for (int i = 0; i < PER; ++i) p.xres[(size_t)b * D + lane + 64 * i] = v[i];
                float mean, var;
                wave_meanvar<PER>(v, mean, var);
                const float rstd = 1.0f / sqrtf(var + p.eps);
#pragma unroll
                for (int i = 0; i < PER; ++i) {
                    const int k = lane + 64 * i;
                    act[b * K + k] = ((v[i] - mean) * rstd) * g[i];
                }
            }
        }
        lds_sync();

}

// Batch-1 LayerNorm row (PRO_LN, NB = 1): every wave loads the whole row and runs
// the same DPP statistics (identical results, no barrier), then writes its quarter
// of act. Loads and arithmetic apart, as ln_load / ln_finish.
template <int K>
struct Ln1Row {
    static constexpr int PER = K / 64;
    float v[PER], g[PER];
    int s;  // trace row (block 0 with a trace only)
};
template <int K>
__device__ __forceinline__ void ln1_load(const GemvP &p, Ln1Row<K> &r) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int i = 0; i < Ln1Row<K>::PER; ++i) r.v[i] = p.src[lane + 64 * i];
    load_lnw<Ln1Row<K>::PER>(p.lnw, r.g);
    r.s = (p.trace && blockIdx.x == 0) ? p.step[0] : 0;
}
template <int K>
__device__ __forceinline__ void ln1_finish(const GemvP &p, Ln1Row<K> &r, float *act) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    constexpr int PER = K / 64, Q = PER / MP_NWAVES;
    float mean, var;
    wave_meanvar<PER>(r.v, mean, var);
    const float rstd = 1.0f / sqrtf(var + p.eps);
    const bool st = p.hidden_out && blockIdx.x == 0;
    const int s = r.s;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        if (i / Q != w) continue;
        const int k = lane + 64 * i;
        const float y = ((r.v[i] - mean) * rstd) * r.g[i];
        act[k] = y;
        if (st) p.hidden_out[k] = y;
        if (p.trace && blockIdx.x == 0 && s < p.trace_steps) p.trace[(size_t)s * K + k] = y;
    }
    lds_sync();
}

// A prologue whose global loads a kernel issues AHEAD of its weight stream
// (vector-memory loads complete in issue order: rows loaded behind the weights are
// only usable once every weight has landed). PRO_LN, plain rows, the SA / XA split
// merges (up to 4 slots) and the LT head's FFN merge at batch 1: their loads are
// independent of the launch's other work; the arithmetic after them is unchanged.
template <int NB, int K, int PRO>
struct PreRows {
    static constexpr bool ON = false;
};
template <int NB, int K>
struct PreRows<NB, K, PRO_LN> {
    static constexpr bool ON = true;
    typename std::conditional<NB == 1, Ln1Row<K>, LnRows<NB, K>>::type r;
};
// register arrays of these structs hold native 4-float vectors (an array of HIP's
// float4 struct in a struct member was kept in scratch memory)
typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4 to_v4(float4 a) { return f32x4{a.x, a.y, a.z, a.w}; }
__device__ __forceinline__ float4 to_f4(f32x4 a) { return make_float4(a.x, a.y, a.z, a.w); }
// Plain rows (PRO_PLAIN) while they fit in 12 float4 per thread
template <int NB, int K>
struct PreRows<NB, K, PRO_PLAIN> {
    static constexpr int PT = (NB * K / 4 + MP_BLOCK - 1) / MP_BLOCK;
    static constexpr bool ON = NB * K <= 12288;
    f32x4 v[ON ? PT : 1];
};
// The SA / XA split merges while every item fits in one round of the prologue's
// (batches up to 4): the split outputs, the split (m, l) pairs and, for XA, x and the
// LN weights
template <int NB, int K, int NS, int NQ, int PART>
struct PreMerge {
    static constexpr int PT = (NB * (K / 4) + MP_BLOCK - 1) / MP_BLOCK;
    static constexpr bool ON = PT <= 4 && NQ <= MP_BLOCK;
    f32x4 o[ON ? PT : 1][NS], xv[ON ? PT : 1];
    float ms[NS], ls[NS];
    float g[K / 64];
};
template <int NB, int K>
struct PreRows<NB, K, PRO_SA_MERGE> : PreMerge<NB, K, SA_SPLITS, NB * NH, SA_PART> {};
template <int NB, int K>
struct PreRows<NB, K, PRO_XA_LN> : PreMerge<NB, K, XA_SPLITS, NB, XA_PART> {};
// the LT head's FFN merge at batch 1: the 64 partial sums and y of output tid
template <int NB, int K>
struct PreRows<NB, K, PRO_LTFFN_MERGE> {
    static constexpr bool ON = NB == 1 && K == MP_BLOCK;
    float pp[LT_FFN_P], y;
};
template <int NB, int K>
struct PreRows<NB, K, PRO_LTQ_MERGE> {
    static constexpr bool ON = NB == 1 && K == MP_BLOCK;
    float pp[LTQ_P], y;
};
template <int NB, int K, int PRO>
__device__ __forceinline__ void pre_load(const GemvP &p, PreRows<NB, K, PRO> &pr) {
    const int tid = threadIdx.x;
    if constexpr (!PreRows<NB, K, PRO>::ON) {
        return;
    } else if constexpr (PRO == PRO_LN) {
        if constexpr (NB == 1) ln1_load<K>(p, pr.r);
        else ln_load<NB, K>(p, pr.r);
    } else if constexpr (PRO == PRO_PLAIN) {
#pragma unroll
        for (int u = 0; u < PreRows<NB, K, PRO>::PT; ++u) {
            const int e = min(u * MP_BLOCK + tid, NB * (K / 4) - 1);  // every element assigned (no scratch)
            pr.v[u] = *(const f32x4 *)(p.src + (size_t)(e / (K / 4)) * p.src_ld + (e % (K / 4)) * 4);
        }
    } else if constexpr (PRO == PRO_SA_MERGE || PRO == PRO_XA_LN) {
        constexpr bool SA = PRO == PRO_SA_MERGE;
        constexpr int NS = SA ? SA_SPLITS : XA_SPLITS, PART = SA ? SA_PART : XA_PART, NQ = SA ? NB * NH : NB;
        static_assert(K == D, "d_model wide");
#pragma unroll
        for (int u = 0; u < PreRows<NB, K, PRO>::PT; ++u) {
            const int e = u * MP_BLOCK + tid;
            if (e >= NB * (K / 4)) break;
            const int b = e / (K / 4), k = (e % (K / 4)) * 4, q = SA ? b * NH + k / DH : b;
            if constexpr (!SA) pr.xv[u] = *(const f32x4 *)(p.src + (size_t)b * p.src_ld + k);
#pragma unroll
            for (int s2 = 0; s2 < NS; ++s2)
                pr.o[u][s2] = *(const f32x4 *)(p.part + ((size_t)q * NS + s2) * PART + 4 + (SA ? k % DH : k));
        }
        if (tid < NQ) {
#pragma unroll
            for (int s2 = 0; s2 < NS; ++s2) {
                pr.ms[s2] = p.part[((size_t)tid * NS + s2) * PART];
                pr.ls[s2] = p.part[((size_t)tid * NS + s2) * PART + 1];
            }
        }
        if constexpr (!SA) load_lnw<K / 64>(p.lnw, pr.g);
    } else if constexpr (PRO == PRO_LTFFN_MERGE) {
#pragma unroll
        for (int q = 0; q < LT_FFN_P; q += 4) {
            const f32x4 v = *(const f32x4 *)(p.part + ltp_idx(0, q, tid));
            pr.pp[q] = v.x; pr.pp[q + 1] = v.y; pr.pp[q + 2] = v.z; pr.pp[q + 3] = v.w;
        }
        pr.y = p.addsrc[tid];
    } else if constexpr (PRO == PRO_LTQ_MERGE) {
        const float *pp = p.part + tid;
#pragma unroll
        for (int q = 0; q < LTQ_P; ++q) pr.pp[q] = pp[(size_t)q * LTD];
        pr.y = p.addsrc[tid];
    }
}
// the prologue's arithmetic on preloaded rows: act[NB][K] f32, as prologue<NB, K, PRO>
template <int NB, int K, int PRO>
__device__ __forceinline__ void pre_finish(const GemvP &p, PreRows<NB, K, PRO> &pr, float *act, float *sc) {
    const int tid = threadIdx.x;
    if constexpr (!PreRows<NB, K, PRO>::ON) {
        return;
    } else if constexpr (PRO == PRO_LN) {
        if constexpr (NB == 1) {
            ln1_finish<K>(p, pr.r, act);
        } else {
            ln_finish<NB, K>(p, pr.r, [&](int b, int k, float y) { act[b * K + k] = y; });
            lds_sync();
        }
    } else if constexpr (PRO == PRO_PLAIN) {
#pragma unroll
        for (int u = 0; u < PreRows<NB, K, PRO>::PT; ++u) {
            const int e = u * MP_BLOCK + tid;
            if (e < NB * (K / 4)) *(f32x4 *)(act + (e / (K / 4)) * K + (e % (K / 4)) * 4) = pr.v[u];
        }
        lds_sync();
    } else if constexpr (PRO == PRO_SA_MERGE || PRO == PRO_XA_LN) {
        // merge_weights' and the merge loop's arithmetic (split_weights, split_merge4, xa_x2)
        constexpr bool SA = PRO == PRO_SA_MERGE;
        constexpr int NS = SA ? SA_SPLITS : XA_SPLITS, NQ = SA ? NB * NH : NB;
        if (tid < NQ) {
            float e[NS], rd;
            split_weights<NS>(pr.ms, pr.ls, e, rd);
#pragma unroll
            for (int s2 = 0; s2 < NS; ++s2) sc[tid * (NS + 1) + s2] = e[s2];
            sc[tid * (NS + 1) + NS] = rd;
        }
        lds_sync();
#pragma unroll
        for (int u = 0; u < PreRows<NB, K, PRO>::PT; ++u) {
            const int e = u * MP_BLOCK + tid;
            if (e >= NB * (K / 4)) break;
            const int b = e / (K / 4), k = (e % (K / 4)) * 4, q = SA ? b * NH + k / DH : b;
            float4 ou[NS];
#pragma unroll
            for (int s2 = 0; s2 < NS; ++s2) ou[s2] = to_f4(pr.o[u][s2]);
            const float4 a = split_merge4<NS>(sc + q * (NS + 1), ou, sc[q * (NS + 1) + NS]);
            if constexpr (SA) *(float4 *)(act + b * K + k) = a;
            else *(float4 *)(act + b * K + k) = xa_x2(a, to_f4(pr.xv[u]));
        }
        lds_sync();
        if constexpr (!SA) xa_ln_rows<NB, K>(p, act, pr.g);
    } else if constexpr (PRO == PRO_LTFFN_MERGE || PRO == PRO_LTQ_MERGE) {
        // lt_ffn_merge's arithmetic: partial sums in ascending order, then the residual
        float s2 = pr.pp[0];
#pragma unroll
        for (int q = 1; q < ltm_count<PRO>(); ++q) s2 += pr.pp[q];
        act[tid] = s2 + pr.y;
        lds_sync();
    }
}

template <int NB, int K, int PRO>
__device__ __forceinline__ void prologue(const GemvP &p, float *act, float *red, float *sc) {
    const int tid = threadIdx.x;
    constexpr int IB = 4;  // merge items per thread with all their loads in flight
    if constexpr (PRO == PRO_SA_MERGE) {
        // self-attention output of every head: its SA_SPLITS key-split states merged
        static_assert(K == D, "SA output is d_model wide");
        constexpr int ITEMS = NB * (K / 4);
        float4 o[IB][SA_SPLITS];
        // the first round's split outputs are loaded together with the split weights'
        // (m, l): one memory round trip before the first combine, not two
        auto load_o = [&](int base) {
#pragma unroll
            for (int u = 0; u < IB; ++u) {
                const int e = base + u * MP_BLOCK + tid;
                if (e >= ITEMS) break;
                const int b = e / (K / 4), k = (e % (K / 4)) * 4, q = b * NH + k / DH;
#pragma unroll
                for (int s2 = 0; s2 < SA_SPLITS; ++s2)
                    o[u][s2] = *(const float4 *)(p.part + ((size_t)q * SA_SPLITS + s2) * SA_PART + 4 + k % DH);
            }
        };
        load_o(0);
        merge_weights<SA_SPLITS>(p.part, SA_PART, NB * NH, sc);
        lds_sync();
        for (int base = 0; base < ITEMS; base += MP_BLOCK * IB) {
            if (base) load_o(base);
#pragma unroll
            for (int u = 0; u < IB; ++u) {
                const int e = base + u * MP_BLOCK + tid;
                if (e >= ITEMS) break;
                const int b = e / (K / 4), k = (e % (K / 4)) * 4, q = b * NH + k / DH;
                *(float4 *)(act + b * K + k) =
                    split_merge4<SA_SPLITS>(sc + q * (SA_SPLITS + 1), o[u], sc[q * (SA_SPLITS + 1) + SA_SPLITS]);
            }
        }
        lds_sync();
    } else if constexpr (PRO == PRO_XA_LN) {
        // x2 = x + XA (its XA_SPLITS text-key split states merged, magpie.cpp:3519); block 0
        // stores x2 (the FFN's residual input); act = LN(x2) * lnw with the same one-wave
        // DPP statistics as PRO_LN, so batch 1 and batched prologues agree bit for bit
        static_assert(K == D, "XA output is d_model wide");
        constexpr int ITEMS = NB * (K / 4);
        float4 o[IB][XA_SPLITS], xv[IB];
        // the first round's inputs are loaded together with the split weights' (m, l)
        auto load_o = [&](int base) {
#pragma unroll
            for (int u = 0; u < IB; ++u) {
                const int e = base + u * MP_BLOCK + tid;
                if (e >= ITEMS) break;
                const int b = e / (K / 4), k = (e % (K / 4)) * 4;
                xv[u] = *(const float4 *)(p.src + (size_t)b * p.src_ld + k);
#pragma unroll
                for (int s2 = 0; s2 < XA_SPLITS; ++s2)
                    o[u][s2] = *(const float4 *)(p.part + ((size_t)b * XA_SPLITS + s2) * XA_PART + 4 + k);
            }
        };
        load_o(0);
        merge_weights<XA_SPLITS>(p.part, XA_PART, NB, sc);
        lds_sync();
        for (int base = 0; base < ITEMS; base += MP_BLOCK * IB) {
            if (base) load_o(base);
#pragma unroll
            for (int u = 0; u < IB; ++u) {
                const int e = base + u * MP_BLOCK + tid;
                if (e >= ITEMS) break;
                const int b = e / (K / 4), k = (e % (K / 4)) * 4;
                const float4 a = split_merge4<XA_SPLITS>(sc + b * (XA_SPLITS + 1), o[u], sc[b * (XA_SPLITS + 1) + XA_SPLITS]);
                *(float4 *)(act + b * K + k) = xa_x2(a, xv[u]);
            }
        }
        lds_sync();
        constexpr int PER = K / 64;
        float g[PER];
        load_lnw<PER>(p.lnw, g);
        xa_ln_rows<NB, K>(p, act, g);
    } else if constexpr (PRO == PRO_LTFFN_MERGE || PRO == PRO_LTQ_MERGE) {
        static_assert(K == LTD, "LT is 256 wide");
        for (int e = tid; e < NB * K; e += MP_BLOCK)
            act[e] = lt_ffn_merge<ltm_count<PRO>(), PRO == PRO_LTFFN_MERGE>(p.part, p.addsrc, e / K, e % K);
        lds_sync();
    } else if constexpr (PRO == PRO_LTS_MERGE) {
        static_assert(K == LTD, "LT is 256 wide");
        for (int e = tid; e < NB * K; e += MP_BLOCK) act[e] = lts_merge(p.part, p.addsrc, e / K, e % K);
        lds_sync();

    } else if constexpr (PRO == PRO_PLAIN) {
        // PG float4 loads in flight per thread, then their LDS stores: the rolled
        // load -> store loop waited one memory round trip per float4 (the Q8_0 file's F32
        // FFN down at 16 slots: 24 per thread, 18.9 us per launch)
        constexpr int ITEMS = NB * (K / 4), PT = (ITEMS + MP_BLOCK - 1) / MP_BLOCK, PG = PT < 12 ? PT : 12;
        for (int u0 = 0; u0 < PT; u0 += PG) {
            f32x4 v[PG];
#pragma unroll
            for (int u = 0; u < PG; ++u) {
                const int e = min((u0 + u) * MP_BLOCK + tid, ITEMS - 1);  // every element assigned
                v[u] = *(const f32x4 *)(p.src + (size_t)(e / (K / 4)) * p.src_ld + (e % (K / 4)) * 4);
            }
#pragma unroll
            for (int u = 0; u < PG; ++u) {
                const int e = (u0 + u) * MP_BLOCK + tid;
                if (u0 + u < PT && e < ITEMS) *(f32x4 *)(act + (e / (K / 4)) * K + (e % (K / 4)) * 4) = v[u];
            }
        }
        lds_sync();
    } else if constexpr (PRO == PRO_LN && NB >= 2) {
        ln_slots<NB, K>(p, [&](int b, int k, float y) { act[b * K + k] = y; });
        lds_sync();
    } else if constexpr (PRO == PRO_LN) {
        Ln1Row<K> r;
        ln1_load<K>(p, r);
        ln1_finish<K>(p, r, act);
    } else if constexpr (PRO == PRO_LTX_LN) {
        // one wave per slot at every batch size (wave_block_meanvar), so a batch
        // reproduces its utterances run alone bit for bit
        // (every owned slot's row loaded before the first slot's arithmetic: one memory
        // round trip per wave, not one per slot)
        const int lane = tid & 63, w = tid >> 6;
        constexpr int SPW = (NB + MP_NWAVES - 1) / MP_NWAVES;
        float g[4], ps[4], xs[SPW][4];
        load_lnw<4>(p.lnw, g);
#pragma unroll
        for (int i = 0; i < 4; ++i) ps[i] = p.lt_pos[(size_t)p.cb * LTD + lane + 64 * i];
#pragma unroll
        for (int j = 0; j < SPW; ++j) {
            const int b = min(w + MP_NWAVES * j, NB - 1);  // every element assigned
#pragma unroll
            for (int i = 0; i < 4; ++i) xs[j][i] = p.lt_s[((size_t)b * 9 + p.cb) * LTD + lane + 64 * i];
        }
#pragma unroll
        for (int j = 0; j < SPW; ++j) {
            const int b = w + MP_NWAVES * j;
            if (b >= NB) break;  // wave-uniform
            float X[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) X[i] = xs[j][i] + ps[i];
            if (blockIdx.x == 0)
#pragma unroll
                for (int i = 0; i < 4; ++i) p.ltX[(size_t)b * LTD + lane + 64 * i] = X[i];
            float mean, var;
            wave_block_meanvar<1>(X, mean, var);
            const float rstd = 1.0f / sqrtf(var + p.eps);
#pragma unroll
            for (int i = 0; i < 4; ++i) act[b * K + lane + 64 * i] = ((X[i] - mean) * rstd) * g[i];
        }
        lds_sync();
    } else if constexpr (PRO == PRO_LTARG_ATTN) {
        // wave w owns slots w, w+4, ... at every batch size. Phase 1 picks codebook
        // cb-1's code of each (the next slot's logits in flight); phase 2 issues every
        // gather at once: q|k|v of position cb from the load-time table and the residual
        // row P[cb-1][code] + lt_pos[cb]; phase 3 attends over positions 0..cb. At one
        // slot per wave the earlier positions' k/v are loaded before the pick.
        static_assert(K == LTD, "LT is 256 wide");
        constexpr int SPW = (NB + MP_NWAVES - 1) / MP_NWAVES;
        const int lane = tid & 63, w = tid >> 6;
        float *wsc = sc + ltc_off<NB>() + w * 2 * VCB;
        float cur[PICK_R], nxt[PICK_R];
        if (w < NB) load_logits(p.logits + (size_t)w * VCB, cur);
        float4 kr[NCB], vr[NCB];
        if constexpr (SPW == 1) {
            if (w < NB) {
                const float *kb = p.ltk + (size_t)w * NCB * LTD + 4 * lane, *vb = p.ltv + (size_t)w * NCB * LTD + 4 * lane;
#pragma unroll
                for (int j = 0; j < NCB - 1; ++j)
                    if (j < p.cb) { kr[j] = *(const float4 *)(kb + j * LTD); vr[j] = *(const float4 *)(vb + j * LTD); }
            }
        }
        int stp[SPW];  // every owned slot's step up front, not one dependent load per pick
#pragma unroll
        for (int j = 0; j < SPW; ++j) stp[j] = w + MP_NWAVES * j < NB ? p.step[w + MP_NWAVES * j] : 0;
        unsigned long long codes = 0ull;  // 16 bits per owned slot (codes < 2048)
#pragma unroll
        for (int j = 0; j < SPW; ++j) {
            const int b = w + MP_NWAVES * j;
            if (b >= NB) break;  // wave-uniform
            const int bn = b + MP_NWAVES;
            if (bn < NB) load_logits(p.logits + (size_t)bn * VCB, nxt);
            int amax;
            const int code = wave_pick_v(cur, p.ignore_eos || stp[j] < 4, p.audio_bos, p.audio_eos, p.smp, b,
                                         stp[j], p.cb - 1, wsc, amax);
            if (blockIdx.x == 0 && lane == 0) {
                p.codes_cur[b * NCB + p.cb - 1] = code;
                if (amax == p.audio_eos) p.smp.argeos[b] = 1;
                if (p.smp.amax) p.smp.amax[b * NCB + p.cb - 1] = amax;
            }
            codes |= (unsigned long long)code << (16 * j);
#pragma unroll
            for (int r = 0; r < PICK_R; ++r) cur[r] = nxt[r];
        }
        float4 q4[SPW], k4[SPW], v4[SPW], x4[SPW];
        const float4 pos4 = *(const float4 *)(p.lt_pos + (size_t)p.cb * LTD + 4 * lane);
#pragma unroll
        for (int j = 0; j < SPW; ++j) {
            if (w + MP_NWAVES * j < NB) {
                const int code = (int)((codes >> (16 * j)) & 0xffffull);
                const size_t r = (size_t)(p.cb - 1) * VCB + code;
                const float *row = p.qkvtab + r * (3 * LTD) + 4 * lane;
                q4[j] = *(const float4 *)row;
                k4[j] = *(const float4 *)(row + LTD);
                v4[j] = *(const float4 *)(row + 2 * LTD);
                x4[j] = *(const float4 *)(p.ptab + r * LTD + 4 * lane);
            }
        }
#pragma unroll
        for (int j = 0; j < SPW; ++j) {
            const int b = w + MP_NWAVES * j;
            if (b >= NB) continue;
            if (blockIdx.x == 0) {  // position cb's k/v for the later codebooks
                *(float4 *)(p.lk + ((size_t)b * NCB + p.cb) * LTD + 4 * lane) = k4[j];
                *(float4 *)(p.lv + ((size_t)b * NCB + p.cb) * LTD + 4 * lane) = v4[j];
            }
            *(float4 *)(sc + b * LTD + 4 * lane) =
                make_float4(x4[j].x + pos4.x, x4[j].y + pos4.y, x4[j].z + pos4.z, x4[j].w + pos4.w);
            *(float4 *)(act + b * K + 4 * lane) = lt_attend<true, SPW == 1>(p, b, q4[j], k4[j], v4[j], kr, vr);
        }
        lds_sync();
    } else if constexpr (PRO == PRO_LT_ATTN) {
        // codebook 0 (q|k|v from the lt_a GEMV): the same per-slot wave code
        static_assert(K == LTD, "LT is 256 wide");
        const int lane = tid & 63, w = tid >> 6;
        float4 kr[NCB], vr[NCB];
        for (int b = w; b < NB; b += MP_NWAVES) {
            const float4 q4 = *(const float4 *)(p.ltq + (size_t)b * LTD + 4 * lane);
            *(float4 *)(act + b * K + 4 * lane) = lt_attend<false, false>(p, b, q4, q4, q4, kr, vr);
        }
        lds_sync();
    }
}

// The epilogue's own operand of output (row n, slot b) -- the bias, the residual row, the
// added row -- loaded when the launch starts: read in the epilogue it was a dependent L2 /
// Infinity-Cache round trip after the dot products, on every such launch's critical path.
// Each element is read and rewritten by the one lane that owns it, so the early value is
// the value the epilogue read; epi_store_op / publish_x1_op compute the same expressions.
template <int EPI>
constexpr bool epi_has_operand() {
    return EPI == EPI_BIAS || EPI == EPI_RESID || EPI == EPI_ADD_STORE || EPI == EPI_RESID_XA;
}
template <int EPI>
__device__ __forceinline__ float epi_operand(const GemvP &p, int n, int b) {
    if constexpr (EPI == EPI_BIAS) return p.bias[n];
    else if constexpr (EPI == EPI_RESID || EPI == EPI_RESID_XA) return p.resid[(size_t)b * D + n];
    else if constexpr (EPI == EPI_ADD_STORE) return p.addsrc[(size_t)b * p.out_ld + n];
    else return 0.f;
}
template <int EPI>
__device__ __forceinline__ void epi_store_op(const GemvP &p, float v, int n, int b, float op) {
    static_assert(EPI == EPI_BIAS || EPI == EPI_RESID || EPI == EPI_ADD_STORE, "epilogues with an operand");
    if constexpr (EPI == EPI_BIAS) p.out[(size_t)b * p.out_ld + n] = v + op;
    else if constexpr (EPI == EPI_RESID) p.resid[(size_t)b * D + n] = v + op;
    else p.out[(size_t)b * p.out_ld + n] = v + op;
}

// Epilogue of output (row n, slot b) of a fused projection.
template <int EPI>
__device__ __forceinline__ void epi_store(const GemvP &p, float v, int n, int b, float extra = 0.f) {
    if constexpr (EPI == EPI_STORE) p.out[(size_t)b * p.out_ld + n] = v;
    else if constexpr (EPI == EPI_BIAS) p.out[(size_t)b * p.out_ld + n] = v + p.bias[n];
    else if constexpr (EPI == EPI_GELU) p.out[(size_t)b * p.out_ld + n] = gelu_tanh(v);
    else if constexpr (EPI == EPI_GELU_B16) {
        const __bf16 h = (__bf16)gelu_tanh(v);  // round to nearest even, as the consumer's staging would
        p.out_b16[(size_t)b * p.out_ld + n] = __builtin_bit_cast(unsigned short, h);
    }
    else if constexpr (EPI == EPI_GELU_F16) {
        const _Float16 h = (_Float16)gelu_tanh(v);
        p.out_b16[(size_t)b * p.out_ld + n] = __builtin_bit_cast(unsigned short, h);
    }
    else if constexpr (EPI == EPI_RESID) p.resid[(size_t)b * D + n] = v + p.resid[(size_t)b * D + n];
    else if constexpr (EPI == EPI_ADD_STORE) p.out[(size_t)b * p.out_ld + n] = v + p.addsrc[(size_t)b * p.out_ld + n];
    else if constexpr (EPI == EPI_LTX_ADD) p.out[(size_t)b * p.out_ld + n] = v + extra;  // extra = X[b][n]
    else if constexpr (EPI == EPI_QKV) {
        const size_t slot = ((size_t)(b * p.nlayers + p.layer) * p.max_seq + p.pos[b]) * D;
        if (n < D) p.out[(size_t)b * D + n] = v;
        else kv_store(n < 2 * D ? p.kc : p.vc, slot + (n < 2 * D ? n - D : n - 2 * D), v, p.kv16);
    } else if constexpr (EPI == EPI_LTKVO) {
        if (n < LTD) p.lk[(size_t)b * NCB * LTD + n] = v;
        else p.lv[(size_t)b * NCB * LTD + n - LTD] = v;
    } else if constexpr (EPI == EPI_LTQKV) {
        if (n < LTD) p.lq[(size_t)b * LTD + n] = v;
        else if (n < 2 * LTD) p.lk[((size_t)b * NCB + p.cb) * LTD + n - LTD] = v;
        else p.lv[((size_t)b * NCB + p.cb) * LTD + n - 2 * LTD] = v;
    }
}

}  // namespace mp
