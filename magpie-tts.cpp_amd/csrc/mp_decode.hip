// Per-frame decode kernels for gfx950 (f32 path, batch NB <= 8 utterances).
//
// One decode iteration = 12 decoder layers (magpie_build_decoder_layer_gpu_cached,
// magpie.cpp:3484-3528) + the 8-codebook local transformer
// (magpie_local_transformer_sample_all, magpie.cpp:1113-1317) + EOS bookkeeping
// (magpie.cpp:4340-4358), all device-resident and captured in one hipGraph.
//
// At batch <= 8 every projection is a weight-streaming GEMV: HBM-bound, each
// weight byte is read once per step and reused across the NB utterances from
// registers. The fused GEMV family below streams W with 16-byte per-lane loads
// (one 1 KiB wave-instruction per 256 floats of a row), keeps the activation
// vector in LDS, and fuses whatever tiny op precedes / follows the projection
// (LayerNorm, frame embedding, attention combine, argmax, GELU, residual, KV
// append) into its prologue / epilogue so no extra launch is paid for it.
#include <hip/hip_runtime.h>
#include <math.h>

#include "mp_device.hpp"
#include "mp_params.hpp"

namespace mp {

// ---------------------------------------------------------------- prologues
// Each prologue fills act[NB][K] (LDS) with the activation vector of every slot.

template <int NB, int K>
__device__ __forceinline__ void pro_ln_vec(const float *x, const float *lnw, float eps, float *act, float *red,
                                           float *store) {
    // ggml_norm + ggml_mul (magpie.cpp:2255-2258): (x - mean) / sqrt(var + eps) * w
    constexpr int PER = K / MP_BLOCK;
    float v[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) v[i] = x[threadIdx.x + MP_BLOCK * i];
    float mean, var;
    block_meanvar<PER>(v, red, mean, var);
    const float rstd = 1.0f / sqrtf(var + eps);
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int k = threadIdx.x + MP_BLOCK * i;
        const float y = ((v[i] - mean) * rstd) * lnw[k];
        act[k] = y;
        if (store) store[k] = y;
    }
}

// Masked first-max argmax of slot b's logits (magpie.cpp:1133-1145, 1243-1259):
// 2016 and 2018..2023 always forbidden, 2017 (EOS) too while step < 4 or in
// fixed-length mode. Every thread returns the winner.
__device__ __forceinline__ int block_masked_argmax(const GemvP &p, int b, float *red) {
    const int tid = threadIdx.x;
    const float *lg = p.logits + (size_t)b * VCB;
    const bool forbid_eos = p.ignore_eos || p.step[b] < 4;
    constexpr int R = (VCB + MP_BLOCK - 1) / MP_BLOCK;
    float lv[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int i = tid + MP_BLOCK * r;
        lv[r] = i < VCB ? lg[i] : -INFINITY;
    }
    float bv = -INFINITY;
    int bi = 0x7fffffff;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int i = tid + MP_BLOCK * r;
        float v = lv[r];
        if (i >= VCB || (i >= p.audio_bos && i <= p.audio_bos + 7 && (i != p.audio_eos || forbid_eos))) v = -INFINITY;
        argmax_merge(bv, bi, v, i);
    }
    wave_argmax(bv, bi);
    if ((tid & 63) == 0) { red[tid >> 6] = bv; ((int *)red)[4 + (tid >> 6)] = bi; }
    lds_sync();
    float v0 = red[0];
    int i0 = ((int *)red)[4];
    for (int w = 1; w < MP_NWAVES; ++w) argmax_merge(v0, i0, red[w], ((int *)red)[4 + w]);
    lds_sync();
    if (i0 < 0 || i0 >= VCB) i0 = 0;  // all -inf / NaN: the reference's argmax stays 0
    return i0;
}

// Wave-level variant of the masked argmax (one wave owns one slot).
__device__ __forceinline__ int wave_masked_argmax(const GemvP &p, int b) {
    const int lane = threadIdx.x & 63;
    const float *lg = p.logits + (size_t)b * VCB;
    const bool forbid_eos = p.ignore_eos || p.step[b] < 4;
    constexpr int R = (VCB + 63) / 64;
    float lv[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int i = lane + 64 * r;
        lv[r] = i < VCB ? lg[i] : -INFINITY;
    }
    float bv = -INFINITY;
    int bi = 0x7fffffff;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int i = lane + 64 * r;
        float v = lv[r];
        if (i >= VCB || (i >= p.audio_bos && i <= p.audio_bos + 7 && (i != p.audio_eos || forbid_eos))) v = -INFINITY;
        argmax_merge(bv, bi, v, i);
    }
    wave_argmax(bv, bi);
    if (bi < 0 || bi >= VCB) bi = 0;
    return bi;
}

// One wave picks slot b's code for codebook `cb` of this frame: masked first-max
// argmax (always, for EOS detection, magpie.cpp:1250-1259), and at temperature
// >= 0.01 a top-k draw with the reference's sample_top_k arithmetic
// (magpie.cpp:1072-1109): the k largest masked logits in descending order (ties by
// ascending index), p_i = exp((l_i - l_max) / T) summed sequentially, normalised,
// and the first i with u < cumsum_i (fallback: the k-th). Radix-select finds the
// k-th key, a ballot compaction gathers the k candidates into LDS, a counting rank
// orders them, lane 0 runs the two sequential float loops. scratch: 2*VCB floats.
__device__ int wave_pick(const float *lg, bool forbid_eos, int audio_bos, int audio_eos, const Sampling &smp,
                         int stream, int step, int cb, float *scratch, int &amax) {
    const int lane = threadIdx.x & 63;
    constexpr int R = (VCB + 63) / 64;
    float lv[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int i = lane + 64 * r;
        lv[r] = i < VCB ? lg[i] : -INFINITY;
    }
    float bv = -INFINITY;
    int bi = 0x7fffffff;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int i = lane + 64 * r;
        if (i >= VCB || (i >= audio_bos && i <= audio_bos + 7 && (i != audio_eos || forbid_eos))) lv[r] = -INFINITY;
        argmax_merge(bv, bi, lv[r], i);
    }
    wave_argmax(bv, bi);
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
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
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
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    for (int j = 0; j < RK; ++j) {
        if (j * 64 >= k) break;
        if (lane + 64 * j < k) { sv[rk[j]] = ev[j]; si[rk[j]] = ei[j]; }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    int code = 0;
    if (lane == 0) {
        float sum = 0.f;
        for (int i = 0; i < k; ++i) sum += sv[i];
        const float u = mp_uniform(smp.cfg->seed, stream, step, cb);
        float cum = 0.f;
        code = si[k - 1];
        for (int i = 0; i < k; ++i) {
            cum += sv[i] / sum;
            if (u < cum) { code = si[i]; break; }
        }
    }
    code = __shfl(code, 0, 64);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    return code;
}

template <int NB, int K, int PRO>
__device__ __forceinline__ void prologue(const GemvP &p, float *act, float *red, float *sc) {
    const int tid = threadIdx.x;
    if constexpr (PRO == PRO_PLAIN) {
        for (int b = 0; b < NB; ++b)
            for (int k = tid * 4; k < K; k += MP_BLOCK * 4)
                *(float4 *)(act + b * K + k) = *(const float4 *)(p.src + (size_t)b * p.src_ld + k);
        lds_sync();
    } else if constexpr (PRO == PRO_LN && NB >= 2) {
        // batched: wave w owns slots w, w+4 (DPP-only statistics, one barrier)
        const int lane = tid & 63, w = tid >> 6;
        for (int b = w; b < NB; b += MP_NWAVES) {
            constexpr int PER = K / 64;
            float v[PER];
#pragma unroll
            for (int i = 0; i < PER; ++i) v[i] = p.src[(size_t)b * p.src_ld + lane + 64 * i];
            float mean, var;
            wave_meanvar<PER>(v, mean, var);
            const float rstd = 1.0f / sqrtf(var + p.eps);
            const bool st = p.hidden_out && blockIdx.x == 0;
            const int s = (p.trace && blockIdx.x == 0) ? p.step[b] : 0;
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int k = lane + 64 * i;
                const float y = ((v[i] - mean) * rstd) * p.lnw[k];
                act[b * K + k] = y;
                if (st) p.hidden_out[(size_t)b * K + k] = y;
                if (p.trace && blockIdx.x == 0 && s < p.trace_steps) p.trace[((size_t)b * p.trace_steps + s) * K + k] = y;
            }
        }
        lds_sync();
    } else if constexpr (PRO == PRO_LN) {
        for (int b = 0; b < NB; ++b) {
            float *store = nullptr;
            if (p.hidden_out && blockIdx.x == 0) store = p.hidden_out + (size_t)b * K;
            pro_ln_vec<NB, K>(p.src + (size_t)b * p.src_ld, p.lnw, p.eps, act + b * K, red, store);
            if (p.trace && blockIdx.x == 0) {
                lds_sync();
                const int s = p.step[b];
                if (s < p.trace_steps)
                    for (int k = tid; k < K; k += MP_BLOCK)
                        p.trace[((size_t)b * p.trace_steps + s) * K + k] = act[b * K + k];
            }
        }
        lds_sync();
    } else if constexpr (PRO == PRO_EMBED_LN && NB >= 2) {
        static_assert(K == D, "embed prologue is d_model wide");
        const int lane = tid & 63, w = tid >> 6;
        for (int b = w; b < NB; b += MP_NWAVES) {
            const int *c = p.codes + b * NCB;
            const int ps = p.pos[b];
            float x[K / 64];
#pragma unroll
            for (int i = 0; i < K / 64; ++i) {
                const int k = lane + 64 * i;
                float s = p.emb[((size_t)0 * VCB + c[0]) * D + k];
#pragma unroll
                for (int cb = 1; cb < NCB; ++cb) s = s + p.emb[((size_t)cb * VCB + c[cb]) * D + k];
                x[i] = s * 0.125f + p.pos_emb[(size_t)ps * D + k];
                if (blockIdx.x == 0) p.xres[(size_t)b * D + k] = x[i];
            }
            float mean, var;
            wave_meanvar<K / 64>(x, mean, var);
            const float rstd = 1.0f / sqrtf(var + p.eps);
#pragma unroll
            for (int i = 0; i < K / 64; ++i) {
                const int k = lane + 64 * i;
                act[b * K + k] = ((x[i] - mean) * rstd) * p.lnw[k];
            }
        }
        lds_sync();
    } else if constexpr (PRO == PRO_EMBED_LN) {
        static_assert(K == D, "embed prologue is d_model wide");
        for (int b = 0; b < NB; ++b) {
            const int *c = p.codes + b * NCB;
            const int ps = p.pos[b];
            float x[K / MP_BLOCK];
#pragma unroll
            for (int i = 0; i < K / MP_BLOCK; ++i) {
                const int k = tid + MP_BLOCK * i;
                float s = p.emb[((size_t)0 * VCB + c[0]) * D + k];
#pragma unroll
                for (int cb = 1; cb < NCB; ++cb) s = s + p.emb[((size_t)cb * VCB + c[cb]) * D + k];
                x[i] = s * 0.125f + p.pos_emb[(size_t)ps * D + k];
                if (blockIdx.x == 0) p.xres[(size_t)b * D + k] = x[i];
            }
            // LN over the freshly built x
            float mean, var;
            block_meanvar<K / MP_BLOCK>(x, red, mean, var);
            const float rstd = 1.0f / sqrtf(var + p.eps);
#pragma unroll
            for (int i = 0; i < K / MP_BLOCK; ++i) {
                const int k = tid + MP_BLOCK * i;
                act[b * K + k] = ((x[i] - mean) * rstd) * p.lnw[k];
            }
        }
        lds_sync();
    } else if constexpr (PRO == PRO_LTX_LN && NB >= 2) {
        const int lane = tid & 63, w = tid >> 6;
        for (int b = w; b < NB; b += MP_NWAVES) {
            float X[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int k = lane + 64 * i;
                X[i] = p.lt_s[((size_t)b * 9 + p.cb) * LTD + k] + p.lt_pos[(size_t)p.cb * LTD + k];
                if (blockIdx.x == 0) p.ltX[(size_t)b * LTD + k] = X[i];
            }
            float mean, var;
            wave_meanvar<4>(X, mean, var);
            const float rstd = 1.0f / sqrtf(var + p.eps);
#pragma unroll
            for (int i = 0; i < 4; ++i) act[b * K + lane + 64 * i] = ((X[i] - mean) * rstd) * p.lnw[lane + 64 * i];
        }
        lds_sync();
    } else if constexpr (PRO == PRO_LTARG_LN && NB >= 2) {
        const int lane = tid & 63, w = tid >> 6;
        for (int b = w; b < NB; b += MP_NWAVES) {
            int amax;
            const int code = wave_pick(p.logits + (size_t)b * VCB, p.ignore_eos || p.step[b] < 4, p.audio_bos, p.audio_eos,
                                       p.smp, b, p.step[b], p.cb - 1, sc + w * 2 * VCB, amax);
            if (blockIdx.x == 0 && lane == 0) {
                p.codes_cur[b * NCB + p.cb - 1] = code;
                if (amax == p.audio_eos) p.smp.argeos[b] = 1;
            }
            float X[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int k = lane + 64 * i;
                X[i] = p.ptab[((size_t)(p.cb - 1) * VCB + code) * LTD + k] + p.lt_pos[(size_t)p.cb * LTD + k];
                if (blockIdx.x == 0) p.ltX[(size_t)b * LTD + k] = X[i];
            }
            float mean, var;
            wave_meanvar<4>(X, mean, var);
            const float rstd = 1.0f / sqrtf(var + p.eps);
#pragma unroll
            for (int i = 0; i < 4; ++i) act[b * K + lane + 64 * i] = ((X[i] - mean) * rstd) * p.lnw[lane + 64 * i];
        }
        lds_sync();
    } else if constexpr (PRO == PRO_LT_ATTN && NB >= 2) {
        const int lane = tid & 63, w = tid >> 6;
        const int nk = p.cb + 1;
        for (int b = w; b < NB; b += MP_NWAVES) {
            const float4 q4 = *(const float4 *)(p.ltq + (size_t)b * LTD + 4 * lane);
            float sj[NCB];
#pragma unroll
            for (int j = 0; j < NCB; ++j)
                sj[j] = j < nk ? wave_sum(dotv(q4, *(const float4 *)(p.ltk + ((size_t)b * NCB + j) * LTD + 4 * lane))) *
                                     (1.0f / 16.0f)
                               : -INFINITY;
            float m = -INFINITY;
#pragma unroll
            for (int j = 0; j < NCB; ++j) m = fmaxf(m, sj[j]);
            float l = 0.f;
            float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int j = 0; j < NCB; ++j) {
                if (j >= nk) break;
                const float e = expf(sj[j] - m);
                l += e;
                const float4 v4 = *(const float4 *)(p.ltv + ((size_t)b * NCB + j) * LTD + 4 * lane);
                a.x += e * v4.x; a.y += e * v4.y; a.z += e * v4.z; a.w += e * v4.w;
            }
            const float il = 1.0f / l;
            *(float4 *)(act + b * K + 4 * lane) = make_float4(a.x * il, a.y * il, a.z * il, a.w * il);
        }
        lds_sync();
    } else if constexpr (PRO == PRO_LTX_LN) {
        static_assert(K == LTD, "LT is 256 wide");
        for (int b = 0; b < NB; ++b) {
            const int k = tid;
            const float X = p.lt_s[((size_t)b * 9 + p.cb) * LTD + k] + p.lt_pos[(size_t)p.cb * LTD + k];
            if (blockIdx.x == 0) p.ltX[(size_t)b * LTD + k] = X;
            const float xv[1] = {X};
            float mean, var;
            block_meanvar<1>(xv, red, mean, var);
            const float rstd = 1.0f / sqrtf(var + p.eps);
            act[b * K + k] = ((X - mean) * rstd) * p.lnw[k];
        }
        lds_sync();
    } else if constexpr (PRO == PRO_LT_ATTN) {
        static_assert(K == LTD, "LT is 256 wide");
        const int lane = tid & 63, w = tid >> 6;
        const int nk = p.cb + 1;
        for (int b = 0; b < NB; ++b) {
            const float4 q4 = *(const float4 *)(p.ltq + (size_t)b * LTD + 4 * lane);
            for (int j = w; j < nk; j += MP_NWAVES) {
                float v = dotv(q4, *(const float4 *)(p.ltk + ((size_t)b * NCB + j) * LTD + 4 * lane));
                v = wave_sum(v);
                if (lane == 0) sc[j] = v * (1.0f / 16.0f);  // 1/sqrt(256)
            }
            lds_sync();
            float m = -INFINITY;
            for (int j = 0; j < nk; ++j) m = fmaxf(m, sc[j]);
            float l = 0.f, a = 0.f;
            for (int j = 0; j < nk; ++j) {
                const float e = expf(sc[j] - m);
                l += e;
                a += e * p.ltv[((size_t)b * NCB + j) * LTD + tid];
            }
            act[b * K + tid] = a / l;
            lds_sync();
        }
    } else if constexpr (PRO == PRO_LTARG_LN) {
        static_assert(K == LTD, "LT is 256 wide");
        const int lane = tid & 63, w = tid >> 6;
        for (int b = 0; b < NB; ++b) {
            int code;
            if (p.smp.on) {
                if (w == 0) {
                    int amax;
                    code = wave_pick(p.logits + (size_t)b * VCB, p.ignore_eos || p.step[b] < 4, p.audio_bos,
                                     p.audio_eos, p.smp, b, p.step[b], p.cb - 1, sc, amax);
                    if (lane == 0) {
                        red[0] = __int_as_float(code);
                        if (blockIdx.x == 0 && amax == p.audio_eos) p.smp.argeos[b] = 1;
                    }
                }
                lds_sync();
                code = __float_as_int(red[0]);
                lds_sync();
            } else {
                code = block_masked_argmax(p, b, red);  // codebook cb-1's code
            }
            if (blockIdx.x == 0 && tid == 0) p.codes_cur[b * NCB + p.cb - 1] = code;
            const int k = tid;
            const float X = p.ptab[((size_t)(p.cb - 1) * VCB + code) * LTD + k] + p.lt_pos[(size_t)p.cb * LTD + k];
            if (blockIdx.x == 0) p.ltX[(size_t)b * LTD + k] = X;
            const float xv[1] = {X};
            float mean, var;
            block_meanvar<1>(xv, red, mean, var);
            const float rstd = 1.0f / sqrtf(var + p.eps);
            act[b * K + k] = ((X - mean) * rstd) * p.lnw[k];
        }
        lds_sync();
    }
}

// ---------------------------------------------------------------- GEMV core
// Rows [row0, row0+RW) of W (row-major [N][K]) dotted with act[NB][K].
// Lane l owns elements 4*(l + 64*i): every weight load is a 1 KiB coalesced
// wave-instruction; activations come from LDS with conflict-free ds_read_b128.
template <int NB, int RW, int K, int PRO, int EPI>
__global__ __launch_bounds__(MP_BLOCK) void gemv_kernel(GemvP p) {
    // No early exit on the done counter: a dependent load there would sit in
    // front of the weight stream of every launch. Once every slot is done the
    // iteration recomputes identical values (codes_prev / pos are frozen) and
    // lt_finalize_kernel refuses to touch the outputs.
    constexpr int VW = K >= 256 ? 4 : K / 64;
    constexpr int NV = K / (64 * VW);
    using VT = typename vecf<VW>::T;
    constexpr int SC = (PRO == PRO_LT_ATTN) ? 16
                       : (PRO == PRO_LTARG_LN) ? (NB >= 2 ? MP_NWAVES : 1) * 2 * VCB
                       : 1;
    __shared__ __attribute__((aligned(16))) float act[NB * K];
    __shared__ float red[8];
    __shared__ float sc[SC];

    // The weight rows do not depend on the prologue: issue the whole stream first
    // so the HBM latency overlaps the prologue's own dependent loads/reductions.
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int row0 = (blockIdx.x * MP_NWAVES + w) * RW;
    VT wv[RW][NV];
#pragma unroll
    for (int r = 0; r < RW; ++r) {
        const int n = row0 + r < p.N ? row0 + r : p.N - 1;
        const VT *wr = (const VT *)(p.W + (size_t)n * K);
#pragma unroll
        for (int i = 0; i < NV; ++i) wv[r][i] = wr[lane + 64 * i];
    }
    prologue<NB, K, PRO>(p, act, red, sc);
    float acc[RW][NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        VT av[NV];
#pragma unroll
        for (int i = 0; i < NV; ++i) av[i] = ((const VT *)(act + b * K))[lane + 64 * i];
#pragma unroll
        for (int r = 0; r < RW; ++r) {
            float s = 0.f;
#pragma unroll
            for (int i = 0; i < NV; ++i) s += dotv(wv[r][i], av[i]);
            acc[r][b] = wave_sum(s);
        }
    }
    if (lane != 0) return;
#pragma unroll
    for (int r = 0; r < RW; ++r) {
        const int n = row0 + r;
        if (n >= p.N) break;
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            const float v = acc[r][b];
            if constexpr (EPI == EPI_STORE) p.out[(size_t)b * p.out_ld + n] = v;
            else if constexpr (EPI == EPI_BIAS) p.out[(size_t)b * p.out_ld + n] = v + p.bias[n];
            else if constexpr (EPI == EPI_GELU) p.out[(size_t)b * p.out_ld + n] = gelu_tanh(v);
            else if constexpr (EPI == EPI_RESID) p.resid[(size_t)b * D + n] = v + p.resid[(size_t)b * D + n];
            else if constexpr (EPI == EPI_ADD_STORE) p.out[(size_t)b * p.out_ld + n] = v + p.addsrc[(size_t)b * p.out_ld + n];
            else if constexpr (EPI == EPI_QKV) {
                const size_t slot = ((size_t)(b * p.nlayers + p.layer) * p.max_seq + p.pos[b]) * D;
                if (n < D) p.out[(size_t)b * D + n] = v;
                else if (n < 2 * D) p.kc[slot + n - D] = v;
                else p.vc[slot + n - 2 * D] = v;
            } else if constexpr (EPI == EPI_LTQKV) {
                if (n < LTD) p.lq[(size_t)b * LTD + n] = v;
                else if (n < 2 * LTD) p.lk[((size_t)b * NCB + p.cb) * LTD + n - LTD] = v;
                else p.lv[((size_t)b * NCB + p.cb) * LTD + n - 2 * LTD] = v;
            }
        }
    }
}

// ---------------------------------------------------------------- SA decode attention
// Split-K over the key axis: workgroup (chunk, head, slot) handles 64 keys and
// writes (max, sum, o[64]); the last of a head's active chunks to arrive
// combines them in-launch (a[d] = sum_c e^(m_c-M) o_c[d] / sum_c e^(m_c-M) l_c)
// and writes the head's 64 outputs, so the O-projection reads a plain vector.
// 16 lanes x float4 cover one 64-dim key row (256 B, coalesced); a wave does 4
// keys per instruction. Keys j > pos are masked (L = pos + 1, magpie.cpp:3412).
__global__ __launch_bounds__(MP_BLOCK) void sa_attn_kernel(AttnP p) {
    const int c = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    __shared__ float sc[SA_CHUNK + MP_NWAVES * DH + 4];
    float *ow = sc + SA_CHUNK;  // [MP_NWAVES][DH]
    const int j0 = c * SA_CHUNK;
    const int kk = lane >> 4, dc = lane & 15;
    // Issue q, all 4 K rows and all 4 V rows of this lane first: rows j < max_seq
    // are always valid memory, so no load waits for the live length L = pos + 1.
    const float4 q4 = *(const float4 *)(p.q + (size_t)b * D + h * DH + 4 * dc);
    const size_t base = ((size_t)(b * p.nlayers + p.layer) * p.max_seq) * D + h * DH + 4 * dc;
    float4 k4[4], v4[4];
#pragma unroll
    for (int it = 0; it < 4; ++it) {
        const int j = j0 + w * 16 + it * 4 + kk;
        k4[it] = *(const float4 *)(p.kc + base + (size_t)j * D);
        v4[it] = *(const float4 *)(p.vc + base + (size_t)j * D);
    }
    const int L = p.pos[b] + 1;
    if (j0 >= L) return;  // inactive chunk: takes no ticket
    const int nact = (L + SA_CHUNK - 1) / SA_CHUNK;
    float *P = p.part + ((size_t)(b * NH + h) * p.nch + c) * PART_STRIDE;
    float s[4];
#pragma unroll
    for (int it = 0; it < 4; ++it) {
        const int j = j0 + w * 16 + it * 4 + kk;
        const float v = group_sum<16>(dotv(q4, k4[it]));
        s[it] = j < L ? v * 0.125f : -INFINITY;  // 1/sqrt(64)
    }
    if (dc == 0)
#pragma unroll
        for (int it = 0; it < 4; ++it) sc[w * 16 + it * 4 + kk] = s[it];
    lds_sync();
    // every wave reduces the chunk's 64 scores itself: lane i holds key i
    const float si = sc[lane];
    const float m = wave_max(si);
    const float l = wave_sum(si == -INFINITY ? 0.f : expf(si - m));
    float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int it = 0; it < 4; ++it) {
        const int j = j0 + w * 16 + it * 4 + kk;
        if (j < L) {
            const float e = expf(s[it] - m);
            o.x += e * v4[it].x; o.y += e * v4[it].y; o.z += e * v4[it].z; o.w += e * v4[it].w;
        }
    }
#pragma unroll
    for (int msk = 16; msk <= 32; msk <<= 1) {
        o.x += __shfl_xor(o.x, msk, 64); o.y += __shfl_xor(o.y, msk, 64);
        o.z += __shfl_xor(o.z, msk, 64); o.w += __shfl_xor(o.w, msk, 64);
    }
    if (lane < 16) *(float4 *)(&ow[w * DH + 4 * lane]) = o;
    lds_sync();
    if (tid < DH / 2) {
        const int d = 2 * tid;
        st_sc1(P + 16 + d, (ow[d] + ow[DH + d]) + (ow[2 * DH + d] + ow[3 * DH + d]),
               (ow[d + 1] + ow[DH + d + 1]) + (ow[2 * DH + d + 1] + ow[3 * DH + d + 1]));
    } else if (tid == 64) {
        st_sc1(P, m, l);
    }
    if (!arrive_last(p.cnt + b * NH + h, (unsigned)nact, sc + SA_CHUNK + MP_NWAVES * DH, p.sc1_loads != 0)) return;
    if (tid >= DH) return;
    const float *Pb = p.part + (size_t)(b * NH + h) * p.nch * PART_STRIDE;
    float mv[NCH_MAX], lv[NCH_MAX], ov[NCH_MAX];
#pragma unroll
    for (int cc = 0; cc < NCH_MAX; ++cc) {  // unconditional (clamped) loads: no branch per load
        const float *Pc = Pb + min(cc, nact - 1) * PART_STRIDE;
        mv[cc] = ld_sc1(Pc);
        lv[cc] = ld_sc1(Pc + 1);
        ov[cc] = ld_sc1(Pc + 16 + tid);
    }
#pragma unroll
    for (int cc = 0; cc < NCH_MAX; ++cc)
        if (cc >= nact) { mv[cc] = -INFINITY; lv[cc] = 0.f; ov[cc] = 0.f; }
    float M = -INFINITY;
#pragma unroll
    for (int cc = 0; cc < NCH_MAX; ++cc) M = fmaxf(M, mv[cc]);
    float num = 0.f, den = 0.f;
#pragma unroll
    for (int cc = 0; cc < NCH_MAX; ++cc) {
        const float e = mv[cc] == -INFINITY ? 0.f : expf(mv[cc] - M);
        den += e * lv[cc];
        num += e * ov[cc];
    }
    p.out[(size_t)b * D + h * DH + tid] = num / den;
}

// ---------------------------------------------------------------- fused XA
// grid (768/64, B): every workgroup recomputes LN(x) and all T scores (K' rows
// are L2-resident after the first workgroup), then owns 64 output dims.
__global__ __launch_bounds__(MP_BLOCK) void xa_fused_kernel(XaP p) {
    __shared__ __attribute__((aligned(16))) float act[D];
    __shared__ float red[8];
    __shared__ float sc[TMAX_LIMIT];
    __shared__ float part[MP_NWAVES][64];
    const int b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int d0 = blockIdx.x * 64;
    const int Tb = p.T[b];
    const size_t base = ((size_t)(b * p.nlayers + p.layer) * p.Tmax) * D;
    const float *Kp = p.kp + base, *Vp = p.vp + base;
    // LN(x) (magpie.cpp:3513)
    {
        float v[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) v[i] = p.x[(size_t)b * D + tid + MP_BLOCK * i];
        float mean, var;
        block_meanvar<3>(v, red, mean, var);
        const float rstd = 1.0f / sqrtf(var + p.eps);
#pragma unroll
        for (int i = 0; i < 3; ++i) act[tid + MP_BLOCK * i] = ((v[i] - mean) * rstd) * p.lnw[tid + MP_BLOCK * i];
    }
    lds_sync();
    const float4 a0 = *(const float4 *)(act + 4 * lane), a1 = *(const float4 *)(act + 256 + 4 * lane),
                 a2 = *(const float4 *)(act + 512 + 4 * lane);
    const float scale = 1.0f / sqrtf((float)DXA);
    // scores: wave w takes rows w, w+4, ...; 4 rows (12 float4 per lane) in flight
    for (int tb = w; tb < Tb; tb += 16) {
        float4 k[4][3];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int t = tb + 4 * u;
            const float *kr = Kp + (size_t)(t < Tb ? t : 0) * D;
            k[u][0] = *(const float4 *)(kr + 4 * lane);
            k[u][1] = *(const float4 *)(kr + 256 + 4 * lane);
            k[u][2] = *(const float4 *)(kr + 512 + 4 * lane);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int t = tb + 4 * u;
            const float sv = wave_sum(dotv(k[u][0], a0) + dotv(k[u][1], a1) + dotv(k[u][2], a2));
            if (lane == 0 && t < Tb) sc[t] = sv * scale;
        }
    }
    lds_sync();
    float m = -INFINITY;
    for (int t = tid; t < Tb; t += MP_BLOCK) m = fmaxf(m, sc[t]);
    m = block_max(m, red);
    float l = 0.f;
    for (int t = tid; t < Tb; t += MP_BLOCK) { const float e = expf(sc[t] - m); sc[t] = e; l += e; }
    l = block_sum(l, red);
    // out[d] = sum_t e_t V'_t[d] / l for the workgroup's 64 dims; 4 time groups
    float acc = 0.f;
#pragma unroll 8
    for (int t = w; t < Tb; t += MP_NWAVES) acc += sc[t] * Vp[(size_t)t * D + d0 + lane];
    part[w][lane] = acc;
    lds_sync();
    if (tid < 64) {
        const float o = ((part[0][tid] + part[1][tid]) + (part[2][tid] + part[3][tid])) / l;
        p.x_out[(size_t)b * D + d0 + tid] = o + p.x[(size_t)b * D + d0 + tid];
    }
}

hipError_t op_xa(const XaP &p, int B, hipStream_t s) {
    if (!p.x || !p.x_out || !p.lnw || !p.kp || !p.vp || !p.T || p.Tmax < 1 || p.Tmax > TMAX_LIMIT) return hipErrorInvalidValue;
    hipLaunchKernelGGL(xa_fused_kernel, dim3(D / 64, B), dim3(MP_BLOCK), 0, s, p);
    return hipGetLastError();
}

// ---------------------------------------------------------------- frame finalize
// Codebook 7's masked argmax, then the reference's loop bookkeeping
// (magpie.cpp:4340-4358): stop on EOS in any codebook (frame not emitted), else
// append the frame; stop at max_dec_steps; otherwise the frame becomes the next
// decoder input and the position advances.
__global__ __launch_bounds__(MP_BLOCK) void lt_finalize_kernel(FinP p) {
    const int b = blockIdx.x, tid = threadIdx.x;
    if (p.done[b]) return;
    __shared__ float red[8];
    int i0, amax;
    if (p.smp.on) {  // one wave draws
        __shared__ float scratch[2 * VCB];
        if (tid >= 64) return;
        i0 = wave_pick(p.logits + (size_t)b * VCB, p.ignore_eos || p.step[b] < 4, p.audio_bos, p.audio_eos, p.smp, b,
                       p.step[b], NCB - 1, scratch, amax);
        if (tid != 0) return;
    } else {
        const float *lg = p.logits + (size_t)b * VCB;
        const bool forbid_eos = p.ignore_eos || p.step[b] < 4;
        float bv = -INFINITY;
        int bi = 0x7fffffff;
        for (int i = tid; i < VCB; i += MP_BLOCK) {
            float v = lg[i];
            if (i >= p.audio_bos && i <= p.audio_bos + 7 && (i != p.audio_eos || forbid_eos)) v = -INFINITY;
            argmax_merge(bv, bi, v, i);
        }
        wave_argmax(bv, bi);
        if ((tid & 63) == 0) { red[tid >> 6] = bv; ((int *)red)[4 + (tid >> 6)] = bi; }
        lds_sync();
        if (tid != 0) return;
        float v0 = red[0];
        i0 = ((int *)red)[4];
        for (int w = 1; w < MP_NWAVES; ++w) argmax_merge(v0, i0, red[w], ((int *)red)[4 + w]);
        if (i0 < 0 || i0 >= VCB) i0 = 0;
        amax = i0;
    }
    int *cc = p.codes_cur + b * NCB;
    cc[NCB - 1] = i0;
    // EOS if any codebook's sampled code or argmax is EOS (magpie.cpp:4340-4348)
    bool eos = amax == p.audio_eos;
    eos |= p.smp.argeos[b] != 0;
    p.smp.argeos[b] = 0;
    for (int cb = 0; cb < NCB; ++cb) eos |= cc[cb] == p.audio_eos;
    const int s = p.step[b];
    if (eos) {
        p.done[b] = 1;
        p.nframes[b] = s;
        atomicAdd(p.ndone, 1);
        return;
    }
    for (int cb = 0; cb < NCB; ++cb) p.codes_out[((size_t)b * p.max_steps + s) * NCB + cb] = cc[cb];
    p.step[b] = s + 1;
    if (s + 1 >= p.max_steps) {
        p.done[b] = 1;
        p.nframes[b] = s + 1;
        atomicAdd(p.ndone, 1);
        return;
    }
    for (int cb = 0; cb < NCB; ++cb) p.codes_prev[b * NCB + cb] = cc[cb];
    p.pos[b] += 1;
}

// ---------------------------------------------------------------- host launchers
// Host-side check that every pointer the (PRO, EPI) pair dereferences is set:
// a mismatch between an op's compile-time epilogue and its arguments must fail
// at launch, not fault on the device.
template <int PRO, int EPI>
static bool gemv_args_ok(const GemvP &p) {
    if (!p.W || p.N <= 0) return false;
    bool ok = true;
    if constexpr (PRO == PRO_PLAIN) ok &= p.src != nullptr;
    if constexpr (PRO == PRO_LN) ok &= p.src && p.lnw;
    if constexpr (PRO == PRO_EMBED_LN) ok &= p.emb && p.codes && p.pos_emb && p.pos && p.xres && p.lnw;
    if constexpr (PRO == PRO_LTX_LN) ok &= p.lt_s && p.lt_pos && p.ltX && p.lnw;
    if constexpr (PRO == PRO_LT_ATTN) ok &= p.ltq && p.ltk && p.ltv;
    if constexpr (PRO == PRO_LTARG_LN) ok &= p.logits && p.codes_cur && p.ptab && p.lt_pos && p.ltX && p.lnw && p.step && p.smp.cfg && p.smp.argeos;
    if constexpr (EPI == EPI_STORE || EPI == EPI_GELU) ok &= p.out != nullptr;
    if constexpr (EPI == EPI_BIAS) ok &= p.out && p.bias;
    if constexpr (EPI == EPI_RESID) ok &= p.resid != nullptr;
    if constexpr (EPI == EPI_ADD_STORE) ok &= p.out && p.addsrc;
    if constexpr (EPI == EPI_QKV) ok &= p.out && p.kc && p.vc && p.pos;
    if constexpr (EPI == EPI_LTQKV) ok &= p.lq && p.lk && p.lv;
    return ok;
}

template <int NB, int RW, int K, int PRO, int EPI>
static hipError_t launch_gemv(const GemvP &p, hipStream_t s) {
    if (!gemv_args_ok<PRO, EPI>(p)) return hipErrorInvalidValue;
    const int rows_per_block = MP_NWAVES * RW;
    const int grid = (p.N + rows_per_block - 1) / rows_per_block;
    hipLaunchKernelGGL((gemv_kernel<NB, RW, K, PRO, EPI>), dim3(grid), dim3(MP_BLOCK), 0, s, p);
    return hipGetLastError();
}

// Named entry points (one per fused op of the decode iteration), instantiated
// for NB in {1, 2, 4, 8}.
#define MP_DECODE_OPS(NB)                                                                                        \
    hipError_t op_qkv_embed_##NB(const GemvP &p, hipStream_t s) { return launch_gemv<NB, 2, D, PRO_EMBED_LN, EPI_QKV>(p, s); } \
    hipError_t op_qkv_##NB(const GemvP &p, hipStream_t s) { return launch_gemv<NB, 2, D, PRO_LN, EPI_QKV>(p, s); }             \
    hipError_t op_oproj_##NB(const GemvP &p, hipStream_t s) { return launch_gemv<NB, 1, D, PRO_PLAIN, EPI_RESID>(p, s); }    \
    hipError_t op_ff1_##NB(const GemvP &p, hipStream_t s) { return launch_gemv<NB, 2, D, PRO_LN, EPI_GELU>(p, s); }            \
    hipError_t op_ff2_##NB(const GemvP &p, hipStream_t s) { return launch_gemv<NB, 1, DFF, PRO_PLAIN, EPI_ADD_STORE>(p, s); }  \
    hipError_t op_lt_in0_##NB(const GemvP &p, hipStream_t s) { return launch_gemv<NB, 1, D, PRO_LN, EPI_BIAS>(p, s); }         \
    hipError_t op_lt_a_##NB(const GemvP &p, hipStream_t s) { return launch_gemv<NB, 1, LTD, PRO_LTX_LN, EPI_LTQKV>(p, s); }    \
    hipError_t op_lt_ag_##NB(const GemvP &p, hipStream_t s) { return launch_gemv<NB, 1, LTD, PRO_LTARG_LN, EPI_LTQKV>(p, s); } \
    hipError_t op_lt_b_##NB(const GemvP &p, hipStream_t s) { return launch_gemv<NB, 1, LTD, PRO_LT_ATTN, EPI_ADD_STORE>(p, s); } \
    hipError_t op_lt_c_##NB(const GemvP &p, hipStream_t s) { return launch_gemv<NB, 1, LTD, PRO_LN, EPI_GELU>(p, s); }         \
    hipError_t op_lt_d_##NB(const GemvP &p, hipStream_t s) { return launch_gemv<NB, 1, LTF, PRO_PLAIN, EPI_ADD_STORE>(p, s); } \
    hipError_t op_lt_e_##NB(const GemvP &p, hipStream_t s) { return launch_gemv<NB, 2, LTD, PRO_PLAIN, EPI_BIAS>(p, s); }      \


MP_DECODE_OPS(1)
MP_DECODE_OPS(2)
MP_DECODE_OPS(4)
MP_DECODE_OPS(8)

hipError_t op_sa_attn(const AttnP &p, int B, hipStream_t s) {
    if (!p.q || !p.kc || !p.vc || !p.pos || !p.part || !p.out || !p.cnt || p.nch < 1 || p.nch > NCH_MAX ||
        p.nch * SA_CHUNK > p.max_seq)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(sa_attn_kernel, dim3(p.nch, NH, B), dim3(MP_BLOCK), 0, s, p);
    return hipGetLastError();
}

hipError_t op_finalize(const FinP &p, int B, hipStream_t s) {
    if (!p.smp.cfg || !p.smp.argeos) return hipErrorInvalidValue;
    hipLaunchKernelGGL(lt_finalize_kernel, dim3(B), dim3(MP_BLOCK), 0, s, p);
    return hipGetLastError();
}

}  // namespace mp
