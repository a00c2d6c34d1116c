// The fused cross-attention (XA) body shared by xa_part_kernel and the
// O-projection launches that carry it (EPI_RESID_XA: the f32 GEMV and the 16-bit
// MFMA families), and the O-projection side of that hand-off.
#pragma once
#include "mp_device.hpp"
#include "mp_fused.hpp"
#include "mp_params.hpp"

namespace mp {

// XA reassociated: with K'_t = W_q^T K_t and V'_t = W_o V_t precomputed per
// utterance and layer, x += sum_t softmax_t(K'_t . LN(x) / sqrt(128)) V'_t.
// Split over text keys: grid (split, slot), 8 waves. Split s takes keys
// [s*chunk, (s+1)*chunk) of T; wave w takes t = t0 + w, t0 + w + 8, ... with its
// first keys' K' and V' rows issued before x is fetched (one round trip), every
// wave normalises x itself (DPP statistics, no barrier), keeps an online softmax
// (m, l, o[768] in 12 registers per lane); the 8 wave states merge in LDS and
// the split's state (m, l, unnormalised O[768]) is stored. The next op (FFN up,
// PRO_XA_LN) merges the XA_SPLITS states, adds x and normalises.
#ifndef MP_XA_WAVES
#define MP_XA_WAVES 4
#define MP_XA_KPW 4
#endif
constexpr int XA_WAVES = MP_XA_WAVES, XA_THREADS = XA_WAVES * 64, XA_KPW = MP_XA_KPW;  // keys in flight per wave
constexpr int XA_V = D / 256;  // float4 per lane per 768-row: lane owns elements 4 lane + 256 i + (0..3)
static_assert(XA_THREADS == MP_BLOCK, "XA workgroups ride in the O-projection launch (EPI_RESID_XA)");
// Hand-off bound: polls of the x1 granules before an XA workgroup gives up (with
// s_sleep between polls this is far beyond any O-projection's duration)
constexpr unsigned HX_SPIN_LIMIT = 1u << 20;
using gu64 = __attribute__((address_space(1))) unsigned long long;
using gi32 = __attribute__((address_space(1))) int;

// a {tag, value} granule's value once the wave sees the tag on every lane (bounded)
__device__ __forceinline__ float gh_wait(const unsigned long long *g, unsigned tag, int *err) {
    for (unsigned spins = 0;; ++spins) {
        const unsigned long long u = __hip_atomic_load((const gu64 *)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__all((unsigned)(u >> 32) == tag)) return __uint_as_float((unsigned)u);
        if (spins >= HX_SPIN_LIMIT) {  // never seen: poison and say so (HX_ERR_LT: the LT's edges use it)
            if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_or((gi32 *)err, HX_ERR_LT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return __builtin_nanf("");
        }
        __builtin_amdgcn_s_sleep(1);
    }
}
// N granules per lane (g[STRIDE j], j < N) polled together: one memory round trip per
// poll for all of them (N gh_wait calls in a row cost N round trips even when every
// granule is already there)
template <int N, int STRIDE>
__device__ __forceinline__ void gh_wait_n(const unsigned long long *g, unsigned tag, float (&v)[N], int *err) {
    for (unsigned spins = 0;; ++spins) {
        bool ok = true;
#pragma unroll
        for (int j = 0; j < N; ++j) {
            const unsigned long long u = __hip_atomic_load((const gu64 *)g + STRIDE * j, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT);
            v[j] = __uint_as_float((unsigned)u);
            ok &= (unsigned)(u >> 32) == tag;
        }
        if (__all(ok)) return;
        if (spins >= HX_SPIN_LIMIT) {  // never seen: poison and say so (HX_ERR_LT: the LT's edges use it)
            if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_or((gi32 *)err, HX_ERR_LT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
            for (int j = 0; j < N; ++j) v[j] = __builtin_nanf("");
            return;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}
// One round of the XA online softmax: keys tb + XA_WAVES u (u < XA_KPW; those >= t1
// are masked), K' rows k[u], V' rows vv[u], query h (this lane's elements).
// score_u = wave_sum(fmaf chain of k . h over the lane's elements) * scale; one
// rescale c = exp(m - mn) for the round, then the keys' e_u = exp(score_u - mn) added
// in key order: l = l c + Σ e_u, o = o c + Σ e_u v_u (each term an explicit fmaf).
__device__ __forceinline__ void xa_round(const float4 (&k)[XA_KPW][XA_V], const float4 (&vv)[XA_KPW][XA_V],
                                         const float4 (&h)[XA_V], float scale, int tb, int t1, float &m, float &l,
                                         float4 (&o)[XA_V]) {
#pragma clang fp contract(off)
    float sv[XA_KPW], mn = m;
#pragma unroll
    for (int u = 0; u < XA_KPW; ++u) {
        float acc = 0.f;
#pragma unroll
        for (int i = 0; i < XA_V; ++i) {
            acc = fmaf(k[u][i].x, h[i].x, acc);
            acc = fmaf(k[u][i].y, h[i].y, acc);
            acc = fmaf(k[u][i].z, h[i].z, acc);
            acc = fmaf(k[u][i].w, h[i].w, acc);
        }
        sv[u] = acc;
    }
    // the keys' wave sums advanced together, unconditionally (wave_sum_n: wave_sum's tree per
    // key), then the keys past t1 masked: the same values as one guarded wave_sum per key
    wave_sum_n<XA_KPW>(sv);
#pragma unroll
    for (int u = 0; u < XA_KPW; ++u) {
        sv[u] = tb + XA_WAVES * u < t1 ? sv[u] * scale : -INFINITY;
        mn = fmaxf(mn, sv[u]);
    }
    const float c = expf(m - mn);
    l = l * c;
#pragma unroll
    for (int i = 0; i < XA_V; ++i) { o[i].x = o[i].x * c; o[i].y = o[i].y * c; o[i].z = o[i].z * c; o[i].w = o[i].w * c; }
#pragma unroll
    for (int u = 0; u < XA_KPW; ++u) {
        const float e = expf(sv[u] - mn);
        l = l + e;
#pragma unroll
        for (int i = 0; i < XA_V; ++i) {
            o[i].x = fmaf(e, vv[u][i].x, o[i].x); o[i].y = fmaf(e, vv[u][i].y, o[i].y);
            o[i].z = fmaf(e, vv[u][i].z, o[i].z); o[i].w = fmaf(e, vv[u][i].w, o[i].w);
        }
    }
    m = mn;
}

// Split sp of slot b. HANDOFF: x1 comes from the O-projection in the same launch,
// as {tag, value} granules xh[b][768] (EPI_RESID_XA): every wave sweeps all 768
// with relaxed agent-scope loads (write-through producer stores, so no fence is
// needed) until every tag matches, after its K'/V' rows are already in flight.
template <bool HANDOFF>
__device__ __forceinline__ void xa_part(const XaP &p, int sp, int b, unsigned long long *xh, unsigned tag, int *err,
                                        int dep, unsigned long long *ts = nullptr, unsigned long long t_start = 0) {
    __shared__ float wm[XA_WAVES], wl[XA_WAVES];
    __shared__ __attribute__((aligned(16))) float wo[XA_WAVES][D];
    __shared__ __attribute__((aligned(16))) float x1row[HANDOFF ? D : 4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int Tb = p.T[b];
    const int chunk = (Tb + XA_SPLITS - 1) / XA_SPLITS;
    const int t0 = sp * chunk, t1 = min(Tb, t0 + chunk);
    const size_t base = ((size_t)(b * p.nlayers + p.layer) * p.Tmax) * D;
    const float *Kp = p.kp + base + 4 * lane + dep, *Vp = p.vp + base + 4 * lane;
    float4 k[XA_KPW][XA_V], vv[XA_KPW][XA_V];
#pragma unroll
    for (int u = 0; u < XA_KPW; ++u) {
        const int t = t0 + w + XA_WAVES * u;
        const size_t r = (size_t)(t < t1 ? t : 0) * D;
#pragma unroll
        for (int i = 0; i < XA_V; ++i) {
            k[u][i] = *(const float4 *)(Kp + r + 256 * i);
            vv[u][i] = *(const float4 *)(Vp + r + 256 * i);
        }
    }
    float4 h[XA_V];
    {   // LN(x) (magpie.cpp:3513), every wave for itself (DPP statistics, no barrier)
        float4 x4[XA_V], g4[XA_V];
#pragma unroll
        for (int i = 0; i < XA_V; ++i) g4[i] = *(const float4 *)(p.lnw + 4 * lane + 256 * i);
        if constexpr (HANDOFF) {
            // wave w sweeps its quarter of x1 (3 granules per lane) into the shared row, the
            // workgroup barrier publishes it (one poller per granule: with every wave
            // polling the whole row, the merge barrier waited for the unluckiest wave's
            // next round trip after x1 was complete)
            constexpr int PQ = D / 64 / XA_WAVES;
            static_assert(PQ * XA_WAVES * 64 == D, "x1 splits into one quarter per wave");
            gu64 *g = (gu64 *)(xh + (size_t)b * D) + w * PQ * 64;
            float xv[PQ];
            for (unsigned spins = 0;; ++spins) {
                bool ok = true;
#pragma unroll
                for (int j = 0; j < PQ; ++j) {
                    const unsigned long long u = __hip_atomic_load(g + lane + 64 * j, __ATOMIC_RELAXED,
                                                                   __HIP_MEMORY_SCOPE_AGENT);
                    xv[j] = __uint_as_float((unsigned)u);
                    ok &= (unsigned)(u >> 32) == tag;
                }
                if (__all(ok)) break;
                if (spins >= HX_SPIN_LIMIT) {  // never seen: poison the output and say so
                    if (lane == 0) __hip_atomic_fetch_or((gi32 *)err, HX_ERR_XA, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
                    for (int j = 0; j < PQ; ++j) xv[j] = __builtin_nanf("");
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
#pragma unroll
            for (int j = 0; j < PQ; ++j) x1row[w * PQ * 64 + lane + 64 * j] = xv[j];
            lds_sync();
            ts_phase<0>(ts, t_start);  // profiling: when the workgroup saw all of x1
#pragma unroll
            for (int i = 0; i < XA_V; ++i) x4[i] = *(const float4 *)&x1row[4 * lane + 256 * i];
        } else {
#pragma unroll
            for (int i = 0; i < XA_V; ++i) x4[i] = *(const float4 *)(p.x + (size_t)b * D + 4 * lane + 256 * i);
        }
        float v[4 * XA_V];
#pragma unroll
        for (int i = 0; i < XA_V; ++i) { v[4 * i] = x4[i].x; v[4 * i + 1] = x4[i].y; v[4 * i + 2] = x4[i].z; v[4 * i + 3] = x4[i].w; }
        float mean, var;
        wave_meanvar<4 * XA_V>(v, mean, var);
        const float rstd = 1.0f / sqrtf(var + p.eps);
#pragma unroll
        for (int i = 0; i < XA_V; ++i)
            h[i] = make_float4(((x4[i].x - mean) * rstd) * g4[i].x, ((x4[i].y - mean) * rstd) * g4[i].y,
                               ((x4[i].z - mean) * rstd) * g4[i].z, ((x4[i].w - mean) * rstd) * g4[i].w);
        if (p.q_f16)  // h . K'_t = q . K_t with q = W_q f16(h): the rounding commutes through K'
#pragma unroll
            for (int i = 0; i < XA_V; ++i)
                h[i] = make_float4((float)(_Float16)h[i].x, (float)(_Float16)h[i].y, (float)(_Float16)h[i].z,
                                   (float)(_Float16)h[i].w);
    }
    ts_phase<1>(ts, t_start);  // profiling: LN done
    const float scale = 1.0f / sqrtf((float)DXA);
    float m = -INFINITY, l = 0.f;
    float4 o[XA_V];
#pragma unroll
    for (int i = 0; i < XA_V; ++i) o[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int tb = t0 + w; tb < t1; tb += XA_WAVES * XA_KPW) {
        // A round's XA_KPW scores first (independent wave reductions the scheduler
        // interleaves), then one online-softmax update for the set (keys past t1 weigh
        // 0). Every rounding is spelled out (contraction off, explicit fmaf in a fixed
        // order), so each instantiation of this body (batch 1 / batched, handed-off /
        // standalone, f32 / 16-bit families) computes the same bits.
        xa_round(k, vv, h, scale, tb, t1, m, l, o);
        const int tn = tb + XA_WAVES * XA_KPW;
        if (tn >= t1) break;
#pragma unroll
        for (int u = 0; u < XA_KPW; ++u) {  // next keys (long texts)
            const int t = tn + XA_WAVES * u;
            const size_t r = (size_t)(t < t1 ? t : 0) * D;
#pragma unroll
            for (int i = 0; i < XA_V; ++i) {
                k[u][i] = *(const float4 *)(Kp + r + 256 * i);
                vv[u][i] = *(const float4 *)(Vp + r + 256 * i);
            }
        }
    }
    ts_phase<2>(ts, t_start);  // profiling: this (first) wave's keys done
#pragma unroll
    for (int i = 0; i < XA_V; ++i) *(float4 *)&wo[w][4 * lane + 256 * i] = o[i];
    if (lane == 0) { wm[w] = m; wl[w] = l; }
    lds_sync();
    ts_phase<3>(ts, t_start);  // profiling: every wave's keys done
    float M = -INFINITY;
#pragma unroll
    for (int q = 0; q < XA_WAVES; ++q) M = fmaxf(M, wm[q]);
    float den = 0.f, e[XA_WAVES];
#pragma unroll
    for (int q = 0; q < XA_WAVES; ++q) {
        e[q] = wm[q] == -INFINITY ? 0.f : expf(wm[q] - M);
        den = fmaf(e[q], wl[q], den);
    }
    float *pp = p.part + ((size_t)b * XA_SPLITS + sp) * XA_PART;
    const unsigned long long tagx = (unsigned long long)tag << 32;  // XaP::x2: the granules' tag
    if (tid < D / 4) {
        float4 num = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int q = 0; q < XA_WAVES; ++q) {
            const float4 v4 = *(const float4 *)&wo[q][4 * tid];
            num.x = fmaf(e[q], v4.x, num.x); num.y = fmaf(e[q], v4.y, num.y);
            num.z = fmaf(e[q], v4.z, num.z); num.w = fmaf(e[q], v4.w, num.w);
        }
        if (p.x2) {  // granules: the slot's split workgroups merge them (xa_merge_split)
            gu64 *g = (gu64 *)p.gh + ((size_t)b * XA_SPLITS + sp) * XA_PART + 4 + 4 * tid;
            __hip_atomic_store(g, tagx | __float_as_uint(num.x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(g + 1, tagx | __float_as_uint(num.y), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(g + 2, tagx | __float_as_uint(num.z), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(g + 3, tagx | __float_as_uint(num.w), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            *(float4 *)(pp + 4 + 4 * tid) = num;
        }
    }
    if (tid == 0) {
        if (p.x2) {
            gu64 *g = (gu64 *)p.gh + ((size_t)b * XA_SPLITS + sp) * XA_PART;
            __hip_atomic_store(g, tagx | __float_as_uint(M), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(g + 1, tagx | __float_as_uint(den), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            pp[0] = M; pp[1] = den;
        }
    }
}

// XaP::x2 (16 slots), after xa_part: split sp of slot b merges outputs
// [192 sp, 192 sp + 192) from the XA_SPLITS states' granules (one thread per output, a
// bounded sweep) and writes x2 = x1 + merged XA with PRO_XA_LN's arithmetic
// (split_weights, split_merge, xa_x2), x1 from the granules this workgroup saw complete.
__device__ __forceinline__ void xa_merge_split(const XaP &p, int sp, int b, const unsigned long long *xh, unsigned tag,
                                               int *err) {
    constexpr int MO = D / XA_SPLITS;
    const int tid = threadIdx.x;
    if (tid >= MO) return;  // no barrier follows
    const gu64 *g = (const gu64 *)p.gh + (size_t)b * XA_SPLITS * XA_PART;
    const int k = MO * sp + tid;
    float ms[XA_SPLITS], ls[XA_SPLITS], o[XA_SPLITS], e[XA_SPLITS], rd;
    // x1 (complete: this workgroup saw all of it) issued ahead of the sweep, not a round
    // trip after it
    const float x1 = __uint_as_float((unsigned)__hip_atomic_load((const gu64 *)xh + (size_t)b * D + k, __ATOMIC_RELAXED,
                                                                  __HIP_MEMORY_SCOPE_AGENT));
    for (unsigned spins = 0;; ++spins) {
        bool ok = true;
#pragma unroll
        for (int s = 0; s < XA_SPLITS; ++s) {
            const unsigned long long um = __hip_atomic_load(g + s * XA_PART, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long ul = __hip_atomic_load(g + s * XA_PART + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long uo = __hip_atomic_load(g + s * XA_PART + 4 + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ok &= (unsigned)(um >> 32) == tag && (unsigned)(ul >> 32) == tag && (unsigned)(uo >> 32) == tag;
            ms[s] = __uint_as_float((unsigned)um);
            ls[s] = __uint_as_float((unsigned)ul);
            o[s] = __uint_as_float((unsigned)uo);
        }
        if (__all(ok)) break;
        if (spins >= HX_SPIN_LIMIT) {  // never seen: poison the output and say so
            if ((tid & 63) == 0) __hip_atomic_fetch_or((gi32 *)err, HX_ERR_XA, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
            for (int s = 0; s < XA_SPLITS; ++s) o[s] = __builtin_nanf("");
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    split_weights<XA_SPLITS>(ms, ls, e, rd);
    const float a = split_merge<XA_SPLITS>(e, o, rd);
    p.x2[(size_t)b * D + k] = xa_x2(make_float4(a, 0.f, 0.f, 0.f), make_float4(x1, 0.f, 0.f, 0.f)).x;
}

// EPI_RESID_XA epilogue, output (row n, slot b): resid += v, and the new x1 value
// published as a {tag, value} granule with a relaxed agent-scope (write-through) store
__device__ __forceinline__ void publish_x1(const GemvP &p, float v, int n, int b) {
    float *r = p.resid + (size_t)b * D + n;
    const float x1 = v + *r;
    *r = x1;
    const unsigned tag = (unsigned)p.iter[0] * 64u + p.layer + 1u;
    __hip_atomic_store((gu64 *)(p.xh + (size_t)b * D + n), ((unsigned long long)tag << 32) | __float_as_uint(x1),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the same with the residual element loaded at launch start (epi_operand)
__device__ __forceinline__ void publish_x1_op(const GemvP &p, float v, int n, int b, float r0) {
    const float x1 = v + r0;
    p.resid[(size_t)b * D + n] = x1;
    const unsigned tag = (unsigned)p.iter[0] * 64u + p.layer + 1u;
    __hip_atomic_store((gu64 *)(p.xh + (size_t)b * D + n), ((unsigned long long)tag << 32) | __float_as_uint(x1),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the launch's XA workgroups (blockIdx.x >= nrow_blocks): split k % XA_SPLITS of slot k / XA_SPLITS
__device__ __forceinline__ void xa_tail(const GemvP &p, unsigned long long t_start) {
    const int k = blockIdx.x - p.nrow_blocks;
    xa_part<true>(p.xa, k % XA_SPLITS, k / XA_SPLITS, p.xh, (unsigned)p.iter[0] * 64u + p.layer + 1u, p.hx_err,
                  ts_dep(t_start), p.ts, t_start);
    if (p.xa.x2) xa_merge_split(p.xa, k % XA_SPLITS, k / XA_SPLITS, p.xh, (unsigned)p.iter[0] * 64u + p.layer + 1u, p.hx_err);
    ts_end(p.ts, t_start);
}

// ---------------------------------------------------------------- text attention, direct form
// a = softmax_t(q . K_t / sqrt(128)) V  of slot b into a_s[128] (every thread
// returns after a barrier); pr: per-key scores, then weights [TMAX_LIMIT]. getq() makes
// q readable (whatever hand-off that takes) and returns it (16 B aligned, global or LDS).
// The first 64 keys' K rows and V rows are issued at entry, before getq: one memory
// round trip for a text of up to 64 tokens; longer texts load 64 keys per round.
//  1. scores: key t = 64 c + 16 w + lane / 4 of wave w, 4 lanes per key (32 dims each,
//     one fmaf chain), the quad summed by two DPP steps (no cross-row exchange);
//  2. weights: thread t exponentiates key t (one expf per key), sums its keys, the
//     denominator is the wave sums in wave order;
//  3. a[d] = sum_t e_t V_t[d] / den: wave w takes keys w, w + 4, ... in ascending order
//     (lane owns dims lane, 64 + lane), the 4 waves' partials summed in order.
// Branch-free per key (clamped loads, selects), so the DPP and LDS traffic of a round
// issues back to back.
constexpr int XA_PF_V = 4;  // rounds of 16 value rows issued at entry
template <typename QF>
__device__ __forceinline__ void xa_text_attention_q(QF getq, const float *Kb, const float *Vb, int Tb, float *pr,
                                                    float *a_s) {
#pragma clang fp contract(off)
    __shared__ __attribute__((aligned(16))) float pv[MP_NWAVES][DXA];
    __shared__ float wred[2 * MP_NWAVES];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int kq = 16 * w + (lane >> 2), dq = 32 * (lane & 3);  // pass 1: key in the round, dims
    f32x4 kpf[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) kpf[i] = *(const f32x4 *)(Kb + (size_t)min(kq, Tb - 1) * DXA + dq + 4 * i);
    float v0pf[XA_PF_V][4], v1pf[XA_PF_V][4];
#pragma unroll
    for (int r = 0; r < XA_PF_V; ++r)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int t = min(w + 16 * r + MP_NWAVES * u, Tb - 1);
            v0pf[r][u] = Vb[(size_t)t * DXA + lane];
            v1pf[r][u] = Vb[(size_t)t * DXA + 64 + lane];
        }
    const float *qp = getq();
    f32x4 q4[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) q4[i] = *(const f32x4 *)(qp + dq + 4 * i);
    const float scale = 1.0f / sqrtf((float)DXA);
    float mx = -INFINITY;
    auto score = [&](int t, const f32x4 (&k4)[8]) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            s = fmaf(q4[i].x, k4[i].x, s);
            s = fmaf(q4[i].y, k4[i].y, s);
            s = fmaf(q4[i].z, k4[i].z, s);
            s = fmaf(q4[i].w, k4[i].w, s);
        }
        s += dpp_mov<0xB1>(s);  // (s0 + s1) + (s2 + s3) in every lane of the quad
        s += dpp_mov<0x4E>(s);
        const float sv = s * scale;
        if ((lane & 3) == 0 && t < Tb) pr[t] = sv;
        mx = fmaxf(mx, t < Tb ? sv : -INFINITY);
    };
    score(kq, kpf);
    for (int t0 = 64; t0 < Tb; t0 += 64) {
        f32x4 k4[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) k4[i] = *(const f32x4 *)(Kb + (size_t)min(t0 + kq, Tb - 1) * DXA + dq + 4 * i);
        score(t0 + kq, k4);
    }
    mx = wave_max(mx);
    if (lane == 0) wred[w] = mx;
    lds_sync();
    const float M = fmaxf(fmaxf(wred[0], wred[1]), fmaxf(wred[2], wred[3]));
    float l = 0.f;
    for (int t = tid; t < Tb; t += MP_BLOCK) {
        const float e = expf(pr[t] - M);
        pr[t] = e;
        l += e;
    }
    l = wave_sum(l);
    if (lane == 0) wred[MP_NWAVES + w] = l;
    lds_sync();
    // o[d] = sum_t e_t V_t[d]: wave w takes keys t = w + 4 u, lane owns dims lane, 64 + lane
    float o0 = 0.f, o1 = 0.f;
    auto accum = [&](int t0, const float (&v0)[4], const float (&v1)[4]) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int t = t0 + MP_NWAVES * u;
            const float e = t < Tb ? pr[min(t, Tb - 1)] : 0.f;
            o0 = fmaf(e, v0[u], o0);
            o1 = fmaf(e, v1[u], o1);
        }
    };
#pragma unroll
    for (int r = 0; r < XA_PF_V; ++r) accum(w + 16 * r, v0pf[r], v1pf[r]);
    for (int t0 = w + 16 * XA_PF_V; t0 < Tb; t0 += MP_NWAVES * 4) {
        float v0[4], v1[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int t = min(t0 + MP_NWAVES * u, Tb - 1);
            v0[u] = Vb[(size_t)t * DXA + lane];
            v1[u] = Vb[(size_t)t * DXA + 64 + lane];
        }
        accum(t0, v0, v1);
    }
    pv[w][lane] = o0;
    pv[w][64 + lane] = o1;
    lds_sync();
    if (tid < DXA) {
        const float den = ((wred[4] + wred[5]) + wred[6]) + wred[7];
        a_s[tid] = (((pv[0][tid] + pv[1][tid]) + pv[2][tid]) + pv[3][tid]) / den;
    }
    lds_sync();
}

__device__ __forceinline__ void xa_text_attention(const float *q, const float *Kb, const float *Vb, int Tb,
                                                  float *pr, float *a_s) {
    xa_text_attention_q([&]() { return q; }, Kb, Vb, Tb, pr, a_s);
}

}  // namespace mp
