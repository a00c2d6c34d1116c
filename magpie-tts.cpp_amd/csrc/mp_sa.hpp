// The decode self-attention body (one query per utterance, split over the live
// cache) shared by sa_attn_kernel and the QKV launches that carry it
// (EPI_QKV_SA: the f32 GEMV and 16-bit MFMA families), and the QKV side of that
// hand-off. Both run 4 waves per workgroup with the same key order and merge, and
// the handed-off new key equals its cache row, so every path computes the same bits.
#pragma once
#include "mp_device.hpp"
#include "mp_params.hpp"
#include "mp_xa.hpp"

namespace mp {

constexpr int SA_IF = 4;  // key rounds in flight per wave

// Split sp of head h, slot b: keys [sp*chunk, (sp+1)*chunk) of L = pos + 1
// (magpie.cpp:3412); wave w takes keys 4(w + NW r) + kk of it (16 lanes x float4
// cover one 64-dim row, a wave does 4 keys per instruction) with SA_IF rounds'
// K and V loads in flight, keeps an online softmax (m, l, o[64]); the NW wave
// states are merged in LDS and the split's state (m, l, unnormalised O) is
// stored; the O-projection's PRO_SA_MERGE prologue merges the splits
// (softmax(K q / 8) V per head, 3457-3476).
// HANDOFF: q and the new key's k, v come from the QKV workgroups of the same
// launch as {tag, value} granules qh[b][2304] (EPI_QKV_SA), swept by every wave
// after its first cache rows are in flight; the cache rows read are those of keys
// < pos (the row at pos is being written by this launch), key pos uses the
// granules.
// The arithmetic is spelled out (contraction off, explicit fmaf): the handed-off
// and standalone instantiations must round identically, whatever code surrounds them.
__device__ __forceinline__ float sa_dot(float4 q, float4 k) {
    return fmaf(q.w, k.w, fmaf(q.z, k.z, fmaf(q.y, k.y, q.x * k.x)));
}
template <bool KV16, int NW, bool HANDOFF>
__device__ __forceinline__ void sa_part(const AttnP &p, int h, int sp, int b, const unsigned long long *qh,
                                        unsigned tag, int *err, int dep, unsigned long long *ts = nullptr,
                                        unsigned long long t_start = 0) {
#pragma clang fp contract(off)
    __shared__ float wm[NW], wl[NW];
    __shared__ __attribute__((aligned(16))) float wo[NW][DH];
    __shared__ __attribute__((aligned(16))) float wq[1][3 * DH];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int kk = lane >> 4, dc = lane & 15;
    const size_t base = ((size_t)(b * p.nlayers + p.layer) * p.max_seq) * D + h * DH + 4 * dc + dep;
    const int L = p.pos[b] + 1, jn = L - 1;  // jn: this step's key
    const int chunk = (L + SA_SPLITS - 1) / SA_SPLITS;
    const int j0 = sp * chunk, j1 = min(L, j0 + chunk);
    // keys past the split re-read its last cached row (an L1/L2 hit, no extra HBM
    // traffic); rows < max_seq are valid memory: no load waits for the mask
    const int jcap = HANDOFF ? max(min(j1, jn) - 1, 0) : max(j1 - 1, 0);
    float4 k4[SA_IF], v4[SA_IF];
#pragma unroll
    for (int u = 0; u < SA_IF; ++u) {
        const int j = min(j0 + 4 * (w + NW * u) + kk, jcap);
        k4[u] = kv_load4<KV16>(p.kc, base + (size_t)j * D);
        v4[u] = kv_load4<KV16>(p.vc, base + (size_t)j * D);
    }
    float4 q4, kn4 = make_float4(0.f, 0.f, 0.f, 0.f), vn4 = kn4;
    if constexpr (HANDOFF) {
        // one poller per array: wave 0 sweeps q, waves 1 and 2 the new key's k and v (when
        // this split holds it), then the workgroup barrier publishes them (every wave
        // polling all three made the merge barrier wait for the unluckiest wave's next
        // round trip after the granules were complete)
        const bool has_new = j0 <= jn && jn < j1;  // workgroup-uniform
        if (w < (has_new ? 3 : 1)) {
            gu64 *g = (gu64 *)const_cast<unsigned long long *>(qh) + (size_t)b * 3 * D + w * D + h * DH + lane;
            float val;
            for (unsigned spins = 0;; ++spins) {
                const unsigned long long u = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                val = __uint_as_float((unsigned)u);
                if (__all((unsigned)(u >> 32) == tag)) break;
                if (spins >= HX_SPIN_LIMIT) {  // never seen: poison the output and say so
                    if (lane == 0) __hip_atomic_fetch_or((gi32 *)err, HX_ERR_SA, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    val = __builtin_nanf("");
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if constexpr (KV16)  // the new row as the cache holds it (kv_store's rounding)
                if (w > 0) val = __uint_as_float((unsigned)f32_to_bf16_rne(val) << 16);
            wq[0][w * DH + lane] = val;
        }
        lds_sync();
        ts_phase<0>(ts, t_start);  // profiling: q (and the new key) seen
        q4 = *(const float4 *)&wq[0][4 * dc];
        if (has_new) {
            kn4 = *(const float4 *)&wq[0][DH + 4 * dc];
            vn4 = *(const float4 *)&wq[0][2 * DH + 4 * dc];
        }
    } else {
        q4 = *(const float4 *)(p.q + (size_t)b * D + h * DH + 4 * dc);
    }
    float m = -INFINITY, l = 0.f;
    float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int r0 = 0; j0 + 4 * NW * r0 < j1; r0 += SA_IF) {
        if (r0) {
#pragma unroll
            for (int u = 0; u < SA_IF; ++u) {
                const int j = min(j0 + 4 * (w + NW * (r0 + u)) + kk, jcap);
                k4[u] = kv_load4<KV16>(p.kc, base + (size_t)j * D);
                v4[u] = kv_load4<KV16>(p.vc, base + (size_t)j * D);
            }
        }
        float sv[SA_IF];
        float mb = -INFINITY;
#pragma unroll
        for (int u = 0; u < SA_IF; ++u) {
            const int j = j0 + 4 * (w + NW * (r0 + u)) + kk;
            if (HANDOFF && j == jn) { k4[u] = kn4; v4[u] = vn4; }
            const float v = group_sum<16>(sa_dot(q4, k4[u])) * 0.125f;  // 1/sqrt(64)
            sv[u] = j < j1 ? v : -INFINITY;
            mb = fmaxf(mb, sv[u]);
        }
        mb = wave_max(mb);
        if (mb == -INFINITY) continue;  // nothing live for this wave in this round
        const float mn = fmaxf(m, mb), c = expf(m - mn);
        l *= c;
        o.x *= c; o.y *= c; o.z *= c; o.w *= c;
#pragma unroll
        for (int u = 0; u < SA_IF; ++u) {
            const float e = sv[u] == -INFINITY ? 0.f : expf(sv[u] - mn);
            l += e;  // per lane: its key group's keys; summed over the wave below
            o.x = fmaf(e, v4[u].x, o.x); o.y = fmaf(e, v4[u].y, o.y);
            o.z = fmaf(e, v4[u].z, o.z); o.w = fmaf(e, v4[u].w, o.w);
        }
        m = mn;
    }
    ts_phase<1>(ts, t_start);  // profiling: this (first) wave's keys done
    // merge the 4 key groups of the wave (lanes l, l^16, l^32, l^48 share dims)
#pragma unroll
    for (int msk = 16; msk <= 32; msk <<= 1) {
        o.x += __shfl_xor(o.x, msk, 64); o.y += __shfl_xor(o.y, msk, 64);
        o.z += __shfl_xor(o.z, msk, 64); o.w += __shfl_xor(o.w, msk, 64);
        l += __shfl_xor(l, msk, 64);
    }
    if (lane < 16) *(float4 *)(&wo[w][4 * lane]) = o;
    if (lane == 0) { wm[w] = m; wl[w] = l; }
    lds_sync();
    ts_phase<2>(ts, t_start);  // profiling: every wave's keys done
    if (tid >= DH) return;
    float M = -INFINITY;
#pragma unroll
    for (int q = 0; q < NW; ++q) M = fmaxf(M, wm[q]);
    float num = 0.f, den = 0.f;
#pragma unroll
    for (int q = 0; q < NW; ++q) {
        const float e = wm[q] == -INFINITY ? 0.f : expf(wm[q] - M);
        den = fmaf(e, wl[q], den);
        num = fmaf(e, wo[q][tid], num);
    }
    float *pp = p.part + ((size_t)(b * NH + h) * SA_SPLITS + sp) * SA_PART;
    if (p.merged) {  // granules: the head's split workgroups merge them (sa_merge_split)
        const unsigned long long tag = (unsigned long long)((unsigned)p.iter[0] * 64u + p.layer + 1u) << 32;
        gu64 *g = (gu64 *)p.gh + ((size_t)(b * NH + h) * SA_SPLITS + sp) * SA_PART;
        __hip_atomic_store(g + 4 + tid, tag | __float_as_uint(num), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (tid == 0) {
            __hip_atomic_store(g, tag | __float_as_uint(M), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(g + 1, tag | __float_as_uint(den), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
    pp[4 + tid] = num;  // relative to M (an empty split stores M = -inf, l = 0, O = 0)
    if (tid == 0) { pp[0] = M; pp[1] = den; }
}

// AttnP::merged (16 slots), after sa_part: split sp of head h merges dims
// [16 sp, 16 sp + 16) of the head from the SA_SPLITS states' granules (one lane per dim,
// a bounded sweep), with PRO_SA_MERGE's arithmetic (split_weights, split_merge)
__device__ __forceinline__ void sa_merge_split(const AttnP &p, int h, int sp, int b) {
    constexpr int MD = DH / SA_SPLITS;
    const int tid = threadIdx.x;
    if (tid >= MD) return;  // one partial wave: no barrier follows
    const unsigned tag = (unsigned)p.iter[0] * 64u + p.layer + 1u;
    const gu64 *g = (const gu64 *)p.gh + (size_t)(b * NH + h) * SA_SPLITS * SA_PART;
    const int d = MD * sp + tid;
    float ms[SA_SPLITS], ls[SA_SPLITS], o[SA_SPLITS], e[SA_SPLITS], rd;
    for (unsigned spins = 0;; ++spins) {
        bool ok = true;
#pragma unroll
        for (int s = 0; s < SA_SPLITS; ++s) {
            const unsigned long long um = __hip_atomic_load(g + s * SA_PART, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long ul = __hip_atomic_load(g + s * SA_PART + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long uo = __hip_atomic_load(g + s * SA_PART + 4 + d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ok &= (unsigned)(um >> 32) == tag && (unsigned)(ul >> 32) == tag && (unsigned)(uo >> 32) == tag;
            ms[s] = __uint_as_float((unsigned)um);
            ls[s] = __uint_as_float((unsigned)ul);
            o[s] = __uint_as_float((unsigned)uo);
        }
        if (__all(ok)) break;
        if (spins >= HX_SPIN_LIMIT) {  // never seen: poison the output and say so
            if (tid == 0) __hip_atomic_fetch_or((gi32 *)p.hx_err, HX_ERR_SA, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
            for (int s = 0; s < SA_SPLITS; ++s) o[s] = __builtin_nanf("");
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    split_weights<SA_SPLITS>(ms, ls, e, rd);
    p.merged[(size_t)b * D + h * DH + d] = split_merge<SA_SPLITS>(e, o, rd);
}

// EPI_QKV_SA epilogue, output (row n, slot b): EPI_QKV's stores, and the value
// published as a {tag, value} granule with a relaxed agent-scope (write-through) store
__device__ __forceinline__ void publish_qkv(const GemvP &p, float v, int n, int b) {
    epi_store<EPI_QKV>(p, v, n, b);
    const unsigned tag = (unsigned)p.iter[0] * 64u + p.layer + 1u;
    __hip_atomic_store((gu64 *)(p.qh + (size_t)b * 3 * D + n), ((unsigned long long)tag << 32) | __float_as_uint(v),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// host-side: the hand-off arguments of an EPI_QKV_SA launch agree with its QKV ones
inline bool qkv_sa_args_ok(const GemvP &p) {
    return p.qh && p.iter && p.hx_err && p.N == 3 * D && p.sa.kc == p.kc && p.sa.vc == p.vc && p.sa.pos == p.pos &&
           p.sa.part && p.sa.layer == p.layer && p.sa.nlayers == p.nlayers && p.sa.kv16 == p.kv16 &&
           p.sa.max_seq == p.max_seq && p.sa.max_seq >= 1 && p.sa.max_seq <= NCH_MAX * SA_CHUNK;
}

// the launch's SA workgroups (blockIdx.x >= nrow_blocks): (head, split, slot) of
// k = blockIdx.x - nrow_blocks, head fastest
__device__ __forceinline__ void sa_tail(const GemvP &p, unsigned long long t_start) {
    const int k = blockIdx.x - p.nrow_blocks;
    const int h = k % NH, sp = (k / NH) % SA_SPLITS, b = k / (NH * SA_SPLITS);
    const unsigned tag = (unsigned)p.iter[0] * 64u + p.layer + 1u;
    if (p.sa.kv16) sa_part<true, MP_NWAVES, true>(p.sa, h, sp, b, p.qh, tag, p.hx_err, ts_dep(t_start), p.ts, t_start);
    else sa_part<false, MP_NWAVES, true>(p.sa, h, sp, b, p.qh, tag, p.hx_err, ts_dep(t_start), p.ts, t_start);
    ts_phase<3>(p.ts, t_start);  // profiling: split state stored
    if (p.sa.merged) sa_merge_split(p.sa, h, sp, b);
    ts_end(p.ts, t_start);
}

}  // namespace mp
