// Device-side helpers shared by the gfx950 kernels (wave64 reductions, vector
// loads, block reductions). CDNA4 only: wave = 64 lanes, 256-thread workgroups.
#pragma once
#include <stdint.h>
#include <vector>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <hip/hip_ext.h>

#define MP_WAVE 64
#define MP_BLOCK 256
#define MP_NWAVES (MP_BLOCK / MP_WAVE)

namespace mp {
// Per-launch kernel timing (mp_hip_profile_ops_kev). While g_kev is set on the
// launching thread, decode launches go through hipExtLaunchKernel with these
// events, which then carry the dispatch's own begin/end timestamps: the interval
// rocprofv3's kernel trace reports, measured live without the profiler.
inline thread_local hipEvent_t g_kev[2] = {nullptr, nullptr};
template <typename... A, typename... P>
inline void launch(void (*k)(A...), dim3 grid, dim3 block, unsigned shm, hipStream_t s, P... args) {
    if (g_kev[0]) hipExtLaunchKernelGGL(k, grid, block, shm, s, g_kev[0], g_kev[1], 0, args...);
    else hipLaunchKernelGGL(k, grid, block, shm, s, args...);
}

// Host: the CU mask of a stream confined to `cus` of `ncu` CUs (every (ncu / cus)-th CU, so the
// share is spread over the XCDs), or its complement. The codec's background stream takes the
// share, the frame loop's stream during an overlapped streaming round the complement
// (hipExtStreamCreateWithCUMask): the two never wait for each other's workgroups.
inline std::vector<uint32_t> cu_share_mask(int ncu, int cus, bool complement) {
    std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
    std::vector<char> in(ncu, 0);
    const int step = cus > 0 ? (ncu / cus > 1 ? ncu / cus : 1) : ncu + 1;
    for (int i = 0, n = 0; i < ncu && n < cus; i += step, ++n) in[i] = 1;
    for (int i = 0; i < ncu; ++i)
        if ((in[i] != 0) != complement) mask[i / 32] |= 1u << (i % 32);
    return mask;
}

}  // namespace mp

// ---- wave64 reductions on DPP (data-parallel primitives move lanes inside the
// VALU; no LDS round trip per step, unlike __shfl_xor's ds_bpermute).
// ctrl: quad_perm(1,0,3,2)=0xB1, quad_perm(2,3,0,1)=0x4E, row_half_mirror=0x141,
// row_mirror=0x140, row_bcast15=0x142, row_bcast31=0x143.
template <int CTRL, int ROWMASK = 0xF>
__device__ __forceinline__ float dpp_mov(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROWMASK, 0xF, false));
}
__device__ __forceinline__ float bcast_lane63(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}
// every lane gets the sum of its 16-lane row
__device__ __forceinline__ float row_sum16(float v) {
    v += dpp_mov<0xB1>(v);
    v += dpp_mov<0x4E>(v);
    v += dpp_mov<0x141>(v);
    v += dpp_mov<0x140>(v);
    return v;
}
__device__ __forceinline__ float row_max16(float v) {
    v = fmaxf(v, dpp_mov<0xB1>(v));
    v = fmaxf(v, dpp_mov<0x4E>(v));
    v = fmaxf(v, dpp_mov<0x141>(v));
    v = fmaxf(v, dpp_mov<0x140>(v));
    return v;
}
// full-wave sum / max, returned uniformly (SGPR broadcast of lane 63)
__device__ __forceinline__ float wave_sum(float v) {
    v = row_sum16(v);
    v += dpp_mov<0x142, 0xA>(v);
    v += dpp_mov<0x143, 0xC>(v);
    return bcast_lane63(v);
}
__device__ __forceinline__ float wave_max(float v) {
    v = row_max16(v);
    v = fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, v),
                                                                    __builtin_bit_cast(int, v), 0x142, 0xA, 0xF, false)));
    v = fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, v),
                                                                    __builtin_bit_cast(int, v), 0x143, 0xC, 0xF, false)));
    return bcast_lane63(v);
}
// wave_sum of N values at once (value j: v[j]), the N DPP chains advanced in lockstep so
// their dependent steps overlap; each total is wave_sum's exactly (same tree, same order).
// Returns the totals uniformly in v.
template <int N>
__device__ __forceinline__ void wave_sum_n(float (&v)[N]) {
#define MP_WSN_STEP(...) _Pragma("unroll") for (int j = 0; j < N; ++j) v[j] += __VA_ARGS__(v[j]);
    MP_WSN_STEP(dpp_mov<0xB1>)
    MP_WSN_STEP(dpp_mov<0x4E>)
    MP_WSN_STEP(dpp_mov<0x141>)
    MP_WSN_STEP(dpp_mov<0x140>)
    MP_WSN_STEP((dpp_mov<0x142, 0xA>))
    MP_WSN_STEP((dpp_mov<0x143, 0xC>))
#undef MP_WSN_STEP
#pragma unroll
    for (int j = 0; j < N; ++j) v[j] = bcast_lane63(v[j]);
}
// full-wave minimum of a non-negative int, returned uniformly (DPP, no LDS)
__device__ __forceinline__ int wave_min_u(int v) {
    auto step = [&](int x) { return x < v ? x : v; };
    v = step(__builtin_amdgcn_update_dpp(v, v, 0xB1, 0xF, 0xF, false));
    v = step(__builtin_amdgcn_update_dpp(v, v, 0x4E, 0xF, 0xF, false));
    v = step(__builtin_amdgcn_update_dpp(v, v, 0x141, 0xF, 0xF, false));
    v = step(__builtin_amdgcn_update_dpp(v, v, 0x140, 0xF, 0xF, false));
    v = step(__builtin_amdgcn_update_dpp(v, v, 0x142, 0xA, 0xF, false));
    v = step(__builtin_amdgcn_update_dpp(v, v, 0x143, 0xC, 0xF, false));
    return __builtin_amdgcn_readlane(v, 63);
}
// sum over lanes that differ only in the low log2(W) bits (W = 16 or 32)
template <int W>
__device__ __forceinline__ float group_sum(float v) {
    static_assert(W == 16 || W == 32, "group_sum: 16 or 32 lanes");
    v = row_sum16(v);
    if constexpr (W == 32) v += __shfl_xor(v, 16, 64);
    return v;
}

// Workgroup barrier for LDS hand-offs only: LDS-scoped release/acquire fences
// around s_barrier lower to `s_waitcnt lgkmcnt(0); s_barrier` and do NOT wait
// for outstanding global loads, so a weight stream issued before a prologue
// stays in flight across it (__syncthreads() would drain it with vmcnt(0)).
// Compiler-visible (no inline asm): the waitcnt and scheduling passes see it.
__device__ __forceinline__ void lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
// LDS ordering among the lanes of one wave (wave-private LDS scratch)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Optional in-kernel timing for the bench's per-op table (ts != nullptr only in
// mp_hip_profile_ops_ts): every wave records (its workgroup's start, its own end
// after its stores completed) as one plain 16-byte store into its slot
// ts[2 * (block * TS_WAVES + wave)]; the host takes min(start) .. max(end). No
// atomics (no contention, and no store before the kernel's loads, so the compiler
// keeps its scalar loads), s_memrealtime at 100 MHz.
constexpr int TS_WAVES = 8, TS_BLOCKS = 1024;
// The start stamp is a non-volatile asm (no modelled side effect: a volatile one or
// the builtin would stop the compiler from turning the kernel's later uniform loads
// into scalar loads); ts_dep(t) (always 0, opaque to the compiler) is added to the
// kernel's first load address so the stamp stays at the start.
__device__ __forceinline__ unsigned long long ts_begin(const unsigned long long *ts) {
    unsigned long long t = 0;
    if (ts) asm("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : "s"(ts));
    return t;
}
__device__ __forceinline__ int ts_dep(unsigned long long t) { return (int)(t >> 63); }
// an intermediate stamp (t0, now) of wave w into wave slot TS_WAVES/2 + w (4-wave kernels)
__device__ __forceinline__ void ts_mark(unsigned long long *ts, unsigned long long t0) {
    if (ts) {
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        const int blk = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
        if ((threadIdx.x & 63) == 0 && blk < TS_BLOCKS && (threadIdx.x >> 6) < TS_WAVES / 2)
            *(ulonglong2 *)(ts + 2 * ((size_t)blk * TS_WAVES + TS_WAVES / 2 + (threadIdx.x >> 6))) =
                make_ulonglong2(t0, t1);
    }
}
// stamp K (0 .. TS_WAVES/2 - 1) of a workgroup's phases, from wave 0, into slot TS_WAVES/2 + K
// (diagnostics of kernels whose phases are workgroup-wide: use instead of ts_mark)
template <int K>
__device__ __forceinline__ void ts_phase(unsigned long long *ts, unsigned long long t0) {
    static_assert(K >= 0 && K < TS_WAVES / 2, "phase slot");
    if (ts) {
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        const int blk = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
        if (threadIdx.x == 0 && blk < TS_BLOCKS)
            *(ulonglong2 *)(ts + 2 * ((size_t)blk * TS_WAVES + TS_WAVES / 2 + K)) = make_ulonglong2(t0 ? t0 : t1, t1);
    }
}
// the same, stamped by the calling wave's lane 0 (a phase that one wave of the workgroup
// reaches, whichever it is)
template <int K>
__device__ __forceinline__ void ts_phase_w(unsigned long long *ts) {
    static_assert(K >= 0 && K < TS_WAVES / 2, "phase slot");
    if (ts) {
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        const int blk = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
        if ((threadIdx.x & 63) == 0 && blk < TS_BLOCKS)
            *(ulonglong2 *)(ts + 2 * ((size_t)blk * TS_WAVES + TS_WAVES / 2 + K)) = make_ulonglong2(t1, t1);
    }
}
__device__ __forceinline__ void ts_end(unsigned long long *ts, unsigned long long t0) {
    if (ts) {
        __builtin_amdgcn_s_waitcnt(0);
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        const int blk = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
        if ((threadIdx.x & 63) == 0 && blk < TS_BLOCKS)
            *(ulonglong2 *)(ts + 2 * ((size_t)blk * TS_WAVES + (threadIdx.x >> 6))) = make_ulonglong2(t0, t1);
    }
}

// Block-wide reduction for 256 threads; `red` is an LDS scratch of >= 4 floats.
// Every thread returns the total. Contains two barriers.
__device__ __forceinline__ float block_sum(float v, float *red) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) red[w] = v;
    lds_sync();
    const float r = (red[0] + red[1]) + (red[2] + red[3]);
    lds_sync();
    return r;
}
__device__ __forceinline__ float block_max(float v, float *red) {
    v = wave_max(v);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) red[w] = v;
    lds_sync();
    const float r = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    lds_sync();
    return r;
}

// LayerNorm statistics of K elements held PER per thread (256 threads):
// one pass, numerically stable pairwise combination of (mean, M2) — groups
// combined at every step have equal element counts. Returns biased variance.
template <int PER>
__device__ __forceinline__ void block_meanvar(const float (&v)[PER], float *red, float &mean, float &var) {
    float m = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) m += v[i];
    m *= 1.0f / PER;
    float M2 = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) { const float d = v[i] - m; M2 += d * d; }
    float n = (float)PER;  // elements per side at the current step
    auto comb = [&](float mb, float M2b) {
        const float d = mb - m;
        m = m + 0.5f * d;
        M2 = M2 + M2b + d * d * (0.5f * n);
        n *= 2.f;
    };
    comb(dpp_mov<0xB1>(m), dpp_mov<0xB1>(M2));
    comb(dpp_mov<0x4E>(m), dpp_mov<0x4E>(M2));
    comb(dpp_mov<0x141>(m), dpp_mov<0x141>(M2));
    comb(dpp_mov<0x140>(m), dpp_mov<0x140>(M2));
    comb(dpp_mov<0x142, 0xA>(m), dpp_mov<0x142, 0xA>(M2));  // valid in rows 1,3
    comb(dpp_mov<0x143, 0xC>(m), dpp_mov<0x143, 0xC>(M2));  // valid in row 3 (lane 63 = whole wave)
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 63) { red[2 * w] = m; red[2 * w + 1] = M2; }
    lds_sync();
    float m0 = red[0], q0 = red[1], m1 = red[2], q1 = red[3], m2 = red[4], q2 = red[5], m3 = red[6], q3 = red[7];
    lds_sync();
    const float nw = 64.f * PER;
    float d = m1 - m0;
    const float ma = m0 + 0.5f * d, Qa = q0 + q1 + d * d * (0.5f * nw);
    d = m3 - m2;
    const float mb = m2 + 0.5f * d, Qb = q2 + q3 + d * d * (0.5f * nw);
    d = mb - ma;
    mean = ma + 0.5f * d;
    const float Q = Qa + Qb + d * d * nw;
    var = Q * (1.0f / (4.f * nw));
}

// block_meanvar<PER> of a 256-thread block, computed by ONE wave bit for bit:
// x[j] holds element lane + 64 j (j < 4 PER), i.e. virtual thread 64 (j%4) + lane's
// value i = j/4. The four virtual waves run the same DPP trees, then the same
// final combination, so a batched prologue (one wave per slot) reproduces the
// batch-1 statistics exactly. Uniform result, no barrier.
template <int PER>
__device__ __forceinline__ void wave_block_meanvar(const float (&x)[4 * PER], float &mean, float &var) {
    float mw[4], qw[4];
#pragma unroll
    for (int v = 0; v < 4; ++v) {
        float m = 0.f;
#pragma unroll
        for (int i = 0; i < PER; ++i) m += x[v + 4 * i];
        m *= 1.0f / PER;
        float M2 = 0.f;
#pragma unroll
        for (int i = 0; i < PER; ++i) { const float d = x[v + 4 * i] - m; M2 += d * d; }
        float n = (float)PER;
        auto comb = [&](float mb, float M2b) {
            const float d = mb - m;
            m = m + 0.5f * d;
            M2 = M2 + M2b + d * d * (0.5f * n);
            n *= 2.f;
        };
        comb(dpp_mov<0xB1>(m), dpp_mov<0xB1>(M2));
        comb(dpp_mov<0x4E>(m), dpp_mov<0x4E>(M2));
        comb(dpp_mov<0x141>(m), dpp_mov<0x141>(M2));
        comb(dpp_mov<0x140>(m), dpp_mov<0x140>(M2));
        comb(dpp_mov<0x142, 0xA>(m), dpp_mov<0x142, 0xA>(M2));
        comb(dpp_mov<0x143, 0xC>(m), dpp_mov<0x143, 0xC>(M2));
        mw[v] = bcast_lane63(m);
        qw[v] = bcast_lane63(M2);
    }
    const float nw = 64.f * PER;
    float d = mw[1] - mw[0];
    const float ma = mw[0] + 0.5f * d, Qa = qw[0] + qw[1] + d * d * (0.5f * nw);
    d = mw[3] - mw[2];
    const float mb = mw[2] + 0.5f * d, Qb = qw[2] + qw[3] + d * d * (0.5f * nw);
    d = mb - ma;
    mean = ma + 0.5f * d;
    const float Q = Qa + Qb + d * d * nw;
    var = Q * (1.0f / (4.f * nw));
}

// Wave-level LayerNorm statistics of 64*PER elements (PER per lane), same
// pairwise (mean, M2) combination as block_meanvar; uniform result, no barrier.
template <int PER>
__device__ __forceinline__ void wave_meanvar(const float (&v)[PER], float &mean, float &var) {
    float m = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) m += v[i];
    m *= 1.0f / PER;
    float M2 = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) { const float d = v[i] - m; M2 += d * d; }
    float n = (float)PER;
    auto comb = [&](float mb, float M2b) {
        const float d = mb - m;
        m = m + 0.5f * d;
        M2 = M2 + M2b + d * d * (0.5f * n);
        n *= 2.f;
    };
    comb(dpp_mov<0xB1>(m), dpp_mov<0xB1>(M2));
    comb(dpp_mov<0x4E>(m), dpp_mov<0x4E>(M2));
    comb(dpp_mov<0x141>(m), dpp_mov<0x141>(M2));
    comb(dpp_mov<0x140>(m), dpp_mov<0x140>(M2));
    comb(dpp_mov<0x142, 0xA>(m), dpp_mov<0x142, 0xA>(M2));
    comb(dpp_mov<0x143, 0xC>(m), dpp_mov<0x143, 0xC>(M2));
    mean = bcast_lane63(m);
    var = bcast_lane63(M2) * (1.0f / (64.f * PER));
}

// wave_meanvar of S rows at once (row j: v[j]), the S chains advanced in lockstep so
// their dependent DPP steps overlap; each row's arithmetic is wave_meanvar's exactly.
template <int PER, int S>
__device__ __forceinline__ void wave_meanvar_n(const float (&v)[S][PER], float (&mean)[S], float (&var)[S]) {
    float m[S], M2[S];
#pragma unroll
    for (int j = 0; j < S; ++j) {
        m[j] = 0.f;
#pragma unroll
        for (int i = 0; i < PER; ++i) m[j] += v[j][i];
        m[j] *= 1.0f / PER;
    }
#pragma unroll
    for (int j = 0; j < S; ++j) {
        M2[j] = 0.f;
#pragma unroll
        for (int i = 0; i < PER; ++i) { const float d = v[j][i] - m[j]; M2[j] += d * d; }
    }
    float n = (float)PER;
    auto comb = [&](const float (&mb)[S], const float (&M2b)[S]) {
#pragma unroll
        for (int j = 0; j < S; ++j) {
            const float d = mb[j] - m[j];
            m[j] = m[j] + 0.5f * d;
            M2[j] = M2[j] + M2b[j] + d * d * (0.5f * n);
        }
        n *= 2.f;
    };
    float mb[S], qb[S];
#define MP_COMB_STEP(...)                                                            \
    _Pragma("unroll") for (int j = 0; j < S; ++j) { mb[j] = __VA_ARGS__(m[j]); qb[j] = __VA_ARGS__(M2[j]); } \
    comb(mb, qb);
    MP_COMB_STEP(dpp_mov<0xB1>)
    MP_COMB_STEP(dpp_mov<0x4E>)
    MP_COMB_STEP(dpp_mov<0x141>)
    MP_COMB_STEP(dpp_mov<0x140>)
    MP_COMB_STEP(dpp_mov<0x142, 0xA>)
    MP_COMB_STEP(dpp_mov<0x143, 0xC>)
#undef MP_COMB_STEP
#pragma unroll
    for (int j = 0; j < S; ++j) {
        mean[j] = bcast_lane63(m[j]);
        var[j] = bcast_lane63(M2[j]) * (1.0f / (64.f * PER));
    }
}

// (value, index) argmax with the reference's tie rule: the FIRST maximal index
// wins (strict '>' scan from index 0, magpie.cpp:1250-1258).
__device__ __forceinline__ void argmax_merge(float &v, int &i, float v2, int i2) {
    if (v2 > v || (v2 == v && i2 < i)) { v = v2; i = i2; }
}
__device__ __forceinline__ void wave_argmax(float &v, int &i) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float v2 = __shfl_xor(v, o, 64);
        const int i2 = __shfl_xor(i, o, 64);
        argmax_merge(v, i, v2, i2);
    }
}

__device__ __forceinline__ float gelu_tanh(float x) {
    // ggml_gelu: 0.5 x (1 + tanh(sqrt(2/pi) x (1 + 0.044715 x^2)))
    return 0.5f * x * (1.0f + tanhf(0.79788456080286535588f * x * (1.0f + 0.044715f * x * x)));
}
// One wave's FFN-up units: v[r] holds this lane's part of unit r's dot product; the N
// totals (wave_sum_n: wave_sum's tree for each) go through GELU on lanes 0..N-1 in
// parallel, lane r storing post(gelu(unit r)) to dst[r] (before: N wave sums and N GELUs
// in sequence on lane 0 behind exec masks). Same value per unit.
template <int N, typename F>
__device__ __forceinline__ void ffn_units_store(float (&v)[N], float *dst, F post) {
    static_assert(N <= 64, "one lane per unit");
    wave_sum_n<N>(v);
    const int lane = threadIdx.x & 63;
    float mine = v[0];
#pragma unroll
    for (int r = 1; r < N; ++r)
        if (lane == r) mine = v[r];
    if (lane < N) dst[lane] = post(gelu_tanh(mine));
}

template <int VW> struct vecf;
template <> struct vecf<4> { using T = float4; };
template <> struct vecf<2> { using T = float2; };
template <> struct vecf<1> { using T = float; };

// SA cache element store / load (MP_KV_BF16: bf16, round to nearest even on the
// f32 bits; K/V values are finite). The cache pointer is typed float in both modes.
__device__ __forceinline__ unsigned short f32_to_bf16_rne(float v) {
    const unsigned u = __float_as_uint(v);
    return (unsigned short)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ void kv_store(float *c, size_t i, float v, int kv16) {
    if (kv16) ((unsigned short *)c)[i] = f32_to_bf16_rne(v);
    else c[i] = v;
}
__device__ __forceinline__ float4 bf16x4_to_f32(uint2 u) {
    return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xFFFF0000u), __uint_as_float(u.y << 16),
                       __uint_as_float(u.y & 0xFFFF0000u));
}
// 4 consecutive cache elements starting at element i (i a multiple of 4)
template <bool KV16>
__device__ __forceinline__ float4 kv_load4(const float *c, size_t i) {
    if constexpr (KV16) return bf16x4_to_f32(*(const uint2 *)((const unsigned short *)c + i));
    else return *(const float4 *)(c + i);
}

// Weight-stream loads (read once per launch by one CU), issued non-temporal
// (global_load ... nt: the guide's nt-weights row). Measured on this path, two
// alternating rounds on one box (gpurun_out/r04j_ab.txt): f32 B=1 2,677 / 2,596 ->
// 2,724 / 2,725 frames/s, bf16 B=8 +2.7 %, B=16 +2 %, bf16 B=1 and Q8_0 B=1 within noise.
// MP_NO_NT_WEIGHTS builds use the default policy.
template <typename T>
__device__ __forceinline__ T ld_weight(const T *p) {
#ifndef MP_NO_NT_WEIGHTS
    if constexpr (sizeof(T) == 16) {
        typedef unsigned u4 __attribute__((ext_vector_type(4)));
        return __builtin_bit_cast(T, __builtin_nontemporal_load((const u4 *)p));
    } else if constexpr (sizeof(T) == 8) {
        typedef unsigned u2 __attribute__((ext_vector_type(2)));
        return __builtin_bit_cast(T, __builtin_nontemporal_load((const u2 *)p));
    } else {
        static_assert(sizeof(T) == 4, "4, 8 or 16 B");
        return __builtin_bit_cast(T, __builtin_nontemporal_load((const unsigned *)p));
    }
#else
    return *p;
#endif
}

// The library is built with -ffp-contract=off (Makefile): every fused multiply-add is
// written out, so an instantiation change cannot move a rounding (batch == single).
// The local transformer's weights (LT FFN, heads, in_proj, [W_k ; W_o W_v]) are re-read
// every frame (the FFN 8 times per frame) and are 5 % of the frame's bytes: MP_LT_NT=0
// loads them with the default cache policy (left in the Infinity Cache between uses)
// instead of non-temporal.
#ifndef MP_LT_NT
#define MP_LT_NT 1
#endif
template <typename T>
__device__ __forceinline__ T ld_lt(const T *p) {
#if MP_LT_NT
    return ld_weight(p);
#else
    return *p;
#endif
}
// The LT FFN's W1 / W2 slices: read by the same workgroup index 8 times per frame (every
// codebook's step), so the default cache policy keeps them on die between steps
// (measured: lt_ffn2 6.24 -> 5.69 us at f32 batch 1, gpurun_out/r05b_ops_f32_b1_ltdef.txt);
// MP_LTFFN_NT=1 restores the non-temporal loads.
#ifndef MP_LTFFN_NT
#define MP_LTFFN_NT 0
#endif
template <typename T>
__device__ __forceinline__ T ld_ltffn(const T *p) {
#if MP_LTFFN_NT
    return ld_weight(p);
#else
    return *p;
#endif
}

__device__ __forceinline__ float dotv(float4 a, float4 b) { return fmaf(a.w, b.w, fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x))); }
__device__ __forceinline__ float dotv(float2 a, float2 b) { return fmaf(a.y, b.y, a.x * b.x); }
__device__ __forceinline__ float dotv(float a, float b) { return a * b; }
