// bf16 weight mode of the decode projections on MFMA (gfx950).
//
// Every fused projection of the decode step (qkv, O, FFN up/down of the 12
// decoder layers; the LT layer and its 8 output heads) as a skinny GEMM
//   out[b][n] = sum_k W[n][k] * bf16(act[b][k]),  b < NB <= 16
// on v_mfma_f32_16x16x32_bf16: the A operand is a 16-row x 32-k weight
// fragment, the B operand 32 k x 16 utterance columns (columns >= NB are zero),
// f32 accumulation. Activations are rounded to bf16 exactly as ggml rounds src1
// for a BF16 mul_mat (vec_dot_type BF16); the products are exact in f32.
//
// Layout in HBM: weights are repacked once at load into fragment order,
// [N/16][K/32][64 lanes][8 bf16], so each wave-instruction of the weight stream
// is one contiguous 1 KiB global_load_dwordx4 (lane l holds row l&15, k
// 8(l>>4)..+8 of the fragment). One workgroup owns one 16-row tile; its four
// waves split K in four and reduce their 16x16 accumulators through LDS in a
// fixed order, so every output's arithmetic is independent of NB (a batch
// reproduces its utterances run alone bit for bit).
#include <hip/hip_runtime.h>
#include <math.h>

#include "mp_device.hpp"
#include "mp_fused.hpp"
#include "mp_params.hpp"
#include "mp_sa.hpp"
#include "mp_xa.hpp"

namespace mp {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

// f32 -> bf16 bits, round to nearest even (ggml_compute_fp32_to_bf16)
__device__ __forceinline__ unsigned short f2bf(float x) {
    unsigned u = __float_as_uint(x);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (unsigned short)((u >> 16) | 64);
    return (unsigned short)((u + (0x7fffu + ((u >> 16) & 1u))) >> 16);
}
// two f32 -> packed bf16 pair on one v_cvt_pk_bf16_f32 (round to nearest even,
// identical to f2bf for every non-NaN input)
__device__ __forceinline__ unsigned pk_bf16(float a, float b) {
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
    const bf16x2 v = {(__bf16)a, (__bf16)b};
    return __builtin_bit_cast(unsigned, v);
}

// two f32 -> packed f16 pair, round to nearest even (ggml_fp32_to_fp16)
__device__ __forceinline__ unsigned pk_f16(float a, float b) {
    typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
    const f16x2 v = {(_Float16)a, (_Float16)b};
    return __builtin_bit_cast(unsigned, v);
}
// the 16-bit element type of a weight mode: F16 = true -> f16, else bf16
template <bool F16>
__device__ __forceinline__ unsigned pk16(float a, float b) {
    if constexpr (F16) return pk_f16(a, b);
    else return pk_bf16(a, b);
}
template <bool F16>
__device__ __forceinline__ floatx4 mfma16(uint4 a, uint4 b, floatx4 c) {
    if constexpr (F16)
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// KS > 1: split-K. A row tile's K is cut into KS slices, one workgroup each (blocks
// tile * KS + ks, consecutive, so a tile's workgroups are dispatched together); each
// stages only its slice of the activations, publishes its 16 x 16 partial tile as
// {tag, value} granules and merges 16 / KS of the tile's rows from the KS partials,
// added in slice order, then runs the epilogue. KS is a function of the op (K) only,
// never of NB, so every batch size computes the same bits.
template <int NB, int K, int PRO, int EPI, bool F16 = false, int KS = 1>
__global__ __launch_bounds__(MP_BLOCK) void gemm_b16_kernel(GemvP p) {
    const unsigned long long t_start = ts_begin(p.ts);
    static_assert(NB >= 1 && NB <= 16, "one 16-column MFMA tile of utterances");
    static_assert(K % (128 * KS) == 0, "K splits into KS slices of 4 waves x 32-wide chunks");
    static_assert(KS == 1 || PRO == PRO_PLAIN || PRO == PRO_PLAIN_B16 || PRO == PRO_SA_MERGE,
                  "split-K stages plain rows or the SA merge of its slice's heads");
    static_assert(16 % KS == 0, "a split workgroup merges 16 / KS rows");
    constexpr int KL = K / KS;  // this workgroup's K slice
    constexpr int KC = K / 32, KCS = KL / 32, KW = KCS / MP_NWAVES;
    constexpr int KP = KL + 8;  // padded bf16 row: rows land 16 B apart in the banks
    constexpr int NR = NB + 1;  // NB activation rows + one zero row for the unused MFMA columns
    constexpr bool STAGE = PRO != PRO_PLAIN && PRO != PRO_PLAIN_B16 && !(PRO == PRO_LN && NB >= 2) && KS == 1;
    constexpr int SC = pro_scratch<NB, PRO>();
    __shared__ __attribute__((aligned(16))) float actf[STAGE ? NB * K : 4];
    __shared__ __attribute__((aligned(16))) unsigned short actb[NR * KP];
    __shared__ __attribute__((aligned(16))) floatx4 part[MP_NWAVES][64];
    __shared__ float red[8];
    __shared__ float sc[SC];
    if constexpr (EPI == EPI_RESID_XA) {
        // the launch's last XA_SPLITS x NB workgroups: cross-attention on this launch's x1 (mp_xa.hpp)
        if ((int)blockIdx.x >= p.nrow_blocks) {
            xa_tail(p, t_start);
            return;
        }
    }
    if constexpr (EPI == EPI_QKV_SA) {
        // the launch's last NH x SA_SPLITS x NB workgroups: self-attention on this launch's q|k|v
        if ((int)blockIdx.x >= p.nrow_blocks) {
            sa_tail(p, t_start);
            return;
        }
    }
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int rt = KS == 1 ? (int)blockIdx.x : (int)blockIdx.x / KS, ks = KS == 1 ? 0 : (int)blockIdx.x % KS;

    // The activation loads go ahead of the weight stream (vector loads complete in
    // issue order, so rows loaded behind the weights would wait for all of them): the
    // PreRows prologues (LN rows, split merges), and plain 16-bit / f32 rows of up to 8
    // items per thread. The arithmetic after them is unchanged.
    constexpr bool LNB = PRO == PRO_LN && NB >= 2;
    constexpr bool PRE = PreRows<NB, K, PRO>::ON && (LNB || STAGE);
    constexpr int ITEMS8 = NB * (KL / 8), PT8 = (ITEMS8 + MP_BLOCK - 1) / MP_BLOCK;
    constexpr bool PLB = PRO == PRO_PLAIN_B16 && PT8 <= 8, PLF = PRO == PRO_PLAIN && PT8 <= 8;
    PreRows<NB, K, PRO> pre;
    // native vector types, every element assigned: an array of HIP's uint4 / float4 structs
    // assigned under a condition was kept in scratch memory
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    u32x4 vb[PLB ? PT8 : 1];
    f32x4 x0p[PLF ? PT8 : 1], x1p[PLF ? PT8 : 1];
    if constexpr (PRE) pre_load<NB, K, PRO>(p, pre);
    if constexpr (PLB) {
        const unsigned short *src = p.src_b16 + ks * KL;
#pragma unroll
        for (int u = 0; u < PT8; ++u) {
            const int e = u * MP_BLOCK + tid;
            vb[u] = e < ITEMS8 ? *(const u32x4 *)(src + (size_t)(e / (KL / 8)) * p.src_ld + (e % (KL / 8)) * 8)
                               : u32x4{0u, 0u, 0u, 0u};
        }
    }
    if constexpr (PLF) {
#pragma unroll
        for (int u = 0; u < PT8; ++u) {
            const int e = u * MP_BLOCK + tid;
            const float *src = p.src + ks * KL + (size_t)(min(e, ITEMS8 - 1) / (KL / 8)) * p.src_ld +
                               (min(e, ITEMS8 - 1) % (KL / 8)) * 8;
            x0p[u] = *(const f32x4 *)src;
            x1p[u] = *(const f32x4 *)(src + 4);
        }
    }
    if constexpr (PRE || PLB || PLF) __builtin_amdgcn_sched_barrier(0);  // issue order: rows, weights, arithmetic

    // weight fragments of this wave's K slice, issued before the prologue
    const uint4 *wf = (const uint4 *)p.Wb + ((size_t)rt * KC + ks * KCS + w * KW) * 64 + lane + ts_dep(t_start);
    uint4 a[KW];
#pragma unroll
    for (int i = 0; i < KW; ++i) a[i] = K == LTD ? ld_lt(wf + (size_t)i * 64) : ld_weight(wf + (size_t)i * 64);
    // the epilogue's operand of this thread's output (row, column below), behind the weights
    float eop = 0.f;
    if constexpr (epi_has_operand<EPI>()) {
        const int rq = KS == 1 ? tid >> 4 : ks * (16 / KS) + (tid >> 4), cq = tid & 15, nq = rt * 16 + rq;
        if (cq < NB && nq < p.N && (KS == 1 || tid < (16 / KS) * 16)) eop = epi_operand<EPI>(p, nq, cq);
    }
    if constexpr (PRE || PLB || PLF || epi_has_operand<EPI>()) __builtin_amdgcn_sched_barrier(0);

    // activation rows -> bf16 in LDS; row NB is zero and feeds MFMA columns NB..15
    if constexpr (LNB) {
        // LN rows rounded straight into the 16-bit tile (no f32 staging pass): the same
        // y values the f32 rows held, rounded by the same RNE conversion
        // (contraction off: the LN's last multiply is rounded to f32 before the conversion,
        // as on the batch-1 path, not fused into it as v_fma_mixlo_f16)
        ln_finish<NB, K>(p, pre.r, [&](int b, int k, float y) {
            if constexpr (F16) actb[b * KP + k] = __builtin_bit_cast(unsigned short, (_Float16)y);
            else actb[b * KP + k] = __builtin_bit_cast(unsigned short, (__bf16)y);
        });
        for (int e = tid; e < K / 8; e += MP_BLOCK) *(uint4 *)(actb + NB * KP + e * 8) = make_uint4(0, 0, 0, 0);
    } else if constexpr (PRO == PRO_SA_MERGE && KS > 1) {
        // the SA output of this slice's heads only: their SA_SPLITS key-split states merged
        // with PRO_SA_MERGE's arithmetic (split_weights, split_merge4), rounded to 16 bits
        static_assert(K == D && KL % DH == 0, "whole heads per slice");
        constexpr int HS = KL / DH;
        const int h0 = ks * HS;
        for (int q = tid; q < NB * HS; q += MP_BLOCK) {
            const float *pp = p.part + (size_t)((q / HS) * NH + h0 + q % HS) * SA_SPLITS * SA_PART;
            float ms[SA_SPLITS], ls[SA_SPLITS], e[SA_SPLITS], rd;
#pragma unroll
            for (int s2 = 0; s2 < SA_SPLITS; ++s2) { ms[s2] = pp[s2 * SA_PART]; ls[s2] = pp[s2 * SA_PART + 1]; }
            split_weights<SA_SPLITS>(ms, ls, e, rd);
#pragma unroll
            for (int s2 = 0; s2 < SA_SPLITS; ++s2) sc[q * (SA_SPLITS + 1) + s2] = e[s2];
            sc[q * (SA_SPLITS + 1) + SA_SPLITS] = rd;
        }
        constexpr int ITEMS = NB * (KL / 8);
        constexpr int PT = (ITEMS + MP_BLOCK - 1) / MP_BLOCK;
        float4 o0[PT][SA_SPLITS], o1[PT][SA_SPLITS];
#pragma unroll
        for (int u = 0; u < PT; ++u) {
            const int e = u * MP_BLOCK + tid;
            if (e < ITEMS) {
                const int b = e / (KL / 8), k = ks * KL + (e % (KL / 8)) * 8;
                const float *pp = p.part + (size_t)(b * NH + k / DH) * SA_SPLITS * SA_PART + 4 + k % DH;
#pragma unroll
                for (int s2 = 0; s2 < SA_SPLITS; ++s2) {
                    o0[u][s2] = *(const float4 *)(pp + s2 * SA_PART);
                    o1[u][s2] = *(const float4 *)(pp + s2 * SA_PART + 4);
                }
            }
        }
        lds_sync();  // the merge weights
#pragma unroll
        for (int u = 0; u < PT; ++u) {
            const int e = u * MP_BLOCK + tid;
            if (e < ITEMS) {
                const int b = e / (KL / 8), kk = (e % (KL / 8)) * 8, q = b * HS + (ks * KL + kk) / DH - h0;
                const float *eq = sc + q * (SA_SPLITS + 1);
                const float4 x0 = split_merge4<SA_SPLITS>(eq, o0[u], eq[SA_SPLITS]);
                const float4 x1 = split_merge4<SA_SPLITS>(eq, o1[u], eq[SA_SPLITS]);
                uint4 o;
                o.x = pk16<F16>(x0.x, x0.y);
                o.y = pk16<F16>(x0.z, x0.w);
                o.z = pk16<F16>(x1.x, x1.y);
                o.w = pk16<F16>(x1.z, x1.w);
                *(uint4 *)(actb + b * KP + kk) = o;
            }
        }
        for (int e = tid; e < KL / 8; e += MP_BLOCK) *(uint4 *)(actb + NB * KP + e * 8) = make_uint4(0, 0, 0, 0);
    } else if constexpr (STAGE) {
        if constexpr (PRE) pre_finish<NB, K, PRO>(p, pre, actf, sc);  // loads issued first
        else prologue<NB, K, PRO>(p, actf, red, sc);
        for (int e = tid; e < NR * (K / 8); e += MP_BLOCK) {
            const int b = e / (K / 8), k = (e % (K / 8)) * 8;
            uint4 o = make_uint4(0, 0, 0, 0);
            if (b < NB) {
                const float4 x0 = *(const float4 *)(actf + b * K + k), x1 = *(const float4 *)(actf + b * K + k + 4);
                o.x = pk16<F16>(x0.x, x0.y);
                o.y = pk16<F16>(x0.z, x0.w);
                o.z = pk16<F16>(x1.x, x1.y);
                o.w = pk16<F16>(x1.z, x1.w);
            }
            *(uint4 *)(actb + b * KP + k) = o;
        }
    } else if constexpr (PLB) {
#pragma unroll
        for (int u = 0; u < PT8; ++u) {
            const int e = u * MP_BLOCK + tid;
            if (e < ITEMS8) *(u32x4 *)(actb + (e / (KL / 8)) * KP + (e % (KL / 8)) * 8) = vb[u];
        }
        for (int e = tid; e < KL / 8; e += MP_BLOCK) *(uint4 *)(actb + NB * KP + e * 8) = make_uint4(0, 0, 0, 0);
    } else if constexpr (PLF) {
#pragma unroll
        for (int u = 0; u < PT8; ++u) {
            const int e = u * MP_BLOCK + tid;
            if (e < ITEMS8) {
                uint4 o;
                o.x = pk16<F16>(x0p[u].x, x0p[u].y);
                o.y = pk16<F16>(x0p[u].z, x0p[u].w);
                o.z = pk16<F16>(x1p[u].x, x1p[u].y);
                o.w = pk16<F16>(x1p[u].z, x1p[u].w);
                *(uint4 *)(actb + (e / (KL / 8)) * KP + (e % (KL / 8)) * 8) = o;
            }
        }
        for (int e = tid; e < KL / 8; e += MP_BLOCK) *(uint4 *)(actb + NB * KP + e * 8) = make_uint4(0, 0, 0, 0);
    } else if constexpr (PRO == PRO_PLAIN_B16) {
        // bf16 rows (written by the FFN-up epilogue): copied as they are, 12 uint4
        // per thread in flight
        constexpr int ITEMS = NB * (KL / 8), BATCH = 12;
        const unsigned short *src = p.src_b16 + ks * KL;
        for (int base = 0; base < ITEMS; base += BATCH * MP_BLOCK) {
            uint4 v[BATCH];
#pragma unroll
            for (int u = 0; u < BATCH; ++u) {
                const int e = base + u * MP_BLOCK + tid;
                v[u] = e < ITEMS ? *(const uint4 *)(src + (size_t)(e / (KL / 8)) * p.src_ld + (e % (KL / 8)) * 8)
                                 : make_uint4(0u, 0u, 0u, 0u);
            }
#pragma unroll
            for (int u = 0; u < BATCH; ++u) {
                const int e = base + u * MP_BLOCK + tid;
                if (e < ITEMS) *(uint4 *)(actb + (e / (KL / 8)) * KP + (e % (KL / 8)) * 8) = v[u];
            }
        }
        for (int e = tid; e < KL / 8; e += MP_BLOCK) *(uint4 *)(actb + NB * KP + e * 8) = make_uint4(0, 0, 0, 0);
    } else {
        // NB rows straight from HBM/L2, in batches of 8 items per thread with all
        // 16 loads issued before the first conversion (one latency per batch)
        constexpr int ITEMS = NB * (KL / 8), BATCH = 8;
        for (int base = 0; base < ITEMS; base += BATCH * MP_BLOCK) {
            float4 x0[BATCH], x1[BATCH];
#pragma unroll
            for (int u = 0; u < BATCH; ++u) {
                const int e = base + u * MP_BLOCK + tid;
                if (e < ITEMS) {
                    const float *src = p.src + ks * KL + (size_t)(e / (KL / 8)) * p.src_ld + (e % (KL / 8)) * 8;
                    x0[u] = *(const float4 *)src;
                    x1[u] = *(const float4 *)(src + 4);
                }
            }
#pragma unroll
            for (int u = 0; u < BATCH; ++u) {
                const int e = base + u * MP_BLOCK + tid;
                if (e < ITEMS) {
                    uint4 o;
                    o.x = pk16<F16>(x0[u].x, x0[u].y);
                    o.y = pk16<F16>(x0[u].z, x0[u].w);
                    o.z = pk16<F16>(x1[u].x, x1[u].y);
                    o.w = pk16<F16>(x1[u].z, x1[u].w);
                    *(uint4 *)(actb + (e / (KL / 8)) * KP + (e % (KL / 8)) * 8) = o;
                }
            }
        }
        for (int e = tid; e < KL / 8; e += MP_BLOCK) *(uint4 *)(actb + NB * KP + e * 8) = make_uint4(0, 0, 0, 0);
    }
    lds_sync();
#ifndef MP_TS_PROBE
    ts_mark(p.ts, t_start);  // profiling: activation tile staged
#endif

    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    const unsigned short *brow = actb + min(lane & 15, NB) * KP + 8 * (lane >> 4);
#pragma unroll
    for (int i = 0; i < KW; ++i) {
        const int kc = w * KW + i;
        const uint4 bv = *(const uint4 *)(brow + kc * 32);
        acc = mfma16<F16>(a[i], bv, acc);
    }
    part[w][lane] = acc;
    lds_sync();
    // thread t -> (row t/16, column t%16); D[row][col] sits in lane (row/4)*16 + col, register row%4
    int row = tid >> 4;
    const int col = tid & 15;
    float v;
    {
        const int ls = (row >> 2) * 16 + col, rg = row & 3;
        v = ((part[0][ls][rg] + part[1][ls][rg]) + part[2][ls][rg]) + part[3][ls][rg];
    }
    if constexpr (KS > 1) {
        // publish this slice's partial (row, col) ...
        using gu64 = __attribute__((address_space(1))) unsigned long long;
        const unsigned tag = (unsigned)p.iter[0] * 64u + p.layer + 1u;
        gu64 *gt = (gu64 *)p.kgh + (size_t)rt * KS * 256;
        __hip_atomic_store(gt + ks * 256 + tid, ((unsigned long long)tag << 32) | __float_as_uint(v), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        // ... and merge rows [ks * 16 / KS, (ks + 1) * 16 / KS) of the tile: the KS partials
        // of (row, col), added in slice order (a bounded sweep; poisoned + HX_ERR_KS if a
        // sibling never publishes)
        constexpr int MR = 16 / KS;
        if (tid >= MR * 16) return;
        row = ks * MR + (tid >> 4);
        const int gi = row * 16 + col;
        float pv[KS];
        for (unsigned spins = 0;; ++spins) {
            bool ok = true;
#pragma unroll
            for (int s2 = 0; s2 < KS; ++s2) {
                const unsigned long long u = __hip_atomic_load(gt + s2 * 256 + gi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok &= (unsigned)(u >> 32) == tag;
                pv[s2] = __uint_as_float((unsigned)u);
            }
            if (__all(ok)) break;
            if (spins >= HX_SPIN_LIMIT) {
                if ((tid & 63) == 0) __hip_atomic_fetch_or((__attribute__((address_space(1))) int *)p.hx_err, HX_ERR_KS,
                                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
                for (int s2 = 0; s2 < KS; ++s2) pv[s2] = __builtin_nanf("");
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        v = pv[0];
#pragma unroll
        for (int s2 = 1; s2 < KS; ++s2) v = v + pv[s2];
    }
    if (col >= NB) return;
    const int n = rt * 16 + row;
    if (n >= p.N) return;
    if constexpr (EPI == EPI_RESID_XA) publish_x1_op(p, v, n, col, eop);
    else if constexpr (EPI == EPI_QKV_SA) publish_qkv(p, v, n, col);
    else if constexpr (EPI == EPI_BIAS || EPI == EPI_RESID || EPI == EPI_ADD_STORE) epi_store_op<EPI>(p, v, n, col, eop);
    else epi_store<EPI>(p, v, n, col, EPI == EPI_LTX_ADD ? sc[col * LTD + n] : 0.f);
    ts_end(p.ts, t_start);
}

template <int PRO, int EPI>
static bool b16_args_ok(const GemvP &p) {
    if (!p.Wb || p.N <= 0) return false;
    bool ok = true;
    if constexpr (PRO == PRO_PLAIN) ok &= p.src != nullptr;
    if constexpr (PRO == PRO_PLAIN_B16) ok &= p.src_b16 != nullptr;
    if constexpr (PRO == PRO_SA_MERGE) ok &= p.part != nullptr;
    if constexpr (PRO == PRO_LTS_MERGE) ok &= p.part && p.addsrc;
    if constexpr (PRO == PRO_XA_LN) ok &= p.part && p.src && p.lnw && p.xres;
    if constexpr (PRO == PRO_LN) ok &= p.src && p.lnw;
    if constexpr (PRO == PRO_LTX_LN) ok &= p.lt_s && p.lt_pos && p.ltX && p.lnw;
    if constexpr (PRO == PRO_LT_ATTN) ok &= p.ltq && p.ltk && p.ltv;
    if constexpr (PRO == PRO_LTARG_ATTN)
        ok &= p.logits && p.codes_cur && p.qkvtab && p.lk && p.lv && p.ltk && p.ltv && p.step && p.smp.cfg && p.smp.argeos;
    if constexpr (EPI == EPI_STORE || EPI == EPI_GELU) ok &= p.out != nullptr;
    if constexpr (EPI == EPI_GELU_B16 || EPI == EPI_GELU_F16) ok &= p.out_b16 != nullptr;
    if constexpr (EPI == EPI_BIAS) ok &= p.out && p.bias;
    if constexpr (EPI == EPI_RESID) ok &= p.resid != nullptr;
    if constexpr (EPI == EPI_ADD_STORE) ok &= p.out && p.addsrc;
    if constexpr (EPI == EPI_LTX_ADD) ok &= p.out && p.ptab && p.lt_pos && p.cb >= 1;
    if constexpr (EPI == EPI_QKV || EPI == EPI_QKV_SA) ok &= p.out && p.kc && p.vc && p.pos;
    if constexpr (EPI == EPI_QKV_SA) ok &= qkv_sa_args_ok(p);
    if constexpr (EPI == EPI_LTQKV) ok &= p.lq && p.lk && p.lv;
    if constexpr (EPI == EPI_RESID_XA)
        ok &= p.resid && p.xh && p.iter && p.hx_err && p.N == D && p.xa.part && p.xa.lnw && p.xa.kp && p.xa.vp &&
              p.xa.T && p.xa.Tmax >= 1 && p.xa.Tmax <= TMAX_LIMIT;
    return ok;
}

template <int NB, int K, int PRO, int EPI, bool F16 = false, int KS = 1>
static hipError_t launch_b16(const GemvP &p, hipStream_t s) {
    if (!b16_args_ok<PRO, EPI>(p)) return hipErrorInvalidValue;
    if (KS > 1 && (!p.kgh || !p.iter || !p.hx_err)) return hipErrorInvalidValue;
    GemvP q = p;
    q.nrow_blocks = (p.N + 15) / 16 * KS;  // row workgroups (KS per 16-row tile)
    const int grid = q.nrow_blocks + (EPI == EPI_RESID_XA ? XA_SPLITS * NB : EPI == EPI_QKV_SA ? NH * SA_SPLITS * NB : 0);
    mp::launch((gemm_b16_kernel<NB, K, PRO, EPI, F16, KS>), dim3(grid), dim3(MP_BLOCK), 0, s, q);
    return hipGetLastError();
}
// split-K of the FFN-down projection (K = 3072, 48 row tiles): a function of the op only.
// 4 slices = 192 workgroups of 24 KiB weights + the slice's activations each: bf16 B=16
// ff2 5.21 -> 4.37 us, 28.5k -> 29.3k frames/s, B=8 17.4k -> 17.6k, B=1 within 1 %
// (gpurun_out/r04h_ab.txt, r04h_ops16_ks.txt)
#ifndef MP_FF2_KS
#define MP_FF2_KS 4
#endif
constexpr int FF2_KS = MP_FF2_KS;
// split-K of the O-projection (K = 768, 48 row tiles): whole SA heads per slice. Measured
// and left off: 2 slices moved bf16 B=16 by +0.5 % and B=8 / B=1 by -1.5 .. -3 %
#ifndef MP_OPROJ_KS
#define MP_OPROJ_KS 1
#endif
constexpr int OPROJ_KS = MP_OPROJ_KS;
int b16_oproj_ks() { return OPROJ_KS; }

#define MP_B16_OPS(NB)                                                                                                  \
    hipError_t b16_qkv_##NB(const GemvP &p, hipStream_t s) { return launch_b16<NB, D, PRO_LN, EPI_QKV>(p, s); }             \
    hipError_t b16_qkv_sa_##NB(const GemvP &p, hipStream_t s) { return launch_b16<NB, D, PRO_LN, EPI_QKV_SA>(p, s); }       \
    hipError_t b16_oproj_##NB(const GemvP &p, hipStream_t s) { return launch_b16<NB, D, PRO_SA_MERGE, EPI_RESID, false, OPROJ_KS>(p, s); }   \
    hipError_t b16_oproj_xa_##NB(const GemvP &p, hipStream_t s) {                                                      \
        return launch_b16<NB, D, PRO_SA_MERGE, EPI_RESID_XA, false, OPROJ_KS>(p, s);                                   \
    }                                                                                                                   \
    hipError_t b16_ff1_##NB(const GemvP &p, hipStream_t s) { return launch_b16<NB, D, PRO_XA_LN, EPI_GELU_B16>(p, s); }     \
    hipError_t b16_ff1p_##NB(const GemvP &p, hipStream_t s) { return launch_b16<NB, D, PRO_LN, EPI_GELU_B16>(p, s); }       \
    hipError_t b16_ff2_##NB(const GemvP &p, hipStream_t s) { return launch_b16<NB, DFF, PRO_PLAIN_B16, EPI_ADD_STORE, false, FF2_KS>(p, s); }  \
    hipError_t b16_lt_a_##NB(const GemvP &p, hipStream_t s) { return launch_b16<NB, LTD, PRO_LTX_LN, EPI_LTQKV>(p, s); }    \
    hipError_t b16_lt_bg_##NB(const GemvP &p, hipStream_t s) { return launch_b16<NB, LTD, PRO_LTARG_ATTN, EPI_LTX_ADD>(p, s); } \
    hipError_t b16_lt_b_##NB(const GemvP &p, hipStream_t s) { return launch_b16<NB, LTD, PRO_LT_ATTN, EPI_ADD_STORE>(p, s); } \
    hipError_t b16_lt_c_##NB(const GemvP &p, hipStream_t s) { return launch_b16<NB, LTD, PRO_LN, EPI_GELU>(p, s); }         \
    hipError_t b16_lt_d_##NB(const GemvP &p, hipStream_t s) { return launch_b16<NB, LTF, PRO_PLAIN, EPI_ADD_STORE>(p, s); } \
    hipError_t b16_lt_e_##NB(const GemvP &p, hipStream_t s) { return launch_b16<NB, LTD, PRO_PLAIN, EPI_BIAS>(p, s); }      \
    hipError_t b16_lt_es_##NB(const GemvP &p, hipStream_t s) { return launch_b16<NB, LTD, PRO_PLAIN, EPI_BIAS>(p, s); }      \
    hipError_t b16_lt_em_##NB(const GemvP &p, hipStream_t s) { return launch_b16<NB, LTD, PRO_LTS_MERGE, EPI_BIAS>(p, s); }

#define MP_F16_OPS(NB)                                                                                                  \
    hipError_t f16_qkv_##NB(const GemvP &p, hipStream_t s) { return launch_b16<NB, D, PRO_LN, EPI_QKV, true>(p, s); }             \
    hipError_t f16_qkv_sa_##NB(const GemvP &p, hipStream_t s) { return launch_b16<NB, D, PRO_LN, EPI_QKV_SA, true>(p, s); }       \
    hipError_t f16_oproj_##NB(const GemvP &p, hipStream_t s) { return launch_b16<NB, D, PRO_SA_MERGE, EPI_RESID, true, OPROJ_KS>(p, s); }   \
    hipError_t f16_oproj_xa_##NB(const GemvP &p, hipStream_t s) {                                                      \
        return launch_b16<NB, D, PRO_SA_MERGE, EPI_RESID_XA, true, OPROJ_KS>(p, s);                                   \
    }                                                                                                                   \
    hipError_t f16_ff1_##NB(const GemvP &p, hipStream_t s) { return launch_b16<NB, D, PRO_XA_LN, EPI_GELU_F16, true>(p, s); }     \
    hipError_t f16_ff2_##NB(const GemvP &p, hipStream_t s) { return launch_b16<NB, DFF, PRO_PLAIN_B16, EPI_ADD_STORE, true, FF2_KS>(p, s); }  \
    hipError_t f16_lt_a_##NB(const GemvP &p, hipStream_t s) { return launch_b16<NB, LTD, PRO_LTX_LN, EPI_LTQKV, true>(p, s); }    \
    hipError_t f16_lt_bg_##NB(const GemvP &p, hipStream_t s) { return launch_b16<NB, LTD, PRO_LTARG_ATTN, EPI_LTX_ADD, true>(p, s); } \
    hipError_t f16_lt_b_##NB(const GemvP &p, hipStream_t s) { return launch_b16<NB, LTD, PRO_LT_ATTN, EPI_ADD_STORE, true>(p, s); } \
    hipError_t f16_lt_c_##NB(const GemvP &p, hipStream_t s) { return launch_b16<NB, LTD, PRO_LN, EPI_GELU, true>(p, s); }         \
    hipError_t f16_lt_d_##NB(const GemvP &p, hipStream_t s) { return launch_b16<NB, LTF, PRO_PLAIN, EPI_ADD_STORE, true>(p, s); } \
    hipError_t f16_lt_e_##NB(const GemvP &p, hipStream_t s) { return launch_b16<NB, LTD, PRO_PLAIN, EPI_BIAS, true>(p, s); }

MP_B16_OPS(1)
MP_B16_OPS(2)
MP_B16_OPS(4)
MP_B16_OPS(8)
MP_B16_OPS(16)
MP_F16_OPS(1)
MP_F16_OPS(2)
MP_F16_OPS(4)
MP_F16_OPS(8)
MP_F16_OPS(16)
// bf16 mode at 8 and 16 slots: the O-projection + XA launch reads the SA output its
// split workgroups merged (plain rows), and its XA workgroups merge x2
hipError_t b16_oproj_xa_pm_16(const GemvP &p, hipStream_t s) {
    return launch_b16<16, D, PRO_PLAIN, EPI_RESID_XA, false, OPROJ_KS>(p, s);
}
hipError_t b16_oproj_xa_pm_8(const GemvP &p, hipStream_t s) {
    return launch_b16<8, D, PRO_PLAIN, EPI_RESID_XA, false, OPROJ_KS>(p, s);
}
// the LT in_proj of an F16 file is F16 too (the bf16 mode keeps it f32)
hipError_t f16_lt_in0_1(const GemvP &p, hipStream_t s) { return launch_b16<1, D, PRO_LN, EPI_BIAS, true>(p, s); }
hipError_t f16_lt_in0_2(const GemvP &p, hipStream_t s) { return launch_b16<2, D, PRO_LN, EPI_BIAS, true>(p, s); }
hipError_t f16_lt_in0_4(const GemvP &p, hipStream_t s) { return launch_b16<4, D, PRO_LN, EPI_BIAS, true>(p, s); }
hipError_t f16_lt_in0_8(const GemvP &p, hipStream_t s) { return launch_b16<8, D, PRO_LN, EPI_BIAS, true>(p, s); }
hipError_t f16_lt_in0_16(const GemvP &p, hipStream_t s) { return launch_b16<16, D, PRO_LN, EPI_BIAS, true>(p, s); }
hipError_t f16_lt_inh_1(const GemvP &p, hipStream_t s) { return launch_b16<1, D, PRO_PLAIN, EPI_BIAS, true>(p, s); }
// o_net + residual after lt_pick_kernel (large batches)
hipError_t b16_lt_bo_8(const GemvP &p, hipStream_t s) { return launch_b16<8, LTD, PRO_PLAIN, EPI_ADD_STORE>(p, s); }
hipError_t b16_lt_bo_16(const GemvP &p, hipStream_t s) { return launch_b16<16, LTD, PRO_PLAIN, EPI_ADD_STORE>(p, s); }
hipError_t f16_lt_bo_8(const GemvP &p, hipStream_t s) { return launch_b16<8, LTD, PRO_PLAIN, EPI_ADD_STORE, true>(p, s); }
hipError_t f16_lt_bo_16(const GemvP &p, hipStream_t s) { return launch_b16<16, LTD, PRO_PLAIN, EPI_ADD_STORE, true>(p, s); }

// f32 [N][K] -> bf16 (F16: f16) fragment order [ceil(N/16)][K/32][64][8], rows >= N
// zero. f16: round to nearest even; exact for an F16 file's (widened) values.
template <bool F16>
__global__ void pack_16_kernel(const float *W, int N, int K, unsigned short *out) {
    const size_t total = (size_t)((N + 15) / 16) * (K / 32) * 64;
    for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
        const int lane = (int)(e % 64);
        const size_t frag = e / 64;
        const int kc = (int)(frag % (K / 32)), rt = (int)(frag / (K / 32));
        const int n = rt * 16 + (lane & 15), k0 = kc * 32 + 8 * (lane >> 4);
        unsigned short *o = out + e * 8;
        for (int j = 0; j < 8; ++j) {
            const float w = n < N ? W[(size_t)n * K + k0 + j] : 0.f;
            o[j] = F16 ? __builtin_bit_cast(unsigned short, (_Float16)w) : f2bf(w);
        }
    }
}

hipError_t pack_b16(const float *W, int N, int K, unsigned short *out, hipStream_t s, bool f16) {
    if (!W || !out || N <= 0 || K % 32) return hipErrorInvalidValue;
    if (f16) mp::launch(pack_16_kernel<true>, dim3(1024), dim3(256), 0, s, W, N, K, out);
    else mp::launch(pack_16_kernel<false>, dim3(1024), dim3(256), 0, s, W, N, K, out);
    return hipGetLastError();
}

}  // namespace mp
