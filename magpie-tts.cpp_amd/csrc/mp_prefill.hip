// Per-utterance preamble kernels (run once per batch, outside the frame loop):
// text encoder (magpie_encode_text, magpie.cpp:2284-2374), cross-attention K/V
// precompute (magpie.cpp:1663-1711, 4098-4136) and the batched 110-frame context
// prefill (magpie.cpp:3911-4060, 4167-4238).
//
// Rows are (utterance, position) pairs laid out r = b * rows_per_utt + t. The
// projections are an LDS-tiled f32 GEMM (64x64 tile, 4x4 per thread) with the
// tiny neighbouring ops fused into its operand loader (causal k=3 conv taps) or
// its epilogue (residual, GELU, KV-cache scatter, XA K/V split).
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <math.h>

#include <algorithm>
#include <cstdlib>

#include "mp_device.hpp"
#include "mp_params.hpp"
#include "mp_prefill_api.hpp"
#include "mp_xa.hpp"

#ifndef MP_PRE_PF
#define MP_PRE_PF 4  // K steps of operand loads in flight per thread (8 measured slower, round 6)
#endif

namespace mp {

// Epilogue of output (m, n) (bias, residual, GELU, KV-cache scatter, XA K/V split).
template <int EPI>
__device__ __forceinline__ void gemm_store1(const GemmP &p, int m, int n, float v) {
    const int b = m / p.rows_per_utt, t = m % p.rows_per_utt;
    if (p.bias) v += p.bias[n];
    if constexpr (EPI == GE_STORE) p.C[(size_t)m * p.ldc + n] = v;
    else if constexpr (EPI == GE_RESID) p.C[(size_t)m * p.ldc + n] = v + p.C[(size_t)m * p.ldc + n];
    else if constexpr (EPI == GE_GELU) p.C[(size_t)m * p.ldc + n] = gelu_tanh(v);
    else if constexpr (EPI == GE_QKV_CACHE) {
        const size_t slot = ((size_t)(b * p.nlayers + p.layer) * p.max_seq + t) * D;
        if (n < D) p.C[(size_t)m * p.ldc + n] = v;
        else kv_store(n < 2 * D ? p.kc : p.vc, slot + (n < 2 * D ? n - D : n - 2 * D), v, p.kv16);
    } else if constexpr (EPI == GE_XAKV) {
        const size_t slot = ((size_t)(b * p.nlayers + p.layer) * p.Tmax + t) * DXA;
        if (n < DXA) p.xak[slot + n] = v;
        else p.xav[slot + n - DXA] = v;
    }
}

// A 4x4 register tile at rows m0.., columns n0..: the epilogue, or (split-K)
// the raw partial sums into split blockIdx.z's slice of p.part.
template <int EPI>
__device__ __forceinline__ void gemm_store(const GemmP &p, const float (&acc)[4][4], int m0, int n0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int m = m0 + i;
        if (m >= p.M) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int n = n0 + j;
            if (n >= p.N) continue;
            if (p.part) p.part[((size_t)blockIdx.z * p.M + m) * p.N + n] = acc[i][j];
            else gemm_store1<EPI>(p, m, n, acc[i][j]);
        }
    }
}

// Split-K reduction: v = sum of the splits in order, then the epilogue.
template <int EPI>
__global__ __launch_bounds__(256) void gemm_reduce_kernel(GemmP p, int splits) {
    const size_t total = (size_t)p.M * p.N;
    const int nb = p.nbatch > 1 ? p.nbatch : 1;  // batched GEMM: partials [batch][split][M][N]
    for (size_t e = (size_t)blockIdx.x * 256 + threadIdx.x; e < total * nb; e += (size_t)gridDim.x * 256) {
        const int bz = (int)(e / total);
        const size_t ee = e % total, base = (size_t)bz * splits * total + ee;
        float v = p.part[base];
        for (int s = 1; s < splits; ++s) v += p.part[base + (size_t)s * total];
        GemmP q = p;
        if (bz) { q.C += bz * p.sC; q.layer += bz; }
        gemm_store1<EPI>(q, (int)(ee / p.N), (int)(ee % p.N), v);
    }
}

// K steps of 16 with PF = 8 steps' operand loads in flight per thread (register ring):
// a step's loads are issued PF steps before its tile is staged, so the global latency
// is paid once per PF steps (once per PRE_KS-wide split slice), not per step (the preamble GEMMs have small grids: one
// workgroup per CU or fewer). The arithmetic (k order, FMA order) is the plain
// LDS-tiled GEMM's.
template <int EPI, int TAPS>
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmP p) {
    constexpr int BM = 64, BN = 64, BK = 16, PF = MP_PRE_PF;
    __shared__ float As[BK][BM + 4];
    __shared__ float Ws[BK][BN + 4];
    const int tid = threadIdx.x;
    const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
    const int tx = tid & 15, ty = tid >> 4;
    float acc[4][4] = {};
    const int lr = tid >> 2, lk = (tid & 3) * 4;  // loader: row lr, k lk..lk+3
    int zs;
    const int S = gemm_batch_enter(p, zs);
    const int ks = p.K / S, kbeg = zs * ks;  // split-K slice (S == 1: all of K)
    const int nsteps = ks / BK;
    const int m = m0 + lr, n = n0 + lr;
    auto load_a = [&](int k0) {
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (m < p.M) {
            if constexpr (TAPS == 0) {
                v = *(const float4 *)(p.A + (size_t)m * p.lda + k0 + lk);
            } else {
                // weights are tap-major [N][tap][Cin] (re-laid out at load), so a
                // 16-wide K step lies inside one tap: one float4 of input row t-2+tap
                const int t = m % p.rows_per_utt;
                const int tap = k0 / p.lda, i = k0 % p.lda + lk;
                if (t - (TAPS - 1) + tap >= 0) v = *(const float4 *)(p.A + (size_t)(m - (TAPS - 1) + tap) * p.lda + i);
            }
        }
        return v;
    };
    auto load_w = [&](int k0) {
        return n < p.N ? *(const float4 *)(p.W + (size_t)n * p.K + k0 + lk) : make_float4(0.f, 0.f, 0.f, 0.f);
    };
    float4 ra[PF], rw[PF];
#pragma unroll
    for (int u = 0; u < PF; ++u)
        if (u < nsteps) { ra[u] = load_a(kbeg + u * BK); rw[u] = load_w(kbeg + u * BK); }
    for (int base = 0; base < nsteps; base += PF) {
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            const int step = base + u;
            if (step >= nsteps) break;
            float a[4] = {ra[u].x, ra[u].y, ra[u].z, ra[u].w};
            if (p.xround)  // F16 weights: the operand ggml's F16 mul_mat multiplies (uniform branch)
#pragma unroll
                for (int e = 0; e < 4; ++e) a[e] = (float)(_Float16)a[e];
#pragma unroll
            for (int e = 0; e < 4; ++e) As[lk + e][lr] = a[e];
            Ws[lk + 0][lr] = rw[u].x; Ws[lk + 1][lr] = rw[u].y; Ws[lk + 2][lr] = rw[u].z; Ws[lk + 3][lr] = rw[u].w;
            if (step + PF < nsteps) { ra[u] = load_a(kbeg + (step + PF) * BK); rw[u] = load_w(kbeg + (step + PF) * BK); }
            __syncthreads();
#pragma unroll
            for (int kk = 0; kk < BK; ++kk) {
                const float4 a4 = *(const float4 *)&As[kk][ty * 4];
                const float4 w4 = *(const float4 *)&Ws[kk][tx * 4];
                const float av[4] = {a4.x, a4.y, a4.z, a4.w}, wv[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(av[i], wv[j], acc[i][j]);
            }
            __syncthreads();
        }
    }
    gemm_store<EPI>(p, acc, m0 + ty * 4, n0 + tx * 4);
}

// The same GEMM on the exact-f32 matrix cores (v_mfma_f32_16x16x4_f32: one k-ordered
// fmaf chain per output, bitwise the VALU kernel's acc = fmaf(a_k, w_k, acc) for k
// ascending; MI355X_MICROARCH.md, FP32-input MFMA), at twice the unpacked VALU rate and
// without the 4x4-per-thread LDS operand traffic. Same tiles, loader (register ring,
// causal conv taps), split-K slices and epilogue. Wave w owns the 32 x 32 quadrant
// (rows 32 (w & 1), columns 32 (w >> 1)) of the 64 x 64 tile: 2 x 2 MFMA tiles; lane l
// feeds A[row l & 15][k l >> 4] and B[k l >> 4][col l & 15] and holds C rows
// 4 (l >> 4) + i, column l & 15.
template <int EPI, int TAPS>
__global__ __launch_bounds__(256) void gemm_f32_mfma_kernel(GemmP p) {
    constexpr int BM = 64, BN = 64, BK = 16, PF = MP_PRE_PF;
    typedef float f4v __attribute__((ext_vector_type(4)));
    __shared__ float As[BK][BM + 4];
    __shared__ float Ws[BK][BN + 4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
    const int rq = 32 * (w & 1), cq = 32 * (w >> 1);  // the wave's quadrant
    f4v acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};
    f4v tot[2][2];
    const int lr = tid >> 2, lk = (tid & 3) * 4;  // loader: row lr, k lk..lk+3
    // split-K: one split per blockIdx.z (gridDim.z == nsplit: partials, summed after), or
    // (large grids, gridDim.z == 1 < nsplit) every split of the tile here in turn, each its
    // own chain from 0, folded into tot in split order: tot = p0, tot += p1, ... - the same
    // float operations as the reduction of the partials, without writing them
    int zs;
    const int S = gemm_batch_enter(p, zs);
    const int ks = p.K / S, kbeg = zs * ks;
    const int nsteps = ks / BK;
    const int sl = (S == 1 && p.nsplit > 1) ? (p.K / p.nsplit) / BK : nsteps;  // steps per split
    const int m = m0 + lr, n = n0 + lr;
    auto load_a = [&](int k0) {
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (m < p.M) {
            if constexpr (TAPS == 0) {
                v = *(const float4 *)(p.A + (size_t)m * p.lda + k0 + lk);
            } else {
                const int t = m % p.rows_per_utt;
                const int tap = k0 / p.lda, i = k0 % p.lda + lk;
                if (t - (TAPS - 1) + tap >= 0) v = *(const float4 *)(p.A + (size_t)(m - (TAPS - 1) + tap) * p.lda + i);
            }
        }
        return v;
    };
    auto load_w = [&](int k0) {
        return n < p.N ? *(const float4 *)(p.W + (size_t)n * p.K + k0 + lk) : make_float4(0.f, 0.f, 0.f, 0.f);
    };
    float4 ra[PF], rw[PF];
#pragma unroll
    for (int u = 0; u < PF; ++u)
        if (u < nsteps) { ra[u] = load_a(kbeg + u * BK); rw[u] = load_w(kbeg + u * BK); }
    const int fr = lane & 15, fk = lane >> 4;
    for (int base = 0; base < nsteps; base += PF) {
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            const int step = base + u;
            if (step >= nsteps) break;
            float a[4] = {ra[u].x, ra[u].y, ra[u].z, ra[u].w};
            if (p.xround)
#pragma unroll
                for (int e = 0; e < 4; ++e) a[e] = (float)(_Float16)a[e];
#pragma unroll
            for (int e = 0; e < 4; ++e) As[lk + e][lr] = a[e];
            Ws[lk + 0][lr] = rw[u].x; Ws[lk + 1][lr] = rw[u].y; Ws[lk + 2][lr] = rw[u].z; Ws[lk + 3][lr] = rw[u].w;
            if (step + PF < nsteps) { ra[u] = load_a(kbeg + (step + PF) * BK); rw[u] = load_w(kbeg + (step + PF) * BK); }
            __syncthreads();
#pragma unroll
            for (int k4 = 0; k4 < BK; k4 += 4) {
                float af[2], bf[2];
#pragma unroll
                for (int i = 0; i < 2; ++i) af[i] = As[k4 + fk][rq + 16 * i + fr];
#pragma unroll
                for (int j = 0; j < 2; ++j) bf[j] = Ws[k4 + fk][cq + 16 * j + fr];
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bf[j], acc[i][j], 0, 0, 0);
            }
            __syncthreads();
            if ((step + 1) % sl == 0) {  // a split's chain is complete: fold it in, split order
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        tot[i][j] = step + 1 == sl ? acc[i][j] : tot[i][j] + acc[i][j];
                        acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};
                    }
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int nn = n0 + cq + 16 * j + fr;
            if (nn >= p.N) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int mm = m0 + rq + 16 * i + 4 * fk + r;
                if (mm >= p.M) continue;
                if (p.part) p.part[((size_t)blockIdx.z * p.M + mm) * p.N + nn] = tot[i][j][r];
                else gemm_store1<EPI>(p, mm, nn, tot[i][j][r]);
            }
        }
}

// Q8_0 weights (weight mode MP_WEIGHTS_Q8): ggml's quantised mul_mat. Every K
// step is one 32-wide Q8_0 block; the A tile is quantised as it is loaded
// (quantize_row_q8_0_ref: d = amax/127, id = 1/d, q = roundf(x*id), d kept as
// fp16; the four loader lanes of a row share amax through DPP), the block dot
// products are exact int32 (v_dot4c_i32_i8) and are scaled by d_w * d_a
// (ggml_vec_dot_q8_0_q8_0).
__device__ __forceinline__ int pack_i8x4(float a, float b, float c, float d) {
    return (int)(((unsigned)(int)a & 0xffu) | (((unsigned)(int)b & 0xffu) << 8) | (((unsigned)(int)c & 0xffu) << 16) |
                 ((unsigned)(int)d << 24));
}

template <int EPI>
__global__ __launch_bounds__(256) void gemm_q8_kernel(GemmP p) {
    constexpr int BM = 64, BN = 64;
    __shared__ int Aq[BM][9];
    __shared__ int Wq[BN][9];
    __shared__ float Ad[BM], Wd[BN];
    const int tid = threadIdx.x;
    const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
    const int tx = tid & 15, ty = tid >> 4;
    const int lr = tid >> 2, part = tid & 3;  // loader: row lr, elements 8 part .. 8 part + 7 of the block
    const int nblk = p.K / 32;
    int zs;
    const int S = gemm_batch_enter(p, zs);
    const int bs = nblk / S, bbeg = zs * bs;  // split-K slice in whole blocks
    float acc[4][4] = {};
    // PF blocks' operand loads in flight per thread (register ring), as gemm_f32_kernel
    constexpr int PF = 4;
    const int m = m0 + lr, n = n0 + lr;
    float4 ra0[PF], ra1[PF];
    uint2 rwv[PF];
    float rwd[PF];
    auto load = [&](int u, int kb) {
        const int k0 = kb * 32 + part * 8;
        ra0[u] = ra1[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (m < p.M) {
            ra0[u] = *(const float4 *)(p.A + (size_t)m * p.lda + k0);
            ra1[u] = *(const float4 *)(p.A + (size_t)m * p.lda + k0 + 4);
        }
        rwv[u] = make_uint2(0u, 0u);
        rwd[u] = 0.f;
        if (n < p.N) {
            rwv[u] = *(const uint2 *)(p.Wq + (size_t)n * p.K + k0);
            rwd[u] = __half2float(__ushort_as_half(p.Wd[(size_t)n * nblk + kb]));
        }
    };
#pragma unroll
    for (int u = 0; u < PF; ++u)
        if (u < bs) load(u, bbeg + u);
    for (int base = 0; base < bs; base += PF)
#pragma unroll
    for (int u = 0; u < PF; ++u) {
        const int step = base + u;
        if (step >= bs) break;
        {   // A rows -> Q8_0
            float a[8] = {ra0[u].x, ra0[u].y, ra0[u].z, ra0[u].w, ra1[u].x, ra1[u].y, ra1[u].z, ra1[u].w};
            float amax = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(a[e]));
            amax = fmaxf(amax, dpp_mov<0xB1>(amax));
            amax = fmaxf(amax, dpp_mov<0x4E>(amax));
            const float dd = amax / 127.0f;
            const float id = dd != 0.f ? 1.0f / dd : 0.0f;
            Aq[lr][2 * part] = pack_i8x4(roundf(a[0] * id), roundf(a[1] * id), roundf(a[2] * id), roundf(a[3] * id));
            Aq[lr][2 * part + 1] = pack_i8x4(roundf(a[4] * id), roundf(a[5] * id), roundf(a[6] * id), roundf(a[7] * id));
            if (part == 0) Ad[lr] = __half2float(__float2half(dd));
        }
        {   // W rows: int8 + block scale
            Wq[lr][2 * part] = (int)rwv[u].x;
            Wq[lr][2 * part + 1] = (int)rwv[u].y;
            if (part == 0) Wd[lr] = rwd[u];
        }
        if (step + PF < bs) load(u, bbeg + step + PF);
        __syncthreads();
        int s[4][4] = {};
#pragma unroll
        for (int w = 0; w < 8; ++w) {
            int av[4], wv[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) { av[i] = Aq[ty * 4 + i][w]; wv[i] = Wq[tx * 4 + i][w]; }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) s[i][j] = __builtin_amdgcn_sdot4(av[i], wv[j], s[i][j], false);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] += (float)s[i][j] * (Wd[tx * 4 + j] * Ad[ty * 4 + i]);
        __syncthreads();
    }
    gemm_store<EPI>(p, acc, m0 + ty * 4, n0 + tx * 4);
}

// Y[m] = LN(X[m]) * w for rows of width 768 (ggml_norm + ggml_mul): one 768-thread block per
// row, thread n element n; mean and variance in two passes (wave sums, the 12 wave partials
// added in wave order). ln_row768 is shared with gemm_reduce_ln_kernel, so a row normalised
// there or here (the large-grid GEMMs that reduce inside the workgroup) has the same bits.
constexpr int RLN_T = D;  // threads per row
__device__ __forceinline__ void ln_row768(float x, const float *w, float *y, float eps) {
    __shared__ float red[RLN_T / 64];
    const int n = threadIdx.x, lane = n & 63, wv = n >> 6;
    auto block_sum = [&](float v) {
        v = wave_sum(v);
        if (lane == 0) red[wv] = v;
        __syncthreads();
        float t = red[0];
#pragma unroll
        for (int i = 1; i < RLN_T / 64; ++i) t += red[i];
        __syncthreads();
        return t;
    };
    const float mean = block_sum(x) * (1.0f / D);
    const float d = x - mean;
    const float var = block_sum(d * d) * (1.0f / D);
    const float rstd = 1.0f / sqrtf(var + eps);
    y[n] = (d * rstd) * w[n];
}
__global__ __launch_bounds__(RLN_T) void ln_rows_kernel(const float *X, int ldx, const float *w, float *Y, int ldy,
                                                        float eps) {
    const int m = blockIdx.x;
    ln_row768(X[(size_t)m * ldx + threadIdx.x], w, Y + (size_t)m * ldy, eps);
}
// The same rows normalised with nw weight vectors at once (grid.y = g: w + g sw -> Y + g sy):
// the XA K/V precompute's LN(encoder output) with every layer's norm_xmem in one launch
__global__ __launch_bounds__(RLN_T) void ln_rows_multi_kernel(const float *X, int ldx, const float *w, long long sw,
                                                              float *Y, int ldy, long long sy, float eps) {
    const int m = blockIdx.x, g = blockIdx.y;
    ln_row768(X[(size_t)m * ldx + threadIdx.x], w + g * sw, Y + g * sy + (size_t)m * ldy, eps);
}

// Split-K reduction of a residual GEMM whose rows are normalised next (GemmP::ln_w, N = 768):
// one 768-thread workgroup per row, thread n: x = C + the splits summed in order
// (gemm_reduce_kernel<GE_RESID>'s arithmetic) stored to C, then ln_row768 (ln_rows_kernel's
// arithmetic) into ln_out. One launch where the preamble had two, with the reduce kernel's
// parallelism (one output per thread; round 6's first form, 3 outputs per thread of a
// 256-thread block, took 19 us per row block against 5 + 5 as two launches).
__global__ __launch_bounds__(RLN_T) void gemm_reduce_ln_kernel(GemmP p, int splits) {
    const int m = blockIdx.x, n = threadIdx.x;
    const size_t total = (size_t)p.M * p.N;
    const size_t e = (size_t)m * p.N + n;
    float a = p.part[e];
#pragma unroll 8
    for (int s = 1; s < splits; ++s) a += p.part[(size_t)s * total + e];
    if (p.bias) a += p.bias[n];
    const float x = a + p.C[(size_t)m * p.ldc + n];
    p.C[(size_t)m * p.ldc + n] = x;
    ln_row768(x, p.ln_w, p.ln_out + (size_t)m * p.ln_ld, p.ln_eps);
}

// Causal multi-head attention for every (row, head): one wave per pair.
// Keys for row (b, t) are rows j <= t of the same utterance, read through
// (kbase, vbase) + b * utt_stride + j * row_stride + h * 64.

template <bool KV16>
__global__ __launch_bounds__(256) void row_attn_kernel(RowAttnP p) {
    __shared__ float pr[4][TMAX_LIMIT];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int pair = blockIdx.x * 4 + w;
    if (pair >= p.M * p.heads) return;
    const int m = pair / p.heads, h = pair % p.heads;
    const int b = m / p.rows_per_utt, t = m % p.rows_per_utt;
    const int nk = t + 1;
    const float *q = p.Q + (size_t)m * p.ldq + h * DH;
    const size_t kb0 = b * p.utt_stride + h * DH;
    float mx = -INFINITY;
    for (int j = lane; j < nk; j += 64) {
        const size_t k = kb0 + (size_t)j * p.row_stride;
        float s = 0.f;
        for (int d = 0; d < DH; d += 4) s += dotv(*(const float4 *)(q + d), kv_load4<KV16>(p.Kb, k + d));
        s *= 0.125f;
        pr[w][j] = s;
        mx = fmaxf(mx, s);
    }
    mx = wave_max(mx);
    float l = 0.f;
    for (int j = lane; j < nk; j += 64) { const float e = expf(pr[w][j] - mx); pr[w][j] = e; l += e; }
    l = wave_sum(l);
    __builtin_amdgcn_wave_barrier();
    float o = 0.f;
    for (int j = 0; j < nk; ++j) {
        const size_t vi = kb0 + (size_t)j * p.row_stride + lane;
        o += pr[w][j] * (KV16 ? __uint_as_float((unsigned)((const unsigned short *)p.Vb)[vi] << 16) : p.Vb[vi]);
    }
    p.O[(size_t)m * D + h * DH + lane] = o / l;
}

// The same causal attention, one workgroup per (row, head), in the direct-form pattern of
// the decode's text attention (xa_text_attention, mp_xa.hpp): keys in rounds of 64, 4 lanes
// per key (16 dims each, one chain, the quad summed by DPP), every key's K row of a round
// issued at once, one exp per key by its own thread, the values summed by 4 waves (keys
// w, w + 4, ...; lane = dim) and the wave partials added in wave order. round 5's wave per
// (row, head) made a dependent memory round trip per key of its value loop.
template <bool KV16>
__global__ __launch_bounds__(MP_BLOCK) void row_attn_wg_kernel(RowAttnP p) {
    __shared__ float pr[TMAX_LIMIT];
    __shared__ float pv[MP_NWAVES][DH];
    __shared__ float wred[2 * MP_NWAVES];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int m = blockIdx.x, h = blockIdx.y;
    const int b = m / p.rows_per_utt, t = m % p.rows_per_utt;
    const int nk = t + 1;
    const size_t kb0 = b * p.utt_stride + h * DH;
    const int kq = 16 * w + (lane >> 2), dq = 16 * (lane & 3);
    float4 q4[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) q4[i] = *(const float4 *)(p.Q + (size_t)m * p.ldq + h * DH + dq + 4 * i);
    float mx = -INFINITY;
    for (int j0 = 0; j0 < nk; j0 += 64) {
        const int j = j0 + kq;
        const size_t k = kb0 + (size_t)min(j, nk - 1) * p.row_stride + dq;
        float4 k4[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) k4[i] = kv_load4<KV16>(p.Kb, k + 4 * i);
        float sv = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) sv += dotv(q4[i], k4[i]);
        sv += dpp_mov<0xB1>(sv);
        sv += dpp_mov<0x4E>(sv);
        sv *= 0.125f;
        if ((lane & 3) == 0 && j < nk) pr[j] = sv;
        mx = fmaxf(mx, j < nk ? sv : -INFINITY);
    }
    mx = wave_max(mx);
    if (lane == 0) wred[w] = mx;
    lds_sync();
    const float M = fmaxf(fmaxf(wred[0], wred[1]), fmaxf(wred[2], wred[3]));
    float l = 0.f;
    for (int j = tid; j < nk; j += MP_BLOCK) {
        const float e = expf(pr[j] - M);
        pr[j] = e;
        l += e;
    }
    l = wave_sum(l);
    if (lane == 0) wred[MP_NWAVES + w] = l;
    lds_sync();
    float o = 0.f;
    for (int j0 = w; j0 < nk; j0 += 4 * MP_NWAVES) {  // 4 keys' V rows in flight per wave
        float v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int j = min(j0 + MP_NWAVES * u, nk - 1);
            const size_t vi = kb0 + (size_t)j * p.row_stride + lane;
            v[u] = KV16 ? __uint_as_float((unsigned)((const unsigned short *)p.Vb)[vi] << 16) : p.Vb[vi];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int j = j0 + MP_NWAVES * u;
            o += (j < nk ? pr[min(j, nk - 1)] : 0.f) * v[u];
        }
    }
    pv[w][lane] = o;
    lds_sync();
    if (tid < DH) {
        const float den = ((wred[4] + wred[5]) + wred[6]) + wred[7];
        p.O[(size_t)m * D + h * DH + tid] = (((pv[0][tid] + pv[1][tid]) + pv[2][tid]) + pv[3][tid]) / den;
    }
}

// Cross-attention for a block of rows: 1 head x 128 over the utterance's T[b]
// text positions (no mask).

__global__ __launch_bounds__(256) void row_xa_kernel(RowXaP p) {
    __shared__ float pr[4][TMAX_LIMIT];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int m = blockIdx.x * 4 + w;
    if (m >= p.M) return;
    const int b = m / p.rows_per_utt, Tb = p.T[b];
    const float *q = p.Q + (size_t)m * DXA;
    const float *Kb = p.xak + ((size_t)(b * p.nlayers + p.layer) * p.Tmax) * DXA;
    const float *Vb = p.xav + ((size_t)(b * p.nlayers + p.layer) * p.Tmax) * DXA;
    const float scale = 1.0f / sqrtf((float)DXA);
    float mx = -INFINITY;
    for (int j = lane; j < Tb; j += 64) {
        float s = 0.f;
        for (int d = 0; d < DXA; d += 4) s += dotv(*(const float4 *)(q + d), *(const float4 *)(Kb + (size_t)j * DXA + d));
        s *= scale;
        pr[w][j] = s;
        mx = fmaxf(mx, s);
    }
    mx = wave_max(mx);
    float l = 0.f;
    for (int j = lane; j < Tb; j += 64) { const float e = expf(pr[w][j] - mx); pr[w][j] = e; l += e; }
    l = wave_sum(l);
    __builtin_amdgcn_wave_barrier();
    float o0 = 0.f, o1 = 0.f;
    for (int j0 = 0; j0 < Tb; j0 += 8) {  // 8 keys' V rows in flight, summed in key order
        float v0[8], v1[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int j = min(j0 + u, Tb - 1);
            v0[u] = Vb[(size_t)j * DXA + lane];
            v1[u] = Vb[(size_t)j * DXA + 64 + lane];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (j0 + u < Tb) {
                o0 += pr[w][j0 + u] * v0[u];
                o1 += pr[w][j0 + u] * v1[u];
            }
    }
    p.O[(size_t)m * DXA + lane] = o0 / l;
    p.O[(size_t)m * DXA + 64 + lane] = o1 / l;
}

// The same cross-attention, one workgroup per row, on the decode's direct-form text
// attention (xa_text_attention, mp_xa.hpp: 4 lanes per key, the first 64 keys' K and V
// rows issued at entry, one exp per key, wave partials summed in wave order): a row's
// attention is one memory round trip and a few DPP steps instead of a wave's serial
// key loop (13.3 us per prefill layer at T = 64 with a wave per row, round 5).
__global__ __launch_bounds__(MP_BLOCK) void row_xa_wg_kernel(RowXaP p) {
    __shared__ float pr[TMAX_LIMIT];
    __shared__ __attribute__((aligned(16))) float a_s[DXA];
    const int m = blockIdx.x;
    const int b = m / p.rows_per_utt;
    const size_t kv = ((size_t)(b * p.nlayers + p.layer) * p.Tmax) * DXA;
    xa_text_attention(p.Q + (size_t)m * DXA, p.xak + kv, p.xav + kv, p.T[b], pr, a_s);
    if (threadIdx.x < DXA) p.O[(size_t)m * DXA + threadIdx.x] = a_s[threadIdx.x];
}

// x[b][t] = text_emb[tok] + enc_pos[t] (t < T[b]), zero rows for padding.
__global__ void embed_text_kernel(const int *tok, const int *T, int Tmax, const float *text_emb,
                                  const float *enc_pos, float *X) {
    const int m = blockIdx.x, b = m / Tmax, t = m % Tmax;
    const bool valid = t < T[b];
    const int id = valid ? tok[m] : 0;
    for (int k = threadIdx.x; k < D; k += blockDim.x)
        X[(size_t)m * D + k] = valid ? text_emb[(size_t)id * D + k] + enc_pos[(size_t)t * D + k] : 0.f;
}

// x[b][t] = baked_context[spk_b][t] + dec_pos[t] for the 110 context frames (4138-4189).
__global__ void embed_context_kernel(const int *spk, const float *baked, const float *dec_pos, float *X) {
    const int m = blockIdx.x, b = m / CTX, t = m % CTX;
    const float *src = baked + (size_t)spk[b] * CTX * D + (size_t)t * D;
    for (int k = threadIdx.x; k < D; k += blockDim.x) X[(size_t)m * D + k] = src[k] + dec_pos[(size_t)t * D + k];
}

// LT table rows (see pre_lt_tab_rows): one 256-thread block per row, the
// block statistics PRO_LTARG_ATTN's per-wave statistics reproduce
__global__ __launch_bounds__(256) void lt_tab_rows_kernel(const float *P, const float *lt_pos, const float *w, float eps,
                                                          float *Y, int round) {
    __shared__ float red[8];
    const int r = blockIdx.x, k = threadIdx.x, cb = r / VCB + 1;
    const float X = P[(size_t)r * LTD + k] + lt_pos[(size_t)cb * LTD + k];
    const float xv[1] = {X};
    float mean, var;
    block_meanvar<1>(xv, red, mean, var);
    const float rstd = 1.0f / sqrtf(var + eps);
    float y = ((X - mean) * rstd) * w[k];
    if (round == 1) y = (float)(__bf16)y;
    else if (round == 2) y = (float)(_Float16)y;
    Y[(size_t)r * LTD + k] = y;
}
__global__ void round_bf16_kernel(const float *src, float *dst, size_t n) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        dst[i] = (float)(__bf16)src[i];
}

// ---------------------------------------------------------------- launchers
// MAGPIE_PRE_VALU=1 runs the preamble GEMMs on the f32 VALU kernel (A/B, and the test
// that both give the same bits; read at every launch, a few per preamble layer)
static bool gemm_mfma() {
    const char *e = getenv("MAGPIE_PRE_VALU");
    return !(e && *e == '1');
}
// GemmP::ln_w: the rows this GEMM completes are normalised next (LN(C) * ln_w -> ln_out):
// in the split reduction when there is one (gemm_reduce_ln_kernel), else as ln_rows_kernel
static hipError_t launch_ln_after(const GemmP &p, hipStream_t s) {
    if (!p.ln_w) return hipSuccess;
    hipLaunchKernelGGL(ln_rows_kernel, dim3(p.M), dim3(RLN_T), 0, s, p.C, p.ldc, p.ln_w, p.ln_out, p.ln_ld, p.ln_eps);
    return hipGetLastError();
}
template <int EPI>
static hipError_t launch_reduce(const GemmP &p, int splits, hipStream_t s) {
    if constexpr (EPI == GE_RESID) {
        if (p.ln_w && p.N == D) {
            hipLaunchKernelGGL(gemm_reduce_ln_kernel, dim3(p.M), dim3(RLN_T), 0, s, p, splits);
            return hipGetLastError();
        }
    }
    const size_t total = (size_t)p.M * p.N * (p.nbatch > 1 ? p.nbatch : 1);
    const int grid = (int)std::min<size_t>((total + 255) / 256, 4096);
    hipLaunchKernelGGL((gemm_reduce_kernel<EPI>), dim3(grid), dim3(256), 0, s, p, splits);
    if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
    return launch_ln_after(p, s);
}
template <int EPI, int TAPS>
static hipError_t launch_gemm(const GemmP &p, hipStream_t s) {
    const int splits = p.part ? gemm_splits(p.K) : 1;
    const int nb = p.nbatch > 1 ? p.nbatch : 1;
    if (p.K % (16 * splits) || (nb > 1 && p.ln_w)) return hipErrorInvalidValue;
    dim3 grid((p.N + 63) / 64, (p.M + 63) / 64, splits * nb);
    GemmP q = p;
    if (splits == 1) q.part = nullptr;
    const bool mfma = gemm_mfma();
    q.nsplit = splits;
    if (mfma && splits > 1 && grid.x * grid.y * nb >= PRE_INWG_TILES) {
        // enough output tiles to fill the chip: each workgroup runs its tile's splits in turn
        // (no partial sums through memory: 0.1-0.2 GB per GEMM at 16 utterances)
        grid.z = nb;
        q.part = nullptr;
        hipLaunchKernelGGL((gemm_f32_mfma_kernel<EPI, TAPS>), grid, dim3(256), 0, s, q);
        if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
        return launch_ln_after(p, s);
    }
    if (mfma) hipLaunchKernelGGL((gemm_f32_mfma_kernel<EPI, TAPS>), grid, dim3(256), 0, s, q);
    else hipLaunchKernelGGL((gemm_f32_kernel<EPI, TAPS>), grid, dim3(256), 0, s, q);
    if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
    if (splits == 1) return launch_ln_after(p, s);
    return launch_reduce<EPI>(p, splits, s);
}
template <int EPI>
static hipError_t launch_gemm_q8(const GemmP &p, hipStream_t s) {
    if (!p.Wd || p.K % 32 || p.conv_taps) return hipErrorInvalidValue;
    const int splits = p.part ? gemm_splits_q8(p.K) : 1;
    const int nb = p.nbatch > 1 ? p.nbatch : 1;
    if (nb > 1 && p.ln_w) return hipErrorInvalidValue;
    dim3 grid((p.N + 63) / 64, (p.M + 63) / 64, splits * nb);
    GemmP q = p;
    if (splits == 1) q.part = nullptr;
    hipLaunchKernelGGL((gemm_q8_kernel<EPI>), grid, dim3(256), 0, s, q);
    if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
    if (splits == 1) return launch_ln_after(p, s);
    return launch_reduce<EPI>(p, splits, s);
}
hipError_t pre_gemm(const GemmP &p, int epi, hipStream_t s) {
    if (p.Wq) {
        switch (epi) {
        case GE_STORE: return launch_gemm_q8<GE_STORE>(p, s);
        case GE_RESID: return launch_gemm_q8<GE_RESID>(p, s);
        case GE_QKV_CACHE: return launch_gemm_q8<GE_QKV_CACHE>(p, s);
        case GE_XAKV: return launch_gemm_q8<GE_XAKV>(p, s);
        }
        return hipErrorInvalidValue;
    }
    if (p.conv_taps == 3) {
        if (epi == GE_GELU) return launch_gemm<GE_GELU, 3>(p, s);
        if (epi == GE_RESID) return launch_gemm<GE_RESID, 3>(p, s);
        return hipErrorInvalidValue;
    }
    switch (epi) {
    case GE_STORE: return launch_gemm<GE_STORE, 0>(p, s);
    case GE_RESID: return launch_gemm<GE_RESID, 0>(p, s);
    case GE_GELU: return launch_gemm<GE_GELU, 0>(p, s);
    case GE_QKV_CACHE: return launch_gemm<GE_QKV_CACHE, 0>(p, s);
    case GE_XAKV: return launch_gemm<GE_XAKV, 0>(p, s);
    }
    return hipErrorInvalidValue;
}
hipError_t pre_ln_rows(const float *X, int ldx, const float *w, float *Y, int ldy, int M, float eps, hipStream_t s) {
    hipLaunchKernelGGL(ln_rows_kernel, dim3(M), dim3(RLN_T), 0, s, X, ldx, w, Y, ldy, eps);
    return hipGetLastError();
}
hipError_t pre_ln_rows_multi(const float *X, int ldx, const float *w, long long sw, float *Y, int ldy, long long sy,
                             int M, int nw, float eps, hipStream_t s) {
    hipLaunchKernelGGL(ln_rows_multi_kernel, dim3(M, nw), dim3(RLN_T), 0, s, X, ldx, w, sw, Y, ldy, sy, eps);
    return hipGetLastError();
}
hipError_t pre_lt_tab_rows(const float *P, const float *lt_pos, const float *w, float eps, float *Y, int round,
                           hipStream_t s) {
    hipLaunchKernelGGL(lt_tab_rows_kernel, dim3(7 * VCB), dim3(256), 0, s, P, lt_pos, w, eps, Y, round);
    return hipGetLastError();
}
hipError_t pre_round_bf16(const float *src, float *dst, size_t n, hipStream_t s) {
    hipLaunchKernelGGL(round_bf16_kernel, dim3((unsigned)std::min<size_t>((n + 255) / 256, 4096)), dim3(256), 0, s, src,
                       dst, n);
    return hipGetLastError();
}
hipError_t pre_row_attn(const RowAttnP &p, hipStream_t s) {
    static const bool old = getenv("MAGPIE_PRE_ROWATTN_OLD") != nullptr;  // A/B: a wave per (row, head)
    if (!old) {
        if (p.kv16) hipLaunchKernelGGL(row_attn_wg_kernel<true>, dim3(p.M, p.heads), dim3(MP_BLOCK), 0, s, p);
        else hipLaunchKernelGGL(row_attn_wg_kernel<false>, dim3(p.M, p.heads), dim3(MP_BLOCK), 0, s, p);
        return hipGetLastError();
    }
    if (p.kv16) hipLaunchKernelGGL(row_attn_kernel<true>, dim3((p.M * p.heads + 3) / 4), dim3(256), 0, s, p);
    else hipLaunchKernelGGL(row_attn_kernel<false>, dim3((p.M * p.heads + 3) / 4), dim3(256), 0, s, p);
    return hipGetLastError();
}
hipError_t pre_row_xa(const RowXaP &p, hipStream_t s) {
    static const bool old = getenv("MAGPIE_PRE_ROWXA_OLD") != nullptr;  // A/B: a wave per row (round 5)
    if (!old) {
        hipLaunchKernelGGL(row_xa_wg_kernel, dim3(p.M), dim3(MP_BLOCK), 0, s, p);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(row_xa_kernel, dim3((p.M + 3) / 4), dim3(256), 0, s, p);
    return hipGetLastError();
}
hipError_t pre_embed_text(const int *tok, const int *T, int B, int Tmax, const float *te, const float *ep, float *X,
                          hipStream_t s) {
    hipLaunchKernelGGL(embed_text_kernel, dim3(B * Tmax), dim3(256), 0, s, tok, T, Tmax, te, ep, X);
    return hipGetLastError();
}
hipError_t pre_embed_context(const int *spk, int B, const float *baked, const float *dp, float *X, hipStream_t s) {
    hipLaunchKernelGGL(embed_context_kernel, dim3(B * CTX), dim3(256), 0, s, spk, baked, dp, X);
    return hipGetLastError();
}

}  // namespace mp
