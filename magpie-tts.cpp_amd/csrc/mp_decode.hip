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
#include "mp_fused.hpp"
#include "mp_params.hpp"

namespace mp {

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
                       : (PRO == PRO_LTARG_LN) ? (NB < MP_NWAVES ? NB : MP_NWAVES) * 2 * VCB
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
    // acc[][] is wave-uniform: lane r*NB + b owns output (row0 + r, slot b), so the
    // epilogue (GELU, KV append, residual) runs on RW*NB lanes in parallel.
    static_assert(RW * NB <= 64, "one lane per output");
    float v = 0.f;
#pragma unroll
    for (int r = 0; r < RW; ++r)
#pragma unroll
        for (int b = 0; b < NB; ++b)
            if (lane == r * NB + b) v = acc[r][b];
    if (lane >= RW * NB) return;
    const int b = lane % NB, n = row0 + lane / NB;
    if (n >= p.N) return;
    epi_store<EPI>(p, v, n, b);
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
    if (p.mode == SA_PARTIALS) {  // plain stores; the combine is the next launch
        if (tid < DH) P[16 + tid] = (ow[tid] + ow[DH + tid]) + (ow[2 * DH + tid] + ow[3 * DH + tid]);
        else if (tid == 64) { P[0] = m; P[1] = l; }
        return;
    }
    if (tid < DH / 2) {
        const int d = 2 * tid;
        st_sc1(P + 16 + d, (ow[d] + ow[DH + d]) + (ow[2 * DH + d] + ow[3 * DH + d]),
               (ow[d + 1] + ow[DH + d + 1]) + (ow[2 * DH + d + 1] + ow[3 * DH + d + 1]));
    } else if (tid == 64) {
        st_sc1(P, m, l);
    }
    if (!arrive_last(p.cnt + b * NH + h, (unsigned)nact, sc + SA_CHUNK + MP_NWAVES * DH, p.mode == SA_COMBINE_SC1))
        return;
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
        i0 = wave_pick(p.logits + (size_t)b * VCB, p.ignore_eos || p.step[b] < 4, p.audio_bos, p.audio_eos, p.smp,
                       b, p.step[b], NCB - 1, scratch, amax);
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
    if (p.smp.amax) p.smp.amax[b * NCB + NCB - 1] = amax;
    // EOS if any codebook's sampled code or argmax is EOS (magpie.cpp:4340-4348)
    bool eos = amax == p.audio_eos;
    eos |= p.smp.argeos[b] != 0;
    p.smp.argeos[b] = 0;
    if (p.lt_only) return;  // magpie_local_transformer_sample_all: codes only
    for (int cb = 0; cb < NCB; ++cb) eos |= cc[cb] == p.audio_eos;
    const int s = p.step[b];
    if (eos) {
        // graph_reuse drops the EOS frame (4349-4352); the streaming loop emits it (4800-4806)
        if (p.emit_eos)
            for (int cb = 0; cb < NCB; ++cb) p.codes_out[((size_t)b * p.max_steps + s) * NCB + cb] = cc[cb];
        p.done[b] = 1;
        p.nframes[b] = p.emit_eos ? s + 1 : s;
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
// LT in_proj of a caller-supplied (already normalised) hidden vector, batch 1
// (magpie_local_transformer_sample_all, magpie.cpp:1161-1163)
hipError_t op_lt_inh_1(const GemvP &p, hipStream_t s) { return launch_gemv<1, 1, D, PRO_PLAIN, EPI_BIAS>(p, s); }
// bf16 weight mode at 16 slots: only the f32 LT in_proj runs on the GEMV family
hipError_t op_lt_in0_16(const GemvP &p, hipStream_t s) { return launch_gemv<16, 1, D, PRO_LN, EPI_BIAS>(p, s); }

// Combine of the SA_PARTIALS mode: one wave per (head, slot), the same arithmetic
// as the in-launch combiner (identical results in every mode).
__global__ __launch_bounds__(64) void sa_combine_kernel(AttnP p) {
    const int h = blockIdx.x, b = blockIdx.y, d = threadIdx.x;
    const int nact = (p.pos[b] + 1 + SA_CHUNK - 1) / SA_CHUNK;
    const float *Pb = p.part + (size_t)(b * NH + h) * p.nch * PART_STRIDE;
    float mv[NCH_MAX], lv[NCH_MAX], ov[NCH_MAX];
#pragma unroll
    for (int cc = 0; cc < NCH_MAX; ++cc) {
        const float *Pc = Pb + min(cc, nact - 1) * PART_STRIDE;
        mv[cc] = Pc[0];
        lv[cc] = Pc[1];
        ov[cc] = Pc[16 + d];
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
    p.out[(size_t)b * D + h * DH + d] = num / den;
}

hipError_t op_sa_combine(const AttnP &p, int B, hipStream_t s) {
    if (!p.part || !p.out || !p.pos || p.nch < 1 || p.nch > NCH_MAX) return hipErrorInvalidValue;
    hipLaunchKernelGGL(sa_combine_kernel, dim3(NH, B), dim3(64), 0, s, p);
    return hipGetLastError();
}

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
