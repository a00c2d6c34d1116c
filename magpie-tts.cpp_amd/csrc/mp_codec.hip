// Nano-codec decoder on gfx950 (magpie_codec_decode, nano-codec.cpp:758-845).
//
// codes [8][F] -> FSQ latent -> pre-conv 32->864 k7 -> 5 x (HalfSnake -> grouped
// convT up x{8,8,4,2,2} -> ResLayer = mean of 3 HiFiGAN blocks k{3,7,11} x
// dilations {1,3,5}) -> HalfSnake -> conv 27->1 k3 -> tanh   
//
// MI355X design:
//  * Every causal conv is an implicit GEMM on MFMA v_mfma_f32_16x16x32_f16:
//    M = out channels, N = time, K = taps x in channels. f16 operands with f32
//    accumulation is exactly ggml_conv_1d's semantics (F16 im2col + mul_mat,
//    A.7), so the MFMA path is the reference's numerics, not an approximation.
//  * Activations live in HBM as [chunk][time][channel] f32 (channel fastest,
//    channels zero-padded to a multiple of 32): a 32-channel K-block of one time
//    step is 64 contiguous bytes, so an input tile is staged once into LDS (with
//    its causal halo) as f16 and reused by all ks taps -> the B fragment of every
//    tap is one ds_read_b128.
//  * Each conv's input activation is produced ONCE, by the epilogue of the op
//    that writes its input: HalfSnake (nano-codec.cpp:376-426) with the
//    consumer's alpha, rounded to f16 exactly as ggml's F16 im2col rounds it, is
//    stored next to (or instead of) the f32 output, so a conv's operand loader is
//    a plain 16-byte f16 copy into LDS (no sinf per M-tile and per halo row). The
//    FSQ dequant (721-752) stays in the pre-conv's loader. Bias and the residual
//    add (568-599) are fused into the epilogue. The 3 HiFiGAN branches of a
//    ResLayer run in one launch (grid.z). The A fragments of all taps of a
//    32-channel block are issued before the block's input rows are staged.
//  * Weight-norm is already folded in the GGUF (convert_codec_to_gguf.py:169-221);
//    weights are re-laid out once at init as f16 [Cout_p][tap][Cin_p].
//  * The grouped ConvTranspose1d (481-565) is 4 MACs per output: an f32 kernel
//    (ggml's conv_transpose_1d with F32 weights is an f32 dot, A.7) with one
//    thread per (input step, group): the 3-branch ResLayer mean (619-641) and
//    HalfSnake of its 4 inputs are computed once and reused by its s outputs;
//    it emits the k=0 in_conv activations of the 3 branches.
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/magpie_hip.h"
#include "mp_device.hpp"
#include "mp_gguf.hpp"

namespace mpc {

constexpr int NSTAGE = 5;
constexpr int CH[6] = {864, 432, 216, 108, 54, 27};   // real channels (stage i input CH[i], output CH[i+1])
constexpr int CP[5] = {448, 224, 128, 64, 32};         // padded channels of stage i's output
constexpr int BMS[5] = {64, 32, 64, 64, 32};           // MFMA tile rows per stage
constexpr int CP_PRE = 896;                            // pre-conv output 864 padded
constexpr int RATE[5] = {8, 8, 4, 2, 2};
constexpr int KS[3] = {3, 7, 11};
constexpr int DIL[3] = {1, 3, 5};
constexpr int HOP = 1024;
// LDS bytes per time row of a 32-channel f16 operand block: 64 B of data + 16 B of pad.
// Measured and kept (round 5): a B fragment is one ds_read_b128 per lane at row base + l16,
// byte 16 kg; by the 16-lane groups gfx950 serves a ds_read_b128 in (MI355X_MICROARCH.md
// §LDS) an 80-byte row stride puts 3 lanes of each group on a taken bank quad and 96 bytes
// none, yet 96 made the codec slower (8 x 32 frames 1.620 -> 1.637 / 1.654 ms, rb_kernel at
// 64 channels 322 -> 345 us; gpurun_out/r05h_codec*.txt): the A-fragment stream and the
// workgroups per CU, not LDS reads, bound these kernels.
#ifndef MP_CODEC_ROWB
#define MP_CODEC_ROWB 80
#endif
constexpr int LDS_ROWB = MP_CODEC_ROWB;
// conv2_kernel pins each A-fragment ring load at its place in the tap loop (a scheduling
// barrier after it): left free, the scheduler sank the loads to just before their MFMAs
// (issue, then s_waitcnt vmcnt(1) four instructions later), exposing the L2 latency at
// every step. Measured (gpurun_out/r05q_*): the 448-channel stage's conv2_kernel 241 ->
// 180 us per decode. rb_kernel: its steps run as one flat (channel block, tap) sequence,
// each step's B fragments read one step ahead (across channel blocks too) and pinned
// before the step's MFMAs, the ring loads pinned after them (MP_RB_PIN 2): 8 x 32 frames
// 1.58 -> 1.48 ms (gpurun_out/r05ze_*; the ring loads alone, 1: 1.49; a 2-slot ring 1.53;
// a 4-slot one takes more than 128 VGPRs). Pinned per tap loop with the B reads fenced at
// every channel block's start, it had cost 5-7 %.
#ifndef MP_CONV2_PIN
#define MP_CONV2_PIN 1
#endif
#ifndef MP_RB_PIN
#define MP_RB_PIN 2
#endif
constexpr bool CONV2_PIN = MP_CONV2_PIN != 0;
constexpr int RB_PIN = MP_RB_PIN;  // 1: sched barrier after the ring loads, 2: and after the B loads

enum InMode { IN_F16 = 0, IN_FSQ = 1 };

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

struct ConvP {
    // per-branch (grid.z) operands
    const _Float16 *W[3];    // [Coutp][ks][Cinp] f16
    const _Float16 *Wf[3];   // the same in MFMA A-fragment order [Coutp/16][Cinp/32][ks][64 lanes][8] (conv2)
    const float *bias[3];    // [Coutp] (zero padded)
    const _Float16 *x[3];    // input activation, block-major [chunk][Cinp/32][T][32] f16 (already HalfSnake'd)
    float *out[3];           // optional f32 output [chunk][T][Coutp]
    const float *resid[3];   // optional residual [chunk][T][Coutp]
    _Float16 *act[3];        // optional f16 HalfSnake(output) for the next conv, block-major [chunk][Coutp/32][T][32]
    const float *act_alpha[3];
    int ks[3];
    const int *codes;        // IN_FSQ: [chunk][8][T]
    int act_nsnake, cout_real;
    int Cinp, Coutp, T, dil;
    int tiles_per_chunk;
    int zorder[3];           // conv2_kernel: branch of grid.z slice z (most taps first)
};

__device__ __forceinline__ float half_snake(float v, int c, int n_snake, int cin_real, const float *alpha) {
    // nano-codec.cpp:401-417 in ggml op order: mul, sin, sqr, div, add | leaky 0.01
    if (c < n_snake) {
        // hardware sin (v_sin_f32) and the hardware reciprocal (v_rcp_f32, 1 ulp) instead
        // of the libm sinf and an IEEE division (__fdividef compiles to the full
        // div_scale / div_fmas / div_fixup sequence here): ~1e-7 relative, far below the
        // f16 rounding every HalfSnake output gets next (the next conv's operand)
        const float a = alpha[c];
        const float s = __sinf(v * a);
        return v + (s * s) * __builtin_amdgcn_rcpf(a);
    }
    if (c < cin_real) return fmaxf(v, 0.01f * v);  // leaky 0.01: v > 0 ? v : 0.01 v
    return 0.f;
}

// half_snake with the channel's alpha already in a register, both forms computed
// and selected (no divergent branch; same arithmetic as half_snake)
__device__ __forceinline__ float half_snake_sel(float v, int c, int n_snake, int cin_real, float a) {
    const float s = __sinf(v * a);
    const float snake = v + (s * s) * __builtin_amdgcn_rcpf(a);  // 1 / a: loop-invariant per channel, hoisted
    const float leaky = fmaxf(v, 0.01f * v);
    return c < n_snake ? snake : (c < cin_real ? leaky : 0.f);
}

// The two HalfSnake forms apart (the same arithmetic as half_snake_sel's), for waves whose
// channels are all of one kind: HalfSnake's split (C / 2) is a multiple of 16 on every
// stage, so a wave's fragment or row piece is snake-only or leaky-only and computes one
// form instead of both (hs_wave_kind's vote; mixed or padded channels take the select)
__device__ __forceinline__ float hs_snake(float v, float a) {
    const float s = __sinf(v * a);
    return v + (s * s) * __builtin_amdgcn_rcpf(a);
}
__device__ __forceinline__ float hs_leaky(float v) { return fmaxf(v, 0.01f * v); }
// 0: every lane's channels [c0, c1] snake, 1: every lane's leaky, 2: otherwise
#ifndef MP_HS_SPLIT
#define MP_HS_SPLIT 1
#endif
__device__ __forceinline__ int hs_wave_kind(int c0, int c1, int n_snake, int cin_real) {
    if (!MP_HS_SPLIT) return 2;
    if (__all(c1 < n_snake)) return 0;
    if (__all(c0 >= n_snake && c1 < cin_real)) return 1;
    return 2;
}

// Residual convs (x' = x + conv(h) + b): the accumulators start at the residual x, the
// bias is added after the MFMAs -- (x + sum) + b in every kernel (conv_mfma_kernel,
// conv2_kernel, rb_kernel, which loads x as phase C frees the registers, under conv_1's
// MFMAs), the same bits across them; 0: (sum + b) + x, x loaded in the epilogue.
// Measured (gpurun_out/r05zs_*): 1.49-1.51 -> 1.42-1.43 ms per 8 x 32-frame decode.
#ifndef MP_RESINIT
#define MP_RESINIT 1
#endif
constexpr bool RESINIT = MP_RESINIT != 0;

// fsq_dequantize_cpu (nano-codec.cpp:721-752): channel c = 4*cb + d
__device__ __forceinline__ float fsq(int code, int d) {
    const int base = d == 0 ? 1 : d == 1 ? 8 : d == 2 ? 56 : 336;
    const int lev = d == 0 ? 8 : d == 1 ? 7 : 6;
    const int half = lev / 2;
    return (float)((code / base) % lev - half) / (float)half;
}

// Implicit-GEMM causal conv. Block tile BM (out ch) x BN (time), 4 waves.
constexpr int MAXTAPS = 11;
// PIPE: the software-pipelined channel loop (twice the registers: 2 waves/SIMD),
// for grids too small to hide latency by occupancy; same arithmetic either way.
template <int BM, int BN, int MODE, bool PIPE>
__global__ __launch_bounds__(256) void conv_mfma_kernel(ConvP p) {
    constexpr int RW = BM / 16;          // row blocks of 16
    constexpr int CWN = 4 / RW;          // column groups
    constexpr int WCOLS = BN / CWN;      // columns per wave
    constexpr int NT = WCOLS / 16;       // MFMA column tiles per wave
    constexpr int ROWB = LDS_ROWB;       // LDS bytes per time row: 32 halves + pad
    constexpr int MAXHALO = 50;          // (11 - 1) * 5
    __shared__ __attribute__((aligned(16))) char xs[PIPE ? 2 : 1][(BN + MAXHALO) * ROWB];

    const int br = blockIdx.z;
    const int ks = p.ks[br];
    const int pad = (ks - 1) * p.dil;
    const int m0 = blockIdx.x * BM;
    const int chunk = blockIdx.y / p.tiles_per_chunk;
    const int t0 = (blockIdx.y % p.tiles_per_chunk) * BN;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int rw = w % RW, cw = w / RW;
    const int kg = lane >> 4, l16 = lane & 15;
    const size_t chunk_in = (size_t)chunk * p.T * p.Cinp;
    const _Float16 *xin = p.x[br] + chunk_in;
    const _Float16 *W = p.W[br];
    const int Kw = ks * p.Cinp;
    const int orow = m0 + rw * 16 + l16;

    floatx4 acc[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
    if (RESINIT && p.resid[br]) {  // the accumulators start at the residual (MP_RESINIT)
        const int o = m0 + rw * 16 + 4 * kg;
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            const int t = t0 + cw * WCOLS + j * 16 + l16;
            if (t < p.T) {
                const float4 r = *(const float4 *)(p.resid[br] + (size_t)chunk * p.T * p.Coutp + (size_t)t * p.Coutp + o);
                acc[j] = floatx4{r.x, r.y, r.z, r.w};
            }
        }
    }

    const int rows = BN + pad;
    if constexpr (!PIPE) {
        // single-buffered: A fragments and input rows of a channel block issued
        // together, one wait, MFMAs; latency hidden by other resident workgroups
        for (int i0 = 0; i0 < p.Cinp; i0 += 32) {
            half8 af[MAXTAPS];
#pragma unroll
            for (int k = 0; k < MAXTAPS; ++k)
                if (k < ks) af[k] = *(const half8 *)(W + (size_t)orow * Kw + k * p.Cinp + i0 + 8 * kg);
            if constexpr (MODE == IN_FSQ) {
                for (int e = tid; e < rows * 8; e += 256) {
                    const int r = e >> 3, c4 = (e & 7) * 4;
                    const int t = t0 - pad + r;
                    _Float16 *dst = (_Float16 *)(xs[0] + r * ROWB) + c4;
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int c = i0 + c4 + u;
                        dst[u] = (t >= 0 && t < p.T)
                                     ? (_Float16)fsq(p.codes[((size_t)chunk * 8 + (c >> 2)) * p.T + t], c & 3)
                                     : (_Float16)0.f;
                    }
                }
            } else {
                for (int e = tid; e < rows * 4; e += 256) {
                    const int r = e >> 2, q = e & 3;
                    const int t = t0 - pad + r;
                    uint4 v = make_uint4(0u, 0u, 0u, 0u);
                    if (t >= 0 && t < p.T) v = *(const uint4 *)(xin + ((size_t)(i0 >> 5) * p.T + t) * 32 + 8 * q);
                    *(uint4 *)(xs[0] + r * ROWB + 16 * q) = v;
                }
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < MAXTAPS; ++k) {
                if (k < ks) {
#pragma unroll
                    for (int j = 0; j < NT; ++j) {
                        const int col = cw * WCOLS + j * 16 + l16;
                        const half8 b = *(const half8 *)(xs[0] + (col + k * p.dil) * ROWB + 16 * kg);
                        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[k], b, acc[j], 0, 0, 0);
                    }
                }
            }
            __syncthreads();
        }
    } else {
        static_assert(MODE == IN_F16, "pipelined loop: f16 inputs");
        // software pipeline over 32-channel blocks: block i+1's A fragments and input
        // rows are loaded into registers while block i's MFMAs run on the LDS buffer
        // filled last iteration (two LDS buffers, one barrier per block)
        constexpr int RPT = ((BN + MAXHALO) * 4 + 255) / 256;  // 16-byte row pieces per thread
        const int items = rows * 4;
        half8 an[MAXTAPS];
        uint4 xv[RPT];
        auto load_blk = [&](int i0) {
#pragma unroll
            for (int k = 0; k < MAXTAPS; ++k)
                if (k < ks) an[k] = *(const half8 *)(W + (size_t)orow * Kw + k * p.Cinp + i0 + 8 * kg);
#pragma unroll
            for (int u = 0; u < RPT; ++u) {
                const int e = tid + 256 * u;
                const int t = t0 - pad + (e >> 2);
                xv[u] = make_uint4(0u, 0u, 0u, 0u);
                if (e < items && t >= 0 && t < p.T) xv[u] = *(const uint4 *)(xin + ((size_t)(i0 >> 5) * p.T + t) * 32 + 8 * (e & 3));
            }
        };
        load_blk(0);
        int buf = 0;
        for (int i0 = 0; i0 < p.Cinp; i0 += 32) {
            half8 af[MAXTAPS];
#pragma unroll
            for (int k = 0; k < MAXTAPS; ++k) af[k] = an[k];
#pragma unroll
            for (int u = 0; u < RPT; ++u) {
                const int e = tid + 256 * u;
                if (e < items) *(uint4 *)(xs[buf] + (e >> 2) * ROWB + 16 * (e & 3)) = xv[u];
            }
            if (i0 + 32 < p.Cinp) load_blk(i0 + 32);
            __syncthreads();
#pragma unroll
            for (int k = 0; k < MAXTAPS; ++k) {
                if (k < ks) {
#pragma unroll
                    for (int j = 0; j < NT; ++j) {
                        const int col = cw * WCOLS + j * 16 + l16;
                        const half8 b = *(const half8 *)(xs[buf] + (col + k * p.dil) * ROWB + 16 * kg);
                        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[k], b, acc[j], 0, 0, 0);
                    }
                }
            }
            buf ^= 1;
        }
    }
    // ---- epilogue: C[row = 4*kg + r][col = l16] -> 4 consecutive channels of one time step
    const int o = m0 + rw * 16 + 4 * kg;
    const float4 bb = *(const float4 *)(p.bias[br] + o);
    const size_t chunk_out = (size_t)chunk * p.T * p.Coutp;
    const float *aal = p.act_alpha[br];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int t = t0 + cw * WCOLS + j * 16 + l16;
        if (t >= p.T) continue;
        float4 v = make_float4(acc[j][0] + bb.x, acc[j][1] + bb.y, acc[j][2] + bb.z, acc[j][3] + bb.w);
        const size_t off = chunk_out + (size_t)t * p.Coutp + o;
        if (!RESINIT && p.resid[br]) {
            const float4 r = *(const float4 *)(p.resid[br] + off);
            v.x = r.x + v.x; v.y = r.y + v.y; v.z = r.z + v.z; v.w = r.w + v.w;  // input + h (568-599)
        }
        if (p.out[br]) *(float4 *)(p.out[br] + off) = v;
        if (p.act[br]) {  // the next conv's operand: f16(HalfSnake(v)) (ggml F16 im2col)
            typedef _Float16 half4 __attribute__((ext_vector_type(4)));
            half4 h;
            h[0] = (_Float16)half_snake(v.x, o + 0, p.act_nsnake, p.cout_real, aal);
            h[1] = (_Float16)half_snake(v.y, o + 1, p.act_nsnake, p.cout_real, aal);
            h[2] = (_Float16)half_snake(v.z, o + 2, p.act_nsnake, p.cout_real, aal);
            h[3] = (_Float16)half_snake(v.w, o + 3, p.act_nsnake, p.cout_real, aal);
            *(half4 *)(p.act[br] + (size_t)chunk * p.T * p.Coutp + ((size_t)(o >> 5) * p.T + t) * 32 + (o & 31)) = h;
        }
    }
}

// Wide-tile implicit-GEMM causal conv for the ResLayer convs (f16 operands):
// RWV x CWV waves, each wave owns 32 output channels (2 A fragments) x 64 time
// steps (4 B fragments), so every B fragment read from LDS feeds 2 MFMAs and every
// A fragment 4. The tap count is a compile-time constant per branch (grid.z picks
// the instantiation), so the tap loop is straight-line code: the B fragments of
// tap k+1 are read while tap k's MFMAs run, and the A fragment of (block b, tap k)
// is re-loaded for block b+1 right after its last use (one register set, a whole
// block of lead time). Channel blocks are software-pipelined: block b+1's input
// rows go to registers during block b's MFMAs, two LDS buffers, one barrier per
// block. Accumulation order (block, tap ascending) equals conv_mfma_kernel's, so
// the two kernels give the same bits.
constexpr int C2_WR = 2, C2_NT = 4;
template <int KS, int RWV, int CWV, int NCB, int R>
__device__ __forceinline__ void conv2_body(const ConvP &p, char *xs) {
    constexpr int NTH = 64 * RWV * CWV;
    constexpr int BN = CWV * 16 * C2_NT;
    constexpr int ROWB = LDS_ROWB;       // LDS bytes per time row: 32 halves + pad
    constexpr int MAXHALO = 50;          // (11 - 1) * 5
    constexpr int BUFB = (BN + MAXHALO) * ROWB;
    constexpr int RPT = ((BN + MAXHALO) * 4 + NTH - 1) / NTH;  // 16-byte row pieces per thread
    const int br = p.zorder[blockIdx.z];
    const int dil = p.dil;
    const int pad = (KS - 1) * dil;
    const int m0 = blockIdx.x * (RWV * 32);
    const int chunk = blockIdx.y / p.tiles_per_chunk;
    const int t0 = (blockIdx.y % p.tiles_per_chunk) * BN;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int rw = w % RWV, cw = w / RWV;
    const int kg = lane >> 4, l16 = lane & 15;
    const _Float16 *xin = p.x[br] + (size_t)chunk * p.T * p.Cinp;
    // A fragment (16-row tile mt, channel block cb, tap k) = 1 KiB contiguous (Wf layout)
    const _Float16 *wrow0 = p.Wf[br] + (size_t)((m0 >> 4) + rw * 2) * NCB * KS * 512 + lane * 8;
    const _Float16 *wrow1 = wrow0 + (size_t)NCB * KS * 512;
    const int rows = BN + pad, items = rows * 4;

    floatx4 acc[C2_WR][C2_NT];
#pragma unroll
    for (int a = 0; a < C2_WR; ++a)
#pragma unroll
        for (int j = 0; j < C2_NT; ++j) acc[a][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    if (RESINIT && p.resid[br]) {  // the accumulators start at the residual (MP_RESINIT)
#pragma unroll
        for (int a = 0; a < C2_WR; ++a)
#pragma unroll
            for (int j = 0; j < C2_NT; ++j) {
                const int t = t0 + cw * (16 * C2_NT) + j * 16 + l16;
                if (t < p.T) {
                    const float4 r = *(const float4 *)(p.resid[br] + (size_t)chunk * p.T * p.Coutp + (size_t)t * p.Coutp +
                                                       m0 + rw * 32 + a * 16 + 4 * kg);
                    acc[a][j] = floatx4{r.x, r.y, r.z, r.w};
                }
            }
    }

    // A stream: step s = cb * KS + k (channel block, tap) is the 1 KiB fragment at
    // wrow + s * 512. The channel-block loop is unrolled (NCB is a template
    // argument), so the ring of R A-slots is indexed at compile time: step s + R is
    // loaded into slot s % R right after step s's MFMAs (R steps of lead; R >= KS
    // keeps every A wait behind loads issued before the next block's input rows,
    // vmcnt being in order), and the compiler counts vmcnt exactly.
    constexpr int NS = NCB * KS;
    half8 ring[R][C2_WR];
#pragma unroll
    for (int q = 0; q < R; ++q)
        if (q < NS) {
            ring[q][0] = *(const half8 *)(wrow0 + (size_t)q * 512);
            ring[q][1] = *(const half8 *)(wrow1 + (size_t)q * 512);
        }
    uint4 xv[RPT];
    auto load_x = [&](int cb) {
#pragma unroll
        for (int u = 0; u < RPT; ++u) {
            const int e = tid + NTH * u;
            const int t = t0 - pad + (e >> 2);
            xv[u] = make_uint4(0u, 0u, 0u, 0u);
            if (e < items && t >= 0 && t < p.T) xv[u] = *(const uint4 *)(xin + ((size_t)cb * p.T + t) * 32 + 8 * (e & 3));
        }
    };
    load_x(0);
    const int colb = cw * (16 * C2_NT) + l16;
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) {
        char *xb = xs + (cb & 1) * BUFB;
#pragma unroll
        for (int u = 0; u < RPT; ++u) {
            const int e = tid + NTH * u;
            if (e < items) *(uint4 *)(xb + (e >> 2) * ROWB + 16 * (e & 3)) = xv[u];
        }
        if (cb + 1 < NCB) load_x(cb + 1);
        __syncthreads();
        const char *bbase = xb + colb * ROWB + 16 * kg;
        half8 bc[C2_NT], bn[C2_NT];
#pragma unroll
        for (int j = 0; j < C2_NT; ++j) bc[j] = *(const half8 *)(bbase + j * 16 * ROWB);
#pragma unroll
        for (int k = 0; k < KS; ++k) {
            const int st = cb * KS + k;
            if (k + 1 < KS) {
#pragma unroll
                for (int j = 0; j < C2_NT; ++j) bn[j] = *(const half8 *)(bbase + (j * 16 + (k + 1) * dil) * ROWB);
            }
#pragma unroll
            for (int j = 0; j < C2_NT; ++j) {
                acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ring[st % R][0], bc[j], acc[0][j], 0, 0, 0);
                acc[1][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ring[st % R][1], bc[j], acc[1][j], 0, 0, 0);
            }
            if (st + R < NS) {
                ring[st % R][0] = *(const half8 *)(wrow0 + (size_t)(st + R) * 512);
                ring[st % R][1] = *(const half8 *)(wrow1 + (size_t)(st + R) * 512);
            }
            if constexpr (CONV2_PIN) __builtin_amdgcn_sched_barrier(0);  // the ring loads stay R steps ahead
            if (k + 1 < KS) {
#pragma unroll
                for (int j = 0; j < C2_NT; ++j) bc[j] = bn[j];
            }
        }
    }
    // ---- epilogue through LDS: the accumulator tile (C[row = 4*kg + r][col = l16] per
    // fragment) is written as [time][channel] f32, then every thread handles 4
    // consecutive channels of one time step in linear order, so bias / residual /
    // output / f16 operand accesses are contiguous rows (the whole [t0, t0 + BN) x
    // Coutp range when the tile spans every channel)
    constexpr int BM = RWV * 32, CST = BM + 4;  // +4 floats: row stride off the bank period
    float *ct = (float *)xs;
    __syncthreads();  // every wave is done with the input buffers
#pragma unroll
    for (int a = 0; a < C2_WR; ++a)
#pragma unroll
        for (int j = 0; j < C2_NT; ++j)
            *(floatx4 *)(ct + (colb + j * 16) * CST + rw * 32 + a * 16 + 4 * kg) = acc[a][j];
    __syncthreads();
    const size_t chunk_out = (size_t)chunk * p.T * p.Coutp;
    // NTH is a multiple of BM / 4: every thread keeps the same 4 channels for the
    // whole loop, so bias and HalfSnake alphas are loaded once (alpha arrays are
    // zero-padded to Coutp at load, the HalfSnake select is branch-free)
    static_assert(NTH % (BM / 4) == 0, "fixed channels per thread");
    const int cl = (tid % (BM / 4)) * 4, o = m0 + cl;
    const float4 bb = *(const float4 *)(p.bias[br] + o);
    float al[4] = {0.f, 0.f, 0.f, 0.f};
    if (p.act[br]) {
        const float4 a4 = *(const float4 *)(p.act_alpha[br] + o);
        al[0] = a4.x; al[1] = a4.y; al[2] = a4.z; al[3] = a4.w;
    }
    // the residual rows of every step this thread stores, loaded before the first store
    // (a load behind a store to another buffer waited one round trip per step)
    constexpr int RSTEP = NTH / (BM / 4), IT = BN / RSTEP;
    static_assert(BN % RSTEP == 0, "whole steps per thread");
    const int tl0 = tid / (BM / 4);
    float4 rres[IT];
    if (!RESINIT && p.resid[br]) {
#pragma unroll
        for (int i = 0; i < IT; ++i) {
            const int t = t0 + tl0 + i * RSTEP;
            rres[i] = t < p.T ? *(const float4 *)(p.resid[br] + chunk_out + (size_t)t * p.Coutp + o)
                              : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
#pragma unroll
    for (int i = 0; i < IT; ++i) {
        const int tl = tl0 + i * RSTEP;
        const int t = t0 + tl;
        if (t >= p.T) break;
        const float4 a4 = *(const float4 *)(ct + tl * CST + cl);
        float4 v = make_float4(a4.x + bb.x, a4.y + bb.y, a4.z + bb.z, a4.w + bb.w);
        const size_t off = chunk_out + (size_t)t * p.Coutp + o;
        if (!RESINIT && p.resid[br]) {
            const float4 r = rres[i];
            v.x = r.x + v.x; v.y = r.y + v.y; v.z = r.z + v.z; v.w = r.w + v.w;  // input + h (568-599)
        }
        if (p.out[br]) *(float4 *)(p.out[br] + off) = v;
        if (p.act[br]) {  // the next conv's operand: f16(HalfSnake(v)) (ggml F16 im2col), block-major
            typedef _Float16 half4 __attribute__((ext_vector_type(4)));
            half4 h;
            const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int u = 0; u < 4; ++u) h[u] = (_Float16)half_snake_sel(vv[u], o + u, p.act_nsnake, p.cout_real, al[u]);
            *(half4 *)(p.act[br] + chunk_out + ((size_t)(o >> 5) * p.T + t) * 32 + (o & 31)) = h;
        }
    }
}

// NCB = Cinp / 32 channel blocks (unrolled); DEEP: an A ring of max(KS, 6) slots
// (a block or more of lead, for grids of about one wave per SIMD whose weights come
// from the Infinity Cache) instead of 3 (occupancy-hidden latency, <= 128 VGPRs).
template <int RWV, int CWV, int NCB, bool DEEP>
__global__ __launch_bounds__(64 * RWV * CWV, DEEP ? 1 : 2) void conv2_kernel(ConvP p) {
    constexpr int BN = CWV * 16 * C2_NT;
    constexpr int XSB = 2 * (BN + 50) * LDS_ROWB, CTB = BN * (RWV * 32 + 4) * 4;  // input buffers / epilogue tile
    __shared__ __attribute__((aligned(16))) char xs[XSB > CTB ? XSB : CTB];
    switch (p.ks[p.zorder[blockIdx.z]]) {
        case 3: conv2_body<3, RWV, CWV, NCB, DEEP ? 6 : 3>(p, xs); break;
        case 7: conv2_body<7, RWV, CWV, NCB, DEEP ? 7 : 3>(p, xs); break;
        default: conv2_body<11, RWV, CWV, NCB, DEEP ? 11 : 3>(p, xs); break;
    }
}

// ---------------------------------------------------------------- fused residual block
// One HiFiGAN residual block of one branch (nano-codec.cpp:568-599) in one launch,
// for the stages of 224 / 128 / 64 / 32 padded channels (where the f32 residual
// stream and the f16 operands between the two convs were the traffic):
//   x' = x + conv_{KS,1}(HS_sk(conv_{KS,d}(HS_in(x)))).
// A workgroup owns output steps [t0, t0 + BN) of one chunk and every channel:
//  A. the x rows [t0 - 16 - (KS-1)d, t0 - 16 + 64 CWV) are read once (f32), HalfSnake'd
//     with the in_act alphas and rounded to f16 (ggml's F16 im2col) into LDS
//     [channel block][row][32 halves + 16 B pad];
//  B. conv_d over the 64 CWV columns [t0 - 16, t0 - 16 + 64 CWV): each wave owns 32
//     channels x 64 steps (conv2's wave tile, A fragments through a register ring);
//  C. bias + sk HalfSnake + f16 into LDS over the dead x rows (steps < 0 are zero:
//     conv_1's causal padding);
//  D. conv_1 (dilation 1) over [t0, t0 + BN), BN = 64 CWV - 16, then bias + x -> x'.
// The intermediate never leaves the CU; x is read once per block (not as an f32
// residual plus an f16 operand) and no f16 operand is written. Operand values,
// fragments and accumulation order (channel block, tap ascending) are conv2's: the
// same bits.
struct RbP {
    const float *x[3];              // residual stream in, [chunk][T][CP] f32 (block 0: the convT output)
    float *out[3];                  // residual stream out: another buffer (the next tile reads x's halo)
    const _Float16 *Wd[3], *W1[3];  // conv_d / conv_1 weights in A-fragment order (Conv::wf)
    const float *bd[3], *b1[3];     // biases, zero padded to CP
    const float *al_in[3], *al_sk[3];  // HalfSnake alphas, zero padded to CP
    int ks[3];
    int nsnake, creal, T, dil, tiles_per_chunk, nchunk;
    int ntiles;     // tiles per branch (nchunk x tiles_per_chunk)
    int order[3];   // item order: branch of items [k ntiles, (k + 1) ntiles), most taps first
    int *ctr;       // this launch's item counter (zeroed once per decode)
    unsigned long long *ts;  // diagnostics (MAGPIE_CODEC_TS): per workgroup RB_TS_N phase stamps, else null
};
constexpr int RB_ROWB = LDS_ROWB;  // LDS bytes per time row of a 32-channel block
constexpr int RB_TS_GX = 16384;    // diagnostics: stamp rows per branch (workgroups beyond: none)
constexpr int RB_TS_N = 48;        // diagnostics: stamps per workgroup (16 + 2 per wave)
// A-fragment ring slots of the residual-block convs (steps of lead for the weight loads)
#ifndef MP_RB_RING
#define MP_RB_RING 3
#endif
constexpr int RB_RING = MP_RB_RING;
// rb_kernel's work items: (branch, tile), heaviest branch (most taps) first, one workgroup
// per item in a 1-D grid. MP_RB_PERSIST=1: persistent workgroups taking items from a
// counter, the next item's x rows prefetched into registers during the current item's
// convolutions. Measured (gpurun_out/r05z_*, 8 x 32 frames): per-item with heaviest-first
// order 1.584-1.599 ms against 1.647-1.649 for the earlier branch-major 2-D grid
// (the 11-tap branch's workgroups no longer start last); persistent 1.91-1.92 ms -- the
// prefetched rows (48 VGPRs at 128 channels) halve the workgroups per CU. Off.
#ifndef MP_RB_PERSIST
#define MP_RB_PERSIST 0
#endif
constexpr bool RB_PERSIST = MP_RB_PERSIST != 0;
// rb_kernel's conv_d bias, HS_sk alpha and conv_1 bias staged in LDS with the x rows (1), or
// loaded from global memory where phases C / E use them (0)
#ifndef MP_RB_PRM
#define MP_RB_PRM 1
#endif
constexpr bool RB_PRM = MP_RB_PRM != 0;
// rb_kernel's residual rows (phase E) loaded before conv_1 (1) or after it (0)
#ifndef MP_RB_RXPRE
#define MP_RB_RXPRE 0
#endif
constexpr bool RB_RXPRE = MP_RB_RXPRE != 0;
constexpr bool RB_RESINIT = RESINIT;
constexpr int RB_MAXHALO = 50;  // (11 - 1) * 5

template <int RWV, int CWV, int NT>
constexpr int rb_lds_bytes() { return RWV * (16 * NT * CWV + RB_MAXHALO) * RB_ROWB; }
// + the staged parameters (RB_PRM): bd, al_sk, b1, CP floats each
template <int RWV, int CWV, int NT>
constexpr int rb_lds_total() { return rb_lds_bytes<RWV, CWV, NT>() + (RB_PRM ? 3 * RWV * 32 * 4 : 0); }

// Work items (branch, tile), heaviest branch first (RB_PERSIST above). With PERSIST the
// grid holds as many workgroups as the chip runs at once; workgroup g starts with item g,
// takes the next from a per-launch counter and loads its x rows into registers right after
// the current item's rows are staged (their HBM latency under the current item's convs:
// tools_dev/codec_rb_timeline.py shows ~6 us of rows per workgroup on every stage). Tiles
// and their arithmetic are the same in every form: the same bits.
template <int RWV, int CWV, int NT>
struct RbGeo {
    static constexpr int NCB = RWV, CPD = NCB * 32, NTH = 64 * RWV * CWV;
    static constexpr int NCD = 16 * NT * CWV;       // conv_d columns
    static constexpr int BN = NCD - 16;             // outputs per tile
    static constexpr int XR = NCD + RB_MAXHALO;     // LDS rows per channel block
    static constexpr int PPR = NCB * 4, RSTEP = NTH / PPR, NU = (XR + RSTEP - 1) / RSTEP;
    static_assert(NTH % PPR == 0, "fixed piece per thread");
    // the x-row pieces (8 channels) of a thread: with HALF, wave pair (2k, 2k + 1) holds
    // rows k 64 / PH ... of the low / high channel half, so a wave's pieces are all snake
    // or all leaky (hs_wave_kind); else thread t holds piece t % PPR of row t / PPR
    static constexpr int PH = PPR / 2;
    static constexpr bool HALF = PPR % 2 == 0 && 64 % PH == 0 && (NTH / 64) % 2 == 0;
    __device__ static int piece(int tid) { return HALF ? ((tid >> 6) & 1) * PH + (tid & 63) % PH : tid % PPR; }
    __device__ static int row0(int tid) { return HALF ? (tid >> 7) * (64 / PH) + (tid & 63) / PH : tid / PPR; }
};
// the x rows item `it` stages (thread: piece pc of rows r0 + u RSTEP), zero outside the chunk
template <int RWV, int CWV, int NT>
__device__ __forceinline__ void rb_load_rows(const RbP &p, int it, float4 (&v)[RbGeo<RWV, CWV, NT>::NU][2]) {
    using G = RbGeo<RWV, CWV, NT>;
    const int tid = threadIdx.x, pc = G::piece(tid), r0 = G::row0(tid);
    const int br = p.order[it / p.ntiles], tile = it % p.ntiles;
    const int halo = (p.ks[br] - 1) * p.dil, rows = G::NCD + halo;
    const int chunk = tile / p.tiles_per_chunk, t0 = (tile % p.tiles_per_chunk) * G::BN, tx0 = t0 - 16 - halo;
    const float *src = p.x[br] + (size_t)chunk * p.T * G::CPD + pc * 8;
#pragma unroll
    for (int u = 0; u < G::NU; ++u) {
        const int r = r0 + u * G::RSTEP, t = tx0 + r;
        v[u][0] = v[u][1] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (r < rows && t >= 0 && t < p.T) {
            v[u][0] = *(const float4 *)(src + (size_t)t * G::CPD);
            v[u][1] = *(const float4 *)(src + (size_t)t * G::CPD + 4);
        }
    }
}
// One item: branch br's tile `tile`, its rows in v. `next`: the item whose rows are loaded
// into v once this item's rows are staged (none if >= 3 ntiles).
template <int KS, int RWV, int CWV, int NT, int R, bool PERSIST>
__device__ __forceinline__ void rb_body(const RbP &p, char *xs, int br, int tile, int next,
                                        float4 (&v)[RbGeo<RWV, CWV, NT>::NU][2], bool first) {
    using G = RbGeo<RWV, CWV, NT>;
    constexpr int NCB = G::NCB, CPD = G::CPD, NCD = G::NCD, BN = G::BN, XR = G::XR, RSTEP = G::RSTEP, NU = G::NU;
    constexpr int NS = NCB * KS;  // A-stream steps (channel block, tap)
    // diagnostics: thread 0 stamps the phases of its first item (A x rows staged, B conv_d,
    // C the intermediate staged, D conv_1, E stored; wave 0's own: 9 conv_d done, 6 its part
    // of C computed, 7 its residual rows landed, 8 its stores done)
    unsigned long long *tsw = p.ts && first && blockIdx.x < RB_TS_GX ? p.ts + RB_TS_N * ((size_t)br * RB_TS_GX + blockIdx.x) : nullptr;
    auto stamp = [&](int k) {
        if (tsw && threadIdx.x == 0) tsw[k] = __builtin_amdgcn_s_memrealtime();
    };
    stamp(0);
    const int d = p.dil, halo = (KS - 1) * d;
    const int chunk = tile / p.tiles_per_chunk;
    const int t0 = (tile % p.tiles_per_chunk) * BN;
    const int tx0 = t0 - 16 - halo;           // time of x row 0 (conv_d column 0 is t0 - 16)
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int rw = w % RWV, cw = w / RWV;
    const int kg = lane >> 4, l16 = lane & 15;
    const size_t cbase = (size_t)chunk * p.T * CPD;

    // the staged parameters: [bd | al_sk | b1], CPD floats each, behind the row blocks
    float *prm = (float *)(xs + rb_lds_bytes<RWV, CWV, NT>());
    constexpr int NPRM = 3 * CPD / 4;  // float4 pieces
    static_assert(NPRM <= G::NTH, "one piece per thread");
    float4 pv = make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (RB_PRM) {
        if (tid < NPRM) {
            const int which = tid / (CPD / 4), o = (tid % (CPD / 4)) * 4;
            const float *src = which == 0 ? p.bd[br] : which == 1 ? p.al_sk[br] : p.b1[br];
            pv = *(const float4 *)(src + o);
        }
    }
    // ---- A: x rows -> HS_in -> f16 -> LDS (each thread keeps one 8-channel piece)
    {
        const int pc = G::piece(tid), c0 = pc * 8, r0 = G::row0(tid);
        float al[8];
        {
            const float4 a0 = *(const float4 *)(p.al_in[br] + c0), a1 = *(const float4 *)(p.al_in[br] + c0 + 4);
            al[0] = a0.x; al[1] = a0.y; al[2] = a0.z; al[3] = a0.w;
            al[4] = a1.x; al[5] = a1.y; al[6] = a1.z; al[7] = a1.w;
        }
        const int rows = NCD + halo;
        char *dst = xs + (pc >> 2) * XR * RB_ROWB + 16 * (pc & 3);
        auto stage_rows = [&](auto hs) {
#pragma unroll
            for (int u = 0; u < NU; ++u) {
                const int r = r0 + u * RSTEP, t = tx0 + r;
                if (r >= rows) break;
                const float vv[8] = {v[u][0].x, v[u][0].y, v[u][0].z, v[u][0].w, v[u][1].x, v[u][1].y, v[u][1].z, v[u][1].w};
                half8 h;
#pragma unroll
                for (int i = 0; i < 8; ++i) h[i] = (_Float16)hs(vv[i], i);
                if (t < 0 || t >= p.T) h = half8{0, 0, 0, 0, 0, 0, 0, 0};  // causal zero padding / past the chunk
                *(half8 *)(dst + r * RB_ROWB) = h;
            }
        };
        const int kind = hs_wave_kind(c0, c0 + 7, p.nsnake, p.creal);
        if (kind == 0) stage_rows([&](float x, int i) { return hs_snake(x, al[i]); });
        else if (kind == 1) stage_rows([&](float x, int) { return hs_leaky(x); });
        else stage_rows([&](float x, int i) { return half_snake_sel(x, c0 + i, p.nsnake, p.creal, al[i]); });
    }
    if constexpr (RB_PRM)
        if (tid < NPRM) *(float4 *)(prm + 4 * tid) = pv;
    // the next item's rows, in flight during this item's convolutions
    if constexpr (PERSIST)
        if (next < 3 * p.ntiles) rb_load_rows<RWV, CWV, NT>(p, next, v);
    __syncthreads();
    stamp(1);

    // ---- B / D: one causal conv from the LDS operand (rows: column c, tap k -> row
    // c * 1 + rowoff + k * dk), A stream from `wf` (conv2's ring), NT column tiles
    floatx4 acc[C2_WR][NT];
    half8 ring[R][C2_WR];
    const int colb = cw * 16 * NT + l16;
    auto conv = [&](const _Float16 *wf, int rowoff, int dk, int nt, bool init) {
        if (init) {
#pragma unroll
            for (int a = 0; a < C2_WR; ++a)
#pragma unroll
                for (int j = 0; j < NT; ++j) acc[a][j] = floatx4{0.f, 0.f, 0.f, 0.f};
        }
        const _Float16 *wrow0 = wf + (size_t)(rw * 2) * NS * 512 + lane * 8, *wrow1 = wrow0 + (size_t)NS * 512;
#pragma unroll
        for (int q = 0; q < R; ++q)
            if (q < NS) {
                ring[q][0] = *(const half8 *)(wrow0 + (size_t)q * 512);
                ring[q][1] = *(const half8 *)(wrow1 + (size_t)q * 512);
            }
        // B fragment j of step (cb, k): x / h rows colb + rowoff + 16 j + k dk of channel block cb
        const char *bbase = xs + (colb + rowoff) * RB_ROWB + 16 * kg;
        auto bfrag = [&](int st, int j) {
            return *(const half8 *)(bbase + (st / KS) * XR * RB_ROWB + (j * 16 + (st % KS) * dk) * RB_ROWB);
        };
        half8 bc[NT], bn[NT];
#pragma unroll
        for (int j = 0; j < NT; ++j) bc[j] = bfrag(0, j);
#pragma unroll
        for (int st = 0; st < NS; ++st) {
            if (st + 1 < NS) {  // the next step's B fragments (across channel blocks too)
#pragma unroll
                for (int j = 0; j < NT; ++j) bn[j] = bfrag(st + 1, j);
            }
            if constexpr (RB_PIN >= 2) __builtin_amdgcn_sched_barrier(0);  // ... issued before this step's MFMAs
#pragma unroll
            for (int j = 0; j < NT; ++j) {
                if (j < nt) {
                    acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ring[st % R][0], bc[j], acc[0][j], 0, 0, 0);
                    acc[1][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ring[st % R][1], bc[j], acc[1][j], 0, 0, 0);
                }
            }
            if (st + R < NS) {
                ring[st % R][0] = *(const half8 *)(wrow0 + (size_t)(st + R) * 512);
                ring[st % R][1] = *(const half8 *)(wrow1 + (size_t)(st + R) * 512);
            }
            if constexpr (RB_PIN >= 1) __builtin_amdgcn_sched_barrier(0);  // the ring loads stay R steps ahead
            if (st + 1 < NS) {
#pragma unroll
                for (int j = 0; j < NT; ++j) bc[j] = bn[j];
            }
        }
    };
    // B: conv_d, column c = time t0 - 16 + c, x row c + k d
    conv(p.Wd[br], 0, d, NT, true);
    // each lane's 8 channels: rw * 32 + a * 16 + 4 kg + r
    const int chl = rw * 32 + 4 * kg;
    stamp(9);
    if (tsw && lane == 0) tsw[16 + 2 * w] = __builtin_amdgcn_s_memrealtime();  // every wave's conv_d end
    __syncthreads();  // every wave is done reading x rows
    stamp(2);
    const int nt = cw == CWV - 1 ? NT - 1 : NT;  // conv_1: BN = 16 NT CWV - 16 outputs
    // ---- C: h = f16(HS_sk(conv_d + b)) into LDS rows 0 .. NCD-1 (row c = time t0 - 16 + c)
    {
        typedef _Float16 half4 __attribute__((ext_vector_type(4)));
        // the bias / alpha rows of both fragments first: one round trip, not one per fragment
        float4 bbs[C2_WR], als[C2_WR];
#pragma unroll
        for (int a = 0; a < C2_WR; ++a) {
            if constexpr (RB_PRM) {
                bbs[a] = *(const float4 *)(prm + chl + a * 16);
                als[a] = *(const float4 *)(prm + CPD + chl + a * 16);
            } else {
                bbs[a] = *(const float4 *)(p.bd[br] + chl + a * 16);
                als[a] = *(const float4 *)(p.al_sk[br] + chl + a * 16);
            }
        }
#pragma unroll
        for (int a = 0; a < C2_WR; ++a) {
            const int ch = chl + a * 16;
            const float4 bb = bbs[a], al = als[a];
            const float bv[4] = {bb.x, bb.y, bb.z, bb.w}, av[4] = {al.x, al.y, al.z, al.w};
            auto stage_frag = [&](auto hs) {
#pragma unroll
                for (int j = 0; j < NT; ++j) {
                    const int c = cw * 16 * NT + j * 16 + l16, t = t0 - 16 + c;
                    half4 h;
#pragma unroll
                    for (int r = 0; r < 4; ++r) h[r] = (_Float16)hs(acc[a][j][r] + bv[r], r);
                    if (t < 0) h = half4{0, 0, 0, 0};
                    *(half4 *)(xs + rw * XR * RB_ROWB + c * RB_ROWB + (a * 16 + 4 * kg) * 2) = h;
                    if constexpr (RB_RESINIT) {  // conv_1's accumulator starts at its residual rows
                        const int to = t0 + cw * 16 * NT + j * 16 + l16;
                        float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
                        if (j < nt && to < p.T) r = *(const float4 *)(p.x[br] + cbase + (size_t)to * CPD + chl + a * 16);
                        acc[a][j] = floatx4{r.x, r.y, r.z, r.w};
                    }
                }
            };
            const int kind = hs_wave_kind(ch, ch + 3, p.nsnake, p.creal);
            if (kind == 0) stage_frag([&](float x, int r) { return hs_snake(x, av[r]); });
            else if (kind == 1) stage_frag([&](float x, int) { return hs_leaky(x); });
            else stage_frag([&](float x, int r) { return half_snake_sel(x, ch + r, p.nsnake, p.creal, av[r]); });
        }
    }
    stamp(6);
    __syncthreads();
    stamp(3);
    // ---- D: conv_1, output column o = time t0 + o, h row o + 16 - (KS - 1) + k
    // ---- E's operands: every residual element and bias before the stores (a load after a
    // store to the other buffer may alias it, so per fragment the loop had waited one L2
    // round trip each); with RB_RXPRE before conv_1, their latency under its MFMAs
    float4 bb1[C2_WR], rx[C2_WR][NT];
    auto load_e = [&]() {
#pragma unroll
        for (int a = 0; a < C2_WR; ++a) {
            const int ch = chl + a * 16;
            bb1[a] = RB_PRM ? *(const float4 *)(prm + 2 * CPD + ch) : *(const float4 *)(p.b1[br] + ch);
#pragma unroll
            for (int j = 0; j < NT; ++j) {
                const int t = t0 + cw * 16 * NT + j * 16 + l16;
                rx[a][j] = make_float4(0.f, 0.f, 0.f, 0.f);
                if (!RB_RESINIT && j < nt && t < p.T) rx[a][j] = *(const float4 *)(p.x[br] + cbase + (size_t)t * CPD + ch);
            }
        }
    };
    if constexpr (RB_RXPRE) {
        load_e();
        __builtin_amdgcn_sched_barrier(0);  // issued here, not sunk to their use
    }
    conv(p.W1[br], 16 - (KS - 1), 1, nt, !RB_RESINIT);
    stamp(4);
    if (tsw && lane == 0) tsw[17 + 2 * w] = __builtin_amdgcn_s_memrealtime();  // every wave's conv_1 end
    // ---- E: + bias + x -> x'
    if constexpr (!RB_RXPRE) load_e();
    if (tsw) {  // diagnostics: wave 0's residual rows landed
        __builtin_amdgcn_s_waitcnt(0);
        stamp(7);
    }
#pragma unroll
    for (int a = 0; a < C2_WR; ++a) {
        const int ch = chl + a * 16;
        const float4 bb = bb1[a];
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            const int t = t0 + cw * 16 * NT + j * 16 + l16;
            if (j >= nt || t >= p.T) continue;
            const size_t off = cbase + (size_t)t * CPD + ch;
            const floatx4 y = acc[a][j];
            const float4 vo = make_float4(y[0] + bb.x, y[1] + bb.y, y[2] + bb.z, y[3] + bb.w);
            if constexpr (RB_RESINIT) {
                *(float4 *)(p.out[br] + off) = vo;  // (input + conv_1) + bias
                continue;
            }
            const float4 r = rx[a][j];
            *(float4 *)(p.out[br] + off) = make_float4(r.x + vo.x, r.y + vo.y, r.z + vo.z, r.w + vo.w);  // input + h
        }
    }
    if (tsw) {
        __builtin_amdgcn_s_waitcnt(0);
        stamp(8);
        __syncthreads();
        stamp(5);
    }
}

// PERSIST false: one item per workgroup (the grid covers every item), no prefetch -- for
// the 224-channel stage, whose 14-wave workgroups cannot hold a second tile's rows
// minimum waves per SIMD the register allocation must allow (launch bounds): MP_RB3_W /
// MP_RB4_W for the 64- / 32-channel stages' kernels (<2,4,4> / <1,8,2>), 0: the default
#ifndef MP_RB3_W
#define MP_RB3_W 0
#endif
#ifndef MP_RB4_W
#define MP_RB4_W 0
#endif
// per stage (224 / 128 / 64 / 32 channels): column waves (CWV) and 16-column fragments
// per wave (NT); a tile is 16 NT CWV - 16 outputs
#ifndef MP_RB1_CWV
#define MP_RB1_CWV 2
#endif
#ifndef MP_RB1_NT
#define MP_RB1_NT 4
#endif
#ifndef MP_RB2_CWV
#define MP_RB2_CWV 2
#endif
#ifndef MP_RB2_NT
#define MP_RB2_NT 4
#endif
#ifndef MP_RB3_CWV
#define MP_RB3_CWV 4
#endif
#ifndef MP_RB3_NT
#define MP_RB3_NT 4
#endif
#ifndef MP_RB4_CWV
#define MP_RB4_CWV 8
#endif
#ifndef MP_RB4_NT
#define MP_RB4_NT 2
#endif
#ifndef MP_RB1_W
#define MP_RB1_W 0
#endif
template <int RWV, int CWV, int NT>
constexpr int rb_minw() {
    if (RWV == 2 && CWV == 4 && NT == 4 && MP_RB3_W) return MP_RB3_W;
    if (RWV == 1 && CWV == 8 && NT == 2 && MP_RB4_W) return MP_RB4_W;
    if (RWV == 7 && MP_RB1_W) return MP_RB1_W;
    if (NT >= 8) return 2;  // <= 256 registers
    return RWV * CWV > 8 || NT > 4 ? 1 : 2;
}
template <int RWV, int CWV, int NT, bool PERSIST>
__global__ __launch_bounds__(64 * RWV * CWV, (rb_minw<RWV, CWV, NT>())) void rb_kernel(RbP p) {
    __shared__ __attribute__((aligned(16))) char xs[rb_lds_total<RWV, CWV, NT>()];
    __shared__ int sh_next;
    using G = RbGeo<RWV, CWV, NT>;
    const int total = 3 * p.ntiles;
    int it = blockIdx.x;
    if (it >= total) return;
    float4 v[G::NU][2];
    if constexpr (!PERSIST) {  // one item: its rows loaded and staged in one place
        const int br = p.order[it / p.ntiles], tile = it % p.ntiles;
        switch (p.ks[br]) {
            case 3: rb_load_rows<RWV, CWV, NT>(p, it, v); rb_body<3, RWV, CWV, NT, RB_RING, false>(p, xs, br, tile, total, v, true); break;
            case 7: rb_load_rows<RWV, CWV, NT>(p, it, v); rb_body<7, RWV, CWV, NT, RB_RING, false>(p, xs, br, tile, total, v, true); break;
            default: rb_load_rows<RWV, CWV, NT>(p, it, v); rb_body<11, RWV, CWV, NT, RB_RING, false>(p, xs, br, tile, total, v, true); break;
        }
        return;
    }
    rb_load_rows<RWV, CWV, NT>(p, it, v);
    for (bool first = true; it < total; first = false) {
        // the next item: from the per-launch counter (items below gridDim.x are the static
        // first ones); the previous item's barriers have retired every read of sh_next
        if (threadIdx.x == 0) sh_next = PERSIST ? (int)gridDim.x + atomicAdd(p.ctr, 1) : total;
        __syncthreads();  // sh_next published; the previous item's conv_1 is done with the LDS rows
        const int next = sh_next;
        const int br = p.order[it / p.ntiles], tile = it % p.ntiles;
        switch (p.ks[br]) {
            case 3: rb_body<3, RWV, CWV, NT, RB_RING, PERSIST>(p, xs, br, tile, next, v, first); break;
            case 7: rb_body<7, RWV, CWV, NT, RB_RING, PERSIST>(p, xs, br, tile, next, v, first); break;
            default: rb_body<11, RWV, CWV, NT, RB_RING, PERSIST>(p, xs, br, tile, next, v, first); break;
        }
        it = next;
    }
}

// ---- A whole ResLayer branch per item (rl_kernel, the 64- and 32-channel stages): the
// three residual blocks of one branch (dilations 1, 3, 5) over one time tile, x kept in
// registers between them. rb_kernel reads and writes every block's f32 residual stream
// (these stages' T is 131k-262k steps per 8 chunks: 100-200 MB per launch); here each tile
// reads x once and writes the layer's output once. A tile of W columns (column c = time
// ts + c) computes block b's outputs only where they are complete: a block's causal
// receptive field is (ks - 1)(d + 1) columns, so after block b the columns from H_b =
// (ks - 1) sum_{b' <= b} (d_b' + 1) on are exact and the tile outputs columns
// [12 (ks - 1), W) (fragments wholly left of what a block needs are skipped). Rows left of
// column 0 and times < 0 are zero, as every conv's causal padding is. Per time step the
// operands, A / B fragments, (channel block, tap) accumulation order and the (x + conv_1) + b
// epilogue are rb_kernel's: the same bits (tests/test_codec_gpu.py).
struct RlP {
    const float *x;                        // the ResLayer input (the convT output) [chunk][T][CP] f32
    float *out[3];                         // each branch's output
    const _Float16 *Wd[3][3], *W1[3][3];   // [branch][block] A-fragment order (Conv::wf)
    const float *bd[3][3], *b1[3][3], *al_in[3][3], *al_sk[3][3];
    int ks[3];
    int nsnake, creal, T;
    int bn[3], tpc[3];  // per branch: outputs per tile (W - 12 (ks - 1)), tiles per chunk
    int order[3];       // branches heaviest first: items [first[k], first[k + 1]) are branch order[k]
    int first[4];
};
constexpr int RL_HALO = RB_MAXHALO;  // zero rows left of column 0: conv_d's (ks - 1) d at most
#ifndef MP_RL_NT32
#define MP_RL_NT32 4  // 16-column fragments per wave, 32-channel stage
#endif
#ifndef MP_RL_NT64
#define MP_RL_NT64 4  // 64-channel stage (4 column waves)
#endif

template <int KS, int RWV, int CWV, int NT, int R>
__device__ __forceinline__ void rl_body(const RlP &p, char *xs, int br, int tile) {
    constexpr int NCB = RWV, CPD = NCB * 32, W = 16 * NT * CWV, XR = W + RL_HALO, NTH = 64 * RWV * CWV;
    constexpr int NS = NCB * KS;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int rw = w % RWV, cw = w / RWV;
    const int kg = lane >> 4, l16 = lane & 15;
    const int chunk = tile / p.tpc[br];
    const int ts = (tile % p.tpc[br]) * p.bn[br] - 12 * (KS - 1);  // time of column 0
    const size_t cbase = (size_t)chunk * p.T * CPD;
    const int chl = rw * 32 + 4 * kg;       // each lane's channels: chl + 16 a + r
    const int cwb = cw * 16 * NT;           // this wave's first column
    // x in the accumulator layout: fragment (a, j), lane: column cwb + 16 j + l16
    floatx4 xr[C2_WR][NT];
#pragma unroll
    for (int a = 0; a < C2_WR; ++a)
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            const int t = ts + cwb + 16 * j + l16;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (t >= 0 && t < p.T) v = *(const float4 *)(p.x + cbase + (size_t)t * CPD + chl + 16 * a);
            xr[a][j] = floatx4{v.x, v.y, v.z, v.w};
        }
    // the zero rows left of column 0, every channel block (never written after)
    constexpr int ZQ = RL_HALO * RB_ROWB / 16;
    for (int i = tid; i < NCB * ZQ; i += NTH)
        *(uint4 *)(xs + (size_t)(i / ZQ) * XR * RB_ROWB + (i % ZQ) * 16) = make_uint4(0, 0, 0, 0);
    // v -> HalfSnake(v [+ bias]) -> f16 -> LDS row HALO + c of this lane's channel block; 0 at t < 0
    auto put = [&](const floatx4 (&v)[C2_WR][NT], const float *alpha, const float *bias) {
        typedef _Float16 half4 __attribute__((ext_vector_type(4)));
        float4 als[C2_WR], bbs[C2_WR];
#pragma unroll
        for (int a = 0; a < C2_WR; ++a) {
            als[a] = *(const float4 *)(alpha + chl + a * 16);
            bbs[a] = bias ? *(const float4 *)(bias + chl + a * 16) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int a = 0; a < C2_WR; ++a) {
            const int ch = chl + a * 16;
            const float av[4] = {als[a].x, als[a].y, als[a].z, als[a].w};
            const float bv[4] = {bbs[a].x, bbs[a].y, bbs[a].z, bbs[a].w};
            auto frag = [&](auto hs) {
#pragma unroll
                for (int j = 0; j < NT; ++j) {
                    const int c = cwb + j * 16 + l16;
                    half4 h;
                    if (bias) {
#pragma unroll
                        for (int r = 0; r < 4; ++r) h[r] = (_Float16)hs(v[a][j][r] + bv[r], r);
                    } else {
#pragma unroll
                        for (int r = 0; r < 4; ++r) h[r] = (_Float16)hs(v[a][j][r], r);
                    }
                    if (ts + c < 0) h = half4{0, 0, 0, 0};
                    *(half4 *)(xs + rw * XR * RB_ROWB + (RL_HALO + c) * RB_ROWB + (a * 16 + 4 * kg) * 2) = h;
                }
            };
            const int kind = hs_wave_kind(ch, ch + 3, p.nsnake, p.creal);
            if (kind == 0) frag([&](float x, int r) { return hs_snake(x, av[r]); });
            else if (kind == 1) frag([&](float x, int) { return hs_leaky(x); });
            else frag([&](float x, int r) { return half_snake_sel(x, ch + r, p.nsnake, p.creal, av[r]); });
        }
    };
    // one causal conv from the LDS operand: column c, tap k reads row rowoff + c + k dk; the
    // fragments below jlo are skipped (wave-uniform)
    floatx4 acc[C2_WR][NT];
    half8 ring[R][C2_WR];
    auto conv = [&](const _Float16 *wf, int rowoff, int dk, int jlo) {
        const _Float16 *wrow0 = wf + (size_t)(rw * 2) * NS * 512 + lane * 8, *wrow1 = wrow0 + (size_t)NS * 512;
#pragma unroll
        for (int q = 0; q < R; ++q)
            if (q < NS) {
                ring[q][0] = *(const half8 *)(wrow0 + (size_t)q * 512);
                ring[q][1] = *(const half8 *)(wrow1 + (size_t)q * 512);
            }
        const char *bbase = xs + (cwb + l16 + rowoff) * RB_ROWB + 16 * kg;
        auto bfrag = [&](int st, int j) {
            return *(const half8 *)(bbase + (st / KS) * XR * RB_ROWB + (j * 16 + (st % KS) * dk) * RB_ROWB);
        };
        half8 bc[NT], bn[NT];
#pragma unroll
        for (int j = 0; j < NT; ++j) bc[j] = bfrag(0, j);
#pragma unroll
        for (int st = 0; st < NS; ++st) {
            if (st + 1 < NS) {
#pragma unroll
                for (int j = 0; j < NT; ++j) bn[j] = bfrag(st + 1, j);
            }
            if constexpr (RB_PIN >= 2) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < NT; ++j) {
                if (j >= jlo) {
                    acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ring[st % R][0], bc[j], acc[0][j], 0, 0, 0);
                    acc[1][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ring[st % R][1], bc[j], acc[1][j], 0, 0, 0);
                }
            }
            if (st + R < NS) {
                ring[st % R][0] = *(const half8 *)(wrow0 + (size_t)(st + R) * 512);
                ring[st % R][1] = *(const half8 *)(wrow1 + (size_t)(st + R) * 512);
            }
            if constexpr (RB_PIN >= 1) __builtin_amdgcn_sched_barrier(0);
            if (st + 1 < NS) {
#pragma unroll
                for (int j = 0; j < NT; ++j) bc[j] = bn[j];
            }
        }
    };
    // the first fragment of this wave holding a column >= need
    auto first_frag = [&](int need) { return need > cwb ? (need - cwb) >> 4 : 0; };
    int hdone = 0;  // columns from which the current x is exact
#pragma unroll 1
    for (int b = 0; b < 3; ++b) {
        const int d = DIL[b];
        put(xr, p.al_in[br][b], nullptr);  // HS_in(x)
        __syncthreads();
        // conv_d: column c = time ts + c, x row HALO + c - (KS - 1) d + k d
#pragma unroll
        for (int a = 0; a < C2_WR; ++a)
#pragma unroll
            for (int j = 0; j < NT; ++j) acc[a][j] = floatx4{0.f, 0.f, 0.f, 0.f};
        const int need_d = hdone + (KS - 1) * d, need_1 = need_d + (KS - 1);
        conv(p.Wd[br][b], RL_HALO - (KS - 1) * d, d, first_frag(need_d));
        __syncthreads();  // every wave is done reading the x rows
        put(acc, p.al_sk[br][b], p.bd[br][b]);  // h = HS_sk(conv_d + bd)
#pragma unroll
        for (int a = 0; a < C2_WR; ++a)
#pragma unroll
            for (int j = 0; j < NT; ++j) acc[a][j] = xr[a][j];  // conv_1's accumulator starts at x
        __syncthreads();
        conv(p.W1[br][b], RL_HALO - (KS - 1), 1, first_frag(need_1));
        {
            float4 bb[C2_WR];
#pragma unroll
            for (int a = 0; a < C2_WR; ++a) bb[a] = *(const float4 *)(p.b1[br][b] + chl + a * 16);
#pragma unroll
            for (int a = 0; a < C2_WR; ++a)
#pragma unroll
                for (int j = 0; j < NT; ++j)
                    xr[a][j] = floatx4{acc[a][j][0] + bb[a].x, acc[a][j][1] + bb[a].y, acc[a][j][2] + bb[a].z,
                                       acc[a][j][3] + bb[a].w};  // (x + conv_1) + b
        }
        hdone = need_1;
        if (b < 2) __syncthreads();  // conv_1's h reads done before the next HS_in rows
    }
    // the exact columns [12 (KS - 1), W) inside the chunk
#pragma unroll
    for (int a = 0; a < C2_WR; ++a)
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            const int c = cwb + 16 * j + l16, t = ts + c;
            if (c < hdone || t >= p.T) continue;
            *(float4 *)(p.out[br] + cbase + (size_t)t * CPD + chl + 16 * a) =
                make_float4(xr[a][j][0], xr[a][j][1], xr[a][j][2], xr[a][j][3]);
        }
}

#ifndef MP_RL_W32
#define MP_RL_W32 2  // minimum waves per SIMD the register allocation must allow, 32-channel stage
#endif
#ifndef MP_RL_W64
#define MP_RL_W64 2
#endif
#ifndef MP_RL_CWV32
#define MP_RL_CWV32 4  // column waves, 32-channel stage
#endif
#ifndef MP_RL_CWV64
#define MP_RL_CWV64 4  // column waves, 64-channel stage
#endif
template <int RWV, int CWV, int NT>
__global__ __launch_bounds__(64 * RWV * CWV, RWV == 1 ? MP_RL_W32 : MP_RL_W64) void rl_kernel(RlP p) {
    __shared__ __attribute__((aligned(16))) char xs[RWV * (16 * NT * CWV + RL_HALO) * RB_ROWB];
    const int it = blockIdx.x;
    if (it >= p.first[3]) return;
    const int k = it < p.first[1] ? 0 : it < p.first[2] ? 1 : 2;
    const int br = p.order[k], tile = it - p.first[k];
    switch (p.ks[br]) {
        case 3: rl_body<3, RWV, CWV, NT, RB_RING>(p, xs, br, tile); break;
        case 7: rl_body<7, RWV, CWV, NT, RB_RING>(p, xs, br, tile); break;
        default: rl_body<11, RWV, CWV, NT, RB_RING>(p, xs, br, tile); break;
    }
}

// Grouped ConvTranspose1d (nano-codec.cpp:481-565), HalfSnake on its input,
// optional 3-branch mean before it: out[t][g] = b[g] + sum_{c in {2g,2g+1}}
// sum_{tau: 0 <= t - tau*s < 2s} x[tau][c] * w[c][t - tau*s]; kept length T*s.
// input steps per thread of the later stages' ConvTranspose (each thread re-reads one step
// of halo: R = 8 reads 1.125x the input; 4: 1.25x, 1.45-1.47 vs 1.44-1.45 ms per decode)
#ifndef MP_CT_R
#define MP_CT_R 8
#endif
struct ConvTP {
    const float *x, *xa, *xb;  // input [chunk][Tin][Cinp] (xa/xb: AVG3)
    const float *alpha;
    int n_snake, cin_real, Cinp;
    const float *w;            // [Cin_real][2s] f32
    const float *bias;         // [Cout_real]
    float *out;                // [chunk][Tin*s][Coutp]
    _Float16 *act[3];          // f16 HalfSnake_{act_alpha[j]}(out): the k=0 in_conv operands
    const float *act_alpha[3];
    int cout_real, Coutp, Tin, s, nchunk;
};
// One thread per (chunk, input step tau, output group g): its outputs are
// t in [tau*s, tau*s + s), fed by inputs tau-1 and tau of channels 2g, 2g+1
// (the 3-branch mean and HalfSnake of those 4 values computed once).
template <bool AVG>
__global__ __launch_bounds__(256) void conv_transpose_kernel(ConvTP p) {
    const size_t total = (size_t)p.nchunk * p.Tin * p.Coutp;
    for (size_t e = (size_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (size_t)gridDim.x * 256) {
        const int g = (int)(e % p.Coutp);
        const size_t tt = e / p.Coutp;
        const int tau = (int)(tt % p.Tin), chunk = (int)(tt / p.Tin);
        const int K = 2 * p.s;
        float in[2][2] = {{0.f, 0.f}, {0.f, 0.f}};  // [tau-1, tau][channel 2g, 2g+1]
        if (g < p.cout_real) {
#pragma unroll
            for (int dt = 0; dt < 2; ++dt) {
                const int ta = tau - 1 + dt;
                if (ta < 0) continue;
#pragma unroll
                for (int ci = 0; ci < 2; ++ci) {
                    const int c = 2 * g + ci;
                    const size_t xo = ((size_t)chunk * p.Tin + ta) * p.Cinp + c;
                    float v = p.x[xo];
                    if constexpr (AVG) v = ((v + p.xa[xo]) + p.xb[xo]) * (1.0f / 3.0f);
                    in[dt][ci] = half_snake(v, c, p.n_snake, p.cin_real, p.alpha);
                }
            }
        }
        for (int u = 0; u < p.s; ++u) {
            const int t = tau * p.s + u;
            float acc = 0.f;
            if (g < p.cout_real) {
                // ggml order: channel c outer, tau = t/s - 1 then t/s inner
#pragma unroll
                for (int ci = 0; ci < 2; ++ci) {
                    const int c = 2 * g + ci;
                    if (tau >= 1) acc += in[0][ci] * p.w[(size_t)c * K + (t - (tau - 1) * p.s)];
                    acc += in[1][ci] * p.w[(size_t)c * K + (t - tau * p.s)];
                }
                acc += p.bias[g];
            }
            const size_t oo = ((size_t)chunk * p.Tin * p.s + t) * p.Coutp + g;
            p.out[oo] = acc;
            // the f16 operands block-major [chunk][Coutp/32][T][32]
            const size_t ob = (size_t)chunk * p.Tin * p.s * p.Coutp + ((size_t)(g >> 5) * p.Tin * p.s + t) * 32 + (g & 31);
#pragma unroll
            for (int j = 0; j < 3; ++j)
                p.act[j][ob] = (_Float16)half_snake(acc, g, p.cout_real / 2, p.cout_real, p.act_alpha[j]);
        }
    }
}

// The same grouped ConvTranspose1d with the shape compile-time per stage: one thread
// per (chunk, run of R input steps, output channel pair). The channel pair's 4
// input channels arrive as one float4 per branch and step (the previous step kept in
// registers), its 4 x 2s weights and all alphas stay in registers, outputs go out as
// float2 (f32) and half2 (block-major f16 operands). Same arithmetic and summation
// order as conv_transpose_kernel.
// ACT: also emit the 3 branches' k=0 in_conv operands (the stages whose residual
// blocks are fused compute them from the f32 output instead).
template <int CINP, int COUTP, int S, bool AVG, int R, bool ACT = true>
__global__ __launch_bounds__(256) void conv_transpose2_kernel(ConvTP p) {
    constexpr int NG = COUTP / 2, K = 2 * S;
    const int e = blockIdx.x * 256 + threadIdx.x;
    const int gp = e % NG, rest = e / NG;
    const int tiles = (p.Tin + R - 1) / R;
    const int tt = rest % tiles, chunk = rest / tiles;
    if (chunk >= p.nchunk) return;
    const int g = 2 * gp, c0 = 2 * g;  // outputs g, g + 1 <- inputs c0 .. c0 + 3
    const bool live0 = g < p.cout_real, live1 = g + 1 < p.cout_real;
    float w[4][K];
    float ia[4], bias0 = 0.f, bias1 = 0.f, oa[3][2];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int c = c0 + i;
        const bool lv = i < 2 ? live0 : live1;
#pragma unroll
        for (int k = 0; k < K; ++k) w[i][k] = lv ? p.w[(size_t)c * K + k] : 0.f;
        ia[i] = c < p.n_snake ? p.alpha[c] : 0.f;
    }
    if (live0) bias0 = p.bias[g];
    if (live1) bias1 = p.bias[g + 1];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        oa[j][0] = g < p.cout_real / 2 ? p.act_alpha[j][g] : 0.f;
        oa[j][1] = g + 1 < p.cout_real / 2 ? p.act_alpha[j][g + 1] : 0.f;
    }
    const int nsn = p.cout_real / 2;
    const size_t cin_base = (size_t)chunk * p.Tin * CINP;
    auto load_in = [&](int tau, float *v) {  // HalfSnake(mean of the branches) of inputs c0..c0+3 at step tau
        if (c0 >= CINP) {  // padded output pairs past the padded input (stage 2: 2 x 128 > 224)
            v[0] = v[1] = v[2] = v[3] = 0.f;
            return;
        }
        const size_t xo = cin_base + (size_t)tau * CINP + c0;
        float4 a = *(const float4 *)(p.x + xo);
        if constexpr (AVG) {
            const float4 b = *(const float4 *)(p.xa + xo), d = *(const float4 *)(p.xb + xo);
            a.x = ((a.x + b.x) + d.x) * (1.0f / 3.0f);
            a.y = ((a.y + b.y) + d.y) * (1.0f / 3.0f);
            a.z = ((a.z + b.z) + d.z) * (1.0f / 3.0f);
            a.w = ((a.w + b.w) + d.w) * (1.0f / 3.0f);
        }
        const float av[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = half_snake_sel(av[i], c0 + i, p.n_snake, p.cin_real, ia[i]);
    };
    const int tau0 = tt * R;
    float prev[4] = {0.f, 0.f, 0.f, 0.f}, cur[4];
    if (tau0 >= 1) load_in(tau0 - 1, prev);
    const int Tout = p.Tin * S;
    const size_t cout_base = (size_t)chunk * Tout * COUTP;
    const size_t act_base = cout_base + (size_t)(g >> 5) * Tout * 32 + (g & 31);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int tau = tau0 + r;
        if (tau >= p.Tin) break;
        load_in(tau, cur);
#pragma unroll
        for (int u = 0; u < S; ++u) {
            const int t = tau * S + u;
            float a0 = 0.f, a1 = 0.f;
            // ggml order: channel c outer, tau = t/s - 1 then t/s inner
#pragma unroll
            for (int ci = 0; ci < 2; ++ci) {
                if (tau >= 1) {
                    a0 = fmaf(prev[ci], w[ci][u + S], a0);
                    a1 = fmaf(prev[2 + ci], w[2 + ci][u + S], a1);
                }
                a0 = fmaf(cur[ci], w[ci][u], a0);
                a1 = fmaf(cur[2 + ci], w[2 + ci][u], a1);
            }
            if (live0) a0 += bias0;
            if (live1) a1 += bias1;
            *(float2 *)(p.out + cout_base + (size_t)t * COUTP + g) = make_float2(a0, a1);
            if constexpr (!ACT) continue;
            typedef _Float16 half2v __attribute__((ext_vector_type(2)));
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                half2v h;
                h[0] = (_Float16)half_snake_sel(a0, g, nsn, p.cout_real, oa[j][0]);
                h[1] = (_Float16)half_snake_sel(a1, g + 1, nsn, p.cout_real, oa[j][1]);
                *(half2v *)(p.act[j] + act_base + (size_t)t * 32) = h;
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) prev[i] = cur[i];
    }
}

// HalfSnake(post) -> causal conv 27->1 k3 (f16 operands, ggml_conv_1d) -> +b -> tanh
// (nano-codec.cpp:702-712) on the 3-branch mean of the last ResLayer.
struct PostP {
    const float *x, *xa, *xb;  // [chunk][T][32]
    const float *alpha;        // 13
    const float *w;            // [27][3] f32
    const float *bias;
    float *audio;              // [chunk][T]
    int T, nchunk;
};
// One workgroup = 256 consecutive output samples of one chunk. HalfSnake of the
// 3-branch mean is computed once per (time, channel) into LDS (with the 2-sample
// causal halo), rounded to f16 like ggml's im2col, then each thread dots its 3
// taps x 27 channels against the f16-rounded weights.
__global__ __launch_bounds__(256) void post_conv_kernel(PostP p) {
    __shared__ __attribute__((aligned(16))) float hs[258][28];
    __shared__ float wh[27 * 3];
    const int tiles = (p.T + 255) / 256;
    const int chunk = blockIdx.x / tiles, t0 = (blockIdx.x % tiles) * 256;
    const size_t cbase = (size_t)chunk * p.T;
    if (threadIdx.x < 81) wh[threadIdx.x] = (float)(_Float16)p.w[threadIdx.x];
    // channel quads: item e = (row e / 7, channels 4 (e % 7) ..): a float4 per branch, the
    // rows' 28 stored channels (27 real + 1 zero pad), 4 items per thread in flight
    constexpr int NQ = 7, NI = 258 * NQ;
#pragma unroll 4
    for (int e = threadIdx.x; e < NI; e += 256) {
        const int r = e / NQ, i0 = 4 * (e % NQ), t = t0 - 2 + r;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (t >= 0 && t < p.T) {
            const size_t o = (cbase + t) * 32 + i0;
            const float4 a = *(const float4 *)(p.x + o), b = *(const float4 *)(p.xa + o), d = *(const float4 *)(p.xb + o);
            const float m[4] = {((a.x + b.x) + d.x) * (1.0f / 3.0f), ((a.y + b.y) + d.y) * (1.0f / 3.0f),
                                ((a.z + b.z) + d.z) * (1.0f / 3.0f), ((a.w + b.w) + d.w) * (1.0f / 3.0f)};
            float hv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) hv[u] = i0 + u < 27 ? (float)(_Float16)half_snake(m[u], i0 + u, 13, 27, p.alpha) : 0.f;
            v = make_float4(hv[0], hv[1], hv[2], hv[3]);
        }
        *(float4 *)&hs[r][i0] = v;
    }
    __syncthreads();
    const int t = t0 + threadIdx.x;
    if (t >= p.T) return;
    float acc = 0.f;
    for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int i = 0; i < 27; ++i) acc = fmaf(hs[threadIdx.x + k][i], wh[i * 3 + k], acc);
    p.audio[cbase + t] = tanhf(acc + p.bias[0]);
}

}  // namespace mpc

// ====================================================================== runtime
struct mp_codec {
    int device = 0;
    std::string err;
    hipStream_t stream = nullptr;
    // weights
    struct Conv { _Float16 *w = nullptr, *wf = nullptr; float *b = nullptr; int ks = 0, cin = 0, cout = 0, cinp = 0, coutp = 0; };
    Conv pre, rb[5][3][3][2];  // [stage][kernel j][dilation k][in/skip]
    float *rb_alpha[5][3][3][2] = {};
    float *up_alpha[5] = {}, *up_w[5] = {}, *up_b[5] = {};
    float *post_alpha = nullptr, *post_w = nullptr, *post_b = nullptr;
    std::vector<void *> weight_allocs;
    // activations (grown on demand)
    size_t cap_elems = 0;
    float *x_pre = nullptr, *x0 = nullptr, *brb[3] = {}, *audio = nullptr;
    float *rbt[3] = {};  // fused residual blocks: block 1's output (block 2 reads its halo)
    _Float16 *a16[3] = {}, *b16[3] = {};  // f16 conv operands: in_conv (HS_in x), sk_conv (HS_sk h)
    int *codes = nullptr;
    size_t codes_cap = 0, audio_cap = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // background decodes (mp_codec_set_background): a second stream confined to a share of the
    // CUs (hipExtStreamCreateWithCUMask), for codec rounds that run beside a decode in flight
    hipStream_t bg_stream = nullptr;
    int bg = 0, bg_cus = 0;
    // pinned host staging of the codes in / audio out: a copy from or to pageable memory is
    // staged synchronously by the runtime and waited for the decode's queued work too
    // (configs[2]: each overlapped round's codec finished only after the decode's next chunk)
    int32_t *h_codes_pin = nullptr;
    float *h_audio_pin = nullptr;
    size_t h_codes_cap = 0, h_audio_cap = 0;
    float last_ms = 0.f;  // device time of the last decode (launch sequence only)
    int *rb_ctr = nullptr;  // rb_kernel's item counters, one per launch of a decode (zeroed per decode)
    // diagnostics (MAGPIE_CODEC_TS=stage,block,file): the phase stamps of one rb_kernel launch
    unsigned long long *ts_dev = nullptr;
    int ts_stage = -1, ts_block = -1;
    std::string ts_file;
};

namespace {

#define CHK(expr)                                                                                  \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess) {                                                                    \
            c->err = std::string(#expr) + " failed: " + hipGetErrorString(e_);                     \
            return MP_ERR_HIP;                                                                     \
        }                                                                                          \
    } while (0)

template <class T> int upload(mp_codec *c, T **dst, const std::vector<T> &h) {
    void *p = nullptr;
    CHK(hipMalloc(&p, h.size() * sizeof(T) + 64));
    CHK(hipMemcpy(p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
    c->weight_allocs.push_back(p);
    *dst = (T *)p;
    return MP_OK;
}

int load_f32(mp_codec *c, const mp::Gguf &g, const std::string &name, int64_t n, std::vector<float> &out) {
    const mp::GgufTensor *t = g.find(name);
    if (!t) { c->err = "missing codec tensor " + name; return MP_ERR_FORMAT; }
    if (n >= 0 && t->nelements() != n) { c->err = "unexpected shape for " + name; return MP_ERR_FORMAT; }
    out.resize((size_t)t->nelements());
    if (!g.to_f32(*t, out.data())) { c->err = "unsupported tensor type in " + name; return MP_ERR_FORMAT; }
    return MP_OK;
}

// conv weight [cout][cin][ks] (PyTorch) -> f16 [coutp][ks][cinp] zero padded
int load_conv(mp_codec *c, const mp::Gguf &g, const std::string &wname, const std::string &bname, int cout, int cin,
              int ks, int coutp, int cinp, mp_codec::Conv &cv) {
    std::vector<float> w, b;
    if (int rc = load_f32(c, g, wname, (int64_t)cout * cin * ks, w)) return rc;
    if (int rc = load_f32(c, g, bname, cout, b)) return rc;
    std::vector<_Float16> wi((size_t)coutp * ks * cinp, (_Float16)0.f);
    for (int o = 0; o < cout; ++o)
        for (int i = 0; i < cin; ++i)
            for (int k = 0; k < ks; ++k) wi[((size_t)o * ks + k) * cinp + i] = (_Float16)w[((size_t)o * cin + i) * ks + k];
    // MFMA A-fragment order for conv2: [coutp/16][cinp/32][ks][lane = 16*kg + l16][8]
    std::vector<_Float16> wf(wi.size());
    const int ncb = cinp / 32;
    for (int mt = 0; mt < coutp / 16; ++mt)
        for (int cb = 0; cb < ncb; ++cb)
            for (int k = 0; k < ks; ++k)
                for (int ln = 0; ln < 64; ++ln)
                    for (int e = 0; e < 8; ++e)
                        wf[((((size_t)mt * ncb + cb) * ks + k) * 64 + ln) * 8 + e] =
                            wi[((size_t)(mt * 16 + (ln & 15)) * ks + k) * cinp + cb * 32 + 8 * (ln >> 4) + e];
    if (int rc = upload(c, &cv.wf, wf)) return rc;
    b.resize(coutp, 0.f);
    cv.ks = ks; cv.cin = cin; cv.cout = cout; cv.cinp = cinp; cv.coutp = coutp;
    if (int rc = upload(c, &cv.w, wi)) return rc;
    return upload(c, &cv.b, b);
}

int load_codec(mp_codec *c, const char *path) {
    mp::Gguf g;
    std::string err;
    if (!g.open(path, err)) { c->err = err; return MP_ERR_IO; }
    if (g.get_u32("codec.num_codebooks", 8) != 8 || g.get_u32("codec.hop_length", 1024) != 1024 ||
        g.get_u32("codec.latent_dim", 32) != 32) {
        c->err = "codec hyperparameters differ from the nano-codec (kernels are specialised)";
        return MP_ERR_UNSUPPORTED;
    }
    using namespace mpc;
    if (int rc = load_conv(c, g, "dec.pre.weight", "dec.pre.bias", 864, 32, 7, CP_PRE, 32, c->pre)) return rc;
    std::vector<float> v;
    for (int i = 0; i < NSTAGE; ++i) {
        const int cin = CH[i], C = CH[i + 1];
        if (int rc = load_f32(c, g, "dec.act." + std::to_string(i) + ".activation.snake_act.alpha", cin / 2, v)) return rc;
        if (int rc = upload(c, &c->up_alpha[i], v)) return rc;
        if (int rc = load_f32(c, g, "dec.up." + std::to_string(i) + ".c.weight", (int64_t)cin * 2 * RATE[i], v)) return rc;
        if (int rc = upload(c, &c->up_w[i], v)) return rc;
        if (int rc = load_f32(c, g, "dec.up." + std::to_string(i) + ".c.bias", C, v)) return rc;
        if (int rc = upload(c, &c->up_b[i], v)) return rc;
        for (int j = 0; j < 3; ++j)
            for (int k = 0; k < 3; ++k) {
                const std::string p = "dec.rl." + std::to_string(i) + ".rb." + std::to_string(j) + ".rb." + std::to_string(k) + ".";
                // alphas zero-padded to the padded channel count (conv2's epilogue loads 4 at a time)
                if (int rc = load_f32(c, g, p + "in_act.alpha", C / 2, v)) return rc;
                v.resize(CP[i], 0.f);
                if (int rc = upload(c, &c->rb_alpha[i][j][k][0], v)) return rc;
                if (int rc = load_f32(c, g, p + "sk_act.alpha", C / 2, v)) return rc;
                v.resize(CP[i], 0.f);
                if (int rc = upload(c, &c->rb_alpha[i][j][k][1], v)) return rc;
                if (int rc = load_conv(c, g, p + "in_conv.weight", p + "in_conv.bias", C, C, KS[j], CP[i], CP[i], c->rb[i][j][k][0])) return rc;
                if (int rc = load_conv(c, g, p + "sk_conv.weight", p + "sk_conv.bias", C, C, KS[j], CP[i], CP[i], c->rb[i][j][k][1])) return rc;
            }
    }
    if (int rc = load_f32(c, g, "dec.post_act.alpha", 13, v)) return rc;
    if (int rc = upload(c, &c->post_alpha, v)) return rc;
    if (int rc = load_f32(c, g, "dec.post.weight", 27 * 3, v)) return rc;
    if (int rc = upload(c, &c->post_w, v)) return rc;
    if (int rc = load_f32(c, g, "dec.post.bias", 1, v)) return rc;
    return upload(c, &c->post_b, v);
}

int ensure_buffers(mp_codec *c, int nchunk, int F) {
    using namespace mpc;
    size_t need = 0;
    for (int i = 0; i < NSTAGE; ++i) {
        size_t T = (size_t)F;
        for (int s = 0; s <= i; ++s) T *= RATE[s];
        need = std::max(need, (size_t)nchunk * T * CP[i]);
    }
    need = std::max(need, (size_t)nchunk * F * CP_PRE);
    if (need > c->cap_elems) {
        float **bufs[8] = {&c->x_pre, &c->x0, &c->brb[0], &c->brb[1], &c->brb[2], &c->rbt[0], &c->rbt[1], &c->rbt[2]};
        for (auto b : bufs) if (*b) { hipFree(*b); *b = nullptr; }
        for (auto b : bufs) CHK(hipMalloc((void **)b, need * 4 + 256));
        _Float16 **hb[6] = {&c->a16[0], &c->a16[1], &c->a16[2], &c->b16[0], &c->b16[1], &c->b16[2]};
        for (auto b : hb) if (*b) { hipFree(*b); *b = nullptr; }
        for (auto b : hb) CHK(hipMalloc((void **)b, need * 2 + 256));
        c->cap_elems = need;
    }
    const size_t ncodes = (size_t)nchunk * 8 * F, naudio = (size_t)nchunk * F * HOP;
    if (ncodes > c->codes_cap) {
        if (c->codes) hipFree(c->codes);
        CHK(hipMalloc((void **)&c->codes, ncodes * 4));
        c->codes_cap = ncodes;
    }
    if (naudio > c->audio_cap) {
        if (c->audio) hipFree(c->audio);
        CHK(hipMalloc((void **)&c->audio, naudio * 4));
        c->audio_cap = naudio;
    }
    return MP_OK;
}

template <int BM, int BN, int MODE>
hipError_t launch_conv(const mpc::ConvP &p, int nchunk, int nbranch, hipStream_t s) {
    dim3 grid(p.Coutp / BM, nchunk * p.tiles_per_chunk, nbranch);
    // fewer workgroups than ~4 per CU cannot hide the channel loop's load latency by
    // occupancy: pipeline it instead (streaming chunks, the small early stages)
    const bool pipe = MODE == mpc::IN_F16 && (size_t)grid.x * grid.y * grid.z < 1024;
    if (pipe) hipLaunchKernelGGL((mpc::conv_mfma_kernel<BM, BN, mpc::IN_F16, true>), grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((mpc::conv_mfma_kernel<BM, BN, MODE, false>), grid, dim3(256), 0, s, p);
    return hipGetLastError();
}

template <int RWV, int CWV, int NCB, bool DEEP>
hipError_t launch_conv2(mpc::ConvP p, int nchunk, int nbranch, hipStream_t s) {
    constexpr int BN = CWV * 16 * mpc::C2_NT;
    if (p.Cinp != NCB * 32) return hipErrorInvalidValue;
    p.tiles_per_chunk = (p.T + BN - 1) / BN;
    // grid.z slices heaviest branch first (dispatched first)
    for (int j = 0; j < 3; ++j) p.zorder[j] = j;
    std::sort(p.zorder, p.zorder + nbranch, [&](int a, int b) { return p.ks[a] > p.ks[b]; });
    dim3 grid(p.Coutp / (RWV * 32), nchunk * p.tiles_per_chunk, nbranch);
    hipLaunchKernelGGL((mpc::conv2_kernel<RWV, CWV, NCB, DEEP>), grid, dim3(64 * RWV * CWV), 0, s, p);
    return hipGetLastError();
}

template <int RWV, int CWV, int NT = 4, bool PERSIST = mpc::RB_PERSIST>
hipError_t launch_rb(mpc::RbP p, int nchunk, hipStream_t s) {
    constexpr int BN = 16 * NT * CWV - 16;
    p.tiles_per_chunk = (p.T + BN - 1) / BN;
    p.nchunk = nchunk;
    p.ntiles = nchunk * p.tiles_per_chunk;
    // items heaviest first: the branches by tap count, descending
    for (int j = 0; j < 3; ++j) p.order[j] = j;
    std::sort(p.order, p.order + 3, [&](int a, int b) { return p.ks[a] > p.ks[b]; });
    const int total = 3 * p.ntiles;
    // persistent: as many workgroups as the chip runs at once (the kernel's occupancy
    // times the CU count), each taking items from the counter; else one per item
    int gx = total;
    if (PERSIST) {
        // cached per device (a process may drive devices of different CU counts)
        constexpr int MAXDEV = 64;
        static int per_cu_d[MAXDEV], ncu_d[MAXDEV];
        int dev = 0;
        hipGetDevice(&dev);
        int per_cu = 1, ncu = 1;
        if (dev >= 0 && dev < MAXDEV && per_cu_d[dev] > 0) {
            per_cu = per_cu_d[dev];
            ncu = ncu_d[dev];
        } else {
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, mpc::rb_kernel<RWV, CWV, NT, PERSIST>, 64 * RWV * CWV, 0) !=
                    hipSuccess || per_cu < 1)
                per_cu = 1;
            if (dev >= 0 && dev < MAXDEV) { ncu_d[dev] = ncu; per_cu_d[dev] = per_cu; }
        }
        gx = std::min(total, std::max(1, per_cu * ncu));
    }
    hipLaunchKernelGGL((mpc::rb_kernel<RWV, CWV, NT, PERSIST>), dim3(gx), dim3(64 * RWV * CWV), 0, s, p);
    return hipGetLastError();
}
// the fused residual block for a stage's padded channel count (0: not fused)
bool rb_fused(int Cp) {
    const char *unf = getenv("MAGPIE_CODEC_UNFUSED");
    const bool off = unf && atoi(unf) != 0;  // A/B switch (read per decode): the two-launch blocks
    return !off && (Cp == 224 || Cp == 128 || Cp == 64 || Cp == 32);
}
hipError_t run_rb(const mpc::RbP &p, int Cp, int nchunk, hipStream_t s) {
    // waves x steps per wave, measured per stage (8 x 32-frame chunks, same box): 64 steps
    // per wave everywhere but the 32-channel stage (32: 240 vs 273 us); 128 per wave took
    // 1.2-1.5x longer (one workgroup per CU), 32 per wave 1.3x on 128 / 64 channels
    switch (Cp) {
        case 224: return launch_rb<7, MP_RB1_CWV, MP_RB1_NT, false>(p, nchunk, s);
        case 128: return launch_rb<4, MP_RB2_CWV, MP_RB2_NT>(p, nchunk, s);
        case 64: return launch_rb<2, MP_RB3_CWV, MP_RB3_NT>(p, nchunk, s);
        case 32: return launch_rb<1, MP_RB4_CWV, MP_RB4_NT>(p, nchunk, s);
    }
    return hipErrorInvalidValue;
}

// one launch per ResLayer (rl_kernel) on the 32-channel stage; MAGPIE_CODEC_RL=0: rb_kernel's
// three launches there too, 2: rl_kernel on the 64-channel stage as well. Measured per stage
// (8 x 32 frames, gpurun_out/r06j_cprof*): 32 channels 232 us (rb, 3 launches) -> 193 us
// (rl, 4 waves x 64 columns) / 225-238 us (8 waves x 32 or 64 columns); 64 channels 274 us
// (rb) against 340-394 us (rl: 167 VGPRs, one 8-wave workgroup per CU).
bool rl_fused(int Cp) {
    const char *e = getenv("MAGPIE_CODEC_RL");
    const int mode = e ? atoi(e) : 1;
    return (Cp == 32 && mode >= 1) || (Cp == 64 && mode >= 2);
}
template <int RWV, int CWV, int NT>
hipError_t launch_rl(mpc::RlP p, int nchunk, hipStream_t s) {
    constexpr int W = 16 * NT * CWV;
    static_assert(W > 12 * 10, "a tile must be wider than the 11-tap branch's receptive field");
    for (int j = 0; j < 3; ++j) {
        p.bn[j] = W - 12 * (p.ks[j] - 1);
        p.tpc[j] = (p.T + p.bn[j] - 1) / p.bn[j];
        p.order[j] = j;
    }
    std::sort(p.order, p.order + 3, [&](int a, int b) { return p.ks[a] > p.ks[b]; });
    p.first[0] = 0;
    for (int k = 0; k < 3; ++k) p.first[k + 1] = p.first[k] + nchunk * p.tpc[p.order[k]];
    hipLaunchKernelGGL((mpc::rl_kernel<RWV, CWV, NT>), dim3(p.first[3]), dim3(64 * RWV * CWV), 0, s, p);
    return hipGetLastError();
}
hipError_t run_rl(const mpc::RlP &p, int Cp, int nchunk, hipStream_t s) {
    switch (Cp) {
        case 64: return launch_rl<2, MP_RL_CWV64, MP_RL_NT64>(p, nchunk, s);
        case 32: return launch_rl<1, MP_RL_CWV32, MP_RL_NT32>(p, nchunk, s);
    }
    return hipErrorInvalidValue;
}

hipError_t run_conv(const mpc::ConvP &p, int BM, int mode, int nchunk, int nbranch, hipStream_t s) {
    using namespace mpc;
    // ResLayer convs: the wide-tile kernel once a chunk fills at least half a tile
    // (per-chunk length decides, so a chunk decodes the same alone or batched)
    static const bool v1 = getenv("MAGPIE_CODEC_V1") != nullptr;  // A/B switch: the narrow-tile kernel only
    if (mode == IN_F16 && !v1) {
        switch (p.Coutp) {
            case 448: if (p.T >= 64) return launch_conv2<2, 2, 14, true>(p, nchunk, nbranch, s); break;
            case 224: if (p.T >= 128) return launch_conv2<1, 4, 7, true>(p, nchunk, nbranch, s); break;
            case 128: if (p.T >= 64) return launch_conv2<4, 2, 4, false>(p, nchunk, nbranch, s); break;
            case 64: if (p.T >= 128) return launch_conv2<2, 4, 2, false>(p, nchunk, nbranch, s); break;
            case 32: if (p.T >= 128) return launch_conv2<1, 4, 1, false>(p, nchunk, nbranch, s); break;
        }
    }
    if (BM == 64) {
        if (mode == IN_FSQ) return launch_conv<64, 64, IN_FSQ>(p, nchunk, nbranch, s);
        return launch_conv<64, 64, IN_F16>(p, nchunk, nbranch, s);
    }
    return launch_conv<32, 128, IN_F16>(p, nchunk, nbranch, s);
}

// Decode nchunk independent chunks of F frames each (codes [chunk][8][F]).
int codec_run(mp_codec *c, int nchunk, int F) {
    using namespace mpc;
    hipStream_t s = c->stream;
    constexpr size_t NCTR = (size_t)NSTAGE * 3 * 16;
    if (!c->rb_ctr) CHK(hipMalloc((void **)&c->rb_ctr, NCTR * sizeof(int)));
    CHK(hipMemsetAsync(c->rb_ctr, 0, NCTR * sizeof(int), s));
    // pre-conv with the FSQ dequant in its loader
    {
        ConvP p{};
        p.W[0] = c->pre.w; p.bias[0] = c->pre.b; p.x[0] = nullptr; p.out[0] = c->x_pre;
        p.resid[0] = nullptr; p.act[0] = nullptr; p.ks[0] = 7; p.codes = c->codes; p.cout_real = 864;
        p.Cinp = 32; p.Coutp = CP_PRE; p.T = F; p.dil = 1; p.tiles_per_chunk = (F + 63) / 64;
        CHK(run_conv(p, 64, IN_FSQ, nchunk, 1, s));
    }
    int T = F;
    for (int i = 0; i < NSTAGE; ++i) {
        const int cin = CH[i], C = CH[i + 1], Cin_p = i == 0 ? CP_PRE : CP[i - 1], Cp = CP[i];
        // HalfSnake -> grouped convT (input: pre-conv, or mean of the previous ResLayer's
        // branches); emits x0 and the 3 branches' first in_conv operands HS_in(x0)
        ConvTP tp{};
        tp.x = i == 0 ? c->x_pre : c->brb[0];
        tp.xa = c->brb[1]; tp.xb = c->brb[2];
        tp.alpha = c->up_alpha[i]; tp.n_snake = cin / 2; tp.cin_real = cin; tp.Cinp = Cin_p;
        tp.w = c->up_w[i]; tp.bias = c->up_b[i]; tp.out = c->x0; tp.cout_real = C; tp.Coutp = Cp;
        for (int j = 0; j < 3; ++j) { tp.act[j] = c->a16[j]; tp.act_alpha[j] = c->rb_alpha[i][j][0][0]; }
        tp.Tin = T; tp.s = RATE[i]; tp.nchunk = nchunk;
        // R input steps per thread: 1 on the short early stages (threads), 4 later (re-reads)
        const int R = i == 0 ? 1 : i == 1 ? 2 : MP_CT_R;
        const dim3 g2((nchunk * ((T + R - 1) / R) * (Cp / 2) + 255) / 256);
        const bool fused = rb_fused(Cp);
        switch (i) {
            case 0: hipLaunchKernelGGL((conv_transpose2_kernel<896, 448, 8, false, 1>), g2, dim3(256), 0, s, tp); break;
            case 1:
                if (fused) hipLaunchKernelGGL((conv_transpose2_kernel<448, 224, 8, true, 2, false>), g2, dim3(256), 0, s, tp);
                else hipLaunchKernelGGL((conv_transpose2_kernel<448, 224, 8, true, 2>), g2, dim3(256), 0, s, tp);
                break;
            case 2:
                if (fused) hipLaunchKernelGGL((conv_transpose2_kernel<224, 128, 4, true, MP_CT_R, false>), g2, dim3(256), 0, s, tp);
                else hipLaunchKernelGGL((conv_transpose2_kernel<224, 128, 4, true, MP_CT_R>), g2, dim3(256), 0, s, tp);
                break;
            case 3:
                if (fused) hipLaunchKernelGGL((conv_transpose2_kernel<128, 64, 2, true, MP_CT_R, false>), g2, dim3(256), 0, s, tp);
                else hipLaunchKernelGGL((conv_transpose2_kernel<128, 64, 2, true, MP_CT_R>), g2, dim3(256), 0, s, tp);
                break;
            default:
                if (fused) hipLaunchKernelGGL((conv_transpose2_kernel<64, 32, 2, true, MP_CT_R, false>), g2, dim3(256), 0, s, tp);
                else hipLaunchKernelGGL((conv_transpose2_kernel<64, 32, 2, true, MP_CT_R>), g2, dim3(256), 0, s, tp);
                break;
        }
        CHK(hipGetLastError());
        T *= RATE[i];
        if (fused && rl_fused(Cp)) {
            RlP lp{};
            lp.x = c->x0;
            for (int j = 0; j < 3; ++j) {
                lp.out[j] = c->brb[j];
                lp.ks[j] = KS[j];
                for (int k = 0; k < 3; ++k) {
                    const mp_codec::Conv &cd = c->rb[i][j][k][0], &c1 = c->rb[i][j][k][1];
                    lp.Wd[j][k] = cd.wf; lp.W1[j][k] = c1.wf; lp.bd[j][k] = cd.b; lp.b1[j][k] = c1.b;
                    lp.al_in[j][k] = c->rb_alpha[i][j][k][0]; lp.al_sk[j][k] = c->rb_alpha[i][j][k][1];
                }
            }
            lp.nsnake = C / 2; lp.creal = C; lp.T = T;
            CHK(run_rl(lp, Cp, nchunk, s));
            continue;
        }
        if (fused) {
            // x0 -> brb (block 0) -> rbt (block 1) -> brb (block 2): out of place, since a
            // tile reads its left neighbour's rows as halo
            for (int k = 0; k < 3; ++k) {
                RbP rp{};
                for (int j = 0; j < 3; ++j) {
                    const mp_codec::Conv &cd = c->rb[i][j][k][0], &c1 = c->rb[i][j][k][1];
                    rp.x[j] = k == 0 ? c->x0 : k == 1 ? c->brb[j] : c->rbt[j];
                    rp.out[j] = k == 1 ? c->rbt[j] : c->brb[j];
                    rp.Wd[j] = cd.wf; rp.W1[j] = c1.wf; rp.bd[j] = cd.b; rp.b1[j] = c1.b;
                    rp.al_in[j] = c->rb_alpha[i][j][k][0]; rp.al_sk[j] = c->rb_alpha[i][j][k][1];
                    rp.ks[j] = KS[j];
                }
                rp.nsnake = C / 2; rp.creal = C; rp.T = T; rp.dil = DIL[k];
                rp.ts = (c->ts_dev && i == c->ts_stage && k == c->ts_block) ? c->ts_dev : nullptr;
                rp.ctr = c->rb_ctr + (i * 3 + k) * 16;  // 64 B apart
                CHK(run_rb(rp, Cp, nchunk, s));
            }
            continue;
        }
        const int BM = BMS[i], BN = BM == 64 ? 64 : 128;
        for (int k = 0; k < 3; ++k) {
            // h = conv_{ks_j, d_k}(HS_in(x)) for the 3 branches j; only HS_sk(h) (f16) is kept
            ConvP p{};
            for (int j = 0; j < 3; ++j) {
                const mp_codec::Conv &cv = c->rb[i][j][k][0];
                p.W[j] = cv.w; p.Wf[j] = cv.wf; p.bias[j] = cv.b; p.x[j] = c->a16[j]; p.out[j] = nullptr; p.resid[j] = nullptr;
                p.act[j] = c->b16[j]; p.act_alpha[j] = c->rb_alpha[i][j][k][1]; p.ks[j] = KS[j];
            }
            p.act_nsnake = C / 2; p.cout_real = C; p.Cinp = Cp; p.Coutp = Cp; p.T = T; p.dil = DIL[k];
            p.tiles_per_chunk = (T + BN - 1) / BN;
            CHK(run_conv(p, BM, IN_F16, nchunk, 3, s));
            // x' = x + conv_{ks_j, 1}(HS_sk(h)); plus the next block's operand HS_in(x')
            for (int j = 0; j < 3; ++j) {
                const mp_codec::Conv &cv = c->rb[i][j][k][1];
                p.W[j] = cv.w; p.Wf[j] = cv.wf; p.bias[j] = cv.b; p.x[j] = c->b16[j];
                p.out[j] = c->brb[j]; p.resid[j] = k == 0 ? c->x0 : c->brb[j];
                p.act[j] = k < 2 ? c->a16[j] : nullptr;
                p.act_alpha[j] = k < 2 ? c->rb_alpha[i][j][k + 1][0] : nullptr;
            }
            p.dil = 1;
            CHK(run_conv(p, BM, IN_F16, nchunk, 3, s));
        }
    }
    PostP pp{c->brb[0], c->brb[1], c->brb[2], c->post_alpha, c->post_w, c->post_b, c->audio, T, nchunk};
    hipLaunchKernelGGL(post_conv_kernel, dim3(nchunk * ((T + 255) / 256)), dim3(256), 0, s, pp);
    CHK(hipGetLastError());
    return MP_OK;
}

}  // namespace

extern "C" {

int mp_hip_codec_init(int device, const char *path, mp_codec **out) {
    if (!out || !path) return MP_ERR_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return MP_ERR_HIP;
    mp_codec *c = new mp_codec();
    c->device = device;
    int least = 0, greatest = 0;  // the codec's stream at the least priority (see mp_hip_init)
    if (hipSetDevice(device) != hipSuccess || hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess ||
        hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, least) != hipSuccess) {
        delete c;
        return MP_ERR_HIP;
    }
    if (int rc = load_codec(c, path)) {
        fprintf(stderr, "mp_hip_codec_init: %s\n", c->err.c_str());
        mp_hip_codec_free(c);
        return rc;
    }
    *out = c;
    return MP_OK;
}

// The stream a decode runs on: the background (CU-masked) one while set, else the codec's.
// c->stream is swapped for the call's duration (every launch of codec_run reads it).
struct CodecStreamScope {
    mp_codec *c;
    hipStream_t saved;
    explicit CodecStreamScope(mp_codec *cc) : c(cc), saved(cc->stream) {
        if (c->bg && c->bg_stream) c->stream = c->bg_stream;
    }
    ~CodecStreamScope() { c->stream = saved; }
};

int mp_hip_codec_decode_chunks(mp_codec *c, const int32_t *codes, int n_chunks, int chunk_frames, float *audio_out) {
    if (!c) return MP_ERR_ARG;
    if (!codes || !audio_out || n_chunks < 1 || chunk_frames < 1) { c->err = "invalid arguments"; return MP_ERR_ARG; }
    CHK(hipSetDevice(c->device));
    CodecStreamScope scope(c);
    if (int rc = ensure_buffers(c, n_chunks, chunk_frames)) return rc;
    const size_t ncodes = (size_t)n_chunks * 8 * chunk_frames, nsamp = (size_t)n_chunks * chunk_frames * mpc::HOP;
    if (c->h_codes_cap < ncodes) {
        if (c->h_codes_pin) hipHostFree(c->h_codes_pin);
        c->h_codes_pin = nullptr;
        c->h_codes_cap = 0;
        CHK(hipHostMalloc((void **)&c->h_codes_pin, ncodes * 4, hipHostMallocDefault));
        c->h_codes_cap = ncodes;
    }
    if (c->h_audio_cap < nsamp) {
        if (c->h_audio_pin) hipHostFree(c->h_audio_pin);
        c->h_audio_pin = nullptr;
        c->h_audio_cap = 0;
        CHK(hipHostMalloc((void **)&c->h_audio_pin, nsamp * 4, hipHostMallocDefault));
        c->h_audio_cap = nsamp;
    }
    memcpy(c->h_codes_pin, codes, ncodes * 4);
    CHK(hipMemcpyAsync(c->codes, c->h_codes_pin, ncodes * 4, hipMemcpyHostToDevice, c->stream));
    if (!c->ev0) { CHK(hipEventCreate(&c->ev0)); CHK(hipEventCreate(&c->ev1)); }
    // diagnostics: MAGPIE_CODEC_TS=stage,block,file -> the phase stamps of that stage's
    // rb_kernel launch for residual block `block` (tools_dev/codec_rb_timeline.py)
    constexpr size_t TS_N = (size_t)3 * mpc::RB_TS_GX * mpc::RB_TS_N;
    // (read per call: parsed into locals and committed only when all 3 fields parse;
    // absent or malformed, the stamps are off again)
    {
        const char *e = getenv("MAGPIE_CODEC_TS");
        char file[512] = {0};
        int st = -1, bl = -1;
        if (e && sscanf(e, "%d,%d,%511s", &st, &bl, file) == 3) {
            c->ts_stage = st;
            c->ts_block = bl;
            c->ts_file = file;
            if (!c->ts_dev) CHK(hipMalloc((void **)&c->ts_dev, TS_N * 8));
            CHK(hipMemsetAsync(c->ts_dev, 0, TS_N * 8, c->stream));
        } else {
            c->ts_stage = c->ts_block = -1;
            c->ts_file.clear();
        }
    }
    CHK(hipEventRecord(c->ev0, c->stream));
    if (int rc = codec_run(c, n_chunks, chunk_frames)) return rc;
    CHK(hipEventRecord(c->ev1, c->stream));
    CHK(hipMemcpyAsync(c->h_audio_pin, c->audio, nsamp * 4, hipMemcpyDeviceToHost, c->stream));
    CHK(hipStreamSynchronize(c->stream));
    memcpy(audio_out, c->h_audio_pin, nsamp * 4);
    CHK(hipEventElapsedTime(&c->last_ms, c->ev0, c->ev1));
    if (c->ts_dev && !c->ts_file.empty()) {
        std::vector<unsigned long long> h(TS_N);
        CHK(hipMemcpy(h.data(), c->ts_dev, TS_N * 8, hipMemcpyDeviceToHost));
        if (FILE *f = fopen(c->ts_file.c_str(), "wb")) {
            fwrite(h.data(), 8, h.size(), f);
            fclose(f);
        }
    }
    return MP_OK;
}

int mp_hip_codec_last_ms(mp_codec *c, float *ms) {
    if (!c || !ms) return MP_ERR_ARG;
    *ms = c->last_ms;
    return MP_OK;
}

int mp_hip_codec_decode(mp_codec *c, const int32_t *codes, int n_frames, float *audio_out) {
    return mp_hip_codec_decode_chunks(c, codes, 1, n_frames, audio_out);
}

// Internal (mp_hip_decode_stream): run this codec's next decodes in the background, i.e. on a
// stream confined to `cus` of the device's CUs (0: back to the codec's own stream), so a decode
// in flight on the model's stream keeps the rest of the chip; every decode computes the same bits
// on either stream (the kernels do not depend on where their workgroups run).
extern "C" int mp_codec_set_background(mp_codec *c, int cus) {
    if (!c) return MP_ERR_ARG;
    if (cus <= 0) { c->bg = 0; return MP_OK; }
    CHK(hipSetDevice(c->device));
    if (!c->bg_stream || c->bg_cus != cus) {
        if (c->bg_stream) { CHK(hipStreamSynchronize(c->bg_stream)); hipStreamDestroy(c->bg_stream); c->bg_stream = nullptr; }
        int ncu = 0;
        CHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device));
        if (cus >= ncu) { c->bg = 0; return MP_OK; }
        const std::vector<uint32_t> mask = mp::cu_share_mask(ncu, cus, false);
        CHK(hipExtStreamCreateWithCUMask(&c->bg_stream, (uint32_t)mask.size(), mask.data()));
        c->bg_cus = cus;
    }
    c->bg = 1;
    return MP_OK;
}

void mp_hip_codec_free(mp_codec *c) {
    if (!c) return;
    hipSetDevice(c->device);
    if (c->stream) hipStreamSynchronize(c->stream);
    if (c->bg_stream) { hipStreamSynchronize(c->bg_stream); hipStreamDestroy(c->bg_stream); }
    if (c->h_codes_pin) hipHostFree(c->h_codes_pin);
    if (c->h_audio_pin) hipHostFree(c->h_audio_pin);
    for (void *p : c->weight_allocs) hipFree(p);
    if (c->ts_dev) hipFree(c->ts_dev);
    if (c->rb_ctr) hipFree(c->rb_ctr);
    float *bufs[5] = {c->x_pre, c->x0, c->brb[0], c->brb[1], c->brb[2]};
    for (float *b : bufs) if (b) hipFree(b);
    for (int j = 0; j < 3; ++j) {
        if (c->a16[j]) hipFree(c->a16[j]);
        if (c->b16[j]) hipFree(c->b16[j]);
    }
    if (c->codes) hipFree(c->codes);
    if (c->audio) hipFree(c->audio);
    if (c->ev0) hipEventDestroy(c->ev0);
    if (c->ev1) hipEventDestroy(c->ev1);
    if (c->stream) hipStreamDestroy(c->stream);
    delete c;
}

const char *mp_hip_codec_error(mp_codec *c) { return c ? c->err.c_str() : "null mp_codec"; }

}  // extern "C"
