// Parameter blocks + launchers of the per-utterance preamble kernels
// (mp_prefill.hip), shared with the host runtime.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

namespace mp {

enum GemmEpi {
    GE_STORE = 0,     // C[m][n] = v (+bias)
    GE_RESID = 1,     // C[m][n] += v
    GE_GELU = 2,      // C[m][n] = gelu(v)
    GE_QKV_CACHE = 3, // n < D: q rows; k/v -> SA cache at position t (prefill, 3942-3955)
    GE_XAKV = 4,      // n < 128: XA K, else XA V, at [b][layer][t]  (1689-1710)
};

struct GemmP {
    const float *A;  // [M][lda]
    int lda;
    const float *W;  // [N][K]
    const signed char *Wq;     // Q8_0 weight mode: int8 [N][K] + fp16 block scales [N][K/32]
    const unsigned short *Wd;  //   (ggml's quantised mul_mat, gemm_q8_kernel); null: f32 W
    const float *bias;
    float *C;
    int ldc;
    int M, N, K;
    int conv_taps;     // 0: plain A; 3: causal conv, A[m][k*Cin+i] = X[t-2+k][i] (1816-1866),
                       //    W re-laid out tap-major [N][k][Cin] at load
    int rows_per_utt;  // for (b, t) decomposition of a row
    const int *T;      // valid rows per utterance (conv zero padding / masking)
    float *kc, *vc;    // bf16 elements when kv16
    int kv16;
    int layer, nlayers, max_seq;
    float *xak, *xav;
    int Tmax;
    // deterministic split-K: with part != nullptr the K range is cut into
    // gemm_splits(K) pieces (a function of K only, so the arithmetic does not
    // depend on M, i.e. on the batch), each written raw to part[s][M][N], then
    // summed in split order by a second launch that applies the epilogue.
    float *part;
    int nsplit;        // gemm_splits(K), set by the launcher (the kernel's split length when gridDim.z == 1)
    // optional: the rows of C this GEMM completes are normalised next, LN(C row) * ln_w ->
    // ln_out[m * ln_ld] (N = 768; fused into the split reduction of a GE_RESID GEMM)
    const float *ln_w;
    float *ln_out;
    int ln_ld;
    float ln_eps;
    int xround;        // 2: round every A element to f16 as it is loaded (an F16 weight: ggml's
                       //    F16 mul_mat rounds src1 to f16; products then exact in f32)
    // batched (nbatch > 1): grid.z = nbatch x splits; batch z uses A + z sA, W (and Wq, Wd)
    // + (z % wmod) sW (sWq, sWd), C + z sC and layer + z: every layer's XA K/V, or every
    // (utterance, layer)'s K' / V', in one launch instead of one per layer (each is the same
    // GEMM as alone: the same tiles, splits and order)
    int nbatch, wmod;
    long long sA, sW, sC, sWq, sWd;
};

// the batch of this workgroup (GemmP::nbatch): shifts p to it, returns the split count and
// sets zs to the split index (blockIdx.z otherwise)
__device__ __forceinline__ int gemm_batch_enter(GemmP &p, int &zs) {
    const int nb = p.nbatch > 1 ? p.nbatch : 1;
    const int S = (int)gridDim.z / nb, bz = (int)blockIdx.z / S;
    zs = (int)blockIdx.z % S;
    if (bz) {
        const int wz = bz % (p.wmod > 0 ? p.wmod : nb);
        p.A += bz * p.sA;
        if (p.W) p.W += wz * p.sW;
        if (p.Wq) p.Wq += wz * p.sWq;
        if (p.Wd) p.Wd += wz * p.sWd;
        if (p.C) p.C += bz * p.sC;
        p.layer += bz;
    }
    return S;
}

// Split count of a preamble GEMM over K (fixed per K: batch-invariant results): K / 96
// pieces, at most 16, whole 32-wide blocks (MP_PRE_KS = 128: K / 128 pieces with 8 steps of
// loads in flight, measured slower in round 6: 3.17 vs 2.97 ms per preamble, more
// workgroups each paying its own start-up and partial-tile stores).
#ifndef MP_PRE_KS
#define MP_PRE_KS 0  // 0: K / 96 pieces, at most 16 (round 5's); 128: K / 128 (measured slower, round 6)
#endif
constexpr int PRE_KS = MP_PRE_KS;
#ifndef MP_PRE_INWG_TILES
#define MP_PRE_INWG_TILES 256
#endif
constexpr int PRE_INWG_TILES = MP_PRE_INWG_TILES;  // output tiles from which a GEMM runs its splits inside each workgroup
// The Q8_0 preamble GEMM (gemm_q8_kernel) always uses these pieces: its split order is part
// of the Q8_0 mode's f32 rounding, which moves activation-quantisation flips (the configs[4]
// long-form test's trajectory).
inline int gemm_splits_q8(int K) {
    int s = K / 96;
    if (s < 1) s = 1;
    if (s > 16) s = 16;
    while (s > 1 && (K % (s * 32)) != 0) --s;  // whole 32-wide (Q8_0) blocks per split
    return s;
}
inline int gemm_splits(int K) {
    if (PRE_KS > 0 && K % PRE_KS == 0) return K / PRE_KS;
    return gemm_splits_q8(K);  // (no model K takes this path)
}
// partial-sum capacity of either kernel's pieces
inline int gemm_splits_max(int K) { return gemm_splits(K) > gemm_splits_q8(K) ? gemm_splits(K) : gemm_splits_q8(K); }

// Causal multi-head attention for every (row, head) of a block of rows.
struct RowAttnP {
    const float *Q;  // [M][ldq], head h at +h*64
    int ldq;
    const float *Kb, *Vb;
    size_t utt_stride, row_stride;
    float *O;  // [M][768]
    int M, rows_per_utt, heads;
    int key_limit_T;  // 1: also mask keys j >= T[b] (unused when causal suffices)
    const int *T;
    int kv16;         // Kb / Vb hold bf16 elements (the SA cache in MP_KV_BF16 mode)
};

// Cross-attention for a block of rows (1 head x 128, no mask).
struct RowXaP {
    const float *Q;  // [M][128]
    const float *xak, *xav;
    int layer, nlayers, Tmax, rows_per_utt, M;
    const int *T;
    float *O;  // [M][128]
};

hipError_t pre_gemm(const GemmP &p, int epi, hipStream_t s);
hipError_t pre_ln_rows_multi(const float *X, int ldx, const float *w, long long sw, float *Y, int ldy, long long sy,
                             int M, int nw, float eps, hipStream_t s);
hipError_t pre_ln_rows(const float *X, int ldx, const float *w, float *Y, int ldy, int M, float eps, hipStream_t s);
// LT table rows: Y[r] = LN(P[r] + lt_pos[r / VCB + 1]) * w for r < 7 * VCB (the LN of
// PRO_LTARG_ATTN's position, bit for bit), rounded to bf16 when `b16`
// round: 0 none, 1 bf16, 2 f16 (the rows' operand precision in that weight mode)
hipError_t pre_lt_tab_rows(const float *P, const float *lt_pos, const float *w, float eps, float *Y, int round,
                           hipStream_t s);
// dst = bf16(src) held as f32 (a bf16-mode weight for an f32 GEMM)
hipError_t pre_round_bf16(const float *src, float *dst, size_t n, hipStream_t s);
hipError_t pre_row_attn(const RowAttnP &p, hipStream_t s);
hipError_t pre_row_xa(const RowXaP &p, hipStream_t s);
hipError_t pre_embed_text(const int *tok, const int *T, int B, int Tmax, const float *te, const float *ep, float *X,
                          hipStream_t s);
hipError_t pre_embed_context(const int *spk, int B, const float *baked, const float *dp, float *X, hipStream_t s);

}  // namespace mp
