// Per-frame decode kernels for gfx950 (f32 path, batch NB <= 8 utterances;
// the F32 FFN convs of a Q8_0 / Q4_0 file also at 16).
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
#include "mp_sa.hpp"
#include "mp_xa.hpp"

namespace mp {

// ---------------------------------------------------------------- GEMV core
// Rows [row0, row0+RW) of W (row-major [N][K]) dotted with act[NB][K].
// Lane l owns elements 4*(l + 64*i): every weight load is a 1 KiB coalesced
// wave-instruction; activations come from LDS with conflict-free ds_read_b128.
#ifndef MP_GEMV_WSN
#define MP_GEMV_WSN 1  // the GEMV family's wave sums advanced together (0: one after another)
#endif
template <int NB, int RW, int K, int PRO, int EPI>
__global__ __launch_bounds__(MP_BLOCK) void gemv_kernel(GemvP p) {
    const unsigned long long t_start = ts_begin(p.ts);
    if constexpr (EPI == EPI_RESID_XA) {
        // the launch's last XA_SPLITS x NB workgroups: cross-attention on this launch's x1
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
    // No early exit on the done counter: a dependent load there would sit in
    // front of the weight stream of every launch. Once every slot is done the
    // iteration recomputes identical values (codes_prev / pos are frozen) and
    // lt_finalize_kernel refuses to touch the outputs.
    constexpr int VW = K >= 256 ? 4 : K / 64;
    constexpr int NV = K / (64 * VW);
    using VT = typename vecf<VW>::T;
    // rows too wide for LDS at 16 slots (PRO_PLAIN, K = 3072: 192 KB) are staged
    // 8 slots at a time against the same weight registers; per (row, slot) the
    // arithmetic is the same at every batch size
    constexpr int NBS = (PRO == PRO_PLAIN && NB * K > 32768) ? NB / 2 : NB;
    static_assert(NBS == NB || PRO == PRO_PLAIN, "only plain rows are staged in halves");
    constexpr int SC = pro_scratch<NBS, PRO>();
    __shared__ __attribute__((aligned(16))) float act[NBS * K];
    __shared__ float red[8];
    __shared__ float sc[SC];

    // The weight rows do not depend on the prologue: issue the whole stream first
    // so the HBM latency overlaps the prologue's own dependent loads/reductions.
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int row0 = (blockIdx.x * MP_NWAVES + w) * RW + ts_dep(t_start);
    // PreRows prologues (LN rows, plain rows, split merges): their loads go ahead of the
    // weights (pre_load), the arithmetic after them is unchanged
    PreRows<NB, K, PRO> pre;
    constexpr bool PRE = PreRows<NB, K, PRO>::ON;
    if constexpr (PRE) {
        pre_load<NB, K, PRO>(p, pre);
        __builtin_amdgcn_sched_barrier(0);  // issue order: rows, weights, then arithmetic
    }
    VT wv[RW][NV];
#pragma unroll
    for (int r = 0; r < RW; ++r) {
        const int n = row0 + r < p.N ? row0 + r : p.N - 1;
        const VT *wr = (const VT *)(p.W + (size_t)n * K);
#pragma unroll
        for (int i = 0; i < NV; ++i) wv[r][i] = K == LTD ? ld_lt(wr + lane + 64 * i) : ld_weight(wr + lane + 64 * i);
    }
    // the epilogue's operand of this lane's output (lane r*NB + b), behind the weights
    float eop = 0.f;
    if constexpr (epi_has_operand<EPI>()) {
        const int nq = row0 + lane / NB;
        if (lane < RW * NB && nq < p.N) eop = epi_operand<EPI>(p, nq, lane % NB);
    }
    if constexpr (PRE || epi_has_operand<EPI>()) __builtin_amdgcn_sched_barrier(0);
    if constexpr (EPI != EPI_RESID_XA && EPI != EPI_QKV_SA) ts_phase<1>(p.ts, 0);  // profiling: weights issued
    float acc[RW][NB];
#pragma unroll
    for (int hh = 0; hh < NB / NBS; ++hh) {
        if constexpr (PRE) {
            pre_finish<NB, K, PRO>(p, pre, act, sc);
        } else if constexpr (NBS == NB) {
            prologue<NB, K, PRO>(p, act, red, sc);
        } else {
            if (hh) lds_sync();  // every wave is done with the previous slots' rows
            GemvP ph = p;
            ph.src = p.src + (size_t)hh * NBS * p.src_ld;
            prologue<NBS, K, PRO>(ph, act, red, sc);
        }
        if constexpr (EPI != EPI_RESID_XA && EPI != EPI_QKV_SA) ts_phase<2>(p.ts, 0);  // profiling: prologue done
        // every (row, slot) partial first, then their wave sums advanced together
        // (wave_sum_n: each total is wave_sum's, same tree and order)
        float sv[RW * NBS];
#pragma unroll
        for (int b = 0; b < NBS; ++b) {
            VT av[NV];
#pragma unroll
            for (int i = 0; i < NV; ++i) av[i] = ((const VT *)(act + b * K))[lane + 64 * i];
#pragma unroll
            for (int r = 0; r < RW; ++r) {
                float s = 0.f;
#pragma unroll
                for (int i = 0; i < NV; ++i) s += dotv(wv[r][i], av[i]);
                sv[r * NBS + b] = s;
            }
        }
        if constexpr (MP_GEMV_WSN) {
            wave_sum_n<RW * NBS>(sv);
        } else {
#pragma unroll
            for (int j = 0; j < RW * NBS; ++j) sv[j] = wave_sum(sv[j]);
        }
#pragma unroll
        for (int b = 0; b < NBS; ++b)
#pragma unroll
            for (int r = 0; r < RW; ++r) acc[r][hh * NBS + b] = sv[r * NBS + b];
    }
    // acc[][] is wave-uniform: lane r*NB + b owns output (row0 + r, slot b), so the
    // epilogue (GELU, KV append, residual) runs on RW*NB lanes in parallel.
    static_assert(RW * NB <= 64, "one lane per output");
    if constexpr (EPI != EPI_RESID_XA && EPI != EPI_QKV_SA) ts_phase<3>(p.ts, 0);  // profiling: dot products
    float v = 0.f;
#pragma unroll
    for (int r = 0; r < RW; ++r)
#pragma unroll
        for (int b = 0; b < NB; ++b)
            if (lane == r * NB + b) v = acc[r][b];
    if constexpr (NB == 1 && EPI == EPI_BIAS && PRO == PRO_LTFFN_MERGE) {
        if (p.cand) {  // uniform: the f32 LT head's workgroup candidate (greedy, batch 1)
            // the masked first-max of this workgroup's logits as one ordered key (every special
            // id but EOS masked); EOS's own key goes to slot LT_HEAD_WGS, and the consumer
            // (lt_step_body) drops it while EOS is forbidden (step < 4, or ignore_eos)
            __shared__ unsigned long long ck[MP_NWAVES];
            unsigned long long key = 0;
            const int n = row0 + lane;
            if (lane < RW && n < p.N) {
                const float lv = v + eop;  // the logit epi_store_op<EPI_BIAS> stores
                if (n == p.audio_eos) p.cand[LT_HEAD_WGS] = lt_cand_key(lv, n);
                else if (!lt_forbidden(n, true, p.audio_bos, p.audio_eos)) key = lt_cand_key(lv, n);
            }
            key = wave_max_u64(key);
            if (lane == 0) ck[w] = key;
            lds_sync();
            if (threadIdx.x == 0) {
                unsigned long long k = ck[0];
#pragma unroll
                for (int u = 1; u < MP_NWAVES; ++u) k = ck[u] > k ? ck[u] : k;
                p.cand[blockIdx.x] = k;
            }
        }
    }
    if (lane >= RW * NB) return;
    const int b = lane % NB, n = row0 + lane / NB;
    if (n >= p.N) return;
    if constexpr (EPI == EPI_RESID_XA) {
        publish_x1_op(p, v, n, b, eop);
    } else if constexpr (EPI == EPI_QKV_SA) {
        publish_qkv(p, v, n, b);
    } else if constexpr (EPI == EPI_BIAS || EPI == EPI_RESID || EPI == EPI_ADD_STORE) {
        epi_store_op<EPI>(p, v, n, b, eop);
    } else {
        epi_store<EPI>(p, v, n, b, EPI == EPI_LTX_ADD ? sc[b * LTD + n] : 0.f);
    }
    ts_end(p.ts, t_start);
}

// ---------------------------------------------------------------- SA decode attention
// Split-K over the live cache (sa_part, mp_sa.hpp): grid (head, split, slot), 4
// waves per workgroup; at batch 1 that is 48 workgroups of ~L/4 keys each instead
// of one workgroup streaming a whole head. Layers >= 1 of the f32 and 16-bit
// families run the same body in their QKV launch (EPI_QKV_SA) below 16 slots;
// this kernel serves layer 0, 16 slots and the Q8_0 mode.
constexpr int SA_WAVES = MP_NWAVES, SA_THREADS = SA_WAVES * 64;
template <bool KV16>
__global__ __launch_bounds__(SA_THREADS) void sa_attn_kernel(AttnP p) {
    const unsigned long long t_start = ts_begin(p.ts);
    sa_part<KV16, SA_WAVES, false>(p, blockIdx.x, blockIdx.y, blockIdx.z, nullptr, 0u, nullptr, ts_dep(t_start));
    if (p.merged) sa_merge_split(p, blockIdx.x, blockIdx.y, blockIdx.z);
    ts_end(p.ts, t_start);
}

// ---------------------------------------------------------------- fused XA (xa_part: mp_xa.hpp)
__global__ __launch_bounds__(XA_THREADS) void xa_part_kernel(XaP p) {
    const unsigned long long t_start = ts_begin(p.ts);
    xa_part<false>(p, blockIdx.x, blockIdx.y, nullptr, 0u, nullptr, ts_dep(t_start));
    ts_end(p.ts, t_start);
}

hipError_t op_xa(const XaP &p, int B, hipStream_t s) {
    if (!p.x || !p.part || !p.lnw || !p.kp || !p.vp || !p.T || p.Tmax < 1 || p.Tmax > TMAX_LIMIT) return hipErrorInvalidValue;
    mp::launch(xa_part_kernel, dim3(XA_SPLITS, B), dim3(XA_THREADS), 0, s, p);
    return hipGetLastError();
}

// ---------------------------------------------------------------- frame finalize
// Codebook 7's masked argmax, then the reference's loop bookkeeping
// (magpie.cpp:4340-4358): stop on EOS in any codebook (frame not emitted), else
// append the frame; stop at max_dec_steps; otherwise the frame becomes the next
// decoder input and the position advances.
// Launched with FIN_THREADS = 4 waves per slot. Wave 0 runs codebook 7's pick
// and the books; waves 1-3 (192 lanes, one float4 of the 768 each) meanwhile
// gather the next decoder input's codebook 0-6 rows and its position row, which do
// not depend on the pick, so only codebook 7's row is loaded after it. The sum
// keeps embed_kernel's order (codebooks 0..7 in sequence, / 8, + position): the
// same bits.
constexpr int FIN_THREADS = 256;
__global__ __launch_bounds__(FIN_THREADS) void lt_finalize_kernel(FinP p) {
    const unsigned long long t_start = ts_begin(p.ts);
    const int b = blockIdx.x, tid = threadIdx.x, w = tid >> 6;
    if (p.iter && b == 0 && tid == 0) p.iter[0] += 1;  // the next iteration's hand-off tags
    // a finished slot keeps running with the batch: it gets its frozen input again
    // (codes_prev / pos no longer advance), so every later iteration recomputes the
    // values of the one that ended it (the hidden-state trace row at the frozen step
    // included) instead of running on the last output residual
    const bool done = p.done[b] != 0;
    const bool embed = p.x != nullptr && !p.lt_only;
    const int e = tid - 64;  // waves 1-3: float4 e of the row
    // Σ_cb emb[cb][cs[cb]] over codebooks 0..ncb-1 in sequence, and position row ps
    auto gather = [&](const int *cs, int ps, int ncb, float4 &s, float4 &pe) {
        ps = ps < p.pos_rows ? ps : p.pos_rows - 1;  // a slot that stops this frame reads a row it never uses
        s = *(const float4 *)(p.emb + (size_t)cs[0] * D + 4 * e);
#pragma unroll
        for (int cb = 1; cb < NCB; ++cb) {
            if (cb >= ncb) break;
            const float4 r = *(const float4 *)(p.emb + ((size_t)cb * VCB + cs[cb]) * D + 4 * e);
            s.x = s.x + r.x; s.y = s.y + r.y; s.z = s.z + r.z; s.w = s.w + r.w;
        }
        pe = *(const float4 *)(p.pos_emb + (size_t)ps * D + 4 * e);
    };
    auto store_x = [&](float4 s, float4 pe) {
        *(float4 *)(p.x + (size_t)b * D + 4 * e) = make_float4(s.x * 0.125f + pe.x, s.y * 0.125f + pe.y,
                                                               s.z * 0.125f + pe.z, s.w * 0.125f + pe.w);
    };
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f), pe = s;
    if (embed && w >= 1) {
        if (done) gather(p.codes_prev + b * NCB, p.pos[b], NCB, s, pe);
        else gather(p.codes_cur + b * NCB, p.pos[b] + 1, NCB - 1, s, pe);
    }
    // greedy: codebook 7's pick split over the 4 waves (lt_step_body's split pick: each
    // wave scans PICK_R / 4 logit rows, the pairs meet in LDS; the same code)
    static_assert(FIN_THREADS / 64 == MP_NWAVES, "the split pick's rows per wave");
    const bool quad = !p.smp.on;
    float lq[QPR];
    int stp_q = 0;
    if (quad) {
        const float *lg = p.logits + (size_t)b * VCB + ts_dep(t_start);
#pragma unroll
        for (int q = 0; q < QPR; ++q) {
            const int i = (tid & 63) + 64 * (w * QPR + q);
            lq[q] = i < VCB ? lg[i] : -INFINITY;
        }
        stp_q = p.step[b];
    }
    __shared__ int sh_adv, sh_code, sh_stop;
    __syncthreads();  // every read of pos / codes / step above precedes wave 0's updates
    if (done) {
        if (embed && w >= 1) store_x(s, pe);
        return;
    }
    int i0 = 0, amax = 0;
    if (quad) {
        float bv;
        int bi = wave_pick_rows(lq, w, p.ignore_eos || stp_q < 4, p.audio_bos, p.audio_eos, bv);
        if (bi < 0 || bi >= VCB) bi = 0;
        pick_exchange(bv, bi, i0);
        amax = i0;
    }
    if (w == 0) {
        // codebook 7's pick with the same wave_pick as every other codebook (masked
        // first-max argmax; top-k draw when sampling); lane 0 keeps the books
        if (!quad) {
            __shared__ float scratch[2 * VCB];
            const int stp = p.step[b];
            i0 = wave_pick(p.logits + (size_t)b * VCB + ts_dep(t_start), p.ignore_eos || stp < 4, p.audio_bos,
                           p.audio_eos, p.smp, b, stp, NCB - 1, scratch, amax);
        }
        if (tid == 0) {
            int adv = 0, stop = 0;
            int cc[NCB];
            int *ccp = p.codes_cur + b * NCB;
            ccp[NCB - 1] = i0;
#pragma unroll
            for (int cb = 0; cb < NCB - 1; ++cb) cc[cb] = ccp[cb];
            cc[NCB - 1] = i0;
            if (p.smp.amax) p.smp.amax[b * NCB + NCB - 1] = amax;
            // EOS if any codebook's sampled code or argmax is EOS (magpie.cpp:4340-4348)
            bool eos = amax == p.audio_eos;
            eos |= p.smp.argeos[b] != 0;
            p.smp.argeos[b] = 0;
            if (!p.lt_only) {  // magpie_local_transformer_sample_all: codes only
                for (int cb = 0; cb < NCB; ++cb) eos |= cc[cb] == p.audio_eos;
                const int st = p.step[b];
                if (eos) {
                    // graph_reuse drops the EOS frame (4349-4352); the streaming loop emits it (4800-4806)
                    if (p.emit_eos)
                        for (int cb = 0; cb < NCB; ++cb) p.codes_out[((size_t)b * p.max_steps + st) * NCB + cb] = cc[cb];
                    p.done[b] = 1;
                    p.nframes[b] = p.emit_eos ? st + 1 : st;
                    atomicAdd(p.ndone, 1);
                    stop = 1;
                } else {
                    for (int cb = 0; cb < NCB; ++cb) p.codes_out[((size_t)b * p.max_steps + st) * NCB + cb] = cc[cb];
                    p.step[b] = st + 1;
                    if (st + 1 >= p.max_steps) {
                        p.done[b] = 1;
                        p.nframes[b] = st + 1;
                        atomicAdd(p.ndone, 1);
                        stop = 1;
                    } else {
                        for (int cb = 0; cb < NCB; ++cb) p.codes_prev[b * NCB + cb] = cc[cb];
                        p.pos[b] = p.pos[b] + 1;
                        adv = 1;
                    }
                }
            }
            sh_adv = adv;
            sh_stop = stop;
            sh_code = i0;
        }
    }
    __syncthreads();
    if (sh_adv && embed && w >= 1) {
        const float4 r = *(const float4 *)(p.emb + ((size_t)(NCB - 1) * VCB + sh_code) * D + 4 * e);
        s.x = s.x + r.x; s.y = s.y + r.y; s.z = s.z + r.z; s.w = s.w + r.w;
        store_x(s, pe);
    } else if (sh_stop && embed && w >= 1) {
        // the slot stopped this frame: from the next iteration on it gets its frozen
        // input (the done branch's gather), so the iterations the batch still runs
        // recompute this frame's values instead of running on the last FFN output
        gather(p.codes_prev + b * NCB, p.pos[b], NCB, s, pe);
        store_x(s, pe);
    }
    ts_end(p.ts, t_start);
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
    if constexpr (PRO == PRO_SA_MERGE) ok &= p.part != nullptr;
    if constexpr (PRO == PRO_LTFFN_MERGE) ok &= p.part && p.addsrc;
    if constexpr (PRO == PRO_XA_LN) ok &= p.part && p.src && p.lnw && p.xres;
    if constexpr (PRO == PRO_LN) ok &= p.src && p.lnw;
    if constexpr (PRO == PRO_LTX_LN) ok &= p.lt_s && p.lt_pos && p.ltX && p.lnw;
    if constexpr (PRO == PRO_LT_ATTN) ok &= p.ltq && p.ltk && p.ltv;
    if constexpr (PRO == PRO_LTARG_ATTN)
        ok &= p.logits && p.codes_cur && p.qkvtab && p.lk && p.lv && p.ltk && p.ltv && p.step && p.smp.cfg && p.smp.argeos;
    if constexpr (EPI == EPI_STORE || EPI == EPI_GELU) ok &= p.out != nullptr;
    if constexpr (EPI == EPI_BIAS) ok &= p.out && p.bias;
    if constexpr (EPI == EPI_RESID) ok &= p.resid != nullptr;
    if constexpr (EPI == EPI_ADD_STORE) ok &= p.out && p.addsrc;
    if constexpr (EPI == EPI_LTX_ADD) ok &= p.out && p.ptab && p.lt_pos && p.cb >= 1;
    if constexpr (EPI == EPI_QKV || EPI == EPI_QKV_SA) ok &= p.out && p.kc && p.vc && p.pos;
    if constexpr (EPI == EPI_QKV_SA) ok &= qkv_sa_args_ok(p);
    if constexpr (EPI == EPI_LTQKV) ok &= p.lq && p.lk && p.lv;
    if constexpr (EPI == EPI_LTKVO) ok &= p.lk && p.lv && p.N == 2 * LTD;
    if constexpr (EPI == EPI_RESID_XA)
        ok &= p.resid && p.xh && p.iter && p.hx_err && p.N == D && p.xa.part && p.xa.lnw && p.xa.kp && p.xa.vp &&
              p.xa.T && p.xa.Tmax >= 1 && p.xa.Tmax <= TMAX_LIMIT;
    return ok;
}

template <int NB, int RW, int K, int PRO, int EPI>
static hipError_t launch_gemv(const GemvP &p, hipStream_t s) {
    if (!gemv_args_ok<PRO, EPI>(p)) return hipErrorInvalidValue;
    const int rows_per_block = MP_NWAVES * RW;
    GemvP q = p;
    q.nrow_blocks = (p.N + rows_per_block - 1) / rows_per_block;
    const int grid = q.nrow_blocks + (EPI == EPI_RESID_XA ? XA_SPLITS * NB : EPI == EPI_QKV_SA ? NH * SA_SPLITS * NB : 0);
    mp::launch((gemv_kernel<NB, RW, K, PRO, EPI>), dim3(grid), dim3(MP_BLOCK), 0, s, q);
    return hipGetLastError();
}

// Named entry points (one per fused op of the decode iteration), instantiated
// for NB in {1, 2, 4, 8}.
// rows per wave of the QKV and FFN-up GEMVs (2: 288 / 384 workgroups at 2304 / 3072 rows);
// any value computes the same bits (each wave's rows are independent)
#ifndef MP_RW_QKV
#define MP_RW_QKV 2
#endif
#ifndef MP_RW_FF1
#define MP_RW_FF1 2
#endif
constexpr int RW_QKV = MP_RW_QKV, RW_FF1 = MP_RW_FF1;
#define MP_DECODE_OPS(NB)                                                                                        \
    hipError_t op_qkv_##NB(const GemvP &p, hipStream_t s) { return launch_gemv<NB, RW_QKV, D, PRO_LN, EPI_QKV>(p, s); }        \
    hipError_t op_qkv_sa_##NB(const GemvP &p, hipStream_t s) { return launch_gemv<NB, RW_QKV, D, PRO_LN, EPI_QKV_SA>(p, s); }  \
    hipError_t op_xq_##NB(const GemvP &p, hipStream_t s) { return launch_gemv<NB, 1, D, PRO_LN, EPI_STORE>(p, s); }            \
    hipError_t op_oproj_##NB(const GemvP &p, hipStream_t s) { return launch_gemv<NB, 1, D, PRO_SA_MERGE, EPI_RESID>(p, s); } \
    hipError_t op_oproj_xa_##NB(const GemvP &p, hipStream_t s) {                                                   \
        return launch_gemv<NB, 1, D, PRO_SA_MERGE, EPI_RESID_XA>(p, s);                                            \
    }                                                                                                              \
    hipError_t op_ff1_##NB(const GemvP &p, hipStream_t s) { return launch_gemv<NB, RW_FF1, D, PRO_LN, EPI_GELU>(p, s); }       \
    hipError_t op_ff1x_##NB(const GemvP &p, hipStream_t s) { return launch_gemv<NB, RW_FF1, D, PRO_XA_LN, EPI_GELU>(p, s); }   \
    hipError_t op_ff2_##NB(const GemvP &p, hipStream_t s) { return launch_gemv<NB, 1, DFF, PRO_PLAIN, EPI_ADD_STORE>(p, s); }  \
    hipError_t op_lt_in0_##NB(const GemvP &p, hipStream_t s) { return launch_gemv<NB, 1, D, PRO_LN, EPI_BIAS>(p, s); }         \
    hipError_t op_lt_a_##NB(const GemvP &p, hipStream_t s) { return launch_gemv<NB, 1, LTD, PRO_LTX_LN, EPI_LTQKV>(p, s); }    \
    hipError_t op_lt_bg_##NB(const GemvP &p, hipStream_t s) { return launch_gemv<NB, 1, LTD, PRO_LTARG_ATTN, EPI_LTX_ADD>(p, s); } \
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
// Q8_0 weight mode at 16 slots: the FFN convs (F32 in the reference's Q8 file)
hipError_t op_ff1_16(const GemvP &p, hipStream_t s) { return launch_gemv<16, 2, D, PRO_LN, EPI_GELU>(p, s); }
#ifndef MP_RW_FF2_16
#define MP_RW_FF2_16 1
#endif
hipError_t op_ff2_16(const GemvP &p, hipStream_t s) { return launch_gemv<16, MP_RW_FF2_16, DFF, PRO_PLAIN, EPI_ADD_STORE>(p, s); }
// the direct XA's f32 q_net at 16 slots (bf16 mode)
hipError_t op_xq_16(const GemvP &p, hipStream_t s) { return launch_gemv<16, 1, D, PRO_LN, EPI_STORE>(p, s); }


hipError_t op_sa_attn(const AttnP &p, int B, hipStream_t s) {
    if (!p.q || !p.kc || !p.vc || !p.pos || !p.part || p.max_seq < 1 || p.max_seq > NCH_MAX * SA_CHUNK)
        return hipErrorInvalidValue;
    if (p.kv16) mp::launch(sa_attn_kernel<true>, dim3(NH, SA_SPLITS, B), dim3(SA_THREADS), 0, s, p);
    else mp::launch(sa_attn_kernel<false>, dim3(NH, SA_SPLITS, B), dim3(SA_THREADS), 0, s, p);
    return hipGetLastError();
}

// ---------------------------------------------------------------- LT pick (large batches)
// PRO_LTARG_ATTN's per-slot work as its own launch, one wave per slot, for
// NB >= 8 (where the fused prologue would run several slots' picks in sequence
// per wave): codebook cb-1's pick, the gathers of position cb's q|k|v and
// residual rows, the causal attention. The attention output goes to ltq (out),
// the residual row to ltX; the o_net GEMV (PRO_PLAIN + EPI_ADD_STORE) follows.
// Same functions, same arithmetic as the fused path: batches stay bit-identical.
__global__ __launch_bounds__(64) void lt_pick_kernel(GemvP p) {
    __shared__ float wsc[2 * VCB];
    const int b = blockIdx.x, lane = threadIdx.x;
    float4 kr[NCB], vr[NCB];
    {
        const float *kb = p.ltk + (size_t)b * NCB * LTD + 4 * lane, *vb = p.ltv + (size_t)b * NCB * LTD + 4 * lane;
#pragma unroll
        for (int j = 0; j < NCB - 1; ++j)
            if (j < p.cb) { kr[j] = *(const float4 *)(kb + j * LTD); vr[j] = *(const float4 *)(vb + j * LTD); }
    }
    float lv[PICK_R];
    load_logits(p.logits + (size_t)b * VCB, lv);
    const int stp = p.step[b];
    int amax;
    const int code = wave_pick_v(lv, p.ignore_eos || stp < 4, p.audio_bos, p.audio_eos, p.smp, b, stp, p.cb - 1, wsc,
                                 amax);
    if (lane == 0) {
        p.codes_cur[b * NCB + p.cb - 1] = code;
        if (amax == p.audio_eos) p.smp.argeos[b] = 1;
        if (p.smp.amax) p.smp.amax[b * NCB + p.cb - 1] = amax;
    }
    const size_t r = (size_t)(p.cb - 1) * VCB + code;
    const float *row = p.qkvtab + r * (3 * LTD) + 4 * lane;
    const float4 q4 = *(const float4 *)row, k4 = *(const float4 *)(row + LTD), v4 = *(const float4 *)(row + 2 * LTD);
    const float4 x4 = *(const float4 *)(p.ptab + r * LTD + 4 * lane);
    const float4 pos4 = *(const float4 *)(p.lt_pos + (size_t)p.cb * LTD + 4 * lane);
    *(float4 *)(p.lk + ((size_t)b * NCB + p.cb) * LTD + 4 * lane) = k4;
    *(float4 *)(p.lv + ((size_t)b * NCB + p.cb) * LTD + 4 * lane) = v4;
    *(float4 *)(p.ltX + (size_t)b * LTD + 4 * lane) =
        make_float4(x4.x + pos4.x, x4.y + pos4.y, x4.z + pos4.z, x4.w + pos4.w);
    *(float4 *)(p.out + (size_t)b * LTD + 4 * lane) = lt_attend<true, true>(p, b, q4, k4, v4, kr, vr);
}
hipError_t op_lt_pick(const GemvP &p, int NB, hipStream_t s) {
    if (!p.logits || !p.codes_cur || !p.qkvtab || !p.ptab || !p.lt_pos || !p.ltk || !p.ltv || !p.lk || !p.lv ||
        !p.ltX || !p.out || !p.step || !p.smp.cfg || !p.smp.argeos || p.cb < 1)
        return hipErrorInvalidValue;
    mp::launch(lt_pick_kernel, dim3(NB), dim3(64), 0, s, p);
    return hipGetLastError();
}
// o_net + residual after lt_pick_kernel (its attention output in src, residual in addsrc)
hipError_t op_lt_bo_8(const GemvP &p, hipStream_t s) { return launch_gemv<8, 1, LTD, PRO_PLAIN, EPI_ADD_STORE>(p, s); }

// ---------------------------------------------------------------- frame embedding
// One workgroup per slot; each element summed over the 8 codebooks in order, /8,
// + position: the first frame's decoder input (reset_decode_state); every later
// frame's is written by lt_finalize_kernel with the same arithmetic.
__global__ __launch_bounds__(MP_BLOCK) void embed_kernel(EmbP p) {
    const int b = blockIdx.x;
    int c[NCB];
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) c[cb] = p.codes[b * NCB + cb];
    const int ps = p.pos[b];
    for (int k = threadIdx.x; k < D; k += MP_BLOCK) {
        float s = p.emb[((size_t)0 * VCB + c[0]) * D + k];
#pragma unroll
        for (int cb = 1; cb < NCB; ++cb) s = s + p.emb[((size_t)cb * VCB + c[cb]) * D + k];
        p.x[(size_t)b * D + k] = s * 0.125f + p.pos_emb[(size_t)ps * D + k];
    }
}
hipError_t op_embed(const EmbP &p, int NB, hipStream_t s) {
    if (!p.emb || !p.codes || !p.pos_emb || !p.pos || !p.x) return hipErrorInvalidValue;
    mp::launch(embed_kernel, dim3(NB), dim3(MP_BLOCK), 0, s, p);
    return hipGetLastError();
}

// ---------------------------------------------------------------- LT FFN
// FFN up + GELU + FFN down of the local transformer in one launch
// (magpie.cpp:983-992): workgroup p owns hidden units j in [16p, 16p+16). Its
// weights (16 rows of W1, the 16-column slice of W2 that row n = thread n
// reads, one contiguous 16 KiB block of the slice-major copy) are issued first; every slot's LN(y) row is built by one wave (DPP
// statistics, the same code at every batch size), a wave computes 4 units per
// slot (float4 lanes, DPP sum, GELU) into LDS, then thread n adds its 16 units'
// contributions to output n in ascending order. The LT_FFN_P partial sums are
// merged (ascending p) by the head's prologue at batch 1 or by lt_merge_kernel.
template <int NB>
__global__ __launch_bounds__(MP_BLOCK) void lt_ffn_kernel(LtFfnP p) {
    constexpr int U = LTF / LT_FFN_P, UPW = U / MP_NWAVES;
    static_assert(U % MP_NWAVES == 0 && U % 4 == 0 && LTD == MP_BLOCK, "unit split");
    __shared__ __attribute__((aligned(16))) float xs[NB][LTD];
    __shared__ __attribute__((aligned(16))) float fs[NB][U];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, j0 = blockIdx.x * U;
    float4 a1[UPW], a2[U / 4];
#pragma unroll
    for (int r = 0; r < UPW; ++r) a1[r] = *(const float4 *)(p.w1 + (size_t)(j0 + w * UPW + r) * LTD + 4 * lane);
#pragma unroll
    for (int i = 0; i < U / 4; ++i) a2[i] = *(const float4 *)(p.w2 + (size_t)j0 * LTD + tid * U + 4 * i);
    for (int b = w; b < NB; b += MP_NWAVES) {
        float x[LTD / 64];
#pragma unroll
        for (int i = 0; i < LTD / 64; ++i) x[i] = p.y[(size_t)b * LTD + lane + 64 * i];
        float mean, var;
        wave_meanvar<LTD / 64>(x, mean, var);
        const float rstd = 1.0f / sqrtf(var + p.eps);
#pragma unroll
        for (int i = 0; i < LTD / 64; ++i) xs[b][lane + 64 * i] = ((x[i] - mean) * rstd) * p.lnw[lane + 64 * i];
    }
    lds_sync();
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const float4 xv = *(const float4 *)&xs[b][4 * lane];
        float v[UPW];
#pragma unroll
        for (int r = 0; r < UPW; ++r) v[r] = dotv(a1[r], xv);
        ffn_units_store<UPW>(v, &fs[b][w * UPW], [](float g) { return g; });
    }
    lds_sync();
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        float acc = 0.f;
#pragma unroll
        for (int i = 0; i < U / 4; ++i) {
            const float4 f4 = *(const float4 *)&fs[b][4 * i];
            acc = fmaf(a2[i].x, f4.x, acc);
            acc = fmaf(a2[i].y, f4.y, acc);
            acc = fmaf(a2[i].z, f4.z, acc);
            acc = fmaf(a2[i].w, f4.w, acc);
        }
        p.part[ltp_idx(b, blockIdx.x, tid)] = acc;
    }
}
template <int NB>
__global__ __launch_bounds__(MP_BLOCK) void lt_merge_kernel(LtFfnP p) {
    for (int e = threadIdx.x; e < NB * LTD; e += MP_BLOCK) p.out[e] = lt_ffn_merge(p.part, p.y, e / LTD, e % LTD);
}
hipError_t op_lt_ffn(const LtFfnP &p, int NB, hipStream_t s) {
    if (!p.y || !p.lnw || !p.w1 || !p.w2 || !p.part) return hipErrorInvalidValue;
    switch (NB) {
    case 1: mp::launch(lt_ffn_kernel<1>, dim3(LT_FFN_P), dim3(MP_BLOCK), 0, s, p); break;
    case 2: mp::launch(lt_ffn_kernel<2>, dim3(LT_FFN_P), dim3(MP_BLOCK), 0, s, p); break;
    case 4: mp::launch(lt_ffn_kernel<4>, dim3(LT_FFN_P), dim3(MP_BLOCK), 0, s, p); break;
    case 8: mp::launch(lt_ffn_kernel<8>, dim3(LT_FFN_P), dim3(MP_BLOCK), 0, s, p); break;
    case 16: mp::launch(lt_ffn_kernel<16>, dim3(LT_FFN_P), dim3(MP_BLOCK), 0, s, p); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
hipError_t op_lt_merge(const LtFfnP &p, int NB, hipStream_t s) {
    if (!p.y || !p.part || !p.out) return hipErrorInvalidValue;
    switch (NB) {
    case 1: mp::launch(lt_merge_kernel<1>, dim3(1), dim3(MP_BLOCK), 0, s, p); break;
    case 2: mp::launch(lt_merge_kernel<2>, dim3(1), dim3(MP_BLOCK), 0, s, p); break;
    case 4: mp::launch(lt_merge_kernel<4>, dim3(1), dim3(MP_BLOCK), 0, s, p); break;
    case 8: mp::launch(lt_merge_kernel<8>, dim3(1), dim3(MP_BLOCK), 0, s, p); break;
    case 16: mp::launch(lt_merge_kernel<16>, dim3(1), dim3(MP_BLOCK), 0, s, p); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
// ---------------------------------------------------------------- LT, f32 mode
// One wave computes slot b's LT residual row y at position cb (LtFfn2P): cb = 0:
// y = X_0 + vo_0; cb >= 1: codebook cb-1's pick (wave_pick_v, the same draw as
// every other path), the q|k|vo gathers of that code's table rows, the causal
// softmax over positions 0..cb and y = X_cb + sum_j p_j vo_j. Lane l returns
// elements 4l..4l+3. `wb0`: this is workgroup 0, which publishes the code and the
// position's k / vo rows for the later codebooks. One body for every batch size
// (one wave per slot), so a batch reproduces its utterances run alone.
// lt_y_slot's global loads (earlier positions' k / vo, the logits, the step; cb = 0:
// X_0 and vo_0), apart from its arithmetic so a kernel can issue them ahead of its
// weight stream (vector loads complete in issue order). Native vectors, every element
// assigned (an array of HIP's float4 struct in a struct member went to scratch).
struct LtYPre {
    f32x4 kr[NCB - 1], vr[NCB - 1];
    float lv[PICK_R];
    int stp;
};
__device__ __forceinline__ void lt_y_load(const LtFfn2P &p, int b, LtYPre &r) {
    const int lane = threadIdx.x & 63, cb = p.cb;
    const size_t row = (size_t)b * NCB * LTD + 4 * lane;
    if (cb == 0) {
        r.kr[0] = *(const f32x4 *)(p.ltX + (size_t)b * LTD + 4 * lane);
        r.vr[0] = *(const f32x4 *)(p.ltv + row);
        return;
    }
#pragma unroll
    for (int j = 0; j < NCB - 1; ++j) {
        const int jj = j < cb ? j : 0;  // every element assigned; positions >= cb unused
        r.kr[j] = *(const f32x4 *)(p.ltk + row + jj * LTD);
        r.vr[j] = *(const f32x4 *)(p.ltv + row + jj * LTD);
    }
    load_logits(p.logits + (size_t)b * VCB, r.lv);
    r.stp = p.step[b];
}
// position cb's table rows for `code` (codebook cb-1's pick): q | k, o_net(v), P[code]
// and the position embedding
struct LtRows {
    float4 q4, k4, vo4, x4, pos4;
};
__device__ __forceinline__ LtRows lt_gather(const LtFfn2P &p, int code) {
    const int lane = threadIdx.x & 63, cb = p.cb;
    const size_t rr = (size_t)(cb - 1) * VCB + code;
    const float *qkv = p.qkvtab + rr * (3 * LTD) + 4 * lane;
    LtRows g;
    g.q4 = *(const float4 *)qkv;
    g.k4 = *(const float4 *)(qkv + LTD);
    g.vo4 = *(const float4 *)(p.votab + rr * LTD + 4 * lane);
    g.x4 = *(const float4 *)(p.ptab + rr * LTD + 4 * lane);
    g.pos4 = *(const float4 *)(p.lt_pos + (size_t)cb * LTD + 4 * lane);
    return g;
}
// the code's bookkeeping (workgroup 0) and y = X_cb + sum_j softmax_j(q k_j / 16) vo_j
__device__ __forceinline__ float4 lt_y_attend(const LtFfn2P &p, int b, bool wb0, int code, int amax, const LtYPre &r,
                                              const LtRows &g) {
    const int lane = threadIdx.x & 63, cb = p.cb;
    const size_t row = (size_t)b * NCB * LTD + 4 * lane;
    const float4 q4 = g.q4, k4 = g.k4, vo4 = g.vo4, x4 = g.x4, pos4 = g.pos4;
    if (wb0) {
        if (lane == 0) {
            p.codes_cur[b * NCB + cb - 1] = code;
            if (amax == p.audio_eos) p.smp.argeos[b] = 1;
            if (p.smp.amax) p.smp.amax[b * NCB + cb - 1] = amax;
        }
        *(float4 *)(p.ltk + row + cb * LTD) = k4;
        *(float4 *)(p.ltv + row + cb * LTD) = vo4;
    }
    // the cb + 1 scores' wave sums advanced together (wave_sum_n: each wave_sum's tree)
    float sj[NCB];
#pragma unroll
    for (int j = 0; j < NCB; ++j) sj[j] = dotv(q4, j < cb ? to_f4(r.kr[j < NCB - 1 ? j : 0]) : k4);
    wave_sum_n<NCB>(sj);
#pragma unroll
    for (int j = 0; j < NCB; ++j) sj[j] = j <= cb ? sj[j] * (1.0f / 16.0f) : -INFINITY;
    float m = -INFINITY;
#pragma unroll
    for (int j = 0; j < NCB; ++j) m = fmaxf(m, sj[j]);
    float l = 0.f;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int j = 0; j < NCB; ++j) {
        if (j > cb) break;
        const float e = expf(sj[j] - m);
        l += e;
        const float4 v4 = j == cb ? vo4 : to_f4(r.vr[j < NCB - 1 ? j : 0]);
        a.x = fmaf(e, v4.x, a.x); a.y = fmaf(e, v4.y, a.y); a.z = fmaf(e, v4.z, a.z); a.w = fmaf(e, v4.w, a.w);
    }
    return make_float4(x4.x + pos4.x + a.x / l, x4.y + pos4.y + a.y / l, x4.z + pos4.z + a.z / l,
                       x4.w + pos4.w + a.w / l);
}
__device__ __forceinline__ float4 lt_y_finish(const LtFfn2P &p, int b, bool wb0, float *wsc, LtYPre &r) {
    const int cb = p.cb;
    if (cb == 0) {
        const float4 x = to_f4(r.kr[0]), v = to_f4(r.vr[0]);
        return make_float4(x.x + v.x, x.y + v.y, x.z + v.z, x.w + v.w);
    }
    const int stp = r.stp;
    int amax;
    const int code = wave_pick_v(r.lv, p.ignore_eos || stp < 4, p.audio_bos, p.audio_eos, p.smp, b, stp, cb - 1, wsc,
                                 amax);
    ts_phase<0>(p.f.ts, 0);  // profiling: code picked
    return lt_y_attend(p, b, wb0, code, amax, r, lt_gather(p, code));
}

// Batch 1, greedy (codebooks >= 1): the pick split over the workgroup's MP_NWAVES waves.
// One wave's pick is ~300 dependent VALU / DPP instructions (~0.9 us of the step, while
// the other waves wait); here wave w scans logit rows [w QPR, (w + 1) QPR) with
// wave_pick_v's mask and first-max rule, gathers its own candidate's table rows at once,
// and the waves' (max, first index) pairs meet in LDS: the first wave holding the global
// maximum has the global first index (its ids are the lowest), so the code is
// wave_pick_v's, and that wave, whose rows are already in flight, computes y.
__device__ __forceinline__ void lt_y_load_q(const LtFfn2P &p, int b, int w, LtYPre &r, float (&lq)[QPR]) {
    const int lane = threadIdx.x & 63, cb = p.cb;
    const size_t row = (size_t)b * NCB * LTD + 4 * lane;
#pragma unroll
    for (int j = 0; j < NCB - 1; ++j) {
        const int jj = j < cb ? j : 0;
        r.kr[j] = *(const f32x4 *)(p.ltk + row + jj * LTD);
        r.vr[j] = *(const f32x4 *)(p.ltv + row + jj * LTD);
    }
    const float *lg = p.logits + (size_t)b * VCB;
#pragma unroll
    for (int q = 0; q < QPR; ++q) {
        const int i = lane + 64 * (w * QPR + q);
        lq[q] = i < VCB ? lg[i] : -INFINITY;
    }
    r.stp = p.step[b];
}
// every wave: its rows' pick, its candidate's table rows (g, in flight during the exchange),
// the exchange; returns the wave holding the code (code: the code, in every wave)
__device__ __forceinline__ int lt_pick_split(const LtFfn2P &p, int w, const LtYPre &yp, float (&lq)[QPR], LtRows &g,
                                             int &code) {
    float bv;
    int bi = wave_pick_rows(lq, w, p.ignore_eos || yp.stp < 4, p.audio_bos, p.audio_eos, bv);
    if (bi < 0 || bi >= VCB) bi = 0;
    g = lt_gather(p, bi);
    return pick_exchange(bv, bi, code);
}

// The same pick from the head's workgroup candidates (GemvP::cand, batch 1 greedy): wave w
// holds candidates 64 w .. 64 w + 63 (one ordered key per lane; slot LT_HEAD_WGS is EOS's key,
// dropped while EOS is forbidden), one 64-bit wave max gives the wave's (value, first index),
// then the same gather and exchange as lt_pick_split. The candidates cover ascending row
// ranges wave by wave, so the exchange's first wave at the maximum holds the first index:
// the code is wave_pick_rows'.
__device__ __forceinline__ void lt_y_load_c(const LtFfn2P &p, int w, LtYPre &r, unsigned long long &ck) {
    const int lane = threadIdx.x & 63, cb = p.cb;
    const size_t row = 4 * (size_t)lane;  // slot 0
#pragma unroll
    for (int j = 0; j < NCB - 1; ++j) {
        const int jj = j < cb ? j : 0;
        r.kr[j] = *(const f32x4 *)(p.ltk + row + jj * LTD);
        r.vr[j] = *(const f32x4 *)(p.ltv + row + jj * LTD);
    }
    const int slot = 64 * w + lane;
    ck = slot <= p.ncand ? p.cand[slot] : 0ull;
    r.stp = p.step[0];
}
__device__ __forceinline__ int lt_pick_cand(const LtFfn2P &p, int w, const LtYPre &yp, unsigned long long ck, LtRows &g,
                                            int &code) {
    const int lane = threadIdx.x & 63;
    if (64 * w + lane == p.ncand && (p.ignore_eos || yp.stp < 4)) ck = 0;  // EOS forbidden
    ck = wave_max_u64(ck);
    const float bv = ck ? lt_cand_value(ck) : -INFINITY;
    int bi = ck ? lt_cand_index(ck) : 0;
    if (bi < 0 || bi >= VCB) bi = 0;
    g = lt_gather(p, bi);
    return pick_exchange(bv, bi, code);
}

__device__ __forceinline__ float4 lt_y_slot(const LtFfn2P &p, int b, bool wb0, float *wsc) {
    LtYPre r;
    lt_y_load(p, b, r);
    return lt_y_finish(p, b, wb0, wsc, r);
}

// The LT step of codebook cb in f32 mode: y (lt_y_slot, every workgroup for itself;
// workgroup 0 stores it as the head's residual), then LN + FFN up + GELU + FFN down
// partial sums exactly as lt_ffn_kernel (workgroup pb owns hidden units [16pb,
// 16pb+16)). acc[b]: this thread's (output tid) partial sum of slot b; ys (nullable):
// slot 0's y for the caller.
template <int NB>
__device__ __forceinline__ void lt_step_body(const LtFfn2P &p, int pb, int dep, float (&accs)[NB], float *ys) {
    constexpr int U = LTF / LT_FFN_P, UPW = U / MP_NWAVES;
    static_assert(U % MP_NWAVES == 0 && U % 4 == 0 && LTD == MP_BLOCK, "unit split");
    __shared__ __attribute__((aligned(16))) float xs[NB][LTD];
    __shared__ __attribute__((aligned(16))) float fs[NB][U];
    __shared__ __attribute__((aligned(16))) float wsc_all[MP_NWAVES][2 * VCB];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, j0 = pb * U + dep;
    // the wave's first slot's loads (logits, earlier positions) ahead of the weights
    LtYPre yp;
    float lq[QPR];
    unsigned long long ck = 0;
    const bool quad = NB == 1 && p.cb > 0 && !p.smp.on;  // uniform: the split greedy pick
    const bool cand = quad && p.cand;                      // uniform: ... from the head's candidates
    if (cand) lt_y_load_c(p, w, yp, ck);
    else if (quad) lt_y_load_q(p, 0, w, yp, lq);
    else if (w < NB) lt_y_load(p, w, yp);
    // the LN weights with the first loads: loaded after y (behind its stores) they cost an
    // L2 round trip on the step's critical path
    const float4 gln = *(const float4 *)(p.f.lnw + 4 * lane);
    __builtin_amdgcn_sched_barrier(0);
    float4 a1[UPW], a2[U / 4];
#pragma unroll
    for (int r = 0; r < UPW; ++r) a1[r] = ld_ltffn((const float4 *)(p.f.w1 + (size_t)(j0 + w * UPW + r) * LTD + 4 * lane));
#pragma unroll
    for (int i = 0; i < U / 4; ++i) a2[i] = ld_ltffn((const float4 *)(p.f.w2 + (size_t)j0 * LTD + tid * U + 4 * i));
    __builtin_amdgcn_sched_barrier(0);
    if (NB == 1 && p.f.ts && w == 0) {  // diagnostics: when wave 0's own loads (not the 8 weight loads) have landed
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        ts_phase<3>(p.f.ts, 0);
    }
    auto y_ln = [&](int b, float4 y) {  // y -> the head's residual row (workgroup 0), LN(y) -> xs[b]
        if (pb == 0) *(float4 *)((float *)p.f.y + (size_t)b * LTD + 4 * lane) = y;
        if (ys && b == 0) *(float4 *)&ys[4 * lane] = y;
        const float x[4] = {y.x, y.y, y.z, y.w};
        float mean, var;
        wave_meanvar<4>(x, mean, var);
        const float rstd = 1.0f / sqrtf(var + p.f.eps);
        const float4 g = gln;
        *(float4 *)&xs[b][4 * lane] = make_float4(((x[0] - mean) * rstd) * g.x, ((x[1] - mean) * rstd) * g.y,
                                                  ((x[2] - mean) * rstd) * g.z, ((x[3] - mean) * rstd) * g.w);
    };
    if (quad) {
        LtRows g;
        int code;
        if ((cand ? lt_pick_cand(p, w, yp, ck, g, code) : lt_pick_split(p, w, yp, lq, g, code)) == w) {
            ts_phase_w<0>(p.f.ts);  // profiling: code picked
            const float4 y = lt_y_attend(p, 0, pb == 0, code, code, yp, g);
            ts_phase_w<1>(p.f.ts);  // profiling: y (gathers + attention)
            y_ln(0, y);
        }
    } else {
        for (int b = w; b < NB; b += MP_NWAVES) {
            const float4 y = b == w ? lt_y_finish(p, b, pb == 0, wsc_all[w], yp) : lt_y_slot(p, b, pb == 0, wsc_all[w]);
            if (b == 0) ts_phase<1>(p.f.ts, 0);  // profiling: y (gathers + attention)
            y_ln(b, y);
        }
    }
    lds_sync();
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const float4 xv = *(const float4 *)&xs[b][4 * lane];
        float v[UPW];
#pragma unroll
        for (int r = 0; r < UPW; ++r) v[r] = dotv(a1[r], xv);
        ffn_units_store<UPW>(v, &fs[b][w * UPW], [](float g) { return g; });
    }
    lds_sync();
    ts_phase<2>(p.f.ts, 0);  // profiling: FFN up
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        float acc = 0.f;
#pragma unroll
        for (int i = 0; i < U / 4; ++i) {
            const float4 f4 = *(const float4 *)&fs[b][4 * i];
            acc = fmaf(a2[i].x, f4.x, acc);
            acc = fmaf(a2[i].y, f4.y, acc);
            acc = fmaf(a2[i].z, f4.z, acc);
            acc = fmaf(a2[i].w, f4.w, acc);
        }
        accs[b] = acc;
    }
}
template <int NB>
__global__ __launch_bounds__(MP_BLOCK) void lt_ffn2_kernel(LtFfn2P p) {
    const unsigned long long t_start = ts_begin(p.f.ts);
    float accs[NB];
    lt_step_body<NB>(p, blockIdx.x, ts_dep(t_start), accs, nullptr);
#pragma unroll
    for (int b = 0; b < NB; ++b) p.f.part[ltp_idx(b, blockIdx.x, threadIdx.x)] = accs[b];
    ts_end(p.f.ts, t_start);
}

hipError_t op_lt_ffn2(const LtFfn2P &p, int NB, hipStream_t s) {
    if (!p.f.y || !p.f.lnw || !p.f.w1 || !p.f.w2 || !p.f.part || !p.ltX || !p.ltk || !p.ltv || !p.qkvtab ||
        !p.votab || !p.ptab || !p.lt_pos || !p.logits || !p.codes_cur || !p.step || !p.smp.cfg || !p.smp.argeos ||
        p.cb < 0 || p.cb >= NCB)
        return hipErrorInvalidValue;
    switch (NB) {
    case 1: mp::launch(lt_ffn2_kernel<1>, dim3(LT_FFN_P), dim3(MP_BLOCK), 0, s, p); break;
    case 2: mp::launch(lt_ffn2_kernel<2>, dim3(LT_FFN_P), dim3(MP_BLOCK), 0, s, p); break;
    case 4: mp::launch(lt_ffn2_kernel<4>, dim3(LT_FFN_P), dim3(MP_BLOCK), 0, s, p); break;
    case 8: mp::launch(lt_ffn2_kernel<8>, dim3(LT_FFN_P), dim3(MP_BLOCK), 0, s, p); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------- LT step, bf16 weight mode
// The bf16 mode's LT step of codebook cb, workgroup (q, b): slot b's y through
// lt_y_slot (wave 0; the attention in f32 through the load-time q|k|vo tables, as
// the f32 mode computes it), LN(y) rounded to bf16, then the FFN for hidden units
// [32q, 32q + 32): up (bf16 W1 rows, f32 sums, GELU, rounded to bf16) and its share
// of FFN down (bf16 W2 slice) as partial sums. From 2 slots up the partials are
// published as {tag, value} granules and every workgroup of the slot merges 8 of the
// 256 outputs (all-to-all over 32 workgroups, 2 KiB swept each, in q order whoever
// publishes last) into y2 = y + FFN(y) for the bf16 head; at batch 1 the head's
// prologue merges (the same operations in the same order).
// LTS_P workgroups per slot at every batch size (16 KiB of W1 and of W2 each): no
// slot's pick waits behind another's, and a batch reproduces its utterances run
// alone. The weights are issued before the pick.
constexpr int LTS_U = LTF / LTS_P, LTS_UPW = LTS_U / MP_NWAVES;
__device__ __forceinline__ float bf16_round(float v) { return __uint_as_float((unsigned)f32_to_bf16_rne(v) << 16); }
__device__ __forceinline__ float bf16_lo(unsigned u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf16_hi(unsigned u) { return __uint_as_float(u & 0xffff0000u); }
__global__ __launch_bounds__(MP_BLOCK) void lt_slot_kernel(LtFfn2P p) {
    const unsigned long long t_start = ts_begin(p.f.ts);
    static_assert(LTD == MP_BLOCK && LTS_U % 8 == 0 && LTS_U % MP_NWAVES == 0, "unit split");
    __shared__ __attribute__((aligned(16))) float xs[LTD];
    __shared__ __attribute__((aligned(16))) float ys[LTD];
    __shared__ __attribute__((aligned(16))) float hs[LTS_U];
    __shared__ __attribute__((aligned(16))) float wsc[2 * VCB];
    const int q = blockIdx.x, b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int u0 = q * LTS_U + ts_dep(t_start);
    // wave 0's logits / earlier positions first, then the weights (in-order completion)
    LtYPre yp;
    float lq[QPR];
    const bool quad = p.cb > 0 && !p.smp.on;  // uniform: the greedy pick split over the waves
    if (quad) lt_y_load_q(p, b, w, yp, lq);
    else if (w == 0) lt_y_load(p, b, yp);
    const float4 gln = *(const float4 *)(p.f.lnw + 4 * lane);  // LN weights with the first loads
    __builtin_amdgcn_sched_barrier(0);
    uint2 a1[LTS_UPW];  // W1 rows u0 + LTS_UPW w + r, elements 4 lane .. 4 lane + 3
#pragma unroll
    for (int r = 0; r < LTS_UPW; ++r) a1[r] = ld_ltffn((const uint2 *)(p.w1h + (size_t)(u0 + w * LTS_UPW + r) * LTD + 4 * lane));
    uint4 a2[LTS_U / 8];  // W2 row tid, units u0 .. u0 + LTS_U - 1
#pragma unroll
    for (int i = 0; i < LTS_U / 8; ++i) a2[i] = ld_ltffn((const uint4 *)(p.w2h + ((size_t)q * LTD + tid) * LTS_U + 8 * i));
    __builtin_amdgcn_sched_barrier(0);
    int yw = 0;  // the wave computing y
    float4 y;
    if (quad) {
        LtRows g;
        int code;
        yw = lt_pick_split(p, w, yp, lq, g, code);
        if (w == yw) y = lt_y_attend(p, b, q == 0, code, code, yp, g);
    } else if (w == 0) {
        y = lt_y_finish(p, b, q == 0, wsc, yp);
    }
    if (w == yw) {
        if (q == 0) *(float4 *)((float *)p.f.y + (size_t)b * LTD + 4 * lane) = y;
        *(float4 *)&ys[4 * lane] = y;
        const float x[4] = {y.x, y.y, y.z, y.w};
        float mean, var;
        wave_meanvar<4>(x, mean, var);
        const float rstd = 1.0f / sqrtf(var + p.f.eps);
        const float4 g = gln;
        *(float4 *)&xs[4 * lane] =
            make_float4(bf16_round(((x[0] - mean) * rstd) * g.x), bf16_round(((x[1] - mean) * rstd) * g.y),
                        bf16_round(((x[2] - mean) * rstd) * g.z), bf16_round(((x[3] - mean) * rstd) * g.w));
    }
    lds_sync();
    const float4 xv = *(const float4 *)&xs[4 * lane];
    {
        float v[LTS_UPW];
#pragma unroll
        for (int r = 0; r < LTS_UPW; ++r)
            v[r] = dotv(make_float4(bf16_lo(a1[r].x), bf16_hi(a1[r].x), bf16_lo(a1[r].y), bf16_hi(a1[r].y)), xv);
        ffn_units_store<LTS_UPW>(v, &hs[w * LTS_UPW], [](float g) { return bf16_round(g); });
    }
    lds_sync();
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < LTS_U / 8; ++i) {
        const float4 h0 = *(const float4 *)&hs[8 * i], h1 = *(const float4 *)&hs[8 * i + 4];
        acc = fmaf(bf16_lo(a2[i].x), h0.x, acc);
        acc = fmaf(bf16_hi(a2[i].x), h0.y, acc);
        acc = fmaf(bf16_lo(a2[i].y), h0.z, acc);
        acc = fmaf(bf16_hi(a2[i].y), h0.w, acc);
        acc = fmaf(bf16_lo(a2[i].z), h1.x, acc);
        acc = fmaf(bf16_hi(a2[i].z), h1.y, acc);
        acc = fmaf(bf16_lo(a2[i].w), h1.z, acc);
        acc = fmaf(bf16_hi(a2[i].w), h1.w, acc);
    }
    if (!p.gh) {  // batch 1: the head's prologue merges (PRO_LTS_MERGE)
        p.f.part[((size_t)b * LTS_P + q) * LTD + tid] = acc;
        ts_end(p.f.ts, t_start);
        return;
    }
    // the partial sums as {tag, value} granules; workgroup q then merges outputs
    // [ME q, ME q + ME) of its slot: thread t sweeps partial t / ME's granule of output
    // ME q + t % ME, and ME threads add the LTS_P values in q order (lts_merge's order)
    constexpr int ME = LTD / LTS_P;
    static_assert(ME * LTS_P == LTD && ME * LTS_P == MP_BLOCK, "one granule per thread");
    __shared__ float mv[LTS_P][ME];
    const unsigned tag = (unsigned)p.iter[0] * 64u + 32u + (unsigned)p.cb;
    gu64 *gh = (gu64 *)p.gh + (size_t)b * LTS_P * LTD;
    __hip_atomic_store(gh + (size_t)q * LTD + tid, ((unsigned long long)tag << 32) | __float_as_uint(acc),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    {
        const gu64 *g = gh + (size_t)(tid / ME) * LTD + ME * q + tid % ME;
        float v;
        for (unsigned spins = 0;; ++spins) {
            const unsigned long long u = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            v = __uint_as_float((unsigned)u);
            if (__all((unsigned)(u >> 32) == tag)) break;
            if (spins >= HX_SPIN_LIMIT) {  // never seen: poison the output and say so
                if (lane == 0) __hip_atomic_fetch_or((gi32 *)p.hx_err, HX_ERR_LT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                v = __builtin_nanf("");
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        mv[tid / ME][tid % ME] = v;
    }
    lds_sync();
    if (tid < ME) {
        float s = mv[0][tid];
#pragma unroll 8
        for (int k = 1; k < LTS_P; ++k) s += mv[k][tid];
        p.f.out[(size_t)b * LTD + ME * q + tid] = s + ys[ME * q + tid];
    }
    ts_end(p.f.ts, t_start);
}
hipError_t op_lt_slot(const LtFfn2P &p, int NB, hipStream_t s) {
    if (!p.f.y || !p.f.lnw || !p.w1h || !p.w2h || !p.f.part || (p.gh && (!p.f.out || !p.iter || !p.hx_err)) || !p.ltX || !p.ltk || !p.ltv ||
        !p.qkvtab || !p.votab || !p.ptab || !p.lt_pos || !p.logits || !p.codes_cur || !p.step || !p.smp.cfg ||
        !p.smp.argeos || p.cb < 0 || p.cb >= NCB || NB < 1 || NB > 16)
        return hipErrorInvalidValue;
    mp::launch(lt_slot_kernel, dim3(LTS_P, NB), dim3(MP_BLOCK), 0, s, p);
    return hipGetLastError();
}

// ---------------------------------------------------------------- LT front, f32 batch 1
// LtFrontP (mp_params.hpp). Workgroup p, wave w: in_proj row 4p + w exactly as
// gemv_kernel<1, 1, 768, PRO_LN, EPI_BIAS> computes it, rows 4p + w and 256 + 4p + w of
// [W_k ; W_o W_v] as gemv_kernel<1, 1, 256, PRO_LTX_LN, EPI_LTKVO> does, then the FFN
// step of lt_ffn2_kernel<1> for codebook 0 (y = X_0 + vo_0). The two all-to-all edges
// (in_proj output -> LN(X_0); vo_0 -> y) are 256-value granule sweeps (2 KiB) by the
// 64 workgroups of the launch, all co-resident.
// The front's work after its weight loads: LN(x) -> in_proj row n_in (published) ->
// X_0, LN(X_0) -> k_0 / vo_0 row n_in (vo_0 published) -> y = X_0 + vo_0 (wave 0; *y4
// and the lane's vo_0 elements *v4 when non-null) -> LN(y) -> this workgroup's 16 FFN
// units -> returns this thread's FFN-down partial sum (output tid) of codebook 0.
constexpr int LTF_U = LTF / LT_FFN_P, LTF_UPW = LTF_U / MP_NWAVES;
constexpr int LTFR_G = LTD / MP_NWAVES;  // lt_front workgroups: one in_proj / k / vo row per wave
// the front's small operands, loaded with the decoder row ahead of the weights: each read
// where it is used was a dependent L2 round trip on the front's chain (after the in_proj
// dot, after the in_proj / vo_0 granules, after y)
struct LtFrontPre {
    float bin;       // in_proj bias of this wave's row
    float posa[4];   // lt_pos[0][lane + 64 i]
    float gself[4];  // norm_self[lane + 64 i]
    float4 posb;     // lt_pos[0][4 lane .. 4 lane + 3]
    float4 gff;      // the LT FFN LayerNorm weights [4 lane .. 4 lane + 3]
};
__device__ __forceinline__ void lt_front_pre(const LtFrontP &p, int n_in, LtFrontPre &q) {
    const int lane = threadIdx.x & 63;
    q.bin = p.b_in[n_in];
#pragma unroll
    for (int i = 0; i < 4; ++i) q.posa[i] = p.lt_pos[lane + 64 * i];
    load_lnw<4>(p.norm_self, q.gself);
    q.posb = *(const float4 *)(p.lt_pos + 4 * lane);
    q.gff = *(const float4 *)(p.l.f.lnw + 4 * lane);
}
__device__ __forceinline__ float lt_front_core(const LtFrontP &p, int pb, int n_in, const float4 (&wi)[3], float4 wk,
                                               float4 wv, const float4 (&a1)[LTF_UPW], const float4 (&a2)[LTF_U / 4],
                                               const float (&v)[D / 64], const float (&g)[D / 64], const LtFrontPre &q,
                                               float *act, float *act2, float *xs, float *fs, float4 *y4, float4 *v4,
                                               float4 *k4 = nullptr) {
    constexpr int U = LTF_U, UPW = LTF_UPW, PER = D / 64, Q = PER / MP_NWAVES;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const unsigned tag_s = (unsigned)p.iter[0] * 64u + 40u, tag_v = tag_s + 1u;
    // ---- LN(x) (PRO_LN, batch 1: every wave the whole row, writes its quarter); the row
    // and the LN weights v, g were loaded by the caller ahead of the weight stream
    {
        float mean, var;
        wave_meanvar<PER>(v, mean, var);
        const float rstd = 1.0f / sqrtf(var + p.l.f.eps);
        const bool st = p.hidden_out && pb == 0;
        const int s = (p.trace && pb == 0) ? p.l.step[0] : 0;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            if (i / Q != w) continue;
            const int k = lane + 64 * i;
            const float y = ((v[i] - mean) * rstd) * g[i];
            act[k] = y;
            if (st) p.hidden_out[k] = y;
            if (p.trace && pb == 0 && s < p.trace_steps) p.trace[(size_t)s * D + k] = y;
        }
    }
    lds_sync();
    // ---- in_proj row n_in (+ bias), published
    {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < 3; ++i) s += dotv(wi[i], ((const float4 *)act)[lane + 64 * i]);
        const float v = wave_sum(s) + q.bin;
        if (lane == 0) {
            p.lt_s[n_in] = v;
            __hip_atomic_store((gu64 *)p.gh + n_in, ((unsigned long long)tag_s << 32) | __float_as_uint(v),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    // ---- X_0 = s + lt_pos[0], LN(X_0) (PRO_LTX_LN's one-wave statistics): wave 0
    if (w == 0) {
        float X[4], sv[4];
        const float(&g)[4] = q.gself;
        gh_wait_n<4, 64>(p.gh + lane, tag_s, sv, p.hx_err);  // in_proj outputs lane + 64 i
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int k = lane + 64 * i;
            xs[k] = sv[i];  // kept for the FFN step below (xs is free until then)
            X[i] = sv[i] + q.posa[i];
        }
        if (pb == 0)
#pragma unroll
            for (int i = 0; i < 4; ++i) const_cast<float *>(p.l.ltX)[lane + 64 * i] = X[i];  // lt_kvo wrote it
        float mean, var;
        wave_block_meanvar<1>(X, mean, var);
        const float rstd = 1.0f / sqrtf(var + p.l.f.eps);
#pragma unroll
        for (int i = 0; i < 4; ++i) act2[lane + 64 * i] = ((X[i] - mean) * rstd) * g[i];
    }
    lds_sync();
    // ---- k_0 row and vo_0 row n_in (EPI_LTKVO); vo_0 published
    {
        const float4 av = *(const float4 *)&act2[4 * lane];
        float sk = 0.f, sv = 0.f;  // gemv_kernel's accumulation, term for term
        sk += dotv(wk, av);
        sv += dotv(wv, av);
        const float k0 = wave_sum(sk), vo0 = wave_sum(sv);
        if (lane == 0) {
            p.l.ltk[n_in] = k0;
            p.l.ltv[n_in] = vo0;
            __hip_atomic_store((gu64 *)p.gh + LTD + n_in, ((unsigned long long)tag_v << 32) | __float_as_uint(vo0),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (k4)  // (lt_all_kernel: k_0 too, every workgroup attends over it)
                __hip_atomic_store((gu64 *)p.gh + 2 * LTD + n_in, ((unsigned long long)tag_v << 32) | __float_as_uint(k0),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    // ---- codebook 0's FFN step (lt_ffn2_kernel<1>: y = X_0 + vo_0, wave 0), in the
    // LT_FFN_P workgroups that own FFN units
    if (pb >= LT_FFN_P) return 0.f;
    if (w == 0) {
        float xv[4], vv[4];
        gh_wait_n<4, 1>(p.gh + LTD + 4 * lane, tag_v, vv, p.hx_err);  // vo_0 outputs 4 lane + c
        if (k4) {
            float kk[4];
            gh_wait_n<4, 1>(p.gh + 2 * LTD + 4 * lane, tag_v, kk, p.hx_err);
            *k4 = make_float4(kk[0], kk[1], kk[2], kk[3]);
        }
        wave_lds_sync();  // (xs: the in_proj outputs this wave stored above)
        const float pb4[4] = {q.posb.x, q.posb.y, q.posb.z, q.posb.w};
#pragma unroll
        for (int c = 0; c < 4; ++c) xv[c] = xs[4 * lane + c] + pb4[c];
        const float4 y = make_float4(xv[0] + vv[0], xv[1] + vv[1], xv[2] + vv[2], xv[3] + vv[3]);
        if (pb == 0) *(float4 *)((float *)p.l.f.y + 4 * lane) = y;
        if (y4) *y4 = y;
        if (v4) *v4 = make_float4(vv[0], vv[1], vv[2], vv[3]);
        const float x[4] = {y.x, y.y, y.z, y.w};
        float mean, var;
        wave_meanvar<4>(x, mean, var);
        const float rstd = 1.0f / sqrtf(var + p.l.f.eps);
        const float4 g = q.gff;
        *(float4 *)&xs[4 * lane] = make_float4(((x[0] - mean) * rstd) * g.x, ((x[1] - mean) * rstd) * g.y,
                                               ((x[2] - mean) * rstd) * g.z, ((x[3] - mean) * rstd) * g.w);
    }
    lds_sync();
    {
        const float4 xv = *(const float4 *)&xs[4 * lane];
        float v[UPW];
#pragma unroll
        for (int r = 0; r < UPW; ++r) v[r] = dotv(a1[r], xv);
        ffn_units_store<UPW>(v, &fs[w * UPW], [](float g) { return g; });
    }
    lds_sync();
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < U / 4; ++i) {
        const float4 f4 = *(const float4 *)&fs[4 * i];
        acc = fmaf(a2[i].x, f4.x, acc);
        acc = fmaf(a2[i].y, f4.y, acc);
        acc = fmaf(a2[i].z, f4.z, acc);
        acc = fmaf(a2[i].w, f4.w, acc);
    }
    return acc;
}
// the front's weights (issued first): in_proj row n_in, k and vo rows, the FFN slice
__device__ __forceinline__ void lt_front_weights(const LtFrontP &p, int pb, int n_in, float4 (&wi)[3], float4 &wk,
                                                 float4 &wv, float4 (&a1)[LTF_UPW], float4 (&a2)[LTF_U / 4]) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
#pragma unroll
    for (int i = 0; i < 3; ++i) wi[i] = ld_lt((const float4 *)(p.w_in + (size_t)n_in * D + 4 * (lane + 64 * i)));
    wk = ld_lt((const float4 *)(p.w_kvo + (size_t)n_in * LTD + 4 * lane));
    wv = ld_lt((const float4 *)(p.w_kvo + (size_t)(LTD + n_in) * LTD + 4 * lane));
    const int j0 = pb * LTF_U;
    if (pb >= LT_FFN_P) {  // no FFN units in this workgroup (every element assigned: no scratch)
#pragma unroll
        for (int r = 0; r < LTF_UPW; ++r) a1[r] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int i = 0; i < LTF_U / 4; ++i) a2[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        return;
    }
#pragma unroll
    for (int r = 0; r < LTF_UPW; ++r)
        a1[r] = ld_ltffn((const float4 *)(p.l.f.w1 + (size_t)(j0 + w * LTF_UPW + r) * LTD + 4 * lane));
#pragma unroll
    for (int i = 0; i < LTF_U / 4; ++i) a2[i] = ld_ltffn((const float4 *)(p.l.f.w2 + (size_t)j0 * LTD + tid * LTF_U + 4 * i));
}
__global__ __launch_bounds__(MP_BLOCK) void lt_front_kernel(LtFrontP p) {
    const unsigned long long t_start = ts_begin(p.l.f.ts);
    static_assert(LTF_U % MP_NWAVES == 0 && LTD == MP_BLOCK && LT_FFN_P <= LTFR_G, "unit split");
    __shared__ __attribute__((aligned(16))) float act[D];
    __shared__ __attribute__((aligned(16))) float act2[LTD];
    __shared__ __attribute__((aligned(16))) float xs[LTD];
    __shared__ __attribute__((aligned(16))) float fs[LTF_U];
    const int tid = threadIdx.x, w = tid >> 6, pb = blockIdx.x;
    const int n_in = pb * MP_NWAVES + w + ts_dep(t_start);  // this wave's in_proj / k / vo row
    // the decoder output row and the final LN's weights first (vector loads complete in
    // issue order: behind the weights they would wait for all of them), then the weights
    constexpr int PER = D / 64;
    float v[PER], g[PER];
    const int lane = tid & 63;
#pragma unroll
    for (int i = 0; i < PER; ++i) v[i] = p.x[lane + 64 * i];
    load_lnw<PER>(p.norm_out, g);
    LtFrontPre q;
    lt_front_pre(p, n_in, q);
    __builtin_amdgcn_sched_barrier(0);
    float4 wi[3], wk, wv, a1[LTF_UPW], a2[LTF_U / 4];
    lt_front_weights(p, pb, n_in, wi, wk, wv, a1, a2);
    __builtin_amdgcn_sched_barrier(0);
    const float acc = lt_front_core(p, pb, n_in, wi, wk, wv, a1, a2, v, g, q, act, act2, xs, fs, nullptr, nullptr);
    if (pb < LT_FFN_P) p.l.f.part[ltp_idx(0, pb, tid)] = acc;
    ts_end(p.l.f.ts, t_start);
}
hipError_t op_lt_front(const LtFrontP &p, hipStream_t s) {
    static_assert(sizeof(LtFrontP) < 4096, "kernel argument size");
    if (!p.x || !p.norm_out || !p.w_in || !p.b_in || !p.lt_s || !p.lt_pos || !p.norm_self || !p.w_kvo || !p.gh ||
        !p.iter || !p.hx_err || !p.l.f.y || !p.l.f.lnw || !p.l.f.w1 || !p.l.f.w2 || !p.l.f.part || !p.l.ltX ||
        !p.l.ltk || !p.l.ltv || !p.l.step || p.l.cb != 0)
        return hipErrorInvalidValue;
    mp::launch(lt_front_kernel, dim3(LTFR_G), dim3(MP_BLOCK), 0, s, p);
    return hipGetLastError();
}

// ---------------------------------------------------------------- the whole LT, f32 batch 1 greedy
// LtAllP (mp_params.hpp). Workgroup pb: the front (lt_front_core), then per codebook cb its
// FFN-down partial sums published, outputs 4 pb .. 4 pb + 3 merged (lt_ffn_merge's order: the
// 64 partials ascending, then + y), y2 swept, head rows 32 pb .. 32 pb + 31 of codebook cb
// (gemv_kernel<1, *, 256, PRO_LTFFN_MERGE, EPI_BIAS>'s per-row arithmetic) and the workgroup's
// masked first-max key; wave 0 then picks codebook cb's code from the 64 keys (+ EOS's while
// EOS is allowed: the first max of wave_pick_rows), gathers position cb + 1's table rows and
// computes y as lt_y_attend with the earlier positions' k / vo rows kept in registers, and the
// workgroup runs its 16 FFN units (lt_step_body's arithmetic). Codebook 7's code is the
// finalize's pick from the logits. Three granule edges per codebook instead of two launches.
constexpr int LTA_ROWS = 32, LTA_RPW = LTA_ROWS / MP_NWAVES;  // head rows per workgroup / wave
static_assert(LTA_ROWS * LT_FFN_P >= VCB && LTFR_G == LT_FFN_P && LTA_RPW <= 64, "head split");
// candidate key: the logit's order bits, then 2047 - id (lower ids win ties), then a 21-bit tag
__device__ __forceinline__ unsigned long long lta_key(float v, int i, unsigned tc) {
    const unsigned u = __float_as_uint(v);
    const unsigned o = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    return ((unsigned long long)o << 32) | ((unsigned long long)(2047u - (unsigned)i) << 21) | tc;
}
__device__ __forceinline__ int lta_index(unsigned long long k) { return 2047 - (int)((k >> 21) & 2047u); }
__global__ __launch_bounds__(MP_BLOCK) void lt_all_kernel(LtAllP p) {
    const unsigned long long t_start = ts_begin(p.f.l.f.ts);
    __shared__ __attribute__((aligned(16))) float act[D];
    __shared__ __attribute__((aligned(16))) float act2[LTD];
    __shared__ __attribute__((aligned(16))) float xs[LTD];
    __shared__ __attribute__((aligned(16))) float fs[LTF_U];
    __shared__ __attribute__((aligned(16))) float ys[LTD];
    __shared__ float mv[LT_FFN_P][4];
    __shared__ unsigned long long ck[MP_NWAVES];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, pb = blockIdx.x;
    const int n_in = pb * MP_NWAVES + w + ts_dep(t_start);
    constexpr int PER = D / 64;
    float v[PER], g[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) v[i] = p.f.x[lane + 64 * i];
    load_lnw<PER>(p.f.norm_out, g);
    LtFrontPre q;
    lt_front_pre(p.f, n_in, q);
    const int stp = p.f.l.step[0];
    const unsigned it = (unsigned)p.f.iter[0];
    const float4 gln = q.gff;  // the LT FFN LayerNorm weights [4 lane .. 4 lane + 3]
    __builtin_amdgcn_sched_barrier(0);
    float4 wi[3], wk, wv, a1[LTF_UPW], a2[LTF_U / 4];
    lt_front_weights(p.f, pb, n_in, wi, wk, wv, a1, a2);
    __builtin_amdgcn_sched_barrier(0);
    float4 y4 = make_float4(0.f, 0.f, 0.f, 0.f), v4 = y4, k4 = y4;
    float acc = lt_front_core(p.f, pb, n_in, wi, wk, wv, a1, a2, v, g, q, act, act2, xs, fs, &y4, &v4, &k4);
    LtYPre r;  // wave 0: the positions' k / vo rows (lt_y_attend's operands)
#pragma unroll
    for (int j = 0; j < NCB - 1; ++j) r.kr[j] = r.vr[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    r.kr[0] = to_v4(k4);
    r.vr[0] = to_v4(v4);
    if (w == 0) *(float4 *)&ys[4 * lane] = y4;
    LtFfn2P lp = p.f.l;
    const bool eos_ok = !(lp.ignore_eos || stp < 4);
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) {
        const unsigned tag_p = it * 64u + 48u + (unsigned)cb, tag_y = it * 64u + 56u + (unsigned)cb;
        const unsigned tc = ((it * 8u + (unsigned)cb) % 0x1FFFFFu) + 1u;
        // codebook cb's head rows first: their latency under the two sweeps
        const int n0 = pb * LTA_ROWS + w * LTA_RPW, nl = n0 + lane;
        float4 hw[LTA_RPW];
#pragma unroll
        for (int rr = 0; rr < LTA_RPW; ++rr) {
            const int n = min(n0 + rr, VCB - 1);
            hw[rr] = ld_lt((const float4 *)(p.w_out + ((size_t)cb * VCB + n) * LTD + 4 * lane));
        }
        const float hb = lane < LTA_RPW && nl < VCB ? p.b_out[(size_t)cb * VCB + nl] : 0.f;
        __builtin_amdgcn_sched_barrier(0);
        // this thread's FFN-down partial sum (output tid), then outputs 4 pb + t % 4 from
        // partial t / 4 (the 64 partials in ascending order, + y: lt_ffn_merge)
        __hip_atomic_store((gu64 *)p.gp + pb * LTD + tid, ((unsigned long long)tag_p << 32) | __float_as_uint(acc),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        {
            float vv[1];
            gh_wait_n<1, 1>(p.gp + (tid >> 2) * LTD + 4 * pb + (tid & 3), tag_p, vv, p.f.hx_err);
            mv[tid >> 2][tid & 3] = vv[0];
        }
        lds_sync();
        if (tid < 4) {
            float s2 = mv[0][tid];
#pragma unroll 8
            for (int q2 = 1; q2 < LT_FFN_P; ++q2) s2 += mv[q2][tid];
            const float y2 = s2 + ys[4 * pb + tid];
            __hip_atomic_store((gu64 *)p.gy + 4 * pb + tid, ((unsigned long long)tag_y << 32) | __float_as_uint(y2),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        {
            float vv[1];
            gh_wait_n<1, 1>(p.gy + tid, tag_y, vv, p.f.hx_err);
            act2[tid] = vv[0];
        }
        lds_sync();
        // the head rows and this workgroup's masked first-max key
        {
            const float4 av = *(const float4 *)&act2[4 * lane];
            float lv = 0.f;
#pragma unroll
            for (int rr = 0; rr < LTA_RPW; ++rr) {
                float sacc = 0.f;
                sacc += dotv(hw[rr], av);
                const float sr = wave_sum(sacc);
                if (lane == rr) lv = sr;
            }
            unsigned long long key = tc;  // no candidate: below every real key, this codebook's tag
            if (lane < LTA_RPW && nl < VCB) {
                const float logit = lv + hb;
                p.logits[nl] = logit;
                if (nl == lp.audio_eos)
                    __hip_atomic_store((gu64 *)p.gc + LT_FFN_P, lta_key(logit, nl, tc), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                else if (!lt_forbidden(nl, true, lp.audio_bos, lp.audio_eos)) key = lta_key(logit, nl, tc);
            }
            key = wave_max_u64(key);
            if (lane == 0) ck[w] = key;
        }
        if (cb == NCB - 1) break;  // codebook 7's code: the finalize's pick
        lds_sync();
        if (tid == 0) {
            unsigned long long k = ck[0];
#pragma unroll
            for (int u = 1; u < MP_NWAVES; ++u) k = ck[u] > k ? ck[u] : k;
            __hip_atomic_store((gu64 *)p.gc + pb, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (w == 0) {
            // codebook cb's code from the 64 workgroup keys (+ EOS's while allowed)
            unsigned long long k1 = 0, k2 = 0;
            for (unsigned spins = 0;; ++spins) {
                k1 = __hip_atomic_load((const gu64 *)p.gc + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                k2 = __hip_atomic_load((const gu64 *)p.gc + LT_FFN_P, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (__all((unsigned)(k1 & 0x1FFFFFull) == tc && (unsigned)(k2 & 0x1FFFFFull) == tc)) break;
                if (spins >= HX_SPIN_LIMIT) {  // never seen: say so (the code falls back to 0)
                    if (lane == 0) __hip_atomic_fetch_or((gi32 *)p.f.hx_err, HX_ERR_LT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    k1 = k2 = 0;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if (lane == 0 && eos_ok && k2 > k1) k1 = k2;
            k1 = wave_max_u64(k1);
            int code = k1 ? lta_index(k1) : 0;
            if (code < 0 || code >= VCB) code = 0;
            // position cb + 1: the code's table rows, y = X + sum_j softmax_j vo_j (lt_y_attend)
            lp.cb = cb + 1;
            const LtRows gr = lt_gather(lp, code);
            const float4 y = lt_y_attend(lp, 0, pb == 0, code, code, r, gr);
            if (cb + 1 < NCB - 1) {
                r.kr[cb + 1] = to_v4(gr.k4);
                r.vr[cb + 1] = to_v4(gr.vo4);
            }
            if (pb == 0) *(float4 *)((float *)lp.f.y + 4 * lane) = y;
            *(float4 *)&ys[4 * lane] = y;
            const float x[4] = {y.x, y.y, y.z, y.w};
            float mean, var;
            wave_meanvar<4>(x, mean, var);
            const float rstd = 1.0f / sqrtf(var + lp.f.eps);
            *(float4 *)&xs[4 * lane] = make_float4(((x[0] - mean) * rstd) * gln.x, ((x[1] - mean) * rstd) * gln.y,
                                                   ((x[2] - mean) * rstd) * gln.z, ((x[3] - mean) * rstd) * gln.w);
        }
        lds_sync();
        // this workgroup's 16 FFN units of position cb + 1 (lt_step_body)
        {
            const float4 xv = *(const float4 *)&xs[4 * lane];
            float uv[LTF_UPW];
#pragma unroll
            for (int rr = 0; rr < LTF_UPW; ++rr) uv[rr] = dotv(a1[rr], xv);
            ffn_units_store<LTF_UPW>(uv, &fs[w * LTF_UPW], [](float gg) { return gg; });
        }
        lds_sync();
        acc = 0.f;
#pragma unroll
        for (int i = 0; i < LTF_U / 4; ++i) {
            const float4 f4 = *(const float4 *)&fs[4 * i];
            acc = fmaf(a2[i].x, f4.x, acc);
            acc = fmaf(a2[i].y, f4.y, acc);
            acc = fmaf(a2[i].z, f4.z, acc);
            acc = fmaf(a2[i].w, f4.w, acc);
        }
    }
    ts_end(p.f.l.f.ts, t_start);
}
hipError_t op_lt_all(const LtAllP &p, hipStream_t s) {
    static_assert(sizeof(LtAllP) < 4096, "kernel argument size");
    if (!p.f.x || !p.f.norm_out || !p.f.w_in || !p.f.b_in || !p.f.lt_s || !p.f.lt_pos || !p.f.norm_self || !p.f.w_kvo ||
        !p.f.gh || !p.f.iter || !p.f.hx_err || !p.f.l.f.y || !p.f.l.f.lnw || !p.f.l.f.w1 || !p.f.l.f.w2 ||
        !p.f.l.ltX || !p.f.l.ltk || !p.f.l.ltv || !p.f.l.step || !p.f.l.qkvtab || !p.f.l.votab || !p.f.l.ptab ||
        !p.f.l.lt_pos || !p.f.l.codes_cur || !p.f.l.smp.argeos || p.f.l.cb != 0 || p.f.l.smp.on || !p.w_out ||
        !p.b_out || !p.logits || !p.gp || !p.gy || !p.gc)
        return hipErrorInvalidValue;
    mp::launch(lt_all_kernel, dim3(LT_FFN_P), dim3(MP_BLOCK), 0, s, p);
    return hipGetLastError();
}

// the LT head at batch 1 with the FFN merge as its prologue
hipError_t op_lt_em_1(const GemvP &p, hipStream_t s) { return launch_gemv<1, MP_RW_LTE, LTD, PRO_LTFFN_MERGE, EPI_BIAS>(p, s); }
// f32 LT position 0: LN(X_0) -> [k_0 | vo_0] (W = [W_k ; W_o W_v], 512 x 256)
hipError_t op_lt_kvo(const GemvP &p, int NB, hipStream_t s) {
    switch (NB) {
    case 1: return launch_gemv<1, 1, LTD, PRO_LTX_LN, EPI_LTKVO>(p, s);
    case 2: return launch_gemv<2, 1, LTD, PRO_LTX_LN, EPI_LTKVO>(p, s);
    case 4: return launch_gemv<4, 1, LTD, PRO_LTX_LN, EPI_LTKVO>(p, s);
    case 8: return launch_gemv<8, 1, LTD, PRO_LTX_LN, EPI_LTKVO>(p, s);
    case 16: return launch_gemv<16, 1, LTD, PRO_LTX_LN, EPI_LTKVO>(p, s);
    }
    return hipErrorInvalidValue;
}

hipError_t op_finalize(const FinP &p, int B, hipStream_t s) {
    if (!p.smp.cfg || !p.smp.argeos) return hipErrorInvalidValue;
    if (p.x && (!p.emb || !p.pos_emb || p.pos_rows < 1)) return hipErrorInvalidValue;
    mp::launch(lt_finalize_kernel, dim3(B), dim3(FIN_THREADS), 0, s, p);
    return hipGetLastError();
}

}  // namespace mp
