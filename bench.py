#!/usr/bin/env python3
"""bench.py — frames/s of the MI355X-native Magpie decode loop.

Metric (BASELINE.json): audio-codec frames/sec + real-time factor, Magpie-357M.
Workload at N=1 is BASELINE.json configs[1]: Magpie-357M f32, batch=1, one
MI355X, HIP decoder-step kernels + hipGraph, KV cache resident in HBM.

A "step" is one decode pass of the batch: the BOS step + 255 autoregressive
iterations = 256 codec frames per utterance (fixed length, EOS masked; SURVEY
§8d), exactly what magpie_synthesize_codes_graph_reuse times as gen_time
(magpie.cpp:4265,4409-4427). Inputs are resident in HBM when the timed region
starts: the per-utterance preamble (encoder, XA K/V, 110-frame prefill) runs
once before warm-up; re-decoding re-initialises every per-step state on the
device, so each step is a complete, identical synthesis of the batch.

value = frames produced by all ranks / max-over-ranks wall time of the K timed
steps. Multi-GPU: one process per GPU (torchrun), independent utterances per
rank, no collective on the data path; `gloo` only carries the barrier and the
max-reduction of the timings ("scaling": "weak").

Weights are synthetic (no checkpoints offline) with the exact GGUF layout.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "magpie-tts.cpp_amd"))

import numpy as np  # noqa: E402

import magpie_amd as ma  # noqa: E402

# libmagpie_hip.so (hipcc 7.2, NEEDs libamdhip64.so.7) is loaded before anything can
# import torch, whose wheel bundles its own libamdhip64.so.7 (ROCm 7.0): the first
# object of that soname in the process is the one every later NEEDED entry binds to,
# so every N runs the kernels on /opt/rocm's runtime (tests/test_dist_cpu.py checks
# /proc/self/maps after this import sequence).
ma.load_library()
LIB_SHA16 = ma.lib_sha16()  # the committed PMC profiles name the build they counted

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
MFMA_F16_PEAK_TFS = 2500.0  # dense f16/bf16 MFMA peak (MI355X_MICROARCH.md; no sparsity)
CODEC_FLOP_PER_FRAME = 2.447e9  # 1.2234 G MAC per codec frame
CODEC_CHUNK = 32  # the CLI decodes stateless 32-frame chunks (magpie-tts.cpp:181-206)
FRAMES = 256
SCALE_BATCH = 8  # configs[3]: batch 64 split 8 per GPU
TEXT_TOKENS = 64
PMC_TRAFFIC = "r06fin_pmc_decode_f32_b1.json"  # per-op HBM bytes of the N=1 workload (tools_dev/pmc_report.py)
PMC_CODEC = "r06fin_pmc_codec.json"  # codec MFMA busy cycles + bytes per kernel (tools_dev/pmc_report.py)


def decoder_bytes_per_frame(B: int, L_mean: float, T: int, dec_layers: int = 12, weights: str = "f32") -> float:
    """Algorithmic HBM bytes per frame, f32 KV. weights="bf16": the
    decode projections (decoder qkv/o/ff1/ff2 = 7,077,888 params per layer; LT
    layer + 8 heads = 4,931,584 params) at 2 B, the rest f32."""
    W_dec = dec_layers * 7_276_800 + 768
    W_lt = 5_147_200
    per_utt = 73_728 * L_mean * dec_layers / 12 + 12_288 * T * dec_layers / 12 + 49_152 + 73_728 * dec_layers / 12
    if weights == "bf16":
        half = dec_layers * 7_077_888 + 4_931_584
        return (2.0 * half + 4.0 * (W_dec + W_lt - half)) / B + per_utt
    return 4.0 * (W_dec + W_lt) / B + per_utt


def _decode_fps(dev, B, frames, steps=2):
    ms = []
    for _ in range(steps):
        ms.append(dev.decode(B, frames).decode_ms)
    return B * frames * 1e3 / float(np.median(ms))


def measure_extra(model_path: str, codec_path, args) -> dict:
    """Throughput of the BASELINE configs' other shapes on this one GPU (fixed-length
    greedy decode, same synthetic prompts): bf16 projections at batch 1, 8
    (configs[3]'s per-GPU share of batch 64) and 16 (configs[2]), and at 8 / 16 with a
    bf16 SA cache as well; Q8_0 weights at
    batch 1 and 16 (int8 MFMA) and 60 s of long-form streaming (configs[4]); and the streaming path
    (sentence streaming, 4-frame codec chunks): time to first audio and real-time
    factor of one utterance."""
    out = {}
    dev = ma.Device(model_path, weights="bf16")
    for B in (1, 8, 16):
        toks = [ma.synthetic_tokens(args.tokens, seed=1000 + b) for b in range(B)]
        dev.synthesize(toks, speakers=[b % 5 for b in range(B)], max_dec_steps=args.frames, ignore_eos=True)
        out[f"bf16_batch{B}_fps"] = round(_decode_fps(dev, B, args.frames), 1)
    dev.close()
    # the same bf16 batches with the SA cache in bf16 too (mp_hip_set_kv_mode MP_KV_BF16: rows
    # rounded on append; half the attention bytes, which dominate from 8 slots up)
    dev = ma.Device(model_path, weights="bf16", kv="bf16")
    for B in (8, 16):
        toks = [ma.synthetic_tokens(args.tokens, seed=1000 + b) for b in range(B)]
        dev.synthesize(toks, speakers=[b % 5 for b in range(B)], max_dec_steps=args.frames, ignore_eos=True)
        out[f"bf16_kv16_batch{B}_fps"] = round(_decode_fps(dev, B, args.frames), 1)
    dev.close()
    # the reference converter's other file types at batch 1: F16 (ggml F16 mul_mat
    # semantics, f16 MFMA) and Q4_0 (on the Q8_0 kernels, int8 q - 8)
    for dt, wm in (("f16", "f16"), ("q4_0", "q4")):
        pth = os.path.join(os.path.dirname(model_path), f"magpie_357m_{dt}_k32.gguf")
        ma.synth_gguf(pth, dtype=dt, lt_head_scale=ma.DECISIVE)
        dev = ma.Device(pth, weights=wm)
        dev.synthesize([ma.synthetic_tokens(args.tokens, seed=1000)], speakers=[0], max_dec_steps=args.frames,
                       ignore_eos=True)
        out[f"{wm}_batch1_fps"] = round(_decode_fps(dev, 1, args.frames), 1)
        dev.close()
    # configs[4]: Q8_0 GGUF (the reference converter's default patterns), 60 s of
    # long-form audio streamed sentence by sentence with 4-frame codec chunks; the
    # sentences run as one device batch (magpie_synthesize_streaming's sentence
    # batching), fixed 216 frames each (EOS masked) -> 6 x 216 = 1296 frames = 60.2 s.
    q8_path = os.path.join(os.path.dirname(model_path), "magpie_357m_q8_k32.gguf")
    ma.synth_gguf(q8_path, dtype="q8_0", lt_head_scale=ma.DECISIVE)
    dev = ma.Device(q8_path, weights="q8")
    tok1 = [ma.synthetic_tokens(args.tokens, seed=1000)]
    dev.synthesize(tok1, speakers=[0], max_dec_steps=args.frames, ignore_eos=True)
    out["q8_batch1_fps"] = round(_decode_fps(dev, 1, args.frames), 1)
    toks16 = [ma.synthetic_tokens(args.tokens, seed=1000 + b) for b in range(16)]
    dev.synthesize(toks16, speakers=[b % 5 for b in range(16)], max_dec_steps=args.frames, ignore_eos=True)
    out["q8_batch16_fps"] = round(_decode_fps(dev, 16, args.frames), 1)
    if codec_path:
        cdc = ma.Codec(codec_path)
        sents = [ma.synthetic_tokens(40, seed=5000 + i) for i in range(6)]
        dev.synthesize_stream(cdc, sents[:1], lambda u, a: True, max_dec_steps=8, ignore_eos=True)  # warm-up
        n = [0]
        first = [None]
        t0 = time.perf_counter()

        def on_audio_q8(u, a):
            if first[0] is None:
                first[0] = time.perf_counter() - t0
            n[0] += len(a)
            return True
        codes, total, tm = dev.synthesize_stream(cdc, sents, on_audio_q8, max_dec_steps=216, ignore_eos=True)
        wall = time.perf_counter() - t0
        audio_s = total / 22050.0
        out["q8_longform_60s"] = {"sentences": len(sents), "frames": int(sum(len(c) for c in codes)),
                                  "audio_s": round(audio_s, 1), "wall_s": round(wall, 3),
                                  "rtf": round(audio_s / wall, 1), "first_audio_ms": round(first[0] * 1e3, 2),
                                  "chunk_frames": 4}
        cdc.close()
    dev.close()
    if codec_path:
        dev = ma.Device(model_path)
        cdc = ma.Codec(codec_path)
        tok = [ma.synthetic_tokens(args.tokens, seed=1000)]
        dev.synthesize_stream(cdc, tok, lambda u, a: True, max_dec_steps=32)  # warm-up
        t0 = time.perf_counter()
        n = [0]

        def on_audio(u, a):
            n[0] += len(a)
            return True
        codes, total, tm = dev.synthesize_stream(cdc, tok, on_audio, max_dec_steps=args.frames)
        wall = time.perf_counter() - t0
        out["stream_f32_batch1"] = {"frames": int(len(codes[0])), "first_audio_ms": round(tm.preamble_ms +
                                    tm.first_audio_ms, 2), "preamble_ms": round(tm.preamble_ms, 2),
                                    "rtf": round(total / 22050.0 / wall, 1), "chunk_frames": 4}
        cdc.close()
        dev.close()
    if codec_path:
        out["configs2_e2e"] = measure_configs2_e2e(model_path, codec_path, args)
    return out


def measure_configs2_e2e(model_path: str, codec_path: str, args) -> dict:
    """configs[2] end to end: bf16, 16 utterances, codes -> waveform on the device. The
    decode runs on the model's stream; as every slot completes a 32-frame chunk (the CLI's
    stateless chunks, magpie-tts.cpp:181-206) the codec decodes it on its own stream while
    the decode continues (mp_hip_decode_stream, frames_per_chunk = 32). Reported against
    the decode alone and against the serial form (decode, then the codec over all chunks)
    measured in the same run on the same prompts."""
    B, F = 16, args.frames
    dev = ma.Device(model_path, weights="bf16")
    cdc = ma.Codec(codec_path)
    toks = [ma.synthetic_tokens(args.tokens, seed=1000 + b) for b in range(B)]
    spk = [b % 5 for b in range(B)]
    r = dev.synthesize(toks, speakers=spk, max_dec_steps=F, ignore_eos=True)
    dec_ms = []
    for _ in range(3):
        dec_ms.append(dev.decode(B, F).decode_ms)
    chunks = np.stack([c[s0:s0 + CODEC_CHUNK].T for c in r.codes for s0 in range(0, len(c), CODEC_CHUNK)
                       if len(c[s0:s0 + CODEC_CHUNK]) == CODEC_CHUNK]).astype(np.int32)
    cdc.decode_chunks(chunks)  # warm-up
    cod_ms = []
    for _ in range(3):
        t0 = time.perf_counter()
        cdc.decode_chunks(chunks)
        cod_ms.append((time.perf_counter() - t0) * 1e3)
    n = [0]

    def on_audio(u, a):
        n[0] += len(a)
        return True
    dev.synthesize_stream(cdc, toks, on_audio, speakers=spk, max_dec_steps=F, frames_per_chunk=CODEC_CHUNK,
                          ignore_eos=True)  # warm-up (and the preamble, outside the timing below)
    walls = []
    for _ in range(3):
        n[0] = 0
        t0 = time.perf_counter()
        codes, total, tm = dev.decode_stream_only(cdc, on_audio, B, F, CODEC_CHUNK)
        walls.append(time.perf_counter() - t0)
    wall = float(np.median(walls))
    frames = B * F
    dec = float(np.median(dec_ms)) * 1e-3
    serial = dec + float(np.median(cod_ms)) * 1e-3
    cdc.close()
    dev.close()
    return {"workload": f"Magpie-357M bf16, batch={B}, {F} frames/utterance, T={args.tokens}, codes -> waveform "
                        f"({CODEC_CHUNK}-frame codec chunks overlapped with the decode on a second stream)",
            "frames": frames, "samples": int(n[0]), "wall_s": round(wall, 4),
            "fps": round(frames / wall, 1), "rtf": round(n[0] / 22050.0 / wall, 1),
            "decode_only_fps": round(frames / dec, 1), "serial_fps": round(frames / serial, 1),
            "e2e_over_decode_only": round(dec / wall, 4)}


def spawn_ranks(n: int) -> int:
    """`bench.py --gpus N` run directly (no torchrun env): start N ranks, one
    process per GPU, through torch.distributed.run on 127.0.0.1 as CHILD
    processes (this process never touches the GPU) and return their exit code."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="GPUs of this node, one rank each")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=None,
                    help="utterances per GPU (default: configs[1]'s 1 at N=1, configs[3]'s 8 at N>1)")
    ap.add_argument("--frames", type=int, default=FRAMES)
    ap.add_argument("--tokens", type=int, default=TEXT_TOKENS)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=4,
                    help="oracle threads for cpu_baseline (ggml's default n_threads, magpie.h:298,306)")
    ap.add_argument("--profile-ops", type=int, default=32, help="in-situ event-timed iterations for the op table")
    ap.add_argument("--no-codec", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the bf16 batch / streaming measurements")
    ap.add_argument("--dry-run", action="store_true",
                    help="resolve ranks / workload, rendezvous over gloo, print one line per rank, no GPU work")
    ap.add_argument("--weights", choices=["f32", "bf16"], default=None,
                    help="f32 = configs[1]; bf16 = configs[2]/[3] (decode projections on bf16 MFMA, batch <= 16); "
                         "default f32 at N=1, bf16 at N>1")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU")
    # N=1: configs[1] (f32, one utterance); N>1: configs[3] (bf16, 8 utterances per GPU)
    if args.weights is None:
        args.weights = "f32" if world == 1 else "bf16"
    if args.batch is None:
        args.batch = 1 if world == 1 else 8
    dist = None
    if world > 1:
        import torch.distributed as dist  # noqa: E402  (gloo: barrier + max only)
        dist.init_process_group("gloo")
    if args.dry_run:
        seen = [None] * world
        if dist is not None:
            dist.all_gather_object(seen, rank)
            dist.destroy_process_group()
        else:
            seen = [rank]
        # one write(2) per line: the ranks share the launcher's stdout pipe
        os.write(1, (json.dumps({"rank": rank, "local_rank": local, "world": world, "ranks_seen": seen,
                                 "weights": args.weights, "batch_per_gpu": args.batch,
                                 "scaling_baseline": {"weights": "bf16", "batch_per_gpu": SCALE_BATCH,
                                                      "measured": "rank 0 alone" if world > 1 else "after the headline"}})
                     + "\n").encode())
        return
    # one rank per GPU; with fewer GPUs than ranks (a rehearsal) ranks share devices
    ndev = ma.device_count()
    if ndev < 1:
        sys.exit("bench.py: no HIP device visible")
    device = local % ndev

    cache = os.environ.get("MAGPIE_CACHE", "/tmp/magpie_amd_cache")
    os.makedirs(cache, exist_ok=True)
    # the parity tests' model (decisive LT heads; the shapes, bytes and timings are those of any Magpie-357M)
    model_path = os.path.join(cache, "magpie_357m_f32_k32.gguf")
    if rank == 0 or world == 1:
        ma.synth_gguf(model_path, lt_head_scale=ma.DECISIVE)
    if dist is not None:
        dist.barrier()
        ma.synth_gguf(model_path, lt_head_scale=ma.DECISIVE)  # no-op once rank 0 wrote it

    dev = ma.Device(model_path, device=device, weights=args.weights)
    B = args.batch
    toks = [ma.synthetic_tokens(args.tokens, seed=1000 + rank * B + b) for b in range(B)]
    speakers = [(rank * B + b) % 5 for b in range(B)]

    # preamble (untimed, inputs resident) + warm-up decodes
    t_pre = time.perf_counter()
    r = dev.synthesize(toks, speakers=speakers, max_dec_steps=args.frames, ignore_eos=True)
    e2e_first_s = time.perf_counter() - t_pre
    preamble_ms = r.preamble_ms
    for _ in range(max(args.warmup - 1, 0)):
        dev.decode(B, args.frames)

    def barrier():
        if dist is not None:
            dist.barrier()

    def timed_decodes():
        t0 = time.perf_counter()
        ms, fr = [], 0
        for _ in range(args.steps):
            res = dev.decode(B, args.frames)  # synchronises its stream before returning
            ms.append(res.decode_ms)
            fr += int(res.n_frames.sum())
        return time.perf_counter() - t0, ms, fr, res

    # N > 1: the like-for-like 1-GPU point of the weak-scaling curve, measured in this
    # run on this node: rank 0 decodes its share alone (the other ranks wait at the
    # barrier, their GPUs idle), then every rank decodes together
    solo = None
    if dist is not None:
        barrier()
        if rank == 0:
            s_el, _, s_fr, _ = timed_decodes()
            solo = s_fr / s_el
        barrier()

    barrier()
    elapsed, decode_ms, frames, rr = timed_decodes()
    barrier()
    assert frames == args.steps * B * args.frames, f"expected fixed-length output, got {frames} frames"

    t_max = elapsed
    per_rank = [{"rank": rank, "device": device, "frames": frames, "s": round(elapsed, 4),
                 "fps": round(frames / elapsed, 1)}]
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        t_max = float(t.item())
        allr = [None] * world
        dist.all_gather_object(allr, per_rank[0])
        per_rank = allr
    total_frames = sum(r["frames"] for r in per_rank)
    value = total_frames / t_max
    ms_per_step = 1e3 * t_max / args.steps

    # ---- weak-scaling baseline: configs[3]'s per-GPU share (bf16, 8 utterances per GPU)
    # on ONE GPU. At N > 1 that is the workload itself, timed on rank 0 alone above;
    # at N = 1 (configs[1], f32 batch 1) it is timed here, after the headline decode, so a
    # SCALE series divides like by like: efficiency(N) = value(N) / (N x this value).
    scaling = None
    sb_desc = f"Magpie-357M bf16, batch={SCALE_BATCH}/GPU, {args.frames} frames/utterance, T={args.tokens} (configs[3] per-GPU share), one GPU"
    if dist is not None:
        scaling = {"workload": sb_desc if (args.weights, B) == ("bf16", SCALE_BATCH) else
                   f"this line's workload on one GPU", "value": round(solo, 2) if solo else None,
                   "unit": "frames/s", "measured": "rank 0 alone in this run (other ranks idle at a barrier)"}
    elif rank == 0:
        if (args.weights, B) == ("bf16", SCALE_BATCH):
            sval = value
        else:
            sdev = ma.Device(model_path, device=device, weights="bf16")
            stoks = [ma.synthetic_tokens(args.tokens, seed=1000 + b) for b in range(SCALE_BATCH)]
            sdev.synthesize(stoks, speakers=[b % 5 for b in range(SCALE_BATCH)], max_dec_steps=args.frames,
                            ignore_eos=True)
            t0 = time.perf_counter()
            sfr = 0
            for _ in range(args.steps):
                sfr += int(sdev.decode(SCALE_BATCH, args.frames).n_frames.sum())
            sval = sfr / (time.perf_counter() - t0)
            sdev.close()
        scaling = {"workload": sb_desc, "value": round(sval, 2), "unit": "frames/s",
                   "measured": "this run, after the headline decode, same steps"}

    # ---- nano-codec on the device: every utterance's 256 frames as 32-frame chunks
    codec = None
    codec_path = os.path.join(cache, "nano_codec.gguf")
    if not args.no_codec:
        if rank == 0 or world == 1:
            ma.synth_gguf(codec_path, kind="codec")
        if dist is not None:
            dist.barrier()
        cdc = ma.Codec(codec_path, device=device)
        chunks = []
        for b in range(B):
            c = rr.codes[b]
            for s0 in range(0, len(c), CODEC_CHUNK):
                ch = c[s0:s0 + CODEC_CHUNK]
                if len(ch) == CODEC_CHUNK:
                    chunks.append(ch.T)  # frame-major -> codebook-major (magpie-tts.cpp:186-191)
        chunks = np.stack(chunks).astype(np.int32)
        cdc.decode_chunks(chunks)  # warm-up
        cms = []
        for _ in range(3):
            audio = cdc.decode_chunks(chunks)
            cms.append(cdc.last_ms())
        cdc.close()
        codec_ms = float(np.median(cms))
        cframes = chunks.shape[0] * CODEC_CHUNK
        tfs = CODEC_FLOP_PER_FRAME * cframes / (codec_ms * 1e-3) / 1e12
        codec = {"frames": cframes, "ms": round(codec_ms, 3), "fps": round(cframes / (codec_ms * 1e-3), 1),
                 "tflops": round(tfs, 1), "mfma_f16_peak_tflops": MFMA_F16_PEAK_TFS,
                 "frac": round(tfs / MFMA_F16_PEAK_TFS, 4), "audio_peak": round(float(np.abs(audio).max()), 4)}
        pmc_codec = os.path.join(REPO, "profiles", PMC_CODEC)
        if os.path.exists(pmc_codec):  # counters of the same codec shape (tools_dev/pmc_report.py)
            pj = json.load(open(pmc_codec))
            sm = pj["summary"]
            stale = pj.get("lib_sha16") != LIB_SHA16  # counted on another build: not this run's kernels
            # MFMA utilisation: the MFMA FLOPs the codec issues per decode of this shape
            # (SQ_INSTS_VALU_MFMA_MOPS_F16 x 512, padding included) over the live decode
            # time above, against the dense f16 peak; traffic: FETCH_SIZE + WRITE_SIZE per
            # decode over the same live time (the PMC runs themselves are slowed by the
            # counters, so their own durations are not used)
            issued = None if stale else sm.get("per_decode_mfma_flops")
            nbytes = None if stale else sm.get("per_decode_bytes")
            pmc_chunks = sm.get("chunks", 8)
            scale = (cframes / CODEC_CHUNK) / pmc_chunks
            codec["pmc"] = {
                "mfma_util": round(issued * scale / (codec_ms * 1e-3) / (MFMA_F16_PEAK_TFS * 1e12), 4) if issued else None,
                "mfma_flops_issued_per_useful": round(issued / (CODEC_FLOP_PER_FRAME * pmc_chunks * CODEC_CHUNK), 3)
                if issued else None,
                "hbm_tbs": round(nbytes * scale / (codec_ms * 1e-3) / 1e12, 3) if nbytes else None,
                "bytes_per_decode": nbytes,
                "source": f"profiles/{PMC_CODEC}: MFMA op counts and FETCH_SIZE/WRITE_SIZE passes of the same "
                          f"{pmc_chunks} x {CODEC_CHUNK}-frame decode, over this run's live decode time",
                "pmc_lib_sha16": pj.get("lib_sha16"), "stale": stale}

    # ---- roofline of the dominant kernel, timed in situ: whole decode iterations
    # launched eagerly on the decode stream, each kernel through hipExtLaunchKernel
    # with a start/stop event pair that the dispatch itself stamps
    # (mp_hip_profile_ops_kev): the interval rocprofv3's kernel trace reports, in
    # the cache state a real frame leaves each op. The batch is first decoded to
    # mid-utterance (cache length L = 110 + frames/2 + 1, the mean over the decode),
    # so length-dependent kernels (attention) run at the average length of the
    # timed decode. Also recorded per op: the first-wave-start to last-wave-end span
    # from in-kernel timestamps (wave_span_us, mp_hip_profile_ops_ts) and a plain
    # event pair around the launch (event_pair_us, mp_hip_profile_ops).
    roofline = None
    op_table = {}
    if rank == 0:
        dev.synthesize(toks, speakers=speakers, max_dec_steps=args.frames // 2, ignore_eos=True)
        names = dev.ops()
        kev = dev.profile_ops_kev(iters=args.profile_ops)
        tsu = dev.profile_ops_ts(iters=args.profile_ops)
        us = dev.profile_ops(iters=args.profile_ops)
        groups = {}
        for i, n in enumerate(names):
            groups.setdefault(n, []).append(i)
        for n, idxs in groups.items():
            dur = float(np.mean([kev[i] for i in idxs]))
            own = [tsu[i] for i in idxs if tsu[i] > 0]
            rec = {"launches_per_frame": len(idxs), "avg_us": round(dur, 3),
                   "wave_span_us": round(float(np.mean(own)), 3) if own else None,
                   "event_pair_us": round(float(np.mean([us[i] for i in idxs])), 3),
                   "us_per_frame": round(dur * len(idxs), 2)}
            if n != "finalize":
                rec["bytes"] = dev.op_bytes(idxs[0])
                # back to back (one event pair around 50 launches; weights warm in L2/MALL)
                # (not for ops carrying an in-launch hand-off: relaunched with the same
                # iteration tag their consumers would not wait; the library refuses)
                try:
                    rec["b2b_us"] = round(dev.time_op(idxs[0], reps=50), 3)
                except ma.MagpieError:
                    rec["b2b_us"] = None
            op_table[n] = rec
        dom = max(((n, r) for n, r in op_table.items() if "bytes" in r), key=lambda kv: kv[1]["us_per_frame"])
        name, rec = dom
        achieved = rec["bytes"] / (rec["avg_us"] * 1e-6) / 1e9
        roofline = {"bound": "hbm", "kernel": name, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                    "algorithmic_bytes_per_launch": rec["bytes"], "avg_launch_us": rec["avg_us"],
                    "timing": "dispatch begin/end stamped on the kernel's own start/stop events "
                              "(hipExtLaunchKernel; the rocprofv3 kernel-trace interval), whole eager "
                              "iterations at the mid-utterance state (mp_hip_profile_ops_kev)"}
        # HBM bytes per launch from the committed PMC passes (tools_dev/pmc_collect.sh +
        # pmc_report.py: separate FETCH_SIZE / WRITE_SIZE passes, gfx950 FETCH_SIZE
        # correction for the 16 B/lane kernels)
        pmc_path = os.path.join(REPO, "profiles", PMC_TRAFFIC)
        if args.weights == "f32" and B == 1 and os.path.exists(pmc_path):
            pj = json.load(open(pmc_path))
            pmc_ops = pj["ops"] if pj.get("lib_sha16") == LIB_SHA16 else {}  # another build's counters: unused
            roofline["traffic_lib_sha16"] = pj.get("lib_sha16")
            roofline["lib_sha16"] = LIB_SHA16
            pmc = pmc_ops.get(name)
            if pmc:
                roofline["traffic"] = pmc["traffic_bytes"]
                roofline["traffic_source"] = f"profiles/{PMC_TRAFFIC} ({pmc['kernel']})"
            for n, r in op_table.items():
                if n in pmc_ops:
                    r["pmc_traffic_bytes"] = pmc_ops[n]["traffic_bytes"]

    # ---- CPU baseline: the oracle (C restatement, f32 accumulation) on the host cores
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, REPO)
        from oracle import oracle as orc  # cpu_baseline leg only
        res = orc.time_decode_fps(model_path, toks[0], args.frames, threads=args.cpu_threads, acc64=False)
        cpu = {"value": round(res["frames"] / res["decode_s"], 2), "unit": "frames/s", "cores": args.cpu_threads,
               "kind": "port",
               "sample": f"1 utterance x {res['frames']} frames (T={args.tokens}), decode loop only "
                         f"(preamble {res['preamble_s']:.2f}s excluded), oracle f32-accumulate mode",
               "cpu_model": cpu_model_name()}
        # also at every core this process may use. The GPU box leases 16 CPUs per
        # GPU (its OMP_NUM_THREADS) out of a machine whose affinity mask shows all of them; the
        # operators' rule caps a one-GPU job's worker pool at that share, so it is a named
        # cap here, not the machine's core count.
        LEASE_CAP = 16
        nall = max(1, min(LEASE_CAP, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))))
        if nall != args.cpu_threads:
            ra = orc.time_decode_fps(model_path, toks[0], args.frames, threads=nall, acc64=False)
            try:
                visible = len(os.sched_getaffinity(0))
            except (AttributeError, OSError):
                visible = os.cpu_count() or 1
            cpu["all_cores"] = {"value": round(ra["frames"] / ra["decode_s"], 2), "cores": nall,
                                "cores_cap": LEASE_CAP,
                                "note": f"the lease's CPU share: OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS', '-')}, "
                                        f"{visible} CPUs in this process's affinity mask, "
                                        f"{os.cpu_count()} on the machine"}

    # ---- the other BASELINE configs' shapes on this GPU (rank 0 at N=1 only)
    extra = None
    if rank == 0 and world == 1 and not args.no_extra:
        extra = measure_extra(model_path, codec_path if not args.no_codec else None, args)

    if rank == 0:
        L_mean = 110 + (args.frames + 1) / 2.0  # keys 111..366 over BOS + 255 steps
        bpf = decoder_bytes_per_frame(B, L_mean, args.tokens, weights=args.weights)
        fps_per_gpu = value / world
        line = {
            "metric": "audio-codec frames/sec (decode loop), Magpie-357M",
            "value": round(value, 2),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.weights,
            "data": "synthetic (deterministic random weights, exact GGUF layout; synthetic T=64 prompts)",
            "config": {"workload": f"Magpie-357M {args.weights}, batch={B}/GPU, {args.frames} frames/utterance, "
                                   f"T={args.tokens}, greedy, EOS masked "
                                   f"({'configs[1]' if args.weights == 'f32' else 'configs[2]/[3] shape'})",
                       "global_batch": B * world, "frames_per_utterance": args.frames, "text_tokens": args.tokens,
                       "parallelism": f"replicas x{world} (utterance-partitioned, no collectives)"},
            "ranks": {"seen": len(per_rank), "devices_visible": ndev, "per_rank": per_rank},
            "rtf_per_stream": round(value / world / B / ma.FRAMES_PER_SECOND, 2),
            "decode_fps_events": round(B * args.frames * 1e3 / float(np.mean(decode_ms)), 2),
            "e2e_fps_first_call": round(B * args.frames / e2e_first_s, 2),
            "preamble_ms": round(preamble_ms, 2),
            "codec": codec,
            "e2e_fps_per_gpu": (round(B * args.frames / ((ms_per_step + preamble_ms + (codec["ms"] if codec else 0))
                                                        * 1e-3), 1)),
            "rtf_e2e_per_stream": (round(args.frames / ma.FRAMES_PER_SECOND /
                                         ((ms_per_step + preamble_ms + (codec["ms"] if codec else 0)) * 1e-3), 1)),
            "decode_roofline": {"bytes_per_frame": round(bpf), "achieved_GBs": round(bpf * fps_per_gpu / 1e9, 1),
                                "frac": round(bpf * fps_per_gpu / 1e9 / HBM_PEAK_GBS, 4)},
            "scaling_baseline": scaling,
            "roofline": roofline,
            "cpu_baseline": cpu,
            "ops": op_table,
            "extra_configs": extra,
        }
        print(json.dumps(line), flush=True)
    dev.close()
    if dist is not None:
        dist.destroy_process_group()


def cpu_model_name() -> str:
    """The host CPU the cpu_baseline ran on (/proc/cpuinfo 'model name')."""
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


if __name__ == "__main__":
    main()
