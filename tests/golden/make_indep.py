#!/usr/bin/env python3
"""Independent f64 restatement of the reference's decode path and nano-codec,
written from the reference source (not from oracle/magpie_oracle.c), and the
fixtures it produces (tests/golden/indep_*.npz) that hold the C oracle to it
(tests/test_indep_cpu.py).

*** TEST INFRASTRUCTURE (build side only). *** Nothing here travels to the GPU box
or is loaded by the product; it reads a synthetic GGUF with its own reader
(tests/gguf_raw.py, tests/gguf_kv.py) and computes everything in numpy float64.

Each function cites the reference lines it restates (/root/reference/src/...):
  layer_norm            magpie.cpp:2237-2259 (ggml_norm: (x - mean) / sqrt(var + eps), * w; no bias)
  gelu                  ggml_gelu (tanh form, magpie.cpp:1799 / 1869; the f16 table of the
                        CPU backend is not restated: the oracle's plain-f32 mode is compared)
  qkv_split + attend    magpie.cpp:1477-1575 (qkv split q|k|v, heads of d/heads, K^T Q / sqrt(dh),
                        causal mask j <= i filled at 2343-2353 / 1224-1234, softmax over keys,
                        o_net); the cached form 3395-3480 and the batched prefill 3911-3988
                        (ggml_diag_mask_inf) are the same arithmetic on a longer key range
  conv_ffn              magpie.cpp:1769-1917 (k = 1: pointwise; k = 3: causal, left pad k-1,
                        tap k reads x[t - (k-1) + k], ggml_permute(w, 2, 0, 1, 3) = w[f][m][k])
  encoder               magpie.cpp:1929-1995, 2284-2374 (text embedding rows, + pos rows 0..T-1,
                        layers, final norm)
  xa_kv                 magpie.cpp:1663-1711 (LN(enc) with norm_xattn_memory, kv_net, K = rows
                        0..127, V = rows 128..255 of the [256] output)
  cross_attention       magpie.cpp:1713-1767 (q_net, 1 head x 128, K^T q / sqrt(128), o_net)
  decoder_layer         magpie.cpp:3484-3528 (cached) / 3991-4060 (batched prefill)
  synthesize            magpie.cpp:4063-4432 (baked context rows of the speaker, + pos 0..109,
                        prefill into cache rows 0..109; BOS frame = sum of the 8 audio_emb rows of
                        code 2016 / 8 + pos[110]; per step: LT on the final-normed hidden,
                        EOS rule 4340-4352, frame embedding 2746-2787 + pos[cache_pos])
  lt_sample_all         magpie.cpp:1113-1317 in the reference's RECOMPUTE form: for codebook cb
                        the whole sequence (in_proj(h), in_proj(emb_c(code_c)) ...) + pos rows
                        0..cb runs through the layer (946-976) with a causal mask, the last
                        position's out_proj[cb] (1037-1048); forbidden ids 2016, 2018..2023
                        (+ 2017 while step < 4), first-max argmax (1250-1258)
  codec_decode          nano-codec.cpp:676-715, 758-845: FSQ (721-752), causal conv1d
                        (429-466, left pad (K-1) d), HalfSnake (376-426: first numel(alpha)
                        channels x + sin^2(a x) / a, the rest leaky 0.01), grouped ConvTranspose
                        (481-565: group g = input channels 2g, 2g+1, out length (T-1) s + K,
                        trimmed right by K - s), residual block (568-599), HiFiGAN block
                        dilations 1, 3, 5 (602-616), ResLayer mean of 3 (619-641), post conv + tanh

usage: python tests/golden/make_indep.py [--small-only]
  (writes tests/golden/indep_small.npz, indep_codec.npz; then indep_codec32.npz, a full 32-frame
  codec chunk, and indep_full.npz, 32 frames of Magpie-357M's 12-layer / 6-encoder-layer shape)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "magpie-tts.cpp_amd"))

from gguf_raw import GgufRaw  # noqa: E402

# magpie.h:40-95 defaults (the synthetic file writes the same values)
D, H, DH, DFF = 768, 12, 64, 3072
XA_D = 128
LT_D, LT_F, VCB = 256, 1024, 2024
CTX_FRAMES = 110
AUDIO_BOS, AUDIO_EOS = 2016, 2017
EPS = 1e-5
# nano-codec: magpie.h:655-678
UP_RATES = (8, 8, 4, 2, 2)


class Weights:
    def __init__(self, path):
        self.g = GgufRaw(path)

    def __call__(self, name):
        return self.g.f32(name).astype(np.float64)


# ------------------------------------------------------------------ magpie decode path
def layer_norm(x, w):
    mu = x.mean(axis=-1, keepdims=True)
    var = ((x - mu) ** 2).mean(axis=-1, keepdims=True)
    return (x - mu) / np.sqrt(var + EPS) * w


def gelu(x):
    return 0.5 * x * (1.0 + np.tanh(np.sqrt(2.0 / np.pi) * x * (1.0 + 0.044715 * x * x)))


def softmax(s):
    s = s - s.max(axis=-1, keepdims=True)
    e = np.exp(s)
    return e / e.sum(axis=-1, keepdims=True)


def qkv_split(x, wqkv):
    """x: [S, d] normalised rows -> q, k, v [S, d] (qkv_net output rows 0..d-1 | d..2d-1 | 2d..3d-1)"""
    d = x.shape[1]
    qkv = x @ wqkv.T
    return qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:]


def attend(q, k, v, heads, causal_offset):
    """q: [S, d] queries at absolute positions causal_offset .. causal_offset+S-1; k, v: [L, d]
    keys 0..L-1. Query at position p sees keys j <= p."""
    S, d = q.shape
    L = k.shape[0]
    dh = d // heads
    out = np.zeros((S, d))
    for h in range(heads):
        sl = slice(h * dh, (h + 1) * dh)
        sc = q[:, sl] @ k[:, sl].T / np.sqrt(dh)
        pos = causal_offset + np.arange(S)[:, None]
        sc = np.where(np.arange(L)[None, :] <= pos, sc, -np.inf)
        out[:, sl] = softmax(sc) @ v[:, sl]
    return out


def conv_ffn(x, w1, w2, ksize):
    """x: [S, d]; w1: [f][d][k], w2: [d][f][k] (PyTorch Conv1d layout). Causal, left pad k-1."""
    S = x.shape[0]

    def cconv(inp, w):
        pad = np.concatenate([np.zeros((ksize - 1, inp.shape[1])), inp], axis=0)
        out = np.zeros((S, w.shape[0]))
        for tap in range(ksize):
            out += pad[tap:tap + S] @ w[:, :, tap].T
        return out

    return cconv(gelu(cconv(x, w1)), w2)


class Magpie:
    def __init__(self, path):
        W = Weights(path)
        self.W = W
        n_enc = sum(1 for n in W.g.tensors if n.startswith("encoder.layers.") and n.endswith("norm_self.weight"))
        n_dec = sum(1 for n in W.g.tensors if n.startswith("decoder.layers.") and n.endswith("norm_self.weight"))
        self.n_enc, self.n_dec = n_enc, n_dec
        self.text_emb = W("text_embedding.weight")
        self.enc_pos = W("encoder.position_embeddings.weight")
        self.enc = []
        for l in range(n_enc):
            p = f"encoder.layers.{l}."
            self.enc.append({k: W(p + n) for k, n in [
                ("ln1", "norm_self.weight"), ("qkv", "self_attention.qkv_net.weight"),
                ("o", "self_attention.o_net.weight"), ("ln2", "norm_pos_ff.weight"),
                ("f1", "pos_ff.proj.conv.weight"), ("f2", "pos_ff.o_net.conv.weight")]})
        self.enc_norm = W("encoder.norm_out.weight")
        self.dec_pos = W("decoder.position_embeddings.weight")
        self.dec = []
        for l in range(n_dec):
            p = f"decoder.layers.{l}."
            self.dec.append({k: W(p + n) for k, n in [
                ("ln1", "norm_self.weight"), ("qkv", "self_attention.qkv_net.weight"),
                ("o", "self_attention.o_net.weight"), ("lnq", "norm_xattn_query.weight"),
                ("xq", "cross_attention.q_net.weight"), ("xkv", "cross_attention.kv_net.weight"),
                ("xo", "cross_attention.o_net.weight"), ("lnm", "norm_xattn_memory.weight"),
                ("ln2", "norm_pos_ff.weight"), ("f1", "pos_ff.proj.conv.weight"),
                ("f2", "pos_ff.o_net.conv.weight")]})
        self.dec_norm = W("decoder.norm_out.weight")
        self.audio_emb = [W(f"audio_embeddings.{c}.weight") for c in range(8)]
        self.baked = W("baked_context_embedding.weight")
        self.lt_in_w = W("local_transformer_in_projection.weight")
        self.lt_in_b = W("local_transformer_in_projection.bias")
        self.lt_pos = W("local_transformer.position_embeddings.weight")
        p = "local_transformer.layers.0."
        self.lt = {k: W(p + n) for k, n in [
            ("ln1", "norm_self.weight"), ("qkv", "self_attention.qkv_net.weight"), ("o", "self_attention.o_net.weight"),
            ("ln2", "norm_pos_ff.weight"), ("f1", "pos_ff.proj.conv.weight"), ("f2", "pos_ff.o_net.conv.weight")]}
        self.lt_out_w = [W(f"local_transformer_out_projections.{c}.weight") for c in range(8)]
        self.lt_out_b = [W(f"local_transformer_out_projections.{c}.bias") for c in range(8)]

    # magpie.cpp:1929-1995, 2284-2374
    def encode(self, tokens):
        T = len(tokens)
        x = self.text_emb[np.asarray(tokens)] + self.enc_pos[:T]
        for L in self.enc:
            h = layer_norm(x, L["ln1"])
            q, k, v = qkv_split(h, L["qkv"])
            x = attend(q, k, v, H, 0) @ L["o"].T + x
            h = layer_norm(x, L["ln2"])
            x = conv_ffn(h, L["f1"], L["f2"], L["f1"].shape[2]) + x
        return layer_norm(x, self.enc_norm)

    # one decoder layer over S new rows at cache positions pos0..pos0+S-1 (3484-3528, 3991-4060)
    def dec_layer(self, l, x, pos0, cache, xk, xv):
        L = self.dec[l]
        h = layer_norm(x, L["ln1"])
        q, k, v = qkv_split(h, L["qkv"])
        kc, vc = cache[l]
        S = x.shape[0]
        kc[pos0:pos0 + S], vc[pos0:pos0 + S] = k, v
        x = attend(q, kc[:pos0 + S], vc[:pos0 + S], H, pos0) @ L["o"].T + x
        hq = layer_norm(x, L["lnq"])
        qx = hq @ L["xq"].T
        a = softmax(qx @ xk[l].T / np.sqrt(XA_D)) @ xv[l]
        x = a @ L["xo"].T + x
        h = layer_norm(x, L["ln2"])
        return conv_ffn(h, L["f1"], L["f2"], 1) + x

    # magpie.cpp:2746-2787
    def frame_embedding(self, codes):
        s = self.audio_emb[0][codes[0]].copy()
        for c in range(1, 8):
            s = s + self.audio_emb[c][codes[c]]
        return s * (1.0 / 8.0)

    # magpie.cpp:946-976 on a whole sequence (recompute form), 1015-1034
    def lt_layer(self, seq):
        S = seq.shape[0]
        x = seq + self.lt_pos[:S]
        h = layer_norm(x, self.lt["ln1"])
        q, k, v = qkv_split(h, self.lt["qkv"])
        x = attend(q, k, v, 1, 0) @ self.lt["o"].T + x
        h = layer_norm(x, self.lt["ln2"])
        return conv_ffn(h, self.lt["f1"], self.lt["f2"], 1) + x

    # magpie.cpp:1113-1317, greedy (temperature < 0.01)
    def lt_sample_all(self, hidden, forbid_eos):
        seq = [self.lt_in_w @ hidden + self.lt_in_b]
        codes, margins, logits_all = [], [], []
        forbidden = [AUDIO_BOS] + list(range(AUDIO_BOS + 2, AUDIO_BOS + 8)) + ([AUDIO_EOS] if forbid_eos else [])
        for cb in range(8):
            out = self.lt_layer(np.array(seq))
            logits = self.lt_out_w[cb] @ out[-1] + self.lt_out_b[cb]
            logits_all.append(logits.copy())
            logits[forbidden] = -np.inf
            am = int(np.argmax(logits))  # first maximal index
            top2 = np.sort(logits)[-2:]
            margins.append(top2[1] - top2[0])
            codes.append(am)
            if cb < 7:
                seq.append(self.lt_in_w @ self.audio_emb[cb][am] + self.lt_in_b)
        return codes, margins, logits_all

    # magpie.cpp:4063-4432 (graph reuse, greedy)
    def synthesize(self, tokens, speaker, max_steps):
        enc = self.encode(tokens)
        xk, xv = [], []
        for L in self.dec:
            kv = layer_norm(enc, L["lnm"]) @ L["xkv"].T
            xk.append(kv[:, :XA_D])
            xv.append(kv[:, XA_D:])
        max_seq = CTX_FRAMES + max_steps + 16
        cache = [(np.zeros((max_seq, D)), np.zeros((max_seq, D))) for _ in range(self.n_dec)]
        ctx = self.baked[speaker].reshape(CTX_FRAMES, D)
        x = ctx + self.dec_pos[:CTX_FRAMES]
        for l in range(self.n_dec):
            x = self.dec_layer(l, x, 0, cache, xk, xv)
        pos = CTX_FRAMES
        frames, hidden, margins, logits0 = [], [], [], []
        prev = [AUDIO_BOS] * 8
        for step in range(-1, max_steps):
            if step >= 0:
                codes, mg, lg = self.lt_sample_all(hidden[-1], forbid_eos=step < 4)
                margins.append(mg)
                logits0.append(lg[0])
                eos = any(c == AUDIO_EOS for c in codes)  # sampled == argmax at temperature 0
                if eos:
                    break
                frames.append(codes)
                if step + 1 >= max_steps:
                    break
                prev = codes
            x = (self.frame_embedding(prev) + self.dec_pos[pos])[None, :]
            for l in range(self.n_dec):
                x = self.dec_layer(l, x, pos, cache, xk, xv)
            hidden.append(layer_norm(x[0], self.dec_norm))
            pos += 1
        return {"enc": enc, "codes": np.array(frames, np.int32).reshape(-1, 8), "hidden": np.array(hidden),
                "margins": np.array(margins), "logits_cb0": np.array(logits0)}


# ------------------------------------------------------------------ nano-codec decoder
class Codec:
    def __init__(self, path):
        W = Weights(path)
        self.W = W
        self.pre_w, self.pre_b = W("dec.pre.weight"), W("dec.pre.bias")
        self.up = []
        for i in range(len(UP_RATES)):
            self.up.append((W(f"dec.act.{i}.activation.snake_act.alpha").ravel(), W(f"dec.up.{i}.c.weight"),
                            W(f"dec.up.{i}.c.bias").ravel()))
        self.rl = []
        for i in range(len(UP_RATES)):
            blocks = []
            for j in range(3):
                inner = []
                for k in range(3):
                    p = f"dec.rl.{i}.rb.{j}.rb.{k}."
                    inner.append((W(p + "in_act.alpha").ravel(), W(p + "in_conv.weight"), W(p + "in_conv.bias").ravel(),
                                  W(p + "sk_act.alpha").ravel(), W(p + "sk_conv.weight"), W(p + "sk_conv.bias").ravel()))
                blocks.append(inner)
            self.rl.append(blocks)
        self.post_alpha = W("dec.post_act.alpha").ravel()
        self.post_w, self.post_b = W("dec.post.weight"), W("dec.post.bias").ravel()

    # nano-codec.cpp:721-752
    @staticmethod
    def fsq(codes):
        """codes [8][n] -> latent [n][32]"""
        base, levels = (1, 8, 56, 336), (8, 7, 6, 6)
        n = codes.shape[1]
        lat = np.zeros((n, 32))
        for cb in range(8):
            for d in range(4):
                nonneg = (codes[cb] // base[d]) % levels[d]
                half = levels[d] // 2
                lat[:, cb * 4 + d] = (nonneg - half) / half
        return lat

    # nano-codec.cpp:376-426 (x: [T][C])
    @staticmethod
    def half_snake(x, alpha):
        n = alpha.size
        a = x[:, :n]
        first = a + np.sin(a * alpha) ** 2 / alpha
        b = x[:, n:]
        second = np.where(b >= 0, b, 0.01 * b)
        return np.concatenate([first, second], axis=1)

    # nano-codec.cpp:429-466: w [OC][IC][K], x [T][IC]
    @staticmethod
    def cconv(x, w, b, dil=1):
        K = w.shape[2]
        pad = (K - 1) * dil
        T = x.shape[0]
        xp = np.concatenate([np.zeros((pad, x.shape[1])), x], axis=0)
        out = np.zeros((T, w.shape[0]))
        for k in range(K):
            out += xp[k * dil:k * dil + T] @ w[:, :, k].T
        return out + b

    # nano-codec.cpp:481-565: w [IC][1][K], groups of 2 input channels per output channel
    @staticmethod
    def conv_t(x, w, b, s):
        T, IC = x.shape
        K = w.shape[2]
        OC = IC // 2
        full = np.zeros(((T - 1) * s + K, OC))
        for g in range(OC):
            for ic in (2 * g, 2 * g + 1):
                for t in range(T):
                    full[t * s:t * s + K, g] += x[t, ic] * w[ic, 0, :]
        return full[:T * s] + b

    def decode(self, codes):
        x = self.cconv(self.fsq(codes), self.pre_w, self.pre_b)
        for i, s in enumerate(UP_RATES):
            alpha, w, b = self.up[i]
            x = self.conv_t(self.half_snake(x, alpha), w, b, s)
            acc = None
            for j in range(3):
                h = x
                for k, dil in enumerate((1, 3, 5)):
                    ia, iw, ib, sa, sw, sb = self.rl[i][j][k]
                    r = self.cconv(self.half_snake(h, ia), iw, ib, dil)
                    r = self.cconv(self.half_snake(r, sa), sw, sb, 1)
                    h = h + r
                acc = h if acc is None else acc + h
            x = acc * (1.0 / 3.0)
        x = self.cconv(self.half_snake(x, self.post_alpha), self.post_w, self.post_b)
        return np.tanh(x[:, 0])


CASES = [  # (seed, T, speaker, max_steps)
    (1000, 24, 1, 16),
    (11, 40, 3, 12),
]
CODEC_CODES_SEED, CODEC_FRAMES = 5, 6
# the shipped shape: Magpie-357M's 12 decoder / 6 encoder layers, 32 frames of
# the bench's T = 64 prompt; and one full 32-frame codec chunk (the CLI's chunk,
# magpie-tts.cpp:181-206)
FULL_CASE = (1004, 64, 0, 32)  # the prompt seed whose 256 decisions have no near-tie (min margin 2.5e-3)
CODEC32_SEED, CODEC32_FRAMES = 7, 32


def main():
    import magpie_amd as ma
    cache = os.environ.get("MAGPIE_CACHE", "/tmp/magpie_amd_cache")
    os.makedirs(cache, exist_ok=True)
    path = ma.synth_gguf(os.path.join(cache, "magpie_small_l2e1_k32.gguf"), dec_layers=2, enc_layers=1,
                         lt_head_scale=ma.DECISIVE)
    m = Magpie(path)
    out = {}
    for i, (seed, T, spk, steps) in enumerate(CASES):
        tok = ma.synthetic_tokens(T, seed=seed)
        r = m.synthesize(tok, spk, steps)
        out[f"c{i}_tokens"] = tok
        out[f"c{i}_meta"] = np.array([spk, steps], np.int32)
        out[f"c{i}_enc"] = r["enc"]
        out[f"c{i}_codes"] = r["codes"]
        out[f"c{i}_hidden"] = r["hidden"]
        out[f"c{i}_margins"] = r["margins"]
        print(f"case {i}: {len(r['codes'])} frames, min margin {r['margins'].min():.4f}")
    np.savez_compressed(os.path.join(HERE, "indep_small.npz"), **out)

    cpath = ma.synth_gguf(os.path.join(cache, "nano_codec.gguf"), kind="codec")
    c = Codec(cpath)
    rng = np.random.default_rng(CODEC_CODES_SEED)
    codes = rng.integers(0, 2016, (8, CODEC_FRAMES)).astype(np.int32)
    audio = c.decode(codes)
    np.savez_compressed(os.path.join(HERE, "indep_codec.npz"), codes=codes, audio=audio)
    print(f"codec: {audio.size} samples, peak {np.abs(audio).max():.4f}")
    if "--small-only" in sys.argv:
        return
    # one full 32-frame chunk, stored as f32 (the values are within f32 rounding of the f64
    # restatement's; the bars are 1e-6 and up)
    codes = np.random.default_rng(CODEC32_SEED).integers(0, 2016, (8, CODEC32_FRAMES)).astype(np.int32)
    audio = c.decode(codes)
    np.savez_compressed(os.path.join(HERE, "indep_codec32.npz"), codes=codes, audio=audio.astype(np.float32))
    print(f"codec 32-frame chunk: {audio.size} samples, peak {np.abs(audio).max():.4f}")
    del c
    # Magpie-357M (12 / 6 layers), the bench's prompt: codes, margins and the hidden state after
    # every step (f32), 32 frames
    fpath = ma.synth_gguf(os.path.join(cache, "magpie_357m_f32_k32.gguf"), lt_head_scale=ma.DECISIVE)
    m = Magpie(fpath)
    seed, T, spk, steps = FULL_CASE
    tok = ma.synthetic_tokens(T, seed=seed)
    r = m.synthesize(tok, spk, steps)
    np.savez_compressed(os.path.join(HERE, "indep_full.npz"), tokens=tok, meta=np.array([spk, steps], np.int32),
                        codes=r["codes"], hidden=r["hidden"].astype(np.float32), margins=r["margins"])
    print(f"Magpie-357M: {len(r['codes'])} frames, min margin {r['margins'].min():.4f}")


if __name__ == "__main__":
    main()
