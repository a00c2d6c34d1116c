"""Offline check of a diag_ops.py divergence (ff1, layer 0): recompute the
divergent workgroup's rows in float64 under stale-input hypotheses (diagnostic)."""
import struct, sys, numpy as np, math
sys.path.insert(0, "magpie-tts.cpp_amd")
import magpie_amd as ma
p = ma.synth_gguf("/tmp/magpie_amd_cache/magpie_small_l2e1.gguf", dec_layers=2, enc_layers=1)
def tensors(path):
    f = open(path, "rb"); data = f.read()
    o = 4; ver, = struct.unpack_from("<I", data, o); o += 4
    nt, nkv = struct.unpack_from("<QQ", data, o); o += 16
    sizes = {0:1,1:1,2:2,3:2,4:4,5:4,6:4,7:1,10:8,11:8,12:8}
    def rstr(o):
        n, = struct.unpack_from("<Q", data, o); return data[o+8:o+8+n], o+8+n
    def rval(t, o):
        if t == 8: return rstr(o)
        if t == 9:
            et, n = struct.unpack_from("<IQ", data, o); o += 12; v = []
            for _ in range(n): x, o = rval(et, o); v.append(x)
            return v, o
        return data[o:o+sizes[t]], o + sizes[t]
    align = 32
    for _ in range(nkv):
        k, o = rstr(o); t, = struct.unpack_from("<I", data, o); o += 4; v, o = rval(t, o)
        if k == b"general.alignment": align = struct.unpack("<I", v)[0]
    infos = []
    for _ in range(nt):
        nm, o = rstr(o); nd, = struct.unpack_from("<I", data, o); o += 4
        dims = struct.unpack_from("<%dQ" % nd, data, o); o += 8 * nd
        ty, off = struct.unpack_from("<IQ", data, o); o += 12
        infos.append((nm.decode(), dims, ty, off))
    base = (o + align - 1) // align * align
    out = {}
    for nm, dims, ty, off in infos:
        if ty != 0: continue
        n = int(np.prod(dims))
        out[nm] = np.frombuffer(data, np.float32, n, base + off).reshape(dims[::-1])
    return out
T = tensors(p)
ks = [k for k in T if "decoder.layers.0." in k]; print(ks)
lnw = T["decoder.layers.0.norm_pos_ff.weight"].reshape(-1)
W1 = T["decoder.layers.0.pos_ff.proj.conv.weight"]; W1 = W1.reshape(W1.shape[0], -1); print("W1", W1.shape)
NAMES = [("x", 768), ("x2", 768), ("q", 768), ("h", 3072), ("logits", 2024), ("ltY", 256), ("sa_part", 3264), ("xa_part", 3088)]
REC = sum(n for _, n in NAMES); offs = {}; o = 0
for nm, n in NAMES: offs[nm] = (o, n); o += n
g = lambda r, nm: r[offs[nm][0]:offs[nm][0]+offs[nm][1]].astype(np.float64)
a = np.fromfile("gpurun_out/ops_a.bin", np.float32).reshape(-1, REC)
b = np.fromfile("gpurun_out/ops_b0.bin", np.float32).reshape(-1, REC)
def merge(xp):
    xp = xp.reshape(4, 772); m = xp[:, 0]; l = xp[:, 1]; M = m.max(); e = np.exp(m - M)
    return (e[:, None] * xp[:, 4:]).sum(0) / (e * l).sum()
def ff1(x, xp):
    x2 = x + merge(xp); mu = x2.mean(); var = ((x2 - mu) ** 2).mean()
    act = (x2 - mu) / math.sqrt(var + 1e-5) * lnw
    y = W1.astype(np.float64) @ act
    return 0.5 * y * (1 + np.vectorize(math.erf)(y / math.sqrt(2))), x2
rows = slice(1392, 1400)
ha, hb = g(a[4], "h")[rows], g(b[4], "h")[rows]
print("x2 check", np.abs(ff1(g(a[2], "x"), g(a[3], "xa_part"))[1] - g(a[4], "x2")).max())
hyp = {"correct": (g(a[2], "x"), g(a[3], "xa_part")),
       "stale x (pre-oproj)": (g(a[1], "x"), g(a[3], "xa_part")),
       "stale xa_part (leftover)": (g(a[2], "x"), g(b[2], "xa_part")),
       "both stale": (g(a[1], "x"), g(b[2], "xa_part"))}
print("a vs b0 rows", np.abs(ha - hb).max())
for k, (x, xp) in hyp.items():
    h, _ = ff1(x, xp)
    print(f"{k:28s} |h-a| {np.abs(h[rows]-ha).max():.2e}  |h-b0| {np.abs(h[rows]-hb).max():.2e}")
print("--- single-line staleness search")
xc, xpc = g(a[2], "x"), g(a[3], "xa_part")
xs, xps = g(a[1], "x"), g(b[2], "xa_part")
best = []
for L in (16, 32):
    for st in range(0, 768, L):
        x = xc.copy(); x[st:st+L] = xs[st:st+L]
        h, _ = ff1(x, xpc); best.append((np.abs(h[rows]-hb).max(), f"x line {st}/{L}"))
    for st in range(0, 3088, L):
        xp = xpc.copy(); xp[st:st+L] = xps[st:st+L]
        h, _ = ff1(xc, xp); best.append((np.abs(h[rows]-hb).max(), f"xa_part line {st}/{L}"))
best.sort()
for e, nm in best[:8]: print(f"{e:.2e} {nm}")
print("--- pre-gelu comparison")
from scipy.optimize import brentq
def inv_gelu(h):
    return brentq(lambda y: 0.5*y*(1+math.erf(y/math.sqrt(2))) - h, -0.75, 50) if h > -0.16 else float('nan')
h0, _ = ff1(xc, xpc)
x2 = xc + merge(xpc); mu = x2.mean(); var = ((x2-mu)**2).mean(); act = (x2-mu)/math.sqrt(var+1e-5)*lnw
y = W1.astype(np.float64) @ act
for i, r in enumerate(range(1392, 1400)):
    print(r, f"y {y[r]:+.5f} ha {ha[i]:+.6f} hb {hb[i]:+.6f} d {hb[i]-ha[i]:+.2e}")
# what if rstd / mean off: fit hb ~ gelu(alpha*y + beta*sum(W1*lnw))
s = W1.astype(np.float64) @ lnw
print("row sums W1*lnw", s[rows])
print("--- rank-1 (single act element) fit")
def inv_near(h, y0):
    f = lambda t: 0.5*t*(1+math.erf(t/math.sqrt(2))) - h
    lo, hi = (-0.75, 5.0)
    return brentq(f, lo, hi)
ya = np.array([inv_near(v, y[r]) for v, r in zip(ha, range(1392, 1400))])
yb = np.array([inv_near(v, y[r]) for v, r in zip(hb, range(1392, 1400))])
dy = yb - ya
print("dy", dy)
Wr = W1[1392:1400].astype(np.float64)
res = []
for k in range(768):
    c = Wr[:, k]; d = (c @ dy) / (c @ c); res.append((np.linalg.norm(dy - c * d) / np.linalg.norm(dy), k, d))
res.sort()
for r_, k, d in res[:5]: print(f"k {k} delta {d:+.4f} rel resid {r_:.3f} act[k] {act[k]:+.4f} x2[k] {x2[k]:+.4f}")
print("--- structured fits")
def fit(cols, name):
    A = np.stack(cols, 1); coef, *_ = np.linalg.lstsq(A, dy, rcond=None)
    print(f"{name:40s} rel resid {np.linalg.norm(dy - A @ coef)/np.linalg.norm(dy):.3f} coef {coef}")
fit([Wr @ act, Wr @ lnw], "global rstd/mean error")
for q in range(4):
    sl = slice(192*q, 192*q+192)
    fit([Wr[:, sl] @ act[sl], Wr[:, sl] @ lnw[sl]], f"quarter {q} rstd/mean")
    fit([Wr[:, sl] @ (x2[sl] - act[sl])], f"quarter {q} raw x2 instead of LN")
    fit([Wr[:, sl] @ (-act[sl])], f"quarter {q} zero")
for j in range(0, 768, 64):
    sl = slice(j, j+64)
    fit([Wr[:, sl] @ (-act[sl])], f"64-chunk {j} zero")
