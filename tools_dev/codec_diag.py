import sys, os, numpy as np
sys.path.insert(0,'magpie-tts.cpp_amd'); sys.path.insert(0,'.')
import magpie_amd as ma
from oracle import oracle as orc
orc.set_mode(True, False, 16)
path = ma.synth_gguf('/tmp/magpie_amd_cache/nano_codec.gguf', kind='codec')
g = ma.Codec(path); o = orc.Codec(path)
for F in [1, 2, 4, 5, 8]:
    codes = np.random.default_rng(100 + F).integers(0, 2016, (8, F)).astype(np.int32)
    a = g.decode(codes); b = o.decode(codes, True); c = o.decode(codes, False)
    d = np.abs(a-b)
    print(F, 'gpu-o16 max', d.max(), 'mean', d.mean(), 'argmax', d.argmax(), 'o16-o32 max', np.abs(b-c).max(), 'gpu-o32', np.abs(a-c).max())
    blk = d.reshape(-1, 256).max(axis=1)
    print('   per-256 max:', np.round(blk, 5).tolist()[:24])
