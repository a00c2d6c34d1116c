"""Minimal GGUF v3 key/value reader for tests (strings and integers only)."""
import struct


def read_kv(path):
    out = {}
    with open(path, "rb") as f:
        assert f.read(4) == b"GGUF"
        (ver,) = struct.unpack("<I", f.read(4))
        assert ver == 3
        _nt, nkv = struct.unpack("<QQ", f.read(16))
        sizes = {0: 1, 1: 1, 2: 2, 3: 2, 4: 4, 5: 4, 6: 4, 7: 1, 10: 8, 11: 8, 12: 8}
        fmts = {4: "<I", 5: "<i", 10: "<Q", 11: "<q"}

        def rstr():
            (n,) = struct.unpack("<Q", f.read(8))
            return f.read(n)

        def rval(t):
            if t == 8:
                return rstr()
            if t == 9:
                et, n = struct.unpack("<IQ", f.read(12))
                return [rval(et) for _ in range(n)]
            raw = f.read(sizes[t])
            return struct.unpack(fmts[t], raw)[0] if t in fmts else raw

        for _ in range(nkv):
            key = rstr().decode()
            (t,) = struct.unpack("<I", f.read(4))
            out[key] = rval(t)
    return out
