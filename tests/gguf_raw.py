"""Minimal GGUF v3 reader for tests: metadata skipped, tensor infos parsed, a
tensor's bytes returned as stored (tests compare the synthetic files' quantised
blocks with numpy restatements of the reference converter)."""
import struct

import numpy as np

_SCALAR = {0: 1, 1: 1, 2: 2, 3: 2, 4: 4, 5: 4, 6: 4, 7: 1, 10: 8, 11: 8, 12: 8}
_TYPE_BYTES = {0: lambda n: 4 * n, 1: lambda n: 2 * n, 2: lambda n: n // 32 * 18, 8: lambda n: n // 32 * 34}


class GgufRaw:
    def __init__(self, path):
        self.buf = open(path, "rb").read()
        self.p = 0
        magic, version = self._u32(), self._u32()
        assert magic == 0x46554747 and version == 3, (hex(magic), version)
        n_t, n_kv = self._u64(), self._u64()
        for _ in range(n_kv):
            self._str()
            self._skip(self._u32())
        self.tensors = {}
        for _ in range(n_t):
            name = self._str()
            nd = self._u32()
            ne = [self._u64() for _ in range(nd)]
            typ, off = self._u32(), self._u64()
            self.tensors[name] = (ne, typ, off)
        align = 32
        self.data = (self.p + align - 1) // align * align

    def _u32(self):
        v = struct.unpack_from("<I", self.buf, self.p)[0]
        self.p += 4
        return v

    def _u64(self):
        v = struct.unpack_from("<Q", self.buf, self.p)[0]
        self.p += 8
        return v

    def _str(self):
        n = self._u64()
        s = self.buf[self.p:self.p + n].decode()
        self.p += n
        return s

    def _skip(self, t):
        if t == 8:
            self._str()
        elif t == 9:
            et, n = self._u32(), self._u64()
            for _ in range(n):
                self._skip(et)
        else:
            self.p += _SCALAR[t]

    def raw(self, name):
        ne, typ, off = self.tensors[name]
        n = int(np.prod(ne))
        start = self.data + off
        return typ, ne, self.buf[start:start + _TYPE_BYTES[typ](n)]

    def f32(self, name):
        typ, ne, b = self.raw(name)
        assert typ == 0
        return np.frombuffer(b, np.float32).reshape(list(reversed(ne)))
