#!/usr/bin/env python3
"""Per-kernel census of f32 FMA / multiply / add instructions in two library builds
(diagnostic for the contraction setting): prints the kernels whose counts differ.
usage: fma_census.py A.so B.so"""
import re
import struct
import subprocess
import sys
import tempfile
from collections import Counter
from pathlib import Path

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def code_objects(so, tmp):
    sec = tmp / "fatbin.bin"
    subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objcopy", f"--dump-section=.hip_fatbin={sec}", so,
                    str(tmp / "discard.so")], check=True)
    data = sec.read_bytes()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    out, pos = [], data.find(magic)
    while pos >= 0:
        n, = struct.unpack_from("<Q", data, pos + 24)
        p = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if "gfx950" in triple and size:
                co = tmp / f"co{len(out)}.elf"
                co.write_bytes(data[pos + off:pos + off + size])
                out.append(co)
        pos = data.find(magic, pos + 1)
    return out


def census(so):
    res = {}
    with tempfile.TemporaryDirectory() as d:
        for co in code_objects(so, Path(d)):
            dis = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", str(co)], capture_output=True, text=True,
                                 check=True).stdout
            cur = None
            for line in dis.splitlines():
                m = re.match(r"^[0-9a-f]+ <(.+)>:", line)
                if m:
                    cur = m.group(1)
                    res[cur] = Counter()
                    continue
                if cur is None:
                    continue
                m = re.search(r"\b(v_(?:fma|fmac|mul|add|sub)_f32|v_fma_mix\w*|v_mad\w*_f32)(?:_e32|_e64|_dpp)?\b", line)
                if m:
                    res[cur][m.group(1)] += 1
    return res


def main():
    a, b = census(sys.argv[1]), census(sys.argv[2])
    for k in sorted(set(a) | set(b)):
        ca, cb = a.get(k, Counter()), b.get(k, Counter())
        if ca != cb:
            name = subprocess.run(["c++filt", k], capture_output=True, text=True).stdout.strip()
            print(f"{name[:110]}\n    A {dict(ca)}\n    B {dict(cb)}")


if __name__ == "__main__":
    main()
