"""Test infrastructure, not product code: a pure-Python restatement of the
reference's text front end (magpie.cpp:124-495) and sentence splitter
(magpie.cpp:4439-4480), used by tests/test_tokenizer_cpu.py as the checker of the
C++ implementation in libmagpie_hip.so. Parity unpinned against the real
reference: its tokenizer data (NeMo IPA vocabulary/dictionary) ships only inside
the released GGUFs, which are not available offline; the synthetic GGUF carries a
small vocabulary/dictionary (tools/mp_synth_gguf.c).
"""
from __future__ import annotations

ONES = ["zero", "one", "two", "three", "four", "five", "six", "seven", "eight", "nine", "ten", "eleven", "twelve",
        "thirteen", "fourteen", "fifteen", "sixteen", "seventeen", "eighteen", "nineteen"]
TENS = ["", "", "twenty", "thirty", "forty", "fifty", "sixty", "seventy", "eighty", "ninety"]


def number_to_words(n: int, use_and: bool = True) -> str:  # magpie.cpp:153-207
    if n < 0:
        return "minus " + number_to_words(-n, use_and)
    if n < 20:
        return ONES[n]
    if n < 100:
        return TENS[n // 10] + ("" if n % 10 == 0 else " " + ONES[n % 10])
    if n < 1000:
        s = ONES[n // 100] + " hundred"
        if n % 100:
            s += (" and" if use_and else "") + " " + number_to_words(n % 100, use_and)
        return s
    if n >= 10**12:
        return str(n)
    for unit, name in ((10**9, " billion"), (10**6, " million"), (1000, " thousand")):
        if n >= unit:
            s = number_to_words(n // unit, use_and) + name
            if n % unit:
                s += " " + number_to_words(n % unit, use_and)
            return s
    return str(n)


def year_to_words(n: int) -> str:  # magpie.cpp:210-227
    if n < 1000 or n > 9999:
        return number_to_words(n)
    hi, lo = divmod(n, 100)
    if lo == 0:
        return number_to_words(hi) + " hundred"
    if lo < 10:
        return number_to_words(n)
    return number_to_words(hi) + " " + number_to_words(lo)


def ordinal_to_words(n: int) -> str:  # magpie.cpp:230-262
    special = ["", "first", "second", "third", "fourth", "fifth", "sixth", "seventh", "eighth", "ninth", "tenth",
               "eleventh", "twelfth"]
    if 1 <= n <= 12:
        return special[n]
    c = number_to_words(n)
    if 13 <= n <= 19:
        return c + "th"
    if n % 10 == 0 and 20 <= n < 100:
        return c[:-1] + "ieth" if c.endswith("y") else c + "th"
    d = n % 10
    if d in (1, 2, 3):
        return c[:c.rfind(" ") + 1] + ["", "first", "second", "third"][d]
    return c + "th"


def normalize_text(t: str) -> str:  # magpie.cpp:265-351, byte-wise (t holds one char per byte)
    out, i = [], 0

    def isd(ch):
        return "0" <= ch <= "9"

    while i < len(t):
        if t[i] == "$" and i + 1 < len(t) and isd(t[i + 1]):
            i += 1
            v = 0
            while i < len(t) and isd(t[i]):
                v = v * 10 + int(t[i])
                i += 1
            out.append(number_to_words(v) + " dollar" + ("" if v == 1 else "s"))
            continue
        if isd(t[i]) or (t[i] == "-" and i + 1 < len(t) and isd(t[i + 1])):
            neg = t[i] == "-"
            if neg:
                i += 1
            v, nd = 0, 0
            while i < len(t) and isd(t[i]):
                v = v * 10 + int(t[i])
                nd += 1
                i += 1
            if i < len(t) and t[i] == "%":
                i += 1
                out.append(("minus " if neg else "") + number_to_words(v) + " percent")
                continue
            ordl = i + 1 < len(t) and t[i:i + 2].lower() in ("st", "nd", "rd", "th")
            if ordl:
                i += 2
                w = ordinal_to_words(v)
            elif nd == 4 and 1000 <= v <= 2099:
                w = year_to_words(v)
            else:
                w = number_to_words(v)
            if neg and v != 0:
                w = "minus " + w
            out.append(w)
            continue
        out.append(t[i])
        i += 1
    return "".join(out)


def load(vocab: str, dictionary: str, space=93, bos=2378, eos=2379):
    """magpie_tokenizer_init (magpie.cpp:353-398): later duplicates win."""
    tid = {}
    for i, s in enumerate(vocab.split("\n")):
        tid[s] = i
    d = {}
    for line in dictionary.split("\n"):
        if "\t" in line:
            w, p = line.split("\t", 1)
            d[w] = p
    return {"tid": tid, "dict": d, "space": space, "bos": bos, "eos": eos}


def tokenize(tk, text: str):  # magpie.cpp:400-492, on UTF-8 bytes like the C++ std::string code
    raw = text.encode("utf-8")
    norm = normalize_text(raw.decode("latin-1")).encode("latin-1")
    low = bytes(c + 32 if 65 <= c <= 90 else c for c in norm)
    proc = bytearray()
    for c in low:
        if c in b",.!?:;":
            proc += b" " + bytes([c]) + b" "
        else:
            proc.append(c)
    tid = {k.encode("utf-8"): v for k, v in tk["tid"].items()}
    dct = {k.encode("utf-8"): v.encode("utf-8") for k, v in tk["dict"].items()}
    ids = [tk["bos"]]
    for w in bytes(proc).split(b" "):
        if not w:
            continue
        if len(w) == 1 and w in tid:
            ids.append(tid[w])
            continue
        if w in dct:
            p, i = dct[w], 0
            while i < len(p):
                for n in range(min(4, len(p) - i), 0, -1):
                    if p[i:i + n] in tid:
                        ids.append(tid[p[i:i + n]])
                        i += n
                        break
                else:
                    i += 1
        else:
            for c in w:
                u = c - 32 if 97 <= c <= 122 else c
                if bytes([u]) in tid:
                    ids.append(tid[bytes([u])])
        if tk["space"] >= 0:
            ids.append(tk["space"])
    if ids and ids[-1] == tk["space"]:
        ids.pop()
    ids.append(tk["eos"])
    return ids


def split_sentences(text: str):  # magpie.cpp:4439-4480
    out, cur = [], ""
    for i, ch in enumerate(text):
        cur += ch
        nx = text[i + 1] if i + 1 < len(text) else ""
        if ch in ".!?" and nx in ("", " ", "\n", "\t"):
            s = cur.lstrip(" \t\n\r")
            if s:
                out.append(s)
            cur = ""
    s = cur.lstrip(" \t\n\r")
    if s:
        out.append(s)
    return out
