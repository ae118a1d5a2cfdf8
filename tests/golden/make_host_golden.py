"""Regenerate tests/golden/host_golden.json — TEST INFRASTRUCTURE.

Inputs and expected outputs of the reference CLI's host side, produced by the REFERENCE's own
code compiled from /root/reference/run.cc (oracle/_ref/librun.so, oracle/run_driver.cpp;
run.cc's tokenizer/sampler are identical to src/llama.cpp's):
  * "kat": the tokenizer known-answer tests of the reference's test.c (prompts and expected ids,
    parsed from test.c and re-checked against librun);
  * "encode": reference encodings of the prompts in the reference's assets/in/*.txt (first
    lines of every file) and of edge-case strings (unicode, byte fallback, whitespace runs);
  * "decode": reference decode() bytes + append_str filter for a spread of (prev, token) pairs;
  * "sample": sample() sequences with their final rng states for seeded logits.
Run from the repo root:  python tests/golden/make_host_golden.py
"""
import ctypes as C
import json
import os
import re
import sys

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
TOK = os.path.join(HERE, "tokenizer.bin")

EDGE = ["", " ", "  ", "\n", "a", "Hello world", "héllo wörld ñ", "日本語のテキスト", "emoji 😀🎉 ok",
        "tabs\tand\nnewlines\r\n", "ŁÓDŹ ąęść", "\x01\x02 control", "<0x41> literal", "1234567890 !@#$%^&*()",
        "a" * 300, " leading and trailing spaces  ", "Ω≈ç√∫˜µ≤≥÷", "🇺🇸🇫🇷"]


def ref():
    L = C.CDLL(os.path.join(REPO, "oracle", "_ref", "librun.so"))
    L.ref_tok_load.restype = C.c_void_p
    L.ref_tok_load.argtypes = [C.c_char_p, C.c_int]
    L.ref_tok_encode.argtypes = [C.c_void_p, C.c_char_p, C.c_int, C.c_int, C.POINTER(C.c_int)]
    L.ref_tok_decode.restype = C.c_void_p
    L.ref_tok_decode.argtypes = [C.c_void_p, C.c_int, C.c_int]
    L.ref_piece_safe.argtypes = [C.c_void_p]
    L.ref_sampler_new.restype = C.c_void_p
    L.ref_sampler_new.argtypes = [C.c_int, C.c_float, C.c_float, C.c_ulonglong]
    L.ref_sample.argtypes = [C.c_void_p, C.POINTER(C.c_float)]
    L.ref_sampler_rng.restype = C.c_ulonglong
    L.ref_sampler_rng.argtypes = [C.c_void_p]
    L.ref_sampler_free.argtypes = [C.c_void_p]
    return L


def encode(L, t, text):
    raw = text.encode() if isinstance(text, str) else text
    buf = (C.c_int * (len(raw) + 3))()
    n = L.ref_tok_encode(t, raw, 1, 0, buf)
    return list(buf[:n])


def parse_test_c():
    src = open(os.path.join(REF, "test.c")).read()
    out = []
    for m in re.finditer(r'char\s*\*\s*(prompt\d*)\s*=\s*((?:"(?:[^"\\]|\\.)*"\s*)+);', src):
        name = m.group(1)
        text = "".join(json.loads('"' + s + '"') for s in re.findall(r'"((?:[^"\\]|\\.)*)"', m.group(2)))
        suffix = name[len("prompt"):]
        em = re.search(r'int\s+expected_tokens' + suffix + r'\[\]\s*=\s*\{([^}]*)\}', src)
        out.append({"text": text, "ids": [int(v) for v in em.group(1).split(",")]})
    return out


def main():
    L = ref()
    t = L.ref_tok_load(TOK.encode(), 32000)
    kat = parse_test_c()
    for k in kat:
        assert encode(L, t, k["text"]) == k["ids"], k["text"]
    texts = list(EDGE)
    for fn in sorted(os.listdir(os.path.join(REF, "assets", "in"))):
        with open(os.path.join(REF, "assets", "in", fn), encoding="utf-8", errors="surrogateescape") as f:
            lines = f.read().split("\n")[1:4]
        texts += [ln for ln in lines if ln]
    enc = [{"text": s, "ids": encode(L, t, s)} for s in texts]
    rng = np.random.default_rng(0)
    pairs = [(1, i) for i in range(0, 32000, 97)] + [(int(a), int(b)) for a, b in rng.integers(0, 32000, (300, 2))]
    pairs += [(1, 29871), (1, 259), (5, 13), (1, 3), (1, 4), (9, 16), (1, 131), (1, 258)]
    dec = []
    for p, tk in pairs:
        ptr = L.ref_tok_decode(t, p, tk)
        dec.append({"prev": p, "token": tk, "hex": C.string_at(ptr).hex(), "safe": int(L.ref_piece_safe(ptr))})
    samples = []
    for seed, (scale, temp, topp) in enumerate([(3.0, 1.0, 0.9), (0.05, 1.0, 0.9), (8.0, 1.0, 0.9), (3.0, 0.7, 0.5),
                                                (3.0, 1.0, 1.0), (3.0, 1.0, 0.0), (3.0, 0.0, 0.9), (1.0, 1.3, 0.95)]):
        r = np.random.default_rng(100 + seed)
        s = L.ref_sampler_new(32000, temp, topp, 314028 + seed)
        toks = []
        for _ in range(12):
            lg = (r.standard_normal(32000) * scale).astype(np.float32)
            lg[r.integers(0, 32000, 40)] = lg.max()  # ties at the top
            toks.append(L.ref_sample(s, lg.ctypes.data_as(C.POINTER(C.c_float))))
        samples.append({"rng_seed": 100 + seed, "scale": scale, "temperature": temp, "topp": topp,
                        "seed": 314028 + seed, "tokens": toks, "final_rng": str(L.ref_sampler_rng(s))})
        L.ref_sampler_free(s)
    out = {"_source": "oracle/_ref/librun.so = reference run.cc (TESTING) + oracle/run_driver.cpp; "
                      "tests/golden/make_host_golden.py", "kat": kat, "encode": enc, "decode": dec,
           "sample": samples}
    with open(os.path.join(HERE, "host_golden.json"), "w") as f:
        json.dump(out, f, indent=0, ensure_ascii=True)
    print(f"kat {len(kat)} encode {len(enc)} decode {len(dec)} sample {len(samples)}")


if __name__ == "__main__":
    sys.exit(main())
