#!/usr/bin/env python3
"""The REFERENCE's own GPU decode on this MI355X (oracle/_ref/libref_gpu.so: its
thaDNN_s_forward_batch, src/thaDNN.cpp:13-82, with its kernels, built for gfx950 by oracle/Makefile)
on a golden case of tests/golden/reference_long.json: greedy tokens against the reference's CPU
decode (src/seq.cpp), the last step's logits against the reference CPU's (max |d|, count beyond
1e-4), and its decode tok/s.  Measurement / test infrastructure only.  Prints one JSON line.
    python tools/ref_gpu.py [case] [--batch B] [--steps N]"""
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(name="llama2_7b", batch=1, steps=None):
    lib = C.CDLL(os.path.join(REPO, "oracle", "_ref", "libref_gpu.so"))
    lib.refgpu_greedy.restype = C.c_int
    lib.refgpu_greedy.argtypes = [C.POINTER(C.c_int), C.c_int, C.c_ulonglong, C.c_int, C.c_int, C.c_int, C.c_int,
                                  C.POINTER(C.c_int), C.POINTER(C.c_float), C.POINTER(C.c_double)]
    with open(os.path.join(REPO, "tests", "golden", "reference_long.json")) as f:
        case = {c["name"]: c for c in json.load(f)["cases"]}[name]
    n = steps or case["steps"]
    cfg = (C.c_int * 7)(*case["config"])
    V = abs(case["config"][5])
    toks = np.zeros((n, batch), np.int32)
    last = np.zeros((batch, V), np.float32)
    secs = C.c_double(0)
    st = lib.refgpu_greedy(cfg, case["shared"], case["seed"], batch, case["start_token"], case["start_pos"], n,
                           toks.ctypes.data_as(C.POINTER(C.c_int)), last.ctypes.data_as(C.POINTER(C.c_float)),
                           C.byref(secs))
    want = case["fp32"]["tokens"][:n]
    seq = toks[:, 0].tolist()
    first = next((i for i, (a, w) in enumerate(zip(seq, want)) if a != w), None)
    out = {"case": name, "batch": batch, "steps": n, "status": st, "seconds": round(secs.value, 4),
           "tok_per_s": round(n * batch / secs.value, 2) if secs.value > 0 else None,
           "ms_per_step": round(1e3 * secs.value / n, 3) if n else None,
           "tokens_match": first is None, "match_prefix": n if first is None else first,
           "rows_agree": bool((toks == toks[:, :1]).all())}
    if n == case["steps"]:
        ref = np.load(os.path.join(REPO, "tests", "golden", "reference_long_logits.npz"))[name + "_fp32_last"]
        d = np.abs(last[0].astype(np.float64) - ref.astype(np.float64))
        tol = 1e-4 * np.maximum(1.0, np.abs(ref))  # the reference's abs-or-rel rule at 1e-4
        out["last_logits_max_abs_diff"] = float(d.max())
        out["last_logits_beyond_1e-4"] = int((d > tol).sum())
    return out


if __name__ == "__main__":
    a = sys.argv[1:]
    name = a[0] if a and not a[0].startswith("-") else "llama2_7b"
    batch = int(a[a.index("--batch") + 1]) if "--batch" in a else 1
    steps = int(a[a.index("--steps") + 1]) if "--steps" in a else None
    print(json.dumps(run(name, batch, steps)), flush=True)
