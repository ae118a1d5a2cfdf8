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


def run_forced(config, shared, seed, tokens, probe_ids, full_steps=()):
    """Teacher-forced decode along `tokens` (step i at position i) with the reference's GPU
    forward_batch: (probe_vals [n][k] at probe_ids [n][k], {step: full logits})."""
    lib = C.CDLL(os.path.join(REPO, "oracle", "_ref", "libref_gpu.so"))
    ip = C.POINTER(C.c_int)
    fpp = C.POINTER(C.c_float)
    lib.refgpu_forced.restype = C.c_int
    lib.refgpu_forced.argtypes = [ip, C.c_int, C.c_ulonglong, ip, C.c_int, C.c_int, ip, C.c_int, fpp, ip, C.c_int, fpp]
    tok = np.ascontiguousarray(tokens, np.int32)
    ids = np.ascontiguousarray(probe_ids, np.int32)
    n, k = ids.shape
    assert tok.size == n
    V = abs(config[5])
    vals = np.zeros((n, k), np.float32)
    fs = np.ascontiguousarray(list(full_steps) or [-1], np.int32)
    full = np.zeros((len(fs), V), np.float32)
    cfg = (C.c_int * 7)(*config)
    st = lib.refgpu_forced(cfg, int(shared), int(seed), tok.ctypes.data_as(ip), 0, n, ids.ctypes.data_as(ip), k,
                           vals.ctypes.data_as(fpp), fs.ctypes.data_as(ip), len(full_steps), full.ctypes.data_as(fpp))
    if st != 0:
        raise RuntimeError(f"refgpu_forced: status {st}")
    return vals, {int(s): full[i] for i, s in enumerate(full_steps)}


def forced_2048(out_path):
    """tests/golden/reference_gpu_drift_2048.json: the reference GPU path's drift from the CPU
    fixture (reference_2048.json) along its tokens, per step (max over the step's probe logits;
    whole logits at steps 255, 1023, 2047) — the yardstick of test_golden_2048_gpu.py."""
    g = os.path.join(REPO, "tests", "golden")
    with open(os.path.join(g, "reference_2048.json")) as f:
        fx = json.load(f)
    npz = np.load(os.path.join(g, "reference_2048_logits.npz"))
    toks = [fx["start_token"]] + fx["tokens"][:-1]
    ids, vals = npz["probe_ids"], npz["probe_vals"].astype(np.float64)
    got, full = run_forced(fx["config"], fx["shared"], fx["seed"], toks, ids, (255, 1023, 2047))
    d = np.abs(got.astype(np.float64) - vals).max(axis=1)
    for p in (255, 1023, 2047):
        d[p] = max(d[p], np.abs(full[p].astype(np.float64) - npz[f"step{p}"].astype(np.float64)).max())
    rec = {"generator": "tools/ref_gpu.py --forced-2048 (oracle/_ref/libref_gpu.so: the reference's "
                        "thaDNN_s_forward_batch, src/thaDNN.cpp:13-82, built for gfx950)",
           "max_drift": float(d.max()), "argmax": int(d.argmax()), "drift": [float(x) for x in d]}
    with open(out_path, "w") as f:
        json.dump(rec, f)
    return rec


if __name__ == "__main__":
    a = sys.argv[1:]
    if "--forced-2048" in a:
        r = forced_2048(a[a.index("--forced-2048") + 1])
        print(json.dumps({"max_drift": r["max_drift"], "argmax": r["argmax"]}), flush=True)
        sys.exit(0)
    name = a[0] if a and not a[0].startswith("-") else "llama2_7b"
    batch = int(a[a.index("--batch") + 1]) if "--batch" in a else 1
    steps = int(a[a.index("--steps") + 1]) if "--steps" in a else None
    print(json.dumps(run(name, batch, steps)), flush=True)
