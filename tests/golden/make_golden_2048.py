#!/usr/bin/env python3
"""Generate tests/golden/reference_2048.json (+ reference_2048_logits.npz): the llama2-7B fp32
greedy decode from BOS over the WHOLE context, positions 0..2047 — the length the reference's
test mode decodes every request to (`steps = seq_len`, src/llama.cpp:1584; the loop ends at
pos >= seq_len, :1036-1064).

Generator: oracle/oracle.c's forward (the bit-exact restatement of src/seq.cpp:53-183, pinned
against the reference compiled in place by tests/test_oracle.py; its matmul rows may run on
several threads without changing any row's summation order), same synthetic model as bench.py
(include/thallama_synth.h generator, seed 20240224).  Its first 256 tokens and digests must equal
tests/golden/reference_long.json's llama2_7b case, which src/seq.cpp itself produced — checked
here before anything is written, and again by tests/test_golden_2048.py.

Recorded per step: the token, the top-2 margin and ids; the digest of make_golden.py at six
steps; and — for the drift curve of a GPU decode against this one — the float32 values at 72 logit
indices (the step's top-8 ids, then 64 fixed ids) in the .npz, with the full float32 logits of
steps 255, 1023 and 2047.  Data only (inputs + outputs).  Run: python tests/golden/make_golden_2048.py [threads]
(~1-2 h on 7 threads, ~32 GB RAM).  Progress is saved every 64 steps; a rerun resumes.
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, HERE)
import oracle as O  # noqa: E402
from make_golden import digest  # noqa: E402

SEED = 20240224
CFG = (4096, 11008, 32, 32, 32, 32000, 2048)
STEPS = 2048
FULL_AT = (255, 1023, 2047)
FIXED_IDS = [int(i) for i in np.random.default_rng(2048).choice(32000, 64, replace=False)]
OUT_JSON = os.path.join(HERE, "reference_2048.json")
OUT_NPZ = os.path.join(HERE, "reference_2048_logits.npz")
PART = "/tmp/reference_2048_partial.json"


def margin(lg):
    top = np.sort(lg.astype(np.float64))[-2:]
    return float(top[1] - top[0])


def main():
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else min(7, os.cpu_count() or 1)
    with open(os.path.join(HERE, "reference_long.json")) as f:
        ref256 = next(c for c in json.load(f)["cases"] if c["name"] == "llama2_7b")["fp32"]
    st = {"tokens": [], "margins": [], "digests": [], "probe_ids": [], "probe_vals": []}
    if os.path.exists(PART):
        with open(PART) as f:
            st = json.load(f)
    full = dict(np.load(OUT_NPZ + ".part.npz")) if os.path.exists(OUT_NPZ + ".part.npz") else {}
    O.set_threads(threads)
    m = O.Model(CFG, 0, seed=SEED)
    tok = 1
    t0 = time.time()
    # replay the saved prefix (rebuilds the K/V cache), then continue
    for p, t in enumerate([1] + st["tokens"][:-1] if st["tokens"] else []):
        m.forward(t, p)
    if st["tokens"]:
        tok = st["tokens"][-1]
    for p in range(len(st["tokens"]), STEPS):
        lg = m.forward(tok, p)
        nxt = int(np.argmax(lg))  # sample_argmax: first index of the maximum
        top8 = [int(i) for i in np.argsort(-lg.astype(np.float64), kind="stable")[:8]]
        ids = top8 + FIXED_IDS
        st["tokens"].append(nxt)
        st["margins"].append(margin(lg))
        st["digests"].append(digest(lg))
        st["probe_ids"].append(ids)
        st["probe_vals"].append([float(v) for v in lg[ids]])
        if p in FULL_AT:
            full[f"step{p}"] = lg.astype(np.float32)
        if p == 255:
            if st["tokens"][:256] != ref256["tokens"] or st["digests"][255] != ref256["digests"][255]:
                raise SystemExit("oracle decode differs from the reference's own 256-step decode")
            print("first 256 tokens and digests equal src/seq.cpp's", file=sys.stderr, flush=True)
        tok = nxt
        if (p + 1) % 64 == 0 or p == STEPS - 1:
            with open(PART, "w") as f:
                json.dump(st, f)
            np.savez(OUT_NPZ + ".part.npz", **full)
            print(f"pos {p} {time.time() - t0:.0f}s min margin {min(st['margins']):.3g}", file=sys.stderr, flush=True)
    m.close()
    out = {"generator": "tests/golden/make_golden_2048.py",
           "reference": "oracle/oracle.c forward (bit-exact src/seq.cpp:53-183 restatement), greedy = sample_argmax "
                        "(src/llama.cpp:275-286); first 256 steps equal reference_long.json (src/seq.cpp itself)",
           "config": list(CFG), "shared": 0, "seed": SEED, "start_token": 1, "start_pos": 0, "steps": STEPS,
           "fixed_probe_ids": FIXED_IDS, "tokens": st["tokens"], "margins": st["margins"],
           "top2": [ids[:2] for ids in st["probe_ids"]],
           "digests_at": {str(k): st["digests"][k] for k in (0, 255, 511, 1023, 1535, 2047)},
           "probes": "reference_2048_logits.npz: probe_ids [2048][72] (the step's top-8 ids, then fixed_probe_ids) "
                     "and probe_vals (float32 logits there)"}
    with open(OUT_JSON, "w") as f:
        json.dump(out, f, separators=(",", ":"))
    np.savez(OUT_NPZ, probe_ids=np.array(st["probe_ids"], np.int32), probe_vals=np.array(st["probe_vals"], np.float32),
             **full)
    os.remove(PART)
    os.remove(OUT_NPZ + ".part.npz")


if __name__ == "__main__":
    main()
