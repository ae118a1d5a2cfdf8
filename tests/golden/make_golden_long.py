#!/usr/bin/env python3
"""Generate tests/golden/reference_long.json (+ reference_long_logits.npz) from the REFERENCE ITSELF:
BASELINE.json configs[1]-[3] as 256-step greedy decodes from BOS.

  * fp32: oracle/_ref/libref_seq.so = /root/reference/src/seq.cpp forward (:53-183) + src/utils.cpp
    loader, compiled in place by oracle/Makefile, single-threaded like the reference;
  * int8: oracle/_ref/librunq.so = /root/reference/runq.c forward (:344-481), OpenMP.

Models are synthetic (include/thallama_synth.h generator, fixed seed; the GPU builds the same
bits on the device), written as a llama2.c v0 model.bin and a runq v2 file.  Recorded per case
and step: the token, the reference's top-2 logit margin and a digest (argmax, top-5 ids and
float32 bit patterns, float64 sum / sum of squares, first 8 logits' bits); plus the full
float32 logits of the last step in the .npz.  These are data (inputs + the reference's
outputs).  Run: python tests/golden/make_golden_long.py [case ...]   (7B: ~25 min, ~35 GB RAM)
"""
import json
import os
import sys
import tempfile
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, HERE)
import oracle as O  # noqa: E402
from make_golden import digest  # noqa: E402

SEED = 20240224  # bench.py's seed: the 7B case is the bench's own model
CASES = [
    # name, (dim, hidden, layers, heads, kv_heads, vocab, seq_len), shared classifier, steps
    ("stories110m_shared", (768, 2048, 12, 12, 12, 32000, 1024), 1, 256),
    ("stories110m_unshared", (768, 2048, 12, 12, 12, 32000, 1024), 0, 256),
    ("llama2_7b", (4096, 11008, 32, 32, 32, 32000, 2048), 0, 256),
]
GS = 64
OUT_JSON = os.path.join(HERE, "reference_long.json")
OUT_NPZ = os.path.join(HERE, "reference_long_logits.npz")


def margin(lg):
    top = np.sort(lg.astype(np.float64))[-2:]
    return float(top[1] - top[0])


def record(toks, logits):
    return {"tokens": [int(t) for t in toks], "margins": [margin(l) for l in logits],
            "digests": [digest(l) for l in logits]}


def main(names):
    if not (O.have_ref() and O.have_ref_q8()):
        raise SystemExit("oracle/_ref missing: build it with `make -C oracle` where /root/reference exists")
    old = {"cases": []}
    if os.path.exists(OUT_JSON):
        with open(OUT_JSON) as f:
            old = json.load(f)
    arrays = dict(np.load(OUT_NPZ)) if os.path.exists(OUT_NPZ) else {}
    cases = {c["name"]: c for c in old["cases"]}
    tmp = tempfile.mkdtemp(dir=os.environ.get("GOLDEN_TMP", "/tmp"))
    for name, cfg, shared, steps in CASES:
        if names and name not in names:
            continue
        t0 = time.time()
        O.set_threads(min(8, os.cpu_count() or 1))  # synthesis / quantisation only
        m = O.Model(cfg, shared, seed=SEED)
        v0, v2 = os.path.join(tmp, name + ".bin"), os.path.join(tmp, name + "_q8.bin")
        m.write_v0(v0)
        m.build_q8(GS)
        m.write_v2(v2)
        m.close()
        del m
        V = abs(cfg[5])
        toks, logits = O.ref_greedy(v0, 1, 0, steps, V)
        os.remove(v0)
        print(f"{name} fp32 {time.time() - t0:.0f}s {toks[:12]}", file=sys.stderr, flush=True)
        qt, ql = O.ref_q8_greedy(v2, 1, 0, steps, V)
        os.remove(v2)
        print(f"{name} int8 {time.time() - t0:.0f}s {qt[:12]}", file=sys.stderr, flush=True)
        cases[name] = {"name": name, "config": list(cfg), "shared": shared, "seed": SEED, "start_token": 1,
                       "start_pos": 0, "steps": steps, "fp32": record(toks, logits),
                       "q8": dict(group_size=GS, **record(qt, ql))}
        arrays[name + "_fp32_last"] = np.asarray(logits[-1], np.float32)
        arrays[name + "_q8_last"] = np.asarray(ql[-1], np.float32)
        out = {"generator": "tests/golden/make_golden_long.py",
               "reference": "src/seq.cpp forward (fp32) and runq.c forward (int8, GS 64), compiled from "
                            "/root/reference by oracle/Makefile; greedy = sample_argmax (src/llama.cpp:275-286)",
               "cases": [cases[n] for n, *_ in CASES if n in cases]}
        with open(OUT_JSON, "w") as f:
            json.dump(out, f, separators=(",", ":"))
        np.savez(OUT_NPZ, **arrays)
    os.rmdir(tmp)


if __name__ == "__main__":
    main(sys.argv[1:])
