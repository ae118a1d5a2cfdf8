#!/usr/bin/env python3
"""Generate tests/golden/*.json from the REFERENCE ITSELF (oracle/_ref, built by
oracle/Makefile from /root/reference/src/seq.cpp + src/utils.cpp and /root/reference/runq.c).

For each case a synthetic model (include/thallama_synth.h generator, fixed seed) is written
as a llama2.c v0 model.bin (and, for int8 cases, a runq v2 file), the reference CPU forward
runs a BOS-started greedy decode, and we record the token ids plus per-step logit digests
(argmax, top-5 ids and values as float32 bit patterns, float64 sum, float64 sum of squares,
and the first 8 logits bit patterns).  The fixtures are data: inputs (config + seed) and the
reference's outputs.  Run: python tests/golden/make_golden.py
"""
import json
import os
import struct
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle as O  # noqa: E402

CASES = [
    # name, config (dim, hidden, layers, heads, kv_heads, vocab, seq_len), shared, seed, steps, q8 group size
    ("tiny_gqa", (64, 172, 2, 4, 2, 512, 64), 0, 7, 24, 32),
    ("small_mha", (256, 768, 2, 4, 4, 1024, 128), 0, 42, 24, 64),
    ("small_shared", (256, 768, 2, 4, 4, 1024, 128), 1, 42, 8, 64),
    ("small_gqa", (512, 1536, 3, 8, 2, 2048, 256), 0, 5, 24, 64),
]


def f32bits(x):
    return struct.unpack("<I", struct.pack("<f", float(x)))[0]


def digest(logits):
    lg = np.asarray(logits, np.float32)
    top = np.argsort(-lg.astype(np.float64), kind="stable")[:5]
    return {"argmax": int(np.argmax(lg)), "top5": [int(i) for i in top],
            "top5_bits": [f32bits(lg[i]) for i in top],
            "sum": float(lg.astype(np.float64).sum()), "sumsq": float((lg.astype(np.float64) ** 2).sum()),
            "head_bits": [f32bits(v) for v in lg[:8]]}


def main():
    if not O.have_ref():
        raise SystemExit("oracle/_ref/libref_seq.so missing: build it with `make -C oracle` where /root/reference exists")
    out = {"generator": "tests/golden/make_golden.py", "reference": "src/seq.cpp forward + runq.c forward, "
           "compiled from /root/reference by oracle/Makefile", "cases": []}
    tmp = tempfile.mkdtemp()
    for name, cfg, shared, seed, steps, gs in CASES:
        m = O.Model(cfg, shared, seed=seed)
        path = os.path.join(tmp, name + ".bin")
        m.write_v0(path)
        toks, logits = O.ref_greedy(path, 1, 0, steps, abs(cfg[5]))
        case = {"name": name, "config": list(cfg), "shared": shared, "seed": seed, "start_token": 1, "steps": steps,
                "tokens": toks, "digests": [digest(l) for l in logits]}
        if gs and O.have_ref_q8():
            m.build_q8(gs)
            qpath = os.path.join(tmp, name + "_q8.bin")
            m.write_v2(qpath)
            qt, ql = O.ref_q8_greedy(qpath, 1, 0, steps, abs(cfg[5]))
            case["q8"] = {"group_size": gs, "tokens": qt, "digests": [digest(l) for l in ql]}
        out["cases"].append(case)
        m.close()
        print(name, toks[:12], file=sys.stderr)
    with open(os.path.join(HERE, "reference_greedy.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
