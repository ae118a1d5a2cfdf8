#!/usr/bin/env python3
"""fp32 drift curve against the reference's 256-step decodes (tests/golden/reference_long.json):
teacher-forced along the reference's own tokens, each step's GPU logits at the reference's top-5
ids against the reference's values (digest bit patterns), plus the full last step (the .npz), for
the persistent, multi-launch and batch-8 paths.  Prints one JSON line.
    python tools/drift_curve.py [case] [--dtype f32|int8]"""
import json
import os
import struct
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    name = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else "llama2_7b"
    q8 = "--dtype" in sys.argv and sys.argv[sys.argv.index("--dtype") + 1] == "int8"
    from __graft_entry__ import _pkg
    _pkg()
    from hip_llama_cpp_amd import thallama as tl
    tl.check(tl.lib().thallama_set_device(0))
    with open(os.path.join(REPO, "tests", "golden", "reference_long.json")) as f:
        case = {c["name"]: c for c in json.load(f)["cases"]}[name]
    g = case["q8" if q8 else "fp32"]
    last = np.load(os.path.join(REPO, "tests", "golden", "reference_long_logits.npz"))[name + ("_q8_last" if q8 else "_fp32_last")]
    c = tl.Config.make(*case["config"])
    m = tl.DeviceModel(c, case["shared"], seed=case["seed"])
    keep = [m]
    if q8:
        m = tl.DeviceModelQ8(c, case["shared"], g["group_size"], from_model=keep[0])
        keep.append(m)
    out = {"case": name, "dtype": "int8" if q8 else "f32", "paths": {}}
    toks = [case["start_token"]] + g["tokens"][:-1]
    for path in ("persistent", "multilaunch", "batch8"):
        B = 8 if path == "batch8" else 1
        st = tl.DeviceState(c, B)
        dec = tl.Decoder(m, st)
        dec.set(tl.OPT_USE_GRAPH, 1)
        if path == "multilaunch":
            dec.set(tl.OPT_PERSISTENT, 0)
        curve = []
        for p, t in enumerate(toks):
            lg = dec.forward([t] * B, [p] * B)
            d = g["digests"][p]
            want = np.array([struct.unpack("<f", struct.pack("<I", b))[0] for b in d["top5_bits"]], np.float64)
            curve.append(float(np.max(np.abs(lg[:, d["top5"]].astype(np.float64) - want))))
        full = float(np.max(np.abs(lg.astype(np.float64) - last)))
        out["paths"][path] = {"max_top5_dlogit_by_step": [round(v, 8) for v in curve], "last_step_max_dlogit": full,
                              "first_step_above_1e-4": next((i for i, v in enumerate(curve) if v > 1e-4), None),
                              "argmax_equal_all_steps": None}
        keep.append((st, dec))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
