"""CPU: tests/golden/reference_2048.json (the 2048-step llama2-7B fp32 greedy decode of the CPU
oracle, tests/golden/make_golden_2048.py) is pinned to the reference: its first 256 tokens and the
step-255 logits digest equal the reference's own src/seq.cpp decode (reference_long.json, made by
the reference compiled from its sources)."""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def test_fixture_pinned_to_reference():
    with open(os.path.join(HERE, "golden", "reference_2048.json")) as f:
        fx = json.load(f)
    with open(os.path.join(HERE, "golden", "reference_long.json")) as f:
        ref = next(c for c in json.load(f)["cases"] if c["name"] == "llama2_7b")["fp32"]
    assert fx["steps"] == len(fx["tokens"]) == len(fx["margins"]) == 2048
    assert fx["tokens"][:256] == ref["tokens"]
    assert fx["digests_at"]["255"] == ref["digests"][255]
    z = np.load(os.path.join(HERE, "golden", "reference_2048_logits.npz"))
    assert z["probe_ids"].shape == z["probe_vals"].shape == (2048, 72)
    # the recorded argmax is the first probe id, and it is the next step's input token
    assert [int(i) for i in z["probe_ids"][:, 0]] == fx["tokens"]
    for k in (255, 1023, 2047):
        assert int(np.argmax(z[f"step{k}"])) == fx["tokens"][k]
