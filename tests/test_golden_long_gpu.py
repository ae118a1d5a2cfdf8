"""BASELINE.json configs[1]-[3] end to end: 256-step greedy decodes from BOS against the
REFERENCE's own 256-step decodes (tests/golden/reference_long.json, generated from the reference's
src/seq.cpp forward (:53-183) and runq.c forward (:344-481) compiled from its sources by
oracle/Makefile; tests/golden/make_golden_long.py).

fp32 bar (north_star): every greedy token identical, last-step logits within 1e-4 under the
reference's abs-or-rel rule (scripts/test/thaDNN.test.cpp:224-229).  The fixture records the
reference's top-2 margin per step: the smallest is 5.2e-4 (7B), far above the fp32 drift.
Cases: stories110M shape with a shared and an unshared classifier, and llama2-7B (the bench's own
model: same seed), each on the persistent one-launch step, the multi-launch step, and — for the
8-GPU config's per-GPU workload — 8 sequences at once on the matrix-core GEMV path.
"""
import json
import os

import numpy as np
import pytest

from helpers import assert_ref_close

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "reference_long.json")) as _f:
    CASES = {c["name"]: c for c in json.load(_f)["cases"]}
LAST = np.load(os.path.join(HERE, "golden", "reference_long_logits.npz"))


def fp32_decoder(tl, case, batch):
    c = tl.Config.make(*case["config"])
    model = tl.DeviceModel(c, case["shared"], seed=case["seed"])
    state = tl.DeviceState(c, batch)
    return (model, state), tl.Decoder(model, state)


@pytest.mark.parametrize("name", ["stories110m_shared", "stories110m_unshared", "llama2_7b"])
@pytest.mark.parametrize("path", ["persistent", "multilaunch", "batch8"])
def test_fp32_256_step_greedy_equals_reference(gpu, name, path):
    case = CASES[name]
    g = case["fp32"]
    B = 8 if path == "batch8" else 1
    keep, dec = fp32_decoder(gpu, case, B)
    dec.set(gpu.OPT_USE_GRAPH, 1)
    if path == "multilaunch":
        dec.set(gpu.OPT_PERSISTENT, 0)
    assert dec.persistent() == (path == "persistent")
    n = case["steps"]
    got = dec.greedy([case["start_token"]] * B, [case["start_pos"]] * B, n)
    for b in range(B):
        seq = got[:, b].tolist()
        first = next((i for i, (a, w) in enumerate(zip(seq, g["tokens"])) if a != w), None)
        assert first is None, (f"{name} {path} seq {b}: token {first} differs (got {seq[first]}, reference "
                               f"{g['tokens'][first]}, reference top-2 margin there {g['margins'][first]:.3g})")
    # the device holds the logits of the last step (pos n-1): the reference's within 1e-4
    lg = dec.logits()
    for b in range(B):
        assert_ref_close(lg[b], LAST[name + "_fp32_last"], 1e-4, f"{name} {path} seq {b} last-step logits")
        d = g["digests"][-1]
        assert int(np.argmax(lg[b])) == d["argmax"]
