"""CPU: the tie-step fixture (tests/golden/request_ties_llama2-7B_f32.{json,npz}, made by
make_golden_request_ties.py with the oracle teacher-forced on each request's own history) agrees with
the request fixture it was cut from — every near-tie under bench.REQUEST_TIE_7B is there, the CPU's
argmax at that step is the fixture's own greedy token, and the stored logit rows carry the recorded
top-2 and margin.  The GPU side (tests/test_requests_gpu.py) replays these steps."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
import bench  # noqa: E402
from make_golden_request_ties import request_inputs  # noqa: E402

G = os.path.join(REPO, "tests", "golden")


def test_tie_fixture_matches_request_fixture():
    with open(os.path.join(G, "request_ties_llama2-7B_f32.json")) as f:
        tf = json.load(f)
    with open(os.path.join(G, "requests_llama2-7B_f32_gen_in_64.json")) as f:
        fx = json.load(f)
    rows = np.load(os.path.join(G, "request_ties_llama2-7B_f32.npz"))["logits"]
    want = sorted((i, t[0]) for i, ts in enumerate(fx["near_ties"]) for t in ts if t[1] < bench.REQUEST_TIE_7B)
    assert sorted((c["request"], c["position"]) for c in tf["cases"]) == want
    assert rows.shape == (len(tf["cases"]), 32000) and rows.dtype == np.float32
    assert tf["config"] == fx["config"] and tf["seed"] == fx["seed"] == bench.SEED
    for k, c in enumerate(tf["cases"]):
        row = rows[k]
        gen = fx["generated_tokens"][c["request"]]
        assert int(np.argmax(row)) == c["top2_ids"][0] == gen[c["position"] - c["prompt_tokens"] + 1]
        assert [float(row[v]) for v in c["top2_ids"]] == c["top2_logits"]
        assert np.sort(row)[-2] == row[c["top2_ids"][1]]
        assert abs(float(row[c["top2_ids"][0]]) - float(row[c["top2_ids"][1]]) - c["margin"]) < 1e-9
        # teacher forcing: the inputs are the prompt, then the fixture's own tokens
        assert len(c["inputs"]) == c["position"] + 1 and c["inputs"][0] == 1
        assert c["inputs"][c["prompt_tokens"]:] == gen[:c["position"] + 1 - c["prompt_tokens"]]


def test_request_inputs():
    assert request_inputs([1, 5, 6], [7, 8, 9], 4) == [1, 5, 6, 7, 8]
    assert request_inputs([1, 5, 6], [7], 1) == [1, 5]
