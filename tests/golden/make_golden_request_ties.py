#!/usr/bin/env python3
"""Generate tests/golden/request_ties_llama2-7B_f32.{json,npz}: the CPU reference's logits at every
near-tie step of the 7B request fixture (tests/golden/requests_llama2-7B_f32_gen_in_64.json) whose
top-2 margin is under bench.REQUEST_TIE_7B — the only steps where the GPU's greedy decode may leave
the fixture (bench.compare_request_file).

For each such (request, position) the oracle (oracle/oracle.c's lockstep forward, bit-identical to the
reference's src/seq.cpp: tests/test_oracle.py) is teacher-forced on the request's own history — its
prompt tokens, then the fixture's generated tokens — up to that position, and the whole logit row of
that step is stored (npz, float32), with the top-2 token ids and values (json).  The GPU test
(tests/test_requests_gpu.py) replays a diverged request on the GPU the same way, with the CLI's own
prefill, and asserts that its logits at that step are within 1e-4 of these under the reference's
abs-or-rel rule (scripts/test/thaDNN.test.cpp:224-229), so the divergence is a flip of a tie the fp32
tolerance covers, not an error.

Run: python tests/golden/make_golden_request_ties.py   (8 cores, ~30 GB of RAM, ~10 min)
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, REPO)

FIXTURE = os.path.join(HERE, "requests_llama2-7B_f32_gen_in_64.json")
OUT_JSON = os.path.join(HERE, "request_ties_llama2-7B_f32.json")
OUT_NPZ = os.path.join(HERE, "request_ties_llama2-7B_f32.npz")
TOK = os.path.join(HERE, "tokenizer.bin")
PROMPTS_FILE = os.path.join(HERE, "gen_in_64.txt")


def request_inputs(ids, gen, t):
    """The input token of each position 0..t of a request: the prompt's ids, then its generated tokens
    (the output of position p >= len(ids) - 1 is gen[p - len(ids) + 1], the input of the next)."""
    return [ids[p] if p < len(ids) else gen[p - len(ids)] for p in range(t + 1)]


def main():
    import bench
    import oracle as O
    from __graft_entry__ import _pkg
    _pkg()
    from hip_llama_cpp_amd import host as H
    with open(FIXTURE) as f:
        fx = json.load(f)
    cfg = tuple(fx["config"])
    O.set_threads(os.cpu_count() or 1)
    tok = H.Tokenizer(TOK, cfg[5])
    req = H.Requests(PROMPTS_FILE, tok.max_token_length, fx["decode_len"])
    cases = []
    for i, ties in enumerate(fx["near_ties"]):
        for pos, margin, off in ties:
            if margin < bench.REQUEST_TIE_7B:
                ids = tok.encode(req.prompt(i))
                cases.append({"request": i, "position": pos, "margin": margin, "byte_offset": off,
                              "prompt_tokens": len(ids),
                              "inputs": request_inputs(ids, fx["generated_tokens"][i], pos)})
    t0 = time.time()
    base = O.Model(cfg, fx["shared"], seed=fx["seed"])
    ls = O.Lockstep(base, len(cases), seq_cap=fx["decode_len"])
    rows = [None] * len(cases)
    for p in range(max(c["position"] for c in cases) + 1):
        act = [k for k, c in enumerate(cases) if p <= c["position"]]
        lg = ls.forward(act, [cases[k]["inputs"][p] for k in act], [p] * len(act))
        for r, k in enumerate(act):
            if p == cases[k]["position"]:
                rows[k] = lg[r].copy()
        if p % 32 == 0:
            print(f"position {p} ({len(act)} active) {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
    ls.close()
    base.close()
    for k, c in enumerate(cases):
        row = rows[k]
        top = np.argsort(-row.astype(np.float64), kind="stable")[:2]  # ties: lowest index first (np.argmax)
        assert int(top[0]) == int(np.argmax(row))
        gen = fx["generated_tokens"][c["request"]]
        assert int(top[0]) == gen[c["position"] - c["prompt_tokens"] + 1], "the fixture's own greedy token"
        c["top2_ids"] = [int(v) for v in top]
        c["top2_logits"] = [float(row[v]) for v in top]
        assert abs((c["top2_logits"][0] - c["top2_logits"][1]) - c["margin"]) < 1e-9
    with open(OUT_JSON, "w") as f:
        json.dump({"generator": "tests/golden/make_golden_request_ties.py (oracle/oracle.c lockstep forward, "
                                "bit-identical to the reference's src/seq.cpp), teacher-forced",
                   "fixture": os.path.relpath(FIXTURE, REPO), "config": list(cfg), "seed": fx["seed"],
                   "tie_margin": bench.REQUEST_TIE_7B, "cases": cases,
                   "logits": os.path.relpath(OUT_NPZ, REPO), "seconds": round(time.time() - t0)}, f)
    np.savez_compressed(OUT_NPZ, logits=np.stack(rows).astype(np.float32))
    print(f"{len(cases)} tie steps -> {OUT_JSON}", file=sys.stderr)


if __name__ == "__main__":
    main()
