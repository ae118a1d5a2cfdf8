#!/usr/bin/env python3
"""Generate tests/golden/requests_llama2-7B_f32_gen_in_64.json: BASELINE.json configs[4]'s request
workload as a fixture made by the pinned CPU path (not by the GPU) — the `-m test -g 1` output of
the first N_PROMPTS prompts of the reference's assets/in/gen_in_64.txt (copied verbatim to
tests/golden/gen_in_64.txt) on the llama2-7B-shaped synthetic model the bench uses (seed 20240224,
unshared classifier), every request run to position DECODE_LEN - 1 or BOS/EOS:
  * forward: oracle/oracle.c's lockstep forward (oracle_forward_multi), bit-identical to its
    single-sequence forward (tests/test_oracle.py::test_lockstep_matches_single_forward), which is
    bit-identical to the reference's src/seq.cpp (tests/test_oracle.py); as a live check at 7B, a
    BOS-started sequence rides along in the first batch and its 256 greedy tokens must equal
    tests/golden/reference_long.json (the reference's own src/seq.cpp, make_golden_long.py);
  * tokenizer encode/decode and the safe-piece rule: libthallama_host.so (bit-exact against the
    reference's run.cc / src/llama.cpp code, tests/test_host.py);
  * scheduling / file format: src/llama.cpp:455-505 and :891-1083 (prompt tokens forced, then one
    greedy token per step until BOS/EOS or the step cap; one "\\n" appended per request, another
    per record when written), with the bench's step cap THALLAMA_TEST_STEPS = DECODE_LEN.
Requests are independent, so the same file is the expected output at any slot count.  Per
generated step the top-2 logit margin is recorded when below NEAR_TIE (near_ties), so a GPU decode
within the fp32 tolerance may be allowed the other branch exactly there (tests/test_requests_gpu.py).

Run: python tests/golden/make_golden_requests.py   (8 cores, ~40 GB of RAM, ~1 h for 64 prompts)
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

CFG = (4096, 11008, 32, 32, 32, 32000, 2048)  # llama2-7B (bench.py MODELS["7b"])
SHARED = 0
SEED = 20240224
DECODE_LEN = 256
N_PROMPTS = int(os.environ.get("N_PROMPTS", "64"))
CHUNK = int(os.environ.get("CHUNK", "32"))  # sequences per lockstep batch (memory: ~270 MB of K/V each)
NEAR_TIE = 1e-3
PROMPTS_FILE = os.path.join(HERE, "gen_in_64.txt")
TOK = os.path.join(HERE, "tokenizer.bin")
OUT = os.path.join(HERE, "requests_llama2-7B_f32_gen_in_64.json")


def main():
    import oracle as O
    from __graft_entry__ import _pkg
    _pkg()
    from hip_llama_cpp_amd import host as H
    O.set_threads(os.cpu_count() or 1)
    tok = H.Tokenizer(TOK, CFG[5])
    mtl = tok.max_token_length
    req = H.Requests(PROMPTS_FILE, mtl, DECODE_LEN)  # read_inputfile, as the CLI reads it
    assert len(req) >= N_PROMPTS
    prompts = [req.prompt(i) for i in range(N_PROMPTS)]
    cap = mtl * DECODE_LEN - 1  # the reference's per-request output buffer, NUL-terminated
    with open(os.path.join(HERE, "reference_long.json")) as f:
        bos_want = next(c for c in json.load(f)["cases"]
                        if tuple(c["config"]) == CFG and c["shared"] == SHARED and c["seed"] == SEED)["fp32"]["tokens"]

    t0 = time.time()
    base = O.Model(CFG, SHARED, seed=SEED)
    print(f"weights made in {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
    results = {}
    bos_got = None
    for c0 in range(0, N_PROMPTS, CHUNK):
        ids_c = list(range(c0, min(N_PROMPTS, c0 + CHUNK)))
        seqs = []  # [request index or -1 (the BOS check), prompt ids]
        for i in ids_c:
            seqs.append([i, tok.encode(prompts[i])])
        if c0 == 0:
            seqs.append([-1, [1]])
        B = len(seqs)
        ls = O.Lockstep(base, B, seq_cap=DECODE_LEN)
        token = [s[1][0] for s in seqs]
        text = [b""] * B
        gen = [[] for _ in range(B)]
        near = [[] for _ in range(B)]
        done = [False] * B
        pos = 0
        while not all(done) and pos < DECODE_LEN:
            act = [b for b in range(B) if not done[b]]
            ts = time.time()
            lg = ls.forward(act, [token[b] for b in act], [pos] * len(act))
            for r, b in enumerate(act):
                ids = seqs[b][1]
                if pos < len(ids) - 1:
                    nxt = ids[pos + 1]
                else:
                    row = lg[r]
                    nxt = int(np.argmax(row))  # sample_argmax: lowest index on ties (src/llama.cpp:275-286)
                    gen[b].append(nxt)
                    top = np.sort(row.astype(np.float64))[-2:]
                    if top[1] - top[0] < NEAR_TIE:  # [position, margin, byte offset of this token's piece]
                        near[b].append([pos, float(top[1] - top[0]), len(text[b])])
                if seqs[b][0] < 0:  # the BOS sequence: greedy from position 0, no text
                    if len(gen[b]) >= len(bos_want):
                        done[b] = True
                    token[b] = nxt
                    continue
                if nxt in (1, 2):
                    done[b] = True
                    continue
                if tok.is_safe(token[b], nxt):
                    text[b] += tok.decode(token[b], nxt)
                token[b] = nxt
                if pos + 1 >= DECODE_LEN:
                    done[b] = True
            pos += 1
            if pos % 16 == 0 or pos < 3:
                print(f"chunk {c0}: position {pos} ({len(act)} active) {time.time() - ts:.1f} s/step, "
                      f"{time.time() - t0:.0f} s total", file=sys.stderr, flush=True)
        for b, (i, _) in enumerate(seqs):
            if i < 0:
                bos_got = gen[b]
                continue
            out = (text[b] + b"\n")[:cap]
            # achieved tokens: pos - 1 at the end of the request (src/llama.cpp:1062)
            n_steps = len(seqs[b][1]) - 1 + len(gen[b])
            results[i] = {"output": out, "generated": gen[b], "near": near[b], "achieved": n_steps - 1}
        ls.close()
    if bos_got != bos_want:
        k = next(i for i, (a, b) in enumerate(zip(bos_got, bos_want)) if a != b)
        raise SystemExit(f"BOS check FAILED: the lockstep decode leaves src/seq.cpp's tokens at step {k}")
    res = [results[i] for i in range(N_PROMPTS)]
    body = f"{N_PROMPTS}\n".encode() + b"".join(r["output"] + b"\n" for r in res)
    fx = {"generator": "tests/golden/make_golden_requests.py (oracle/oracle.c lockstep forward, bit-identical to "
                       "the reference's src/seq.cpp; host tokenizer bit-exact to its run.cc)",
          "model": "llama2-7B", "dtype": "f32", "config": list(CFG), "shared": SHARED, "seed": SEED,
          "decode_len": DECODE_LEN, "prompts": "tests/golden/gen_in_64.txt (reference assets/in/gen_in_64.txt)",
          "n_prompts": N_PROMPTS, "batch_independent": True,
          "bos_check": {"steps": len(bos_want), "tokens_match": True,
                        "source": "tests/golden/reference_long.json (the reference's src/seq.cpp compiled from source)"},
          "output_file": body.decode("latin-1"),
          "outputs": [r["output"].decode("latin-1") for r in res],
          "generated_tokens": [r["generated"] for r in res],
          "achieved_tokens": [r["achieved"] for r in res],
          "total_achieved_tokens": sum(r["achieved"] for r in res),
          "near_ties": [r["near"] for r in res],
          "near_ties_doc": "per prompt: [position, top-2 margin, byte offset of that token's piece in the output] of "
                           "every greedy step with margin < NEAR_TIE; a GPU decode within the fp32 tolerance may take "
                           "the other branch there",
          "seconds": round(time.time() - t0)}
    with open(OUT, "w") as f:
        json.dump(fx, f)
    print(f"{N_PROMPTS} prompts, {fx['total_achieved_tokens']} tokens, {fx['seconds']} s -> {OUT}", file=sys.stderr)


if __name__ == "__main__":
    main()
