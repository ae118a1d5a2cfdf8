#!/usr/bin/env python3
"""Generate tests/golden/cli_gen_in_128_greedy.json: BASELINE.json configs[0] as a fixture — the
`-m test` output file for all 128 prompts of the reference's assets/in/gen_in_128.txt (copied
verbatim to tests/golden/gen_in_128.txt) on a stories110M-shaped synthetic model, decoded
greedily (`-g 1`), produced by the pinned CPU path:
  * forward: oracle/oracle.c, bit-identical to the reference's src/seq.cpp (tests/test_oracle.py);
  * tokenizer encode/decode and the safe-piece rule: libthallama_host.so, bit-exact against the
    reference's own run.cc/src/llama.cpp code (tests/test_host.py);
  * scheduling / file format: src/llama.cpp:455-505 (read_inputfile / write_outputfile) and
    :891-1083 (test_data_parallelism: prompt tokens forced, then one token per step until
    BOS/EOS or seq_len, one "\\n" appended per request, another per line when written).
The model is written as a v0 model.bin from the synthetic generator (config, seed below), so the
GPU test rebuilds the identical file.  Run: python tests/golden/make_golden_cli.py  (~15-20 min, 8 cores)
"""
import json
import multiprocessing as mp
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "hip_llama.cpp_amd"))

CFG = (768, 2048, 12, 12, 12, 32000, 1024)  # stories110M shape
SHARED = 0  # an unshared classifier: a random-init shared one makes every greedy continuation repeat its last token
SEED = 110
N_PROMPTS = 128
NEAR_TIE = 1e-3  # greedy steps whose top-2 logit margin is below this are recorded (near_ties)
PROMPTS_FILE = os.path.join(HERE, "gen_in_128.txt")
TOK = os.path.join(HERE, "tokenizer.bin")
OUT = os.path.join(HERE, "cli_gen_in_128_greedy.json")


def prompts(n):
    with open(PROMPTS_FILE, "rb") as f:
        lines = f.read().split(b"\n")
    assert int(lines[0]) >= n
    return [l.decode() for l in lines[1:1 + n]]


def decode_one(args):
    idx, prompt = args
    import oracle as O
    import host as H
    m = O.Model(CFG, SHARED, seed=SEED)
    tok = H.Tokenizer(TOK, CFG[5])
    ids = tok.encode(prompt)
    token, pos, text, gen, near = ids[0], 0, b"", [], []
    while True:
        lg = m.forward(token, pos)
        nxt = ids[pos + 1] if pos < len(ids) - 1 else int(np.argmax(lg))  # sample_argmax: lowest index on ties
        if pos >= len(ids) - 1:
            gen.append(nxt)
            top = np.sort(lg.astype(np.float64))[-2:]
            if top[1] - top[0] < NEAR_TIE:  # a near-tie: [pos, margin, text offset before this token]
                near.append([pos, float(top[1] - top[0]), len(text)])
        pos += 1
        if nxt in (1, 2):
            break
        if tok.is_safe(token, nxt):
            text += tok.decode(token, nxt)
        token = nxt
        if pos >= CFG[6]:
            break
    return idx, text + b"\n", pos - 1, gen, near


def main():
    ps = prompts(N_PROMPTS)
    with mp.Pool(min(8, os.cpu_count() or 1)) as pool:
        res = sorted(pool.map(decode_one, list(enumerate(ps))))
    body = f"{len(ps)}\n".encode() + b"".join(r[1] + b"\n" for r in res)
    out = {"generator": "tests/golden/make_golden_cli.py", "config": list(CFG), "shared": SHARED, "seed": SEED,
           "prompts_file": "tests/golden/gen_in_128.txt (= reference assets/in/gen_in_128.txt)",
           "n_prompts": len(ps), "batch_independent": True,
           "output_file": body.decode("latin-1"), "total_achieved_tokens": sum(r[2] for r in res),
           "generated_tokens": [r[3] for r in res],
           "outputs": [r[1].decode("latin-1") for r in res], "achieved_tokens": [r[2] for r in res],
           "near_ties": [r[4] for r in res],
           "near_ties_doc": "per prompt: [position, top-2 margin, byte offset of that token's piece in the output] "
                            "of every greedy step with margin < NEAR_TIE; a GPU decode within the fp32 tolerance may "
                            "take the other branch there (tests/test_cli_gpu.py)"}
    with open(OUT, "w") as f:
        json.dump(out, f)
    print(f"{len(ps)} prompts, {out['total_achieved_tokens']} tokens", file=sys.stderr)


if __name__ == "__main__":
    main()
