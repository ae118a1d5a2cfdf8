"""CPU: pin the oracle (oracle/oracle.c) before trusting it.

1. against the committed golden fixtures produced by the REFERENCE itself
   (tests/golden/make_golden.py -> oracle/_ref, i.e. /root/reference/src/seq.cpp and runq.c):
   identical greedy tokens and bit-identical logit digests;
2. against the live reference build (oracle/_ref), when present: bit-identical logits;
3. op-level known answers.
"""
import json
import os
import struct

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden", "reference_greedy.json")


def f32bits(x):
    return struct.unpack("<I", struct.pack("<f", float(x)))[0]


def load_cases():
    with open(GOLDEN) as f:
        return json.load(f)["cases"]


@pytest.mark.parametrize("case", load_cases(), ids=lambda c: c["name"])
def test_oracle_matches_reference_golden(oracle, case):
    cfg = tuple(case["config"])
    m = oracle.Model(cfg, case["shared"], seed=case["seed"])
    tok = case["start_token"]
    toks = []
    for p in range(case["steps"]):
        lg = m.forward(tok, p)
        d = case["digests"][p]
        assert [f32bits(v) for v in lg[:8]] == d["head_bits"], f"step {p}: logits differ from the reference"
        top = np.argsort(-lg.astype(np.float64), kind="stable")[:5]
        assert [int(i) for i in top] == d["top5"]
        assert [f32bits(lg[i]) for i in top] == d["top5_bits"]
        assert float(lg.astype(np.float64).sum()) == d["sum"]
        tok = int(np.argmax(lg))
        toks.append(tok)
    assert toks == case["tokens"]


@pytest.mark.parametrize("case", [c for c in load_cases() if "q8" in c], ids=lambda c: c["name"])
def test_q8_oracle_matches_reference_golden(oracle, case):
    cfg = tuple(case["config"])
    m = oracle.Model(cfg, case["shared"], seed=case["seed"])
    m.build_q8(case["q8"]["group_size"])
    tok = case["start_token"]
    toks = []
    for p in range(case["steps"]):
        lg = m.q8_forward(tok, p)
        d = case["q8"]["digests"][p]
        assert [f32bits(v) for v in lg[:8]] == d["head_bits"], f"q8 step {p}"
        assert float(lg.astype(np.float64).sum()) == d["sum"]
        tok = int(np.argmax(lg))
        toks.append(tok)
    assert toks == case["q8"]["tokens"]


@pytest.mark.skipif(not os.path.exists(os.path.join(os.path.dirname(HERE), "oracle", "_ref", "libref_seq.so")),
                    reason="reference build oracle/_ref absent")
def test_oracle_bitexact_vs_live_reference(oracle, tmp_path):
    cfg = (128, 384, 2, 8, 4, 700, 48)   # GQA, odd vocab
    for shared in (0, 1):
        m = oracle.Model(cfg, shared, seed=99)
        path = str(tmp_path / f"m{shared}.bin")
        m.write_v0(path)
        rtoks, rlog = oracle.ref_greedy(path, 3, 0, 16, cfg[5])
        m2 = oracle.Model(cfg, shared, seed=99)
        seq = [3] + rtoks[:-1]
        for p, t in enumerate(seq):
            np.testing.assert_array_equal(m2.forward(t, p), rlog[p])


def test_oracle_thread_count_invariant(oracle):
    cfg = (256, 768, 2, 4, 4, 1024, 64)
    outs = []
    for th in (1, 4):
        oracle.set_threads(th)
        m = oracle.Model(cfg, 0, seed=3)
        outs.append(np.stack([m.forward(t, p) for p, t in enumerate([1, 2, 3, 4])]))
    oracle.set_threads(1)
    np.testing.assert_array_equal(outs[0], outs[1])


@pytest.mark.skipif(not os.path.exists(os.path.join(os.path.dirname(HERE), "oracle", "_ref", "libref_seq_f64.so")),
                    reason="reference build oracle/_ref absent")
@pytest.mark.parametrize("cfg,shared", [((768, 2048, 2, 12, 12, 32000, 64), 0),   # stories110M-shaped layers
                                        ((128, 384, 2, 8, 4, 700, 48), 1),        # GQA, shared classifier
                                        ((128, 384, 3, 8, 2, 700, 48), 0)])       # kv_mul 4
def test_forward_f64_matches_widened_reference(oracle, tmp_path, cfg, shared):
    """oracle_forward_f64 — the 'exact' forward the GPU's and the CPU's logits are measured against
    (tests/test_golden_2048_gpu.py) — pinned to the reference itself: its src/seq.cpp compiled with
    float widened to double (oracle/ref_f64_driver.cpp, read in place) gives BIT-IDENTICAL logits at
    every position of a teacher-forced run when forward_f64 also computes RoPE's (cos, sin) in double
    and keeps its own double K/V rows.  Its default mode differs from that only by taking the
    reference's float RoPE parameters and the caller's fp32 K/V rows, both inputs rather than
    accumulations; at this size that moves logits by less than the fp32 forward's own rounding."""
    m = oracle.Model(cfg, shared, seed=11)
    path = str(tmp_path / "m.bin")
    m.write_v0(path)
    V = abs(cfg[5])
    toks = [int(t) for t in np.random.default_rng(cfg[2]).integers(0, V, 14)]
    ref = oracle.ref64_forced(path, toks, V)
    worst_default, worst_fp32 = 0.0, 0.0
    for p, t in enumerate(toks):
        np.testing.assert_array_equal(m.forward_f64(t, p, rope_double=True, own_cache=True), ref[p],
                                      err_msg=f"position {p}")
        dflt = m.forward_f64(t, p)  # (reads the fp32 cache rows of the fp32 forwards before it)
        fp32 = m.forward(t, p).astype(np.float64)
        worst_default = max(worst_default, float(np.abs(dflt - ref[p]).max()))
        worst_fp32 = max(worst_fp32, float(np.abs(fp32 - ref[p]).max()))
    assert worst_default < worst_fp32, (worst_default, worst_fp32)


def test_lockstep_matches_single_forward(oracle):
    """oracle_forward_multi (the fixture generator of make_golden_requests.py) is bit-identical to
    the single-sequence forward: 21 sequences (two 16-sequence tiles), GQA, row counts that end
    mid-tile, sequences entering at different steps (ragged positions in one call), a capped cache."""
    cfg = (120, 332, 2, 6, 3, 251, 48)
    B, steps = 21, 14
    oracle.set_threads(4)
    base = oracle.Model(cfg, 0, seed=41)
    ls = oracle.Lockstep(base, B, seq_cap=steps)
    rng = np.random.default_rng(5)
    toks = rng.integers(0, cfg[5], size=(B, steps))
    start = [b % 4 for b in range(B)]  # sequence b enters at step start[b]
    singles = [oracle.Model(cfg, 0, seed=41) for _ in range(3)]  # one reference model reused per b
    want = {}
    for b in range(B):
        m = singles[b % 3]
        m.reset_kv()
        for p in range(steps - start[b]):
            want[(b, p)] = m.forward(int(toks[b, p]), p)
    for s in range(steps):
        idx = [b for b in range(B) if s >= start[b]]
        pos = [s - start[b] for b in idx]
        lg = ls.forward(idx, [toks[b, p] for b, p in zip(idx, pos)], pos)
        for r, (b, p) in enumerate(zip(idx, pos)):
            np.testing.assert_array_equal(lg[r], want[(b, p)], err_msg=f"sequence {b} position {p}")
    oracle.set_threads(1)
    with pytest.raises(ValueError):
        ls.forward([0], [1], [steps])  # past the capped cache


def test_ops_known_answers(oracle):
    # rmsnorm of a constant vector is the weight (ss = 1/|c|): x=2 -> 1/sqrt(4+1e-5)*2
    x = np.full(16, 2.0, np.float32)
    w = np.arange(16, dtype=np.float32)
    o = oracle.rmsnorm(x, w)
    ss = np.float32(1.0) / np.sqrt(np.float32(np.float32(64.0) / 16 + np.float32(1e-5)))
    np.testing.assert_allclose(o, w * (ss * 2), rtol=1e-7)
    # softmax sums to one, is shift-invariant
    s = oracle.softmax(np.array([1.0, 2.0, 3.0], np.float32))
    np.testing.assert_allclose(s.sum(), 1.0, rtol=1e-6)
    np.testing.assert_allclose(s, oracle.softmax(np.array([11.0, 12.0, 13.0], np.float32)), rtol=1e-6)
    # RoPE at pos 0 is the identity
    q = np.arange(8, dtype=np.float32)
    q2, k2 = oracle.rope(q, q, 8, 4, 8, 0)
    np.testing.assert_array_equal(q2, q)
    # matmul
    W = np.arange(12, dtype=np.float32).reshape(3, 4)
    np.testing.assert_array_equal(oracle.matmul(W, np.ones(4, np.float32)), W.sum(1))
    # swiglu(0, anything) = 0 and silu(x)*1 -> x*sigmoid(x)
    np.testing.assert_array_equal(oracle.swiglu(np.zeros(3, np.float32), np.ones(3, np.float32)), 0)


def test_q8_quantize_rules(oracle):
    # runq.c:145-171: scale = max|x|/127, q = round-half-away(x/scale)
    x = np.array([0.5, -1.0, 0.25, 127.0 / 254] * 16, np.float32)
    q, s = oracle.q8_quantize(x, 64)
    assert s[0] == np.float32(1.0) / np.float32(127.0)
    assert q[1] == -127 and q[0] == 64  # 0.5*127 = 63.5 -> 64 (away from zero)
    # export.py weight quantisation rounds half to even
    qw, sw = oracle.q8_quantize_weights(x, 64)
    assert qw[0] == 64 or qw[0] == 63
    # all-zero group: scale 0 -> q = 0 (NaN cast)
    qz, sz = oracle.q8_quantize(np.zeros(64, np.float32), 64)
    assert sz[0] == 0 and (qz == 0).all()


def test_synth_generator_statistics(oracle):
    v = oracle.synth_fill(1 << 20, 123, 3, 0.02)
    assert abs(float(v.mean())) < 1e-3
    assert abs(float(v.std()) - 0.02) < 5e-4
    # deterministic and offset-consistent
    np.testing.assert_array_equal(oracle.synth_fill(100, 123, 3, 0.02, offset=50), v[50:150])
