"""GPU parity of the batched persistent decode step (hip_llama.cpp_amd/csrc/persist_b.hip: the
whole step of 2..8 sequences as ONE launch, fp32) against the CPU oracle (the reference's
src/seq.cpp forward, pinned in tests/test_oracle.py).

Bar (BASELINE.json north_star): every sequence's greedy tokens equal its own CPU decode's; fp32
logits within 1e-4 under the reference's abs-or-rel rule (scripts/test/thaDNN.test.cpp:224-229).
The batched step applies RMSNorm as (W (w * x)) * ss per row (its K-passes cannot see the whole
row's sum of squares first), a last-bit difference from src/seq.cpp:3-16 the same rule covers.
Shapes: head 64 and 128, GQA, a hidden size that ends mid-chunk (W2 in two K-passes, the second
partial), 2..8 sequences at independent positions (the K-pass strip holds 2, 4 or 8 rows).
"""
import numpy as np
import pytest

from helpers import SMALL, SMALL_GQA, assert_ref_close

pytestmark = pytest.mark.gpu

HEAD128 = (512, 1536, 2, 4, 2, 1024, 512)       # head 128, GQA (kv_dim 256)
RAGGED = (1024, 2816, 2, 8, 8, 1024, 256)       # head 128; hidden 2816 = one chunk + 768 (like 11008)


def decoder(tl, cfg, seed, batch, persistent=1):
    c = tl.Config.make(*cfg)
    model = tl.DeviceModel(c, 0, seed=seed)
    state = tl.DeviceState(c, batch)
    dec = tl.Decoder(model, state)
    dec.set(tl.OPT_PERSISTENT, persistent)
    return (model, state), dec


@pytest.mark.parametrize("cfg", [SMALL, HEAD128, RAGGED, SMALL_GQA])
@pytest.mark.parametrize("B", [2, 3, 5, 8])
def test_independent_positions_match_oracle(gpu, oracle, cfg, B):
    """B sequences at different positions, teacher-forced random tokens: every sequence's logits
    within 1e-4 of its own CPU decode at every step."""
    keep, dec = decoder(gpu, cfg, 5, B)
    assert dec.persistent()
    rng = np.random.default_rng(B)
    starts = rng.integers(0, 20, B)
    toks = rng.integers(0, cfg[5], (B, 48))
    refs = [oracle.Model(cfg, 0, seed=5) for _ in range(B)]
    for b in range(B):
        for p in range(int(starts[b])):
            refs[b].forward(int(toks[b, p]), p)
    for p in range(int(starts.max())):
        dec.forward([int(toks[b, p]) for b in range(B)], [p] * B, want_logits=False)
    for step in range(10):
        ps = [int(starts[b]) + step for b in range(B)]
        tk = [int(toks[b, ps[b]]) for b in range(B)]
        got = dec.forward(tk, ps)
        for b in range(B):
            assert_ref_close(got[b], refs[b].forward(tk[b], ps[b]), 1e-4, f"B={B} b={b} pos={ps[b]}")


@pytest.mark.parametrize("cfg", [SMALL, HEAD128])
@pytest.mark.parametrize("B", [4, 8])
@pytest.mark.parametrize("graph", [0, 1])
def test_greedy_matches_oracle(gpu, oracle, cfg, B, graph):
    """Greedy decode of B sequences from different start tokens, on the device (argmax per
    sequence in the step's tail): every sequence's tokens equal the oracle's greedy decode."""
    keep, dec = decoder(gpu, cfg, 42, B)
    dec.set(gpu.OPT_USE_GRAPH, graph)
    starts = [1 + 37 * b for b in range(B)]
    n = 40
    got = dec.greedy(starts, [0] * B, n)
    for b in range(B):
        want = oracle.Model(cfg, 0, seed=42).greedy(starts[b], 0, n)
        assert got[:, b].tolist() == want, f"sequence {b}"


def test_long_context(gpu, oracle):
    """Past many 16-key attention chunks (the units split each head's keys NS ways)."""
    cfg = HEAD128
    B = 4
    keep, dec = decoder(gpu, cfg, 21, B)
    refs = [oracle.Model(cfg, 0, seed=21) for _ in range(B)]
    toks = np.random.default_rng(8).integers(0, cfg[5], (B, 400))
    for p in range(400):
        want = [refs[b].forward(int(toks[b, p]), p) for b in range(B)]
        got = dec.forward(toks[:, p].tolist(), [p] * B, want_logits=(p % 53 == 0 or p == 399))
        if got is not None:
            for b in range(B):
                assert_ref_close(got[b], want[b], 1e-4, f"b={b} pos={p}")


def test_matches_multilaunch_tokens(gpu):
    """Same greedy tokens as the multi-launch batched step on a 110M-class shape."""
    cfg = (768, 2048, 4, 12, 12, 32000, 256)
    B = 8
    keep, dp = decoder(gpu, cfg, 7, B, 1)
    keep2, dm = decoder(gpu, cfg, 7, B, 0)
    assert dp.persistent() and not dm.persistent()
    starts = [1 + 1000 * b for b in range(B)]
    a = dp.greedy(starts, [0] * B, 64)
    m = dm.greedy(starts, [0] * B, 64)
    assert (a == m).all()


@pytest.mark.parametrize("graph", [0, 1])
def test_give_up_falls_back(gpu, oracle, graph):
    """A batched persistent launch missing a block gives up (bounded waits), the path is disabled
    and the call re-runs on the multi-launch step: tokens still the oracle's."""
    B = 4
    keep, dec = decoder(gpu, SMALL, 42, B)
    dec.set(gpu.OPT_USE_GRAPH, graph)
    starts = [1, 5, 9, 200]
    want = [oracle.Model(SMALL, 0, seed=42).greedy(s, 0, 12) for s in starts]
    got = dec.greedy(starts, [0] * B, 4)
    assert [got[:, b].tolist() for b in range(B)] == [w[:4] for w in want]
    assert dec.persistent()
    dec.set(gpu.OPT_PERSIST_FAULT, 1)
    got = dec.greedy([w[3] for w in want], [4] * B, 8)
    assert [got[:, b].tolist() for b in range(B)] == [w[4:12] for w in want]
    assert not dec.persistent()
