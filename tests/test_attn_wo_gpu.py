"""The fused attention + Wo launch of the batched multi-launch step (csrc/attn_wo.hip): 5..8
sequences, fp32, head size 64 / 128.  Each layer's attention units and its Wo GEMV (+ residual and
the next norm's sums of squares) run in one launch, the Wo waves waiting for the heads their K range
needs.  Checked against the CPU oracle (the bit-exact src/seq.cpp restatement) at north_star's 1e-4
(the reference's abs-or-rel rule), against the two-launch step, through a graph, and through the
give-up path (a workgroup that never runs its attention units)."""
import numpy as np
import pytest

from helpers import SMALL_GQA, assert_ref_close

pytestmark = pytest.mark.gpu

HEAD128 = (1024, 2816, 2, 8, 8, 1536, 320)    # head size 128, 64 tiles
HEAD64_MHA = (512, 1376, 3, 8, 8, 1024, 200)  # head size 64, hidden ending mid-chunk


def make(tl, cfg, B, seed, fuse=1):
    c = tl.Config.make(*cfg)
    model = tl.DeviceModel(c, 0, seed=seed)
    state = tl.DeviceState(c, B)
    dec = tl.Decoder(model, state)
    dec.set(tl.OPT_FUSE_ATTN_WO, fuse)
    return (model, state), dec


@pytest.mark.parametrize("cfg", [SMALL_GQA, HEAD128, HEAD64_MHA])
@pytest.mark.parametrize("B", [5, 8])
def test_fused_matches_oracle_independent_positions(gpu, oracle, cfg, B):
    """B sequences at their own positions, up to ~100 keys (several key splits per head, so the
    combining unit is the one that signals the head), every step's logits vs the oracle."""
    keep, dec = make(gpu, cfg, B, seed=17)
    assert dec.fused_attn_wo()
    rng = np.random.default_rng(B + cfg[0])
    starts = rng.integers(0, 60, B)
    toks = rng.integers(0, cfg[5], (B, 120))
    refs = [oracle.Model(cfg, 0, seed=17) for _ in range(B)]
    for b in range(B):
        for p in range(int(starts[b])):
            refs[b].forward(int(toks[b, p]), p)
    for p in range(int(starts.max())):
        dec.forward([int(toks[b, p]) for b in range(B)], [p] * B, want_logits=False)
    for step in range(40):
        ps = [int(starts[b]) + step for b in range(B)]
        tk = [int(toks[b, ps[b]]) for b in range(B)]
        got = dec.forward(tk, ps)
        for b in range(B):
            assert_ref_close(got[b], refs[b].forward(tk[b], ps[b]), 1e-4, f"b={b} pos={ps[b]}")
    assert dec.fused_attn_wo()


def test_fused_equals_two_launch_step(gpu):
    """The fused launch against the two-launch step (attention, then the split-K matrix-core Wo):
    the same arithmetic up to the order the Wo partial sums are added, so within 2e-5."""
    cfg, B = HEAD128, 8
    k1, fused = make(gpu, cfg, B, seed=23, fuse=1)
    k2, plain = make(gpu, cfg, B, seed=23, fuse=0)
    assert fused.fused_attn_wo() and not plain.fused_attn_wo()
    rng = np.random.default_rng(3)
    for p in range(70):
        tk = [int(t) for t in rng.integers(0, cfg[5], B)]
        a, b = fused.forward(tk, [p] * B), plain.forward(tk, [p] * B)
        assert_ref_close(a, b, 2e-5, f"pos {p}")


def test_fused_greedy_graph_matches_oracle(gpu, oracle):
    """Greedy decode of 8 sequences from different start tokens replayed from a captured graph:
    every token equals the oracle's greedy decode."""
    cfg, B, n = SMALL_GQA, 8, 48
    keep, dec = make(gpu, cfg, B, seed=29)
    dec.set(gpu.OPT_USE_GRAPH, 1)
    starts = [1 + 37 * b for b in range(B)]
    got = dec.greedy(starts, [0] * B, n)
    for b in range(B):
        want = oracle.Model(cfg, 0, seed=29).greedy(starts[b], 0, n)
        assert got[:, b].tolist() == want, f"sequence {b}"
    assert dec.fused_attn_wo()


@pytest.mark.parametrize("graph", [0, 1])
def test_fused_give_up_falls_back(gpu, oracle, graph):
    """A fused launch whose workgroup 0 never runs its attention units (THALLAMA_OPT_PERSIST_FAULT,
    the co-residency failure the bounded waits guard against): its waits give up, the call reports
    it, disables the fused launch and re-runs on the two-launch step — the logits are still the
    oracle's and later steps stay correct."""
    cfg, B = SMALL_GQA, 6
    keep, dec = make(gpu, cfg, B, seed=31)
    dec.set(gpu.OPT_USE_GRAPH, graph)
    refs = [oracle.Model(cfg, 0, seed=31) for _ in range(B)]
    for p in range(6):
        tk = [(11 * b + 5 * p) % cfg[5] for b in range(B)]
        if p == 3:
            dec.set(gpu.OPT_PERSIST_FAULT, 1)
        got = dec.forward(tk, [p] * B)
        for b in range(B):
            assert_ref_close(got[b], refs[b].forward(tk[b], p), 1e-4, f"b={b} pos={p}")
        assert dec.fused_attn_wo() == (p < 3)
