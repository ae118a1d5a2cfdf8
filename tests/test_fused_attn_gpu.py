"""GPU: the fused QKV + attention launch of the batched multi-launch fp32 step
(hip_llama.cpp_amd/csrc/qkv_attn.hip, THALLAMA_OPT_FUSED_ATTN, 5..8 sequences, head size 64/128).

The fused launch runs the QKV GEMV's own blocks (same tiles, splits and sums, tiles dealt per
kv-head group), so q / k / v are bitwise the two-launch step's; its attention units walk 16-key
chunks (the register budget of a wave that shares the launch with the GEMV) where the stand-alone
attention kernel walks 32, so the online-softmax merges round differently past 16 keys.  The bar is
therefore the oracle's (the reference's src/seq.cpp forward): every logit within 1e-4 under the
reference's abs-or-rel rule (scripts/test/thaDNN.test.cpp:224-229) at independent positions and
across many chunks, greedy tokens equal to the CPU decode's, a step run twice bitwise identical, and
a launch whose waits give up (the fault hook) disables the path and re-runs on the two-launch step.
"""
import numpy as np
import pytest

from helpers import SMALL, SMALL_GQA, assert_ref_close

pytestmark = pytest.mark.gpu

HEAD128 = (512, 1536, 2, 4, 2, 1024, 512)   # head 128, GQA


def decoder(tl, cfg, seed, batch, fused):
    c = tl.Config.make(*cfg)
    model = tl.DeviceModel(c, 0, seed=seed)
    state = tl.DeviceState(c, batch)
    dec = tl.Decoder(model, state)
    dec.set(tl.OPT_PERSISTENT, 0)
    dec.set(tl.OPT_FUSED_ATTN, fused)
    return (model, state), dec


@pytest.mark.parametrize("cfg", [SMALL, HEAD128, SMALL_GQA])
@pytest.mark.parametrize("B", [5, 8])
@pytest.mark.parametrize("graph", [0, 1])
def test_fused_matches_oracle_independent_positions(gpu, oracle, cfg, B, graph):
    """B sequences at their own positions, teacher-forced random tokens: every sequence's logits
    within 1e-4 of its own CPU decode at every step; the last step run twice is bitwise the same."""
    keep, dec = decoder(gpu, cfg, 11, B, 1)
    assert dec.fused_attn() and not dec.persistent()
    dec.set(gpu.OPT_USE_GRAPH, graph)
    rng = np.random.default_rng(B + 10 * graph)
    starts = rng.integers(0, 40, B)
    toks = rng.integers(0, cfg[5], (B, 120))
    refs = [oracle.Model(cfg, 0, seed=11) for _ in range(B)]
    for b in range(B):
        for p in range(int(starts[b])):
            refs[b].forward(int(toks[b, p]), p)
    # every sequence's cache rows up to the longest prefix (a row past a sequence's own start is
    # rewritten with the same token when its step comes)
    for p in range(int(starts.max())):
        dec.forward([int(toks[b, p]) for b in range(B)], [p] * B, want_logits=False)
    for step in range(40):
        ps = [int(starts[b]) + step for b in range(B)]
        tk = [int(toks[b, ps[b]]) for b in range(B)]
        got = dec.forward(tk, ps)
        for b in range(B):
            assert_ref_close(got[b], refs[b].forward(tk[b], ps[b]), 1e-4, f"B={B} b={b} pos={ps[b]}")
    again = dec.forward(tk, ps)
    assert np.array_equal(again.view(np.uint32), got.view(np.uint32))
    assert dec.fused_attn()


@pytest.mark.parametrize("cfg", [SMALL, HEAD128])
def test_fused_greedy_matches_oracle(gpu, oracle, cfg):
    B = 8
    keep, dec = decoder(gpu, cfg, 42, B, 1)
    starts = [1 + 37 * b for b in range(B)]
    n = 40
    got = dec.greedy(starts, [0] * B, n)
    assert dec.fused_attn()
    for b in range(B):
        assert got[:, b].tolist() == oracle.Model(cfg, 0, seed=42).greedy(starts[b], 0, n), f"sequence {b}"


def test_fused_long_context_and_prefill(gpu, oracle):
    """Past 300 positions (19+ chunks of 16 keys, several per unit), one slot filled by prefill (the
    prefill chunks run unfused) among slots that keep decoding: within 1e-4 of the CPU decode."""
    cfg = HEAD128
    B = 6
    keep, dec = decoder(gpu, cfg, 3, B, 1)
    refs = [oracle.Model(cfg, 0, seed=3) for _ in range(B)]
    toks = np.random.default_rng(4).integers(0, cfg[5], (B, 420))
    dec.forward(toks[:, 0].tolist(), [0] * B, want_logits=False)
    for b in range(B):
        refs[b].forward(int(toks[b, 0]), 0)
    assert dec.prefill(2, toks[2, 1:30].tolist(), 1) == 0
    for p in range(1, 30):
        refs[2].forward(int(toks[2, p]), p)
    for p in range(1, 330):
        ps = [p] * B
        ps[2] = 29 + p
        tk = [int(toks[b, ps[b]]) for b in range(B)]
        want = p % 41 == 0 or p == 329
        got = dec.forward(tk, ps, want_logits=want)
        for b in range(B):
            r = refs[b].forward(tk[b], ps[b])
            if want:
                assert_ref_close(got[b], r, 1e-4, f"b={b} pos={ps[b]}")
    assert dec.fused_attn()


@pytest.mark.parametrize("graph", [0, 1])
def test_fused_give_up_falls_back(gpu, oracle, graph):
    """A fused launch whose granule waits give up sets the error word; the call re-runs on the
    two-launch step and the path stays off: tokens still the oracle's."""
    B = 5
    keep, dec = decoder(gpu, SMALL, 42, B, 1)
    dec.set(gpu.OPT_USE_GRAPH, graph)
    starts = [1, 5, 9, 200, 77]
    want = [oracle.Model(SMALL, 0, seed=42).greedy(s, 0, 12) for s in starts]
    got = dec.greedy(starts, [0] * B, 4)
    assert [got[:, b].tolist() for b in range(B)] == [w[:4] for w in want]
    assert dec.fused_attn()
    dec.set(gpu.OPT_PERSIST_FAULT, 1)
    got = dec.greedy([w[3] for w in want], [4] * B, 8)
    assert [got[:, b].tolist() for b in range(B)] == [w[4:12] for w in want]
    assert not dec.fused_attn()


def test_int8_batches_never_take_the_fused_path(gpu):
    """The fused launch is fp32 only: an int8 decoder of 5..8 sequences (created through the fp32
    create, then switched to its int8 weights) reports it off and keeps it off when asked."""
    cfg = SMALL
    c = gpu.Config.make(*cfg)
    m = gpu.DeviceModel(c, 0, seed=5)
    q = gpu.DeviceModelQ8(c, 0, 64, from_model=m)
    st = gpu.DeviceState(c, 8)
    dec = gpu.Decoder(q, st)
    assert not dec.fused_attn()
    dec.set(gpu.OPT_FUSED_ATTN, 1)
    assert not dec.fused_attn()
    dec.greedy([1] * 8, [0] * 8, 3)
