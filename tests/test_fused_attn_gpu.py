"""GPU: the fused QKV + attention launch of the batched multi-launch fp32 step
(hip_llama.cpp_amd/csrc/qkv_attn.hip, THALLAMA_OPT_FUSED_ATTN, 5..8 sequences, head size 64/128).

The fused launch runs the QKV GEMV's own blocks (same tiles, splits and sums, tiles dealt per
kv-head group) and attn_unit's multi-launch arithmetic (q and this step's k/v row arrive as
granules instead of through the cache), so its logits must be BITWISE those of the two-launch step
— checked at independent positions, across many 16-key chunks, with and without graphs — and the
oracle bar of every batched path holds (greedy tokens equal the CPU decode's).  A launch whose
waits give up (the fault hook) disables the path and the call re-runs on the two-launch step.
"""
import numpy as np
import pytest

from helpers import SMALL, SMALL_GQA

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
def test_fused_bitwise_equals_two_launches(gpu, cfg, B, graph):
    """B sequences at their own positions, teacher-forced: every logit bitwise equal."""
    keep_f, df = decoder(gpu, cfg, 11, B, 1)
    keep_m, dm = decoder(gpu, cfg, 11, B, 0)
    assert df.fused_attn() and not dm.fused_attn() and not df.persistent()
    for d in (df, dm):
        d.set(gpu.OPT_USE_GRAPH, graph)
    rng = np.random.default_rng(B + 10 * graph)
    starts = rng.integers(0, 40, B)
    toks = rng.integers(0, cfg[5], (B, 120))
    for step in range(70):
        ps = [int(starts[b]) + step for b in range(B)]
        tk = [int(toks[b, ps[b]]) for b in range(B)]
        a, m = df.forward(tk, ps), dm.forward(tk, ps)
        assert np.array_equal(a.view(np.uint32), m.view(np.uint32)), f"step {step}"
    assert df.fused_attn()


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


def test_fused_long_context_and_prefill(gpu):
    """Past 300 positions (19+ chunks of 16 keys, several per unit), a slot refilled by prefill (the
    prefill chunks run unfused) among slots that keep decoding: bitwise the two-launch step."""
    cfg = HEAD128
    B = 6
    keep_f, df = decoder(gpu, cfg, 3, B, 1)
    keep_m, dm = decoder(gpu, cfg, 3, B, 0)
    toks = np.random.default_rng(4).integers(0, cfg[5], (B, 420))
    for d in (df, dm):
        d.forward(toks[:, 0].tolist(), [0] * B, want_logits=False)
        assert d.prefill(2, toks[2, :30].tolist(), 0) == 0
    for p in range(1, 330):
        ps = [p] * B
        ps[2] = 29 + p
        tk = [int(toks[b, ps[b]]) for b in range(B)]
        want = p % 41 == 0 or p == 329
        a, m = df.forward(tk, ps, want_logits=want), dm.forward(tk, ps, want_logits=want)
        if want:
            assert np.array_equal(a.view(np.uint32), m.view(np.uint32)), f"position {p}"
    assert df.fused_attn()


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
