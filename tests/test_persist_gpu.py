"""GPU parity of the one-launch persistent decode step (hip_llama.cpp_amd/csrc/persist.hip)
against the CPU oracle (the reference src/seq.cpp forward, pinned in tests/test_oracle.py) and
against the multi-launch step it replaces.

Bar: greedy token ids identical to the oracle's; fp32 logits within 1e-4 (reference abs-or-rel
rule, scripts/test/thaDNN.test.cpp:224-229).  The persistent step sums each 8-KiB row chunk
separately, so its logits are NOT bit-identical to the multi-launch step's: they are compared
under the same 1e-4 rule.
"""
import numpy as np
import pytest

from helpers import SMALL, SMALL_GQA, TINY, assert_ref_close

pytestmark = pytest.mark.gpu

HEAD128 = (512, 1536, 2, 4, 2, 1024, 512)       # head 128, GQA (kv_dim 256)
RAGGED = (1024, 2816, 2, 8, 8, 1024, 256)       # head 128; hidden 2816 ends mid-chunk (like 11008)
HEAD64_GQA = (512, 1536, 3, 8, 2, 2048, 256)   # = SMALL_GQA: head 64, kv_dim 128
WIDE = (2048, 5632, 2, 16, 4, 1024, 256)       # dim >= 2048: late granules re-polled with the back-off


def decoder(tl, cfg, shared, seed, persistent, batch=1):
    c = tl.Config.make(*cfg)
    model = tl.DeviceModel(c, shared, seed=seed)
    state = tl.DeviceState(c, batch)
    dec = tl.Decoder(model, state)
    dec.set(tl.OPT_PERSISTENT, persistent)
    return c, model, state, dec


def test_selection(gpu):
    for cfg, want in [(SMALL, True), (HEAD128, True), (RAGGED, True), (TINY, False)]:
        _, _, _, dec = decoder(gpu, cfg, 0, 1, 1)
        assert dec.persistent() == want, cfg
        dec.set(gpu.OPT_PERSISTENT, 0)
        assert not dec.persistent()
    # 2..8 sequences: the batched persistent step (persist_b.hip, tests/test_persist_b_gpu.py)
    _, _, _, dec = decoder(gpu, SMALL, 0, 1, 1, batch=2)
    assert dec.persistent()
    # 5..8: prepared, but multi-launch unless asked for (forward.hip batch_persist_default_max)
    c = gpu.Config.make(*SMALL)
    model, state = gpu.DeviceModel(c, 0, seed=0), gpu.DeviceState(c, 8)
    dec = gpu.Decoder(model, state)
    assert not dec.persistent()
    dec.set(gpu.OPT_PERSISTENT, 1)
    assert dec.persistent()
    _, _, _, dec = decoder(gpu, SMALL, 0, 1, 1, batch=9)
    assert not dec.persistent()


def test_profiled_as_one_class(gpu):
    _, _, _, dec = decoder(gpu, SMALL, 0, 1, 1)
    dec.set(gpu.OPT_PROFILE, 1)
    dec.prof_reset()
    dec.greedy([1], [0], 5)
    ms, n = dec.prof(gpu.K_STEP)
    assert n == 5 and ms > 0
    assert dec.prof(gpu.K_QKV)[1] == 0


@pytest.mark.parametrize("cfg,shared", [(SMALL, 0), (HEAD128, 0), (RAGGED, 0), (HEAD64_GQA, 0), (SMALL, 1), (WIDE, 0)])
@pytest.mark.parametrize("graph", [0, 1])
def test_greedy_matches_oracle(gpu, oracle, cfg, shared, graph):
    _, _, _, dec = decoder(gpu, cfg, shared, 42, 1)
    assert dec.persistent()
    dec.set(gpu.OPT_USE_GRAPH, graph)
    ref = oracle.Model(cfg, shared, seed=42)
    n = 40
    want = ref.greedy(1, 0, n)
    got = dec.greedy([1], [0], n)[:, 0].tolist()
    assert got == want
    fresh = oracle.Model(cfg, shared, seed=42)
    for p, t in enumerate([1] + want[:-1]):
        last = fresh.forward(t, p)
    assert_ref_close(dec.logits()[0], last, 1e-4, "last-step logits")


@pytest.mark.parametrize("graph", [0, 1])
@pytest.mark.parametrize("cfg", [SMALL, WIDE])
def test_give_up_falls_back(gpu, oracle, graph, cfg):
    """A persistent launch whose grid is not co-resident (simulated: block 0 missing) must not
    hang or return garbage: its bounded waits give up, the call disables the path and re-runs
    on the multi-launch step, and the tokens still equal the oracle's.  WIDE: the waits back off
    to ~2000-cycle pauses (common.hpp gran_backoff), so the give-up takes longer but stays bounded."""
    _, _, _, dec = decoder(gpu, cfg, 0, 42, 1)
    dec.set(gpu.OPT_USE_GRAPH, graph)
    want = oracle.Model(cfg, 0, seed=42).greedy(1, 0, 12)
    assert dec.greedy([1], [0], 4)[:, 0].tolist() == want[:4]
    assert dec.persistent()
    dec.set(gpu.OPT_PERSIST_FAULT, 1)
    assert dec.greedy([want[3]], [4], 8)[:, 0].tolist() == want[4:12]
    assert not dec.persistent()


def test_async_give_up_is_reported(gpu, oracle):
    """An asynchronous greedy call (sync=0, no tokens) returns before its launches run: a give-up
    inside it must be reported by the next call on the decoder (its tokens and K/V rows are
    invalid), not silently repaired by re-running only the later call."""
    _, _, _, dec = decoder(gpu, SMALL, 0, 42, 1)
    dec.set(gpu.OPT_USE_GRAPH, 1)
    want = oracle.Model(SMALL, 0, seed=42).greedy(1, 0, 12)
    assert dec.greedy([1], [0], 4)[:, 0].tolist() == want[:4]
    dec.set(gpu.OPT_PERSIST_FAULT, 1)
    dec.greedy([want[3]], [4], 4, want_tokens=False, sync=False)
    with pytest.raises(RuntimeError):
        dec.sync()
    assert not dec.persistent()
    # the caller re-runs the lost call itself; the multi-launch path then gives the oracle's tokens
    assert dec.greedy([want[3]], [4], 8)[:, 0].tolist() == want[4:12]


def test_cooperative_launch(gpu):
    """The persistent grid is dispatched as a cooperative launch (co-residency guaranteed by the
    runtime) on MI355X unless THALLAMA_PERSIST_COOP=0."""
    import os
    if os.environ.get("THALLAMA_PERSIST_COOP", "1") != "0":
        assert gpu.lib().thallama_persistent_cooperative() == 1


def test_plain_launch_switch(gpu):
    """THALLAMA_PERSIST_COOP=0 — the one launch switch left, for rocprofv3 runs (the profiler fails
    at exit after a cooperative launch, tools/prof_r04.sh) — gives a plain launch of the same grid
    and the same greedy tokens as the CPU oracle (a fresh process: the choice is made once)."""
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = (
        "import sys; sys.path.insert(0, %r); sys.path.insert(0, %r)\n"
        "from __graft_entry__ import _pkg; _pkg()\n"
        "from hip_llama_cpp_amd import thallama as tl\n"
        "import oracle as O\n"
        "tl.check(tl.lib().thallama_set_device(0))\n"
        "cfg = (256, 768, 2, 4, 2, 1024, 128)\n"
        "c = tl.Config.make(*cfg); m = tl.DeviceModel(c, 0, seed=5); st = tl.DeviceState(c, 1)\n"
        "d = tl.Decoder(m, st); assert d.persistent()\n"
        "got = d.greedy([1], [0], 24)[:, 0].tolist()\n"
        "want = O.Model(cfg, 0, seed=5).greedy(1, 0, 24)\n"
        "assert tl.lib().thallama_persistent_cooperative() == 0\n"
        "assert d.persistent() and got == want, (got, want)\n"
        "print('plain launch OK')\n") % (repo, os.path.join(repo, "oracle"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       env={**os.environ, "THALLAMA_PERSIST_COOP": "0"})
    assert r.returncode == 0 and "plain launch OK" in r.stdout, r.stderr[-3000:]


@pytest.mark.parametrize("cfg", [SMALL, HEAD128, RAGGED])
def test_forced_logits_every_step(gpu, oracle, cfg):
    _, _, _, dec = decoder(gpu, cfg, 0, 9, 1)
    ref = oracle.Model(cfg, 0, seed=9)
    toks = np.random.default_rng(3).integers(0, cfg[5], 24)
    for p, t in enumerate(toks):
        got = dec.forward([int(t)], [p])[0]
        want = ref.forward(int(t), p)
        assert_ref_close(got, want, 1e-4, f"logits pos {p}")
        assert int(np.argmax(got)) == oracle.lib().oracle_argmax(oracle.fp(want), cfg[5])


@pytest.mark.parametrize("cfg", [(256, 768, 2, 4, 4, 1024, 1024), (512, 1024, 2, 4, 2, 1024, 1024)])
@pytest.mark.parametrize("splits", [0, 1, 5, 16])
def test_long_context(gpu, oracle, cfg, splits):
    """Far past one attention chunk (16 keys in the persistent step), with 1..16 key-split
    units per head: the in-launch combine of the partials."""
    _, _, _, dec = decoder(gpu, cfg, 0, 21, 1)
    dec.set(gpu.OPT_ATTN_SPLITS, splits)
    assert dec.persistent()
    ref = oracle.Model(cfg, 0, seed=21)
    n = 300
    toks = np.random.default_rng(8).integers(0, cfg[5], n)
    for p, t in enumerate(toks):
        want = ref.forward(int(t), p)
        got = dec.forward([int(t)], [p], want_logits=(p % 29 == 0 or p == n - 1))
        if got is not None:
            assert_ref_close(got[0], want, 1e-4, f"pos {p}")


@pytest.mark.parametrize("cfg", [HEAD128, RAGGED])
def test_matches_multilaunch(gpu, cfg):
    """The persistent step and the multi-launch step agree (1e-4) step for step, and their
    greedy continuations are identical."""
    _, _, _, dp = decoder(gpu, cfg, 0, 77, 1)
    _, _, _, dm = decoder(gpu, cfg, 0, 77, 0)
    assert dp.persistent() and not dm.persistent()
    toks = np.random.default_rng(4).integers(0, cfg[5], 16)
    for p, t in enumerate(toks):
        assert_ref_close(dp.forward([int(t)], [p])[0], dm.forward([int(t)], [p])[0], 1e-4, f"pos {p}")
    n = 64
    start = len(toks)
    a = dp.greedy([1], [start], n)[:, 0].tolist()
    b = dm.greedy([1], [start], n)[:, 0].tolist()
    assert a == b


def test_repeated_launches_stay_consistent(gpu, oracle):
    """Many back-to-back graph replays (barrier counters re-armed by the memset node every
    launch, attention tickets re-armed in-kernel): the same tokens as the oracle."""
    cfg = SMALL
    _, _, _, dec = decoder(gpu, cfg, 0, 5, 1)
    dec.set(gpu.OPT_USE_GRAPH, 1)
    ref = oracle.Model(cfg, 0, seed=5)
    want = ref.greedy(7, 0, 120)
    got = dec.greedy([7], [0], 120)[:, 0].tolist()
    assert got == want
