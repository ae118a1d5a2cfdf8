"""Batched prefill (hip_llama.cpp_amd/csrc/prefill.hip, thallama_decoder_prefill) against the
CPU oracle: prefilling n prompt tokens and then decoding must give the logits the oracle gets
by feeding the same tokens one decode step at a time (src/llama.cpp:1029-1031), within the
reference's 1e-4 abs-or-rel rule, and the same K/V cache rows."""
import numpy as np
import pytest

from helpers import assert_ref_close

pytestmark = pytest.mark.gpu

CFGS = [
    (256, 768, 2, 4, 4, 1000, 512),     # head 64
    (512, 1536, 2, 4, 2, 1000, 512),    # head 128, GQA
    (1024, 2816, 2, 4, 4, 1000, 512),   # head 256; hidden not a multiple of the 128-row tile
]


def build(tl, oracle, cfg, seed, batch=1):
    c = tl.Config.make(*cfg)
    model = tl.DeviceModel(c, 0, seed=seed)
    state = tl.DeviceState(c, batch)
    dec = tl.Decoder(model, state)
    ref = oracle.Model(cfg, 0, seed=seed)
    return model, state, dec, ref


@pytest.mark.parametrize("cfg", CFGS)
@pytest.mark.parametrize("n", [1, 7, 20, 64, 81, 130])
def test_prefill_then_decode_matches_oracle(gpu, oracle, cfg, n):
    model, state, dec, ref = build(gpu, oracle, cfg, 31)
    toks = np.random.default_rng(n).integers(0, cfg[5], n + 1).tolist()
    assert dec.prefill(0, toks[:n], 0) == 0
    got = dec.forward([toks[n]], [n])[0]
    for p, t in enumerate(toks[:n]):
        ref.forward(t, p)
    want = ref.forward(toks[n], n)
    assert_ref_close(got, want, 1e-4, f"logits after prefill of {n}")


def test_prefill_continues_a_sequence(gpu, oracle):
    """Decode some steps, prefill a second chunk at pos0 > 0, decode again."""
    cfg = CFGS[1]
    model, state, dec, ref = build(gpu, oracle, cfg, 8)
    toks = np.random.default_rng(2).integers(0, cfg[5], 60).tolist()
    for p in range(10):
        dec.forward([toks[p]], [p], want_logits=False)
        ref.forward(toks[p], p)
    assert dec.prefill(0, toks[10:50], 10) == 0
    for p in range(10, 50):
        ref.forward(toks[p], p)
    for p in range(50, 60):
        assert_ref_close(dec.forward([toks[p]], [p])[0], ref.forward(toks[p], p), 1e-4, f"pos {p}")


def test_prefill_touches_only_its_slot(gpu, oracle):
    cfg = CFGS[0]
    model, state, dec, ref = build(gpu, oracle, cfg, 5, batch=3)
    toks = np.random.default_rng(4).integers(0, cfg[5], 40).tolist()
    before = state.download_kcache() if hasattr(state, "download_kcache") else None
    assert dec.prefill(1, toks[:33], 0) == 0
    # slot 1 now continues exactly like the oracle; slots 0 and 2 start fresh at position 0
    refs = [oracle.Model(cfg, 0, seed=5) for _ in range(3)]
    for p, t in enumerate(toks[:33]):
        refs[1].forward(t, p)
    got = dec.forward([toks[0], toks[33], toks[1]], [0, 33, 0])
    assert_ref_close(got[1], refs[1].forward(toks[33], 33), 1e-4, "slot 1")
    assert_ref_close(got[0], refs[0].forward(toks[0], 0), 1e-4, "slot 0")
    assert_ref_close(got[2], refs[2].forward(toks[1], 0), 1e-4, "slot 2")
    del before


def test_prefill_rejections(gpu):
    c = gpu.Config.make(64, 172, 2, 4, 2, 512, 64)  # head 16: not supported -> caller falls back
    dec = gpu.Decoder(gpu.DeviceModel(c, 0, seed=1), gpu.DeviceState(c, 1))
    assert dec.prefill(0, [1, 2, 3], 0) != 0
    c = gpu.Config.make(*CFGS[0])
    dec = gpu.Decoder(gpu.DeviceModel(c, 0, seed=1), gpu.DeviceState(c, 1))
    assert dec.prefill(0, [1] * 10, CFGS[0][6] - 5) != 0   # past seq_len
    assert dec.prefill(0, [CFGS[0][5]], 0) != 0            # token out of range
    assert dec.prefill(1, [1], 0) != 0                     # no such slot
