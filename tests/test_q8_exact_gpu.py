"""GPU parity of the multi-launch int8 step in runq's arithmetic order (hip_llama.cpp_amd/csrc/
q8_exact.hip: the batched decoders with group size 64, and batch 1 with the persistent step off)
against the CPU oracle's runq.c restatement (oracle_q8_forward, pinned to the reference runq.c in
tests/test_oracle.py).

Bar: BIT equality.  runq re-quantises the activations before every matmul, so nothing short of
its own summation order and roundings survives more than a few steps (tests/test_q8_gpu.py keeps
the Q8_TOL checks for the reordered kernels, THALLAMA_Q8_EXACT=0, and group sizes 32 / 128).
Shapes: head 64 and 128, GQA, a hidden size of 11 runs of 256 (W2's products span a
non-power-of-two group count), sequences at independent positions, contexts past the V window.
"""
import ctypes as C

import numpy as np
import pytest

from helpers import SMALL, SMALL_GQA

pytestmark = pytest.mark.gpu

HEAD128 = (512, 1536, 2, 4, 2, 1024, 512)     # head 128, GQA
RAGGED = (1024, 2816, 2, 8, 8, 1024, 320)      # head 128, hidden 2816 = 11 runs


def decoders(tl, cfg, seed, B, persistent=0):
    c = tl.Config.make(*cfg)
    m = tl.DeviceModel(c, 0, seed=seed)
    q = tl.DeviceModelQ8(c, 0, 64, from_model=m)
    state = tl.DeviceState(c, B)
    dec = tl.Decoder(q, state)
    dec.set(tl.OPT_PERSISTENT, persistent)
    assert not dec.persistent()
    return (m, q, state), dec


def refs_of(oracle, cfg, seed, B):
    out = []
    for _ in range(B):
        r = oracle.Model(cfg, 0, seed=seed)
        r.build_q8(64)
        out.append(r)
    return out


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@pytest.mark.parametrize("cfg", [SMALL, SMALL_GQA, HEAD128, RAGGED])
@pytest.mark.parametrize("B", [1, 2, 3, 5, 8])
def test_teacher_forced_logits_bitexact(gpu, oracle, cfg, B):
    """B sequences at their own positions (own random tokens): every logit of every step equals
    runq's bit for bit."""
    keep, dec = decoders(gpu, cfg, 17, B)
    refs = refs_of(oracle, cfg, 17, B)
    rng = np.random.default_rng(100 + B)
    starts = rng.integers(0, 12, B)
    toks = rng.integers(0, cfg[5], (B, 24))
    for b in range(B):
        for p in range(int(starts[b])):
            refs[b].q8_forward(int(toks[b, p]), p)
    for p in range(int(starts.max())):  # a sequence past its prefix rewrites its start row (same token)
        dec.forward([int(toks[b, min(p, int(starts[b]))]) for b in range(B)], [min(p, int(starts[b])) for b in range(B)],
                    want_logits=False)
    for step in range(6):
        ps = [int(starts[b]) + step for b in range(B)]
        tk = [int(toks[b, ps[b]]) for b in range(B)]
        got = dec.forward(tk, ps)
        for b in range(B):
            want = refs[b].q8_forward(tk[b], ps[b])
            np.testing.assert_array_equal(bits(got[b]), bits(want), err_msg=f"B={B} b={b} pos={ps[b]}")


@pytest.mark.parametrize("B,graph", [(4, 0), (8, 1)])
def test_greedy_long_context_bitexact(gpu, oracle, B, graph):
    """Greedy decode of B sequences from different start tokens past 300 positions (more than one
    V window of the output kernel): tokens equal runq's greedy decode of each, last logits bit-equal."""
    cfg = HEAD128
    keep, dec = decoders(gpu, cfg, 23, B)
    dec.set(gpu.OPT_USE_GRAPH, graph)
    starts = [1 + 97 * b for b in range(B)]
    n = 300
    got = dec.greedy(starts, [0] * B, n)
    lg = dec.logits()
    for b in range(B):
        r = oracle.Model(cfg, 0, seed=23)
        r.build_q8(64)
        want = r.q8_greedy(starts[b], 0, n)
        assert got[:, b].tolist() == want, f"sequence {b}"
        np.testing.assert_array_equal(bits(lg[b]), bits(r.logits()), err_msg=f"sequence {b} last logits")


def test_forward_batch_c_abi_bitexact(gpu, oracle):
    """thaDNN_q8_forward_batch (the reference-shaped entry point) on 3 sequences: bit-equal logits."""
    cfg = SMALL_GQA
    c = gpu.Config.make(*cfg)
    m = gpu.DeviceModel(c, 0, seed=3)
    q = gpu.DeviceModelQ8(c, 0, 64, from_model=m)
    B = 3
    state = gpu.DeviceState(c, B)
    h = gpu.new_handle()
    refs = refs_of(oracle, cfg, 3, B)
    logits = np.zeros(B * cfg[5], np.float32)
    toks = np.random.default_rng(1).integers(0, cfg[5], (B, 6))
    for p in range(6):
        tk = (C.c_int * B)(*toks[:, p].tolist())
        ps = (C.c_int * B)(*([p] * B))
        assert gpu.lib().thaDNN_q8_forward_batch(h, B, C.byref(c), C.byref(q.w), state.ptr, tk, ps,
                                                 logits.ctypes.data_as(gpu.c_float_p)) == 0
        for b in range(B):
            np.testing.assert_array_equal(bits(logits[b * cfg[5]:(b + 1) * cfg[5]]),
                                          bits(refs[b].q8_forward(int(toks[b, p]), p)), err_msg=f"b={b} pos={p}")


@pytest.mark.parametrize("cfg", [SMALL, HEAD128])
@pytest.mark.parametrize("B,persistent", [(1, 1), (1, 0), (3, 0)])
@pytest.mark.parametrize("n", [1, 7, 8, 21])
def test_int8_prefill_bitexact(gpu, oracle, cfg, B, persistent, n):
    """int8 prefill (thallama_decoder_prefill on an int8 decoder: chunks of up to 8 prompt tokens
    through the exact batched step) leaves slot b's K/V rows as stepping through the prompt would:
    the next forward's logits equal runq's after feeding the prompt one token at a time, bit for
    bit, and so do the following greedy steps."""
    c = gpu.Config.make(*cfg)
    m = gpu.DeviceModel(c, 0, seed=31)
    q = gpu.DeviceModelQ8(c, 0, 64, from_model=m)
    state = gpu.DeviceState(c, B)
    dec = gpu.Decoder(q, state)
    dec.set(gpu.OPT_PERSISTENT, persistent)
    rng = np.random.default_rng(7 + n + B)
    prompt = [int(t) for t in rng.integers(0, cfg[5], n + 1)]
    slot = B - 1
    pos0 = 3 if B > 1 else 0
    ref = oracle.Model(cfg, 0, seed=31)
    ref.build_q8(64)
    if pos0:  # slot's earlier rows, by decode steps on both sides
        pre = [int(t) for t in rng.integers(0, cfg[5], pos0)]
        for p, t in enumerate(pre):
            ref.q8_forward(t, p)
            tk = [0] * B
            ps = [0] * B
            tk[slot], ps[slot] = t, p
            dec.forward(tk, ps, want_logits=False)
    assert dec.prefill(slot, prompt[:n], pos0) == 0, gpu.lib().thallama_last_error()
    for p, t in enumerate(prompt[:n]):
        ref.q8_forward(t, pos0 + p)
    tok, pos = prompt[n], pos0 + n
    for step in range(4):
        want = ref.q8_forward(tok, pos)
        tk = [0] * B
        ps = [0] * B
        tk[slot], ps[slot] = tok, pos
        got = dec.forward(tk, ps)[slot]
        np.testing.assert_array_equal(bits(got), bits(want), err_msg=f"step {step} after a {n}-token prefill")
        tok, pos = int(np.argmax(want)), pos + 1
