"""GPU parity of the fused decode step against the CPU oracle (a bit-exact restatement of the
reference's src/seq.cpp forward, pinned in tests/test_oracle.py).

Bar (BASELINE.json north_star): greedy token ids identical, fp32 logits within 1e-4 under the
reference's abs-or-rel rule (scripts/test/thaDNN.test.cpp:224-229).
"""
import ctypes as C

import numpy as np
import pytest

from helpers import LLAMA2_7B, SMALL, SMALL_GQA, STORIES_110M, TINY, assert_ref_close

pytestmark = pytest.mark.gpu


def build(tl, oracle, cfg, shared, seed, batch=1):
    """Same synthetic weights on both sides: the GPU fills its arena with the device generator,
    the oracle with the host generator (bit-identical, checked in test_synth_bitexact)."""
    c = tl.Config.make(*cfg)
    model = tl.DeviceModel(c, shared, seed=seed)
    state = tl.DeviceState(c, batch)
    dec = tl.Decoder(model, state)
    ref = oracle.Model(cfg, shared, seed=seed)
    return c, model, state, dec, ref


def test_synth_bitexact(gpu, oracle):
    cfg = SMALL_GQA
    c = gpu.Config.make(*cfg)
    m = gpu.DeviceModel(c, 0, seed=1234)
    ref = oracle.Model(cfg, 0, seed=1234)
    np.testing.assert_array_equal(m.download(), ref.arena())


@pytest.mark.parametrize("cfg,shared", [(TINY, 0), (SMALL, 0), (SMALL_GQA, 0), (SMALL, 1)])
@pytest.mark.parametrize("graph", [0, 1])
def test_greedy_matches_oracle(gpu, oracle, cfg, shared, graph):
    c, model, state, dec, ref = build(gpu, oracle, cfg, shared, seed=42)
    dec.set(gpu.OPT_USE_GRAPH, graph)
    n = 40
    want = ref.greedy(1, 0, n)
    got = dec.greedy([1], [0], n)[:, 0].tolist()
    assert got == want
    # the device still holds the last step's logits (token want[-2] at pos n-1)
    fresh = oracle.Model(cfg, shared, seed=42)
    for p, t in enumerate([1] + want[:-1]):
        last = fresh.forward(t, p)
    assert_ref_close(dec.logits()[0], last, 1e-4, "last-step logits")


@pytest.mark.parametrize("cfg,shared", [(TINY, 0), (SMALL, 1), (SMALL_GQA, 0)])
def test_forced_logits_every_step(gpu, oracle, cfg, shared):
    """Teacher-forced random tokens: every step's logits within 1e-4 (also covers shared
    classifiers, whose greedy path degenerates to repeating the input token)."""
    c, model, state, dec, ref = build(gpu, oracle, cfg, shared, seed=9)
    toks = np.random.default_rng(3).integers(0, cfg[5], 24)
    for p, t in enumerate(toks):
        got = dec.forward([int(t)], [p])[0]
        want = ref.forward(int(t), p)
        assert_ref_close(got, want, 1e-4, f"logits pos {p}")
        assert int(np.argmax(got)) == oracle.lib().oracle_argmax(oracle.fp(want), cfg[5])


@pytest.mark.parametrize("cfg", [
    (256, 768, 2, 4, 4, 1024, 1024),    # head 64
    (512, 1024, 2, 4, 2, 1024, 1024),   # head 128, GQA
    (1024, 2048, 1, 4, 4, 512, 512),    # head 256
    (128, 512, 2, 4, 4, 512, 512),      # head 32: block kernel + combine launch
])
def test_long_context_attention(gpu, oracle, cfg):
    """Teacher-forced decode far past one attention chunk (32 keys): exercises the
    multi-chunk path whose last-arriving chunk combines the partials in-kernel."""
    c, model, state, dec, ref = build(gpu, oracle, cfg, 0, seed=21)
    n = min(cfg[6], 700)
    toks = np.random.default_rng(8).integers(0, cfg[5], n)
    for p, t in enumerate(toks):
        want = ref.forward(int(t), p)
        got = dec.forward([int(t)], [p], want_logits=(p % 37 == 0 or p == n - 1))
        if got is not None:
            assert_ref_close(got[0], want, 1e-4, f"pos {p}")


@pytest.mark.parametrize("B", [2, 3, 8])
def test_batch_independent_positions(gpu, oracle, B):
    """B sequences at different positions in one step == B independent CPU decodes."""
    cfg = SMALL_GQA
    c, model, state, dec, _ = build(gpu, oracle, cfg, 0, seed=5, batch=B)
    rng = np.random.default_rng(B)
    starts = rng.integers(0, 20, B)
    toks = rng.integers(0, cfg[5], (B, 64))
    refs = [oracle.Model(cfg, 0, seed=5) for _ in range(B)]
    for b in range(B):
        for p in range(int(starts[b])):
            refs[b].forward(int(toks[b, p]), p)
    # prefix: every lane runs (toks[b,p], p); for p >= starts[b] that row is rewritten by the real
    # step at p before any attention reads it, so the extra work is harmless
    for p in range(int(starts.max())):
        dec.forward([int(toks[b, p]) for b in range(B)], [p] * B, want_logits=False)
    for step in range(12):
        ps = [int(starts[b]) + step for b in range(B)]
        tk = [int(toks[b, ps[b]]) for b in range(B)]
        got = dec.forward(tk, ps)
        for b in range(B):
            assert_ref_close(got[b], refs[b].forward(tk[b], ps[b]), 1e-4, f"b={b} pos={ps[b]}")


def test_forward_batch_c_abi(gpu, oracle):
    """thaDNN_s_forward_batch, called exactly like the reference driver does
    (src/llama.cpp:1017): host token[]/pos[], logits into a host buffer."""
    cfg = SMALL
    c = gpu.Config.make(*cfg)
    model = gpu.DeviceModel(c, 0, seed=77)
    B = 2
    state = gpu.DeviceState(c, B)
    h = gpu.new_handle()
    ref = [oracle.Model(cfg, 0, seed=77) for _ in range(B)]
    logits = np.zeros(B * cfg[5], np.float32)
    toks = [[1, 5, 9, 200, 7], [3, 3, 100, 44, 2]]
    for p in range(5):
        tk = (C.c_int * B)(toks[0][p], toks[1][p])
        ps = (C.c_int * B)(p, p)
        rc = gpu.lib().thaDNN_s_forward_batch(h, h, h, B, C.byref(c), C.byref(model.w), state.ptr, tk, ps,
                                              logits.ctypes.data_as(gpu.c_float_p))
        assert rc == 0
        for b in range(B):
            assert_ref_close(logits[b * cfg[5]:(b + 1) * cfg[5]], ref[b].forward(toks[b][p], p), 1e-4, "abi")


def test_forward_batch_decoder_cache_bounded(gpu, oracle):
    """thaDNN_s_forward_batch keeps one decoder per (device, stream, batch, config): a caller that
    reallocates its RunState every call does not grow the cache, the decoder follows the new
    buffers, and distinct batch sizes stay within the cap of 8."""
    cfg = SMALL
    c = gpu.Config.make(*cfg)
    model = gpu.DeviceModel(c, 0, seed=78)
    h = gpu.new_handle()
    gpu.lib().thallama_forward_batch_cache_clear()
    logits = np.zeros(cfg[5], np.float32)
    toks = [1, 7, 300, 5, 9]
    prev = None
    for p in range(len(toks)):
        state = gpu.DeviceState(c, 1)  # a fresh state for every prefix: the cached decoder is replaced
        want = oracle.Model(cfg, 0, seed=78)
        for q in range(p + 1):
            rc = gpu.lib().thaDNN_s_forward_batch(h, h, h, 1, C.byref(c), C.byref(model.w), state.ptr,
                                                  (C.c_int * 1)(toks[q]), (C.c_int * 1)(q),
                                                  logits.ctypes.data_as(gpu.c_float_p))
            assert rc == 0
            lw = want.forward(toks[q], q)
        assert_ref_close(logits, lw, 1e-4, f"fresh state, prefix {p}")
        assert gpu.lib().thallama_forward_batch_cache_size() == 1
        if prev is not None:
            prev.free()
        prev = state
    gpu.lib().thallama_forward_batch_cache_clear()
    prev.free()
    keep = []
    for B in range(1, 12):
        st = gpu.DeviceState(c, B)
        keep.append(st)
        lg = np.zeros(B * cfg[5], np.float32)
        rc = gpu.lib().thaDNN_s_forward_batch(h, h, h, B, C.byref(c), C.byref(model.w), st.ptr,
                                              (C.c_int * B)(*([1] * B)), (C.c_int * B)(*([0] * B)),
                                              lg.ctypes.data_as(gpu.c_float_p))
        assert rc == 0
        assert gpu.lib().thallama_forward_batch_cache_size() == min(B, 8)
    gpu.lib().thallama_forward_batch_cache_clear()
    assert gpu.lib().thallama_forward_batch_cache_size() == 0


@pytest.mark.parametrize("token,pos", [(0, 0), (3, 4), (4, 4), (64, 64)])
def test_stories110m_reference_cases(gpu, oracle, token, pos):
    """The reference's own forward test points (scripts/test/thaDNN.test.cpp:541-549) on a
    stories110M-shaped synthetic model: fresh state, a single forward at (token, pos)."""
    oracle.set_threads(16)
    c, model, state, dec, ref = build(gpu, oracle, STORIES_110M, 1, seed=110)
    got = dec.forward([token], [pos])[0]
    want = ref.forward(token, pos)
    assert_ref_close(got, want, 1e-4, "110M logits")


def test_stories110m_greedy(gpu, oracle):
    oracle.set_threads(16)
    cfg = (768, 2048, 12, 12, 12, 32000, 1024)
    # unshared classifier so the greedy path does not collapse onto the input token
    c, model, state, dec, ref = build(gpu, oracle, cfg, 0, seed=111)
    dec.set(gpu.OPT_USE_GRAPH, 1)
    n = 48
    want = ref.greedy(1, 0, n)
    got = dec.greedy([1], [0], n)[:, 0].tolist()
    assert got == want


@pytest.mark.slow
def test_llama2_7b_shape(gpu, oracle):
    """Full llama2-7B shape (26.9 GB fp32): greedy tokens and logits vs the CPU oracle for a
    few steps (the oracle runs 16 threads; results are thread-count independent)."""
    oracle.set_threads(16)
    c, model, state, dec, ref = build(gpu, oracle, LLAMA2_7B, 0, seed=7)
    dec.set(gpu.OPT_USE_GRAPH, 1)
    n = 4
    toks = [1]
    for p in range(n):
        want = ref.forward(toks[-1], p)
        got = dec.forward([toks[-1]], [p])[0]
        assert_ref_close(got, want, 1e-4, f"7B logits pos {p}")
        assert int(np.argmax(got)) == int(np.argmax(want))
        toks.append(int(np.argmax(want)))


@pytest.mark.parametrize("B", [4, 8])
@pytest.mark.parametrize("abi", [0, 1])
def test_batched_norm_carry_mixed_paths(gpu, oracle, B, abi):
    """dim % 256 == 0 but hidden % 256 != 0 (stories42M-like 512 / 1376): W2 (K = hidden) takes the
    generic GEMV, which leaves no RMSNorm sums, while QKV / W1-W3 / the classifier (K = dim) take
    the matrix-core kernel — the sums must then not be carried across launches (round-2 review).
    Teacher-forced random tokens through the decoder and through thaDNN_s_forward_batch."""
    cfg = (512, 1376, 3, 8, 8, 1024, 64)
    c, model, state, dec, _ = build(gpu, oracle, cfg, 0, seed=42, batch=B)
    refs = [oracle.Model(cfg, 0, seed=42) for _ in range(B)]
    toks = np.random.default_rng(B + 10 * abi).integers(0, cfg[5], (B, 6))
    h = gpu.new_handle()
    logits = np.zeros(B * cfg[5], np.float32)
    for p in range(6):
        if abi:
            tk = (C.c_int * B)(*toks[:, p].tolist())
            ps = (C.c_int * B)(*([p] * B))
            assert gpu.lib().thaDNN_s_forward_batch(h, h, h, B, C.byref(c), C.byref(model.w), state.ptr, tk, ps,
                                                    logits.ctypes.data_as(gpu.c_float_p)) == 0
            got = logits.reshape(B, cfg[5])
        else:
            got = dec.forward(toks[:, p].tolist(), [p] * B)
        for b in range(B):
            assert_ref_close(got[b], refs[b].forward(int(toks[b, p]), p), 1e-4, f"B={B} b={b} pos={p}")


@pytest.mark.parametrize("B", [4, 7, 16, 17])
def test_batched_matrix_core_gemv(gpu, oracle, B):
    """B >= 4 sequences take the matrix-core GEMV (gemv_mfma.hpp; 17 = a group of 16 + a
    single-sequence group): every sequence's logits match its own CPU decode within 1e-4."""
    cfg = (512, 1536, 2, 8, 2, 2048, 64)   # head 64, GQA
    c, model, state, dec, _ = build(gpu, oracle, cfg, 0, seed=19, batch=B)
    rng = np.random.default_rng(B)
    toks = rng.integers(0, cfg[5], (B, 6))
    refs = [oracle.Model(cfg, 0, seed=19) for _ in range(B)]
    for p in range(6):
        got = dec.forward(toks[:, p].tolist(), [p] * B)
        for b in range(B):
            assert_ref_close(got[b], refs[b].forward(int(toks[b, p]), p), 1e-4, f"B={B} b={b} pos={p}")
