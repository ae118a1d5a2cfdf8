"""Concurrent callers of one library, the way the reference drives it: one host thread per GPU,
each with its own handle/stream, calling thaDNN_s_forward_batch (src/llama.cpp:919-1024), and the
CLI's replicas sharing a device (app/run.cpp, THALLAMA_REPLICAS).

* A graph capture in one thread must survive whatever another thread's decoder does meanwhile
  (prefill, greedy steps, decoder creation): GPUTEST_r03 failed on a legacy-stream hipMemset of
  the lazily allocated prefill workspace issued while a sibling replica was capturing.
* The forward_batch decoder cache may drop a decoder (LRU past 8 keys, or new buffers) while
  another thread is still running it: that decoder must stay alive until the call returns.
"""
import ctypes as C
import threading

import numpy as np
import pytest

from helpers import SMALL, assert_ref_close

pytestmark = pytest.mark.gpu


def _run_threads(fns):
    errs = []
    start = threading.Barrier(len(fns))

    def wrap(f):
        def body():
            try:
                start.wait()
                f()
            except BaseException as e:  # noqa: BLE001 - reported below
                errs.append(e)
        return body

    ts = [threading.Thread(target=wrap(f)) for f in fns]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in ts), "a worker thread did not finish"
    if errs:
        raise errs[0]


def test_forward_batch_cache_two_threads_nine_plus_keys(gpu, oracle):
    """Two threads, each with its own handle (stream), cycle through batch sizes 1..5: 10 keys
    against a cache that starts at 8, so entries the other thread is using get evicted.  Every call's logits
    must still be the oracle's, and once the callers are done every dropped decoder is freed."""
    cfg = SMALL
    c = gpu.Config.make(*cfg)
    model = gpu.DeviceModel(c, 0, seed=91)
    V = cfg[5]
    want = oracle.Model(cfg, 0, seed=91).forward(1, 0)
    gpu.lib().thallama_forward_batch_cache_clear()
    states = {}
    handles = [gpu.new_handle(), gpu.new_handle()]
    for t in range(2):
        for B in range(1, 6):
            states[(t, B)] = gpu.DeviceState(c, B)

    def worker(t):
        def run():
            h = handles[t]
            for rnd in range(4):
                for B in (range(1, 6) if (rnd + t) % 2 == 0 else range(5, 0, -1)):
                    lg = np.zeros(B * V, np.float32)
                    rc = gpu.lib().thaDNN_s_forward_batch(h, h, h, B, C.byref(c), C.byref(model.w),
                                                          states[(t, B)].ptr, (C.c_int * B)(*([1] * B)),
                                                          (C.c_int * B)(*([0] * B)),
                                                          lg.ctypes.data_as(gpu.c_float_p))
                    assert rc == 0, f"thread {t} B={B} round {rnd}: status {rc}"
                    for b in range(B):
                        assert_ref_close(lg[b * V:(b + 1) * V], want, 1e-4, f"thread {t} B={B} b={b}")
        return run

    _run_threads([worker(0), worker(1)])
    n = gpu.lib().thallama_forward_batch_cache_size()
    cap = gpu.lib().thallama_forward_batch_cache_cap()
    assert 8 <= cap <= 10 and n == cap  # the cap grew toward the 10 keys in use
    assert gpu.lib().thallama_forward_batch_live() == n  # evicted decoders were freed by their last user
    gpu.lib().thallama_forward_batch_cache_clear()
    assert gpu.lib().thallama_forward_batch_cache_size() == 0
    assert gpu.lib().thallama_forward_batch_live() == 0


def test_capture_survives_sibling_prefill_and_create(gpu, oracle):
    """Three threads on one device: A replays captured greedy graphs (recaptured every round),
    B alternates prefill with captured greedy steps, C keeps creating and destroying decoders.
    Every token sequence must equal the oracle's."""
    cfg = SMALL
    c = gpu.Config.make(*cfg)
    model = gpu.DeviceModel(c, 0, seed=92)
    n = 24
    want_a = oracle.Model(cfg, 0, seed=92).greedy(1, 0, n)
    prompt = [1, 17, 300, 45, 900, 12, 7]
    ref_b = oracle.Model(cfg, 0, seed=92)
    for p, t in enumerate(prompt[:-1]):
        ref_b.forward(t, p)
    want_b = ref_b.greedy(prompt[-1], len(prompt) - 1, n)
    sa, sb = gpu.DeviceState(c, 1), gpu.DeviceState(c, 1)
    da, db = gpu.Decoder(model, sa), gpu.Decoder(model, sb)

    def run_a():
        for rnd in range(12):
            da.set(gpu.OPT_USE_GRAPH, 1)  # drops the graph: a fresh capture every round
            got = da.greedy([1], [0], n)[:, 0].tolist()
            assert got == want_a, f"A round {rnd}"

    def run_b():
        db.set(gpu.OPT_USE_GRAPH, 1)
        for rnd in range(12):
            assert db.prefill(0, prompt[:-1], 0) == 0, gpu.lib().thallama_last_error()
            got = db.greedy([prompt[-1]], [len(prompt) - 1], n)[:, 0].tolist()
            assert got == want_b, f"B round {rnd}"
            db.set(gpu.OPT_USE_GRAPH, 1)

    def run_c():
        for _ in range(12):
            st = gpu.DeviceState(c, 2)
            d = gpu.Decoder(model, st)
            d.set(gpu.OPT_USE_GRAPH, 1)
            d.greedy([1, 1], [0, 0], 2)
            d.close()
            st.free()

    _run_threads([run_a, run_b, run_c])
    da.close()
    db.close()
