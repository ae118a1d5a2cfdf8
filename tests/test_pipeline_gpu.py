"""the reference's pipeline, layer-swap and 70B layer-streaming drivers
(src/thaDNN.cpp:83-427) and their staging (src/models.cpp:181-758), called the way its
src/llama.cpp test_pipeline_parallelism / test_70B call them (:1085-1485), against the CPU oracle
(the bit-exact src/seq.cpp restatement, tests/test_oracle.py).

Bar: north_star's fp32 1e-4 under the reference's abs-or-rel rule (scripts/test/thaDNN.test.cpp:
224-229), every step of a teacher-forced decode, two sequences at their own positions.  The stages
run on the device of each handle's stream; this box has one GPU, so every stage shares it (the
hand-off is then a same-device copy; the peer copy over xGMI needs two devices).
"""
import ctypes as C

import numpy as np
import pytest

from helpers import assert_ref_close

pytestmark = pytest.mark.gpu

CFG = (256, 768, 4, 4, 2, 1024, 96)   # 4 layers (1, 2 or 4 stages), GQA, unshared classifier


def host_transformer(tl, cfg, arena, shared):
    """A host Transformer over a v0 payload in host memory (the reference's mmapped model)."""
    t = tl.Transformer()
    t.config = tl.Config.make(*cfg)
    tl.lib().thallama_map_weights(C.byref(t.weights), C.byref(t.config), arena.ctypes.data_as(tl.c_float_p), shared)
    t.fd = -1
    return t


def handles(tl, n):
    arr = (tl.Handle * n)()
    for g in range(n):
        arr[g] = tl.new_handle()
    return arr


@pytest.mark.parametrize("n_stages", [1, 2, 4])
@pytest.mark.parametrize("variant", ["multiple", "layer_swap", "pipe_line"])
def test_pipeline_matches_oracle(gpu, oracle, n_stages, variant):
    tl = gpu
    cfg, shared, seed, B, steps = CFG, 0, 41, 2, 10
    base = oracle.Model(cfg, shared, seed=seed)
    arena = base.arena().copy()
    t_h = host_transformer(tl, cfg, arena, shared)
    c = tl.Config.make(*cfg)
    pipe = cfg[2] // n_stages
    hs = handles(tl, n_stages)
    L = tl.lib()
    wps = (C.POINTER(tl.TransformerWeights) * n_stages)()
    sps = (C.POINTER(tl.RunState) * n_stages)()
    hsp = (C.POINTER(tl.RunState) * n_stages)()
    tps = (C.POINTER(tl.Transformer) * n_stages)()
    for g in range(n_stages):  # (each out-parameter is the reference's `T* &`: a pointer to the pointer)
        if variant == "pipe_line":
            tp = C.POINTER(tl.Transformer)()
            L.copy_transformer_pipeline_to_device_batch(hs[g], C.byref(t_h), C.byref(tp), pipe, g, B)
            tps[g] = tp
            continue
        wp, sp, hp = C.POINTER(tl.TransformerWeights)(), C.POINTER(tl.RunState)(), C.POINTER(tl.RunState)()
        L.copy_transformer_weight_pipeline_to_device_batch(C.byref(t_h), C.byref(wp), pipe, g, B)
        if variant == "layer_swap":
            L.alloc_swap_run_state_on_host_batch(hs[g], C.byref(t_h), C.byref(hp), pipe, g, B, cfg[6] // 2)
            L.alloc_swap_run_state_to_device_batch(hs[g], C.byref(t_h), C.byref(sp), pipe, g, B, cfg[6] // 2)
        else:
            L.alloc_run_state_to_device_batch(hs[g], C.byref(t_h), C.byref(sp), pipe, g, B)
        wps[g], sps[g], hsp[g] = wp, sp, hp
    rng = np.random.default_rng(7 + n_stages)
    refs = [oracle.Model(cfg, shared, seed=seed) for _ in range(B)]
    toks = rng.integers(0, cfg[5], (steps + 5, B))
    logits = np.zeros(B * cfg[5], np.float32)
    pos = [0, 0]
    for step in range(steps + 5):
        # slot 1 runs 5 positions ahead of slot 0 after the first 5 steps (independent positions)
        active = [True, True] if step >= 5 else [False, True]
        tk = [int(toks[step, b]) if active[b] else -1 for b in range(B)]  # -1: an idle slot
        ps = [pos[b] if active[b] else -1 for b in range(B)]
        tka, psa = (C.c_int * B)(*tk), (C.c_int * B)(*ps)
        lp = logits.ctypes.data_as(tl.c_float_p)
        if variant == "multiple":
            rc = L.thaDNN_s_forward_batch_multiple_pipe_line(hs, 0, 1, n_stages, B, C.byref(c), wps, sps, tka, psa, lp,
                                                             None, None, None)
        elif variant == "layer_swap":
            rc = L.thaDNN_s_forward_batch_multiple_pipe_line_layer_swap(hs, 0, 1, n_stages, B, cfg[6] // 2, C.byref(c),
                                                                        wps, sps, hsp, tka, psa, lp, None)
        else:
            rc = L.thaDNN_s_forward_batch_pipe_line(hs, n_stages, B, tps, tka, psa, lp)
        assert rc == 0, (variant, step, tl.lib().thallama_last_error())
        for b in range(B):
            if not active[b]:
                continue
            want = refs[b].forward(tk[b], ps[b])
            assert_ref_close(logits[b * cfg[5]:(b + 1) * cfg[5]], want, 1e-4, f"{variant} {n_stages} stages b={b} "
                                                                                f"pos={ps[b]}")
            pos[b] += 1
    tl.lib().thallama_forward_batch_cache_clear()
    for g in range(n_stages):
        if variant != "pipe_line":
            L.free_weight_device(wps[g])
            L.free_state_device(sps[g])


@pytest.mark.parametrize("shared", [0, 1])
def test_forward_70B_layer_streaming_matches_oracle(gpu, oracle, shared):
    """thaDNN_s_forward_70B as test_70B drives it (src/llama.cpp:1105-1209): host layers from
    copy_transformer_to_host_70B, device staging from alloc_weight_to_device_70B /
    alloc_state_to_device_70B, batch 1; greedy tokens and every step's logits vs the oracle."""
    tl = gpu
    cfg = CFG
    base = oracle.Model(cfg, shared, seed=43)
    arena = base.arena().copy()
    t_h = host_transformer(tl, cfg, arena, shared)
    c = tl.Config.make(*cfg)
    L = tl.lib()
    h_w = (C.POINTER(tl.TransformerWeights) * cfg[2])()
    h_s = (C.POINTER(tl.RunState) * 1)()
    L.copy_transformer_to_host_70B(C.byref(t_h), h_w, h_s, 1)
    d_w = C.POINTER(tl.TransformerWeights)()
    d_s = C.POINTER(tl.RunState)()
    L.alloc_weight_to_device_70B(C.byref(t_h), C.byref(d_w))
    L.alloc_state_to_device_70B(C.byref(t_h), C.byref(d_s))
    h = tl.new_handle()
    ref = oracle.Model(cfg, shared, seed=43)
    logits = np.zeros(cfg[5], np.float32)
    token = 1
    for p in range(24):
        rc = L.thaDNN_s_forward_70B(h, 1, C.byref(c), h_w, h_s[0], d_w, d_s, (C.c_int * 1)(token), (C.c_int * 1)(p),
                                    logits.ctypes.data_as(tl.c_float_p))
        assert rc == 0, tl.lib().thallama_last_error()
        want = ref.forward(token, p)
        assert_ref_close(logits, want, 1e-4, f"70B streaming pos={p}")
        assert int(np.argmax(logits)) == int(np.argmax(want))
        token = int(np.argmax(want))
    tl.lib().thallama_forward_batch_cache_clear()
    L.free_weight_device(d_w)
    tl.lib().free_state_device(d_s)


def test_pipeline_four_threads_cache_follows_working_set(gpu, oracle):
    """The reference's test_pipeline_parallelism drives the pipeline from 4 host threads, each with
    its own handle per device (src/llama.cpp:1298): 4 threads x 4 stages = 16 stage decoders, twice
    the decoder cache's starting size.  The cache must grow to that working set (thrashing would
    re-create a decoder — workspaces, RoPE table — on every call): after the first rounds the
    number of live decoders stays flat, and every thread's logits stay the oracle's."""
    import threading
    tl = gpu
    cfg, shared, seed, B, n_stages, n_threads = CFG, 0, 45, 1, 4, 4
    base = oracle.Model(cfg, shared, seed=seed)
    arena = base.arena().copy()
    t_h = host_transformer(tl, cfg, arena, shared)
    c = tl.Config.make(*cfg)
    L = tl.lib()
    L.thallama_forward_batch_cache_clear()
    pipe = cfg[2] // n_stages
    wps = (C.POINTER(tl.TransformerWeights) * n_stages)()
    for g in range(n_stages):
        wp = C.POINTER(tl.TransformerWeights)()
        L.copy_transformer_weight_pipeline_to_device_batch(C.byref(t_h), C.byref(wp), pipe, g, B)
        wps[g] = wp
    per = []
    for t in range(n_threads):
        hs = handles(tl, n_stages)
        sps = (C.POINTER(tl.RunState) * n_stages)()
        for g in range(n_stages):
            sp = C.POINTER(tl.RunState)()
            L.alloc_run_state_to_device_batch(hs[g], C.byref(t_h), C.byref(sp), pipe, g, B)
            sps[g] = sp
        per.append((hs, sps))
    steps = 12
    toks = [[(7 * t + 3 * p) % cfg[5] for p in range(steps)] for t in range(n_threads)]
    got = [[None] * steps for _ in range(n_threads)]
    live = [[0] * steps for _ in range(n_threads)]
    errs = []
    start = threading.Barrier(n_threads)

    def worker(t):
        try:
            hs, sps = per[t]
            start.wait()
            lg = np.zeros(cfg[5], np.float32)
            for p in range(steps):
                rc = L.thaDNN_s_forward_batch_multiple_pipe_line(hs, 0, 1, n_stages, B, C.byref(c), wps, sps,
                                                                 (C.c_int * 1)(toks[t][p]), (C.c_int * 1)(p),
                                                                 lg.ctypes.data_as(tl.c_float_p), None, None, None)
                assert rc == 0, (t, p, L.thallama_last_error())
                got[t][p] = lg.copy()
                live[t][p] = L.thallama_forward_batch_live()
        except BaseException as e:  # noqa: BLE001 - reported below
            errs.append(e)

    ts = [threading.Thread(target=worker, args=(t,)) for t in range(n_threads)]
    for th in ts:
        th.start()
    for th in ts:
        th.join(timeout=300)
    assert not any(th.is_alive() for th in ts), "a worker thread did not finish"
    if errs:
        raise errs[0]
    cap = L.thallama_forward_batch_cache_cap()
    assert cap >= n_threads * n_stages, cap
    assert L.thallama_forward_batch_cache_size() == n_threads * n_stages
    tail = {live[t][p] for t in range(n_threads) for p in range(steps // 2, steps)}
    assert tail == {n_threads * n_stages}, (tail, live)
    for t in range(n_threads):
        ref = oracle.Model(cfg, shared, seed=seed)
        for p in range(steps):
            assert_ref_close(got[t][p], ref.forward(toks[t][p], p), 1e-4, f"thread {t} pos {p}")
    L.thallama_forward_batch_cache_clear()
    for t in range(n_threads):
        for g in range(n_stages):
            L.free_state_device(per[t][1][g])
    for g in range(n_stages):
        L.free_weight_device(wps[g])
