"""The 4x4x1 matrix-core batched GEMV (csrc/gemv_mb.hpp) against the CPU oracle.

One launch through the library's dispatcher (thallama_gemv_check) on the shapes that exercise each
part of the kernel: whole rows in LDS (4 and 8 sequence slots), row groups cut between waves (the
slab + ticket combine), rows too long for the LDS (K slices: W2's K = 11008), a ragged last row
group, the fused RMSNorm, the offset store of thaBLAS_s_matmul_batch (src/thaBLAS.cpp:191-228,
C[Coff + has_pos*pos[b] + b*C_batch_size + i]) and the SwiGLU pair (src/seq.cpp:159-166).  The
acceptance rule is the reference's abs-or-rel 1e-4 (scripts/test/thaDNN.test.cpp:224-229); the
same launch without the kernel's scratch (the previous matrix-core path) is checked alongside.
"""
import ctypes as C

import numpy as np
import pytest

from helpers import assert_ref_close, rng

pytestmark = pytest.mark.gpu


def dev(tl, a):
    return tl.DevBuf.from_array(np.ascontiguousarray(a))


def run(gpu, mode, W0, W1, X, rms, y0, pos, has_pos, y_stride, use_mb):
    M, K = W0.shape
    nb = X.shape[0]
    dW0, dX, dy, dpos = dev(gpu, W0), dev(gpu, X), dev(gpu, y0), dev(gpu, pos)
    dW1 = dev(gpu, W1) if W1 is not None else None
    drms = dev(gpu, rms) if rms is not None else None
    took = C.c_int(-1)
    rc = gpu.lib().thallama_gemv_check(mode, M, K, nb, dW0.ptr, dW1.ptr if dW1 else None, dX.ptr,
                                       drms.ptr if drms else None, dy.ptr, dpos.ptr, has_pos, y_stride,
                                       use_mb, C.byref(took))
    assert rc == 0
    return dy.download(), took.value


def normed(oracle, X, rms):
    return X if rms is None else np.stack([oracle.rmsnorm(x, rms) for x in X])


@pytest.mark.parametrize("M,K,B,norm", [
    (4096, 4096, 8, False),   # whole rows, one row group per wave pair
    (4096, 4096, 3, True),    # 4-sequence slots, fused RMSNorm
    (2000, 4096, 8, True),    # cls-like with the norm, row groups cut between waves
    (1001, 768, 5, False),    # ragged last row group, short rows
    (4096, 11008, 8, False),  # K slices (W2 of llama2-7B): every row group combined from slabs
    (768, 6144, 4, False),    # two K slices at 4 slots
])
def test_store(gpu, oracle, M, K, B, norm):
    r = rng(M * 7 + K + B)
    W = (r.standard_normal((M, K)) * 0.02).astype(np.float32)
    X = r.standard_normal((B, K)).astype(np.float32)
    rms = r.uniform(0.5, 1.5, K).astype(np.float32) if norm else None
    y0 = np.full(B * M, 7.0, np.float32)
    want = np.stack([oracle.matmul(W, x) for x in normed(oracle, X, rms)])
    got, took = run(gpu, 0, W, None, X, rms, y0, np.zeros(B, np.int32), 0, M, 1)
    assert took == 1
    assert_ref_close(got.reshape(B, M), want, 1e-4, f"mb store {M}x{K} B={B}")
    old, took = run(gpu, 0, W, None, X, rms, y0, np.zeros(B, np.int32), 0, M, 0)
    assert took == 0
    assert_ref_close(old.reshape(B, M), want, 1e-4, f"matrix-core store {M}x{K} B={B}")


@pytest.mark.parametrize("B", [2, 6, 8])
def test_store_offsets(gpu, oracle, B):
    """KV-cache addressing of the reference batched GEMV: untouched elements stay untouched."""
    M, K, S = 256, 512, 16
    r = rng(B + 100)
    W = (r.standard_normal((M, K)) * 0.05).astype(np.float32)
    X = r.standard_normal((B, K)).astype(np.float32)
    pos = r.integers(0, S, B).astype(np.int32)
    Cbs = 2 * S * M
    y0 = np.full(B * Cbs, 7.0, np.float32)
    got, took = run(gpu, 0, W, None, X, None, y0, pos, M, Cbs, 1)
    assert took == 1
    want = y0.copy()
    for b in range(B):
        o = M * pos[b] + b * Cbs
        want[o:o + M] = oracle.matmul(W, X[b])
    assert_ref_close(got, want, 1e-4, "mb offsets")
    np.testing.assert_array_equal(got[want == 7.0], 7.0)


@pytest.mark.parametrize("M,K,B", [(4096, 4096, 8), (4096, 11008, 8), (4096, 11008, 4), (512, 1408, 7)])
def test_residual(gpu, oracle, M, K, B):
    r = rng(M + K * 3 + B)
    W = (r.standard_normal((M, K)) * 0.02).astype(np.float32)
    X = r.standard_normal((B, K)).astype(np.float32)
    y0 = r.standard_normal(B * M).astype(np.float32)
    got, took = run(gpu, 1, W, None, X, None, y0, np.zeros(B, np.int32), 0, M, 1)
    assert took == 1
    want = y0.reshape(B, M) + np.stack([oracle.matmul(W, x) for x in X])
    assert_ref_close(got.reshape(B, M), want, 1e-4, f"mb residual {M}x{K} B={B}")


@pytest.mark.parametrize("M,K,B,norm", [(11008, 4096, 8, True), (1378, 512, 5, False), (2048, 768, 2, True)])
def test_swiglu_pair(gpu, oracle, M, K, B, norm):
    r = rng(M + K + B + 5)
    W1 = (r.standard_normal((M, K)) * 0.02).astype(np.float32)
    W3 = (r.standard_normal((M, K)) * 0.02).astype(np.float32)
    X = r.standard_normal((B, K)).astype(np.float32)
    rms = r.uniform(0.5, 1.5, K).astype(np.float32) if norm else None
    got, took = run(gpu, 2, W1, W3, X, rms, np.zeros(B * M, np.float32), np.zeros(B, np.int32), 0, M, 1)
    assert took == 1
    xs = normed(oracle, X, rms)
    want = np.stack([oracle.swiglu(oracle.matmul(W1, x), oracle.matmul(W3, x)) for x in xs])
    assert_ref_close(got.reshape(B, M), want, 1e-4, f"mb swiglu {M}x{K} B={B}")
