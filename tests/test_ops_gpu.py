"""GPU parity of every thaBLAS / thaDNN operator against the CPU oracle.

Cases and tolerances follow the reference's own tests
(scripts/test/thaBLAS.test.cpp:148-160, scripts/test/thaDNN.test.cpp:490-529):
same sizes, same abs-or-rel acceptance rule.  All calls go through the C ABI of
libthallama.so (ctypes); nothing here runs without the HIP library.
"""
import ctypes as C

import numpy as np
import pytest

from helpers import assert_ref_close, rng

pytestmark = pytest.mark.gpu


def dev(tl, a):
    return tl.DevBuf.from_array(np.ascontiguousarray(a))


# ------------------------------------------------------------------ RMSNorm
@pytest.mark.parametrize("size", [1, 111, 11111, 256 * 256])
def test_rmsnorm(gpu, handle, oracle, size):
    r = rng(size)
    x = r.uniform(-0.5, 0.5, size).astype(np.float32)
    w = r.uniform(-0.5, 0.5, size).astype(np.float32)
    dx, dw, do = dev(gpu, x), dev(gpu, w), gpu.DevBuf(size * 4)
    assert gpu.lib().thaDNN_s_rmsnorm_v2_batch(C.byref(handle), 1, do.fptr(), dx.fptr(), dw.fptr(), size, size) == 0
    gpu.sync()
    assert_ref_close(do.download(), oracle.rmsnorm(x, w), 1e-5, "rmsnorm")


@pytest.mark.parametrize("B,size,dim", [(4, 768, 768), (3, 4096, 4100), (2, 333, 400)])
def test_rmsnorm_batch(gpu, handle, oracle, B, size, dim):
    r = rng(B * size)
    x = r.standard_normal((B, dim)).astype(np.float32)
    w = r.standard_normal(size).astype(np.float32)
    dx, dw, do = dev(gpu, x), dev(gpu, w), gpu.DevBuf(B * dim * 4)
    assert gpu.lib().thaDNN_s_rmsnorm_v2_batch(C.byref(handle), B, do.fptr(), dx.fptr(), dw.fptr(), size, dim) == 0
    gpu.sync()
    got = do.download().reshape(B, dim)
    for b in range(B):
        assert_ref_close(got[b, :size], oracle.rmsnorm(x[b, :size], w), 1e-5, f"rmsnorm b={b}")


def test_rmsnorm_in_place(gpu, handle, oracle):
    # the final norm of the reference runs in place: rmsnorm(x, x, w)  (src/thaDNN.cpp:75)
    x = rng(5).standard_normal(768).astype(np.float32)
    w = rng(6).standard_normal(768).astype(np.float32)
    dx, dw = dev(gpu, x), dev(gpu, w)
    assert gpu.lib().thaDNN_s_rmsnorm_v2_batch(C.byref(handle), 1, dx.fptr(), dx.fptr(), dw.fptr(), 768, 768) == 0
    gpu.sync()
    assert_ref_close(dx.download(), oracle.rmsnorm(x, w), 1e-5, "rmsnorm in place")


# ------------------------------------------------------------------ softmax
@pytest.mark.parametrize("size", [1, 111, 11111, 32000])
def test_softmax(gpu, handle, oracle, size):
    x = rng(size).uniform(-0.5, 0.5, size).astype(np.float32) * 10
    dx = dev(gpu, x)
    assert gpu.lib().thaDNN_s_softmax_v2(C.byref(handle), dx.fptr(), size) == 0
    gpu.sync()
    assert_ref_close(dx.download(), oracle.softmax(x), 1e-3, "softmax")


# ------------------------------------------------------------------ RoPE
@pytest.mark.parametrize("dim,hs,kv_dim,pos", [(256, 16, 64, 0), (2, 1, 2, 1), (16384, 256, 11111, 512),
                                               (2222, 333, 2111, 111), (4096, 128, 4096, 2047)])
def test_rope(gpu, handle, oracle, dim, hs, kv_dim, pos):
    r = rng(dim + pos)
    q = r.uniform(-0.5, 0.5, dim).astype(np.float32)
    k = r.uniform(-0.5, 0.5, kv_dim + 1).astype(np.float32)  # odd kv_dim rotates one past the end, like the reference
    dq, dk = dev(gpu, q), dev(gpu, k)
    assert gpu.lib().thaDNN_s_rope(C.byref(handle), dim, hs, kv_dim, pos, dq.fptr(), dk.fptr()) == 0
    gpu.sync()
    q_ref, k_ref = oracle.rope(q, k, dim, hs, kv_dim, pos)
    assert_ref_close(dq.download(), q_ref, 1e-4, "rope q")
    assert_ref_close(dk.download(), k_ref, 1e-4, "rope k")


# ------------------------------------------------------------------ SwiGLU
@pytest.mark.parametrize("n", [256, 1, 1000000, 33333])
def test_swiglu(gpu, handle, oracle, n):
    r = rng(n)
    a = r.uniform(-4, 4, n).astype(np.float32)
    b = r.uniform(-4, 4, n).astype(np.float32)
    da, db = dev(gpu, a), dev(gpu, b)
    assert gpu.lib().thaDNN_s_swiglu(C.byref(handle), da.fptr(), db.fptr(), n) == 0
    gpu.sync()
    assert_ref_close(da.download(), oracle.swiglu(a, b), 1e-4, "swiglu")


# ------------------------------------------------------------------ vector ops
@pytest.mark.parametrize("n", [1, 63, 4096, 11008, 100003])
def test_vecaddvec(gpu, handle, n):
    r = rng(n)
    a = r.standard_normal(n).astype(np.float32)
    b = r.standard_normal(n).astype(np.float32)
    da, db = dev(gpu, a), dev(gpu, b)
    assert gpu.lib().thaBLAS_s_vecaddvec(C.byref(handle), da.fptr(), db.fptr(), n) == 0
    gpu.sync()
    np.testing.assert_array_equal(da.download(), a + b)  # one IEEE add per element: exact


@pytest.mark.parametrize("n", [10, 1000, 100000])
def test_svds(gpu, handle, n):
    a = rng(n).standard_normal(n).astype(np.float32)
    da, db = dev(gpu, a), gpu.DevBuf(n * 4)
    assert gpu.lib().thablas_Svds(handle, n, da.fptr(), db.fptr(), C.c_float(3.7)) == 0
    gpu.sync()
    np.testing.assert_array_equal(db.download(), a / np.float32(3.7))
    assert gpu.lib().thablas_Svds(handle, n, da.fptr(), db.fptr(), C.c_float(0.0)) != 0  # rejected like the reference


# ------------------------------------------------------------------ GEMV / GEMM
@pytest.mark.parametrize("M,K", [(4096, 4096), (11008, 4096), (4096, 11008), (32000, 768), (768, 2048),
                                 (100, 100), (3, 3), (173, 260), (1, 256)])
def test_matmulvec(gpu, handle, oracle, M, K):
    r = rng(M * 7 + K)
    W = (r.standard_normal((M, K)) * 0.02).astype(np.float32)
    x = r.standard_normal(K).astype(np.float32)
    dW, dx, dy = dev(gpu, W), dev(gpu, x), gpu.DevBuf(M * 4)
    assert gpu.lib().thaBLAS_s_matmulvec(handle, dy.fptr(), dx.fptr(), dW.fptr(), K, M) == 0
    gpu.sync()
    assert_ref_close(dy.download(), oracle.matmul(W, x), 1e-4, f"gemv {M}x{K}")


@pytest.mark.parametrize("B", [1, 2, 3, 5, 8, 13, 16, 17])
def test_matmul_batch_offsets(gpu, handle, oracle, B):
    """thaBLAS_s_matmul_batch with the KV-cache addressing of src/thaDNN.cpp:45-46:
    C[Coff + has_pos*pos[b] + b*C_batch_size + i]."""
    M, K, S = 256, 512, 16
    r = rng(B)
    W = (r.standard_normal((M, K)) * 0.05).astype(np.float32)
    X = r.standard_normal((B, K)).astype(np.float32)
    pos = r.integers(0, S, B).astype(np.int32)
    Cbs = 2 * S * M
    Coff = S * M  # "layer 1"
    C0 = np.full(B * Cbs, 7.0, np.float32)
    dW, dX, dC, dpos = dev(gpu, W), dev(gpu, X), dev(gpu, C0), dev(gpu, pos)
    assert gpu.lib().thaBLAS_s_matmul_batch(C.byref(handle), B, dC.fptr(), dX.fptr(), dW.fptr(), K, M, Coff, M,
                                            dpos.iptr(), Cbs, K) == 0
    gpu.sync()
    got = dC.download()
    want = C0.copy()
    for b in range(B):
        o = Coff + M * pos[b] + b * Cbs
        want[o:o + M] = oracle.matmul(W, X[b])
    assert_ref_close(got, want, 1e-4, "matmul_batch")
    untouched = want == 7.0
    np.testing.assert_array_equal(got[untouched], 7.0)


@pytest.mark.parametrize("B", [4, 5, 8])
@pytest.mark.parametrize("M,K", [(4096, 4096), (4096, 11008), (12288, 2048)])
def test_matmul_batch_register_resident(gpu, handle, oracle, M, K, B):
    """Batched GEMV at 7B row counts: B = 4 takes the register-resident kernel (gemv_rr.hpp; K =
    11008 is three passes of 16 / 16 / 11 chunks, the last pass leaves waves idle), B = 5 and 8 the
    matrix-core kernel; 1e-4 vs the oracle."""
    r = rng(M + K + B)
    W = (r.standard_normal((M, K)) * 0.02).astype(np.float32)
    X = r.standard_normal((B, K)).astype(np.float32)
    pos = np.zeros(B, np.int32)
    C0 = np.full(B * M, 7.0, np.float32)
    dW, dX, dC, dpos = dev(gpu, W), dev(gpu, X), dev(gpu, C0), dev(gpu, pos)
    assert gpu.lib().thaBLAS_s_matmul_batch(C.byref(handle), B, dC.fptr(), dX.fptr(), dW.fptr(), K, M, 0, 0,
                                            dpos.iptr(), M, K) == 0
    gpu.sync()
    got = dC.download().reshape(B, M)
    for b in range(B):
        assert_ref_close(got[b], oracle.matmul(W, X[b]), 1e-4, f"rr gemv {M}x{K} b={b}")


@pytest.mark.parametrize("m,n,k", [(3, 3, 3), (100, 100, 100), (1000, 1000, 1000), (65, 130, 33)])
def test_sgemm(gpu, handle, m, n, k):
    r = rng(m + n + k)
    A = r.uniform(-0.5, 0.5, (m, k)).astype(np.float32)
    B = r.uniform(-0.5, 0.5, (k, n)).astype(np.float32)
    dA, dB, dC = dev(gpu, A), dev(gpu, B), gpu.DevBuf(m * n * 4)
    assert gpu.lib().thaBLAS_s_matmul(handle, m, n, k, dA.fptr(), dB.fptr(), dC.fptr()) == 0
    gpu.sync()
    want = (A.astype(np.float64) @ B.astype(np.float64))
    assert_ref_close(dC.download().reshape(m, n), want, 1e-3, "sgemm")  # thaBLAS.test.cpp eps 1e-3


@pytest.mark.parametrize("M,N,K", [(256, 4, 512), (512, 16, 768), (48, 40, 100), (4096, 32, 4096)])
def test_matmul_reduction_and_mfma(gpu, handle, M, N, K):
    r = rng(M * N)
    A = r.uniform(-0.5, 0.5, (M, K)).astype(np.float32)
    B = r.uniform(-0.5, 0.5, (N, K)).astype(np.float32)
    want = (B.astype(np.float64) @ A.astype(np.float64).T)  # [N][M]
    dA, dB = dev(gpu, A), dev(gpu, B)
    for fn in ("thaBLAS_s_matmul_reduction", "thaBLAS_s_sgemm_Mx16xK", "thaBLAS_s_matmul_ifdef"):
        dD = gpu.DevBuf(N * M * 4)
        assert getattr(gpu.lib(), fn)(C.byref(handle), dA.fptr(), dB.fptr(), dD.fptr(), M, N, K) == 0
        gpu.sync()
        assert_ref_close(dD.download().reshape(N, M), want, 1e-3, fn)


# ------------------------------------------------------------------ attention (3-kernel API)
@pytest.mark.parametrize("B,H,kvh,hs,S,L", [(1, 4, 4, 64, 64, 2), (3, 8, 2, 128, 96, 3), (2, 6, 3, 48, 40, 1)])
def test_mha_v1(gpu, handle, oracle, B, H, kvh, hs, S, L):
    r = rng(B * H * hs)
    dim, kv_dim, kv_mul = H * hs, kvh * hs, H // kvh
    layer = L - 1
    loff = layer * S * kv_dim
    pos = r.integers(0, S, B).astype(np.int32)
    q = r.standard_normal((B, dim)).astype(np.float32)
    kc = r.standard_normal((B, L, S, kv_dim)).astype(np.float32)
    vc = r.standard_normal((B, L, S, kv_dim)).astype(np.float32)
    dq, dk, dv = dev(gpu, q), dev(gpu, kc), dev(gpu, vc)
    datt, dxb, dpos = dev(gpu, np.zeros((B, H, S), np.float32)), gpu.DevBuf(B * dim * 4), dev(gpu, pos)
    hpos = (C.c_int * B)(*pos.tolist())
    lib = gpu.lib()
    assert lib.thaDNN_s_multiheads_1_v1_batch(C.byref(handle), B, hpos, dpos.iptr(), H, L, dq.fptr(), datt.fptr(),
                                              dk.fptr(), hs, S, loff, kv_dim, dim, kv_mul) == 0
    assert lib.thaDNN_s_multiheads_2_v1_batch(C.byref(handle), B, datt.fptr(), dpos.iptr(), S, H) == 0
    assert lib.thaDNN_s_multiheads_3_v1_batch(C.byref(handle), B, dpos.iptr(), H, dxb.fptr(), datt.fptr(), dv.fptr(),
                                              hs, S, loff, kv_dim, kv_mul, dim, L) == 0
    gpu.sync()
    xb = dxb.download().reshape(B, dim)
    att = datt.download().reshape(B, H, S)
    for b in range(B):
        xb_ref, att_ref = oracle.attention(q[b], kc[b, layer], vc[b, layer], int(pos[b]), H, hs, kv_dim, kv_mul, S)
        n = pos[b] + 1
        assert_ref_close(att[b, :, :n], att_ref[:, :n], 1e-4, "att probs")
        assert_ref_close(xb[b], xb_ref, 1e-4, "attn out")


def test_mha_v2_layout(gpu, handle, oracle):
    B, H, kvh, hs, W = 3, 4, 2, 32, 50
    r = rng(11)
    dim, kv_dim, kv_mul = H * hs, kvh * hs, H // kvh
    pos = np.array([0, 17, 49], np.int32)
    q = r.standard_normal((B, dim)).astype(np.float32)
    kc = r.standard_normal((W, B, kv_dim)).astype(np.float32)  # [t][b][kv_dim]
    vc = r.standard_normal((W, B, kv_dim)).astype(np.float32)
    dq, dk, dv, dpos = dev(gpu, q), dev(gpu, kc), dev(gpu, vc), dev(gpu, pos)
    datt, dxb = dev(gpu, np.zeros((B, H, W), np.float32)), gpu.DevBuf(B * dim * 4)
    hpos = (C.c_int * B)(*pos.tolist())
    lib = gpu.lib()
    assert lib.thaDNN_s_multiheads_1_v2_batch(C.byref(handle), B, 1, hpos, dpos.iptr(), H, dq.fptr(), datt.fptr(),
                                              dk.fptr(), hs, W, kv_dim, dim, kv_mul) == 0
    assert lib.thaDNN_s_multiheads_2_batch(C.byref(handle), B, datt.fptr(), dpos.iptr(), W, H) == 0
    assert lib.thaDNN_s_multiheads_3_v2_batch(C.byref(handle), B, dpos.iptr(), H, dxb.fptr(), datt.fptr(), dv.fptr(),
                                              hs, W, kv_dim, kv_mul, dim, 1) == 0
    gpu.sync()
    xb = dxb.download().reshape(B, dim)
    for b in range(B):
        xb_ref, _ = oracle.attention(q[b], kc[:, b], vc[:, b], int(pos[b]), H, hs, kv_dim, kv_mul, W)
        assert_ref_close(xb[b], xb_ref, 1e-4, "attn v2")


def test_invalid_arguments(gpu, handle):
    lib = gpu.lib()
    assert lib.thaBLAS_s_matmul(handle, 0, 3, 3, None, None, None) != 0
    assert lib.thaDNN_s_softmax_v2(C.byref(handle), None, 0) != 0
    assert lib.thaBLAS_s_vecaddvec(None, None, None, 4) != 0
