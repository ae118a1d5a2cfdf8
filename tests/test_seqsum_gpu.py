"""GPU: the wave-parallel left-to-right fp32 sum (csrc/seqsum.hpp; used by the int8 path for the
RMSNorm sum of squares, src/seq.cpp:5-8 / runq.c:284-287, and the softmax denominator,
runq.c:306-310) is bit-identical to the sequential chain s = fl(s + a[k]) on typical (squares of
Gaussians: the norm's input), heavy-tailed, tie-rich (small integers), power-of-two, front-loaded
and ragged-length arrays, and on the softmax's own inputs (exp of shifted scores)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def seq_chain(a):
    s = np.float32(0)
    for v in a.astype(np.float32):
        s = np.float32(s + v)
    return s


def arrays(kind, n, count, rng):
    if kind == "gauss_sq":
        x = rng.standard_normal((count, n)).astype(np.float32)
        return x * x
    if kind == "heavy_sq":
        x = (rng.standard_normal((count, n)) * np.exp(3 * rng.standard_normal((count, n)))).astype(np.float32)
        return x * x
    if kind == "ints_sq":
        x = np.trunc(rng.standard_normal((count, n)) * 8).astype(np.float32)
        return x * x
    if kind == "pow2":
        return np.ldexp(np.ones((count, n)), rng.integers(-10, 10, (count, n))).astype(np.float32)
    if kind == "front":
        x = (rng.standard_normal((count, n)) * 1e-3).astype(np.float32)
        x[:, :8] *= 1e6
        return x * x
    if kind == "softmax":
        s = (rng.standard_normal((count, n)) * 3).astype(np.float32)
        return np.exp(s - s.max(axis=1, keepdims=True)).astype(np.float32)
    raise ValueError(kind)


@pytest.mark.parametrize("kind", ["gauss_sq", "heavy_sq", "ints_sq", "pow2", "front", "softmax"])
@pytest.mark.parametrize("n", [4096, 768, 1, 37, 256, 300, 1000, 2048, 5000, 8192])
def test_wave_seqsum_bitexact(gpu, kind, n):
    rng = np.random.default_rng(n * 7 + len(kind))
    count = 64
    a = np.ascontiguousarray(arrays(kind, n, count, rng), np.float32)
    din = gpu.DevBuf.from_array(a)
    dout = gpu.DevBuf(4 * count)
    gpu.check(gpu.lib().thallama_seqsum_check(din.ptr, n, count, dout.ptr), "seqsum_check")
    got = dout.download(np.float32)
    want = np.array([seq_chain(r) for r in a], np.float32)
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("kind", ["gauss_sq", "ints_sq", "softmax"])
@pytest.mark.parametrize("n", [4096, 4095, 3000, 2304, 2049, 768, 200])
def test_wave_seqsum_reg_bitexact(gpu, kind, n):
    """The register form (n <= 4096; the norm and softmax sums of the int8 step) is the chain too;
    it also reports clock cycles per call (printed)."""
    rng = np.random.default_rng(n * 11 + len(kind))
    count = 64
    a = np.ascontiguousarray(arrays(kind, n, count, rng), np.float32)
    din = gpu.DevBuf.from_array(a)
    dout = gpu.DevBuf(4 * count)
    dcyc = gpu.DevBuf(8 * (count + 16))  # (+ array 0's failing lane per round, diagnostics)
    gpu.check(gpu.lib().thallama_seqsum_time(din.ptr, n, count, dout.ptr, dcyc.ptr), "seqsum_time")
    got = dout.download(np.float32)
    want = np.array([seq_chain(r) for r in a], np.float32)
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
    raw = dcyc.download(np.int64)[:count]
    cyc, rounds = raw & ((1 << 48) - 1), raw >> 48
    print(f"seqsum_reg {kind} n={n}: cycles median {int(np.median(cyc))} max {int(cyc.max())}, "
          f"rounds mean {rounds.mean():.2f} max {int(rounds.max())}")

