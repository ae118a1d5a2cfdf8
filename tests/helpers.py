"""Test helpers shared by the CPU and GPU suites."""
import numpy as np

# Small synthetic model shapes.  (dim, hidden, layers, heads, kv_heads, vocab, seq_len)
TINY = (64, 172, 2, 4, 2, 512, 64)          # GQA, K=172 exercises the generic GEMV path
SMALL = (256, 768, 2, 4, 4, 1024, 128)      # every GEMV on the streaming path (K % 256 == 0)
SMALL_GQA = (512, 1536, 3, 8, 2, 2048, 256)
STORIES_110M = (768, 2048, 12, 12, 12, 32000, 1024)   # stories110M shape (shared classifier)
LLAMA2_7B = (4096, 11008, 32, 32, 32, 32000, 2048)    # llama2-7B shape (unshared classifier)


def ref_close_mask(got, ans, eps):
    """The reference tests' acceptance rule (scripts/test/thaDNN.test.cpp:64-69, 224-229):
    an element fails only if BOTH |got-ans| > eps and |got-ans|/|ans| > eps (ans != 0)."""
    got = np.asarray(got, np.float64)
    ans = np.asarray(ans, np.float64)
    d = np.abs(got - ans)
    with np.errstate(divide="ignore", invalid="ignore"):
        rel = np.where(ans != 0, d / np.abs(ans), np.inf)
    return ~((d > eps) & (rel > eps))


def assert_ref_close(got, ans, eps, what=""):
    ok = ref_close_mask(got, ans, eps)
    if not ok.all():
        bad = np.flatnonzero(~ok.ravel())
        g = np.asarray(got).ravel()
        a = np.asarray(ans).ravel()
        i = bad[0]
        raise AssertionError(f"{what}: {bad.size} of {ok.size} elements differ beyond eps={eps} "
                             f"(first at {i}: got {g[i]!r} want {a[i]!r}; max abs diff "
                             f"{np.max(np.abs(g.astype(np.float64) - a)):.3g})")


def rng(seed):
    return np.random.default_rng(seed)
