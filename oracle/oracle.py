"""oracle.py — TEST INFRASTRUCTURE ONLY: ctypes bindings of the CPU oracle.

* ``liboracle.so``  — our C restatement of the reference CPU path (oracle.c);
* ``_ref/libref_seq.so`` / ``_ref/librunq.so`` — the REFERENCE's own seq.cpp /
  runq.c compiled from /root/reference by oracle/Makefile (absent on machines
  where the reference tree was never present and nothing was prebuilt).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module, and only as the checker or the CPU baseline.  The product
(hip_llama.cpp_amd) never imports it.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
REF_SEQ = os.path.join(HERE, "_ref", "libref_seq.so")
REF_RUNQ = os.path.join(HERE, "_ref", "librunq.so")

F = C.POINTER(C.c_float)
I8 = C.POINTER(C.c_int8)
IP = C.POINTER(C.c_int)


class OCfg(C.Structure):
    _fields_ = [("dim", C.c_int), ("hidden_dim", C.c_int), ("n_layers", C.c_int), ("n_heads", C.c_int),
                ("n_kv_heads", C.c_int), ("vocab_size", C.c_int), ("seq_len", C.c_int)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        V, S, U64 = C.c_void_p, C.c_size_t, C.c_uint64
        sig = {
            "oracle_set_threads": (None, [C.c_int]),
            "oracle_get_threads": (C.c_int, []),
            "oracle_rmsnorm": (None, [F, F, F, C.c_int]),
            "oracle_softmax": (None, [F, C.c_int]),
            "oracle_matmul": (None, [F, F, F, C.c_int, C.c_int]),
            "oracle_rope": (None, [F, F, C.c_int, C.c_int, C.c_int, C.c_int]),
            "oracle_swiglu": (None, [F, F, C.c_int]),
            "oracle_attention": (None, [F, F, F, F, F, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]),
            "oracle_payload_floats": (S, [C.POINTER(OCfg), C.c_int]),
            "oracle_model_new": (V, [C.POINTER(OCfg), C.c_int, F, U64]),
            "oracle_model_arena": (F, [V]),
            "oracle_model_arena_floats": (S, [V]),
            "oracle_model_logits": (F, [V]),
            "oracle_model_kcache": (F, [V]),
            "oracle_model_vcache": (F, [V]),
            "oracle_model_x": (F, [V]),
            "oracle_model_buf": (F, [V, C.c_int]),
            "oracle_model_reset_kv": (None, [V]),
            "oracle_write_v0": (C.c_int, [V, C.c_char_p]),
            "oracle_model_free": (None, [V]),
            "oracle_forward": (F, [V, C.c_int, C.c_int]),
            "oracle_forward_f64": (C.c_int, [V, C.c_int, C.c_int, C.POINTER(C.c_double)]),
            "oracle_forward_f64_ex": (C.c_int, [V, C.c_int, C.c_int, C.POINTER(C.c_double), C.c_int]),
            "oracle_argmax": (C.c_int, [F, C.c_int]),
            "oracle_greedy": (C.c_int, [V, C.c_int, C.c_int, C.c_int, IP]),
            "oracle_q8_quantize": (None, [I8, F, F, C.c_int, C.c_int]),
            "oracle_q8_quantize_weights": (None, [I8, F, F, S, C.c_int]),
            "oracle_q8_matmul": (None, [F, I8, F, I8, F, C.c_int, C.c_int, C.c_int]),
            "oracle_q8_build": (C.c_int, [V, C.c_int]),
            "oracle_q8_payload": (C.POINTER(C.c_uint8), [V]),
            "oracle_q8_payload_size": (S, [V]),
            "oracle_write_v2": (C.c_int, [V, C.c_char_p]),
            "oracle_q8_forward": (F, [V, C.c_int, C.c_int]),
            "oracle_q8_greedy": (C.c_int, [V, C.c_int, C.c_int, C.c_int, IP]),
            "oracle_synth_fill": (None, [F, S, U64, C.c_int, C.c_double, S]),
            "oracle_aggregate": (C.c_double, [V, C.c_int, C.c_int, IP, C.c_int, C.c_int, IP]),
            "oracle_model_view_cap": (V, [V, C.c_int]),
            "oracle_forward_multi": (C.c_int, [C.POINTER(V), C.c_int, IP, IP]),
        }
        for n, (r, a) in sig.items():
            fn = getattr(L, n)
            fn.restype, fn.argtypes = r, a
        _lib = L
    return _lib


def fp(a):
    return a.ctypes.data_as(F)


def set_threads(n):
    lib().oracle_set_threads(int(n))


# ---------------------------------------------------------------- ops
def rmsnorm(x, w):
    x = np.ascontiguousarray(x, np.float32)
    o = np.empty_like(x)
    lib().oracle_rmsnorm(fp(o), fp(x), fp(np.ascontiguousarray(w, np.float32)), x.size)
    return o


def softmax(x):
    x = np.array(x, np.float32, copy=True)
    lib().oracle_softmax(fp(x), x.size)
    return x


def matmul(w, x):
    """w [d][n] row-major, x [n] -> [d]"""
    w = np.ascontiguousarray(w, np.float32)
    x = np.ascontiguousarray(x, np.float32)
    d, n = w.shape
    o = np.empty(d, np.float32)
    lib().oracle_matmul(fp(o), fp(x), fp(w), n, d)
    return o


def rope(q, k, dim, head_size, kv_dim, pos):
    q = np.array(q, np.float32, copy=True)
    k = np.array(k, np.float32, copy=True)
    lib().oracle_rope(fp(q), fp(k), dim, head_size, kv_dim, pos)
    return q, k


def swiglu(hb, hb2):
    hb = np.array(hb, np.float32, copy=True)
    lib().oracle_swiglu(fp(hb), fp(np.ascontiguousarray(hb2, np.float32)), hb.size)
    return hb


def attention(q, kc, vc, pos, n_heads, head_size, kv_dim, kv_mul, seq_len):
    """q [dim]; kc/vc [seq_len][kv_dim] for one layer -> (xb [dim], att [H][seq_len])"""
    xb = np.zeros(n_heads * head_size, np.float32)
    att = np.zeros(n_heads * seq_len, np.float32)
    lib().oracle_attention(fp(xb), fp(att), fp(np.ascontiguousarray(q, np.float32)),
                           fp(np.ascontiguousarray(kc, np.float32)), fp(np.ascontiguousarray(vc, np.float32)), pos,
                           n_heads, head_size, kv_dim, kv_mul, seq_len)
    return xb, att.reshape(n_heads, seq_len)


def q8_quantize(x, gs):
    x = np.ascontiguousarray(x, np.float32)
    q = np.empty(x.size, np.int8)
    s = np.empty(x.size // gs, np.float32)
    lib().oracle_q8_quantize(q.ctypes.data_as(I8), fp(s), fp(x), x.size, gs)
    return q, s


def q8_quantize_weights(w, gs):
    w = np.ascontiguousarray(w, np.float32).ravel()
    q = np.empty(w.size, np.int8)
    s = np.empty(w.size // gs, np.float32)
    lib().oracle_q8_quantize_weights(q.ctypes.data_as(I8), fp(s), fp(w), w.size, gs)
    return q, s


def q8_matmul(xq, xs, wq, ws, n, d, gs):
    o = np.empty(d, np.float32)
    lib().oracle_q8_matmul(fp(o), np.ascontiguousarray(xq, np.int8).ctypes.data_as(I8), fp(np.ascontiguousarray(xs)),
                           np.ascontiguousarray(wq, np.int8).ctypes.data_as(I8), fp(np.ascontiguousarray(ws)), n, d, gs)
    return o


def synth_fill(n, seed, tid, stddev, offset=0):
    out = np.empty(n, np.float32)
    lib().oracle_synth_fill(fp(out), n, seed, tid, stddev, offset)
    return out


# ---------------------------------------------------------------- model
class Model:
    """Single-sequence CPU model over a v0 payload (synthetic when payload is None)."""

    def __init__(self, cfg_tuple, shared, seed=0, payload=None):
        self.cfg = OCfg(*cfg_tuple)
        self.shared = int(bool(shared))
        self.vocab = abs(cfg_tuple[5])
        arr = None
        if payload is not None:
            arr = np.ascontiguousarray(payload, np.float32)
        self.h = lib().oracle_model_new(C.byref(self.cfg), self.shared, fp(arr) if arr is not None else None,
                                        C.c_uint64(seed))
        if not self.h:
            raise MemoryError("oracle_model_new failed")
        self.q8 = False

    def arena(self):
        n = lib().oracle_model_arena_floats(self.h)
        return np.ctypeslib.as_array(lib().oracle_model_arena(self.h), shape=(n,))

    def forward(self, token, pos):
        p = lib().oracle_forward(self.h, token, pos)
        return np.ctypeslib.as_array(p, shape=(self.vocab,)).copy()

    def forward_f64(self, token, pos, rope_double=False, own_cache=False):
        """The same forward in double precision from this model's K/V rows 0..pos-1 (the fp32 cache
        is not modified): the exact value of the reference's arithmetic, to attribute rounding.
        rope_double: RoPE's (cos, sin) in double too (default: the reference's float values);
        own_cache: earlier positions' K/V from this function's own double cache (written by every
        own_cache call) instead of the fp32 cache — with both, src/seq.cpp widened to double."""
        out = np.zeros(self.vocab, np.float64)
        flags = (1 if rope_double else 0) | (2 if own_cache else 0)
        if lib().oracle_forward_f64_ex(self.h, token, pos, out.ctypes.data_as(C.POINTER(C.c_double)), flags) != 0:
            raise MemoryError("oracle_forward_f64")
        return out

    def greedy(self, token, pos0, n):
        out = (C.c_int * n)()
        lib().oracle_greedy(self.h, token, pos0, n, out)
        return list(out)

    def logits(self):
        """The logits of the last forward (a copy)."""
        return np.ctypeslib.as_array(lib().oracle_model_logits(self.h), shape=(self.vocab,)).copy()

    def buf(self, which, n):
        """RunState buffer after a forward: 0 x, 1 xb, 2 xb2, 3 hb, 4 hb2, 5 q, 6 k, 7 v (diagnostics)."""
        return np.ctypeslib.as_array(lib().oracle_model_buf(self.h, which), shape=(n,)).copy()

    def reset_kv(self):
        lib().oracle_model_reset_kv(self.h)

    def kcache(self):
        c = self.cfg
        n = c.n_layers * c.seq_len * (c.dim * c.n_kv_heads // c.n_heads)
        return np.ctypeslib.as_array(lib().oracle_model_kcache(self.h), shape=(n,)).copy()

    def write_v0(self, path):
        if lib().oracle_write_v0(self.h, path.encode()) != 0:
            raise IOError(path)

    # int8 twin
    def build_q8(self, gs=64):
        if lib().oracle_q8_build(self.h, gs) != 0:
            raise MemoryError("oracle_q8_build")
        self.q8, self.gs = True, gs

    def q8_payload(self):
        n = lib().oracle_q8_payload_size(self.h)
        return np.ctypeslib.as_array(lib().oracle_q8_payload(self.h), shape=(n,)).copy()

    def write_v2(self, path):
        if lib().oracle_write_v2(self.h, path.encode()) != 0:
            raise IOError(path)

    def q8_forward(self, token, pos):
        p = lib().oracle_q8_forward(self.h, token, pos)
        return np.ctypeslib.as_array(p, shape=(self.vocab,)).copy()

    def q8_greedy(self, token, pos0, n):
        out = (C.c_int * n)()
        lib().oracle_q8_greedy(self.h, token, pos0, n, out)
        return list(out)

    def aggregate(self, P, n, cpus=None):
        """BASELINE.md CPU-baseline mode (ii): P independent single-threaded decoders (decoder i
        from token 1+i at pos 0, pinned to cpus[i % len(cpus)]) of n greedy tokens each, at once,
        over these weights.  Returns (wall seconds, tokens [P][n])."""
        cpus = list(cpus or [])
        cp = (C.c_int * max(1, len(cpus)))(*cpus) if cpus else None
        out = (C.c_int * (P * n))()
        secs = lib().oracle_aggregate(self.h, int(self.q8), P, cp, len(cpus), n, out)
        if secs < 0:
            raise MemoryError("oracle_aggregate")
        return secs, np.array(list(out), np.int32).reshape(P, n)

    def close(self):
        if self.h:
            lib().oracle_model_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Lockstep:
    """B sequences over one Model's weights, stepped together (oracle_forward_multi): each
    sequence has its own RunState and K/V cache (positions < seq_cap), and its logits are
    bit-identical to Model.forward's for the same (token, pos) history.  Fixture generation."""

    def __init__(self, model, B, seq_cap=0):
        self.model, self.vocab = model, model.vocab
        self.views = [lib().oracle_model_view_cap(model.h, int(seq_cap)) for _ in range(B)]
        if not all(self.views):
            self.close()
            raise MemoryError("oracle_model_view_cap")

    def forward(self, idx, tokens, pos):
        """One step of the sequences idx (indices into this batch) at (tokens, pos): logits [len(idx)][V]."""
        n = len(idx)
        arr = (C.c_void_p * n)(*[self.views[i] for i in idx])
        tk = (C.c_int * n)(*[int(t) for t in tokens])
        ps = (C.c_int * n)(*[int(p) for p in pos])
        if lib().oracle_forward_multi(arr, n, tk, ps) != 0:
            raise ValueError("oracle_forward_multi: bad position or mixed models")
        return np.stack([np.ctypeslib.as_array(lib().oracle_model_logits(self.views[i]), shape=(self.vocab,)).copy()
                         for i in idx]) if n else np.zeros((0, self.vocab), np.float32)

    def close(self):
        for v in getattr(self, "views", []):
            if v:
                lib().oracle_model_free(v)
        self.views = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---------------------------------------------------------------- the reference itself (oracle/_ref)
def have_ref():
    return os.path.exists(REF_SEQ)


def have_ref_q8():
    return os.path.exists(REF_RUNQ)


_ref = None
_refq = None


def ref_lib():
    global _ref
    if _ref is None:
        L = C.CDLL(REF_SEQ)
        L.ref_greedy.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int, IP, F]
        L.ref_forced.argtypes = [C.c_char_p, IP, C.c_int, C.c_int, F]
        L.ref_rmsnorm.argtypes = [F, F, F, C.c_int]
        L.ref_softmax.argtypes = [F, C.c_int]
        L.ref_matmul.argtypes = [F, F, F, C.c_int, C.c_int]
        _ref = L
    return _ref


def ref_q8_lib():
    global _refq
    if _refq is None:
        L = C.CDLL(REF_RUNQ)
        L.ref_q8_greedy.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int, IP, F]
        _refq = L
    return _refq


REF_SEQ_F64 = os.path.join(HERE, "_ref", "libref_seq_f64.so")


def have_ref_f64():
    return os.path.exists(REF_SEQ_F64)


def ref64_forced(path, tokens, vocab):
    """The reference's src/seq.cpp widened to double (oracle/ref_f64_driver.cpp): teacher-forced
    logits [n][vocab] (float64) of tokens[i] at position i."""
    L = C.CDLL(REF_SEQ_F64)
    L.ref64_forced.argtypes = [C.c_char_p, IP, C.c_int, C.c_int, C.POINTER(C.c_double)]
    n = len(tokens)
    out = np.zeros(n * vocab, np.float64)
    if L.ref64_forced(path.encode(), (C.c_int * n)(*[int(t) for t in tokens]), 0, n,
                      out.ctypes.data_as(C.POINTER(C.c_double))) != 0:
        raise IOError(path)
    return out.reshape(n, vocab)


def ref_greedy(path, token, pos0, n, vocab):
    toks = (C.c_int * n)()
    logits = np.empty(n * vocab, np.float32)
    ref_lib().ref_greedy(path.encode(), token, pos0, n, toks, fp(logits))
    return list(toks), logits.reshape(n, vocab)


def ref_q8_greedy(path, token, pos0, n, vocab):
    toks = (C.c_int * n)()
    logits = np.empty(n * vocab, np.float32)
    ref_q8_lib().ref_q8_greedy(path.encode(), token, pos0, n, toks, fp(logits))
    return list(toks), logits.reshape(n, vocab)
