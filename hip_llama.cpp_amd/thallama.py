"""ctypes bindings of libthallama.so (include/thaBLAS.hpp, include/thaDNN.hpp,
include/models.hpp, include/thallama.h).

Host-side mirror of the reference's operator interface: the same entry-point
names, argument meaning and status codes as /root/reference/include/thaBLAS.hpp
and thaDNN.hpp, so tests read like the reference's own GPU-vs-CPU tests
(scripts/test/thaDNN.test.cpp).  There is deliberately NO fallback: if the HIP
library is missing or no GPU is present, calls raise.
"""
import ctypes as C
import os

import numpy as np

from . import LIB_PATH

# ---------------------------------------------------------------- ABI types
c_float_p = C.POINTER(C.c_float)
c_int_p = C.POINTER(C.c_int)


class Config(C.Structure):
    """reference include/models.hpp:10-18"""
    _fields_ = [("dim", C.c_int), ("hidden_dim", C.c_int), ("n_layers", C.c_int), ("n_heads", C.c_int),
                ("n_kv_heads", C.c_int), ("vocab_size", C.c_int), ("seq_len", C.c_int)]

    @classmethod
    def make(cls, dim, hidden_dim, n_layers, n_heads, n_kv_heads, vocab_size, seq_len):
        return cls(dim, hidden_dim, n_layers, n_heads, n_kv_heads, vocab_size, seq_len)

    def as_tuple(self):
        return tuple(getattr(self, f) for f, _ in self._fields_)

    @property
    def head_size(self):
        return self.dim // self.n_heads

    @property
    def kv_dim(self):
        return self.dim * self.n_kv_heads // self.n_heads


class TransformerWeights(C.Structure):
    """reference include/models.hpp:20-39"""
    _fields_ = [(n, c_float_p) for n in ("token_embedding_table", "rms_att_weight", "rms_ffn_weight", "wq", "wk",
                                          "wv", "wo", "w1", "w2", "w3", "rms_final_weight", "wcls")]


class RunState(C.Structure):
    """reference include/models.hpp:41-60"""
    _fields_ = [(n, c_float_p) for n in ("x", "xb", "xb2", "hb", "hb2", "q", "k", "v", "att", "logits", "key_cache",
                                          "value_cache", "key_matmul", "value_matmul", "key_layer_cache",
                                          "value_layer_cache")]


class Transformer(C.Structure):
    """reference include/models.hpp:62-70"""
    _fields_ = [("config", Config), ("weights", TransformerWeights), ("state", RunState), ("fd", C.c_int),
                ("data", c_float_p), ("file_size", C.c_ssize_t)]


class QuantizedTensor(C.Structure):
    """runq.c:34-37 (include/thaQ8.hpp)"""
    _fields_ = [("q", C.POINTER(C.c_int8)), ("s", c_float_p)]


class Q8TransformerWeights(C.Structure):
    """runq.c:39-59 field order (include/thaQ8.hpp)"""
    _fields_ = [("q_tokens", C.POINTER(QuantizedTensor)), ("token_embedding_table", c_float_p),
                ("rms_att_weight", c_float_p), ("rms_ffn_weight", c_float_p)] + \
               [(n, C.POINTER(QuantizedTensor)) for n in ("wq", "wk", "wv", "wo", "w1", "w2", "w3")] + \
               [("rms_final_weight", c_float_p), ("wcls", C.POINTER(QuantizedTensor)), ("group_size", C.c_int)]


class Q8Checkpoint(C.Structure):
    """include/thaQ8.hpp: a v2 "ak42" file opened like runq.c read_checkpoint (:219-251)"""
    _fields_ = [("config", Config), ("shared_classifier", C.c_int), ("group_size", C.c_int), ("fd", C.c_int),
                ("data", C.c_void_p), ("file_size", C.c_size_t), ("payload", C.c_void_p),
                ("payload_bytes", C.c_size_t)]


class Handle(C.Structure):
    """thablasHandle_t, reference include/thaBLAS.hpp:21-25"""
    _fields_ = [("current_gpu_id", C.c_int), ("calc_stream", C.c_void_p), ("copy_stream", C.c_void_p)]


STATUS = {0: "SUCCESS", 1: "NOT_INITIALIZED", 2: "ALLOC_FAILED", 3: "INVALID_VALUE", 4: "MAPPING_ERROR",
          5: "EXECUTION_FAILED", 6: "INTERNAL_ERROR", 7: "NOT_SUPPORTED", 8: "ARCH_MISMATCH",
          9: "HANDLE_IS_NULLPTR", 10: "INVALID_ENUM", 11: "UNKNOWN"}

# kernel classes (include/thallama.h)
K_QKV, K_ATTN, K_WO, K_FFN_UP, K_FFN_DOWN, K_CLS, K_ARGMAX, K_STEP = range(8)
K_NAMES = ["qkv", "attn", "wo", "ffn_up", "ffn_down", "cls", "argmax", "step"]
OPT_NT_WEIGHTS, OPT_ATTN_SPLITS, OPT_USE_GRAPH, OPT_PROFILE, OPT_PERSISTENT, OPT_PERSIST_FAULT = 1, 2, 3, 4, 5, 6
OPT_KSPLIT = 7

_lib = None


def lib():
    """Load libthallama.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
        L = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        P, I, F, VP, S = c_float_p, C.c_int, C.c_float, C.c_void_p, C.c_size_t
        sig = {
            "thablasCreate": (I, [C.POINTER(Handle)]),
            "thablasDestroy": (I, [Handle]),
            "thablas_Svds": (I, [Handle, I, P, P, F]),
            "thaBLAS_s_vecaddvec": (I, [C.POINTER(Handle), P, P, I]),
            "thaBLAS_s_matmulvec": (I, [Handle, P, P, P, I, I]),
            "thaDNN_s_matmulvec_v2": (I, [Handle, P, P, P, I, I]),
            "thaBLAS_s_matmul": (I, [Handle, I, I, I, P, P, P]),
            "thaBLAS_s_matmul_batch": (I, [C.POINTER(Handle), I, P, P, P, I, I, I, I, c_int_p, I, I]),
            "thaBLAS_s_matmul_reduction": (I, [C.POINTER(Handle), P, P, P, I, I, I]),
            "thaBLAS_s_sgemm_Mx16xK": (I, [C.POINTER(Handle), P, P, P, I, I, I]),
            "thaBLAS_s_matmul_ifdef": (I, [C.POINTER(Handle), P, P, P, I, I, I]),
            "thaDNN_s_rmsnorm_v2_batch": (I, [C.POINTER(Handle), I, P, P, P, I, I]),
            "thaDNN_s_rope": (I, [C.POINTER(Handle), I, I, I, I, P, P]),
            "thaDNN_s_swiglu": (I, [C.POINTER(Handle), P, P, I]),
            "thaDNN_s_softmax_v2": (I, [C.POINTER(Handle), P, I]),
            "thaDNN_s_multiheads_1_v1_batch": (I, [C.POINTER(Handle), I, c_int_p, c_int_p, I, I, P, P, P, I, I, I, I,
                                                   I, I]),
            "thaDNN_s_multiheads_2_v1_batch": (I, [C.POINTER(Handle), I, P, c_int_p, I, I]),
            "thaDNN_s_multiheads_3_v1_batch": (I, [C.POINTER(Handle), I, c_int_p, I, P, P, P, I, I, I, I, I, I, I]),
            "thaDNN_s_multiheads_1_v2_batch": (I, [C.POINTER(Handle), I, I, c_int_p, c_int_p, I, P, P, P, I, I, I, I,
                                                   I]),
            "thaDNN_s_multiheads_2_batch": (I, [C.POINTER(Handle), I, P, c_int_p, I, I]),
            "thaDNN_s_multiheads_3_v2_batch": (I, [C.POINTER(Handle), I, c_int_p, I, P, P, P, I, I, I, I, I, I]),
            "thaDNN_s_forward_batch": (I, [Handle, Handle, Handle, I, C.POINTER(Config), C.POINTER(TransformerWeights),
                                           C.POINTER(RunState), c_int_p, c_int_p, P]),
            "thallama_v0_payload_floats": (S, [C.POINTER(Config), I]),
            "thallama_map_weights": (None, [C.POINTER(TransformerWeights), C.POINTER(Config), P, I]),
            "alloc_state_to_device_batch": (None, [C.POINTER(Transformer), C.POINTER(C.POINTER(RunState)), I]),
            "free_state_device": (None, [C.POINTER(RunState)]),
            "thallama_decoder_create": (I, [C.POINTER(VP), C.POINTER(Config), C.POINTER(TransformerWeights),
                                            C.POINTER(RunState), I, VP]),
            "thallama_decoder_create_q8": (I, [C.POINTER(VP), C.POINTER(Config), C.POINTER(Q8TransformerWeights),
                                               C.POINTER(RunState), I, VP]),
            "thallama_q8_payload_bytes": (S, [C.POINTER(Config), I, I]),
            "thallama_q8_read_checkpoint": (I, [C.c_char_p, C.POINTER(Q8Checkpoint)]),
            "thallama_q8_close_checkpoint": (None, [C.POINTER(Q8Checkpoint)]),
            "read_checkpoint": (None, [C.c_char_p, C.POINTER(Config), C.POINTER(TransformerWeights),
                                       C.POINTER(C.c_int), C.POINTER(P), C.POINTER(C.c_ssize_t)]),
            "thallama_q8_map": (I, [C.POINTER(Q8TransformerWeights), C.POINTER(Config), VP, I, I, P]),
            "thallama_q8_unmap": (None, [C.POINTER(Q8TransformerWeights)]),
            "thallama_q8_dequant_embedding": (I, [C.POINTER(Q8TransformerWeights), C.POINTER(Config), VP]),
            "thallama_q8_quantize_model": (I, [VP, C.POINTER(TransformerWeights), C.POINTER(Config), I, I, VP]),
            "thaBLAS_q8_quantize_batch": (I, [C.POINTER(Handle), I, C.POINTER(C.c_int8), P, P, I, I, I]),
            "thaBLAS_q8_matmul_batch": (I, [C.POINTER(Handle), I, P, P, C.POINTER(C.c_int8), P, I, I, I, I, I]),
            "thaDNN_q8_forward_batch": (I, [Handle, I, C.POINTER(Config), C.POINTER(Q8TransformerWeights),
                                            C.POINTER(RunState), c_int_p, c_int_p, P]),
            "thallama_decoder_destroy": (None, [VP]),
            "thallama_decoder_set": (I, [VP, I, I]),
            "thallama_decoder_persistent": (I, [VP]),
            "thallama_decoder_ksplit": (I, [VP]),
            "thallama_persistent_cooperative": (I, []),
            "thallama_decoder_granules": (I, [VP, C.POINTER(C.c_ulonglong), S]),
            "thallama_decoder_prefill": (I, [VP, I, c_int_p, I, I]),
            "thallama_decoder_ptrace": (I, [VP, I, C.POINTER(C.c_ulonglong), C.c_size_t]),
            "thallama_decoder_stream": (VP, [VP]),
            "thallama_decoder_forward": (I, [VP, c_int_p, c_int_p, P]),
            "thallama_decoder_greedy": (I, [VP, c_int_p, c_int_p, I, c_int_p, I]),
            "thallama_decoder_logits": (I, [VP, P]),
            "thallama_decoder_sync": (I, [VP]),
            "thallama_decoder_prof": (I, [VP, I, C.POINTER(C.c_double), C.POINTER(C.c_longlong)]),
            "thallama_decoder_prof_reset": (None, [VP]),
            "thallama_step_bytes": (C.c_double, [C.POINTER(Config), I, I, c_int_p]),
            "thallama_decoder_stage": (I, [VP, c_int_p, c_int_p, I, P, VP, P, I]),
            "thaDNN_s_forward_70B": (I, [Handle, I, C.POINTER(Config), C.POINTER(C.POINTER(TransformerWeights)),
                                         C.POINTER(RunState), C.POINTER(TransformerWeights), C.POINTER(RunState),
                                         c_int_p, c_int_p, P]),
            "thaDNN_s_forward_batch_pipe_line": (I, [C.POINTER(Handle), I, I, C.POINTER(C.POINTER(Transformer)),
                                                     c_int_p, c_int_p, P]),
            "thaDNN_s_forward_batch_multiple_pipe_line": (
                I, [C.POINTER(Handle), I, I, I, I, C.POINTER(Config), C.POINTER(C.POINTER(TransformerWeights)),
                    C.POINTER(C.POINTER(RunState)), c_int_p, c_int_p, P, c_int_p, c_int_p, VP]),
            "thaDNN_s_forward_batch_multiple_pipe_line_layer_swap": (
                I, [C.POINTER(Handle), I, I, I, I, I, C.POINTER(Config), C.POINTER(C.POINTER(TransformerWeights)),
                    C.POINTER(C.POINTER(RunState)), C.POINTER(C.POINTER(RunState)), c_int_p, c_int_p, P, VP]),
            "copy_transformer_weight_pipeline_to_device_batch": (
                None, [C.POINTER(Transformer), C.POINTER(C.POINTER(TransformerWeights)), I, I, I]),
            "alloc_run_state_to_device_batch": (None, [Handle, C.POINTER(Transformer), C.POINTER(C.POINTER(RunState)),
                                                       I, I, I]),
            "copy_transformer_pipeline_to_device_batch": (
                None, [Handle, C.POINTER(Transformer), C.POINTER(C.POINTER(Transformer)), I, I, I]),
            "alloc_swap_run_state_on_host_batch": (None, [Handle, C.POINTER(Transformer), C.POINTER(C.POINTER(RunState)),
                                                          I, I, I, I]),
            "alloc_swap_run_state_to_device_batch": (None, [Handle, C.POINTER(Transformer),
                                                            C.POINTER(C.POINTER(RunState)), I, I, I, I]),
            "copy_transformer_to_host_70B": (None, [C.POINTER(Transformer), C.POINTER(C.POINTER(TransformerWeights)),
                                                    C.POINTER(C.POINTER(RunState)), I]),
            "alloc_state_to_device_70B": (None, [C.POINTER(Transformer), C.POINTER(C.POINTER(RunState))]),
            "alloc_weight_to_device_70B": (None, [C.POINTER(Transformer), C.POINTER(C.POINTER(TransformerWeights))]),
            "free_weight_device": (None, [C.POINTER(TransformerWeights)]),
            "thallama_forward_batch_cache_size": (I, []),
            "thallama_forward_batch_cache_cap": (I, []),
            "thallama_forward_batch_live": (I, []),
            "thallama_forward_batch_cache_clear": (None, []),
            "thallama_synth_arena": (I, [P, C.POINTER(Config), I, C.c_uint64, VP]),
            "thallama_device_count": (I, []),
            "thallama_set_device": (I, [I]),
            "thallama_malloc": (VP, [S]),
            "thallama_free": (I, [VP]),
            "thallama_memcpy_h2d": (I, [VP, VP, S]),
            "thallama_memcpy_d2h": (I, [VP, VP, S]),
            "thallama_memcpy_d2d": (I, [VP, VP, S]),
            "thallama_memset": (I, [VP, I, S]),
            "thallama_sync": (I, []),
            "thallama_seqsum_check": (I, [VP, I, I, VP]),
            "thallama_seqsum_time": (I, [VP, I, I, VP, VP]),
            "thallama_last_error": (C.c_char_p, []),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc, what="call"):
    if rc != 0:
        err = lib().thallama_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed with status {rc} ({STATUS.get(rc, rc)}) {err}")
    return rc


def device_count():
    return lib().thallama_device_count()


# ---------------------------------------------------------------- device memory
class DevBuf:
    """Owning device allocation (hipMalloc) with numpy transfer helpers."""

    def __init__(self, nbytes):
        self.nbytes = int(nbytes)
        self.ptr = lib().thallama_malloc(self.nbytes)
        if not self.ptr:
            raise MemoryError(f"hipMalloc({self.nbytes}) failed")

    @classmethod
    def from_array(cls, a):
        a = np.ascontiguousarray(a)
        b = cls(a.nbytes)
        b.upload(a)
        return b

    def upload(self, a, offset=0):
        a = np.ascontiguousarray(a)
        check(lib().thallama_memcpy_h2d(C.c_void_p(self.ptr + offset), a.ctypes.data_as(C.c_void_p), a.nbytes), "h2d")

    def download(self, dtype=np.float32, count=None, offset=0):
        dtype = np.dtype(dtype)
        n = (self.nbytes - offset) // dtype.itemsize if count is None else count
        out = np.empty(n, dtype=dtype)
        check(lib().thallama_memcpy_d2h(out.ctypes.data_as(C.c_void_p), C.c_void_p(self.ptr + offset),
                                        out.nbytes), "d2h")
        return out

    def fptr(self, offset_elems=0):
        return C.cast(C.c_void_p(self.ptr + 4 * offset_elems), c_float_p)

    def iptr(self, offset_elems=0):
        return C.cast(C.c_void_p(self.ptr + 4 * offset_elems), c_int_p)

    def free(self):
        if self.ptr:
            lib().thallama_free(C.c_void_p(self.ptr))
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def new_handle():
    h = Handle()
    rc = lib().thablasCreate(C.byref(h))
    if rc != 0:
        raise RuntimeError(f"thablasCreate: {STATUS.get(rc, rc)}")
    return h


def sync():
    check(lib().thallama_sync(), "hipDeviceSynchronize")


# ---------------------------------------------------------------- model / state
class DeviceModel:
    """Weights in ONE device arena with the v0 payload layout (reference src/utils.cpp:119-148).

    Either filled by the deterministic synthetic generator on the device
    (``seed``), or uploaded from a host v0 payload (``payload``, e.g. a model.bin
    minus its 28-byte header, or the oracle's arena)."""

    def __init__(self, cfg, shared, seed=None, payload=None, arena_ptr=None):
        self.cfg = cfg
        self.shared = int(bool(shared))
        self.n = lib().thallama_v0_payload_floats(C.byref(cfg), self.shared)
        self.buf = None
        if arena_ptr is None:
            self.buf = DevBuf(self.n * 4)
            base = self.buf.ptr
        else:
            base = arena_ptr  # caller-owned (e.g. a torch tensor's data_ptr)
        self.base = base
        if payload is not None:
            payload = np.ascontiguousarray(payload, dtype=np.float32)
            assert payload.size == self.n, (payload.size, self.n)
            check(lib().thallama_memcpy_h2d(C.c_void_p(base), payload.ctypes.data_as(C.c_void_p), payload.nbytes))
        elif seed is not None:
            check(lib().thallama_synth_arena(C.cast(C.c_void_p(base), c_float_p), C.byref(cfg), self.shared,
                                             C.c_uint64(seed), None), "synth")
            sync()
        self.w = TransformerWeights()
        lib().thallama_map_weights(C.byref(self.w), C.byref(cfg), C.cast(C.c_void_p(base), c_float_p), self.shared)

    def arena_ptr(self):
        return self.base

    def download(self):
        out = np.empty(self.n, dtype=np.float32)
        check(lib().thallama_memcpy_d2h(out.ctypes.data_as(C.c_void_p), C.c_void_p(self.base), out.nbytes))
        return out


class DeviceModelQ8:
    """int8 twin of a model (include/thaQ8.hpp): a device runq-v2 payload (norms fp32, Q8_0
    tensors in export.py order) mapped like runq.c memory_map_weights, plus the dequantised
    fp32 embedding table runq keeps (runq.c:199-201).

    Built either by quantising a DeviceModel on the device (export.py semantics) or from a
    host payload (e.g. the oracle's, or a v2 file minus its 256-byte header)."""

    def __init__(self, cfg, shared, group_size=64, from_model=None, payload=None, payload_ptr=None):
        self.cfg = cfg
        self.shared = int(bool(shared))
        self.gs = group_size
        self.nbytes = lib().thallama_q8_payload_bytes(C.byref(cfg), self.shared, group_size)
        self.buf = None
        if payload_ptr is None:
            self.buf = DevBuf(self.nbytes)
            payload_ptr = self.buf.ptr
        self.base = payload_ptr  # caller-owned when given (e.g. a torch tensor's data_ptr)
        if from_model is not None:
            check(lib().thallama_q8_quantize_model(C.c_void_p(self.base), C.byref(from_model.w), C.byref(cfg),
                                                   self.shared, group_size, None), "q8 quantize")
        elif payload is not None:
            payload = np.ascontiguousarray(payload, np.uint8)
            assert payload.size == self.nbytes, (payload.size, self.nbytes)
            check(lib().thallama_memcpy_h2d(C.c_void_p(self.base), payload.ctypes.data_as(C.c_void_p), payload.nbytes))
        self.emb = DevBuf(abs(cfg.vocab_size) * cfg.dim * 4)
        self.w = Q8TransformerWeights()
        check(lib().thallama_q8_map(C.byref(self.w), C.byref(cfg), C.c_void_p(self.base), self.shared, group_size,
                                    self.emb.fptr()), "q8 map")
        check(lib().thallama_q8_dequant_embedding(C.byref(self.w), C.byref(cfg), None), "q8 dequant")
        sync()

    def payload(self):
        out = np.empty(self.nbytes, np.uint8)
        check(lib().thallama_memcpy_d2h(out.ctypes.data_as(C.c_void_p), C.c_void_p(self.base), self.nbytes))
        return out

    def close(self):
        if getattr(self, "w", None) is not None:
            lib().thallama_q8_unmap(C.byref(self.w))
            self.w = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceState:
    """Batched RunState (reference src/models.cpp:155-179)."""

    def __init__(self, cfg, batch):
        self.cfg = cfg
        self.batch = batch
        t = Transformer()
        t.config = cfg
        p = C.POINTER(RunState)()
        lib().alloc_state_to_device_batch(C.byref(t), C.byref(p), batch)
        self.ptr = p
        self.s = p.contents

    def free(self):
        if self.ptr:
            lib().free_state_device(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Decoder:
    """The fused decode step (thaDNN_s_forward_batch) as an object (include/thallama.h)."""

    def __init__(self, model, state, batch=None, stream=None):
        self.model, self.state = model, state
        self.cfg = model.cfg
        self.batch = batch or state.batch
        h = C.c_void_p()
        if isinstance(model, DeviceModelQ8):
            check(lib().thallama_decoder_create_q8(C.byref(h), C.byref(self.cfg), C.byref(model.w), C.byref(state.s),
                                                   self.batch, stream), "decoder_create_q8")
        else:
            check(lib().thallama_decoder_create(C.byref(h), C.byref(self.cfg), C.byref(model.w), C.byref(state.s),
                                                self.batch, stream), "decoder_create")
        self.h = h

    @property
    def vocab(self):
        return abs(self.cfg.vocab_size)

    def set(self, key, value):
        check(lib().thallama_decoder_set(self.h, key, int(value)), "decoder_set")

    def prefill(self, b, tokens, pos0):
        """Batched prompt processing for slot b (no logits; K/V rows at pos0..)."""
        arr = (C.c_int * len(tokens))(*[int(t) for t in tokens])
        return lib().thallama_decoder_prefill(self.h, b, arr, len(tokens), pos0)

    def persistent(self):
        """True if steps run as one persistent launch (persist.hip)."""
        return bool(lib().thallama_decoder_persistent(self.h))

    def ksplit(self):
        """True if the persistent step is the K-split one (8 sequences, csrc/persist_k.hip)."""
        return bool(lib().thallama_decoder_ksplit(self.h))

    def ptrace(self, enable=True):
        """Enable the persistent-step timeline; returns the stamps of the last launch as a
        [grid, phases, 8] uint64 array (100-MHz clock) once a launch has run."""
        n = lib().thallama_decoder_ptrace(self.h, int(enable), None, 0)
        check(0 if n >= 0 else n, "decoder_ptrace")
        out = np.zeros(n, np.uint64)
        lib().thallama_decoder_ptrace(self.h, 0, out.ctypes.data_as(C.POINTER(C.c_ulonglong)), n)
        return out

    def forward(self, tokens, pos, want_logits=True):
        tok = (C.c_int * self.batch)(*[int(t) for t in tokens])
        ps = (C.c_int * self.batch)(*[int(p) for p in pos])
        out = np.empty(self.batch * self.vocab, dtype=np.float32) if want_logits else None
        check(lib().thallama_decoder_forward(self.h, tok, ps, out.ctypes.data_as(c_float_p) if want_logits else None),
              "decoder_forward")
        return out.reshape(self.batch, self.vocab) if want_logits else None

    def greedy(self, tokens0, pos0, n_steps, want_tokens=True, sync=True):
        tok = (C.c_int * self.batch)(*[int(t) for t in tokens0])
        ps = (C.c_int * self.batch)(*[int(p) for p in pos0])
        out = (C.c_int * (n_steps * self.batch))() if want_tokens else None
        check(lib().thallama_decoder_greedy(self.h, tok, ps, n_steps, out, int(sync)), "decoder_greedy")
        if want_tokens:
            return np.frombuffer(out, dtype=np.int32).reshape(n_steps, self.batch).copy()
        return None

    def sync(self):
        """Wait for queued work; raises if an earlier asynchronous call's persistent step gave up."""
        check(lib().thallama_decoder_sync(self.h), "decoder_sync")

    def logits(self):
        out = np.empty(self.batch * self.vocab, dtype=np.float32)
        check(lib().thallama_decoder_logits(self.h, out.ctypes.data_as(c_float_p)), "decoder_logits")
        return out.reshape(self.batch, self.vocab)

    def prof(self, kclass):
        ms, n = C.c_double(), C.c_longlong()
        check(lib().thallama_decoder_prof(self.h, kclass, C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def prof_reset(self):
        lib().thallama_decoder_prof_reset(self.h)

    def stream(self):
        return lib().thallama_decoder_stream(self.h)

    def close(self):
        if getattr(self, "h", None):
            lib().thallama_decoder_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def step_bytes(cfg, batch, kclass, pos):
    arr = (C.c_int * batch)(*[int(p) for p in pos])
    return lib().thallama_step_bytes(C.byref(cfg), batch, kclass, arr)


def step_bytes_q8(cfg, batch, kclass, pos, gs):
    """Algorithmic HBM bytes of one launch of kernel class kclass on the int8 path: int8 weights
    + one fp32 scale per group, fp32 norms / activations / KV (as step_bytes)."""
    dim, hid, V = cfg.dim, cfg.hidden_dim, abs(cfg.vocab_size)
    kvd = cfg.kv_dim
    qt = lambda n: n + 4 * n // gs  # noqa: E731
    if kclass == K_QKV:
        return qt(dim * dim + 2 * dim * kvd) + 4 * (dim + batch * (2 * dim + 2 * kvd))
    if kclass == K_WO:
        return qt(dim * dim) + 4 * batch * 3 * dim
    if kclass == K_FFN_UP:
        return qt(2 * hid * dim) + 4 * (dim + batch * (dim + hid))
    if kclass == K_FFN_DOWN:
        return qt(hid * dim) + 4 * batch * (hid + 2 * dim)
    if kclass == K_CLS:
        return qt(V * dim) + 4 * (dim + batch * (dim + V))
    if kclass == K_STEP:  # the persistent step: every class of the step in one launch
        per_layer = sum(step_bytes_q8(cfg, batch, k, pos, gs) for k in (K_QKV, K_ATTN, K_WO, K_FFN_UP, K_FFN_DOWN))
        return (cfg.n_layers * per_layer + step_bytes_q8(cfg, batch, K_CLS, pos, gs)
                + step_bytes_q8(cfg, batch, K_ARGMAX, pos, gs))
    return step_bytes(cfg, batch, kclass, pos)
