"""ctypes binding of lib/libthallama_host.so (include/thallama_host.h): the reference CLI's host
side — BPE tokenizer, sampler, test-mode request files and scheduler (src/llama.cpp:35-505,
891-1083).  CPU only; used by tests/ and by nothing on the GPU path."""
import ctypes as C
import os

import numpy as np

_LIB = None
HERE = os.path.dirname(os.path.abspath(__file__))
STEP_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int),
                      C.POINTER(C.c_float))
PREFILL_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_int), C.c_int, C.c_int)
ARGMAX_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int),
                        C.POINTER(C.c_int))


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "lib", "libthallama_host.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: build with `make -C hip_llama.cpp_amd`")
        L = C.CDLL(path)
        VP, I, F, S = C.c_void_p, C.c_int, C.c_float, C.c_char_p
        IP, FP, ULL = C.POINTER(C.c_int), C.POINTER(C.c_float), C.c_ulonglong
        sig = {
            "thallama_tokenizer_load": (VP, [S, I]),
            "thallama_tokenizer_free": (None, [VP]),
            "thallama_tokenizer_max_token_length": (I, [VP]),
            "thallama_tokenizer_piece": (S, [VP, I]),
            "thallama_tokenizer_score": (F, [VP, I]),
            "thallama_tokenizer_encode": (I, [VP, S, I, I, IP, IP]),
            "thallama_tokenizer_decode": (C.c_void_p, [VP, I, I]),
            "thallama_piece_is_safe": (I, [C.c_void_p]),
            "thallama_sampler_create": (VP, [I, F, F, ULL]),
            "thallama_sampler_free": (None, [VP]),
            "thallama_sample": (I, [VP, FP]),
            "thallama_sampler_rng_state": (ULL, [VP]),
            "thallama_sample_argmax": (I, [FP, I]),
            "thallama_sample_mult": (I, [FP, I, F]),
            "thallama_sample_topp": (I, [FP, I, F, F]),
            "thallama_random_u32": (C.c_uint, [C.POINTER(ULL)]),
            "thallama_random_f32": (F, [C.POINTER(ULL)]),
            "thallama_softmax": (None, [FP, I]),
            "thallama_requests_read": (VP, [S, I, I]),
            "thallama_requests_set_sampling": (None, [VP, C.c_float, C.c_float]),
            "thallama_requests_free": (None, [VP]),
            "thallama_requests_count": (I, [VP]),
            "thallama_requests_prompt": (S, [VP, I]),
            "thallama_requests_output": (S, [VP, I]),
            "thallama_requests_write": (I, [VP, S]),
            "thallama_serve_requests": (I, [VP, S, I, I, I, STEP_FN, VP, C.POINTER(C.c_longlong)]),
            "thallama_serve_requests_prefill": (I, [VP, S, I, I, I, STEP_FN, PREFILL_FN, VP,
                                                    C.POINTER(C.c_longlong)]),
            "thallama_serve_requests_greedy": (I, [VP, S, I, I, I, STEP_FN, ARGMAX_FN, PREFILL_FN, VP,
                                                   C.POINTER(C.c_longlong)]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype, fn.argtypes = res, args
        _LIB = L
    return _LIB


def fp(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


class Tokenizer:
    def __init__(self, path, vocab_size=32000):
        self.h = lib().thallama_tokenizer_load(path.encode(), vocab_size)
        if not self.h:
            raise RuntimeError(f"cannot load tokenizer {path}")
        self.vocab_size = vocab_size

    def encode(self, text, bos=True, eos=False):
        raw = text.encode() if isinstance(text, str) else text
        buf = (C.c_int * (len(raw) + 3))()
        n = C.c_int(0)
        lib().thallama_tokenizer_encode(self.h, raw, int(bos), int(eos), buf, C.byref(n))
        return list(buf[:n.value])

    def decode(self, prev, token):
        """The piece as bytes (raw-byte pieces included)."""
        return C.string_at(lib().thallama_tokenizer_decode(self.h, prev, token))

    def is_safe(self, prev, token):
        return bool(lib().thallama_piece_is_safe(lib().thallama_tokenizer_decode(self.h, prev, token)))

    @property
    def max_token_length(self):
        return lib().thallama_tokenizer_max_token_length(self.h)

    def close(self):
        if self.h:
            lib().thallama_tokenizer_free(self.h)
            self.h = None

    def __del__(self):
        self.close()


class Sampler:
    def __init__(self, vocab_size, temperature, topp, seed):
        self.h = lib().thallama_sampler_create(vocab_size, temperature, topp, seed)

    def sample(self, logits):
        """Like the reference, rescales/softmaxes `logits` (float32 array) in place."""
        return lib().thallama_sample(self.h, fp(logits))

    @property
    def rng(self):
        return lib().thallama_sampler_rng_state(self.h)

    def __del__(self):
        if self.h:
            lib().thallama_sampler_free(self.h)
            self.h = None


class Requests:
    def __init__(self, path, max_token_len, max_seq_len):
        self.h = lib().thallama_requests_read(path.encode(), max_token_len, max_seq_len)
        if not self.h:
            raise RuntimeError(f"cannot read {path}")

    def __len__(self):
        return lib().thallama_requests_count(self.h)

    def set_sampling(self, temperature, topp=0.9):
        """temperature 0 = greedy; default is the reference's 1.0 / 0.9."""
        lib().thallama_requests_set_sampling(self.h, temperature, topp)

    def prompt(self, i):
        return lib().thallama_requests_prompt(self.h, i)

    def output(self, i):
        return lib().thallama_requests_output(self.h, i)

    def write(self, path):
        if lib().thallama_requests_write(self.h, path.encode()):
            raise RuntimeError(f"cannot write {path}")

    def serve(self, tokenizer_path, vocab_size, n_workers, batch, step, prefill=None):
        """step(worker, tokens[batch], pos[batch]) -> logits [batch, vocab] float32;
        prefill(worker, slot, tokens[n], pos0) -> 0 (done) / 1 (not supported), optional."""
        def cb(_ctx, worker, b, tok, pos, out):
            try:
                lg = step(worker, np.ctypeslib.as_array(tok, (b,)).copy(), np.ctypeslib.as_array(pos, (b,)).copy())
                np.ctypeslib.as_array(out, (b * vocab_size,))[:] = np.ascontiguousarray(lg, np.float32).ravel()
                return 0
            except Exception:  # noqa: BLE001 — surfaced as a nonzero status
                import traceback
                traceback.print_exc()
                return 7

        def pcb(_ctx, worker, slot, tok, n, pos0):
            try:
                return int(prefill(worker, slot, np.ctypeslib.as_array(tok, (n,)).copy(), pos0))
            except Exception:  # noqa: BLE001
                import traceback
                traceback.print_exc()
                return -7
        fn = STEP_FN(cb)
        gen = C.c_longlong(0)
        if prefill is None:
            st = lib().thallama_serve_requests(self.h, tokenizer_path.encode(), vocab_size, n_workers, batch, fn,
                                              None, C.byref(gen))
        else:
            pfn = PREFILL_FN(pcb)
            st = lib().thallama_serve_requests_prefill(self.h, tokenizer_path.encode(), vocab_size, n_workers,
                                                      batch, fn, pfn, None, C.byref(gen))
        if st:
            raise RuntimeError(f"serve_requests failed: {st}")
        return gen.value

    def serve_native(self, tokenizer_path, vocab_size, n_workers, batch, step_addr, prefill_addr, ctx,
                     argmax_addr=0):
        """Same scheduler driven by native callbacks (addresses of a thallama_step_fn, an optional
        thallama_prefill_fn and an optional thallama_argmax_step_fn used for greedy sampling, e.g.
        libthallama's thallama_decoder_step_cb / _prefill_cb / _argmax_cb with ctx = the decoder):
        no Python on the per-step path."""
        gen = C.c_longlong(0)
        st = lib().thallama_serve_requests_greedy(self.h, tokenizer_path.encode(), vocab_size, n_workers, batch,
                                                 STEP_FN(step_addr) if step_addr else STEP_FN(),
                                                 ARGMAX_FN(argmax_addr) if argmax_addr else ARGMAX_FN(),
                                                 PREFILL_FN(prefill_addr) if prefill_addr else PREFILL_FN(),
                                                 C.c_void_p(ctx), C.byref(gen))
        if st:
            raise RuntimeError(f"serve_requests failed: {st}")
        return gen.value

    def __del__(self):
        if getattr(self, "h", None):
            lib().thallama_requests_free(self.h)
            self.h = None
