#!/usr/bin/env python3
"""Sweep launch variants of the streaming GEMV on the llama2-7B / stories110M shapes
(thallama_gemv_bench: weights rotate over >= 1.5 GiB, so each launch streams from HBM).
Prints one JSON object: per shape, per variant, us per launch and achieved GB/s."""
import ctypes as C
import itertools
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from __graft_entry__ import _pkg  # noqa: E402

_pkg()
from hip_llama_cpp_amd import thallama as tl  # noqa: E402

L = tl.lib()
L.thallama_gemv_bench.argtypes = [C.c_int] * 9 + [C.POINTER(C.c_double)]
L.thallama_gemv_bench.restype = C.c_int

SHAPES = {  # name: (mode, M, K, weight bytes)
    "7b_qkv": (3, 0, 4096, 3 * 4096 * 4096 * 4),
    "7b_wo": (1, 4096, 4096, 4096 * 4096 * 4),
    "7b_ffn_up": (2, 11008, 4096, 2 * 11008 * 4096 * 4),
    "7b_ffn_down": (1, 4096, 11008, 11008 * 4096 * 4),
    "7b_cls": (0, 32000, 4096, 32000 * 4096 * 4),
    "110m_qkv": (3, 0, 768, 3 * 768 * 768 * 4),
    "110m_ffn_up": (2, 2048, 768, 2 * 2048 * 768 * 4),
    "110m_ffn_down": (1, 768, 2048, 2048 * 768 * 4),
}


def run(mode, M, K, nb, ipw, waves, pf, nt, iters):
    us = C.c_double()
    rc = L.thallama_gemv_bench(mode, M, K, nb, ipw, waves, pf, nt, iters, C.byref(us))
    if rc:
        raise RuntimeError(f"gemv_bench rc={rc}")
    return us.value


def main():
    nbs = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "1").split(",")]
    shapes = sys.argv[2].split(",") if len(sys.argv) > 2 else list(SHAPES)
    out = {}
    for name in shapes:
        mode, M, K, wbytes = SHAPES[name]
        for nb in nbs:
            res = {}
            space = itertools.product([1, 2], [4, 8] if nb == 1 else [4], [0, 1], [0, 1])
            iters = max(20, int(2e9 / wbytes))
            for ipw, waves, pf, nt in space:
                us = run(mode, M, K, nb, ipw, waves, pf, nt, iters)
                res[f"ipw{ipw}_w{waves}_pf{pf}_nt{nt}"] = {"us": round(us, 2), "GBps": round(wbytes / us / 1e3, 1)}
            best = min(res, key=lambda k: res[k]["us"])
            out[f"{name}_nb{nb}"] = {"best": best, **res}
            print(name, nb, best, res[best], file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
