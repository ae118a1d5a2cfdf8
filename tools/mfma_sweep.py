#!/usr/bin/env python3
"""Time the default-dispatch GEMV (matrix-core kernel at nb >= 4) on the llama2-7B shapes
via thallama_gemv_bench(ipw=0); THALLAMA_MFMA_* env variables select kernel variants.
    python tools/mfma_sweep.py [nbs] [shapes]"""
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
from gemv_sweep import L, SHAPES  # noqa: E402


def main():
    nbs = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "4,8,16").split(",")]
    shapes = sys.argv[2].split(",") if len(sys.argv) > 2 else [s for s in SHAPES if s.startswith("7b")]
    tag = {k: v for k, v in os.environ.items() if k.startswith("THALLAMA_MFMA")}
    out = {}
    for name in shapes:
        mode, M, K, wbytes = SHAPES[name]
        iters = max(20, int(2e9 / wbytes))
        for nb in nbs:
            us = C.c_double()
            rc = L.thallama_gemv_bench(mode, M, K, nb, 0, 4, 0, 1, iters, C.byref(us))
            if rc:
                raise RuntimeError(f"gemv_bench rc={rc}")
            out[f"{name}_nb{nb}"] = {"us": round(us.value, 2), "GBps": round(wbytes / us.value / 1e3, 1)}
    print(json.dumps({"env": tag, "res": out}), flush=True)


if __name__ == "__main__":
    main()
