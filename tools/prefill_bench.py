"""Batched prefill vs token-by-token prompt processing.

For a prompt of P tokens on the llama2-7B shape (synthetic fp32 weights): the time of one
thallama_decoder_prefill call against P forced decode steps, and the prefill's matrix-core
rate (2 FLOP per weight per token, fp32 MFMA peak 157.3 TFLOP/s).

    python tools/prefill_bench.py [--model 7b|110m] [--p 16,64,128,512]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from __graft_entry__ import _pkg  # noqa: E402

MODELS = {"7b": (4096, 11008, 32, 32, 32, 32000, 2048), "110m": (768, 2048, 12, 12, 12, 32000, 1024)}
F32_MFMA_PEAK = 157.3  # TFLOP/s, MI355X_MICROARCH.md


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="7b", choices=sorted(MODELS))
    ap.add_argument("--p", default="16,64,128,512")
    args = ap.parse_args()
    _pkg()
    from hip_llama_cpp_amd import thallama as tl
    cfg = MODELS[args.model]
    c = tl.Config.make(*cfg)
    model = tl.DeviceModel(c, 0, seed=7)
    state = tl.DeviceState(c, 1)
    dec = tl.Decoder(model, state)
    dim, hid, L = cfg[0], cfg[1], cfg[2]
    layer_weights = 2 * dim * dim + 2 * dim * (dim * cfg[4] // cfg[3]) + 3 * dim * hid
    out = {"model": args.model, "rows": []}
    for P in [int(v) for v in args.p.split(",")]:
        toks = [(i * 7919) % cfg[5] for i in range(P)]
        dec.prefill(0, toks, 0)  # warm
        t0 = time.perf_counter()
        rc = dec.prefill(0, toks, 0)
        tp = time.perf_counter() - t0
        assert rc == 0
        t0 = time.perf_counter()
        for p in range(P):
            dec.forward([toks[p]], [p], want_logits=False)
        td = time.perf_counter() - t0
        flops = 2.0 * L * layer_weights * P
        row = {"P": P, "prefill_ms": round(tp * 1e3, 3), "decode_ms": round(td * 1e3, 3),
               "speedup": round(td / tp, 2), "prefill_tok_s": round(P / tp, 1),
               "tflops": round(flops / tp / 1e12, 2), "frac_f32_mfma_peak": round(flops / tp / 1e12 / F32_MFMA_PEAK, 4)}
        out["rows"].append(row)
        print(json.dumps(row), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
