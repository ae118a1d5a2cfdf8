#!/usr/bin/env python3
"""Diagnostics for the exact int8 persistent step: after one forward at pos 0..P, compare the last
layer's hand-off granules (q/k/v, attention output codes, SwiGLU output hb, residual x) with the
oracle's runq restatement (oracle.c) state.  python tools/debug_q8.py [cfg index] [positions]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
CFGS = [(256, 768, 2, 4, 4, 1024, 128), (512, 1536, 2, 4, 2, 1024, 512), (512, 1536, 1, 4, 4, 1024, 64)]


def main():
    ci = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    P = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    cfg = CFGS[ci]
    from __graft_entry__ import _pkg
    _pkg()
    from hip_llama_cpp_amd import thallama as tl
    import oracle as O
    import ctypes as C
    tl.check(tl.lib().thallama_set_device(0))
    c = tl.Config.make(*cfg)
    m = tl.DeviceModel(c, 0, seed=31)
    q = tl.DeviceModelQ8(c, 0, 64, from_model=m)
    st = tl.DeviceState(c, 1)
    dec = tl.Decoder(q, st)
    ref = O.Model(cfg, 0, seed=31)
    ref.build_q8(64)
    L = O.lib()
    dim, hid, kvd = cfg[0], cfg[1], cfg[0] * cfg[4] // cfg[3]
    toks = np.random.default_rng(5).integers(0, cfg[5], P)
    for p, t in enumerate(toks):
        got = dec.forward([int(t)], [p])[0]
        want = ref.q8_forward(int(t), p)
        n = tl.lib().thallama_decoder_granules(dec.h, None, 0)
        g = np.zeros(n, np.uint64)
        tl.lib().thallama_decoder_granules(dec.h, g.ctypes.data_as(C.POINTER(C.c_ulonglong)), n)
        vals = (g & 0xFFFFFFFF).astype(np.uint32).view(np.float32)
        gx, gxb, ghb = vals[:dim], vals[dim:2 * dim], vals[2 * dim:2 * dim + hid]
        gq = vals[2 * dim + hid:2 * dim + hid + dim]
        gk = vals[3 * dim + hid:3 * dim + hid + kvd]
        gv = vals[3 * dim + hid + kvd:3 * dim + hid + 2 * kvd]
        print(f"pos {p}: logits differ {np.sum(got.view(np.uint32) != want.view(np.uint32))} of {len(got)}")
        for nm, gpu_v, wh, n_ in (("q", gq, 5, dim), ("k", gk, 6, kvd), ("v", gv, 7, kvd), ("hb", ghb, 3, hid)):
            rv = ref.buf(wh, n_)
            d = gpu_v.view(np.uint32) != rv.view(np.uint32)
            print(f"  {nm:3s} differ {int(d.sum()):5d} of {n_}  max|d| {np.max(np.abs(gpu_v - rv)):.3g}")


if __name__ == "__main__" and len(sys.argv) <= 3:
    main()


def norm_check(ci=2, P=2):
    """The layer-0 QKV norm sum (block 0, trace slot 11) against the CPU chain of the squares of
    the dequantized embedding row."""
    cfg = CFGS[ci]
    from __graft_entry__ import _pkg
    _pkg()
    from hip_llama_cpp_amd import thallama as tl
    import oracle as O
    tl.check(tl.lib().thallama_set_device(0))
    c = tl.Config.make(*cfg)
    m = tl.DeviceModel(c, 0, seed=31)
    q = tl.DeviceModelQ8(c, 0, 64, from_model=m)
    st = tl.DeviceState(c, 1)
    dec = tl.Decoder(q, st)
    dec.ptrace(True)
    ref = O.Model(cfg, 0, seed=31)
    ref.build_q8(64)
    pay = ref.q8_payload()
    dim, V, L = cfg[0], cfg[5], cfg[2]
    off = 4 * (2 * L * dim + dim)
    qe = pay[off:off + V * dim].view(np.int8)
    se = pay[off + V * dim:off + V * dim + 4 * (V * dim // 64)].view(np.float32)
    toks = np.random.default_rng(5).integers(0, cfg[5], P)
    nph = 5 * L + 1
    for p, t in enumerate(toks):
        dec.forward([int(t)], [p])
        tr = dec.ptrace(False).reshape(-1, nph, 12)
        row = (qe[t * dim:(t + 1) * dim].astype(np.float32) * np.repeat(se[t * dim // 64:(t + 1) * dim // 64], 64)).astype(np.float32)
        s = np.float32(0)
        for v in row:
            s = np.float32(s + np.float32(v * v))
        g = int(tr[0, 0, 11])
        gsum = np.uint32(g & 0xFFFFFFFF).view(np.float32)
        print(f"pos {p} tok {t}: layer-0 norm sum gpu {gsum!r} cpu {s!r} equal {gsum == s}; blocks agree "
              f"{len(set(int(v) for v in tr[:, 0, 11]))}")


if __name__ == "__main__" and len(sys.argv) > 3:
    norm_check(int(sys.argv[1]), int(sys.argv[2]))
