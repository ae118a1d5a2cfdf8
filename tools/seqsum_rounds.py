#!/usr/bin/env python3
"""Cycles of the register-form wave seqsum (csrc/seqsum.hpp wave_seqsum_reg, thallama_seqsum_time)
against its repair-round count (a numpy emulation of the same algorithm): a least-squares fit
cycles = base + per_round * rounds, on squares of Gaussians (the RMSNorm input).  One JSON line."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def chain(a, s):
    s = np.float32(s)
    for v in a:
        s = np.float32(s + v)
    return s


def rounds_of(a, lanes=None):
    n = a.size
    ch = 4 * ((n + 255) // 256)
    pad = np.zeros(64 * ch, np.float32)
    pad[:n] = a
    ck = pad.reshape(64, ch)
    e = np.array([chain(ck[L], 0) for L in range(64)], np.float32)
    inc = e.astype(np.float64)
    start = np.zeros(64, np.float32)
    start[1:] = (np.cumsum(inc)[:-1]).astype(np.float32)
    e = np.array([chain(ck[L], start[L]) for L in range(64)], np.float32)
    inc = e.astype(np.float64) - start.astype(np.float64)
    incl = np.cumsum(inc)
    pre = incl - inc
    lo, slo, plo = 0, np.float32(0), 0.0
    for r in range(64):
        st = start.copy()
        st[lo + 1:] = (np.float64(slo) + (pre[lo + 1:] - plo)).astype(np.float32)
        if lo > 0:
            st[lo] = slo
        total = np.float32(np.float64(slo) + (incl[63] - plo)) if r else np.float32(incl[63])
        e = np.array([chain(ck[L], st[L]) for L in range(64)], np.float32)
        nxt = np.append(st[1:], total)
        bad = [L for L in range(lo, 64) if e[L] != nxt[L]]
        if not bad:
            return r + 1
        c = bad[0]
        if lanes is not None:
            lanes.append(c)
        if c == 63:
            return r + 1
        lo, slo, plo = c + 1, e[c], pre[c + 1]
        start = st
    return 64


def fail_lanes(a):
    out = []
    rounds_of(a, out)
    return out


def main():
    from __graft_entry__ import _pkg
    _pkg()
    from hip_llama_cpp_amd import thallama as tl
    tl.check(tl.lib().thallama_set_device(0))
    n, count = 4096, 64
    rng = np.random.default_rng(5)
    x = rng.standard_normal((count, n)).astype(np.float32)
    a = np.ascontiguousarray(x * x)
    din = tl.DevBuf.from_array(a)
    dout = tl.DevBuf(4 * count)
    dcyc = tl.DevBuf(8 * (count + 15))
    tl.check(tl.lib().thallama_seqsum_time(din.ptr, n, count, dout.ptr, dcyc.ptr), "seqsum_time")
    allraw = dcyc.download(np.int64)
    raw = allraw[:count]
    fails0 = allraw[count:count + 15].tolist()
    cyc = (raw & ((1 << 48) - 1)).astype(np.float64)
    rr = (raw >> 48).astype(np.float64)  # the device's own round count
    emu = np.array([rounds_of(a[i]) for i in range(8)], np.float64)
    A = np.stack([np.ones(count), rr], 1)
    (base, per), *_ = np.linalg.lstsq(A, cyc, rcond=None)
    print(json.dumps({"n": n, "arrays": count, "rounds_mean": float(rr.mean()), "rounds_max": int(rr.max()),
                      "cycles_median": float(np.median(cyc)), "fit_base_cycles": round(float(base), 1),
                      "fit_cycles_per_round": round(float(per), 1),
                      "device_rounds_first8": rr[:8].tolist(), "device_failing_lanes_array0": fails0,
                      "emulated_failing_lanes_array0": fail_lanes(a[0]), "emulated_rounds_first8": emu.tolist()}), flush=True)


if __name__ == "__main__":
    main()
