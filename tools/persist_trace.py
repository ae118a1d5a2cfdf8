"""Timeline of the persistent decode step (hip_llama.cpp_amd/csrc/persist.hip).

Wave 0 of every block stamps the 100-MHz real-time clock at: phase start (grid barrier exit),
input staged, all slots reduced, epilogue drained.  This prints, per phase kind averaged over
layers (us): staging, streaming (staged -> reduced, the slowest block), epilogue, the barrier
(last arrival -> first exit) and the whole phase, plus the per-phase weight bytes and the
rate they imply.

    python tools/persist_trace.py --model 7b --steps 4
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from __graft_entry__ import _pkg  # noqa: E402

MODELS = {"7b": (4096, 11008, 32, 32, 32, 32000, 2048), "110m": (768, 2048, 12, 12, 12, 32000, 1024)}
KINDS = ["qkv", "attn", "wo", "ffn_up", "ffn_down"]


def ksplit_report(t, nph, G, wbytes, args):
    """Per phase kind (medians over blocks, then over layers; us): staging (start -> slice staged),
    first slot (staged -> streaming wave 1's first slot consumed), sweep (staged -> wave 1's last
    slot), sweep barrier (staged -> every streaming wave done), reduce (barrier -> reduce done), the
    phase (start -> the next phase's start, median block) and the weight rate it implies."""
    print(f"ksplit B=8: {G} blocks, step {t[:, -1, 5].max() - t[:, 0, 0].min():.1f} us")
    print(f"{'kind':9s}{'phase':>8s}{'stage':>8s}{'slot0':>8s}{'sweep':>8s}{'swbar':>8s}{'prep':>8s}{'reduce':>8s}{'GB/s':>8s}")
    out = {}
    for kind, k in (("qkv", 0), ("attn", 1), ("wo", 2), ("ffn_up", 3), ("ffn_down", 4), ("cls", nph - 1)):
        phs = [k] if kind == "cls" else list(range(k, nph - 1, 5))
        med = lambda a, b: float(np.median([np.median(t[:, ph, a] - t[:, ph, b]) for ph in phs]))  # noqa: E731
        if kind == "cls":
            phase = float(np.median(t[:, -1, 5] - t[:, -1, 0]))
        else:
            phase = float(np.median([np.median(t[:, ph + 1, 0] - t[:, ph, 0]) for ph in phs]))
        if kind == "attn":
            print(f"{kind:9s}{phase:8.2f}   units done {med(3, 0):.2f}")
            out[kind] = {"phase": phase, "units_done": med(3, 0)}
            continue
        row = {"phase": phase, "stage": med(1, 0), "slot0": med(6, 1), "sweep": med(3, 1), "sweep_barrier": med(4, 1),
               "prep": med(2, 1), "reduce": med(5, 4)}
        row["GBps"] = wbytes[kind] / (phase * 1e-6) / 1e9
        print(f"{kind:9s}" + "".join(f"{row[x]:8.2f}" for x in ("phase", "stage", "slot0", "sweep", "sweep_barrier", "prep", "reduce"))
              + f"{row['GBps']:8.0f}")
        out[kind] = row
    # spread of the sweep over blocks (the reduce waits for the row group's slowest K slice)
    bi = np.arange(G)
    kg = (bi >> 3) & 7
    for kind, k in (("qkv", 0), ("wo", 2), ("ffn_up", 3), ("ffn_down", 4)):
        sw = np.mean([t[:, ph, 3] - t[:, ph, 1] for ph in range(k, nph - 1, 5)], axis=0)
        print(f"{kind:9s} sweep per block: min {sw.min():.2f} med {np.median(sw):.2f} max {sw.max():.2f}; by XCD "
              + " ".join(f"{sw[bi % 8 == x].mean():.1f}" for x in range(8)) + "; by K group "
              + " ".join(f"{sw[kg == x].mean():.1f}" for x in range(8)))
        out[kind + "_sweep_by_xcd"] = [float(sw[bi % 8 == x].mean()) for x in range(8)]
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="7b", choices=sorted(MODELS))
    ap.add_argument("--pos", type=int, default=8, help="position of the traced step")
    ap.add_argument("--json", default="")
    ap.add_argument("--npz", default="", help="also save the raw stamps [grid][phase][slot] (100-MHz ticks)")
    ap.add_argument("--dtype", default="f32", choices=["f32", "int8"])
    ap.add_argument("--batch", type=int, default=1, help="sequences (2..8: the batched step, persist_b.hip)")
    args = ap.parse_args()
    _pkg()
    from hip_llama_cpp_amd import thallama as tl
    cfg = MODELS[args.model]
    c = tl.Config.make(*cfg)
    model = tl.DeviceModel(c, 0, seed=7)
    if args.dtype == "int8":
        model = tl.DeviceModelQ8(c, 0, 64, from_model=model)
    B = args.batch
    state = tl.DeviceState(c, B)
    dec = tl.Decoder(model, state)
    if B > 1:
        dec.set(tl.OPT_PERSISTENT, 1)  # (opt-in at 5..8 sequences; at 8 the K-split step)
    assert dec.persistent()
    dec.greedy([1] * B, [0] * B, args.pos, want_tokens=False)
    dec.ptrace(True)
    dec.greedy([1] * B, [args.pos] * B, 1, want_tokens=False)
    t = dec.ptrace(False).astype(np.int64)
    L = cfg[2]
    nph = 5 * L + 1
    NSL = 16  # kTraceSlots (persist.hpp)
    G = t.size // (nph * NSL)
    t = t.reshape(G, nph, NSL)
    raw = t.copy()  # (slot 13 holds a count, not a time)
    if args.npz:
        np.savez_compressed(args.npz, stamps=raw)
    t = (t - t[:, 0, 0].min()) * 0.01  # us
    dim, hid, kvd, V = cfg[0], cfg[1], cfg[0] * cfg[4] // cfg[3], cfg[5]
    esz = 4 if args.dtype == "f32" else 1 + 4 / 64  # int8 + one fp32 scale per 64
    wbytes = {k: v * esz for k, v in {"qkv": dim * (dim + 2 * kvd), "attn": 0, "wo": dim * dim, "ffn_up": 2 * dim * hid,
                                       "ffn_down": dim * hid, "cls": dim * V}.items()}
    if B == 8 and dec.ksplit():  # the K-split step (persist_k.hip): its own slots, see TRACE_K there
        ksplit_report(t, nph, G, wbytes, args)
        return
    if B > 1:  # the batched step (persist_b.hip): its own slots, see TRACE_B there
        print(f"{args.model} B={B}: {G} blocks, step {t[:, -1, 3].max() - t[:, 0, 0].min():.1f} us")
        print(f"{'kind':9s}{'phase':>8s}{'stage0':>8s}{'slot0':>8s}{'passes':>40s}{'epi':>7s}{'GB/s':>8s}")
        out = {}
        for kind, k in (("qkv", 0), ("attn", 1), ("wo", 2), ("ffn_up", 3), ("ffn_down", 4), ("cls", nph - 1)):
            phs = [k] if kind == "cls" else list(range(k, nph - 1, 5))
            phase = np.median([t[:, ph + 1, 0].max() - t[:, ph, 0].max() for ph in phs if ph + 1 < nph]) \
                if kind != "cls" else float(t[:, -1, 3].max() - t[:, -1, 0].max())
            if kind == "attn":
                done = np.median([np.median(t[:, ph, 3] - t[:, ph, 0]) for ph in phs])
                print(f"{kind:9s}{phase:8.2f}   units done (median) {done:.2f}")
                out[kind] = {"phase": float(phase)}
                continue
            stage0 = np.median([np.median(t[:, ph, 1] - t[:, ph, 0]) for ph in phs])
            slot0 = np.median([np.median(t[:, ph, 4] - t[:, ph, 1]) for ph in phs])
            passes = []
            for c in range(6):  # pass q's end is slot 8 + q (stamped only for the passes there were)
                if not all((raw[:, ph, 8 + c] > raw[:, ph, 0]).all() for ph in phs):
                    break
                prev = 1 if c == 0 else 8 + c - 1
                passes.append(float(np.median([np.median(t[:, ph, 8 + c] - t[:, ph, prev]) for ph in phs])))
            epi = np.median([np.median(t[:, ph, 3] - t[:, ph, 2]) for ph in phs])
            med = lambda a, b: float(np.median([np.median(t[:, ph, a] - t[:, ph, b]) for ph in phs]))  # noqa: E731
            # staging of pass 0, from the phase start: control wave first batch in / swept, streaming
            # wave 1 first batch in / swept
            stg = [med(5, 0), med(6, 0), med(14, 0), med(15, 0)]
            print(f"{'':9s} staging c.first {stg[0]:.2f} c.swept {stg[1]:.2f}  s.first {stg[2]:.2f} s.swept {stg[3]:.2f}")
            gbs = wbytes[kind] / (phase * 1e-6) / 1e9
            print(f"{kind:9s}{phase:8.2f}{stage0:8.2f}{slot0:8.2f}{' '.join(f'{v:5.2f}' for v in passes):>40s}"
                  f"{epi:7.2f}{gbs:8.0f}")
            out[kind] = {"phase": float(phase), "stage0": float(stage0), "slot0": float(slot0), "passes": passes,
                         "epilogue": float(epi), "GBps": float(gbs)}
        if args.json:
            with open(args.json, "w") as f:
                json.dump(out, f, indent=1)
        return
    rows = {}
    for ph in range(nph):
        kind = "cls" if ph == nph - 1 else KINDS[ph % 5]
        s0 = t[:, ph, 0]
        end = t[:, ph, 3]
        nxt = t[:, ph + 1, 0] if ph + 1 < nph else None
        r = {"start_skew": s0.max() - s0.min(), "epi_max": (end - t[:, ph, 2]).max() if kind != "attn" else 0.0}
        if kind != "attn":
            r["stage"] = np.median(t[:, ph, 1] - s0)
            r["stream_max"] = (t[:, ph, 2] - t[:, ph, 1]).max()
        if nxt is not None:
            r["barrier"] = nxt.min() - end.max()
            r["phase"] = nxt.max() - s0.max()
        rows.setdefault(kind, []).append(r)
    out = {}
    print(f"{args.model}: {G} blocks, step {t[:, -1, 3].max() - t[:, 0, 0].min():.1f} us")
    print(f"{'kind':9s}{'phase':>8s}{'stage':>8s}{'stream':>8s}{'epi':>7s}{'barrier':>8s}{'skew':>7s}{'GB/s':>8s}")
    for kind, rs in rows.items():
        avg = {k: float(np.mean([r[k] for r in rs if k in r])) for k in rs[0]}
        ph_us = avg.get("phase", float("nan"))
        gbs = wbytes[kind] / (ph_us * 1e-6) / 1e9 if kind != "attn" and ph_us == ph_us else 0.0
        print(f"{kind:9s}{ph_us:8.2f}{avg.get('stage', 0):8.2f}{avg.get('stream_max', 0):8.2f}"
              f"{avg['epi_max']:7.2f}{avg.get('barrier', 0):8.2f}{avg['start_skew']:7.2f}{gbs:8.0f}")
        out[kind] = avg
    # where the skew comes from: per-block streaming time of the big phases, by blockIdx % 8
    # (blocks b and b+8 share an XCD under round-robin dispatch) and over the grid
    for kind, k in (("ffn_up", 3), ("qkv", 0), ("ffn_down", 4)):
        st = np.mean([t[:, ph, 2] - t[:, ph, 1] for ph in range(k, nph - 1, 5)], axis=0)
        byx = [float(np.mean(st[x::8])) for x in range(8)]
        print(f"{kind:9s} stream per block: min {st.min():.2f} med {np.median(st):.2f} max {st.max():.2f}; "
              f"by blockIdx%8: " + " ".join(f"{v:.1f}" for v in byx))
        out[kind + "_stream_by_xcd"] = byx
    # streaming wave 0 of every block: staged -> first slot consumed (waiting for data that was
    # prefetched during the hand-off), first -> last slot, issue of the next phase's slots
    print(f"{'kind':9s}{'first':>8s}{'rest':>8s}{'issue':>8s}   (streaming wave 0, medians over blocks, us)")
    for kind, k in (("qkv", 0), ("wo", 2), ("ffn_up", 3), ("ffn_down", 4)):
        phs = list(range(k, nph - 1, 5))
        f = np.median([t[:, ph, 5] - t[:, ph, 4] for ph in phs])
        r = np.median([t[:, ph, 6] - t[:, ph, 5] for ph in phs])
        i = np.median([t[:, ph, 7] - t[:, ph, 6] for ph in phs])
        print(f"{kind:9s}{f:8.2f}{r:8.2f}{i:8.2f}")
        out[kind + "_stream_wave"] = {"first": float(f), "rest": float(r), "issue": float(i)}
    # inside the staging (us after the control wave's phase start, medians over blocks and layers):
    # control wave gathered / normalised / staged; streaming wave 0 gathered / staged
    print(f"{'kind':9s}{'c.gath':>8s}{'c.norm':>8s}{'c.stgd':>8s}{'s.gath':>8s}{'s.stgd':>8s}   (staging, from phase start)")
    for kind, k in (("qkv", 0), ("wo", 2), ("ffn_up", 3), ("ffn_down", 4)):
        phs = list(range(k, nph - 1, 5))
        med = lambda a, b: float(np.median([t[:, ph, a] - t[:, ph, b] for ph in phs]))
        row = [med(8, 0), med(9, 0), med(1, 0), med(10, 0), med(4, 0)]
        print(f"{kind:9s}" + "".join(f"{v:8.2f}" for v in row))
        out[kind + "_staging"] = row
    # attention phase on the blocks that run a unit (single-chunk contexts): q granule ready,
    # (int8: every score of the head gathered; fp32: k/v granules ready), output computed, unit
    # done (us after the phase start)
    att = [ph for ph in range(1, nph - 1, 5)]
    a = np.stack([t[:, ph, :] for ph in att])  # [layers][G][slots]
    # live: blocks whose unit stamped its granules in (fp32) / its publish (int8); a unit that is
    # not its head's last split publishes nothing (slot 10 stays from an earlier phase)
    live = (a[:, :, 8] > a[:, :, 0]) if args.dtype == "f32" else (a[:, :, 10] > a[:, :, 0])
    if live.any():
        rel = lambda k: float(np.median((a[:, :, k] - a[:, :, 0])[live & (a[:, :, k] > a[:, :, 0])]))
        if args.dtype == "int8":
            print(f"attention units ({int(live.sum() / len(att))} per layer): q {rel(8):.2f}  scores/kv {rel(9):.2f}  "
                  f"summed {rel(11):.2f}  computed {rel(10):.2f}  done {rel(3):.2f} us after phase start")
        else:  # attn_unit_win (fp32, batch 1): granules in, cached keys folded, computed, published
            print(f"attention units ({int(live.sum() / len(att))} per layer): q/k/v in {rel(8):.2f}  first K rows in "
                  f"{rel(12):.2f}  first scores {rel(13):.2f}  cached keys {rel(9):.2f}  computed {rel(11):.2f}  "
                  f"published {rel(10):.2f}  done {rel(3):.2f} us after phase start")
        # the hand-offs around attention, per layer (median over layers): the last QKV epilogue's end,
        # the last head published, and the Wo staging's gather, relative to the median attention start
        qkv_end = np.stack([t[:, ph - 1, 3].max() for ph in att])
        a0 = np.stack([np.median(t[:, ph, 0]) for ph in att])
        pubm = a[:, :, 10] > a[:, :, 0]  # blocks whose unit published a head in this phase
        pub = np.stack([(a[i, :, 10][pubm[i]]).max() if pubm[i].any() else np.nan for i in range(len(att))])
        wo_g = np.stack([np.median(t[:, ph + 1, 8]) for ph in att])
        print(f"around attention (median over layers, us from the median attention start): last QKV epilogue "
              f"{np.nanmedian(qkv_end - a0):.2f}  last head published {np.nanmedian(pub - a0):.2f}  "
              f"Wo gather (median block) {np.nanmedian(wo_g - a0):.2f}")
    # int8: repair rounds of the exact norm sums (slot 13, seqsum.hpp)
    if args.dtype == "int8":
        print("norm-sum repair rounds (mean / max over blocks and layers): " + "  ".join(
            f"{kind} {np.mean([raw[:, ph, 13] for ph in range(k, nph - 1, 5)]):.2f}/"
            f"{np.max([raw[:, ph, 13] for ph in range(k, nph - 1, 5)])}"
            for kind, k in (("qkv", 0), ("ffn_up", 3))))
    # epilogue: row values computed (slot 12, the control wave's first item) after the epilogue start
    print("epilogue row values us after its start (median): " + "  ".join(
        f"{kind} {np.median([np.median(t[:, ph, 12] - t[:, ph, 2]) for ph in range(k, nph - 1, 5)]):.2f}"
        for kind, k in (("qkv", 0), ("wo", 2), ("ffn_up", 3), ("ffn_down", 4))))
    # epilogue (all slots reduced -> epilogue issued), median and max over blocks
    print("epilogue us (median / max over blocks): " + "  ".join(
        f"{kind} {np.median([np.median(t[:, ph, 3] - t[:, ph, 2]) for ph in range(k, nph - 1, 5)]):.2f}/"
        f"{np.mean([np.max(t[:, ph, 3] - t[:, ph, 2]) for ph in range(k, nph - 1, 5)]):.2f}"
        for kind, k in (("qkv", 0), ("wo", 2), ("ffn_up", 3), ("ffn_down", 4))))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
