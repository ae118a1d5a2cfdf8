#!/usr/bin/env python3
"""bench.py — decode tokens/s + achieved HBM GB/s on MI355X (BASELINE.json metric).

One "step" = one greedy decode token for the B sequences a GPU holds, running the whole
thaDNN forward (all layers, classifier, on-device argmax feeding the next token).
Default workload (the N=1 line): llama2-7B-shaped fp32 model, random-init synthetic weights,
one BOS-started greedy sequence per GPU over positions 0..K-1 (BASELINE.json configs[2]).
Other configs: --dtype int8 (configs[3], runq Q8_0 layout), --batch 8 (configs[4] per GPU),
--model 110m (configs[1]).
Multi-GPU: one process per GPU (torch.distributed.run); each rank decodes its own
independent sequences (weak scaling, no collective on the data path); rank 0 synthesises the
weights once and RCCL-broadcasts them over xGMI.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--model 7b|110m] [--dtype f32|int8] [--batch B]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

MODELS = {
    # (dim, hidden, layers, heads, kv_heads, vocab, seq_len), shared classifier, name
    "7b": ((4096, 11008, 32, 32, 32, 32000, 2048), 0, "llama2-7B"),
    "110m": ((768, 2048, 12, 12, 12, 32000, 1024), 1, "stories110M"),
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
SEED = 20240224


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=256)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--model", default="7b", choices=sorted(MODELS))
    ap.add_argument("--dtype", default="f32", choices=["f32", "int8"])
    ap.add_argument("--group-size", type=int, default=64, help="Q8_0 group size (int8)")
    ap.add_argument("--batch", type=int, default=1, help="sequences per GPU")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-nt", action="store_true")
    ap.add_argument("--splits", type=int, default=0)
    ap.add_argument("--no-persistent", action="store_true",
                    help="multi-launch step instead of the one-launch persistent step (batch 1)")
    ap.add_argument("--cpu-baseline-tokens", type=int, default=0,
                    help="greedy tokens the CPU baseline decodes (0: as many as fit --cpu-baseline-seconds)")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-aggregate", type=int, default=1 << 20,
                    help="max decoders of the aggregate CPU baseline (default: the host CPU share)")
    ap.add_argument("--skip-cpu", action="store_true")
    ap.add_argument("--prof-steps", type=int, default=16)
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL over xGMI) or gloo (CPU rehearsal)")
    ap.add_argument("--device-map", default="", help="comma list: local rank -> HIP device (rehearsals that "
                                                     "put several ranks on one GPU)")
    args = ap.parse_args()
    if args.prof_steps < 1:
        ap.error("--prof-steps must be >= 1 (the roofline object times the dominant kernel over them)")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.device_map:
        local = [int(v) for v in args.device_map.split(",")][local]

    import torch
    import torch.distributed as dist
    from __graft_entry__ import _pkg
    _pkg()
    from hip_llama_cpp_amd import thallama as tl
    from hip_llama_cpp_amd import dist as D

    if tl.device_count() < 1:
        raise SystemExit("bench.py: no HIP device")
    torch.cuda.set_device(local)
    tl.check(tl.lib().thallama_set_device(local))
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend=args.dist_backend)
    dev = f"cuda:{local}"

    cfg_t, shared, mname = MODELS[args.model]
    c = tl.Config.make(*cfg_t)
    B, K, W = args.batch, args.steps, args.warmup
    S, L = cfg_t[6], cfg_t[2]
    gs = args.group_size
    if K > S or W > S:
        raise SystemExit(f"--steps/--warmup must be <= seq_len {S}")
    q8 = args.dtype == "int8"

    # ---------------- weights: rank 0 synthesises (and for int8 quantises, export.py
    # semantics), then one RCCL broadcast of the packed weight image to every other rank
    t0 = time.perf_counter()
    n_floats = tl.lib().thallama_v0_payload_floats(tl.C.byref(c), shared)
    if not q8:
        image = torch.empty(n_floats, dtype=torch.float32, device=dev)
        if rank == 0:
            tl.check(tl.lib().thallama_synth_arena(tl.C.cast(tl.C.c_void_p(image.data_ptr()), tl.c_float_p),
                                                   tl.C.byref(c), shared, tl.C.c_uint64(SEED), None), "synth")
    else:
        nbytes = tl.lib().thallama_q8_payload_bytes(tl.C.byref(c), shared, gs)
        image = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        if rank == 0:
            fp = torch.empty(n_floats, dtype=torch.float32, device=dev)
            tl.check(tl.lib().thallama_synth_arena(tl.C.cast(tl.C.c_void_p(fp.data_ptr()), tl.c_float_p),
                                                   tl.C.byref(c), shared, tl.C.c_uint64(SEED), None), "synth")
            fpm = tl.DeviceModel(c, shared, arena_ptr=fp.data_ptr())
            tl.check(tl.lib().thallama_q8_quantize_model(tl.C.c_void_p(image.data_ptr()), tl.C.byref(fpm.w),
                                                         tl.C.byref(c), shared, gs, None), "q8 quantize")
            torch.cuda.synchronize()
            del fpm, fp
            torch.cuda.empty_cache()
    torch.cuda.synchronize()
    t_bcast = 0.0
    if world > 1:
        dist.barrier()
        tb = time.perf_counter()
        D.broadcast_arena(image, src=0)
        torch.cuda.synchronize()
        t_bcast = time.perf_counter() - tb
    t_init = time.perf_counter() - t0
    if q8:
        model = tl.DeviceModelQ8(c, shared, gs, payload_ptr=image.data_ptr())
    else:
        model = tl.DeviceModel(c, shared, arena_ptr=image.data_ptr())
    state = tl.DeviceState(c, B)
    dec = tl.Decoder(model, state)
    dec.set(tl.OPT_USE_GRAPH, 0 if args.no_graph else 1)
    if args.no_nt:
        dec.set(tl.OPT_NT_WEIGHTS, 0)
    if args.splits:
        dec.set(tl.OPT_ATTN_SPLITS, args.splits)
    if args.no_persistent:
        dec.set(tl.OPT_PERSISTENT, 0)
    persistent = dec.persistent()
    log(f"[rank {rank}] {mname} {args.dtype} B={B} init {t_init:.2f}s (broadcast {t_bcast:.2f}s)")

    tok0, pos0 = [1] * B, [0] * B  # BOS at position 0
    if W:
        dec.greedy(tok0, pos0, W, want_tokens=False, sync=True)

    def timed(n):
        """n greedy steps at positions 0..n-1, barrier + synchronize on both sides, max over ranks"""
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t = time.perf_counter()
        dec.greedy(tok0, pos0, n, want_tokens=False, sync=True)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        return D.max_over_ranks(time.perf_counter() - t, device=dev)

    # ---------------- timed region: K greedy steps at positions 0..K-1
    elapsed = timed(K)
    value = world * B * K / elapsed
    ms_step = elapsed / K * 1e3
    # the persistent step gives up (and the call re-runs on the multi-launch path) only if its
    # grid was not co-resident: re-read the path after the timed region, report any fallback
    persistent_after = dec.persistent()
    # BASELINE.json configs[2]: the 256-token decode (positions 0..255), timed in the same run
    # whatever --steps is (about 1.1 s at 7B fp32)
    HEAD = 256
    elapsed_h = elapsed if K == HEAD else (timed(HEAD) if S >= HEAD else None)
    persistent_after = persistent_after and dec.persistent()

    # ---------------- algorithmic bytes per step: weights once + KV rows at each position
    def launch_bytes(kclass, pos):
        return tl.step_bytes_q8(c, B, kclass, pos, gs) if q8 else tl.step_bytes(c, B, kclass, pos)

    layer_classes = (tl.K_QKV, tl.K_ATTN, tl.K_WO, tl.K_FFN_UP, tl.K_FFN_DOWN)
    step_bytes = sum(L * sum(launch_bytes(k, [p] * B) for k in layer_classes) + launch_bytes(tl.K_CLS, [p] * B)
                     + launch_bytes(tl.K_ARGMAX, [p] * B) for p in range(K)) / K
    step_gbs = step_bytes / (ms_step * 1e-3) / 1e9
    headline = None
    if elapsed_h is not None:
        hb = sum(L * sum(launch_bytes(k, [p] * B) for k in layer_classes) + launch_bytes(tl.K_CLS, [p] * B)
                 + launch_bytes(tl.K_ARGMAX, [p] * B) for p in range(HEAD)) / HEAD
        hms = elapsed_h / HEAD * 1e3
        headline = {"workload": f"{mname} {args.dtype} {HEAD}-token greedy decode (BASELINE.json configs), "
                                f"{B} seq/GPU, positions 0..{HEAD - 1}",
                    "value": round(world * B * HEAD / elapsed_h, 3), "unit": "tok/s", "ms_per_step": round(hms, 4),
                    "achieved_GBps": round(hb / (hms * 1e-3) / 1e9, 1),
                    "frac_of_peak": round(hb / (hms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                    "roofline_tok_s": round(HBM_PEAK_GBS * 1e9 / hb * B * world, 1)}

    # ---------------- greedy tokens vs the reference's own 256-step decode (tests/golden/
    # reference_long.json, generated from the reference's seq.cpp / runq.c by make_golden_long.py)
    golden = None
    try:
        with open(os.path.join(REPO, "tests", "golden", "reference_long.json")) as f:
            gcases = json.load(f)["cases"]
    except (OSError, ValueError, KeyError):
        gcases = []
    for gc in gcases:
        if tuple(gc["config"]) == tuple(cfg_t) and gc["shared"] == shared and gc["seed"] == SEED:
            want = gc["q8" if q8 else "fp32"]["tokens"]
            got = dec.greedy(tok0, pos0, len(want))  # [steps][B]
            prefix = min(next((i for i, (a, b) in enumerate(zip(want, got[:, b].tolist())) if a != b), len(want))
                         for b in range(B))
            golden = {"steps": len(want), "tokens_match": prefix == len(want), "match_prefix": prefix,
                      "source": "tests/golden/reference_long.json (" + ("runq.c" if q8 else "src/seq.cpp") +
                                " compiled from the reference, greedy from BOS)"}

    # ---------------- per-kernel-class timing: HIP events around every launch on the decoder's
    # stream, over an eager replay of the first prof-steps positions
    # (the persistent step is ONE launch: class "step"; the multi-launch kernels are profiled
    # as well for the breakdown, with the persistent path switched off)
    prof, prof_ml = {}, {}
    P = min(args.prof_steps, K)  # >= 1 (argument check): the roofline needs a measured kernel
    step_bytes_p = sum(launch_bytes(tl.K_STEP, [p] * B) for p in range(P)) / P

    def profile(into):
        dec.set(tl.OPT_PROFILE, 1)
        dec.prof_reset()
        dec.greedy(tok0, pos0, P, want_tokens=False, sync=True)
        for k, name in enumerate(tl.K_NAMES):
            ms, n = dec.prof(k)
            if n:
                into[name] = {"avg_us": 1e3 * ms / n, "launches": n}
                if k == tl.K_STEP:
                    into[name]["GBps"] = step_bytes_p / (into[name]["avg_us"] * 1e-6) / 1e9
                elif k not in (tl.K_ATTN, tl.K_ARGMAX):
                    into[name]["GBps"] = launch_bytes(k, [0] * B) / (into[name]["avg_us"] * 1e-6) / 1e9
        dec.set(tl.OPT_PROFILE, 0)

    if rank == 0:
        profile(prof)
        if persistent:
            dec.set(tl.OPT_PERSISTENT, 0)
            profile(prof_ml)
            dec.set(tl.OPT_PERSISTENT, 1)

    # ---------------- CPU baseline: the oracle (bit-exact seq.cpp / runq.c restatement), same model,
    # on this box's host cores (BASELINE.md CPU-baseline plan): (i) one decoder on one core, like
    # seq.cpp (int8: runq's OpenMP matmul over the cores we may use); (ii) aggregate: P
    # independent single-threaded decoders at once, one per core, over disjoint sequences
    cpu = None
    if rank == 0 and world == 1 and not args.skip_cpu and args.cpu_baseline_tokens >= 0:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle as O
        nproc = os.cpu_count() or 1
        allowed = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(nproc))
        # the GPU box grants a CPU share per GPU (OMP_NUM_THREADS there); the whole host's nproc
        # is reported beside it
        share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(allowed)
        P = max(1, min(share, len(allowed), args.cpu_aggregate))
        O.set_threads(P)  # weight synthesis (+ int8 quantisation) only
        ref = O.Model(cfg_t, shared, seed=SEED)
        if q8:
            ref.build_q8(gs)
            cores = P  # runq.c's matmul is OpenMP-parallel (runq.c:323-324)
            run = lambda m: ref.q8_greedy(1, 0, m)
        else:
            O.set_threads(1)
            cores = 1  # seq.cpp is single-threaded
            run = lambda m: ref.greedy(1, 0, m)
        n = args.cpu_baseline_tokens
        t1 = None
        if n <= 0:  # bounded sample: as many tokens as fit the time budget (one token calibrates), >= 8
            tc = time.perf_counter()
            run(1)
            t1 = time.perf_counter() - tc
            ref.reset_kv()
            n = max(8, min(K, S, int(args.cpu_baseline_seconds / max(t1, 1e-6))))
        tc = time.perf_counter()
        ctoks = run(n)
        tcpu = time.perf_counter() - tc
        t1 = t1 or tcpu / n
        gtoks = dec.greedy([1] * B, pos0, n)[:, 0].tolist()
        agg = None
        if not q8 and P > 1:
            m_agg = max(1, min(8, int(args.cpu_baseline_seconds / max(t1, 1e-6) / 2)))
            secs, atoks = ref.aggregate(P, m_agg, allowed[:P])
            agg = {"value": round(P * m_agg / secs, 4), "unit": "tok/s", "cores": P, "decoders": P,
                   "sample": f"{P} single-threaded decoders at once (one per core, pinned), decoder i greedy "
                             f"from token 1+i at pos 0, {m_agg} token(s) each",
                   "seconds": round(secs, 2), "decoder0_matches_single": atoks[0].tolist() == ctoks[:m_agg]}
        cpu = {"value": round(n / tcpu, 4), "unit": "tok/s", "cores": cores, "kind": "port",
               "sample": f"{n} greedy tokens (as many as fit ~{args.cpu_baseline_seconds:g} s, at least 8, unless "
                         f"--cpu-baseline-tokens) from BOS (pos 0..{n - 1}) of the same synthetic {mname} "
                         f"{args.dtype} model with oracle/oracle.c (bit-exact "
                         f"{'runq.c' if q8 else 'src/seq.cpp'} restatement), {cores} thread(s)",
               "host": {"nproc": nproc, "affinity_cpus": len(allowed), "cpu_share": share},
               "aggregate": agg,
               "tokens_match_gpu": ctoks == gtoks,
               "tokens_match_prefix": next((i for i, (a, b) in enumerate(zip(ctoks, gtoks)) if a != b),
                                           min(len(ctoks), len(gtoks)))}
        ref.close()

    if rank == 0:
        roof = None
        stp, ffn = prof.get("step"), prof.get("ffn_up")
        # HBM traffic of the same kernel from the committed rocprofv3 PMC passes (FETCH_SIZE and
        # WRITE_SIZE in separate runs, gfx950 FETCH_SIZE x2 correction): profiles/r02_pmc_traffic*.json
        pmc_file = "r02_pmc_traffic_int8.json" if q8 else "r02_pmc_traffic.json"
        pmc = {}
        try:
            with open(os.path.join(REPO, "profiles", pmc_file)) as f:
                pmc = json.load(f)["kernels"]
        except (OSError, ValueError, KeyError):
            pmc = {}

        def traffic_of(prefix):
            if mname != "llama2-7B" or B != 1:
                return None  # the committed PMC passes were taken on the 7B batch-1 workloads
            hits = [v["traffic_bytes"] for k, v in pmc.items() if k.startswith(prefix)]
            return round(hits[0]) if hits else None
        if stp:
            roof = {"bound": "hbm", "achieved": round(stp["GBps"], 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(stp["GBps"] / HBM_PEAK_GBS, 4),
                    "traffic": traffic_of("void tl::persistent_step_kernel<"),
                    "traffic_source": f"profiles/{pmc_file} (rocprofv3 --pmc, mean over the run's launches: "
                                      "positions 0..255, so ~0.1 GB more K/V than positions 0..15)",
                    "kernel": "persistent_step_kernel (the whole decode step, one launch)",
                    "bytes_per_launch": step_bytes_p, "avg_us": round(stp["avg_us"], 2),
                    "positions": f"0..{P - 1}"}
        elif ffn:
            roof = {"bound": "hbm", "achieved": round(ffn["GBps"], 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ffn["GBps"] / HBM_PEAK_GBS, 4),
                    "traffic": None if q8 else traffic_of("void tl::gemv_kernel<2, 1, 1, true, 4, false>"),
                    "traffic_source": f"profiles/{pmc_file} (rocprofv3 --pmc)",
                    "kernel": ("gemv_q8" if q8 else "gemv") + ("_mfma" if B >= 4 else "") + "_kernel<GM_SWIGLU> "
                              "(RMSNorm + W1/W3 + SwiGLU" + (", matrix cores)" if B >= 4 else ")"),
                    "bytes_per_launch": launch_bytes(tl.K_FFN_UP, [0] * B), "avg_us": round(ffn["avg_us"], 2)}
        out = {
            "metric": "decode tokens/sec (greedy, whole model) + achieved HBM GB/s fraction",
            "value": round(value, 3), "unit": "tok/s", "n_gpus": world, "steps": K, "warmup": W,
            "ms_per_step": round(ms_step, 4), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": args.dtype, "data": "synthetic (random-init weights, BOS-started greedy decode)",
            "config": {"workload": f"{mname} {args.dtype} greedy decode, {B} seq/GPU, positions 0..{K - 1}",
                       "model": mname, "global_batch": B * world, "seq_len": S, "parallelism": f"prompt-dp{world}"},
            "hbm": {"step_bytes": step_bytes, "achieved_GBps": round(step_gbs, 1),
                    "frac_of_peak": round(step_gbs / HBM_PEAK_GBS, 4),
                    "roofline_tok_s": round(HBM_PEAK_GBS * 1e9 / step_bytes * B * world, 1)},
            "roofline": roof,
            "step_path": "persistent" if persistent_after else "multi-launch",
            "persistent_fallback": bool(persistent and not persistent_after),
            "persistent_launch": (("cooperative" if tl.lib().thallama_persistent_cooperative() else "plain")
                                  if persistent else None),
            "headline": headline,
            "reference_tokens": golden,
            "kernels": {k: {kk: round(vv, 2) for kk, vv in v.items()} for k, v in prof.items()},
            "kernels_multilaunch": {k: {kk: round(vv, 2) for kk, vv in v.items()} for k, v in prof_ml.items()},
            "cpu_baseline": cpu,
            "init_s": round(t_init, 2), "broadcast_s": round(t_bcast, 2),
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
