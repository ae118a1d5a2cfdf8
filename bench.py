#!/usr/bin/env python3
"""bench.py — decode tokens/s + achieved HBM GB/s on MI355X (BASELINE.json metric).

Workloads (one "step" = one pass of the hot path over one batch of synthetic input):

* ``decode`` (default at N = 1; BASELINE.json configs[2], or [3] with --dtype int8, [1] with
  --model 110m): a step is one 256-token greedy decode (--decode-len) of the B sequences a GPU
  holds, BOS-started at position 0 and run to position 255 — every step the whole thaDNN forward
  (all layers, classifier, on-device argmax feeding the next token).  value = tokens/s over the
  K timed decodes.  The line also carries the long-context tail (positions 1792..2047 of a
  2048-token decode, the length the reference's test mode runs to), the 1-GPU point of the
  request workload below, the dominant kernel's roofline and the CPU baseline.
* ``cli`` (default at N > 1; BASELINE.json configs[4]): the drop-in's own multi-GPU path — the
  CLI build/apps/llama in test mode (src/llama.cpp:891-1083: one host thread per GPU, weights
  uploaded once and RCCL-broadcast over xGMI) over the reference's assets/in/gen_in_64.txt
  prompts: 8 per GPU (--prompts-per-gpu; all 64 at N = 8), greedy (-g 1), prompts prefilled,
  each request to position 255 or EOS/BOS.  A step is one pass over the job; value = the
  reference's token count (sum of pos - 1 over requests, src/llama.cpp:1062) / the CLI's serve
  time.  value runs ONE slot per GPU (-b 1), the per-GPU work of the N = 1 line, so the driver's
  per-N values form a weak-scaling curve; the same job at 8 slots per GPU (-b 8, the batched
  form) rides along as "batched".  Each output file is compared with a committed one-process
  fixture of its slot count.  At N = 1 the decode line carries both CLI runs on the one GPU
  ("cli_1gpu"), the per-GPU base of the N > 1 numbers.
* ``requests``: the same job through a torch.distributed process-per-GPU harness
  (hip_llama_cpp_amd/dist.py over the HIP decoder's native callbacks) — a cross-check of the CLI.

Multi-GPU: ``--gpus N`` with no WORLD_SIZE in the environment starts the N ranks itself
(torch.distributed.run as a child process, before anything touches a GPU) and exits with their
status; under an outer torch.distributed.run it is one rank.  ``cli``: rank 0 starts the CLI over
GPUs 0..N-1, the other ranks wait.  ``requests``/``decode``: rank 0 synthesises the weights once
and RCCL-broadcasts them; no collective on the data path (weak scaling).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload decode|cli|requests]
                    [--model 7b|110m] [--dtype f32|int8] [--batch B]
"""
import argparse
import atexit
import hashlib
import json
import os
import re
import shutil
import socket
import subprocess
import sys
import tempfile
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
GOLDEN = os.path.join(REPO, "tests", "golden")
PROMPTS = os.path.join(GOLDEN, "gen_in_64.txt")  # the reference's assets/in/gen_in_64.txt
TOKENIZER = os.path.join(GOLDEN, "tokenizer.bin")  # the reference's assets/tokenizer.bin


def fixture_path(mname, dtype, T):
    """The expected output file of the request job (prompts of gen_in_64.txt, greedy, each request to
    position T - 1 or BOS/EOS), made by the pinned CPU path: tests/golden/make_golden_requests.py
    (oracle/oracle.c, bit-identical to the reference's src/seq.cpp).  Requests are independent, so
    one file serves every slot count.  None where no such fixture exists."""
    p = os.path.join(GOLDEN, f"requests_{mname}_{dtype}_gen_in_64.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        fx = json.load(f)
    return p if fx.get("decode_len") == T and fx.get("seed") == SEED else None


# llama2-7B fp32: the GPU's teacher-forced logits drift up to 1.75e-4 from the CPU reference's over a
# 2048-step decode (profiles/r03/drift_2048_7b_fp32.json; the reference's own GPU path: 5.35e-4,
# tests/golden/reference_gpu_drift_2048.json), so a greedy step whose top-2 margin is under 2e-4 may
# go either way on any fp32 path with another summation order than src/seq.cpp's: the near-ties a
# request may leave the fixture at (each one then proven by a teacher-forced replay, or under 1e-5)
REQUEST_TIE_7B = 2e-4


def compare_request_file(got, fx, n, tie_margin=1e-4, tight=1e-5, evidence=None):
    """The CLI's output file for the first n requests against the fixture.  Byte-identical, or else
    every request's record equals the fixture's except a request whose greedy decode reaches a
    near-tie of the CPU reference (top-2 logit margin < tie_margin) and leaves the fixture's text
    within that step's piece; the rest of such a request is unpinned.  Such a divergence is PROVEN
    when a teacher-forced GPU replay of that step (evidence[(request, position)], made by
    tests/test_requests_gpu.py against tests/golden/request_ties_llama2-7B_f32.json) shows the GPU's
    argmax there is the CPU's runner-up and both competing logits are within the reference's 1e-4
    rule of the CPU's — the fp32 tolerance covers the flip; without evidence only a tie under `tight`
    (whose margin no fp32 summation order can be trusted to resolve) counts as proven.  Returns
    {"identical", "diverged": [[request, position, margin]], "proven", "unproven", "unexplained",
    "ok"}; ok = identical, or no unexplained difference and every divergence proven."""
    ws = [o.encode("latin-1") + b"\n" for o in fx["outputs"][:n]]  # a record: output + "\n"
    head = f"{n}\n".encode()
    res = {"identical": got == head + b"".join(ws), "requests": n, "diverged": [], "proven": [], "unproven": [],
           "unexplained": []}
    if not res["identical"]:
        if not got.startswith(head):
            res["unexplained"].append("header")
            rest = b""
        else:
            rest = got[len(head):]
        for i, w in enumerate(ws):
            if not rest:
                res["unexplained"].append(f"record {i} missing")
                break
            if rest.startswith(w):
                rest = rest[len(w):]
                continue
            first = next((k for k, (a, b) in enumerate(zip(rest, w)) if a != b), min(len(rest), len(w)))
            ties = [t for t in fx["near_ties"][i] if t[1] < tie_margin and t[2] <= first]
            if ties and first - ties[-1][2] <= 64:
                d = [i, ties[-1][0], ties[-1][1]]
                res["diverged"].append(d)
                ev = (evidence or {}).get((i, d[1]))
                proven = (ev["gpu_flips"] and ev["within_tol"]) if ev else d[2] < tight
                (res["proven"] if proven else res["unproven"]).append(d)
            else:
                res["unexplained"].append(i)
            if i + 1 < n:  # the next record starts with its prompt (forced tokens: never diverges)
                k = rest.find(b"\n\n" + ws[i + 1][:48])
                if k < 0:
                    res["unexplained"].append(f"record {i + 1} not found")
                    rest = b""
                    break
                rest = rest[k + 2:]
            else:
                rest = b""
        if rest:
            res["unexplained"].append("trailing bytes")
    res["ok"] = res["identical"] or (not res["unexplained"] and not res["unproven"])
    return res


_WORKDIRS = []


def workdir(prefix):
    """A scratch directory under the repository (visible to every rank); removed at exit whatever
    happens to the run (atexit also runs on SystemExit and uncaught exceptions)."""
    d = tempfile.mkdtemp(prefix=prefix, dir=REPO)
    if not _WORKDIRS:
        atexit.register(lambda: [shutil.rmtree(x, ignore_errors=True) for x in _WORKDIRS])
    _WORKDIRS.append(d)
    return d


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse_args(argv):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5, help="timed steps (decodes / request passes)")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=["decode", "requests", "cli"], default=None,
                    help="default: decode at N = 1, cli at N > 1 (requests: the torch.distributed cross-check)")
    ap.add_argument("--cli-budget", type=float, default=150.0,
                    help="cli: seconds of serving after which no further pass of the value run starts (the -b 8 "
                         "run gets a third, the same-run 1-GPU point a quarter)")
    ap.add_argument("--no-scaling-point", action="store_true",
                    help="cli, N > 1: skip the same per-GPU job on GPU 0 alone (scaling_vs_1gpu)")
    ap.add_argument("--cli-replicas", type=int, default=0,
                    help="cli: THALLAMA_REPLICAS (more workers than GPUs: a one-GPU rehearsal of the N-GPU split)")
    ap.add_argument("--decode-len", type=int, default=256, help="positions per sequence (configs[2]: 256)")
    ap.add_argument("--model", default="7b", choices=sorted(MODELS))
    ap.add_argument("--dtype", default="f32", choices=["f32", "int8"])
    ap.add_argument("--group-size", type=int, default=64, help="Q8_0 group size (int8)")
    ap.add_argument("--batch", type=int, default=0, help="sequences (slots) per GPU; default 1 decode, 8 requests")
    ap.add_argument("--prompts-per-gpu", type=int, default=8)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-nt", action="store_true")
    ap.add_argument("--splits", type=int, default=0)
    ap.add_argument("--no-persistent", action="store_true",
                    help="multi-launch step instead of the one-launch persistent step")
    ap.add_argument("--persistent", action="store_true",
                    help="the batched persistent step also for 5..8 sequences (opt-in there)")
    ap.add_argument("--no-long", action="store_true", help="skip the positions 1792..2047 line")
    ap.add_argument("--long-kernels", action="store_true",
                    help="also time each kernel class with HIP events over the long-context tail (eager replay)")
    ap.add_argument("--no-requests-point", action="store_true", help="skip the 1-GPU request-workload point")
    ap.add_argument("--no-cli-point", action="store_true", help="skip the 1-GPU CLI runs (-b 1 and -b 8)")
    ap.add_argument("--host-argmax", action="store_true",
                    help="requests: greedy sampling on the host from copied logits (the reference's way)")
    ap.add_argument("--cpu-baseline-tokens", type=int, default=0,
                    help="greedy tokens the CPU baseline decodes (0: as many as fit --cpu-baseline-seconds)")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-aggregate", type=int, default=1 << 20,
                    help="max decoders of the aggregate CPU baseline (default: the host CPU share)")
    ap.add_argument("--skip-cpu", action="store_true")
    ap.add_argument("--prof-steps", type=int, default=0,
                    help="positions the roofline object's HIP events cover (0: all decode-len, the headline's span)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL over xGMI) or gloo (CPU rehearsal)")
    ap.add_argument("--device-map", default="", help="comma list: local rank -> HIP device (rehearsals that "
                                                     "put several ranks on one GPU)")
    ap.add_argument("--plumbing", action="store_true",
                    help="no GPU: ranks, sharding and output gathering over a deterministic CPU step (tests)")
    args = ap.parse_args(argv)
    if args.prof_steps < 0:
        ap.error("--prof-steps must be >= 0 (0: the whole decode, the headline's span)")
    if args.gpus < 1 or args.steps < 1 or args.warmup < 0:
        ap.error("--gpus and --steps must be >= 1, --warmup >= 0")
    return args


def launch_ranks(args, argv):
    """--gpus N > 1 without WORLD_SIZE: one rank per GPU via torch.distributed.run, started as a CHILD
    process (nothing here has touched a GPU); returns its exit status."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + argv
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    log(f"bench.py: starting {args.gpus} ranks: {' '.join(cmd[1:8])} ...")
    return subprocess.run(cmd, env=env).returncode


def read_prompts(path, n):
    """The first n prompts of a reference request file (read_inputfile, src/llama.cpp:424-453)."""
    from hip_llama_cpp_amd import host as H
    r = H.Requests(path, 512, 1024)
    if n > len(r):
        raise SystemExit(f"{n} prompts requested, {path} holds {len(r)}")
    return [r.prompt(i) for i in range(n)]


def write_requests(prompts, d):
    fd, path = tempfile.mkstemp(prefix=".bench_req_", suffix=".txt", dir=d)
    with os.fdopen(fd, "wb") as f:
        f.write(f"{len(prompts)}\n".encode() + b"".join(p + b"\n" for p in prompts))
    return path


def sha(strings):
    return hashlib.sha256("\x00".join(strings).encode()).hexdigest()[:16]


# ---------------------------------------------------------------- --plumbing (CPU only, tests)
def plumbing(args, world, rank):
    """Everything of the request workload except the GPU: rank start-up, prompt sharding, the
    reference scheduler, gathering on rank 0.  The step is a deterministic function of
    (token, pos) — a peaked one-hot — so outputs are comparable across world sizes."""
    import numpy as np
    import torch.distributed as dist
    from hip_llama_cpp_amd import dist as D
    if world > 1:
        dist.init_process_group(backend="gloo")
    V = 32000

    def step(_w, tok, pos):
        lg = np.zeros((len(tok), V), np.float32)
        for b, (t, p) in enumerate(zip(tok, pos)):
            lg[b, (int(t) * 7919 + int(p) * 104729 + 13) % (V - 3) + 3] = 1.0
        return lg
    n = args.prompts_per_gpu * world
    wd = workdir(".bench_")
    req = write_requests(read_prompts(PROMPTS, n), wd) if rank == 0 else None
    if world > 1:
        box = [req]
        dist.broadcast_object_list(box, src=0)
        req = box[0]
    out = os.path.join(wd, "out.txt")
    outs = []
    t = time.perf_counter()
    gen = D.serve_sharded(req, out, TOKENIZER, V, args.batch or 8, step, 64, args.decode_len, temperature=0.0,
                          workdir=wd, outputs=outs)
    el = D.max_over_ranks(time.perf_counter() - t)
    if world > 1:
        dist.barrier()
    if rank == 0:
        outs = [o.decode("utf-8", "replace") for o in outs]
        print(json.dumps({"metric": "plumbing (no GPU)", "plumbing": True, "n_gpus": world, "ranks": world,
                          "prompts": n, "tokens": gen, "seconds": round(el, 3),
                          "outputs_sha": [hashlib.sha256(o.encode()).hexdigest()[:12] for o in outs]}), flush=True)
        os.remove(out)
        os.remove(req)
        os.rmdir(wd)
    if world > 1:
        dist.destroy_process_group()


# ---------------------------------------------------------------- --workload cli (configs[4])
def cli_passes(stdout):
    """(tokens, seconds) of each pass the CLI served: its "pass i: tokens N seconds S" lines
    (app/run.cpp, THALLAMA_PASSES), or, for one pass, the reference's own summary lines
    ("Total achieved token: N", "elapsed time(s): S, ...", src/llama.cpp:1062-1070)."""
    lines = stdout.splitlines()
    runs = [(int(ln.split()[3]), float(ln.split()[5])) for ln in lines
            if ln.startswith("pass ") and ln.split()[1].endswith(":")]
    if not runs:
        tot = [ln for ln in lines if ln.startswith("Total achieved token:")]
        el = [ln for ln in lines if ln.startswith("elapsed time(s):")]
        runs = [(int(tot[-1].split()[-1]), float(el[-1].split()[2].rstrip(",")))]
    return runs


def cli_serve(args, world, B, passes, warmup, budget_s=0.0, devices=None, replicas=None):
    """One run of the drop-in CLI (build/apps/llama, app/run.cpp — the reference's
    test_data_parallelism, src/llama.cpp:891-1083: one host thread per GPU, B slots per thread, one
    weight image made on GPU 0 and RCCL-broadcast over xGMI) serving the first prompts_per_gpu x N
    prompts of gen_in_64.txt greedily (-g 1), each request to position decode_len - 1 or EOS/BOS.
    The weights are the synthetic model made on GPU 0 ("synth:" spec, no 27 GB file).  Started as
    a child process over GPUs 0..N-1; it serves the file warmup + passes times on the same
    resident weights (THALLAMA_PASSES).  Returns tokens / serve time of the timed passes (the CLI's
    own clock, weights already in HBM) and whether the output file equals the committed
    one-process fixture of B slots, byte for byte.  budget_s > 0: no pass starts after budget_s
    seconds of serving (THALLAMA_PASS_BUDGET_S), so the run's wall time is bounded whatever a pass
    costs; the passes actually timed are reported.  devices: HIP_VISIBLE_DEVICES for the child
    (default: GPUs 0..world-1 unless the environment already restricts them); replicas: workers
    (THALLAMA_REPLICAS; default --cli-replicas, 0 = one per GPU)."""
    cfg_t, shared, mname = MODELS[args.model]
    q8 = args.dtype == "int8"
    T = args.decode_len
    n = args.prompts_per_gpu * world
    if n > 64:
        raise SystemExit(f"{n} prompts > the 64 of gen_in_64.txt")
    exe = os.environ.get("THALLAMA_BENCH_CLI") or os.path.join(REPO, "build", "apps", "llama")  # (tests: a stand-in)
    if not os.path.exists(exe):
        raise SystemExit(f"bench.py: {exe} not built (make -C hip_llama.cpp_amd)")
    dims = list(cfg_t)
    dims[5] = dims[5] if shared else -dims[5]
    spec = "synth:" + ",".join(str(v) for v in dims) + f":{SEED}" + (f":q8:{args.group_size}" if q8 else "")
    wd = workdir(".bench_cli_")
    req = write_requests(read_prompts(PROMPTS, n), wd)
    out = os.path.join(wd, "out.txt")
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if devices is not None:
        env["HIP_VISIBLE_DEVICES"] = devices
    elif "HIP_VISIBLE_DEVICES" not in env and "ROCR_VISIBLE_DEVICES" not in env:
        env["HIP_VISIBLE_DEVICES"] = ",".join(str(i) for i in range(world))
    reps = args.cli_replicas if replicas is None else replicas
    if reps:
        env["THALLAMA_REPLICAS"] = str(reps)
    else:
        env.pop("THALLAMA_REPLICAS", None)
    env["THALLAMA_PASSES"] = str(warmup + passes)
    if budget_s > 0:
        env["THALLAMA_PASS_BUDGET_S"] = str(budget_s)
    env["THALLAMA_TEST_STEPS"] = str(T)
    cmd = [exe, spec, "-m", "test", "-f", req, "-o", out, "-b", str(B), "-g", "1", "-z", TOKENIZER]
    log("bench.py: " + " ".join(cmd))
    t0 = time.perf_counter()
    p = subprocess.run(cmd, env=env, cwd=REPO, capture_output=True, text=True)
    wall = time.perf_counter() - t0
    if p.returncode != 0:
        log(p.stdout[-4000:], p.stderr[-4000:])
        raise SystemExit(f"bench.py: the CLI failed ({p.returncode})")
    runs = cli_passes(p.stdout)
    timed_p = runs[warmup:] or runs
    tokens = sum(t for t, _ in timed_p)
    secs = sum(x for _, x in timed_p)
    load = next((float(ln.split()[-1]) for ln in p.stdout.splitlines() if ln.startswith("Load model time")), None)
    with open(out, "rb") as f:
        got = f.read()
    fx_path = fixture_path(mname, args.dtype, T)
    check = None
    if fx_path:
        with open(fx_path) as f:
            fx = json.load(f)
        if len(fx["outputs"]) >= n:
            check = compare_request_file(got, fx, n, REQUEST_TIE_7B)
            check["tokens_equal_fixture"] = tokens == (sum(fx["achieved_tokens"][:n]) * len(timed_p))
    # per pass, per GPU (worker): tokens, requests, seconds from the pass start to its last step
    per_gpu = {}
    for ln in p.stdout.splitlines():
        f_ = ln.replace(":", "").split()
        if ln.startswith("pass ") and len(f_) >= 11 and f_[2] == "worker":
            per_gpu.setdefault(int(f_[1]), []).append({"worker": int(f_[3]), "device": int(f_[5]),
                                                       "tokens": int(f_[7]), "requests": int(f_[9]),
                                                       "seconds": float(f_[11])})
    timed_ids = sorted(per_gpu)[warmup:] or sorted(per_gpu)
    gpus = []
    for w in sorted({g["worker"] for i in timed_ids for g in per_gpu[i]}):
        rows = [g for i in timed_ids for g in per_gpu[i] if g["worker"] == w]
        tk, sc = sum(g["tokens"] for g in rows), sum(g["seconds"] for g in rows)
        gpus.append({"worker": w, "device": rows[0]["device"], "tokens_per_pass": rows[0]["tokens"],
                     "requests_per_pass": rows[0]["requests"], "seconds_per_pass": round(sc / len(rows), 4),
                     "tok_s": round(tk / sc, 2) if sc > 0 else None})
    replication, fallbacks = cli_replication(p.stdout)
    cpus = [ln for ln in p.stdout.splitlines() if ln.startswith("worker ") and " cpu " in ln]
    budget_hit = [ln for ln in p.stdout.splitlines() if ln.startswith("pass budget: ")]
    for f_ in (req, out):
        os.remove(f_)
    os.rmdir(wd)
    return {"value": round(tokens / secs, 3), "unit": "tok/s", "slots_per_gpu": B, "prompts": n,
            "seconds_per_pass": round(secs / len(timed_p), 4), "tokens_per_pass": timed_p[0][0],
            "timed_passes": len(timed_p),
            "cmd": " ".join(os.path.relpath(c, REPO) if c.startswith(REPO) else c for c in cmd),
            "passes": [{"tokens": t, "seconds": x} for t, x in runs], "warmup_passes": warmup,
            "pass_budget_s": budget_s, "pass_budget_hit": budget_hit[0] if budget_hit else None,
            "load_s": load, "wall_s": round(wall, 2), "replicas": reps or world,
            "visible_devices": env.get("HIP_VISIBLE_DEVICES", env.get("ROCR_VISIBLE_DEVICES")),
            "output_matches_fixture": check["identical"] if check else None,
            "fixture_check": check,
            "fixture": os.path.relpath(fx_path, REPO) if fx_path else None,
            "output_sha": hashlib.sha256(got).hexdigest()[:16],
            "replication": replication, "replication_fallbacks": fallbacks, "worker_cpus": cpus,
            "per_gpu": gpus}


_REPLICATION = re.compile(r"^replication: (\w+) to (\d+) replica\(s\) on (\d+) GPU\(s\) in ([\d.]+) s$")


def cli_replication(stdout):
    """The CLI's replication summary ("replication: <path> to R replica(s) on G GPU(s) in S s",
    app/run.cpp) and the fall-back lines printed before it ("replication: RCCL failed (...); falling
    back to peer copies", "replication: hipMemcpyPeer ...; falling back to uploads")."""
    lines = stdout.splitlines()
    m = next((m for m in map(_REPLICATION.match, lines) if m), None)
    summary = ({"path": m.group(1), "replicas": int(m.group(2)), "gpus": int(m.group(3)),
                "seconds": float(m.group(4))} if m else None)
    return summary, [ln for ln in lines if ln.startswith("replication: ") and "falling back" in ln]


def weight_bytes(cfg_t):
    """fp32 weight bytes one decode step of a GPU reads (every layer matrix, norms, classifier)."""
    dim, hid, L, H, KVH, V = cfg_t[:6]
    kvd = dim * KVH // H
    return 4.0 * (L * (dim * dim + 2 * dim * kvd + dim * dim + 3 * dim * hid + 2 * dim) + abs(V) * dim + dim)


def token_bytes_host(cfg_t, B, pos):
    """thallama_step_bytes(K_STEP) + the argmax read, in Python (forward.hip, the §8(d) accounting):
    the weights once for the B slots, activations, and every slot's K/V rows 0..pos."""
    dim, hid, L, H, KVH, V = cfg_t[:6]
    kvd = dim * KVH / H
    V = abs(V)
    per_layer = (4.0 * ((dim * dim + 2 * dim * kvd) + dim + B * (dim + dim + 2 * kvd))
                 + 4.0 * (2 * kvd * B * (pos + 1) + B * 2 * dim)
                 + 4.0 * (dim * dim + B * 3 * dim)
                 + 4.0 * (2 * hid * dim + dim + B * (dim + hid))
                 + 4.0 * (hid * dim + B * (hid + 2 * dim)))
    return L * per_layer + 4.0 * (V * dim + dim + B * (dim + V)) + 4.0 * B * V


def cli_roofline(cfg_t, B, r, decode_frac, T):
    """The HBM-roofline half of the metric for a CLI run (the CLI is a child process, so its kernels
    cannot be timed with HIP events here; the N = 1 line carries those): per GPU, its decode tokens/s
    (the CLI's per-worker tokens x the job's share of decoded — not prefilled — tokens) against the
    token rate the HBM peak allows at B slots and the mean position of a request (the §8(d) bytes of
    one step, token_bytes_host; the same accounting as the N = 1 line's requests_1gpu point)."""
    mean_pos = (T - 1) / 2.0
    step = token_bytes_host(cfg_t, B, mean_pos)
    roof_tok_s = HBM_PEAK_GBS * 1e9 / step * B
    per = []
    for g in r.get("per_gpu") or []:
        if not g.get("tok_s"):
            continue
        dts = g["tok_s"] * decode_frac
        per.append({"worker": g["worker"], "device": g["device"], "decode_tok_s": round(dts, 2),
                    "achieved_GBps": round(dts / B * step / 1e9, 1), "frac": round(dts / roof_tok_s, 4)})
    if not per:
        return None
    ach = sum(p["achieved_GBps"] for p in per) / len(per)
    return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "frac_min_gpu": min(p["frac"] for p in per),
            "traffic": None, "per_gpu": per,
            "kernel": f"the whole decode step of {B} slot(s) per GPU, CLI worker clocks (per-kernel HIP events and "
                      "PMC traffic: the N = 1 line)",
            "bytes_per_step": step, "mean_position": mean_pos, "roofline_decode_tok_s_per_gpu": round(roof_tok_s, 1)}


def _first_device():
    """The first GPU this job may use (HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES, else 0)."""
    for k in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES"):
        v = os.environ.get(k)
        if v:
            return v.split(",")[0]
    return "0"


def cli_run(args, world, rank):
    """BASELINE.json configs[4] through the drop-in's OWN multi-GPU path (cli_serve): rank 0 starts
    the CLI over GPUs 0..N-1 before anything here touches a GPU; other ranks only wait (gloo).
    value: one slot per GPU (-b 1, the per-GPU work of the N = 1 decode line, so the per-N values
    are a weak-scaling curve); "batched": the same job at 8 slots per GPU (-b 8), unless --batch
    picks the slot count of value."""
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group(backend="gloo")
    res = None
    if rank == 0:
        cfg_t, shared, mname = MODELS[args.model]
        T = args.decode_len
        B = args.batch or 1
        # wall-time bounds (the driver's --steps 20 --warmup 5 must finish well inside its lease): at most
        # 2 warm-up passes per run, and no pass starts after the run's serve budget
        warm = min(args.warmup, 2)
        r = cli_serve(args, world, B, args.steps, warm, budget_s=args.cli_budget)
        batched = None if args.batch else cli_serve(args, world, 8, args.steps, warm, budget_s=args.cli_budget / 3)
        # the same per-GPU job on GPU 0 alone, in this run: the 1-GPU end of the weak-scaling curve
        one = None
        if world > 1 and not args.no_scaling_point:
            one = cli_serve(args, 1, B, 3, 1, budget_s=args.cli_budget / 4, devices=_first_device(), replicas=0)
        prompts = read_prompts(PROMPTS, r["prompts"])
        from hip_llama_cpp_amd import host as H
        tok = H.Tokenizer(TOKENIZER)
        prompt_pos = sum(max(0, min(len(tok.encode(p)), T) - 1) for p in prompts)
        prompt_pos_1 = sum(max(0, min(len(tok.encode(p)), T) - 1) for p in prompts[:args.prompts_per_gpu])
        tok.close()
        dfrac = lambda rr, pp: (rr["tokens_per_pass"] - pp) / rr["tokens_per_pass"]  # noqa: E731
        roof = cli_roofline(cfg_t, B, r, dfrac(r, prompt_pos), T)
        if batched:
            batched["roofline"] = cli_roofline(cfg_t, 8, batched, dfrac(batched, prompt_pos), T)
        scaling = None
        if one:
            one["roofline"] = cli_roofline(cfg_t, B, one, dfrac(one, prompt_pos_1), T)
            scaling = {"value_1gpu": one["value"], "unit": "tok/s", "n_gpus": world,
                       "scaling_vs_1gpu": round(r["value"] / (world * one["value"]), 4),
                       "note": f"value / ({world} x the same per-GPU job on GPU 0 alone, this run: "
                               f"{args.prompts_per_gpu} prompts, -b {B})"}
        cpu = cpu_baseline(args, cfg_t, shared, mname) if not args.skip_cpu else None
        res = {"metric": "decode tokens/sec (greedy, whole model) + achieved HBM GB/s fraction",
               "value": r["value"], "unit": "tok/s", "n_gpus": world, "steps": r["timed_passes"],
               "steps_requested": args.steps,
               "warmup": args.warmup, "ms_per_step": round(1e3 * r["seconds_per_pass"], 3),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
               "data": "synthetic weights (random init, seed 20240224, made on GPU 0); prompts: the reference's "
                       "gen_in_64.txt",
               "config": {"workload": f"{mname} {args.dtype} drop-in CLI test mode (build/apps/llama -m test -g 1 "
                                      f"-b {B}; src/llama.cpp:891-1083), {r['prompts']} prompts of gen_in_64.txt "
                                      f"({args.prompts_per_gpu} per GPU, one host thread + RCCL-broadcast replica per "
                                      f"GPU), each request to position {T - 1} or EOS/BOS",
                          "model": mname, "global_batch": r["prompts"], "slots_per_gpu": B, "seq_len": cfg_t[6],
                          "decode_len": T, "parallelism": f"prompt-dp{world} (threads + RCCL broadcast)"},
               "cli": r, "batched": batched, "cli_1gpu_same_run": one,
               "scaling_vs_1gpu": scaling["scaling_vs_1gpu"] if scaling else None, "scaling_point": scaling,
               "roofline": roof,
               "roofline_note": "the CLI runs in a child process, so the roofline is per GPU from the CLI's worker "
                                "clocks and the §8(d) bytes of a step (weights "
                                f"{weight_bytes(cfg_t) / 1e9:.2f} GB once per step for the slots of a GPU, plus "
                                "their K/V rows at the mean position); the per-kernel HIP-event roofline and PMC "
                                "traffic are in the N = 1 decode line",
               "cpu_baseline": cpu}
    if world > 1:
        dist.barrier()
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()



def pmc_traffic_file(mname, q8, B, prefixes):
    """The newest committed rocprofv3 PMC pass (profiles/r*_pmc_traffic*.json: FETCH_SIZE and
    WRITE_SIZE in separate runs, gfx950 FETCH_SIZE x2) of this model, dtype and batch that holds one of
    the kernels `prefixes` names (so a multi-launch pass is never picked for the persistent step, nor
    the other way round).  Returns {"file", "kernels", "decode_len"} ({} if none): decode_len is the
    PMC run's --decode-len (its positions 0..decode_len-1), read from the file's "_how"."""
    import glob
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "r*_pmc_traffic*.json")), reverse=True):
        fn = os.path.basename(path)
        if ("int8" in fn) != q8:
            continue
        try:
            with open(path) as f:
                j = json.load(f)
            if j.get("model", "llama2-7B") != mname or j.get("batch", 1) != B:
                continue
            if not any(k.startswith(p) for k in j["kernels"] for p in prefixes):
                continue
            m = re.search(r"--decode-len (\d+)", j.get("_how", ""))
            return {"file": fn, "kernels": j["kernels"], "decode_len": int(m.group(1)) if m else None}
        except (OSError, ValueError, KeyError):
            continue
    return {}


# ---------------------------------------------------------------- CPU baseline
def cpu_baseline(args, cfg_t, shared, mname, gpu_tokens=None):
    """The oracle (bit-exact seq.cpp / runq.c restatement, oracle/oracle.c), same synthetic model, on
    this box's host cores: (i) one decoder on one core, like seq.cpp (int8: runq's OpenMP matmul over
    the cores we may use); (ii) aggregate: P single-threaded decoders at once, one per core.  A
    bounded sample (one calibration token, then as many greedy tokens from BOS as fit
    --cpu-baseline-seconds).  Its tokens are compared with gpu_tokens(n) when given (the N = 1
    decoder), else with the reference's own 256-step decode (tests/golden/reference_long.json)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    q8 = args.dtype == "int8"
    gs = args.group_size
    T, S = args.decode_len, cfg_t[6]
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
        run = lambda m: ref.q8_greedy(1, 0, m)  # noqa: E731
    else:
        O.set_threads(1)
        cores = 1  # seq.cpp is single-threaded
        run = lambda m: ref.greedy(1, 0, m)  # noqa: E731
    n = args.cpu_baseline_tokens
    t1 = None
    if n <= 0:  # bounded sample: as many tokens as fit the time budget (one token calibrates), >= 8
        tc = time.perf_counter()
        run(1)
        t1 = time.perf_counter() - tc
        ref.reset_kv()
        n = max(8, min(T, S, int(args.cpu_baseline_seconds / max(t1, 1e-6))))
    tc = time.perf_counter()
    ctoks = [int(t) for t in run(n)]
    tcpu = time.perf_counter() - tc
    t1 = t1 or tcpu / n
    agg = None
    if not q8 and P > 1:
        m_agg = max(1, min(8, int(args.cpu_baseline_seconds / max(t1, 1e-6) / 2)))
        secs, atoks = ref.aggregate(P, m_agg, allowed[:P])
        agg = {"value": round(P * m_agg / secs, 4), "unit": "tok/s", "cores": P, "decoders": P,
               "sample": f"{P} single-threaded decoders at once (one per core, pinned), decoder i greedy "
                         f"from token 1+i at pos 0, {m_agg} token(s) each",
               "seconds": round(secs, 2), "decoder0_matches_single": atoks[0].tolist() == ctoks[:m_agg]}
    ref.close()
    # span: the GPU figure covers positions 0..T-1, the sample 0..n-1; what differs is the K/V rows read
    # (the weights are read once per token either way), so the span moves the CPU's bytes per token by
    # this fraction — an upper bound on how much it flatters the CPU rate
    dim, _, L, H, KVH = cfg_t[:5]
    kv = lambda p: 4.0 * L * 2 * (dim * KVH / H) * (p + 1)  # noqa: E731
    wb = weight_bytes(cfg_t) * ((1 + 4.0 / gs) / 4 if q8 else 1.0)
    span_effect = (kv((T - 1) / 2.0) - kv((n - 1) / 2.0)) / (wb + kv((n - 1) / 2.0))
    out = {"value": round(n / tcpu, 4), "unit": "tok/s", "cores": cores, "kind": "port",
           "sample": f"{n} greedy tokens (as many as fit ~{args.cpu_baseline_seconds:g} s, at least 8, unless "
                     f"--cpu-baseline-tokens) from BOS (pos 0..{n - 1}) of the same synthetic {mname} "
                     f"{args.dtype} model with oracle/oracle.c (bit-exact "
                     f"{'runq.c' if q8 else 'src/seq.cpp'} restatement), {cores} thread(s)",
           "span": {"cpu_positions": f"0..{n - 1}", "gpu_positions": f"0..{T - 1}",
                    "bytes_per_token_effect": round(span_effect, 6),
                    "note": "the sample's span is shorter than the GPU figure's; the K/V rows it does not read "
                            "change a token's bytes by bytes_per_token_effect (weights dominate), so the CPU "
                            "rate is flattered by at most that fraction"},
           "host": {"nproc": nproc, "affinity_cpus": len(allowed), "cpu_share": share},
           "aggregate": agg}
    if gpu_tokens is not None:
        gtoks = [int(t) for t in gpu_tokens(n)]
        out["tokens_match_gpu"] = ctoks == gtoks
        out["tokens_match_prefix"] = next((i for i, (a, b) in enumerate(zip(ctoks, gtoks)) if a != b),
                                          min(len(ctoks), len(gtoks)))
    else:
        want = None
        try:
            with open(os.path.join(GOLDEN, "reference_long.json")) as f:
                for gc in json.load(f)["cases"]:
                    if tuple(gc["config"]) == tuple(cfg_t) and gc["shared"] == shared and gc["seed"] == SEED:
                        want = gc["q8" if q8 else "fp32"]["tokens"]
        except (OSError, ValueError, KeyError):
            pass
        out["tokens_match_reference"] = (ctoks == want[:n]) if want else None
    return out

# ---------------------------------------------------------------- GPU
def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args, argv))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"bench.py: --gpus {args.gpus} but {world} rank(s) were started")
        sys.exit(3)
    from __graft_entry__ import _pkg
    _pkg()
    if args.plumbing:
        return plumbing(args, world, rank)
    if args.device_map:
        local = [int(v) for v in args.device_map.split(",")][local]
    workload = args.workload or ("decode" if world == 1 else "cli")
    if workload == "cli":
        return cli_run(args, world, rank)
    # the 1-GPU base of the N > 1 CLI numbers, before this process touches the GPU (7B fp32, the
    # job whose fixtures are committed)
    cli_point = None
    if (workload == "decode" and world == 1 and not args.no_cli_point and args.model == "7b" and
            args.dtype == "f32" and args.decode_len == 256 and not args.batch):
        cli_point = {"b1": cli_serve(args, 1, 1, 2, 1), "b8": cli_serve(args, 1, 8, 2, 1)}

    import torch
    import torch.distributed as dist
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
    S, L = cfg_t[6], cfg_t[2]
    gs = args.group_size
    q8 = args.dtype == "int8"
    T = args.decode_len
    if T > S or T < 2:
        raise SystemExit(f"--decode-len must be in [2, seq_len {S}]")

    # ---------------- weights: rank 0 synthesises (and for int8 quantises, export.py semantics),
    # then one RCCL broadcast of the packed weight image to every other rank
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
    model = (tl.DeviceModelQ8(c, shared, gs, payload_ptr=image.data_ptr()) if q8
             else tl.DeviceModel(c, shared, arena_ptr=image.data_ptr()))

    def make_decoder(B):
        state = tl.DeviceState(c, B)
        dec = tl.Decoder(model, state)
        dec.set(tl.OPT_USE_GRAPH, 0 if args.no_graph else 1)
        if args.no_nt:
            dec.set(tl.OPT_NT_WEIGHTS, 0)
        if args.splits:
            dec.set(tl.OPT_ATTN_SPLITS, args.splits)
        if args.no_persistent:
            dec.set(tl.OPT_PERSISTENT, 0)
        elif args.persistent:
            dec.set(tl.OPT_PERSISTENT, 1)
        return state, dec

    def launch_bytes(B, kclass, pos):
        return tl.step_bytes_q8(c, B, kclass, pos, gs) if q8 else tl.step_bytes(c, B, kclass, pos)

    layer_classes = (tl.K_QKV, tl.K_ATTN, tl.K_WO, tl.K_FFN_UP, tl.K_FFN_DOWN)

    def token_bytes(B, p):
        """Algorithmic bytes of one greedy step of B sequences at position p: weights once, K/V rows."""
        return (L * sum(launch_bytes(B, k, [p] * B) for k in layer_classes) + launch_bytes(B, tl.K_CLS, [p] * B)
                + launch_bytes(B, tl.K_ARGMAX, [p] * B))

    def timed(fn, n):
        """n calls of fn, barrier + synchronize on both sides, max over ranks"""
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        return D.max_over_ranks(time.perf_counter() - t, device=dev)

    def profile_roofline(dec, B):
        """Per-kernel-class HIP events on the decoder's stream over an eager replay of the first
        prof-steps positions; the dominant kernel's roofline object."""
        prof, prof_ml = {}, {}
        P = min(args.prof_steps or T, T)
        persistent = dec.persistent()
        step_bytes_p = sum(launch_bytes(B, tl.K_STEP, [p] * B) for p in range(P)) / P

        def run(into):
            dec.set(tl.OPT_PROFILE, 1)
            dec.prof_reset()
            dec.greedy([1] * B, [0] * B, P, want_tokens=False, sync=True)
            for k, name in enumerate(tl.K_NAMES):
                ms, n = dec.prof(k)
                if n:
                    into[name] = {"avg_us": 1e3 * ms / n, "launches": n}
                    if k == tl.K_STEP:
                        into[name]["GBps"] = step_bytes_p / (into[name]["avg_us"] * 1e-6) / 1e9
                    elif k not in (tl.K_ATTN, tl.K_ARGMAX):
                        into[name]["GBps"] = launch_bytes(B, k, [0] * B) / (into[name]["avg_us"] * 1e-6) / 1e9
            dec.set(tl.OPT_PROFILE, 0)
        run(prof)
        if persistent:
            dec.set(tl.OPT_PERSISTENT, 0)
            run(prof_ml)
            dec.set(tl.OPT_PERSISTENT, 1)
        # HBM traffic of the same kernel from the committed rocprofv3 PMC passes (FETCH_SIZE and
        # WRITE_SIZE in separate runs, gfx950 FETCH_SIZE x2 correction): the newest
        # profiles/r*_pmc_traffic*.json of this model, dtype and batch
        stp, ffn = prof.get("step"), prof.get("ffn_up")
        if stp:
            prefixes = ["void tl::persistent_step_kernel<"]
        else:
            # the W1/W3 kernel the launcher picked for B sequences (gemv_launch.hpp launch_mode), in
            # order of preference: the first of these a PMC pass saw
            pre = "gemv_q8" if q8 else "gemv"
            cands = [f"{pre}_rr_kernel", f"{pre}_mfma_kernel", f"{pre}_kernel"] if B >= 4 else [f"{pre}_kernel"]
            if q8:  # the batched int8 step runs in runq's order by default (q8_exact.hip)
                cands = [f"{pre}_exact_kernel"] + cands
            prefixes = [f"void tl::{c}<2" for c in cands]
        pmc = pmc_traffic_file(mname, q8, B, prefixes)

        def traffic_of(prefix):
            hits = [v["traffic_bytes"] for k, v in pmc.get("kernels", {}).items() if k.startswith(prefix)]
            return round(hits[0]) if hits else None
        roof = None
        if stp:
            tr = traffic_of(prefixes[0]) if pmc else None
            # the PMC pass's own positions (its bench run's --decode-len), so traffic is compared with the
            # algorithmic bytes of the same launches
            pp = pmc.get("decode_len")
            alg_p = sum(launch_bytes(B, tl.K_STEP, [p] * B) for p in range(pp)) / pp if pp else None
            roof = {"bound": "hbm", "achieved": round(stp["GBps"], 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(stp["GBps"] / HBM_PEAK_GBS, 4),
                    "traffic": tr,
                    "traffic_source": f"profiles/{pmc['file']} (rocprofv3 --pmc)" if pmc else None,
                    "traffic_positions": f"0..{pp - 1}" if pp else None,
                    "traffic_bytes_algorithmic": alg_p,
                    "traffic_ratio": round(tr / alg_p, 4) if tr and alg_p else None,
                    "kernel": f"persistent_step_kernel (the whole decode step of {B} sequence(s), one launch)",
                    "bytes_per_launch": step_bytes_p, "avg_us": round(stp["avg_us"], 2),
                    "positions": f"0..{P - 1}"}
        elif ffn:
            seen = [c for c, pf in zip(cands, prefixes) if any(k.startswith(pf) for k in pmc.get("kernels", {}))]
            kname = seen[0] if seen else (cands[0] if q8 else f"{pre}_mfma_kernel" if B > 4 else cands[0])
            tr = traffic_of(f"void tl::{kname}<2") if pmc else None
            fb = launch_bytes(B, tl.K_FFN_UP, [0] * B)
            roof = {"bound": "hbm", "achieved": round(ffn["GBps"], 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ffn["GBps"] / HBM_PEAK_GBS, 4),
                    "traffic": tr,
                    "traffic_source": f"profiles/{pmc['file']} (rocprofv3 --pmc)" if pmc else None,
                    "traffic_ratio": round(tr / fb, 4) if tr else None,
                    "kernel": f"{kname}<GM_SWIGLU> (RMSNorm + W1/W3 + SwiGLU)",
                    "bytes_per_launch": fb, "avg_us": round(ffn["avg_us"], 2)}
        rnd = lambda d: {k: {kk: round(vv, 2) for kk, vv in v.items()} for k, v in d.items()}  # noqa: E731
        return roof, rnd(prof), rnd(prof_ml)

    # ------------------------------------------------------------ request workload (configs[4])
    def requests_run(dec, B, n_per_rank, passes, warm):
        """The reference test mode over gen_in_64.txt: n_per_rank prompts per rank, B slots, greedy,
        each request to position T-1 or EOS/BOS.  Returns the measurement dict (rank 0)."""
        from hip_llama_cpp_amd import host as H
        n = n_per_rank * world
        wd = workdir(".bench_") if rank == 0 else None
        prompts = read_prompts(PROMPTS, n)
        req = write_requests(prompts, wd) if rank == 0 else None
        if world > 1:
            box = [req, wd]
            dist.broadcast_object_list(box, src=0)
            req, wd = box
        out = os.path.join(wd, "out.txt")
        tok = H.Tokenizer(TOKENIZER)
        prompt_pos = sum(max(0, min(len(tok.encode(p)), T) - 1) for p in prompts)  # prefilled / forced positions
        mtl = tok.max_token_length
        tok.close()
        addr = lambda f: tl.C.cast(f, tl.C.c_void_p).value  # noqa: E731
        # step (logits), prefill, decoder, greedy step (device argmax: B ids back instead of B x V logits)
        native = (addr(tl.lib().thallama_decoder_step_cb), addr(tl.lib().thallama_decoder_prefill_cb), dec.h.value,
                  0 if args.host_argmax else addr(tl.lib().thallama_decoder_argmax_cb))
        gen, outs = [0], []

        def one():
            outs.clear()
            gen[0] = D.serve_sharded(req, out, TOKENIZER, abs(c.vocab_size), B, None, mtl, T, temperature=0.0,
                                     workdir=wd, native=native, outputs=outs)
        for _ in range(warm):
            one()
        el = timed(one, passes)
        res = None
        if rank == 0:
            fx_path = fixture_path(mname, args.dtype, T)
            check = None
            if fx_path:
                with open(fx_path) as f:
                    fx = json.load(f)
                if len(fx["outputs"]) >= n:
                    got = f"{n}\n".encode() + b"".join(o + b"\n" for o in outs)
                    check = compare_request_file(got, fx, n, REQUEST_TIE_7B)
            tok_s = gen[0] * passes / el
            dec_tokens = gen[0] - prompt_pos
            per_rank_roof = HBM_PEAK_GBS * 1e9 / token_bytes(B, (T - 1) / 2.0) * B
            res = {"workload": f"{mname} {args.dtype} test mode (src/llama.cpp:891-1083), greedy, {n} prompts of "
                               f"gen_in_64.txt ({n_per_rank} per GPU, {B} slots per GPU, prompt prefilled), each "
                               f"request to position {T - 1} or EOS/BOS",
                   "value": round(tok_s, 3), "unit": "tok/s", "seconds_per_pass": round(el / passes, 4),
                   "passes": passes, "tokens_per_pass": gen[0],
                   "decode_tok_s": round(dec_tokens * passes / el, 3),
                   "prompt_positions_per_pass": prompt_pos,
                   "roofline_decode_tok_s_per_gpu": round(per_rank_roof, 1),
                   "frac_of_roofline": round(dec_tokens * passes / el / world / per_rank_roof, 4),
                   "outputs_sha": sha([o.decode("latin-1") for o in outs]),
                   "output_matches_fixture": check["identical"] if check else None, "fixture_check": check,
                   "fixture": os.path.relpath(fx_path, REPO) if fx_path else None}
            os.remove(out)
            os.remove(req)
            os.rmdir(wd)
        if world > 1:
            dist.barrier()
        return res

    out = None
    if workload == "requests":
        B = args.batch or 8
        state, dec = make_decoder(B)
        log(f"[rank {rank}] {mname} {args.dtype} requests B={B} init {t_init:.2f}s (broadcast {t_bcast:.2f}s) "
            f"path {'persistent' if dec.persistent() else 'multi-launch'}")
        per = args.prompts_per_gpu
        if per * world > 64:
            raise SystemExit(f"{per} prompts per GPU x {world} GPUs > the 64 prompts of gen_in_64.txt")
        r = requests_run(dec, B, per, args.steps, args.warmup)
        roof, prof, prof_ml = profile_roofline(dec, B) if rank == 0 else (None, {}, {})
        if rank == 0:
            out = {"metric": "decode tokens/sec (greedy, whole model) + achieved HBM GB/s fraction",
                   "value": r["value"], "unit": "tok/s", "n_gpus": world, "steps": args.steps,
                   "warmup": args.warmup, "ms_per_step": round(1e3 * r["seconds_per_pass"], 3),
                   "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
                   "data": "synthetic weights (random init, seed 20240224); prompts: the reference's gen_in_64.txt",
                   "config": {"workload": r["workload"], "model": mname, "global_batch": per * world,
                              "slots_per_gpu": B, "seq_len": S, "decode_len": T, "parallelism": f"prompt-dp{world}"},
                   "requests": r, "roofline": roof, "kernels": prof, "kernels_multilaunch": prof_ml,
                   "cpu_baseline": None, "init_s": round(t_init, 2), "broadcast_s": round(t_bcast, 2)}
    else:
        B = args.batch or 1
        state, dec = make_decoder(B)
        persistent = dec.persistent()
        log(f"[rank {rank}] {mname} {args.dtype} B={B} init {t_init:.2f}s (broadcast {t_bcast:.2f}s) "
            f"path {'persistent' if persistent else 'multi-launch'}")
        tok0, pos0 = [1] * B, [0] * B  # BOS at position 0

        def decode():
            dec.greedy(tok0, pos0, T, want_tokens=False, sync=False)
        for _ in range(args.warmup):
            decode()
        elapsed = timed(decode, args.steps)
        dec.sync()
        K = args.steps
        value = world * B * T * K / elapsed
        ms_step = elapsed / K * 1e3
        persistent_after = dec.persistent()
        step_bytes = sum(token_bytes(B, p) for p in range(T)) / T  # per token step, mean over positions
        step_gbs = step_bytes * T * K / elapsed / 1e9

        # greedy tokens vs the reference's own 256-step decode (tests/golden/reference_long.json,
        # generated from the reference's seq.cpp / runq.c by make_golden_long.py)
        golden = None
        try:
            with open(os.path.join(GOLDEN, "reference_long.json")) as f:
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

        # long context: positions 1792..2047 of a 2048-token decode (the reference's test mode runs
        # every request to seq_len, src/llama.cpp:1584), tokens against tests/golden/reference_2048.json
        long_ctx = None
        if not args.no_long and S >= 2048 and rank == 0:
            t_tail = 256
            toks_all = dec.greedy(tok0, pos0, S)  # the whole decode (untimed), tokens for the comparison
            # replay its last t_tail positions: every K/V row before them is in place; the input at
            # position S - t_tail is the token generated at the position before
            last_tok = [int(v) for v in toks_all[S - t_tail - 1]]
            torch.cuda.synchronize()
            tc = time.perf_counter()
            dec.greedy(last_tok, [S - t_tail] * B, t_tail, want_tokens=False, sync=True)
            lt = time.perf_counter() - tc
            tail_bytes = sum(token_bytes(B, p) for p in range(S - t_tail, S)) / t_tail
            long_ctx = {"workload": f"positions {S - t_tail}..{S - 1} of a {S}-token greedy decode from BOS "
                                    f"({B} seq/GPU)",
                        "value": round(B * t_tail / lt, 3), "unit": "tok/s", "ms_per_token": round(lt / t_tail * 1e3, 4),
                        "achieved_GBps": round(tail_bytes * t_tail / lt / 1e9, 1),
                        "frac_of_peak": round(tail_bytes * t_tail / lt / 1e9 / HBM_PEAK_GBS, 4),
                        "roofline_tok_s": round(HBM_PEAK_GBS * 1e9 / tail_bytes * B, 1)}
            if args.long_kernels:
                # per-kernel-class HIP events over the same tail, replayed eagerly (the K/V rows it
                # rewrites are the ones already there); GB/s from each class's algorithmic bytes at
                # the tail's positions (attention: the K/V rows it reads)
                dec.set(tl.OPT_PROFILE, 1)
                dec.prof_reset()
                dec.greedy(last_tok, [S - t_tail] * B, t_tail, want_tokens=False, sync=True)
                kk = {}
                for k, name in enumerate(tl.K_NAMES):
                    ms, n = dec.prof(k)
                    if n:
                        us = 1e3 * ms / n
                        kb = sum(launch_bytes(B, k, [p] * B) for p in range(S - t_tail, S)) / t_tail
                        kk[name] = {"avg_us": round(us, 2), "launches": n, "GBps": round(kb / (us * 1e-6) / 1e9, 1)}
                dec.set(tl.OPT_PROFILE, 0)
                long_ctx["kernels_eager"] = kk
            try:
                with open(os.path.join(GOLDEN, "reference_2048.json")) as f:
                    g2 = json.load(f)
                if not q8 and tuple(g2["config"]) == tuple(cfg_t) and g2["seed"] == SEED:
                    want = g2["tokens"]
                    pre = min(next((i for i, (a, b) in enumerate(zip(want, toks_all[:, b].tolist())) if a != b),
                                   len(want)) for b in range(B))
                    long_ctx["reference_tokens"] = {"steps": len(want), "match_prefix": pre,
                                                    "tokens_match": pre == len(want),
                                                    "source": "tests/golden/reference_2048.json"}
            except (OSError, ValueError, KeyError):
                pass

        roof, prof, prof_ml = profile_roofline(dec, B) if rank == 0 else (None, {}, {})
        if roof:  # the same bytes over the timed region's own clock (graph replays, launch gaps included)
            roof["frac_timed_region"] = round(step_gbs / HBM_PEAK_GBS, 4)

        # the 1-GPU point of the request workload (configs[4]'s per-GPU share), so the N > 1 lines
        # have their own single-GPU reference
        req_point = None
        if world == 1 and not args.no_requests_point and not q8 and mname == "llama2-7B":
            del dec, state
            torch.cuda.empty_cache()
            st8, dec8 = make_decoder(8)
            req_point = requests_run(dec8, 8, args.prompts_per_gpu, 1, 1)
            del dec8, st8
            state, dec = make_decoder(B)  # (the CPU baseline compares against a fresh decoder)

        # CPU baseline: the oracle (bit-exact seq.cpp / runq.c restatement), same model, on this box's
        # host cores: (i) one decoder on one core, like seq.cpp (int8: runq's OpenMP matmul over the
        # cores we may use); (ii) aggregate: P single-threaded decoders at once, one per core
        cpu = None
        if rank == 0 and world == 1 and not args.skip_cpu and args.cpu_baseline_tokens >= 0:
            cpu = cpu_baseline(args, cfg_t, shared, mname, lambda n: dec.greedy([1] * B, pos0, n)[:, 0].tolist())

        if rank == 0:
            out = {
                "metric": "decode tokens/sec (greedy, whole model) + achieved HBM GB/s fraction",
                "value": round(value, 3), "unit": "tok/s", "n_gpus": world, "steps": K, "warmup": args.warmup,
                "ms_per_step": round(ms_step, 3), "ms_per_token": round(ms_step / T, 4), "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
                "data": "synthetic (random-init weights, BOS-started greedy decode)",
                "config": {"workload": f"{mname} {args.dtype} {T}-token greedy decode from BOS (positions 0..{T - 1}), "
                                       f"{B} seq/GPU; one step = one whole decode",
                           "model": mname, "global_batch": B * world, "seq_len": S, "decode_len": T,
                           "parallelism": f"prompt-dp{world}"},
                "hbm": {"step_bytes": step_bytes, "achieved_GBps": round(step_gbs, 1),
                        "frac_of_peak": round(step_gbs / HBM_PEAK_GBS, 4),
                        "roofline_tok_s": round(HBM_PEAK_GBS * 1e9 / step_bytes * B * world, 1)},
                "roofline": roof,
                "step_path": "persistent" if persistent_after else "multi-launch",
                "persistent_fallback": bool(persistent and not persistent_after),
                "persistent_launch": (("cooperative" if tl.lib().thallama_persistent_cooperative() else "plain")
                                      if persistent else None),
                "reference_tokens": golden,
                "long_context": long_ctx,
                "requests_1gpu": req_point,
                "cli_1gpu": cli_point,
                "kernels": prof, "kernels_multilaunch": prof_ml,
                "cpu_baseline": cpu,
                "init_s": round(t_init, 2), "broadcast_s": round(t_bcast, 2),
            }
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
