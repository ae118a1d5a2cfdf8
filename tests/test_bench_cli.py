"""CPU: the pieces of bench.py's CLI workload (`--workload cli`, the default at N > 1) that need
no GPU — the CLI's pass / per-GPU / replication lines, the oracle-made request fixture and the
near-tie comparison rule."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def test_cli_passes_parses_pass_lines_and_reference_summary():
    out = ("loading\npass 0: tokens 2040 seconds 8.742000\npass 0 worker 0 device 0: tokens 2040 requests 8 "
           "seconds 8.700000\npass 1: tokens 2040 seconds 8.665000\n")
    assert bench.cli_passes(out) == [(2040, 8.742), (2040, 8.665)]
    ref = "Total achieved token: 2040\nelapsed time(s): 8.5, achieved throughput TPS (tok/s): 240.0\n"
    assert bench.cli_passes(ref) == [(2040, 8.5)]


def test_fixture_is_oracle_made():
    """One fixture for every slot count, written by the CPU oracle (not by a GPU run)."""
    p = bench.fixture_path("llama2-7B", "f32", 256)
    assert p and p.endswith("requests_llama2-7B_f32_gen_in_64.json")
    assert bench.fixture_path("llama2-7B", "f32", 128) is None
    assert bench.fixture_path("stories110M", "f32", 256) is None
    with open(p) as f:
        fx = json.load(f)
    assert fx["generator"].startswith("tests/golden/make_golden_requests.py") and "oracle" in fx["generator"]
    assert fx["seed"] == bench.SEED and fx["decode_len"] == 256 and len(fx["outputs"]) == 64
    assert fx["bos_check"]["tokens_match"] and fx["bos_check"]["steps"] == 256
    body = "64\n" + "".join(o + "\n" for o in fx["outputs"])
    assert fx["output_file"] == body
    assert len(fx["near_ties"]) == 64 and sum(fx["achieved_tokens"]) == fx["total_achieved_tokens"]


def _fx():
    outs = ["alpha beta gamma\n", "delta epsilon zeta eta\n", "theta iota\n"]
    return {"outputs": outs, "near_ties": [[], [[9, 3e-5, 6]], [[4, 5e-4, 3]]]}


def test_compare_request_file_rule():
    fx = _fx()
    good = ("3\n" + "".join(o + "\n" for o in fx["outputs"])).encode("latin-1")
    r = bench.compare_request_file(good, fx, 3)
    assert r["identical"] and r["ok"] and not r["diverged"]
    # request 1 takes the other branch at its 3e-5 near-tie (byte 6): allowed only with a < 1e-5 tie
    div = good.replace(b"delta epsilon zeta", b"delta xpsilon zeta")
    r = bench.compare_request_file(div, fx, 3)
    assert not r["identical"] and r["diverged"] == [[1, 9, 3e-5]] and not r["unexplained"]
    assert not r["ok"]  # the fixture has no tie under 1e-5
    fx["near_ties"][1][0][1] = 5e-6
    assert bench.compare_request_file(div, fx, 3)["ok"]
    # a difference before any near-tie, or at a tie of 5e-4 (above the 1e-4 bar), is unexplained
    bad = good.replace(b"alpha", b"alphx")
    r = bench.compare_request_file(bad, fx, 3)
    assert r["unexplained"] == [0] and not r["ok"]
    bad2 = good.replace(b"theta iota", b"theta iotx")
    assert bench.compare_request_file(bad2, fx, 3)["unexplained"] == [2]
    # a missing record
    assert not bench.compare_request_file(b"3\nalpha beta gamma\n\n", fx, 3)["ok"]


def test_parse_args_measurement_switches():
    """The round-5 switches: the long-context per-kernel profile and the opt-in batched persistent
    step; --prof-steps 0 (the whole headline span) stays the default."""
    a = bench.parse_args(["--batch", "8", "--long-kernels", "--persistent"])
    assert a.long_kernels and a.persistent and not a.no_persistent and a.batch == 8
    d = bench.parse_args([])
    assert not d.long_kernels and not d.persistent and d.prof_steps == 0 and d.gpus == 1


def test_replication_summary_after_fallback_lines():
    """the fall-back lines come before the summary and must not be parsed as it."""
    out = ("replication: RCCL failed (ncclCommInitAll: invalid usage); falling back to peer copies\n"
           "replication: hipMemcpyPeer to device 1: invalid argument; falling back to uploads\n"
           "replication: upload to 2 replica(s) on 2 GPU(s) in 3.250000 s\nworker 0: device 0 cpu 3\n")
    s, fb = bench.cli_replication(out)
    assert s == {"path": "upload", "replicas": 2, "gpus": 2, "seconds": 3.25}
    assert len(fb) == 2 and "RCCL failed" in fb[0]
    assert bench.cli_replication("no replication line\n") == (None, [])


def test_pmc_file_matches_the_kernel_it_is_read_for():
    """at fp32 B=4 (persistent step) the multi-launch PMC pass must not be picked."""
    pst = bench.pmc_traffic_file("llama2-7B", False, 4, ["void tl::persistent_step_kernel<"])
    if pst:
        assert "multilaunch" not in pst["file"]
        assert any(k.startswith("void tl::persistent_step_kernel<") for k in pst["kernels"])
    b1 = bench.pmc_traffic_file("llama2-7B", False, 1, ["void tl::persistent_step_kernel<"])
    import glob
    newest = sorted(os.path.basename(f) for f in glob.glob(os.path.join(REPO, "profiles", "r*_pmc_traffic_f32_b1.json")))[-1]
    assert b1 and b1["decode_len"] == 8 and b1["file"] == newest


def test_token_bytes_host_matches_library_accounting(tl):
    """token_bytes_host (the CLI roofline's bytes, no GPU library needed) equals the library's
    thallama_step_bytes(K_STEP) at a few batches / positions (host arithmetic, no GPU call)."""
    cfg_t = bench.MODELS["7b"][0]
    c = tl.Config.make(*cfg_t)
    for B, p in ((1, 0), (1, 127.5), (8, 255)):
        lib = tl.step_bytes(c, B, tl.K_STEP, [int(p)] * B) if p == int(p) else None
        host = bench.token_bytes_host(cfg_t, B, p)
        if lib is not None:
            assert abs(host - lib) / lib < 1e-12, (B, p, host, lib)
    assert 26.4e9 < bench.weight_bytes(cfg_t) < 26.5e9


def _fake_cli(tmp_path):
    """A stand-in for build/apps/llama: parses -f/-o/-b, prints the real CLI's replication, worker and
    per-pass lines (app/run.cpp) and writes the oracle fixture's records for the requests it got."""
    fx = bench.fixture_path("llama2-7B", "f32", 256)
    src = f'''#!{sys.executable}
import json, os, sys
a = sys.argv
req, out = a[a.index("-f") + 1], a[a.index("-o") + 1]
fx = json.load(open({fx!r}))
n = int(open(req, "rb").readline())
ndev = len(os.environ.get("HIP_VISIBLE_DEVICES", "0").split(","))
passes = int(os.environ.get("THALLAMA_PASSES", "1"))
print("replication: %s to %d replica(s) on %d GPU(s) in 1.500000 s" % ("rccl" if ndev > 1 else "none", ndev, ndev))
for w in range(ndev):
    print("worker %d: device %d cpu %d" % (w, w, w))
tok = sum(fx["achieved_tokens"][:n])
rate = 200.0 if a[a.index("-b") + 1] == "1" else 1000.0  # tok/s per GPU
for p in range(passes):
    print("pass %d: tokens %d seconds %f" % (p, tok, tok / ndev / rate + 0.1))
    for w in range(ndev):
        print("pass %d worker %d device %d: tokens %d requests %d seconds %f" % (p, w, w, tok // ndev, n // ndev,
                                                                             tok / ndev / rate))
open(out, "wb").write(("%d\\n" % n).encode() + b"".join(o.encode("latin-1") + b"\\n" for o in fx["outputs"][:n]))
'''
    exe = tmp_path / "fake_llama"
    exe.write_text(src)
    exe.chmod(0o755)
    return str(exe)


def test_cli_line_carries_roofline_scaling_and_bounded_passes(tmp_path):
    """The N > 1 line (--workload cli) carries the whole metric: a per-GPU roofline, the same-run
    1-GPU point with scaling_vs_1gpu, and the pass budget (CPU, gloo ranks, a stand-in CLI)."""
    import subprocess
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "HIP_VISIBLE_DEVICES",
              "ROCR_VISIBLE_DEVICES"):
        env.pop(k, None)
    env["THALLAMA_BENCH_CLI"] = _fake_cli(tmp_path)
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--workload", "cli",
                        "--steps", "3", "--warmup", "5", "--skip-cpu"], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["steps"] == 3 and line["scaling"] == "weak"
    assert line["cli"]["warmup_passes"] == 2  # bounded warm-up
    assert line["cli"]["output_matches_fixture"] and line["batched"]["output_matches_fixture"]
    roof = line["roofline"]
    assert roof["bound"] == "hbm" and roof["unit"] == "GB/s" and roof["peak"] == bench.HBM_PEAK_GBS
    assert len(roof["per_gpu"]) == 2 and all(0 < g["frac"] < 1 for g in roof["per_gpu"])
    assert 0 < roof["frac"] < 1 and abs(roof["frac"] - roof["achieved"] / roof["peak"]) < 1e-3
    assert line["batched"]["roofline"]["per_gpu"]
    one = line["cli_1gpu_same_run"]
    assert one["prompts"] == 8 and one["visible_devices"] == "0" and one["output_matches_fixture"]
    # the stand-in serves 2 GPUs x 8 prompts in the time 1 GPU serves 8: scaling 1.0
    assert abs(line["scaling_vs_1gpu"] - 1.0) < 1e-3


def test_compare_request_file_evidence():
    """A divergence at a tie above `tight` is proven only by a teacher-forced GPU replay that flips
    there with both competing logits within the 1e-4 rule."""
    fx = _fx()
    good = ("3\n" + "".join(o + "\n" for o in fx["outputs"])).encode("latin-1")
    div = good.replace(b"delta epsilon zeta", b"delta xpsilon zeta")
    assert bench.compare_request_file(div, fx, 3)["unproven"] == [[1, 9, 3e-5]]
    ok = bench.compare_request_file(div, fx, 3, evidence={(1, 9): {"gpu_flips": True, "within_tol": True}})
    assert ok["ok"] and ok["proven"] == [[1, 9, 3e-5]] and not ok["unproven"]
    for ev in ({"gpu_flips": False, "within_tol": True}, {"gpu_flips": True, "within_tol": False}):
        assert not bench.compare_request_file(div, fx, 3, evidence={(1, 9): ev})["ok"]
