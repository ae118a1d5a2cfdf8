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
