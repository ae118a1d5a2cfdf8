"""CPU: the pieces of bench.py's CLI workload (`--workload cli`, the default at N > 1) that need
no GPU — the CLI's pass lines, the per-slot-count fixtures and their agreement."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def test_cli_passes_parses_pass_lines_and_reference_summary():
    out = "loading\npass 0: tokens 2040 seconds 8.742000\npass 1: tokens 2040 seconds 8.665000\n"
    assert bench.cli_passes(out) == [(2040, 8.742), (2040, 8.665)]
    ref = "Total achieved token: 2040\nelapsed time(s): 8.5, achieved throughput TPS (tok/s): 240.0\n"
    assert bench.cli_passes(ref) == [(2040, 8.5)]


def test_fixture_per_slot_count():
    assert bench.fixture_path("llama2-7B", "f32", 8).endswith("bench_requests_llama2-7B_f32_greedy.json")
    assert bench.fixture_path("llama2-7B", "f32", 1).endswith("bench_requests_llama2-7B_f32_greedy_b1.json")


def test_batch1_and_batch8_fixtures_agree():
    """The batch-1 file (persistent step) and the batch-8 file (multi-launch matrix-core step) hold
    the same 64 outputs: a request's greedy output does not depend on its slot count."""
    fx = [json.load(open(bench.fixture_path("llama2-7B", "f32", b))) for b in (1, 8)]
    for f in fx:
        assert f["seed"] == bench.SEED and f["decode_len"] == 256 and len(f["outputs"]) == 64
    assert fx[0]["outputs"] == fx[1]["outputs"]
