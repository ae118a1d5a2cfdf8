"""CPU: bench.py's multi-GPU launch path (no GPU needed, `--plumbing`).

`python bench.py --gpus N` with no WORLD_SIZE starts the N ranks itself (torch.distributed.run as
a child process, before any GPU call), like the reference starts one worker per device itself
(src/llama.cpp:902-920).  The plumbing mode runs everything of the request workload (BASELINE.json
configs[4]: the reference's test mode over gen_in_64.txt, 8 prompts per rank) except the GPU step:
rank start-up, sharding, the reference scheduler, the gather on rank 0."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(*args, env=None):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], cwd=REPO, env=e,
                       capture_output=True, text=True, timeout=240)
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    return p.returncode, (json.loads(lines[-1]) if lines else None), p.stderr


def test_gpus2_starts_two_ranks_and_gathers_in_order():
    rc1, one, err1 = run_bench("--plumbing")
    assert rc1 == 0, err1[-2000:]
    rc2, two, err2 = run_bench("--gpus", "2", "--plumbing", "--dist-backend", "gloo")
    assert rc2 == 0, err2[-2000:]
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2 and two["ranks"] == 2
    assert one["prompts"] == 8 and two["prompts"] == 16  # 8 prompts per rank (weak scaling)
    # rank 0 of the 2-rank job served prompts 0..7: their outputs equal the 1-rank job's
    assert two["outputs_sha"][:8] == one["outputs_sha"]
    assert len(set(two["outputs_sha"])) > 8


def test_rank_count_mismatch_fails():
    rc, line, err = run_bench("--gpus", "2", "--plumbing", env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert rc == 3 and line is None, err[-500:]
