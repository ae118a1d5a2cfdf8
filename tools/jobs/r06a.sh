#!/bin/bash
# round 6, first GPU pass: the tie-step replay + request files, the 7B drop-in timing, graph capture
# paths, then the N = 2 CLI line rehearsed on one GPU (roofline per GPU, same-run 1-GPU point)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 700 --timeout-method thread -m gpu \
  tests/test_requests_gpu.py tests/test_dropin.py tests/test_forward_gpu.py tests/test_concurrency_gpu.py \
  > gpurun_out/r06a_pytest.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --gpus 2 --steps 2 --warmup 1 --skip-cpu \
  > gpurun_out/r06a_bench_n2.json 2> gpurun_out/r06a_bench_n2.err
