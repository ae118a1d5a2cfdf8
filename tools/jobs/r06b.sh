#!/bin/bash
# round 6: the fused QKV + attention launch (batched multi-launch step) — parity, then same-box A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_fused_attn_gpu.py tests/test_golden_long_gpu.py tests/test_q8_exact_gpu.py > gpurun_out/r06b_pytest.log 2>&1 || exit $?
for v in fused unfused fused unfused; do
  extra=""; [ $v = unfused ] && extra="--no-fused-attn"
  timeout -k 10 300 python -u bench.py --batch 8 --steps 3 --warmup 1 --skip-cpu --no-requests-point --no-cli-point \
    --long-kernels $extra > gpurun_out/r06b_bench_b8_$v.json 2>> gpurun_out/r06b_bench.err || exit $?
  tail -c 300 gpurun_out/r06b_bench_b8_$v.json
done
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread -m gpu \
  tests/test_requests_gpu.py -k "8-64" > gpurun_out/r06b_requests.log 2>&1
