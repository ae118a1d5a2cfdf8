#!/usr/bin/env bash
# round 6: K-split persistent step iteration — B=8 bench line, timeline at position 128, parity subset
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
B="python bench.py --skip-cpu --no-long --no-requests-point --no-cli-point --batch 8 --steps 3"
tools/gpujob.sh \
 "bench_k:300:THALLAMA_KSPLIT=1 $B" \
 "ktrace128:300:python tools/persist_trace.py --model 7b --batch 8 --pos 128 --json gpurun_out/ktrace_pos128.json" \
 "ktests:600:python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_persist_k_gpu.py -k 'independent or bitwise or selected'"
