#!/usr/bin/env bash
# round 6: the K-split persistent step (opt-in) at HEAD — its full parity file, timelines at positions
# 8 and 128, and the B=8 bench line with it (THALLAMA_KSPLIT=1) and without (the default), same box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
B="python bench.py --skip-cpu --no-requests-point --no-cli-point --batch 8 --steps 3"
tools/gpujob.sh \
 "ktests:900:python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_persist_k_gpu.py" \
 "ktrace8:300:python tools/persist_trace.py --model 7b --batch 8 --pos 8 --json gpurun_out/ktrace_pos8.json" \
 "ktrace128:300:python tools/persist_trace.py --model 7b --batch 8 --pos 128 --json gpurun_out/ktrace_pos128.json" \
 "bench_k:300:THALLAMA_KSPLIT=1 $B" \
 "bench_ml:300:$B"
