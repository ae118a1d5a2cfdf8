#!/usr/bin/env bash
# round 6: K-split step with plain-float x / SwiGLU hand-offs behind per-producer flags — parity subset,
# then the B=8 bench line with it and the multi-launch default, twice each, same box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
B="python bench.py --skip-cpu --no-long --no-requests-point --no-cli-point --batch 8 --steps 3"
tools/gpujob.sh \
 "ktests:600:python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_persist_k_gpu.py -k 'independent or bitwise or greedy or give_up'" \
 "bench_k1:300:THALLAMA_KSPLIT=1 $B" \
 "bench_ml1:300:$B" \
 "bench_k2:300:THALLAMA_KSPLIT=1 $B" \
 "bench_ml2:300:$B"
