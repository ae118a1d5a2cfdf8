#!/usr/bin/env bash
# round 6: first GPU run of the K-split persistent step (csrc/persist_k.hip): the wave-reduction
# probe, its parity tests, then the 7B fp32 B=8 bench line with it (default) and without it
# (THALLAMA_KSPLIT=1; the default at 8 sequences is the multi-launch step), same box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
B="python bench.py --skip-cpu --no-long --no-requests-point --no-cli-point --batch 8 --steps 3"
tools/gpujob.sh \
 "probe:60:tools/probes/wave_reduce_probe" \
 "ktests:900:python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_persist_k_gpu.py" \
 "bench_k:300:THALLAMA_KSPLIT=1 $B" \
 "bench_ml:300:$B"
