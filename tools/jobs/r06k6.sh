#!/usr/bin/env bash
# round 6 close: the K-split step's parity file at HEAD, then rocprofv3 kernel stats of its B=8 bench
# line (plain launch: rocprofv3 crashes at exit after a cooperative one), summarised on the box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && rm -rf gpurun_out/prof_k8 && \
tools/gpujob.sh \
 "ktests:900:python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_persist_k_gpu.py" \
 "prof_k8:300:THALLAMA_KSPLIT=1 THALLAMA_PERSIST_COOP=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_k8 -o k8 -- python bench.py --skip-cpu --no-long --no-requests-point --no-cli-point --batch 8 --steps 3" || exit $?
db=$(find gpurun_out/prof_k8 -name '*results.db' | head -1)
[ -n "$db" ] && python tools/rocprof_summary.py stats "$db" gpurun_out/r06_rocprof_kernel_stats_f32_b8_ksplit.csv
rm -rf gpurun_out/prof_k8
