#!/usr/bin/env bash
# int8 B=1 traffic per kernel class on the MULTI-LAUNCH step (bench.py --no-persistent): FETCH_SIZE /
# WRITE_SIZE in separate passes, so each GEMV launch's bytes can be set against its algorithmic
# bytes (which phase kind carries the persistent step's 4% excess).  Eager launches (--no-graph):
# rocprofv3 --pmc died (SIGSEGV, host side) on this path's graph replay.  Summaries on the box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && rm -rf gpurun_out/pmc_ml_* && \
B="python bench.py --dtype int8 --no-persistent --skip-cpu --no-long --no-requests-point --no-cli-point --steps 1 --warmup 0 --decode-len 8 --no-graph" && \
tools/gpujob.sh \
 "pmc_ml_f:200:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_ml_f -o f -- $B" \
 "pmc_ml_w:200:rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_ml_w -o w -- $B"
rc=$?
f=$(find gpurun_out/pmc_ml_f -name '*results.db' | head -1); w=$(find gpurun_out/pmc_ml_w -name '*results.db' | head -1)
[ -n "$f" ] && [ -n "$w" ] && python tools/rocprof_summary.py pmc "$f" "$w" gpurun_out/r05_pmc_traffic_int8_b1_multilaunch.json "round 5: rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs of bench.py --dtype int8 --no-persistent --decode-len 8; traffic = 2*FETCH_SIZE + WRITE_SIZE (gfx950 correction)" llama2-7B-multilaunch 1
rm -rf gpurun_out/pmc_ml_*
exit $rc
