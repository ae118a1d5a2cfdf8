#!/usr/bin/env bash
# Round-3 B=8 / B=4 multi-launch PMC passes.  The matrix-core GEMVs now keep
# their hidden kernel arguments (common.hpp keep_implicit_args): with a 344-B explicit-only kernarg
# segment rocprofv3 --pmc faulted on the host in their dispatch (profiles/r03/pmc_sigsegv_diagnosis.md).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && rm -rf gpurun_out/pmc_* && \
B="python bench.py --skip-cpu --no-long --no-requests-point --steps 1 --warmup 0 --decode-len 8 --prof-steps 2 --no-graph" && \
tools/gpujob.sh \
 "pmc_f_b8:200:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f_b8 -o f -- $B --batch 8" \
 "pmc_w_b8:200:rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w_b8 -o w -- $B --batch 8" \
 "pmc_f_b4ml:200:THALLAMA_BATCH_PERSIST=0 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f_b4ml -o f -- $B --batch 4" \
 "pmc_w_b4ml:200:THALLAMA_BATCH_PERSIST=0 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w_b4ml -o w -- $B --batch 4" \
 "pmc_f_b8g:200:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f_b8g -o f -- python bench.py --skip-cpu --no-long --no-requests-point --steps 1 --warmup 0 --decode-len 8 --prof-steps 2 --batch 8"
