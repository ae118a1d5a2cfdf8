#!/usr/bin/env bash
# Round-4 profiles at HEAD (each step under its own limit, tools/gpujob.sh): rocprofv3 kernel stats
# of the default bench line (B=1 fp32 persistent, plain launch: rocprofv3 crashes at exit after a
# cooperative one), int8 B=1 and fp32 B=8; int8 B=1 FETCH_SIZE / WRITE_SIZE in separate passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && rm -rf gpurun_out/prof_* gpurun_out/pmc_* && \
B="python bench.py --skip-cpu --no-long --no-requests-point --no-cli-point" && \
tools/gpujob.sh \
 "prof_b1:300:THALLAMA_PERSIST_COOP=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b1 -o b1 -- $B --steps 5 --prof-steps 4" \
 "prof_int8:300:THALLAMA_PERSIST_COOP=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_int8 -o i8 -- $B --dtype int8 --steps 5 --prof-steps 4" \
 "prof_b8:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b8 -o b8 -- $B --batch 8 --steps 3 --prof-steps 4" \
 "pmc_f_i8:200:THALLAMA_PERSIST_COOP=0 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f_i8 -o f -- $B --dtype int8 --steps 1 --warmup 0 --decode-len 8 --prof-steps 2" \
 "pmc_w_i8:200:THALLAMA_PERSIST_COOP=0 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w_i8 -o w -- $B --dtype int8 --steps 1 --warmup 0 --decode-len 8 --prof-steps 2"
