#!/usr/bin/env bash
# Round-5 profiles at HEAD (each step under its own limit, tools/gpujob.sh): rocprofv3 kernel stats
# of the default bench line (7B fp32 B=1 persistent, plain launch: rocprofv3 crashes at exit after a
# cooperative one), 7B fp32 B=8 (fused attention + Wo), 7B int8 B=1 and stories110M fp32 B=1, then
# FETCH_SIZE / WRITE_SIZE passes (separate runs) for stories110M B=1 and 7B fp32 B=8.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && rm -rf gpurun_out/prof_* gpurun_out/pmc_* && \
B="python bench.py --skip-cpu --no-long --no-requests-point --no-cli-point" && \
tools/gpujob.sh \
 "prof_b1:300:THALLAMA_PERSIST_COOP=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b1 -o b1 -- $B --steps 5" \
 "prof_b8:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b8 -o b8 -- $B --batch 8 --steps 3" \
 "prof_int8:300:THALLAMA_PERSIST_COOP=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_int8 -o i8 -- $B --dtype int8 --steps 5" \
 "prof_110m:300:THALLAMA_PERSIST_COOP=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_110m -o m -- $B --model 110m --steps 10" \
 "pmc_f_110m:200:THALLAMA_PERSIST_COOP=0 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f_110m -o f -- $B --model 110m --steps 1 --warmup 0 --decode-len 8" \
 "pmc_w_110m:200:THALLAMA_PERSIST_COOP=0 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w_110m -o w -- $B --model 110m --steps 1 --warmup 0 --decode-len 8" \
 "pmc_f_b8:200:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f_b8 -o f -- $B --batch 8 --steps 1 --warmup 0 --decode-len 8" \
 "pmc_w_b8:200:rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w_b8 -o w -- $B --batch 8 --steps 1 --warmup 0 --decode-len 8"
