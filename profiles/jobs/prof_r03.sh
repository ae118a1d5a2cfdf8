#!/usr/bin/env bash
# Round-3 profiles: rocprofv3 kernel stats of the default bench (7B fp32 B=1) and of B=4 / B=8,
# then FETCH_SIZE and WRITE_SIZE in separate --pmc passes (gfx950 rules, MI355X_MICROARCH.md) for
# B=1, B=4 (batched persistent step) and B=8 (multi-launch, eager: --no-graph).  The persistent
# launch is plain (THALLAMA_PERSIST_COOP=0): rocprofv3 crashes at exit after a cooperative one.
# Last, the round-2 SIGSEGV diagnosis: B=4 multi-launch (gemv_rr) eager, then the same with graph replay.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && rm -rf gpurun_out/prof_* gpurun_out/pmc_* && \
B="python bench.py --skip-cpu --no-long --no-requests-point" && \
tools/gpujob.sh \
 "prof_b1:300:THALLAMA_PERSIST_COOP=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b1 -o b1 -- $B --steps 5 --prof-steps 4" \
 "prof_b4:300:THALLAMA_PERSIST_COOP=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b4 -o b4 -- $B --steps 3 --batch 4 --prof-steps 4" \
 "prof_b8:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b8 -o b8 -- $B --steps 3 --batch 8 --prof-steps 4" \
 "pmc_f_b1:200:THALLAMA_PERSIST_COOP=0 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f_b1 -o f -- $B --steps 1 --warmup 0 --decode-len 8 --prof-steps 2" \
 "pmc_w_b1:200:THALLAMA_PERSIST_COOP=0 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w_b1 -o w -- $B --steps 1 --warmup 0 --decode-len 8 --prof-steps 2" \
 "pmc_f_b4:200:THALLAMA_PERSIST_COOP=0 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f_b4 -o f -- $B --steps 1 --warmup 0 --decode-len 8 --prof-steps 2 --batch 4" \
 "pmc_w_b4:200:THALLAMA_PERSIST_COOP=0 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w_b4 -o w -- $B --steps 1 --warmup 0 --decode-len 8 --prof-steps 2 --batch 4" \
 "pmc_f_b8:200:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f_b8 -o f -- $B --steps 1 --warmup 0 --decode-len 8 --prof-steps 2 --batch 8 --no-graph" \
 "pmc_w_b8:200:rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w_b8 -o w -- $B --steps 1 --warmup 0 --decode-len 8 --prof-steps 2 --batch 8 --no-graph" \
 "pmc_f_b4ml:200:THALLAMA_BATCH_PERSIST=0 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f_b4ml -o f -- $B --steps 1 --warmup 0 --decode-len 8 --prof-steps 2 --batch 4 --no-graph" \
 "pmc_w_b4ml:200:THALLAMA_BATCH_PERSIST=0 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w_b4ml -o w -- $B --steps 1 --warmup 0 --decode-len 8 --prof-steps 2 --batch 4 --no-graph" \
 "pmc_f_b4g:200:THALLAMA_BATCH_PERSIST=0 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f_b4g -o f -- $B --steps 1 --warmup 0 --decode-len 8 --prof-steps 2 --batch 4"
