#!/usr/bin/env bash
# Round-5 closing measurements at HEAD (each step under its own limit, tools/gpujob.sh): rocprofv3
# kernel stats of the default line (plain launch: rocprofv3 crashes at exit after a cooperative one)
# and FETCH_SIZE / WRITE_SIZE passes (separate runs) for 7B fp32 B=1, summarised on the box into
# gpurun_out/r05_* (the raw rocprofv3 directories are far over gpurun's 64 MiB copy-back and are
# removed) and copied into profiles/ of the box's tree so the bench lines that follow report this
# round's traffic; then the default bench line, the int8 and the stories110M lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && rm -rf gpurun_out/prof_* gpurun_out/pmc_* && \
B="python bench.py --skip-cpu --no-long --no-requests-point --no-cli-point" && \
tools/gpujob.sh \
 "prof_b1:300:THALLAMA_PERSIST_COOP=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b1 -o b1 -- $B --steps 5" \
 "pmc_f_b1:200:THALLAMA_PERSIST_COOP=0 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f_b1 -o f -- $B --steps 1 --warmup 0 --decode-len 8" \
 "pmc_w_b1:200:THALLAMA_PERSIST_COOP=0 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w_b1 -o w -- $B --steps 1 --warmup 0 --decode-len 8" || exit $?
db=$(find gpurun_out/prof_b1 -name '*results.db' | head -1)
[ -n "$db" ] && python tools/rocprof_summary.py stats "$db" gpurun_out/r05_rocprof_kernel_stats_f32_b1.csv
f=$(find gpurun_out/pmc_f_b1 -name '*results.db' | head -1); w=$(find gpurun_out/pmc_w_b1 -name '*results.db' | head -1)
[ -n "$f" ] && [ -n "$w" ] && python tools/rocprof_summary.py pmc "$f" "$w" gpurun_out/r05_pmc_traffic_f32_b1.json \
  "round 5 HEAD: rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs of bench.py --decode-len 8 (7B fp32 B=1, plain launch); traffic = 2*FETCH_SIZE + WRITE_SIZE (gfx950 correction)" llama2-7B 1 && \
  cp gpurun_out/r05_pmc_traffic_f32_b1.json profiles/
rm -rf gpurun_out/prof_* gpurun_out/pmc_*
tools/gpujob.sh \
 "bench_default:600:python bench.py" \
 "bench_int8:300:python bench.py --dtype int8 --skip-cpu --no-requests-point --no-cli-point" \
 "bench_110m:300:python bench.py --model 110m --skip-cpu"
