#!/usr/bin/env bash
# Round-6 closing measurements at HEAD (each step under its own limit, tools/gpujob.sh): rocprofv3
# kernel stats (plain launch: rocprofv3 crashes at exit after a cooperative one) of the 7B fp32 B=1,
# B=8 and int8 B=1 lines, FETCH_SIZE / WRITE_SIZE passes (separate runs) for 7B fp32 B=1, summarised
# on the box into gpurun_out/r06_* (the raw directories are removed) and the PMC file copied into the
# box's profiles/ so the bench line that follows reports this round's traffic; then the default
# bench line, the int8 and the stories110M lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && rm -rf gpurun_out/prof_* gpurun_out/pmc_* && \
B="python bench.py --skip-cpu --no-long --no-requests-point --no-cli-point" && \
tools/gpujob.sh \
 "prof_b1:300:THALLAMA_PERSIST_COOP=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b1 -o b1 -- $B --steps 5" \
 "pmc_f_b1:200:THALLAMA_PERSIST_COOP=0 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f_b1 -o f -- $B --steps 1 --warmup 0 --decode-len 8" \
 "pmc_w_b1:200:THALLAMA_PERSIST_COOP=0 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w_b1 -o w -- $B --steps 1 --warmup 0 --decode-len 8" \
 "prof_b8:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b8 -o b8 -- $B --batch 8 --steps 3" \
 "prof_i8:300:THALLAMA_PERSIST_COOP=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_i8 -o i8 -- $B --dtype int8 --steps 5" || exit $?
for t in b1:f32_b1 b8:f32_b8 i8:int8_b1; do
  d=${t%%:*}; n=${t#*:}
  db=$(find gpurun_out/prof_$d -name '*results.db' | head -1)
  [ -n "$db" ] && python tools/rocprof_summary.py stats "$db" gpurun_out/r06_rocprof_kernel_stats_$n.csv
done
f=$(find gpurun_out/pmc_f_b1 -name '*results.db' | head -1); w=$(find gpurun_out/pmc_w_b1 -name '*results.db' | head -1)
[ -n "$f" ] && [ -n "$w" ] && python tools/rocprof_summary.py pmc "$f" "$w" gpurun_out/r06_pmc_traffic_f32_b1.json \
  "round 6 HEAD: rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs of bench.py --decode-len 8 (7B fp32 B=1, plain launch); traffic = 2*FETCH_SIZE + WRITE_SIZE (gfx950 correction)" llama2-7B 1 && \
  cp gpurun_out/r06_pmc_traffic_f32_b1.json profiles/
rm -rf gpurun_out/prof_* gpurun_out/pmc_*
tools/gpujob.sh \
 "bench_default:600:python bench.py" \
 "bench_int8:300:python bench.py --dtype int8 --skip-cpu --no-requests-point --no-cli-point" \
 "bench_110m:300:python bench.py --model 110m --skip-cpu"
