#!/usr/bin/env bash
# Round-5 profiles at HEAD (each step under its own limit, tools/gpujob.sh): rocprofv3 kernel stats
# of the default bench line (7B fp32 B=1 persistent, plain launch: rocprofv3 crashes at exit after a
# cooperative one), 7B fp32 B=8, 7B int8 B=1 and stories110M fp32 B=1, then FETCH_SIZE / WRITE_SIZE
# passes (separate runs) for stories110M B=1.  Summaries are written on the box (raw traces are far
# over gpurun's 64 MiB copy-back) into gpurun_out/r05_*; the raw directories are removed.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && rm -rf gpurun_out/prof_* gpurun_out/pmc_* && \
B="python bench.py --skip-cpu --no-long --no-requests-point --no-cli-point" && \
tools/gpujob.sh \
 "prof_b1:300:THALLAMA_PERSIST_COOP=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b1 -o b1 -- $B --steps 5" \
 "prof_b8:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b8 -o b8 -- $B --batch 8 --steps 3" \
 "prof_int8:300:THALLAMA_PERSIST_COOP=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_int8 -o i8 -- $B --dtype int8 --steps 5" \
 "prof_110m:300:THALLAMA_PERSIST_COOP=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_110m -o m -- $B --model 110m --steps 10" \
 "pmc_f_110m:200:THALLAMA_PERSIST_COOP=0 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f_110m -o f -- $B --model 110m --steps 1 --warmup 0 --decode-len 8" \
 "pmc_w_110m:200:THALLAMA_PERSIST_COOP=0 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w_110m -o w -- $B --model 110m --steps 1 --warmup 0 --decode-len 8"
rc=$?
for t in b1:f32_b1 b8:f32_b8 int8:int8_b1 110m:f32_110m_b1; do
  d=${t%%:*}; n=${t#*:}
  db=$(find gpurun_out/prof_$d -name '*results.db' | head -1)
  [ -n "$db" ] && python tools/rocprof_summary.py stats "$db" gpurun_out/r05_rocprof_kernel_stats_$n.csv
done
f=$(find gpurun_out/pmc_f_110m -name '*results.db' | head -1); w=$(find gpurun_out/pmc_w_110m -name '*results.db' | head -1)
[ -n "$f" ] && [ -n "$w" ] && python tools/rocprof_summary.py pmc "$f" "$w" gpurun_out/r05_pmc_traffic_f32_110m_b1.json \
  "round 5 HEAD: rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs of bench.py --model 110m --decode-len 8 (plain launch); traffic = 2*FETCH_SIZE + WRITE_SIZE (gfx950 correction)" stories110M 1
rm -rf gpurun_out/prof_* gpurun_out/pmc_*
exit $rc
