#!/usr/bin/env bash
# Round-5 close: rocprofv3 kernel stats of the int8 B=1 and stories110M B=1 lines at HEAD (after the
# poll back-off), plain launch (rocprofv3 crashes at exit after a cooperative one); summaries on the
# box into gpurun_out/r05_*, raw directories removed.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && rm -rf gpurun_out/prof_* && \
B="python bench.py --skip-cpu --no-long --no-requests-point --no-cli-point" && \
tools/gpujob.sh \
 "prof_int8:300:THALLAMA_PERSIST_COOP=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_int8 -o i8 -- $B --dtype int8 --steps 5" \
 "prof_110m:300:THALLAMA_PERSIST_COOP=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_110m -o m -- $B --model 110m --steps 10"
rc=$?
for t in int8:int8_b1 110m:f32_110m_b1; do
  d=${t%%:*}; n=${t#*:}
  db=$(find gpurun_out/prof_$d -name '*results.db' | head -1)
  [ -n "$db" ] && python tools/rocprof_summary.py stats "$db" gpurun_out/r05_rocprof_kernel_stats_$n.csv
done
rm -rf gpurun_out/prof_*
exit $rc
