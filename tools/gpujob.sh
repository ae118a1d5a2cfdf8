#!/usr/bin/env bash
# gpujob.sh — run GPU steps in order, each under its own time limit, logging to gpurun_out/.
# Usage: tools/gpujob.sh "name:seconds:command" ...
# A step that fails normally (e.g. a test failure, rc 1-123) is logged and the job goes on;
# a step that times out (124/137), aborts (134) or crashes (139, or any signal) ends the job:
# nothing else touches the GPU after a possible fault.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] (limit ${secs}s): $cmd" | tee -a gpurun_out/job.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.out" 2> "gpurun_out/$name.err"
  rc=$?
  echo "=== [$name] rc=$rc after $(( $(date +%s) - start ))s" | tee -a gpurun_out/job.log
  tail -3 "gpurun_out/$name.out" | tee -a gpurun_out/job.log
  if [ $rc -ge 124 ]; then
    echo "=== stopping: step $name ended with rc=$rc (timeout/abort/crash)" | tee -a gpurun_out/job.log
    exit $rc
  fi
done
exit 0
