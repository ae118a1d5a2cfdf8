#!/bin/bash
# round 6: the attention unit's first-round timeline (trace slots 12 / 13), 110M and 7B, batch 1
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python tools/persist_trace.py --model 110m --pos 8 > gpurun_out/att_trace_110m_8.txt 2>&1 &&
timeout -k 10 200 python tools/persist_trace.py --model 110m --pos 40 > gpurun_out/att_trace_110m_40.txt 2>&1 &&
timeout -k 10 300 python tools/persist_trace.py --model 7b --pos 8 > gpurun_out/att_trace_7b_8.txt 2>&1
rc=$?
grep -h "attention units" gpurun_out/att_trace_*.txt
exit $rc
