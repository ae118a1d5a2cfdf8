#!/usr/bin/env bash
# round 6: timeline of the K-split persistent step (7B fp32, 8 sequences) at positions 8 and 128
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
tools/gpujob.sh \
 "ktrace8:300:python tools/persist_trace.py --model 7b --batch 8 --pos 8 --json gpurun_out/ktrace_pos8.json" \
 "ktrace128:300:python tools/persist_trace.py --model 7b --batch 8 --pos 128 --json gpurun_out/ktrace_pos128.json"
