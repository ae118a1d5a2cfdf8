#!/bin/bash
# round 6: short attention rounds score LPK lanes per key (ATTN_SPLIT_KEYS): batch-1 parity, then same-box A/B
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_persist_gpu.py > gpurun_out/split_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/split_pytest.log; [ $rc -ne 0 ] && exit $rc
BENCH_ARGS="--model 110m" bash tools/variant_ab.sh "s0 s1" 2 || exit 1
AB_LONG=" " bash tools/variant_ab.sh "s0 s1" 2 || exit 1
timeout -k 10 200 python tools/persist_trace.py --model 110m --pos 8 > gpurun_out/split_trace_110m_8.txt 2>&1 || exit 1
grep -h "attention units" gpurun_out/split_trace_110m_8.txt
