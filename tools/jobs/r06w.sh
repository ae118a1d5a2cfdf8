#!/bin/bash
# round 6: keys per batch-1 attention unit at least (ATTN_WIN_MIN_KEYS 16 / 32 / 64): parity of the
# 64 build, then same-box A/B
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=hip_llama.cpp_amd/lib
cp $L/libthallama.so.w64 $L/libthallama.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_persist_gpu.py > gpurun_out/w64_pytest.log 2>&1
rc=$?; cp $L/libthallama.so.w16 $L/libthallama.so; tail -3 gpurun_out/w64_pytest.log; [ $rc -ne 0 ] && exit $rc
BENCH_ARGS="--model 110m" bash tools/variant_ab.sh "w16 w32 w64" 2 || exit 1
AB_LONG=" " bash tools/variant_ab.sh "w16 w32 w64" 2 || exit 1
