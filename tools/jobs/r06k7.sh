#!/usr/bin/env bash
# round 6: the K-split step with the attention fused into the QKV reduce (7B shapes) — its parity
# file, then same-box A/B against the unfused form and the multi-launch default
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_persist_k_gpu.py > gpurun_out/ktests_fused.log 2>&1 || { tail -30 gpurun_out/ktests_fused.log; exit 1; }
tail -2 gpurun_out/ktests_fused.log
AB_LONG=" " BENCH_ARGS="--batch 8 --no-cli-point" VARIANT_ENV_fused="THALLAMA_KSPLIT=1" VARIANT_ENV_unfused="THALLAMA_KSPLIT=1" \
  bash tools/variant_ab.sh "ml fused unfused" 2 > gpurun_out/ab14.log 2>&1
cat gpurun_out/ab14.log
