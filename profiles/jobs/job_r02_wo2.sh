# Wo (residual launch, K <= 4096) at half the split depth vs HEAD before it (THALLAMA_MFMA_DEPTH=4
# restores one depth for every launch), same box, two rounds; parity of the batched paths.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && rm -f gpurun_out/job.log && tools/gpujob.sh \
 "t:400:python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_golden_long_gpu.py tests/test_forward_gpu.py tests/test_ops_gpu.py -k 'batch8 or batched or batch_independent or matmul_batch'" \
 "new1:200:python bench.py --batch 8 --skip-cpu" \
 "old1:200:THALLAMA_MFMA_DEPTH=4 python bench.py --batch 8 --skip-cpu" \
 "new2:200:python bench.py --batch 8 --skip-cpu" \
 "old2:200:THALLAMA_MFMA_DEPTH=4 python bench.py --batch 8 --skip-cpu"
