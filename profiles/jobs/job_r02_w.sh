# register-resident GEMV with the gfx950 permlane swaps in the lane reduction: parity at B=4 (default)
# and B=8 (THALLAMA_GEMV_RR=8), then the B=8 / B=4 bench A/B against the matrix-core kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && rm -f gpurun_out/job.log && tools/gpujob.sh \
 "t_rr:300:THALLAMA_GEMV_RR=8 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k 'register_resident or matmul_batch_offsets'" \
 "t_b8:400:THALLAMA_GEMV_RR=8 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_golden_long_gpu.py tests/test_forward_gpu.py -k 'batch8 or batched or batch_independent'" \
 "b_rr:200:THALLAMA_GEMV_RR=8 python bench.py --batch 8 --skip-cpu" \
 "b_mf:200:THALLAMA_GEMV_RR=0 python bench.py --batch 8 --skip-cpu" \
 "b_rr4:200:python bench.py --batch 4 --skip-cpu" \
 "b_rr2:200:THALLAMA_GEMV_RR=8 python bench.py --batch 8 --skip-cpu" \
 "b_mf2:200:THALLAMA_GEMV_RR=0 python bench.py --batch 8 --skip-cpu"
