# register-resident batched GEMV (gemv_rr.hpp): parity, then B=8 bench A/B against the matrix-core kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && rm -f gpurun_out/job.log && tools/gpujob.sh \
 "t_rr:300:python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k 'register_resident or matmul_batch_offsets'" \
 "t_b8:400:python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_golden_long_gpu.py tests/test_forward_gpu.py -k 'batch8 or batched or batch_independent'" \
 "b_rr:200:python bench.py --batch 8 --skip-cpu" \
 "b_mf:200:THALLAMA_GEMV_RR=0 python bench.py --batch 8 --skip-cpu"
