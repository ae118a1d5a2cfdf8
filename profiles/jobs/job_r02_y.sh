# register-resident GEMV at 8 sequences, batch shapes (THALLAMA_RR8_SHAPE 0/1/2) vs the matrix cores.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && rm -f gpurun_out/job.log && tools/gpujob.sh \
 "t_rr:300:THALLAMA_GEMV_RR=8 THALLAMA_RR8_SHAPE=1 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k 'register_resident' && THALLAMA_GEMV_RR=8 THALLAMA_RR8_SHAPE=2 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k 'register_resident'" \
 "s0:200:THALLAMA_GEMV_RR=8 THALLAMA_RR8_SHAPE=0 python bench.py --batch 8 --skip-cpu" \
 "s1:200:THALLAMA_GEMV_RR=8 THALLAMA_RR8_SHAPE=1 python bench.py --batch 8 --skip-cpu" \
 "s2:200:THALLAMA_GEMV_RR=8 THALLAMA_RR8_SHAPE=2 python bench.py --batch 8 --skip-cpu" \
 "mf:200:THALLAMA_GEMV_RR=0 python bench.py --batch 8 --skip-cpu"
