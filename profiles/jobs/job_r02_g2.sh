# register-resident GEMV at 8 sequences as two wave groups of 4 over the same rows (THALLAMA_RR_G2=1):
# parity, then B=8 against the matrix cores and the one-group kernel, same box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && rm -f gpurun_out/job.log && tools/gpujob.sh \
 "t_g2:300:THALLAMA_GEMV_RR=8 THALLAMA_RR_G2=1 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k 'register_resident'" \
 "t_g2b8:400:THALLAMA_GEMV_RR=8 THALLAMA_RR_G2=1 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_golden_long_gpu.py -k 'llama2_7b and batch8'" \
 "g2:200:THALLAMA_GEMV_RR=8 THALLAMA_RR_G2=1 python bench.py --batch 8 --skip-cpu" \
 "g1:200:THALLAMA_GEMV_RR=8 python bench.py --batch 8 --skip-cpu" \
 "mf:200:THALLAMA_GEMV_RR=0 python bench.py --batch 8 --skip-cpu"
