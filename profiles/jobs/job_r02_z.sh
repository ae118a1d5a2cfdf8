# register-resident GEMV: 4 register batches with the next batch issued before each consume
# (RR_BUF4, lib/libthallama.so.buf4) vs HEAD, same box: parity (B=4, forced B=8), B=4 / B=8 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && rm -f gpurun_out/job.log && L=hip_llama.cpp_amd/lib && cp $L/libthallama.so $L/libthallama.so.base && tools/gpujob.sh \
 "t4:300:cp $L/libthallama.so.buf4 $L/libthallama.so && THALLAMA_GEMV_RR=8 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k 'register_resident'" \
 "v4_b4:200:cp $L/libthallama.so.buf4 $L/libthallama.so && python bench.py --batch 4 --skip-cpu" \
 "v4_b8:200:cp $L/libthallama.so.buf4 $L/libthallama.so && THALLAMA_GEMV_RR=8 python bench.py --batch 8 --skip-cpu" \
 "base_b4:200:cp $L/libthallama.so.base $L/libthallama.so && python bench.py --batch 4 --skip-cpu" \
 "base_b8:200:cp $L/libthallama.so.base $L/libthallama.so && THALLAMA_GEMV_RR=8 python bench.py --batch 8 --skip-cpu" \
 "mf_b8:200:cp $L/libthallama.so.base $L/libthallama.so && THALLAMA_GEMV_RR=0 python bench.py --batch 8 --skip-cpu"
cp $L/libthallama.so.base $L/libthallama.so
