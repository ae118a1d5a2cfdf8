cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && rm -f gpurun_out/job.log && tools/gpujob.sh \
 "q8exact:600:python -u -m pytest tests/test_q8_persist_gpu.py tests/test_golden_long_gpu.py -m gpu -q -k 'bitexact' --timeout 300 --timeout-method thread" \
 "tr_q8:200:python tools/persist_trace.py --dtype int8 --pos 8" \
 "tr_q8_200:200:python tools/persist_trace.py --dtype int8 --pos 200" \
 "bench_q8:300:python bench.py --dtype int8 --skip-cpu"
