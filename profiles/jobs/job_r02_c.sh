# Round-2: exact int8 persistent step — bit-exactness tests, the int8 persistent suite, bench int8.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && rm -f gpurun_out/job.log && tools/gpujob.sh \
 "q8exact:600:python -u -m pytest tests/test_q8_persist_gpu.py tests/test_golden_long_gpu.py -m gpu -v -k 'q8 or int8' --timeout 300 --timeout-method thread" \
 "bench_q8:500:python bench.py --dtype int8"
