# Persistent-step change: parity tests on the new build, then same-box A/B (fp32, int8) and traces.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && L=hip_llama.cpp_amd/lib && cp $L/libthallama.so.new $L/libthallama.so && tools/gpujob.sh \
 "ptest:300:python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_persist_gpu.py tests/test_q8_persist_gpu.py" \
 "ab32:400:bash profiles/jobs/job_ab.sh" \
 "ab8:400:BENCH_ARGS='--dtype int8' bash profiles/jobs/job_ab.sh" \
 "tr8:120:python tools/persist_trace.py --model 7b --pos 8" \
 "trq8:120:python tools/persist_trace.py --model 7b --pos 8 --dtype int8"
