set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_q8_persist_gpu.py tests/test_q8_gpu.py tests/test_persist_gpu.py -q -x > gpurun_out/q8p.log 2>&1 || { echo "TESTS rc=$?"; tail -40 gpurun_out/q8p.log; exit 1; }
tail -2 gpurun_out/q8p.log
timeout -k 10 300 python bench.py --dtype int8 --steps 64 --warmup 4 --skip-cpu > gpurun_out/bq8.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/bq8.log; exit 1; }
tail -1 gpurun_out/bq8.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline'], d.get('step_path'))"
