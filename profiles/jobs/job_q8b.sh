set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_q8_gpu.py tests/test_q8_persist_gpu.py tests/test_prefill_gpu.py -q -x > gpurun_out/q8b.log 2>&1 || { echo "TESTS rc=$?"; tail -40 gpurun_out/q8b.log; exit 1; }
tail -1 gpurun_out/q8b.log
for b in 2 8; do
timeout -k 10 300 python bench.py --dtype int8 --batch $b --steps 64 --warmup 4 --skip-cpu > gpurun_out/bq8b.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/bq8b.log; exit 1; }
tail -1 gpurun_out/bq8b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('b$b', d['value'], d['ms_per_step'], {k: v.get('GBps', v['avg_us']) for k, v in d['kernels'].items()})"
done
