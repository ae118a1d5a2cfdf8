export TMPDIR=/tmp
for d in 2 3 4 6 8; do
  THALLAMA_MFMA_DEPTH=$d timeout -k 10 200 python bench.py --batch 8 --steps 128 --warmup 4 --skip-cpu > gpurun_out/sd.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/sd.log; exit 1; }
  tail -1 gpurun_out/sd.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('depth $d', d['value'], {n: k[n]['avg_us'] for n in ('qkv','wo','ffn_up','ffn_down','attn')})"
done
