# int8 B=8: matrix-core GEMV split depth sweep (THALLAMA_MFMA_DEPTH = blocks per CU targeted)
export TMPDIR=/tmp
for d in 2 3 4 6 8; do
  THALLAMA_MFMA_DEPTH=$d timeout -k 10 200 python bench.py --batch 8 --dtype int8 --steps 128 --warmup 4 --skip-cpu > gpurun_out/sq.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/sq.log; exit 1; }
  tail -1 gpurun_out/sq.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('depth $d', d['value'], {n: k[n]['avg_us'] for n in ('qkv','wo','ffn_up','ffn_down','attn','cls')})"
done
