for B in 2 3 4 6 8; do
  python bench.py --batch $B --steps 1 --warmup 1 --skip-cpu --no-long --no-requests-point --prof-steps 1 > gpurun_out/p$B.json 2>/dev/null || exit 1
  THALLAMA_BATCH_PERSIST=0 python bench.py --batch $B --steps 1 --warmup 1 --skip-cpu --no-long --no-requests-point --prof-steps 1 > gpurun_out/m$B.json 2>/dev/null || exit 1
  echo B=$B $(python -c "import json;print(json.load(open('gpurun_out/p$B.json'))['ms_per_token'], json.load(open('gpurun_out/m$B.json'))['ms_per_token'])")
done
