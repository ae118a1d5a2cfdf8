#!/bin/bash
# round 6: stories110M batch 1, persistent grid size (THALLAMA_PERSIST_GRID, measurement only), same box
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
B="python bench.py --model 110m --skip-cpu --no-long --no-requests-point --steps 3 --warmup 1 --prof-steps 4"
for r in 1 2; do
  for g in 256 128 64 192; do
    THALLAMA_PERSIST_GRID=$g timeout -k 10 200 $B > gpurun_out/grid_${g}_$r.json 2> gpurun_out/grid_${g}_$r.err || exit 1
    echo "grid $g run $r: $(python -c "import json;d=json.load(open('gpurun_out/grid_${g}_$r.json'));print(d['ms_per_token'], d['value'], d['roofline']['frac'], d['reference_tokens']['match_prefix'])")"
  done
done
for g in 256 128; do
  THALLAMA_PERSIST_GRID=$g timeout -k 10 200 python tools/persist_trace.py --model 110m --pos 8 > gpurun_out/grid_trace_$g.txt 2>&1 || exit 1
done
