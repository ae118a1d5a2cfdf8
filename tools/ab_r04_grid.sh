#!/usr/bin/env bash
# Round-4: the persistent step on fewer blocks than CUs (THALLAMA_PERSIST_GRID) for the small model
# (stories110M, 60 phase hand-offs per token: fewer producers and consumers per all-gather).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
B="python bench.py --skip-cpu --no-requests-point --warmup 1 --prof-steps 4 --model 110m --steps 5"
for g in ${GRID_LIST:-256 192 128 96 64 32}; do
  THALLAMA_PERSIST_GRID=$g timeout -k 10 200 $B > gpurun_out/grid_110m_$g.json 2> gpurun_out/grid_110m_$g.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/grid_110m_$g.json'));print('grid $g 110m', d['value'], d['reference_tokens']['match_prefix'], d['step_path'], flush=True)"
done
