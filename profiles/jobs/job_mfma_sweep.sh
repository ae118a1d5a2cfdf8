set -o pipefail
export TMPDIR=/tmp
for lay in ${LAYS:-0 1 2}; do
  THALLAMA_MFMA_LAYOUT=$lay timeout -k 10 300 python -m pytest tests/test_forward_gpu.py -q -x -k "batched or batch" > gpurun_out/tl$lay.log 2>&1 || { echo "test lay $lay rc=$?"; tail -30 gpurun_out/tl$lay.log; exit 1; }
  tail -1 gpurun_out/tl$lay.log
  for dep in ${DEPS:-2 4 8}; do
    THALLAMA_MFMA_LAYOUT=$lay THALLAMA_MFMA_DEPTH=$dep timeout -k 10 300 python tools/mfma_sweep.py 4,8,16 >> gpurun_out/sweep.jsonl 2> gpurun_out/sweep_err.log || { echo "sweep rc=$?"; tail gpurun_out/sweep_err.log; exit 1; }
  done
done
python - <<'P'
import json
for l in open("gpurun_out/sweep.jsonl"):
    d=json.loads(l); print(d["env"], {k: v["GBps"] for k, v in d["res"].items()})
P
