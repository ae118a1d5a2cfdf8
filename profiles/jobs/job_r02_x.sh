# Batch-4 256-step golden (register-resident GEMV at 7B) and the 2-rank rehearsal of the N>1 bench
# path on one GPU (gloo, both ranks on device 0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && rm -f gpurun_out/job.log && tools/gpujob.sh \
 "t_b4:400:python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_golden_long_gpu.py -k 'batch4'" \
 "n2:400:python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 32 --warmup 4 --dist-backend gloo --device-map 0,0 --skip-cpu"
