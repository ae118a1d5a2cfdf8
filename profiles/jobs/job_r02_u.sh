# int8 persistent step: register slots in flight per streaming wave (PERSIST_NBUF 2 = HEAD, 3, 4),
# same box, two rounds; the bench checks the 256 greedy tokens against runq's (bit-exact path).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && rm -f gpurun_out/job.log && L=hip_llama.cpp_amd/lib && cp $L/libthallama.so $L/libthallama.so.base
for r in 1 2; do for v in base nb3 nb4; do
  cp $L/libthallama.so.$v $L/libthallama.so
  timeout -k 10 200 python bench.py --dtype int8 --skip-cpu > gpurun_out/u_${v}_${r}.log 2>&1 || { echo "$v rc=$?"; tail -5 gpurun_out/u_${v}_${r}.log; cp $L/libthallama.so.base $L/libthallama.so; exit 1; }
  tail -1 gpurun_out/u_${v}_${r}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], d['reference_tokens']['tokens_match'], d['reference_tokens']['match_prefix'])" | tee -a gpurun_out/job.log
done; done
cp $L/libthallama.so.base $L/libthallama.so
