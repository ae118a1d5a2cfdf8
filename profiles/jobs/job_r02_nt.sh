# B=8: non-temporal weight loads (default) vs default-policy loads (--no-nt), same box, two rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && rm -f gpurun_out/job.log && tools/gpujob.sh \
 "nt1:200:python bench.py --batch 8 --skip-cpu" \
 "nn1:200:python bench.py --batch 8 --skip-cpu --no-nt" \
 "nt2:200:python bench.py --batch 8 --skip-cpu" \
 "nn2:200:python bench.py --batch 8 --skip-cpu --no-nt" \
 "b4nn:200:python bench.py --batch 4 --skip-cpu --no-nt" \
 "b4nt:200:python bench.py --batch 4 --skip-cpu"
