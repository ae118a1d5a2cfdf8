cd /root/repo && export TMPDIR=/tmp && tools/gpujob.sh \
 "gpuall:700:python -m pytest tests -x -q -m \"gpu and not slow\"" \
 "smoke:300:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "prof_ps:400:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ps -o ps -- python bench.py --steps 64 --skip-cpu" \
 "prof_ml:400:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ml -o ml -- python bench.py --steps 64 --skip-cpu --no-persistent" \
 "pmc_ps:500:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_ps -o pmc -- python bench.py --steps 4 --warmup 1 --skip-cpu --prof-steps 2" \
 "pmcw_ps:500:rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw_ps -o pmcw -- python bench.py --steps 4 --warmup 1 --skip-cpu --prof-steps 2"
