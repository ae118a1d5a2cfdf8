cd "${GRAFT_REPO_ROOT:-.}" && export TMPDIR=/tmp && rm -rf gpurun_out/pmc_f_b1 gpurun_out/pmc_w_b1 && \
B="python bench.py --skip-cpu --no-long --no-requests-point" && \
tools/gpujob.sh \
 "pmc_f_b1:200:THALLAMA_PERSIST_COOP=0 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f_b1 -o f -- $B --steps 1 --warmup 0 --decode-len 8 --prof-steps 2" \
 "pmc_w_b1:200:THALLAMA_PERSIST_COOP=0 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w_b1 -o w -- $B --steps 1 --warmup 0 --decode-len 8 --prof-steps 2"
