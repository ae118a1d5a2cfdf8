cd "${GRAFT_REPO_ROOT}" && export TMPDIR=/tmp && rm -rf gpurun_out/pmc_r_* && \
B="python bench.py --skip-cpu --no-long --no-requests-point --no-cli-point --steps 1 --warmup 0 --decode-len 8" && \
tools/gpujob.sh \
 "pmc_r_i8:200:THALLAMA_PERSIST_COOP=0 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_32B_sum -d gpurun_out/pmc_r_i8 -o r -- $B --dtype int8" \
 "pmc_r_f:200:THALLAMA_PERSIST_COOP=0 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_32B_sum -d gpurun_out/pmc_r_f -o r -- $B" \
 "pmc_fi8:200:THALLAMA_PERSIST_COOP=0 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_r_fi8 -o f -- $B --dtype int8" \
 "pmc_wi8:200:THALLAMA_PERSIST_COOP=0 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_r_wi8 -o w -- $B --dtype int8"
rc=$?
for t in i8 f; do db=$(find gpurun_out/pmc_r_$t -name '*results.db' | head -1); [ -n "$db" ] && python tools/rocprof_summary.py counters "$db" gpurun_out/r05b_pmc_rdreq_$t.json "TCC_EA0_RDREQ (all L2 read requests to the fabric, Infinity-Cache hits included) vs TCC_EA0_RDREQ_DRAM; bench.py --decode-len 8, plain launch; round 5 after the poll back-off"; done
f=$(find gpurun_out/pmc_r_fi8 -name '*results.db' | head -1); w=$(find gpurun_out/pmc_r_wi8 -name '*results.db' | head -1)
[ -n "$f" ] && [ -n "$w" ] && python tools/rocprof_summary.py pmc "$f" "$w" gpurun_out/r05_pmc_traffic_int8_b1.json "round 5 HEAD (after the poll back-off): rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs of bench.py --dtype int8 --decode-len 8 (plain launch); traffic = 2*FETCH_SIZE + WRITE_SIZE (gfx950 correction)" llama2-7B 1
rm -rf gpurun_out/pmc_r_*
exit $rc
