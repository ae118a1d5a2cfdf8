#!/bin/bash
# round 6: FETCH_SIZE calibration of the read shapes the persistent steps use (tools/probes/fetch_calib.hip)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/calib_f -o f -- tools/probes/bin/fetch_calib > gpurun_out/calib_f.log 2>&1 || exit $?
timeout -k 10 60 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/calib_w -o w -- tools/probes/bin/fetch_calib > gpurun_out/calib_w.log 2>&1 || exit $?
timeout -k 10 60 rocprofv3 --kernel-trace --stats -d gpurun_out/calib_t -o t -- tools/probes/bin/fetch_calib > gpurun_out/calib_t.log 2>&1 || exit $?
f=$(find gpurun_out/calib_f -name '*results.db' | head -1)
python tools/rocprof_summary.py counters "$f" gpurun_out/r06_fetch_calib.json "FETCH_SIZE per launch: k16 / k4 / k8s each read 536870912 bytes once (nt buffer loads)"
w=$(find gpurun_out/calib_w -name '*results.db' | head -1)
python tools/rocprof_summary.py counters "$w" gpurun_out/r06_write_calib.json "WRITE_SIZE per launch: kst8 / kst16 write 67108864 bytes with sc1 stores"
t=$(find gpurun_out/calib_t -name '*results.db' | head -1)
python tools/rocprof_summary.py stats "$t" gpurun_out/r06_fetch_calib_stats.csv
rm -rf gpurun_out/calib_f gpurun_out/calib_w gpurun_out/calib_t
python -c "import json; [print(n, k, round(v['avg'])) for f in ('gpurun_out/r06_fetch_calib.json', 'gpurun_out/r06_write_calib.json') for n, c in json.load(open(f))['kernels'].items() for k, v in c.items()]"
