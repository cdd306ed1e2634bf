set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v -m gpu --timeout 600 --timeout-method thread tests/test_timing.py > gpurun_out/o_timing.log 2>&1
grep -E "passed|failed|AssertionError" gpurun_out/o_timing.log | tail -4 | cut -c1-700
cp gpurun_out/timing_c3_store.txt gpurun_out/o_timing_store.txt; cp gpurun_out/timing_c3_expiry.txt gpurun_out/o_timing_expiry.txt
bash tools/gpu_bench_profile.sh r04o > gpurun_out/r04o_prof.log 2>&1; rc=$?
tail -3 gpurun_out/r04o_prof.log; python3 -c "
import json
d=json.load(open('gpurun_out/r04o/bench.json')); print(d['value'], d['ms_per_step'], d['roofline'], d['batch_roofline']['frac'], d['cpu_baseline'])"
exit $rc
