set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_full.sh || exit 1
bash tools/gpu_bench_profile.sh r04m > gpurun_out/r04m_prof.log 2>&1; rc=$?
tail -3 gpurun_out/r04m_prof.log; python3 -c "
import json
d=json.load(open('gpurun_out/r04m/bench.json')); print(d['value'], d['ms_per_step'], d['roofline'], d['batch_roofline']['frac'], d['cpu_baseline'])"
exit $rc
