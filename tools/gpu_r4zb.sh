# round-4 final bench line, PMC traffic and kernel stats (tools/gpu_bench_profile.sh)
bash tools/gpu_bench_profile.sh r04zb > gpurun_out/r04zb_prof.log 2>&1; rc=$?
tail -3 gpurun_out/r04zb_prof.log; python3 -c "
import json
d=json.load(open('gpurun_out/r04zb/bench.json')); print(d['value'], d['ms_per_step'], d['roofline'], d['batch_roofline']['frac'], d['cpu_baseline']['value'])"
exit $rc
