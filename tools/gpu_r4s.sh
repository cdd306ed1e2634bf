set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_sharded.py > gpurun_out/s_par.log 2>&1 || { tail -20 gpurun_out/s_par.log; exit 1; }
tail -1 gpurun_out/s_par.log
timeout -k 10 500 python -u tools/l2_diag.py gpurun_out/s_diag_r --counters "FETCH_SIZE" --mixes main,main#2,hot_next_rud,all_miss_read --args "--log2n 20 --batch 32768 --shards 2" > gpurun_out/s_diag_r.log 2>&1 || { tail -5 gpurun_out/s_diag_r.log; exit 1; }
grep -E "k_m2x|k_m1x|check" gpurun_out/s_diag_r/table.txt | cut -c1-250
timeout -k 10 500 python -u tools/l2_diag.py gpurun_out/s_diag_p --counters "FETCH_SIZE" --mixes main,main#2,hot_next_rud,all_miss_read > gpurun_out/s_diag_p.log 2>&1 || { tail -5 gpurun_out/s_diag_p.log; exit 1; }
grep -E "k_m2x|k_m1x|check" gpurun_out/s_diag_p/table.txt | cut -c1-250
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/s_bench.json 2> gpurun_out/s_bench.err && python3 -c "
import json
d=json.load(open('gpurun_out/s_bench.json')); print(d['value'], d['ms_per_step'], d['stage_ms']['m1'], d['stage_ms']['m2'])"
