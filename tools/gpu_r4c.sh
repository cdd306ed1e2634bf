set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/c_bench_base.json 2> gpurun_out/c_bench_base.err &&
GVS_LIB_OVERRIDE=$PWD/build/nts0p/libgvstore.so timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/c_bench_nts0.json 2> gpurun_out/c_bench_nts0.err &&
python3 -c "
import json
for n in ['base','nts0']:
    d=json.load(open(f'gpurun_out/c_bench_{n}.json')); print(n, d['value'], d['ms_per_step'], d['stage_ms']['rpass'], d['stage_ms']['m2'], d['roofline']['frac'])
" &&
timeout -k 10 900 python -u tools/l2_diag.py gpurun_out/c_diag --counters "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" --variants "nts0=build/nts0/libgvstore_test.so,m2s0=build/m2s0/libgvstore_test.so" --mixes main,main#2,all_miss_read,hot_next_rud,deletes > gpurun_out/c_diag.log 2>&1
rc=$?; grep -E "k_rpass2|k_m2x|^===|^---|check|/" gpurun_out/c_diag/table.txt | cut -c1-250; exit $rc
