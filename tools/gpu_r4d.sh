set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for x in 0 2 16 18 3 17; do
  GVS_LIB_OVERRIDE=$PWD/build/aux$x/libgvstore_test.so timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/d_bench_aux$x.json 2> gpurun_out/d_bench_aux$x.err || exit 1
  python3 -c "
import json
d=json.load(open('gpurun_out/d_bench_aux$x.json')); print('aux$x', d['value'], d['ms_per_step'], d['stage_ms']['rpass'], d['stage_ms']['m2'], d['roofline']['frac'])
" || exit 1
done
timeout -k 10 900 python -u tools/l2_diag.py gpurun_out/d_diag --counters "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_BUBBLE_sum" --variants "aux2=build/aux2/libgvstore_test.so,aux16=build/aux16/libgvstore_test.so,aux18=build/aux18/libgvstore_test.so,aux3=build/aux3/libgvstore_test.so,aux17=build/aux17/libgvstore_test.so" --mixes main,main#2,all_create,rud,deletes > gpurun_out/d_diag.log 2>&1
rc=$?; grep -E "k_rpass2|^===|^---|check|/" gpurun_out/d_diag/table.txt | cut -c1-250; exit $rc
