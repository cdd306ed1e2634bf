set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/l2_diag.py gpurun_out/f_diag --counters "TCC_UC_REQ_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" --mixes main,all_create,all_create#2,all_create#3 > gpurun_out/f_diag.log 2>&1 || { tail -20 gpurun_out/f_diag.log; exit 1; }
grep -E "^===|^---|check|/" gpurun_out/f_diag/table.txt | cut -c1-260
