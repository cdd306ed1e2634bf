set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/l2_diag.py gpurun_out/x_diag --counters "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum TCC_UC_REQ_sum" --mixes main,main#2,hot_next_rud,all_miss_read > gpurun_out/x_diag.log 2>&1 || { tail -5 gpurun_out/x_diag.log; exit 1; }
grep -E "^---|k_m2x" gpurun_out/x_diag/table.txt | cut -c1-250
timeout -k 10 500 python -u tools/l2_diag.py gpurun_out/x_diag2 --counters "TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum" --mixes main,main#2,hot_next_rud,all_miss_read > gpurun_out/x_diag2.log 2>&1 || { tail -5 gpurun_out/x_diag2.log; exit 1; }
grep -E "^---|k_m2x" gpurun_out/x_diag2/table.txt | cut -c1-250
