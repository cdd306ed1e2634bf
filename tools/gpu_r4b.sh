set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/l2_diag.py gpurun_out/b_diag --counters "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_BUBBLE_sum" --variants "base=,nts0=build/nts0/libgvstore_test.so,old=@0x400" --mixes main,main#2,all_create,rud,deletes > gpurun_out/b_diag.log 2>&1
rc=$?; grep -E "k_rpass2|^===|^---|check|/" gpurun_out/b_diag/table.txt | cut -c1-250; exit $rc
