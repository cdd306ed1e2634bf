set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/l2_diag.py gpurun_out/e_diag --counters "TCC_UC_REQ_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_sum" --mixes main,main#2,all_create,all_create#2 --args "--log2n 20 --batch 32768 --shards 2" > gpurun_out/e_diag.log 2>&1 || { tail -20 gpurun_out/e_diag.log; exit 1; }
grep -E "^===|^---|check|/|k_route_dest|k_rpass2s|k_m1x" gpurun_out/e_diag/table.txt | cut -c1-260
timeout -k 10 700 python -u -m pytest -v -m gpu --timeout 300 --timeout-method thread tests/test_oblivious.py -k "WRITE_SIZE or wire" tests/test_timing.py > gpurun_out/e_rest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed|Error" gpurun_out/e_rest.log | tail -20; exit $rc
