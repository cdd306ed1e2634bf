set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_oram.py tests/test_gpu_omap.py tests/test_gpu_sharded.py > gpurun_out/a_parity.log 2>&1 && tail -3 gpurun_out/a_parity.log &&
timeout -k 10 300 python -u tools/l2_diag.py gpurun_out/a_diag --counters "TCC_BUBBLE_sum TCP_TCC_READ_REQ_sum TCC_EA0_WRREQ_sum" --mixes main,main#2,hot_next_rud,all_miss_read,deletes > gpurun_out/a_diag.log 2>&1 && tail -40 gpurun_out/a_diag.log &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/a_bench.json 2> gpurun_out/a_bench.err && cat gpurun_out/a_bench.json
