cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1 GVS_PIPELINE=2
mkdir -p gpurun_out/v2a
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_targeted.py tests/test_gpu_sharded.py -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/v2a/parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -30 gpurun_out/v2a/parity.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_configs.py -v -k c3 --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/v2a/c3.log 2>&1
rc=$?; echo "c3 rc=$rc"; tail -15 gpurun_out/v2a/c3.log
timeout -k 10 300 python3 -u -m pytest tests/test_timing.py -v --timeout 280 --timeout-method thread -p no:cacheprovider > gpurun_out/v2a/timing.log 2>&1
rc=$?; echo "timing rc=$rc"; cp gpurun_out/timing_c3.txt gpurun_out/v2a/ 2>/dev/null; tail -3 gpurun_out/v2a/timing.log
