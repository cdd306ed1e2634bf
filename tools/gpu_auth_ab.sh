#!/bin/bash
# Sealed-pass A/B: seal parity tests (4- and 8-wave passes), the C5 config
# test, then bench --auth with 8 and with 4 waves per workgroup.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${1:-auth_ab}
mkdir -p "$O"
PT="python3 -u -m pytest -v --timeout 600 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 $PT tests/test_gpu_seal.py > "$O/seal_tests.log" 2>&1
rc=$?; echo "seal tests rc=$rc"; tail -3 "$O/seal_tests.log"
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 500 $PT tests/test_gpu_configs.py -k c5 > "$O/c5.log" 2>&1
rc=$?; echo "c5 rc=$rc"; tail -3 "$O/c5.log"
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 400 python3 bench.py --auth --no-cpu --steps 5 --warmup 2 --host-steps 0 --wire-steps 0 > "$O/bench_auth8.json" 2> "$O/bench_auth8.err" || exit $?
timeout -k 10 400 python3 bench.py --auth --no-cpu --steps 5 --warmup 2 --host-steps 0 --wire-steps 0 --sealed-waves 4 > "$O/bench_auth4.json" 2> "$O/bench_auth4.err" || exit $?
echo ALL_DONE
