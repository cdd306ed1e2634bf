#!/bin/bash
# Block store / map: the GPU parity tests, then the oram and omap shapes of
# tests/test_oblivious.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${1:-kv_obl}
mkdir -p "$O"
PT="python3 -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $PT tests/test_gpu_oram.py tests/test_gpu_omap.py > "$O/kv_tests.log" 2>&1
rc=$?; echo "kv tests rc=$rc"; tail -3 "$O/kv_tests.log"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 1000 $PT tests/test_oblivious.py -k "oram or omap" > "$O/obl_kv.log" 2>&1
rc=$?; echo "obl kv rc=$rc"; grep -E "^(FAILED|PASSED)|passed|failed" "$O/obl_kv.log" | tail -8
cp gpurun_out/oblivious_*_o*.txt "$O/" 2>/dev/null
echo ALL_DONE
