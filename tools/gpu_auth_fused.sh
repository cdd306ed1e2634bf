#!/bin/bash
# Sealed message pass, interleaved crypto: seal parity tests, then the C5-mode
# bench line with and without the interleaving (same build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${1:-auth_fused}
mkdir -p "$O"
PT="python3 -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $PT tests/test_gpu_seal.py tests/test_expiry.py -m gpu > "$O/seal_tests.log" 2>&1
rc=$?; echo "seal tests rc=$rc"; tail -3 "$O/seal_tests.log"
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python3 bench.py --auth --no-cpu --steps 5 --warmup 2 > "$O/bench_auth_fused.json" 2> "$O/bench_auth_fused.err" || exit 1
timeout -k 10 300 python3 bench.py --auth --no-cpu --steps 5 --warmup 2 --sealed-fused 0 > "$O/bench_auth_phased.json" 2> "$O/bench_auth_phased.err" || exit 1
python3 - "$O" <<'P'
import json, sys
for n in ("fused", "phased"):
    d = json.loads(open(f"{sys.argv[1]}/bench_auth_{n}.json").read().strip().splitlines()[-1])
    print(n, round(d["value"]), "req/s", round(d["ms_per_step"], 2), "ms", d["roofline"].get("kernel_ms"), d.get("stage_ms", {}).get("rpass"))
P
echo ALL_DONE
