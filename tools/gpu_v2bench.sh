cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1 GVS_PIPELINE=${GVS_PIPELINE:-2}
O=gpurun_out/${1:-v2b}
mkdir -p $O
timeout -k 10 300 python3 bench.py --no-cpu > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cat $O/bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'], d['stage_ms'], d['checks'])"
if [ $rc -ne 0 ]; then tail -20 $O/bench.err; exit $rc; fi
timeout -k 10 300 python3 -u -m pytest tests/test_timing.py -v --timeout 280 --timeout-method thread -p no:cacheprovider > $O/timing.log 2>&1
rc=$?; echo "timing rc=$rc"; cp gpurun_out/timing_c3.txt $O/ 2>/dev/null; tail -3 $O/timing.log
