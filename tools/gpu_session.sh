#!/bin/bash
# One GPU session: gpu_session.sh TAG MODE.  Output under gpurun_out/TAG.
#   tests    the GPU test suite without the long obliviousness/timing tests
#   timing   the C3 per-kernel duration test
#   bench    bench.py (default workload)
#   obl      the obliviousness counter tests (plain shapes)
#   all      tests, bench, timing
#   seal     the sealed-storage GPU tests (message store, block store, map, epoch limit)
#   sealobl  seal, then the sealed shape's counter tests and a sealed bench line
#   driver   the driver's round-end command (pytest tests/ -x -q -m gpu)
# Each GPU step runs under its own time limit.  A pytest exit status of 1
# means failed tests (recorded, the session goes on); anything else (time
# limit, abort, crash) ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/$1
mkdir -p "$O"
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2
  shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -4 "$O/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name"; exit $rc; fi
}
PT="python3 -u -m pytest -v --timeout 600 --timeout-method thread -p no:cacheprovider"
tests() { step gpu_tests 600 $PT tests -m gpu --ignore=tests/test_oblivious.py --ignore=tests/test_timing.py "$@"; }
timing() { step timing_c3 300 $PT tests/test_timing.py; cp gpurun_out/timing_c3.txt "$O/" 2>/dev/null; }
bench() { step bench 300 python3 bench.py; }
SEALT="tests/test_gpu_seal.py tests/test_gpu_oram.py tests/test_gpu_omap.py tests/test_gpu_epoch.py"
case "$2" in
  seal) step seal_tests 600 $PT $SEALT ;;
  sealobl) step seal_tests 600 $PT $SEALT && \
    step oblivious_auth 900 $PT tests/test_oblivious.py -k "auth and not oram_auth and not omap_auth" && \
    step bench_auth 400 python3 bench.py --auth --no-cpu --steps 5 ;;
  plaintime)  # the plain pass's timing and counters, then the C3 bench line
    step timing_store 600 $PT tests/test_timing.py -k "independent_of_mix and not sealed and not routed"
    cp gpurun_out/timing_c3_store.txt "$O/" 2>/dev/null
    step oblivious_plain 600 $PT tests/test_oblivious.py -k "plain"
    step bench 400 python3 bench.py --no-cpu ;;
  sealperf)  # the sealed tests, the sealed bench at 12 and 8 waves
    step seal_tests 600 $PT $SEALT
    step bench_auth12 400 python3 bench.py --auth --no-cpu --steps 5 --sealed-waves 12
    step bench_auth8 400 python3 bench.py --auth --no-cpu --steps 5 --sealed-waves 8 ;;
  contract)  # every counter and timing shape
    step oblivious_all 1200 $PT tests/test_oblivious.py
    step timing_all 900 $PT tests/test_timing.py
    cp gpurun_out/timing_c3_*.txt "$O/" 2>/dev/null ;;
  sealab)  # sealed pass A/B: library builds ab/libgvstore_VAR.so x waves (SEALAB="VAR:WAVES ...")
    for v in ${SEALAB:-nb2:12 nb4:12 nb8:12 nosync_nb2:12 nosync_nb4:12 nb2:8 nb4:8}; do
      lib=${v%%:*}; nw=${v##*:}
      GVS_LIB_OVERRIDE=ab/libgvstore_$lib.so step bench_auth_${lib}_nw$nw 300 \
        python3 bench.py --auth --no-cpu --steps 5 --host-steps 0 --wire-steps 0 --sealed-waves $nw
    done ;;
  sealrw)  # the sealed tests, the sealed A/B (SEALAB), then the routed and wire counter shapes
    step seal_tests 600 $PT $SEALT && \
    for v in ${SEALAB:-dual:12 nodual:12 m2a1:12}; do
      lib=${v%%:*}; nw=${v##*:}
      GVS_LIB_OVERRIDE=ab/libgvstore_$lib.so step bench_auth_${lib}_nw$nw 300 \
        python3 bench.py --auth --no-cpu --steps 5 --host-steps 0 --wire-steps 0 --sealed-waves $nw
    done && \
    step obl_rw 900 $PT tests/test_oblivious.py -k "routed or wire"
    cp gpurun_out/oblivious_*_routed.txt gpurun_out/oblivious_*_wire.txt "$O/" 2>/dev/null ;;
  fixcheck)  # the GPU suite (no counters/timing), routed counters, routed and store timing, the bench line
    tests && \
    step obl_routed 600 $PT tests/test_oblivious.py -k "routed" && \
    step timing_rs 600 $PT tests/test_timing.py -k "routed or (independent_of_mix and not sealed)" && \
    step bench 400 python3 bench.py --no-cpu
    cp gpurun_out/timing_c3_*.txt gpurun_out/oblivious_*_routed.txt "$O/" 2>/dev/null ;;
  timeab)  # routed and store timing for the in-tree build and each ab/ library in TIMEAB
    step timing_rs_base 600 $PT tests/test_timing.py -k "routed or (independent_of_mix and not sealed)"
    for f in gpurun_out/timing_c3_*.txt; do cp "$f" "$O/base_$(basename $f)"; done
    for lib in ${TIMEAB:-even}; do
      GVS_LIB_OVERRIDE=ab/libgvstore_$lib.so step timing_rs_$lib 600 $PT tests/test_timing.py -k "routed or (independent_of_mix and not sealed)"
      for f in gpurun_out/timing_c3_*.txt; do cp "$f" "$O/${lib}_$(basename $f)"; done
    done ;;
  admit)  # the GPU suite (no counters/timing), then every timing shape
    tests && \
    step timing_all 900 $PT tests/test_timing.py
    cp gpurun_out/timing_c3_*.txt "$O/" 2>/dev/null ;;
  mbox)  # the plain bench line at several mailbox partition sizes
    for sr in ${MBOX:-256 512 1024}; do
      step bench_mbox$sr 300 python3 bench.py --no-cpu --host-steps 0 --wire-steps 0 --mailbox-slots $sr
    done ;;
  sealchk)  # the sealed tests, the sealed counter shapes, the sealed bench line
    step seal_tests 600 $PT $SEALT && \
    step oblivious_auth 900 $PT tests/test_oblivious.py -k "auth" && \
    step bench_auth 400 python3 bench.py --auth --no-cpu --steps 5 --host-steps 0 --wire-steps 0
    cp gpurun_out/oblivious_*_auth.txt "$O/" 2>/dev/null ;;
  srprof)  # the signature and wire tests, the wire counters, then the profiling session
    step sr_tests 600 $PT tests/test_gpu_sr25519.py tests/test_gpu_wire.py && \
    step obl_wire 600 $PT tests/test_oblivious.py -k "wire" && \
    cp gpurun_out/oblivious_*_wire.txt "$O/" && \
    bash "$0" "$1" prof ;;
  tprof)  # the GPU suite without counters/timing, then the profiling session
    tests && bash "$0" "$1" prof ;;
  scrubab)  # sealed FETCH_SIZE counters: in-tree build, then each ab/ library in SCRUBAB
    step fetch_auth_base 600 $PT tests/test_oblivious.py -k "FETCH_SIZE and auth"
    for f in gpurun_out/oblivious_FETCH_SIZE_*auth.txt; do cp "$f" "$O/base_$(basename $f)"; done
    for lib in ${SCRUBAB:-scrub}; do
      GVS_LIB_OVERRIDE=ab/libgvstore_$lib.so step fetch_auth_$lib 600 $PT tests/test_oblivious.py -k "FETCH_SIZE and auth"
      for f in gpurun_out/oblivious_FETCH_SIZE_*auth.txt; do cp "$f" "$O/${lib}_$(basename $f)"; done
    done ;;
  spassnoise)  # request-level counters of the sealed pass over identical and differing inputs
    PMC_OUT="$O/pmc" PMC_ARGS="--oram --log2n 20 --batch 65536 --auth" PMC_KERN=k_spass \
      PMC_CTRS="${SPN_CTRS:-TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_UC_REQ_sum TCC_HIT_sum}" \
      PMC_RUNS="${SPN_RUNS:-main:1234 main:99 all_read:1234 all_write:1234 all_write:99}" \
      step pmc_spass 900 bash tools/gpu_pmc_mix.sh
    find "$O/pmc" -mindepth 1 -maxdepth 1 -type d -exec rm -rf {} + ;;
  rollab)  # the sealed pass's requests and speed: the in-tree build against ab/libgvstore_roll.so
    GVS_LIB_OVERRIDE=ab/libgvstore_roll.so SPN_CTRS="SQC_TC_INST_REQ SQ_INSTS_VALU TCC_EA0_RDREQ_sum TCC_HIT_sum" \
      bash "$0" "$1/roll" spassnoise && \
    step bench_auth_base 300 python3 bench.py --auth --no-cpu --steps 5 --host-steps 0 --wire-steps 0 && \
    GVS_LIB_OVERRIDE=ab/libgvstore_roll.so step bench_auth_roll 300 \
      python3 bench.py --auth --no-cpu --steps 5 --host-steps 0 --wire-steps 0 ;;
  allfinal)  # the GPU suite without counters/timing, the profiling session, then the driver's command, smoke and bench lines
    tests && bash "$0" "$1" prof && bash "$0" "$1" final ;;
  sealmac)  # the GPU suite without counters/timing, the map and sealed counter shapes, the sealed bench line
    tests && \
    step obl_map 900 $PT tests/test_oblivious.py -k "omap or (auth and not oram)" && \
    step bench_auth 400 python3 bench.py --auth --no-cpu --steps 5 --host-steps 0 --wire-steps 0
    cp gpurun_out/oblivious_*omap*.txt gpurun_out/oblivious_*_auth.txt "$O/" 2>/dev/null ;;
  m21ab)  # the fused mailbox pass: production and the diagnostic builds in ab/ (M21AB="VAR ...")
    step bench_base 300 python3 bench.py --no-cpu --host-steps 0 --wire-steps 0 --steps 10
    for v in ${M21AB:-m21s m21p}; do
      GVS_LIB_OVERRIDE=ab/libgvstore_$v.so step bench_$v 300 python3 bench.py --no-cpu --host-steps 0 --wire-steps 0 --steps 10
    done
    for f in "$O"/bench_*.log; do echo "$f"; grep '^{"metric"' "$f" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3), {k: round(v,3) for k, v in d['stage_ms'].items()})"; done ;;
  fusecheck)  # the GPU suite without counters/timing, the store's timing and plain counters, a bench line
    tests && \
    step timing_store 600 $PT tests/test_timing.py -k "independent_of_mix and not sealed and not routed" && \
    step obl_plain 600 $PT tests/test_oblivious.py -k "plain" && \
    step bench 400 python3 bench.py --no-cpu
    cp gpurun_out/timing_c3_store*.txt gpurun_out/oblivious_*_plain.txt "$O/" 2>/dev/null ;;
  ttime)  # the GPU suite without counters/timing, then every timing shape with per-test durations
    tests && \
    step timing_all 1000 $PT --durations=0 tests/test_timing.py
    cp gpurun_out/timing_c3_*.txt "$O/" 2>/dev/null ;;
  timeall)  # every timing shape, then the default bench line
    step timing_all 1000 $PT tests/test_timing.py
    cp gpurun_out/timing_c3_*.txt "$O/" 2>/dev/null
    step bench 400 python3 bench.py --no-cpu ;;
  routed)  # the sharded path: parity, counters, timing
    step sharded_tests 600 $PT tests/test_gpu_sharded.py
    step obl_routed 900 $PT tests/test_oblivious.py -k "routed"
    step timing_routed 600 $PT tests/test_timing.py -k "routed"
    cp gpurun_out/timing_c3_routed.txt gpurun_out/oblivious_FETCH_SIZE_routed.txt gpurun_out/oblivious_WRITE_SIZE_routed.txt "$O/" 2>/dev/null ;;
  kplain)  # per-kernel stats of the device-buffer C3 batches alone (no host or wire paths)
    step kstats_plain 400 rocprofv3 --kernel-trace --stats -d "$O/kp" -o run --output-format csv -- \
      python3 bench.py --no-cpu --host-steps 0 --wire-steps 0 --steps 10 --warmup 2
    find "$O/kp" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats_plain.csv" \;
    rm -rf "$O/kp" ;;
  kauth)  # the same for the sealed store
    step kstats_auth 400 rocprofv3 --kernel-trace --stats -d "$O/ka" -o run --output-format csv -- \
      python3 bench.py --auth --no-cpu --host-steps 0 --wire-steps 0 --steps 5 --warmup 2
    find "$O/ka" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats_auth.csv" \;
    rm -rf "$O/ka" ;;
  authsq) step auth_sq 900 bash tools/gpu_auth_sq.sh "$1/sq" ;;
  driver) step driver_x 1100 python3 -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread ;;
  final)  # the driver's round-end command, then smoke()
    step driver_x 1100 python3 -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread
    cp gpurun_out/oblivious_*.txt gpurun_out/timing_c3_*.txt "$O/" 2>/dev/null
    step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
    step bench 400 python3 bench.py
    step bench_auth 400 python3 bench.py --auth --no-cpu --steps 5 ;;
  tests) tests ;;
  timing) timing ;;
  bench) bench ;;
  obl) step oblivious 1100 $PT tests/test_oblivious.py -k "plain or launch" ;;
  tobl) tests && step oblivious 900 $PT tests/test_oblivious.py -k "plain or launch" ;;
  oblx) step oblivious_x 1000 $PT tests/test_oblivious.py -k "auth or routed" ;;
  tdiag) tests && bash "$0" "$1" m2diag ;;
  m2diag)  # write/read request counters of the auth mailbox pass under two mixes
    PMC_ARGS=--auth PMC_KERN=k_m2x,k_rpass2 PMC_CTRS="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_HIT_sum TCC_MISS_sum" \
      step pmc_mix 400 bash tools/gpu_pmc_mix.sh
    step oblivious_x 1000 $PT tests/test_oblivious.py -k "auth or routed" ;;
  probe) step hbm_probe 300 tools/hbm_probe 16 ;;
  tob) tests && step oblivious_all 1000 $PT tests/test_oblivious.py && step hbm_probe 300 tools/hbm_probe 16 && bench ;;
  oblall) step oblivious_all 1150 $PT tests/test_oblivious.py ;;
  oblplain)  # plain-shape counters, then L2 hit/miss per kernel for two mixes
    step oblivious_plain 900 $PT tests/test_oblivious.py -k "plain"
    PMC_KERN=${PMC_KERN:-k_vscan_a,k_rr2_c,k_m2r_c,k_bitonic_global2,k_m1x,k_scan_c} \
      step pmc_mix 400 bash tools/gpu_pmc_mix.sh ;;
  all) tests && bench && timing ;;
  full) tests && timing && step oblivious_all 1150 $PT tests/test_oblivious.py ;;
  ktraffic)  # HBM traffic per launch of the headline path's larger kernels (two PMC passes, device batches only)
    BA="python3 bench.py --no-cpu --steps 5 --warmup 1 --host-steps 0 --wire-steps 0"
    step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch" -o run --output-format csv -- $BA && \
    step pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write" -o run --output-format csv -- $BA && \
    for k in k_rpass2s k_m21x k_m1r_c k_rr2_c "k_vscan_a<gvs::Rr2Op>" k_copy k_out k_meta k_alloc_ring; do
      python3 tools/traffic_from_pmc.py "$O/pmc_fetch" "$O/pmc_write" 24 65536 "$k" > "$O/traffic_$(echo $k | tr -c 'a-zA-Z0-9_\n' '_').json"
    done
    rm -rf "$O/pmc_fetch" "$O/pmc_write" ;;
  prof)  # HBM traffic of k_rpass2 (two PMC passes), kernel stats, auth and expiry lines
    step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch" -o run --output-format csv -- python3 bench.py --no-cpu --steps 5 --warmup 1
    step pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write" -o run --output-format csv -- python3 bench.py --no-cpu --steps 5 --warmup 1
    python3 tools/traffic_from_pmc.py "$O/pmc_fetch" "$O/pmc_write" 24 65536 k_rpass2s > "$O/traffic_latest.json" && cp "$O/traffic_latest.json" profiles/traffic_latest.json
    rm -rf "$O/pmc_fetch" "$O/pmc_write"
    step kstats 600 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- python3 bench.py --no-cpu
    find "$O/prof" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats.csv" \;
    find "$O/prof" -name "*kernel_trace.csv" -delete
    step bench_full 300 python3 bench.py
    step pmc_valu 600 rocprofv3 --pmc SQ_INSTS_VALU -d "$O/pmc_valu" -o run --output-format csv -- python3 bench.py --auth --no-cpu --steps 5 --warmup 1
    python3 tools/valu_from_pmc.py "$O/pmc_valu" 24 65536 k_spass > "$O/valu_auth_latest.json" && cp "$O/valu_auth_latest.json" profiles/
    step predict 600 python3 bench.py --predict-shards 8 --steps 3 --warmup 1
    grep '^{"metric": "predicted' "$O/predict.log" | tail -1 > "$O/scale_prediction.json" && \
      python3 -c "import json; d=json.load(open('$O/scale_prediction.json')); json.dump(d, open('profiles/scale_prediction.json','w'), indent=1)"
    rm -rf "$O/pmc_valu"
    step bench_auth 600 python3 bench.py --auth --no-cpu --steps 5
    step bench_expiry 300 python3 bench.py --expiry 1024 --no-cpu
    step kstats_auth 400 rocprofv3 --kernel-trace --stats -d "$O/ka" -o run --output-format csv -- \
      python3 bench.py --auth --no-cpu --host-steps 0 --wire-steps 0 --steps 5 --warmup 2
    find "$O/ka" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats_auth.csv" \;
    rm -rf "$O/ka" ;;
esac
echo ALL_DONE
