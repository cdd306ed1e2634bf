#!/bin/bash
# L2 hit/miss/request counters per kernel for request mixes (oblivious_probe):
# PMC_RUNS="mix:seed ..." (default main:1234 main:99 all_miss_read:1234 all_miss_read:99)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${PMC_OUT:-gpurun_out/pmc_mix}
mkdir -p "$O"
CTRS=${PMC_CTRS:-TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum}
ARGS=${PMC_ARGS:---log2n 20 --batch 65536}
RUNS=${PMC_RUNS:-main:1234 main:99 all_miss_read:1234 all_miss_read:99}
for r in $RUNS; do
  mix=${r%%:*}; seed=${r##*:}
  timeout -k 10 300 rocprofv3 --pmc $CTRS -d "$O/${mix}_$seed" -o run --output-format csv -- \
    python3 tools/oblivious_probe.py $mix --seed $seed --fill-batches 4 $ARGS > "$O/${mix}_$seed.log" 2>&1 || exit 1
done
PMC_RUNS="$RUNS" PMC_KERN="${PMC_KERN:-k_m1r_c,k_rpass2,k_m2x,k_rr2_c}" python3 tools/pmc_mix_table.py "$O" | tee "$O/table.txt"
