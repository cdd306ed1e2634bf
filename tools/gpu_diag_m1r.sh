#!/bin/bash
# Attribution of the k_m1r_c all-miss-read FETCH excess: GVS_DIAG variants of the
# test library (tools/gpu_pmc_mix.sh per variant)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export GVS_TEST_HOOKS=1
for d in ${DIAGS:-0 1 2 3}; do
  GVS_DIAG=$d PMC_ARGS="--log2n 20 --batch 65536 --no-check" PMC_RUNS="main:1234 main:99 all_miss_read:1234" \
    PMC_KERN=k_m1r_c,k_vscan_a bash tools/gpu_pmc_mix.sh > /dev/null || exit 1
  mkdir -p gpurun_out/diag_m1r && cp gpurun_out/pmc_mix/table.txt gpurun_out/diag_m1r/diag$d.txt
  echo "== diag $d"; cat gpurun_out/diag_m1r/diag$d.txt
done
