set -e
cd "$GRAFT_REPO_ROOT"
export PMC_RUNS="main:1234 main:99 all_miss_read:1234 all_miss_read:99 all_create:1234 all_create:99"
export PMC_KERN="k_alloc_ring,k_vscan_a,k_rr2_c,k_m2r_c,k_m1x,k_scan_a,k_rpass2"
PMC_OUT=gpurun_out/pmcA PMC_CTRS="SQC_TC_INST_REQ SQC_TC_DATA_READ_REQ TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum" timeout -k 10 500 bash tools/gpu_pmc_mix.sh > gpurun_out/pmcA.txt 2>&1
PMC_OUT=gpurun_out/pmcB PMC_CTRS="TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_REQ_sum SQC_ICACHE_MISSES" timeout -k 10 500 bash tools/gpu_pmc_mix.sh > gpurun_out/pmcB.txt 2>&1
rm -rf gpurun_out/pmcA/*/ gpurun_out/pmcB/*/
echo DONE
