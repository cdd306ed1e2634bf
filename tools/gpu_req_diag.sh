#!/bin/bash
# Request counters per kernel and mix (tools/req_table.py): vector read/write
# requests to L2, instruction requests, 128-B memory reads.  A kernel whose
# request counts move with the mix has an address or code path that follows
# the data.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/req
rm -rf "$O"; mkdir -p "$O"
RUNS=${REQ_RUNS:-main:1234 main:99 all_miss_read:1234 all_create:1234 hot_next:1234 deletes:1234}
ARGS=${REQ_ARGS:---log2n 20 --batch 65536}
for r in $RUNS; do
  mix=${r%%:*}; seed=${r##*:}
  timeout -k 10 300 rocprofv3 --pmc SQC_TC_INST_REQ TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCC_EA0_RDREQ_128B_sum \
    -d "$O/${mix}_$seed" -o run --output-format csv -- \
    python3 tools/oblivious_probe.py $mix --seed $seed --fill-batches 3 --batches 2 $ARGS > "$O/${mix}_$seed.log" 2>&1 || exit 1
done
REQ_RUNS="$RUNS" python3 tools/req_table.py "$O" > "$O/table.txt"
find "$O" -mindepth 1 -type d -exec rm -rf {} +
cat "$O/table.txt"
