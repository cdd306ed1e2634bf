set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/l2_diag.py gpurun_out/l_diag --counters "FETCH_SIZE" --variants "base=,oldnt=build/oldnt/libgvstore_test.so,drop16=build/drop16/libgvstore_test.so" --mixes main,main#2,all_create,deletes,hot_next_rud --args "--log2n 21 --batch 65536 --auth" > gpurun_out/l_diag.log 2>&1 || { tail -20 gpurun_out/l_diag.log; exit 1; }
grep -E "^===|k_rpass2|check" gpurun_out/l_diag/table.txt | cut -c1-260
