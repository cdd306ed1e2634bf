set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
V="nt=,sc1=build/aa16/libgvstore_test.so,ntsc1=build/aa18/libgvstore_test.so,normal=build/aa0/libgvstore_test.so"
for c in FETCH_SIZE WRITE_SIZE; do
timeout -k 10 500 python -u tools/l2_diag.py gpurun_out/t_$c --counters "$c" --variants "$V" --mixes main,main#2,hot_next_rud,all_create,deletes --args "--log2n 21 --batch 65536 --auth" > gpurun_out/t_$c.log 2>&1 || { tail -5 gpurun_out/t_$c.log; exit 1; }
grep -E "^===|k_rpass2|check" gpurun_out/t_$c/table.txt | cut -c1-250
done
