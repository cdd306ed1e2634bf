# round-end rehearsal: smoke, the driver's -m gpu -x suite, the default bench line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/u_smoke.log 2>&1; echo "smoke rc=$?"; tail -1 gpurun_out/u_smoke.log
timeout -k 10 1000 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/u_gpu_x.log 2>&1; echo "suite rc=$?"; tail -3 gpurun_out/u_gpu_x.log
