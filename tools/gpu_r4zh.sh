# round-4 end: smoke(), the sealed-storage and expiry bench lines at HEAD
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r04zh
timeout -k 10 240 python3 -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/r04zh/smoke.log 2>&1 || { tail -20 gpurun_out/r04zh/smoke.log; exit 1; }
tail -1 gpurun_out/r04zh/smoke.log
timeout -k 10 400 python3 bench.py --auth --no-cpu --steps 5 --warmup 2 > gpurun_out/r04zh/bench_auth.json 2> gpurun_out/r04zh/bench_auth.err || { tail -5 gpurun_out/r04zh/bench_auth.err; exit 1; }
timeout -k 10 300 python3 bench.py --expiry 1024 --no-cpu > gpurun_out/r04zh/bench_expiry.json 2> gpurun_out/r04zh/bench_expiry.err || { tail -5 gpurun_out/r04zh/bench_expiry.err; exit 1; }
python3 -c "
import json
for f in ('bench_auth','bench_expiry'):
    d=json.load(open('gpurun_out/r04zh/'+f+'.json')); print(f, d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'))"
