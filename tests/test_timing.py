"""Timing side of the obliviousness contract (api/proto/grapevine.proto:120-122:
READ, UPDATE and DELETE must be indistinguishable in access patterns *and
timings*) at the headline shape, BASELINE config 3: a 2^24-message store and
64K-request batches.

Each mix runs tools/oblivious_probe.py under `rocprofv3 --kernel-trace`; every
kernel's duration on the measured batches must match the reference mix within
the run-to-run noise, taken from the prefill batches that every process runs
identically.  The mixes include adversarial ones: every request aimed at one
recipient (hot_next, hot_next_rud), every read missing (all_miss_read), only
deletes.  A pass whose workgroups did work in proportion to the ops routed to
them would show the hot mixes here."""
import csv
import glob
import os
import shutil
import statistics
import subprocess
import sys

import pytest

from test_oblivious import PROBE, short, split_batches

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MIXES = ["rud", "main", "hot_next", "hot_next_rud", "all_miss_read", "deletes", "all_create"]
ARGS = ["--log2n", "24", "--batch", "65536", "--identities", "200000", "--fill-batches", "4"]
N_MEAS = 3


def kernel_trace(mix, outdir):
    """(kernel, duration us) of every gvs kernel of one probe process."""
    if shutil.which("rocprofv3") is None:
        pytest.skip("rocprofv3 not available")
    os.makedirs(outdir, exist_ok=True)
    cmd = (["rocprofv3", "--kernel-trace", "-d", outdir, "-o", "run", "--output-format", "csv", "--",
            sys.executable, PROBE, mix] + ARGS)
    env = dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp"))
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    rows = []
    for f in glob.glob(os.path.join(outdir, "**", "*kernel_trace.csv"), recursive=True):
        rows += [x for x in csv.DictReader(open(f)) if "gvs::" in x.get("Kernel_Name", "")]
    key = "Dispatch_Id" if "Dispatch_Id" in rows[0] else "Correlation_Id"
    rows.sort(key=lambda x: int(x[key]))
    return [(short(x["Kernel_Name"]), (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3)
            for x in rows]


def test_kernel_durations_independent_of_mix(tmp_path):
    per_mix = {}
    for mix in MIXES:
        per_mix[mix] = [[(k, v) for k, _, _, v in b] for b in
                        split_batches([(k, None, None, v) for k, v in kernel_trace(mix, str(tmp_path / mix))])]
    ref_b = per_mix["rud"]
    kernels = [k for k, _ in ref_b[-1]]
    n_pre = min(len(bs) for bs in per_mix.values()) - N_MEAS
    lines, bad = [], []
    for idx, k in enumerate(kernels):
        # noise: spread of the identical prefill batches (batch 0: cold) across
        # the processes, and of the reference mix's own measured batches
        spread = 0.0
        for i in range(1, n_pre):
            v = [bs[i][idx][1] for bs in per_mix.values()]
            spread = max(spread, max(v) - min(v))
        own = [b[idx][1] for b in ref_b[-N_MEAS:]]
        spread = max(spread, max(own) - min(own))
        ref = statistics.median(own)
        tol = 3.0 * spread + 2.0  # us; +2 us: launch-to-launch jitter floor of the trace clock
        row = [f"{k[:30]:30s} ref={ref:10.1f}us spread={spread:7.1f} tol={tol:7.1f}"]
        for mix, bs in per_mix.items():
            assert [x[0] for x in bs[-1]] == kernels, f"{mix}: kernel sequence differs"
            med = statistics.median(b[idx][1] for b in bs[-N_MEAS:])
            row.append(f"{mix}:{med - ref:+.1f}")
            if abs(med - ref) > tol:
                bad.append((k, mix, round(med - ref, 1), round(tol, 1)))
        lines.append(" ".join(row))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "timing_c3.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")
        f.write(f"violations: {bad}\n")
    assert not bad, f"kernel durations depend on the request mix: {bad}"
