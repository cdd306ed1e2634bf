#!/usr/bin/env python3
"""Diagnostic A/B of the byte-counter residues (DESIGN.md §3 "What remains"):
run tools/oblivious_probe.py under `rocprofv3 --pmc <counters>` for several
request mixes and engine builds, and print per kernel and counter the mean over
the seed-controlled measured batches of each mix, as a difference from main.

    python tools/l2_diag.py OUTDIR --counters "C1 C2 ..." \
        [--variants base=,nt=build/diag_nt/libgvstore_test.so] \
        [--mixes main,main#2,all_miss_read,hot_next_rud] [--args "--log2n 20 --batch 65536"]

A variant names a library (GVS_LIB_OVERRIDE; an empty path is the in-tree
test library) and optionally, after "@", GVS_DIAG bits (name=lib@0x400).  Test infrastructure only: nothing here is on the product path.
"""
import argparse
import collections
import csv
import glob
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
PROBE = os.path.join(ROOT, "tools", "oblivious_probe.py")
SEEDS = "1234,99,5"
PER_SEED = 2
N_MEAS = 6


def short(name):
    return name.split("(")[0].replace("void ", "").replace("gvs::", "")


def split(vals, first):
    out, cur, prev = [], None, ""
    for v in vals:
        k = v[0]
        starts = k == first and not (first == "k_route_dest" and prev.startswith("k_route_")
                                     and prev != "k_route_gather")
        prev = k
        if starts:
            if cur:
                out.append(cur)
            cur = []
        if cur is not None:
            cur.append(v)
    if cur:
        out.append(cur)
    return out


def run(outdir, counters, mix, lib, args, timeout, diag=None):
    os.makedirs(outdir, exist_ok=True)
    cmd = (["rocprofv3", "--pmc"] + counters + ["-d", outdir, "-o", "run", "--output-format", "csv", "--",
                                                 sys.executable, PROBE, mix, "--fill-batches", "3",
                                                 "--seeds", SEEDS, "--batches", str(PER_SEED)] + args)
    # the test library, as under pytest (tests/conftest.py): GVS_DIAG variants too
    env = dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp"), GVS_TEST_HOOKS="1")
    if lib:
        env["GVS_LIB_OVERRIDE"] = os.path.join(ROOT, lib)
    if diag:
        env["GVS_DIAG"] = diag
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    if r.returncode != 0:
        sys.exit(f"probe failed ({mix}, {lib}):\n" + r.stdout[-3000:] + r.stderr[-3000:])
    rows = []
    for f in glob.glob(os.path.join(outdir, "**", "*counter_collection.csv"), recursive=True):
        rows += [x for x in csv.DictReader(open(f)) if "gvs::" in x.get("Kernel_Name", "")]
    key = "Dispatch_Id" if "Dispatch_Id" in rows[0] else "Correlation_Id"
    per = collections.defaultdict(dict)
    names = {}
    for x in rows:
        d = int(x[key])
        names[d] = short(x["Kernel_Name"])
        per[d][x["Counter_Name"]] = per[d].get(x["Counter_Name"], 0.0) + float(x["Counter_Value"])
    vals = [(names[d], per[d]) for d in sorted(per)]
    ks = {v[0] for v in vals}
    first = ("k_wire_decode" if "k_wire_decode" in ks else "k_route_dest" if "k_route_dest" in ks else
             "k_bcopy" if "k_bcopy" in ks else "k_ocopy" if "k_ocopy" in ks else "k_copy")
    return split(vals, first)


def check(res, counters, mixes):
    """tests/test_oblivious.py's two checks per kernel and counter (the counter
    in its own unit): noise from the prefill batches across the processes and
    main against main#2; every measured batch within 3x range + FLOOR of main's
    median, every mix's mean within 5 standard errors + BIAS_FLOOR of main's."""
    import math
    FLOOR, BIAS_FLOOR, SIG = 2.0, 0.25, 5.0
    out = []
    ref_b = res["main"]
    n_pre = min(len(b) for b in res.values()) - N_MEAS
    for c in counters:
        bad = []
        for idx, (k, _) in enumerate(ref_b[-1]):
            val = lambda b: b[idx][1].get(c, float("nan"))
            rng, ss, dof = 0.0, 0.0, 0
            for i in range(1, n_pre):
                v = [val(res[m][i]) for m in mixes]
                rng = max(rng, max(v) - min(v))
                ss += statistics.variance(v) * (len(v) - 1)
                dof += len(v) - 1
            if "main#2" in res:
                for x, y in zip(res["main"][1:], res["main#2"][1:]):
                    d = val(x) - val(y)
                    rng = max(rng, abs(d))
                    ss += d * d / 2.0
                    dof += 1
            sigma = math.sqrt(ss / dof) if dof else 0.0
            tol = 3.0 * rng + FLOOR
            main_meas = [val(b) for b in ref_b[-N_MEAS:]]
            ref, mu = statistics.median(main_meas), statistics.fmean(main_meas)
            btol = SIG * sigma * math.sqrt(2.0 / N_MEAS) + BIAS_FLOOR
            for m in mixes:
                meas = [val(b) for b in res[m][-N_MEAS:]]
                dev = max(abs(v - ref) for v in meas)
                bias = statistics.fmean(meas) - mu
                if dev > tol:
                    bad.append(f"{k}/{m}: batch {dev:.2f} > {tol:.2f}")
                if m != "main" and abs(bias) > btol:
                    bad.append(f"{k}/{m}: bias {bias:+.2f} > {btol:.2f}")
        out.append(f"### check {c}: {len(bad)} violation(s)")
        out += ["    " + b for b in bad]
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("outdir")
    p.add_argument("--counters", required=True)
    p.add_argument("--variants", default="base=")
    p.add_argument("--mixes", default="main,main#2,all_miss_read,hot_next_rud")
    p.add_argument("--args", default="--log2n 20 --batch 65536")
    p.add_argument("--timeout", type=int, default=300)
    a = p.parse_args()
    counters = a.counters.split()
    variants = [(v.split("=", 1) + [""])[:2] for v in a.variants.split(",")]
    mixes = a.mixes.split(",")
    lines = []
    for vname, spec in variants:
        lib, _, diag = spec.partition("@")
        res = {}
        for mix in mixes:
            d = os.path.join(a.outdir, f"{vname}_{mix.replace('#', '_')}")
            res[mix] = run(d, counters, mix.split("#")[0], lib, a.args.split(), a.timeout, diag)
            print(f"ran {vname} {mix}: {len(res[mix])} batches", flush=True)
        ref = res["main"][-1]
        lines.append(f"=== variant {vname} ({lib or 'in-tree'}); per kernel: main mean, then mix mean - main mean"
                     f" [per-batch range of the mix]")
        for c in counters:
            lines.append(f"--- {c}")
            for idx, (k, _) in enumerate(ref):
                def meas(m):
                    return [b[idx][1].get(c, float("nan")) for b in res[m][-N_MEAS:]]
                mm = statistics.fmean(meas("main"))
                cells = []
                for m in mixes[1:]:
                    v = meas(m)
                    cells.append(f"{m}:{statistics.fmean(v) - mm:+9.1f}[{min(v) - mm:+.0f},{max(v) - mm:+.0f}]")
                lines.append(f"  {idx:2d} {k[:34]:34s} {mm:12.1f}  " + "  ".join(cells))
        lines += check(res, counters, mixes)
    txt = "\n".join(lines) + "\n"
    with open(os.path.join(a.outdir, "table.txt"), "w") as f:
        f.write(txt)
    print(txt)


if __name__ == "__main__":
    main()
