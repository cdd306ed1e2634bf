"""Data-independence of the engine (north_star obliviousness contract,
api/proto/grapevine.proto:120-122): for batches of the same size, the kernel
launch sequence, the grid/workgroup sizes and the HBM byte counters
(rocprofv3 FETCH_SIZE, WRITE_SIZE) must not depend on the request mix.

Shapes: 64K-request batches (the C3 batch, so the multi-tile sorts and every
global merge step run) over a 2^20-message store (2^21 authenticated), plain and authenticated
(DESIGN.md §8); the routed path (2 shards in one process: k_route_* and the
padded all-to-all); the block store and the key-value map;
the expiry sweep; the wire path (decode, schnorrkel check,
store, encode).

Every mix runs tools/oblivious_probe.py under rocprofv3 --pmc in a child
process (one counter per run, never combined with other tracing).  The
measured batches are seed-controlled: SEEDS x PER_SEED batches, the request
generator reseeded before each seed's batches, so a difference between two
mixes can be told from a difference between two draws of the same mix.  The
prefill batches are identical in every process (same seed, same store state):
their spread across the processes, and the difference between main and a
second main process with the same seeds, is the counters' own noise.

Two checks per kernel (DESIGN.md §3 'Results'):
  * every measured batch of every mix lies within 3x the noise range + 2 KiB
    of main's median;
  * no bias: the mean over a mix's measured batches differs from main's mean
    by less than 5 standard errors (sigma pooled from the identical-input
    samples) + 0.25 KiB.  This is the check that caught the all-miss-read
    excess of round 2 (k_m1r_c +20-27 KiB, tests/test_oblivious.py history;
    profiles/r03_oblivious_bias_before.txt).

The environment re-walks the GPU page tables now and then ("A
TLB invalidation nothing in the process causes"): every kernel of one batch
then reads ~140 uncached lines per GiB more.  Each --pmc pass also records
TCC_UC_REQ_sum per dispatch; a process's one batch whose kernels made more
than UC_WALK uncached requests is left out of both checks (exclusions()); the
report lists every batch's count and every exclusion.  A process that
re-walked in every measured batch is measured again in a fresh process
(rewalk_processes())."""
import csv
import ctypes
import glob
import math
import os
import shutil
import statistics
import subprocess
import sys
import time

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = os.path.join(ROOT, "tools", "oblivious_probe.py")
ALL_MIXES = ["main", "rud", "all_create", "all_miss_read", "hot_next", "hot_next_rud", "deletes"]
SHAPES = {
    "plain": dict(args=["--log2n", "20", "--batch", "65536"], mixes=ALL_MIXES),
    # 2^22 messages: 1024-row partitions, 64 transaction slots, so the sealed
    # pass runs its production form (slot lines staged in LDS, 12 waves per
    # workgroup, gvs_spass.h; gvs_engine.hip launch_rpass2) as at C3 / C5
    "auth": dict(args=["--log2n", "22", "--batch", "65536", "--auth"], mixes=ALL_MIXES),
    # hot recipients go through the 2-shard router too: the requests past
    # their routing key's cap are shed (DESIGN.md §6 "Hot keys")
    "routed": dict(args=["--log2n", "20", "--batch", "32768", "--shards", "2"],
                   mixes=["main", "rud", "all_create", "all_miss_read", "hot_next", "hot_next_rud",
                          "deletes"]),
    # the block store and the key-value map (gvs_oram_*, gvs_omap_*, DESIGN.md
    # §10): read-only, write-only, remove-only, insert-only, hot-key, single-block
    # and missing-key mixes (tools/oblivious_probe.py KV_MIXES)
    "oram": dict(args=["--oram", "--log2n", "20", "--batch", "65536"],
                 mixes=["main", "all_read", "all_write", "hot", "chain"]),
    "omap": dict(args=["--omap", "--log2n", "20", "--batch", "65536"],
                 mixes=["main", "all_read", "all_insert", "all_remove", "hot", "miss"]),
    # the same two surfaces sealed (GVS_FLAG_AUTH_STORAGE): the block table
    # through the sealed pass (gvs_spass.h), the map's directory sealed too
    # (README.md:49-50, mc-oblivious's untrusted storage)
    "oram_auth": dict(args=["--oram", "--log2n", "20", "--batch", "65536", "--auth"],
                      mixes=["main", "all_read", "all_write", "hot", "chain"]),
    "omap_auth": dict(args=["--omap", "--log2n", "20", "--batch", "65536", "--auth"],
                      mixes=["main", "all_read", "all_insert", "all_remove", "hot", "miss"]),
    # the expiry sweep (README.md:92-97): the main request mix
    # with nothing, everything, or a few old rows (in a few partitions) past
    # the cutoff (tools/oblivious_probe.py --expiry); main runs without a cutoff
    "expiry": dict(args=["--log2n", "20", "--batch", "65536", "--expiry", "1024"],
                   mixes=["main", "x_all", "x_few"]),
    # the wire path: launches and grids must not depend on forged signatures
    # or malformed messages either; the byte counters of the front-end
    # kernels are compared over requests that verify and decode (canonical or
    # not): a forged or malformed request fails at the gRPC level in the
    # reference (grapevine.proto:57-64), which the host sees.
    "wire": dict(args=["--log2n", "20", "--batch", "16384", "--wire"],
                 mixes=["main", "rud", "wire_forged", "wire_malformed", "wire_noncanonical"],
                 pmc_mixes=["main", "rud", "wire_noncanonical"],
                 pmc_kernels=("k_wire_decode", "sr::k_sr_verify", "k_wire_encode")),
}
FILL_BATCHES = 3
# A batch whose kernels made more uncached L2 requests than half the process's
# first batch (and at least this) re-walked the page tables (an environmental
# GPU TLB invalidation, DESIGN.md §3 "A TLB invalidation nothing in the process
# causes": ~140 per GiB touched); see exclusions() for how such a batch is
# treated.
UC_WALK = 64
SEEDS = (1234, 99, 5)
PER_SEED = 2
N_MEAS = len(SEEDS) * PER_SEED
FLOOR_KIB = 2.0       # per-batch floor (16 lines)
BIAS_FLOOR_KIB = 0.25  # bias floor (2 lines)
BIAS_SIGMAS = 5.0


_HIP = []
_VRAM = {"base": 0, "log": []}


def vram_free():
    """Free device memory (hipMemGetInfo), or None when HIP is unavailable."""
    try:
        if not _HIP:
            _HIP.append(ctypes.CDLL("libamdhip64.so"))
        f, t = ctypes.c_size_t(), ctypes.c_size_t()
        return f.value if _HIP[0].hipMemGetInfo(ctypes.byref(f), ctypes.byref(t)) == 0 else None
    except OSError:
        return None


def quiesce(tag, timeout=90.0, slack=512 << 20):
    """Start a probe process only once the previous one's device memory is back.

    A probe process holds tens of GB of VRAM and pinned memory; releasing
    them after it exits unmaps pages and invalidates GPU TLBs while the next
    probe may already run.  In round 4 one-batch excursions of ~7 KiB (page
    walks, uncached reads counted in FETCH_SIZE) landed twice in the first
    request-reading kernel of the process started right after the first
    one of a shape exited ("What's weak" 2).  Every probe now
    waits until free VRAM is back at the largest value seen this session
    (less `slack`), then one more second; the wait is logged in the report."""
    t0 = time.time()
    free = vram_free()
    while free is not None and free < _VRAM["base"] - slack and time.time() - t0 < timeout:
        time.sleep(0.25)
        free = vram_free()
    if free is not None:
        _VRAM["base"] = max(_VRAM["base"], free)
        time.sleep(1.0)
    _VRAM["log"].append(f"{tag}: waited {time.time() - t0:.1f} s, free {0 if free is None else free >> 20} MiB")


def rocprof(counter, mix, outdir, shape):
    if shutil.which("rocprofv3") is None:
        pytest.skip("rocprofv3 not available")
    os.makedirs(outdir, exist_ok=True)
    quiesce(f"{shape}/{counter}/{mix}")
    cmd = (["rocprofv3", "--pmc", counter, "TCC_UC_REQ_sum", "-d", outdir, "-o", "run", "--output-format", "csv", "--",
            sys.executable, PROBE, mix, "--fill-batches", str(FILL_BATCHES),
            "--seeds", ",".join(map(str, SEEDS)), "--batches", str(PER_SEED)]
           + SHAPES[shape]["args"])
    env = dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp"))
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    files = glob.glob(os.path.join(outdir, "**", "*counter_collection.csv"), recursive=True)
    assert files, outdir
    rows, uc = [], {}
    for f in files:
        for x in csv.DictReader(open(f)):
            if "gvs::" not in x.get("Kernel_Name", ""):
                continue
            key = "Dispatch_Id" if "Dispatch_Id" in x else "Correlation_Id"
            if x.get("Counter_Name") == "TCC_UC_REQ_sum":
                uc[int(x[key])] = float(x["Counter_Value"])
            elif x.get("Counter_Name", counter) == counter:
                rows.append(x)
    key = "Dispatch_Id" if "Dispatch_Id" in rows[0] else "Correlation_Id"
    rows.sort(key=lambda x: int(x[key]))
    # (kernel, grid, workgroup, counter value, uncached L2 requests)
    return [(short(x["Kernel_Name"]), x.get("Grid_Size"), x.get("Workgroup_Size"),
             float(x["Counter_Value"]), uc.get(int(x[key]), 0.0)) for x in rows]


def short(name):
    return name.split("(")[0].replace("void ", "").replace("gvs::", "")


def split_batches(vals):
    """Per-batch lists of (kernel, grid, workgroup, value); launches before
    the first batch (k_seal_init at store creation) are dropped.  Routed
    stores start each batch with the router, one k_route_dest..k_route_fill
    run per source: a batch starts at the k_route_dest that follows a
    non-router kernel."""
    names = {v[0] for v in vals}
    first = ("k_wire_decode" if "k_wire_decode" in names else
             "k_route_dest" if "k_route_dest" in names else
             "k_bcopy" if "k_bcopy" in names else "k_ocopy" if "k_ocopy" in names else "k_copy")
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


_CACHE = {}
_RERUNS = []


def walk_levels(per):
    """{mix: median uncached L2 requests over the process's measured batches}."""
    return {mix: statistics.median(sum(x[4] for x in b) for b in bs[-N_MEAS:]) for mix, bs in per.items()}


def rewalk_processes(per):
    """Processes whose every measured batch re-walked page tables: a measured-
    batch median of uncached L2 requests above 3x the median over all the
    shape's processes (and above UC_WALK).  Seen in one process at a time, a
    different mix in different runs (r05i: expiry x_all; r05r: plain deletes
    and expiry x_few, 300-430 uncached requests in every measured batch against
    20-100, their prefill batches like every other process's), with +0.3-1 KiB
    in a few small kernels.  Such a process is measured again in a fresh
    process, at most twice (the state can outlive one process: r05v, the
    sealed shape's deletes, 318 then 162 against a median of 14, quiet in the
    r05i, r05r and r05u runs); the same rule for every mix, main and main#2
    included, and every re-run is printed in the report.  A byte count that
    follows the mix follows it into the fresh processes too."""
    lv = walk_levels(per)
    med = statistics.median(lv.values())
    return [m for m, v in lv.items() if v > max(UC_WALK, 3.0 * med)]


def measure(shape, counter, tmp_root):
    """{mix: per-batch lists} for every mix of the shape, plus 'main#2' (a
    second main process: identical inputs)."""
    key = (shape, counter)
    if key not in _CACHE:
        mixes = SHAPES[shape]["mixes"] if counter == "FETCH_SIZE" else \
            SHAPES[shape].get("pmc_mixes", SHAPES[shape]["mixes"])  # FETCH runs also serve the launch check
        res = {}
        for mix in list(mixes) + ["main#2"]:
            m = mix.split("#")[0]
            d = os.path.join(tmp_root, f"{shape}_{counter}_{mix.replace('#', '_')}")
            res[mix] = split_batches(rocprof(counter, m, d, shape))
        # a process that re-walked the page tables in every measured batch is
        # measured again in a fresh process, at most twice (rewalk_processes())
        for attempt in range(2):
            for mix in rewalk_processes(res):
                m = mix.split("#")[0]
                d = os.path.join(tmp_root, f"{shape}_{counter}_{mix.replace('#', '_')}_again{attempt}")
                levels = walk_levels(res)
                res[mix] = split_batches(rocprof(counter, m, d, shape))
                _RERUNS.append(f"{shape}/{counter}/{mix}: measured-batch walk level {levels[mix]:.0f} against a "
                               f"median of {statistics.median(levels.values()):.0f}; again: "
                               f"{walk_levels(res)[mix]:.0f}")
        _CACHE[key] = res
    return _CACHE[key]


@pytest.fixture(scope="module")
def tmp_root(tmp_path_factory):
    return str(tmp_path_factory.mktemp("obl"))


@pytest.mark.parametrize("shape", sorted(SHAPES))
def test_launch_sequence_and_grids_identical(shape, tmp_root):
    """Every batch of every mix launches the same kernels with the same grids
    and workgroups, in the same order (from the FETCH_SIZE runs' dispatch
    records)."""
    per = measure(shape, "FETCH_SIZE", tmp_root)
    ref = per["main"]
    seq = [(k, g, w) for k, g, w, *_ in ref[-1]]
    assert len(seq) > (15 if shape.startswith("oram") else 30)
    names = {k for k, _, _ in seq}
    assert any(n.startswith("k_bitonic_global") for n in names), sorted(names)
    if shape == "routed":
        assert {"k_route_dest", "k_route_pos", "k_route_copy", "k_route_fill",
                "k_route_gather"} <= names, sorted(names)
    if shape == "wire":
        assert {"k_wire_decode", "sr::k_sr_verify", "k_wire_encode"} <= names, sorted(names)
    for mix, bs in per.items():
        for i, b in enumerate(bs[1:], 1):
            assert [(k, g, w) for k, g, w, *_ in b] == seq, f"{shape}: {mix} batch {i} launches differ"


def exclusions(per):
    """{mix: {batch index}}: the one measured batch of a process that re-walked
    the page tables, if one did.

    The rule ("Next round" 2): the uncached L2 requests
    (TCC_UC_REQ_sum) are recorded in the same --pmc pass as the byte counter,
    for every dispatch; a measured batch whose kernels made more than UC_WALK
    of them is a re-walk; the rule is the same for every mix (main and main#2
    included); at most one batch per process is set aside, and only when it is
    the process's only re-walk among its measured batches (two or more are all
    kept: the test then fails on them); every exclusion is printed in the
    report.  The prefill batches are not candidates: the first two of every
    process touch their pages for the first time (~4000 walks each, the same in
    every process: identical inputs), and they enter only the noise estimate."""
    out = {}
    for mix, bs in per.items():
        n0 = len(bs) - N_MEAS
        uc = [sum(x[4] for x in b) for b in bs]
        # a re-walk touches every page the batch's kernels touch, as the
        # process's first batch did on first touch: half of that is the bar
        # (hot mixes make up to ~230 uncached requests in every batch)
        bar = max(UC_WALK, uc[0] / 2)
        walks = [i for i in range(n0, len(bs)) if uc[i] > bar]
        out[mix] = set(walks) if len(walks) == 1 else set()
    return out


def noise_stats(per, idx, excl):
    """(range, sigma) of kernel `idx` over identical-input samples: the
    prefill batches (batch 0 excluded: cold start) across every process, and
    main against main#2 over every batch.  sigma is pooled from the sample
    variances of those groups.  Batches in `excl` are left out."""
    n_pre = min(len(bs) for bs in per.values()) - N_MEAS
    rng, ss, dof = 0.0, 0.0, 0
    for i in range(1, n_pre):
        vals = [bs[i][idx][3] for m, bs in per.items() if i not in excl[m]]
        if not vals:
            continue
        rng = max(rng, max(vals) - min(vals))
        if len(vals) > 1:
            ss += statistics.variance(vals) * (len(vals) - 1)
            dof += len(vals) - 1
    for i, (a, b) in enumerate(zip(per["main"][1:], per["main#2"][1:]), 1):
        if i in excl["main"] or i in excl["main#2"]:
            continue
        d = a[idx][3] - b[idx][3]
        rng = max(rng, abs(d))
        ss += d * d / 2.0
        dof += 1
    return rng, math.sqrt(ss / dof) if dof else 0.0


def report(shape, counter, lines, bad):
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"oblivious_{counter}_{shape}.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")
        f.write(f"violations: {bad}\n")
        f.write("probe starts: " + "; ".join(x for x in _VRAM["log"] if x.startswith(f"{shape}/")) + "\n")
        f.write("re-run processes (page-table re-walks in every measured batch, or a violation): "
                + "; ".join(x for x in _RERUNS if x.startswith(f"{shape}/{counter}/")) + "\n")


MAX_RERUNS = 2  # fresh processes per shape and counter


def evaluate_counters(per, only=None):
    """The two checks per kernel on {process: per-batch lists}: (report lines,
    violations).  A violation is (kernel, process, kind, value, bound[,
    measured batch, process index])."""
    ref_b = per["main"]
    kernels = [x[0] for x in ref_b[-1]]
    excl = exclusions(per)
    lines, bad = [], []

    def measured(mix, idx):  # (batch index among the measured, value), exclusions left out
        bs = per[mix]
        n0 = len(bs) - N_MEAS
        return [(i - n0, bs[i][idx][3]) for i in range(n0, len(bs)) if i not in excl[mix]]

    for idx, k in enumerate(kernels):
        if only and k not in only:
            continue
        rng, sigma = noise_stats(per, idx, excl)
        tol = 3.0 * rng + FLOOR_KIB
        main_meas = [v for _, v in measured("main", idx)]
        ref = statistics.median(main_meas)
        mu_main = statistics.fmean(main_meas)
        row = [f"{k[:30]:30s} ref={ref:12.1f} range={rng:8.2f} sigma={sigma:7.2f} tol={tol:7.2f}"]
        for mix, bs in per.items():
            assert [x[0] for x in bs[-1]] == kernels, f"{mix}: kernel sequence differs"
            mm = measured(mix, idx)
            meas = [v for _, v in mm]
            # the bias bound: 5 standard errors of the difference of two means
            btol = BIAS_SIGMAS * sigma * math.sqrt(1.0 / len(meas) + 1.0 / len(main_meas)) + BIAS_FLOOR_KIB
            devs = [abs(v - ref) for v in meas]
            dev = max(devs)
            bias = statistics.fmean(meas) - mu_main
            row.append(f"{mix}:{dev:.2f}/{bias:+.2f}")
            if dev > tol:  # with the measured batch's index and the mix's process index
                bad.append((k, mix, "batch", round(dev, 2), round(tol, 2), mm[devs.index(dev)][0],
                            list(per).index(mix)))
            if mix != "main" and abs(bias) > btol:
                bad.append((k, mix, "bias", round(bias, 2), round(btol, 2)))
        lines.append(" ".join(row))
    lines.append("uncached L2 requests per batch (TCC_UC_REQ_sum over the batch's kernels): " + "; ".join(
        f"{mix}: " + ",".join(str(int(sum(x[4] for x in b))) for b in bs) for mix, bs in per.items()))
    lines.append("excluded (re-walk) batches, by batch index in the process: " + "; ".join(
        f"{mix}: {sorted(e)}" for mix, e in excl.items() if e))
    return lines, bad


def rerun_candidates(bad, mixes, fresh=()):
    """Processes a fresh process could settle: those with violations, or main
    (the reference every bias is taken against) when most other mixes fail one
    kernel's bias in the same direction.  Processes already run again are not
    candidates: their violations stand."""
    others = [m for m in mixes if m != "main"]
    if "main" not in fresh:
        for k in {v[0] for v in bad if v[2] == "bias"}:
            # one vote per mix: a kernel name launched several times per batch
            # (the sort stages) must not outvote the other mixes (r06i: six
            # k_bitonic_tile launches of one hot_next process re-ran main)
            signs = {v[1]: math.copysign(1, v[3]) for v in bad if v[0] == k and v[2] == "bias"}
            if len(signs) > len(others) / 2 and abs(sum(signs.values())) == len(signs):
                return ["main"]
    return [m for m in dict.fromkeys(v[1] for v in bad) if m not in fresh]


@pytest.mark.parametrize("shape", sorted(SHAPES))
@pytest.mark.parametrize("counter", ["FETCH_SIZE", "WRITE_SIZE"])
def test_hbm_bytes_identical(counter, shape, tmp_root):
    """Per kernel, the byte counter of every measured batch of every mix lies
    within 3x the counter's identical-input noise range + 2 KiB of main's
    median, and no mix is biased against main (mean over its measured batches
    within 5 standard errors + 0.25 KiB).

    A process with a violation is measured again once in a fresh process (at
    most MAX_RERUNS per shape and counter, printed in the report), and the
    fresh process must pass: the inputs are seed-controlled, so a byte count
    that follows the data follows it into the fresh process; a one-batch
    excursion of the environment does not (r06h: one `rud` batch of the sealed
    pass wrote +16 KiB of 4.55 GB, the other five batches within 0.25 KiB)."""
    per = measure(shape, counter, tmp_root)
    keep = set(SHAPES[shape].get("pmc_mixes", SHAPES[shape]["mixes"])) | {"main#2"}
    per = {m: bs for m, bs in per.items() if m in keep}
    only = SHAPES[shape].get("pmc_kernels")
    lines, bad = evaluate_counters(per, only)
    fresh = []
    while bad and len(fresh) < MAX_RERUNS:
        cand = rerun_candidates(bad, list(per), fresh)[:MAX_RERUNS - len(fresh)]
        if not cand:
            break
        for m in cand:
            d = os.path.join(tmp_root, f"{shape}_{counter}_{m.replace('#', '_')}_fresh")
            before = [v for v in bad if v[1] == m][:4]
            per[m] = split_batches(rocprof(counter, m.split("#")[0], d, shape))
            _CACHE[(shape, counter)][m] = per[m]
            fresh.append(m)
            _RERUNS.append(f"{shape}/{counter}/{m}: violations {before}; measured again in a fresh process")
        lines, bad = evaluate_counters(per, only)
    report(shape, counter, lines, bad)
    if bad:
        pytest.fail(f"{shape} {counter} depends on the request mix: {bad[:16]}\nrun again: {fresh}", pytrace=False)
