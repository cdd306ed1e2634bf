#!/usr/bin/env python3
"""HBM traffic per launch of the message-table pass from two rocprofv3 --pmc
runs of bench.py (one FETCH_SIZE pass, one WRITE_SIZE pass, never combined).

Correction per /opt/skills/guides/MI355X_MICROARCH.md (HBM section): both
counters are in KiB; on gfx950 FETCH_SIZE reports half of the bytes of wide
coalesced reads, so bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.  The
message pass streams every row with 16-B-per-lane loads and stores, the case
that calibration covers.

    python tools/traffic_from_pmc.py FETCH_DIR WRITE_DIR LOG2N BATCH [KERNEL [EXPIRY]]
"""
import csv
import glob
import json
import os
import statistics
import sys

from srcsha import source_sha


def per_launch(d, counter, kernel):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel not in r.get("Kernel_Name", "") or r.get("Counter_Name") != counter:
                continue
            key = r.get("Dispatch_Id", r.get("Correlation_Id"))
            vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    if not vals:
        sys.exit(f"no {counter} rows for {kernel} under {d}")
    return list(vals.values())


def main():
    fdir, wdir, log2n, batch = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    kernel = sys.argv[5] if len(sys.argv) > 5 else "k_rpass2s"
    expiry = int(sys.argv[6]) if len(sys.argv) > 6 else 0
    f = per_launch(fdir, "FETCH_SIZE", kernel)
    w = per_launch(wdir, "WRITE_SIZE", kernel)
    # the last launches are the timed C3 batches (the prefill batches run on a
    # partly empty table, same footprint); take the median of the last 5
    fm = statistics.median(f[-5:])
    wm = statistics.median(w[-5:])
    out = {
        "kernel": kernel, "log2n": log2n, "batch": batch, "expiry_per_batch": expiry,
        "source_sha": source_sha(),
        "fetch_kib": fm, "write_kib": wm,
        "read_bytes": 2 * fm * 1024, "write_bytes": wm * 1024,
        "rpass_bytes_per_launch": (2 * fm + wm) * 1024,
        "launches_seen": [len(f), len(w)],
        "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) KiB, MI355X_MICROARCH.md HBM section",
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
