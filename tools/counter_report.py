#!/usr/bin/env python3
"""Summarise gpurun_out/oblivious_<COUNTER>.txt: per kernel, the measured
batches of every mix vs 'main', next to the noise seen across the identical
prefill batches of all mixes."""
import collections
import sys


def load(path):
    data = {}
    for line in open(path):
        if ": " not in line or line.split(": ")[0] not in ("main", "all_create", "all_miss_read", "hot_next", "deletes"):
            continue
        mix, rest = line.rstrip("\n").split(": ", 1)
        toks = rest.replace("Key128, 4096", "Key128_4096").replace("unsigned long, 8192", "u64_8192").split()
        data[mix] = [(t.rsplit("=", 1)[0], float(t.rsplit("=", 1)[1])) for t in toks]
    return data


def per_batch(seq):
    # split at each k_copy launch
    out, cur = [], []
    for k, v in seq:
        if k == "k_copy" and cur:
            out.append(cur)
            cur = []
        cur.append((k, v))
    out.append(cur)
    return out


def main(path, n_measured=3):
    data = load(path)
    batches = {m: per_batch(s) for m, s in data.items()}
    kernels = [k for k, _ in batches["main"][-1]]
    noise = collections.defaultdict(list)
    for m, bs in batches.items():
        for b in bs[:-n_measured]:
            for idx, (k, v) in enumerate(b):
                noise[(idx, k)].append(v)
    print(f"{'kernel':28s} {'prefill range':>16s} " + " ".join(f"{m:>22s}" for m in batches))
    for idx, k in enumerate(kernels):
        vals = noise[(idx, k)]
        rng = f"{min(vals):.0f}..{max(vals):.0f}" if vals else "-"
        cells = []
        for m, bs in batches.items():
            meas = [b[idx][1] for b in bs[-n_measured:]]
            cells.append(f"{min(meas):.0f}..{max(meas):.0f}")
        print(f"{k[:28]:28s} {rng:>16s} " + " ".join(f"{c:>22s}" for c in cells))


if __name__ == "__main__":
    main(sys.argv[1])
