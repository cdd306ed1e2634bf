#!/usr/bin/env python3
"""Vector-ALU instructions per launch of the authenticated message pass from a
rocprofv3 --pmc SQ_INSTS_VALU run of `bench.py --auth`.

SQ_INSTS_VALU counts wave-level VALU instructions, summed over the chip.  The
bench divides it by the pass's HIP-event time for `roofline.achieved` and by
the issue peak (one wave64 instruction per SIMD per 2 cycles) for `frac`.

    python tools/valu_from_pmc.py PMC_DIR LOG2N BATCH [KERNEL]
"""
import json
import statistics
import sys

from srcsha import source_sha
from traffic_from_pmc import per_launch


def main():
    d, log2n, batch = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    kernel = sys.argv[4] if len(sys.argv) > 4 else "k_spass"
    v = per_launch(d, "SQ_INSTS_VALU", kernel)
    print(json.dumps({"kernel": kernel, "log2n": log2n, "batch": batch,
                      "valu_insts_per_launch": statistics.median(v[-5:]),
                      "launches_seen": len(v), "source_sha": source_sha()}, indent=1))


if __name__ == "__main__":
    main()
