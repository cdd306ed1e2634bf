#!/usr/bin/env python3
"""Time the message-pass kernel variants (gvs_set_option rpass_variant) on the
C3 workload: one prefilled store, the same batch stream, HIP-event stage times."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    import torch
    from grapevine_amd import abi
    from grapevine_amd.store import ObliviousStore
    log2n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    variants = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else list(range(11))
    rows = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [0]
    copy_reference(torch)
    for S in rows:
        run(torch, abi, ObliviousStore, log2n, variants, S)


def copy_reference(torch):
    """Device-to-device copy of 8 GiB: the read+write streaming rate this box
    reaches with a library kernel (ceiling reference for the table pass)."""
    dev = torch.device("cuda", 0)
    a = torch.empty(1 << 33, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    a.fill_(1)
    ts = []
    for _ in range(6):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        b.copy_(a)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ms = sorted(ts[1:])[len(ts[1:]) // 2]
    print(f"d2d copy 8 GiB: {ms:.3f} ms  {2 * (1 << 33) / ms / 1e6:.0f} GB/s (read+write)", flush=True)
    del a, b
    torch.cuda.empty_cache()


def run(torch, abi, ObliviousStore, log2n, variants, S):
    dev = torch.device("cuda", 0)
    N, B = 1 << log2n, 65536
    cfg = abi.make_config(N, max_batch=B)
    cfg.rows_per_partition = S
    store = ObliviousStore(cfg)
    print(f"rows per partition {store.stats()['msg_partition_slots']}, partitions {store.stats()['msg_partitions']}", flush=True)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    pool = torch.randint(0, 256, (1 << 19, 32), dtype=torch.uint8, device=dev, generator=g)
    known = bench.prefill(torch, store, dev, B, int(N * 0.75), pool, g, 1_700_000_000)
    reps = 4
    batches = bench.gen_batches(torch, dev, B, reps * len(variants) * 2, known, pool, g, 1_800_000_000)
    d_out = torch.empty((B, 1040), dtype=torch.uint8, device=dev)
    store.set_timing(True)
    k = 0
    res = {v: [] for v in variants}
    for rnd in range(2):
        for v in variants:
            store.set_option("rpass_variant", v)
            for _ in range(reps):
                store.process_batch_device(batches[k].data_ptr(), B, d_out.data_ptr())
                k += 1
                if rnd == 1:
                    res[v].append(store.last_timings()["rpass"])
    alg = 2 * N * 1024 + B * (1024 + 1040)
    for v in variants:
        ms = sorted(res[v])[len(res[v]) // 2]
        print(f"variant {v}: rpass {ms:.3f} ms  {alg / ms / 1e6:.0f} GB/s  ({min(res[v]):.3f}..{max(res[v]):.3f})", flush=True)
    store.close()
    del known, batches
    torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
