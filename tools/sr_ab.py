"""A/B timing of gvs_sr25519_verify_device across library builds (not part of
the product):  python tools/sr_ab.py lib1.so lib2.so ...
Each library: a small store, then 6 launches over 64K random (pk, 32-B
message, signature) triples; prints every launch's HIP-event time."""
import ctypes
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__file__)))
from grapevine_amd import abi, store as gs  # noqa: E402


def run(path, n=65536):
    lib = gs.load_library(path)
    cfg = abi.make_config(1 << 16, max_batch=4096)
    h = ctypes.c_void_p()
    assert lib.gvs_create(ctypes.byref(cfg), ctypes.byref(h)) == 0
    lib.gvs_set_timing(h, 1)
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    pks = torch.randint(0, 256, (n, 32), dtype=torch.uint8, device="cuda", generator=g)
    msgs = torch.randint(0, 256, (n, 32), dtype=torch.uint8, device="cuda", generator=g)
    sigs = torch.randint(0, 256, (n, 64), dtype=torch.uint8, device="cuda", generator=g)
    ok = torch.empty((n,), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    ctx = b"grapevine-challenge"
    out = []
    for _ in range(6):
        assert lib.gvs_sr25519_verify_device(h, pks.data_ptr(), 32, msgs.data_ptr(), 32, 32,
                                             sigs.data_ptr(), 64, n, ctx, len(ctx), ok.data_ptr()) == 0
        names = (ctypes.c_char_p * 16)()
        ms = (ctypes.c_float * 16)()
        c = lib.gvs_last_timings(h, names, ms, 16)
        out.append(round(ms[0], 3) if c > 0 else None)
    lib.gvs_destroy(h)
    print(path, out, flush=True)


if __name__ == "__main__":
    for p in sys.argv[1:]:
        run(p)
