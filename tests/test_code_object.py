"""The built engine's gfx950 code object (CPU test: reads kernel metadata only).

Private (scratch) memory lives in HBM behind L2: whether a wave's scratch
lines are written back and fetched again depends on what else the batch
evicted, so a kernel with scratch moves FETCH_SIZE / WRITE_SIZE with the
timing.  Round 5 found `k_route_gather` with a 160-B/lane array in scratch (a
`c ? x : y` over uint4 values compiled to a select of their addresses): 10 MB
of FETCH_SIZE per launch and +-25 KiB of noise that failed the routed counter
test (profiles/r05l_oblivious_FETCH_SIZE_routed.txt, r05m after the fix).
Every kernel is now checked for scratch, and none has any (k_m2a's 24-B
register spills are gone: its per-lane row is recomputed per chunk;
k_sr_verify's 80 B went with its out-of-line curve functions).  ALLOWED would
list an exception with its bound and the reason.
"""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"

# kernel symbol substring -> (max scratch bytes per lane, why)
ALLOWED = {}


def kernel_scratch(lib):
    tmp = tempfile.mkdtemp()
    try:
        fb, co = os.path.join(tmp, "fb.bin"), os.path.join(tmp, "co")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", lib, os.path.join(tmp, "x")],
                       check=True, capture_output=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"],
                       check=True, capture_output=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                               text=True).stdout
    finally:
        shutil.rmtree(tmp)
    out, name = {}, None
    for line in notes.splitlines():
        m = re.match(r"\s*(?:- )?\.name:\s+(\S+)", line)
        if m:
            name = m.group(1)
        m = re.match(r"\s*(?:- )?\.private_segment_fixed_size:\s+(\d+)", line)
        if m and name is not None:
            out[name] = int(m.group(1))
    return out


LIBS = ["grapevine_amd/libgvstore.so", "grapevine_amd/libgvstore_test.so"]


@pytest.mark.parametrize("lib", LIBS)
def test_no_scratch_outside_the_allowlist(lib):
    path = os.path.join(ROOT, lib)
    if not os.path.exists(path) or not os.path.exists(f"{LLVM}/clang-offload-bundler"):
        pytest.skip("library or ROCm LLVM tools not present")
    ks = kernel_scratch(path)
    assert len(ks) > 50, f"kernel metadata not found ({len(ks)} kernels)"
    bad = []
    for k, n in sorted(ks.items()):
        if n == 0:
            continue
        allow = next((v for s, v in ALLOWED.items() if s in k), None)
        if allow is None or n > allow[0]:
            bad.append((k, n))
    assert not bad, f"kernels with scratch: {bad}"
