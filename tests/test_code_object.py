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

The second check is on branches: a conditional branch whose condition comes
from loaded data (tests/isa_taint.py, a dataflow over the disassembly) makes
the instructions a wave issues depend on the data.  The sort kernels must have
none (`key_lt<Key128>` was written with a short-circuit `||`
/ `&&`), nor must the other kernels that have none today; the analysis itself
is checked on compiled positive and negative controls.
"""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

import isa_taint

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"

# kernel symbol substring -> (max scratch bytes per lane, why)
ALLOWED = {}


def code_object(lib, tool):
    """Output of `tool` (a list: program and flags) on the library's gfx950 code object."""
    tmp = tempfile.mkdtemp()
    try:
        fb, co = os.path.join(tmp, "fb.bin"), os.path.join(tmp, "co")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", lib, os.path.join(tmp, "x")],
                       check=True, capture_output=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"],
                       check=True, capture_output=True)
        return subprocess.run(tool + [co], check=True, capture_output=True, text=True).stdout
    finally:
        shutil.rmtree(tmp)


def kernel_scratch(lib):
    notes = code_object(lib, [f"{LLVM}/llvm-readelf", "--notes"])
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


# Kernels that must have no data-dependent conditional branch: the sorts (the
# short-circuit comparison of VERDICT round 5) and every kernel with none
# today.  The others (the table and mailbox passes, the scans with per-op
# guards, the router, the wire codec, the map's key pass) are listed with their
# counts in the report; their memory traffic and durations are what
# tests/test_oblivious.py and tests/test_timing.py check.
STRICT = ("k_bitonic_tile", "k_bitonic_global", "k_copy", "k_meta", "k_alloc_sum", "k_alloc_b", "k_post_sum",
          "k_post_ring", "k_out", "k_rr2_c", "k_m2g", "k_m2r_c", "k_vscan_b1", "k_vscan_b2", "k_vscan_b3",
          "k_scan_b<GtxOp>", "k_scan_a<GtxOp>", "k_scan_a<Rr1Op>", "k_scan_b<Rr1Op>", "k_scan_c<Rr1Op>",
          "k_vscan_a<M1rOp>", "k_vscan_a<Rr2Op>", "k_vscan_a<M2rOp>", "k_seal_init", "k_pseal", "k_sr_verify",
          "k_route_mark", "k_route_hist", "k_err_or", "k_ogather", "k_kdir_seal_init", "k_scan_a<OrowOp>",
          "k_scan_b<OrowOp>", "k_scan_c<OrowOp>", "k_scan_b<OgtOp>")


def demangle(sym):
    """'_ZN3gvs8k_scan_aINS_5GtxOpEEEvNT_4ArgsE' -> 'k_scan_a<GtxOp>' (enough to match STRICT)."""
    import re
    m = re.match(r"_ZN3gvs(?:2sr)?(\d+)", sym)
    if not m:
        return sym
    n = int(m.group(1))
    rest = sym[m.end():]
    name, rest = rest[:n], rest[n:]
    t = re.match(r"INS_(\d+)", rest)
    if t:
        k = int(t.group(1))
        return f"{name}<{rest[t.end():t.end() + k]}>"
    return name


CONTROLS = r"""
#include <hip/hip_runtime.h>
#include <stdint.h>
struct K2 { uint64_t hi, lo; };
__device__ inline bool lt_sc(const K2& a, const K2& b) { return a.hi < b.hi || (a.hi == b.hi && a.lo < b.lo); }
extern "C" __global__ void ctrl_store_on_swap(K2* d, uint32_t j) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  K2 a = d[i], b = d[i + j];
  if (lt_sc(b, a)) { d[i] = b; d[i + j] = a; }
}
extern "C" __global__ void ctrl_loaded_trip(uint32_t* d, const uint32_t* n) {
  uint32_t s = 0;
  for (uint32_t k = 0; k < n[threadIdx.x]; ++k) s += d[k];
  d[threadIdx.x] = s;
}
extern "C" __global__ void ctrl_lds_uniform(uint32_t* d) {
  __shared__ uint32_t s[64];
  s[threadIdx.x] = d[threadIdx.x];
  __syncthreads();
  if (s[0] > 5u) d[threadIdx.x + 64] = 1u;
}
extern "C" __global__ void ctrl_clean(K2* d, uint32_t j, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i + j >= n) return;
  K2 a = d[i], b = d[i + j];
  const bool sw = (b.hi < a.hi) | ((b.hi == a.hi) & (b.lo < a.lo));
  d[i] = K2{sw ? b.hi : a.hi, sw ? b.lo : a.lo};
  d[i + j] = K2{sw ? a.hi : b.hi, sw ? a.lo : b.lo};
}
"""


def test_taint_analysis_catches_the_controls(tmp_path):
    """The analysis flags a store under a key comparison (short-circuit), a loop
    whose trip count is loaded and a uniform branch on an LDS value, and flags
    nothing in the same compare-exchange written with selects."""
    hipcc = "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc) or not os.path.exists(f"{LLVM}/llvm-objdump"):
        pytest.skip("hipcc / llvm-objdump not present")
    src, co = tmp_path / "ctrl.hip", tmp_path / "ctrl.co"
    src.write_text(CONTROLS)
    subprocess.run([hipcc, "--offload-arch=gfx950", "--offload-device-only", "--no-gpu-bundle-output", "-O3", "-c",
                    str(src), "-o", str(co)], check=True, capture_output=True)
    dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", str(co)], check=True,
                         capture_output=True, text=True).stdout
    ks = isa_taint.parse(dis)
    flagged = {k: isa_taint.data_dependent_branches(v) for k, v in ks.items()}
    assert flagged["ctrl_store_on_swap"] and flagged["ctrl_loaded_trip"] and flagged["ctrl_lds_uniform"], flagged
    assert flagged["ctrl_clean"] == [], flagged["ctrl_clean"]
    assert any(x.op.startswith("s_cbranch") for x in ks["ctrl_clean"])  # its bounds branch is not data


@pytest.mark.parametrize("lib", LIBS)
def test_no_data_dependent_branches(lib):
    path = os.path.join(ROOT, lib)
    if not os.path.exists(path) or not os.path.exists(f"{LLVM}/llvm-objdump"):
        pytest.skip("library or ROCm LLVM tools not present")
    ks = isa_taint.parse(code_object(path, [f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn"]))
    assert len(ks) > 50, f"kernels not found ({len(ks)})"
    bad, table, n_sort = [], [], 0
    for sym, ins in sorted(ks.items()):
        name = demangle(sym)
        flagged = isa_taint.data_dependent_branches(ins)
        n_br = sum(1 for x in ins if x.op.startswith("s_cbranch"))
        strict = name.startswith(STRICT)
        n_sort += name.startswith("k_bitonic")
        table.append(f"{name:28s} {len(ins):6d} instructions {n_br:4d} branches {len(flagged):4d} on data"
                     + (" (must be 0)" if strict else ""))
        if strict and flagged:
            bad.append((name, flagged[:6]))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"branches_{os.path.basename(lib)}.txt"), "w") as f:
        f.write("\n".join(table) + "\n")
    assert n_sort >= 8, "sort kernels not found"
    assert not bad, f"data-dependent branches: {bad}"
