#!/usr/bin/env python3
"""Issue ceiling of a kernel's own VALU instruction mix.

The nominal VALU peak (one wave64 instruction per SIMD every 2 cycles) holds
for two-source operations such as v_xor_b32; the three-source operations the
sealed passes are made of (v_perm_b32, v_alignbit_b32, v_bitop3_b32,
v_lshl_add_u64) issue 1.35-1.55x slower on gfx950 (tools/valu_rate_probe.hip,
profiles/r05j_valu_rate_probe.txt).  This tool counts the VALU instructions of
one kernel in the device assembly, prices each with its probe-measured issue
rate at the kernel's waves per SIMD (unmeasured opcodes at the two-source rate)
and prints the mix's ceiling in wave-instructions per cycle per SIMD, and in
G wave-instructions per second over the chip at the probe's clock.

    python tools/valu_mix_peak.py KERNEL_SYMBOL_SUBSTRING WAVES_PER_SIMD [ASM] [PROBE]

Without ASM the engine is compiled to device assembly here (hipcc -S).
"""
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from srcsha import source_sha  # noqa: E402

PROBE_OPS = {  # probe line prefix -> opcode(s) it prices
    "v_lshl_add_u64": ["v_lshl_add_u64"],
    "v_perm_b32": ["v_perm_b32"],
    "v_alignbit_b32": ["v_alignbit_b32"],
    "v_bitop3_b32": ["v_bitop3_b32"],
    "v_xor_b32 ": ["v_xor_b32_e32", "v_xor_b32_e64", "v_xor_b32"],
}
CHIP_SIMDS = 256 * 4
CLOCK_GHZ = 2.4


def probe_rates(path, waves):
    rates = {}
    for line in open(path):
        m = re.match(r"(.+?)\s+waves/SIMD=(\d+)\s+\S+ ms\s+([\d.]+) wave-instr", line)
        if m and int(m.group(2)) == waves:
            rates[m.group(1).strip()] = float(m.group(3))
    out = {}
    for prefix, ops in PROBE_OPS.items():
        for name, r in rates.items():
            if (name + " ").startswith(prefix):
                for op in ops:
                    out[op] = r
    return out, rates.get("v_xor_b32", max(out.values()))


def kernel_counts(asm, sym):
    lines = open(asm).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(rf"^_Z\S*{re.escape(sym)}\S*:", l))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    c = collections.Counter()
    for l in lines[start:end]:
        t = l.strip().split()
        if t and t[0].startswith("v_") and not t[0].startswith(("v_readlane", "v_writelane", "v_readfirstlane")):
            c[t[0]] += 1
    return c


def main():
    sym, waves = sys.argv[1], int(sys.argv[2])
    asm = sys.argv[3] if len(sys.argv) > 3 else None
    probe = sys.argv[4] if len(sys.argv) > 4 else os.path.join(ROOT, "profiles", "r05j_valu_rate_probe.txt")
    if not asm:
        asm = os.path.join(tempfile.mkdtemp(), "engine.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-Wno-unused-function",
                        "-Wno-bitwise-instead-of-logical", "--cuda-device-only", "-S", "-o", asm,
                        os.path.join(ROOT, "grapevine_amd", "csrc", "gvs_engine.hip")], check=True)
    rates, base = probe_rates(probe, waves)
    counts = kernel_counts(asm, sym)
    total = sum(counts.values())
    cycles = sum(n / rates.get(op, base) for op, n in counts.items())
    ceiling = total / cycles
    out = {"kernel": sym, "waves_per_simd": waves, "source_sha": source_sha(),
           "static_valu_instructions": total,
           "priced": {op: {"count": n, "rate": rates.get(op, base)} for op, n in counts.most_common(8)},
           "ceiling_wave_instr_per_cycle_per_simd": ceiling,
           "ceiling_g_wave_instr_per_s": ceiling * CHIP_SIMDS * CLOCK_GHZ,
           "nominal_g_wave_instr_per_s": 0.5 * CHIP_SIMDS * CLOCK_GHZ,
           "probe": os.path.relpath(probe, ROOT)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
