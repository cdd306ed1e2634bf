"""Which branches of a gfx950 kernel depend on the data it loads (test helper).

A static backward slice over the disassembly (`llvm-objdump -d`): a value is
*tainted* when it was loaded from memory (global / buffer / flat / LDS) or
computed from a tainted value; a conditional branch is data-dependent when its
condition (SCC, VCC or EXEC) is tainted.  Kernel arguments (s_load), workitem
and workgroup ids are not data.  The analysis follows the linear order of the
listing and, inside a loop (a backward branch), every writer of a register in
the loop body, so a loop-carried key still counts.  It is approximate the safe
way round for the kernels it is used on (tests/test_code_object.py): it may
flag a branch that does not depend on data, it does not miss one that does,
and the positive controls in that test compile the patterns it must catch.

EXEC is modelled as structured control flow: `s_and_saveexec sX, c` narrows
EXEC by c and saves the old mask in sX (sX itself is not tainted by c);
`s_or_b64 exec, exec, sX` restores the mask saved in sX, whose taint is that
of EXEC where sX was saved.
"""
import re

LOADS = ("global_load", "buffer_load", "flat_load", "scratch_load", "ds_read", "ds_load",
         "global_atomic", "buffer_atomic", "flat_atomic", "ds_add_rtn", "ds_bpermute", "ds_permute",
         "ds_swizzle")
NO_DST = ("global_store", "buffer_store", "flat_store", "scratch_store", "ds_write", "ds_store", "s_waitcnt",
          "s_branch", "s_cbranch", "s_barrier", "s_endpgm", "s_nop", "s_setprio", "s_sleep", "s_dcache",
          "s_set_gpr_idx", "s_sendmsg", "s_trap", "s_setreg", "ds_add_u32", "ds_or_b32", "ds_and_b32",
          "ds_max", "ds_min", "ds_xor", "ds_inc", "ds_dec", "s_icache", "buffer_wbl2", "buffer_inv",
          "s_memtime", "s_memrealtime")
SCC_WRITERS = ("s_cmp", "s_bitcmp", "s_and_", "s_or_", "s_xor_", "s_andn2_", "s_orn2_", "s_nand_", "s_nor_",
               "s_xnor_", "s_add_", "s_sub_", "s_addc_", "s_subb_", "s_lshl", "s_lshr", "s_ashr", "s_bfe_",
               "s_min_", "s_max_", "s_abs_", "s_not_", "s_absdiff", "s_bcnt", "s_quadmask", "s_wqm",
               "s_addk", "s_cmpk")
SCC_READERS = ("s_cselect", "s_cmov", "s_addc_", "s_subb_", "s_cbranch_scc")
REG = re.compile(r"^(v|s|a)\[(\d+):(\d+)\]$|^(v|s|a)(\d+)$")


def expand(tok):
    """Register names of one operand ('v[4:7]' -> v4..v7, 'vcc' -> vcc_lo, vcc_hi)."""
    tok = tok.strip().lstrip("-|").rstrip("|")
    tok = re.sub(r"^(abs|neg|sext)\((.*)\)$", r"\2", tok)
    if tok in ("vcc", "exec"):
        return [tok + "_lo", tok + "_hi"]
    if tok in ("vcc_lo", "vcc_hi", "exec_lo", "exec_hi", "scc", "m0"):
        return [tok]
    m = REG.match(tok)
    if not m:
        return []
    if m.group(1):
        return [f"{m.group(1)}{i}" for i in range(int(m.group(2)), int(m.group(3)) + 1)]
    return [f"{m.group(4)}{m.group(5)}"]


def split_ops(text):
    out, depth, cur = [], 0, ""
    for ch in text:
        if ch in "([":
            depth += 1
        elif ch in ")]":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


class Ins:
    __slots__ = ("i", "op", "ops", "dst", "src", "load", "target", "saved_exec")

    def __init__(self, i, op, ops, target):
        self.i, self.op, self.ops, self.target = i, op, ops, target
        self.saved_exec = None
        regs = [expand(o) for o in ops]
        self.load = op.startswith(LOADS)
        if op.startswith(NO_DST) or not ops:
            dst, src = [], [r for rs in regs for r in rs]
        else:
            dst, src = list(regs[0]), [r for rs in regs[1:] for r in rs]
            # VALU carry-out / 64-bit mad / div_scale: the second operand is a destination too
            if op.startswith("v_") and len(regs) > 2 and ("_co_" in op or "mad_u64" in op or "mad_i64" in op
                                                         or "div_scale" in op) and ops[1][0] in "sv":
                dst += regs[1]
                src = [r for rs in regs[2:] for r in rs]
        if op.startswith("v_cmpx"):
            dst += ["exec_lo", "exec_hi"]
        if "saveexec" in op:  # sX = old exec; exec = f(exec, src)
            self.saved_exec = list(regs[0])
            dst = list(regs[0]) + ["exec_lo", "exec_hi", "scc"]
            src = src + ["exec_lo", "exec_hi"]
        if op.startswith(SCC_WRITERS) and "saveexec" not in op:
            dst.append("scc")
        if op.startswith(SCC_READERS):
            src.append("scc")
        if op.startswith("s_cbranch_vcc"):
            src += ["vcc_lo", "vcc_hi"]
        if op.startswith("s_cbranch_exec"):
            src += ["exec_lo", "exec_hi"]
        self.dst, self.src = dst, src


def parse(listing):
    """{kernel symbol: [Ins]} from an llvm-objdump -d listing."""
    out, cur, addr_of = {}, None, {}
    raw = []
    for line in listing.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.*)>:", line)
        if m:
            cur = m.group(2)
            out[cur] = []
            continue
        if cur is None:
            continue
        m = re.match(r"^\s+([a-z_0-9]+)\s*(.*?)\s*//\s*([0-9A-F]+):", line)
        if not m:
            continue
        op, rest, addr = m.group(1), m.group(2), int(m.group(3), 16)
        tm = re.search(r"<([^>+]+)\+0x([0-9a-f]+)>", line)
        raw.append((cur, op, rest, addr, tm))
    base = {}
    for cur, op, rest, addr, tm in raw:
        base.setdefault(cur, addr)
    for cur, op, rest, addr, tm in raw:
        lst = out[cur]
        target = None
        if op.startswith(("s_cbranch", "s_branch")) and tm and tm.group(1) == cur:
            target = base[cur] + int(tm.group(2), 16)
        ops = split_ops(rest) if rest else []
        if op.startswith(("s_cbranch", "s_branch")):
            ops = []
        ins = Ins(len(lst), op, ops, target)
        lst.append(ins)
        addr_of[(cur, len(lst) - 1)] = addr
    # branch targets as instruction indices
    for cur, lst in out.items():
        idx = {addr_of[(cur, k)]: k for k in range(len(lst))}
        for ins in lst:
            if ins.target is not None:
                ins.target = idx.get(ins.target)
    return out


def blocks(ins):
    """Basic blocks as (first, last) instruction indices, and their successors."""
    lead = {0}
    for x in ins:
        if x.op.startswith(("s_cbranch", "s_branch", "s_endpgm")):
            lead.add(x.i + 1)
            if x.target is not None:
                lead.add(x.target)
    lead = sorted(k for k in lead if k < len(ins))
    spans = [(a, (lead[n + 1] if n + 1 < len(lead) else len(ins)) - 1) for n, a in enumerate(lead)]
    start = {a: n for n, (a, _) in enumerate(spans)}
    succ = []
    for a, b in spans:
        x, s = ins[b], []
        if x.op.startswith(("s_branch", "s_cbranch")) and x.target is not None:
            s.append(start[x.target])
        if not x.op.startswith(("s_branch", "s_endpgm")) and b + 1 < len(ins):
            s.append(start[b + 1])
        succ.append(s)
    return spans, succ


def step(x, t):
    """Transfer function of one instruction on the tainted-register set t (in place)."""
    if x.saved_exec:  # s_*_saveexec sX, c: sX = old exec, exec = f(exec, c)
        old = "exec_lo" in t
        new = old or any(r in t for r in x.src)
        for r in x.saved_exec:
            (t.add if old else t.discard)(r)
        for r in ("exec_lo", "exec_hi"):
            (t.add if new else t.discard)(r)
        (t.add if new else t.discard)("scc")
        return
    if x.op.startswith("s_or_b64") and x.ops[:2] == ["exec", "exec"] and len(x.ops) == 3:
        src = expand(x.ops[2])  # restore of a saved mask
    else:
        src = x.src
    v = x.load or any(r in t for r in src)
    for r in x.dst:
        (t.add if v else t.discard)(r)


def data_dependent_branches(ins):
    """[(index, mnemonic)] of the conditional branches whose condition is tainted
    (forward dataflow over the basic blocks, union at joins, to a fixpoint)."""
    spans, succ = blocks(ins)
    state_in = [None] * len(spans)
    state_in[0] = set()
    work, flagged = [0], set()
    while work:
        n = work.pop()
        t = set(state_in[n])
        a, b = spans[n]
        for k in range(a, b + 1):
            x = ins[k]
            if x.op.startswith("s_cbranch") and any(r in t for r in x.src):
                flagged.add(k)
            step(x, t)
        for m in succ[n]:
            if state_in[m] is None or not t <= state_in[m]:
                state_in[m] = t | (state_in[m] or set())
                work.append(m)
    return [(k, ins[k].op) for k in sorted(flagged)]
