"""Path-sensitive check of a kernel's register reads: a forward "definitely
written" dataflow over the kernel's control-flow graph (branches, and the far jumps
s_getpc_b64 / s_add_u32 / s_addc_u32 / s_setpc_b64 resolved), intersection at merges.  A read of a
register -- or, for the SGPR spill slots, of a VGPR lane: v_writelane defines (vN, lane),
v_readlane uses it -- that is not definitely written on every path from the kernel's entry is
reported with its position.  EXEC masking is ignored (a masked VALU write counts as a write).
usage: python tools/isa_mustdef.py lib_or_obj [kernel-regex]"""
import re
import sys
import os

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from test_isa_hot_loops import disassemble  # noqa: E402
from isa_undef import NODST, regs  # noqa: E402

HW = {("s", 0), ("s", 1), ("v", 0)}  # set by the hardware at wave launch (kernarg ptr, workitem id)


def parse(ins):
    """per instruction: (uses, defs) as sets of keys ('v', n) / ('s', n) / ('a', n) / ('l', vreg, lane)"""
    out = []
    for _, t, _ in ins:
        parts = t.split(None, 1)
        op = parts[0]
        ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
        uses, defs = set(), set()
        if op == "v_writelane_b32":
            defs.add(("l", int(ops[0][1:]), int(ops[2]) if ops[2].isdigit() else -1))
            uses |= set(regs(ops[1]))
        elif op == "v_readlane_b32":
            defs |= set(regs(ops[0]))
            lane = int(ops[2]) if ops[2].isdigit() else -1
            uses.add(("l", int(ops[1][1:]), lane) if lane >= 0 else ("v", int(ops[1][1:])))
        elif not ops:
            pass
        elif NODST.match(t) or (op.startswith("global_atomic") and " sc0" not in t and " glc" not in t):
            for o in ops:
                uses |= set(regs(o))
            if op.startswith("v_cmp"):
                pass
        else:
            defs |= set(regs(ops[0]))
            for o in ops[1:]:
                uses |= set(regs(o))
        if op.startswith("v_cmp_") and ops and ops[0].startswith("s"):
            defs |= set(regs(ops[0]))
            uses -= set(regs(ops[0]))
        out.append((uses, defs))
    return out


def cfg(ins):
    """successors of every instruction (far jumps resolved)"""
    addr = {a: i for i, (a, _, _) in enumerate(ins)}
    succ = []
    n = len(ins)
    for i, (a, t, tgt) in enumerate(ins):
        op = t.split()[0] if t else ""
        s = []
        if op == "s_setpc_b64":
            # s_getpc_b64 s[x:y] ; s_add_u32 sx, sx, OFF ; s_addc_u32 ... ; s_setpc_b64
            g = ins[i - 3]
            add = ins[i - 2][1]
            off = int(add.split(",")[-1].strip(), 16)
            if off >= 1 << 31:
                off -= 1 << 32
            dest = ins[i - 2][0] + off  # s_getpc returns the address of the next instruction
            s.append(addr.get(dest, None))
        elif op == "s_branch":
            s.append(addr.get(tgt))
        elif op.startswith("s_cbranch"):
            s.append(addr.get(tgt))
            s.append(i + 1)
        elif op == "s_endpgm":
            pass
        else:
            s.append(i + 1)
        succ.append([x for x in s if x is not None and x < n])
    return succ


def main():
    path = sys.argv[1]
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"qp_batch_kernelILi2ELi4ELb1ELi0E")
    for name, ins in disassemble(path).items():
        if not pat.search(name):
            continue
        pu = parse(ins)
        succ = cfg(ins)
        keys = {}
        for u, d in pu:
            for k in u | d:
                keys.setdefault(k, len(keys))
        bit = lambda ks: sum(1 << keys[k] for k in ks)  # noqa: E731
        D = [bit(d) for _, d in pu]
        U = [bit(u) for u, _ in pu]
        ALL = (1 << len(keys)) - 1
        IN = [ALL] * len(ins)
        IN[0] = bit(k for k in HW if k in keys)
        work = [0]
        inq = {0}
        while work:
            i = work.pop()
            inq.discard(i)
            out = IN[i] | D[i]
            for j in succ[i]:
                nv = IN[j] & out if j != 0 else IN[j]
                if nv != IN[j]:
                    IN[j] = nv
                    if j not in inq:
                        work.append(j)
                        inq.add(j)
        inv = {v: k for k, v in keys.items()}
        bad = []
        for i in range(len(ins)):
            miss = U[i] & ~IN[i]
            if miss:
                ks = [inv[b] for b in range(len(keys)) if miss >> b & 1]
                bad.append((i, ins[i][1], ks))
        print(name[-48:], "instructions", len(ins), "reads not definitely written:", len(bad))
        for i, t, ks in bad:
            print(f"  {i:6d} {t:60s} {ks}")


if __name__ == "__main__":
    main()
