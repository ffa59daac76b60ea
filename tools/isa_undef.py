"""Registers a kernel reads that no instruction of the kernel writes (the
register-dependent wrong results of high-register builds).  Approximate operand parser: the first
operand is the destination except for stores, atomics without return, s_cbranch/s_setpc and
compares writing vcc/exec; v_writelane writes its VGPR (one lane), v_readlane / v_readfirstlane
write their SGPR.  Registers set by the hardware at wave launch (v0 = workitem id, s[0:1] =
kernarg pointer, the workgroup-id SGPRs the descriptor enables) are listed separately.
usage: python tools/isa_undef.py lib_or_obj.so [kernel-regex]"""
import re
import sys

sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__file__), "..", "tests"))
from test_isa_hot_loops import disassemble  # noqa: E402

REG = re.compile(r"\b([vsa])(\d+)\b|\b([vsa])\[(\d+):(\d+)\]")


def regs(op):
    out = []
    for m in REG.finditer(op):
        if m.group(1):
            out.append((m.group(1), int(m.group(2))))
        else:
            out += [(m.group(3), k) for k in range(int(m.group(4)), int(m.group(5)) + 1)]
    return out


NODST = re.compile(r"^(global_store|buffer_store|ds_write|ds_add_f64|ds_add_u32|ds_max|ds_min|scratch_store|"
                   r"s_cbranch|s_branch|s_setpc|s_waitcnt|s_barrier|s_nop|s_sleep|s_endpgm|"
                   r"s_cmp|v_cmp_|v_cmpx|s_bitcmp|global_atomic_add_f64 v\[|s_store|s_dcache|buffer_inv|"
                   r"buffer_wbl2|s_setprio|s_trap|s_sendmsg)")


def analyse(ins):
    written, read_first = set(), {}
    for i, (_, t, _) in enumerate(ins):
        parts = t.split(None, 1)
        op = parts[0]
        ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
        if not ops:
            continue
        if NODST.match(t) or (op.startswith("global_atomic") and " glc" not in t and " sc0" not in t):
            srcs, dsts = ops, []
        else:
            dsts, srcs = [ops[0]], ops[1:]
        if op.startswith("v_cmp_") or op.startswith("v_cmpx"):
            dsts = [ops[0]] if ops[0].startswith("s") else []
            srcs = ops[1:] if dsts else ops
        for o in srcs:
            for r in regs(o):
                if r not in written and r not in read_first:
                    read_first[r] = i
        for o in dsts:
            for r in regs(o):
                written.add(r)
    return written, read_first


def main():
    path = sys.argv[1]
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"qp_batch_kernelILi2ELi4ELb1ELi0E")
    for name, ins in disassemble(path).items():
        if not pat.search(name):
            continue
        written, first = analyse(ins)
        never = sorted((r for r in first if r not in written), key=lambda r: (r[0], r[1]))
        print(name[-48:], "instructions", len(ins))
        print("  read, never written in the kernel:", " ".join(f"{c}{k}@{first[(c, k)]}" for c, k in never))


if __name__ == "__main__":
    main()
