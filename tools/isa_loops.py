"""Per-region ISA counts inside the N = 20 product kernel's ADMM loop (see isa_stats.py):
every loop nested in it (the solve-step record pipelines, the factorization runners, the Ruiz /
check loops) and the straight-line stretches between them.  usage: python tools/isa_loops.py lib.so"""
import collections
import os
import re
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from test_isa_hot_loops import disassemble, loops  # noqa: E402

PAT = re.compile(os.environ.get("ISA_KERNEL", r"qp_batch_kernelILi2ELi4ELb1ELi0E"))


def cnt(seg):
    c = collections.Counter(x.split()[0] for x in seg)
    return (f"n={len(seg):5d} rl={c['v_readlane_b32']:3d} sl={sum(v for k, v in c.items() if k.startswith('s_load')):3d} "
            f"ds={sum(v for k, v in c.items() if k.startswith('ds_')):4d} "
            f"atom={sum(v for k, v in c.items() if k.startswith('ds_add')):3d} "
            f"buf={sum(v for k, v in c.items() if k.startswith('buffer_')):3d}")


lib = sys.argv[1]
for name, ins in disassemble(lib).items():
    if not PAT.search(name):
        continue
    L = loops(ins)
    admm = max(L, key=lambda x: x[1] - x[0])
    sub = sorted({l for l in L if l != admm and admm[0] <= l[0] and l[1] <= admm[1]})
    # keep only outermost sub-loops
    top = [l for l in sub if not any(o != l and o[0] <= l[0] and l[1] <= o[1] for o in sub)]
    print(name[-44:], "ADMM", admm, cnt([t for _, t, _ in ins[admm[0]:admm[1] + 1]]))
    pos = admm[0]
    for h, e in top:
        if h > pos:
            print(f"   line   {pos:6d}-{h - 1:6d}", cnt([t for _, t, _ in ins[pos:h]]))
        print(f"   LOOP   {h:6d}-{e:6d}", cnt([t for _, t, _ in ins[h:e + 1]]))
        pos = e + 1
    print(f"   line   {pos:6d}-{admm[1]:6d}", cnt([t for _, t, _ in ins[pos:admm[1] + 1]]))
