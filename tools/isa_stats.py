"""ISA statistics of the N = 20 product kernel (qp_batch_kernel<2, 4, paired, KM_LDS>) of a library:
instruction counts of the whole kernel and of its ADMM loop (the outermost loop that holds the
solve steps), SGPR-spill reloads (v_readlane), spill stores (v_writelane), kernel-argument and
other scalar loads, LDS operations.  usage: python tools/isa_stats.py lib.so [lib2.so ...]"""
import collections
import os
import re
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from test_isa_hot_loops import disassemble, loops  # noqa: E402

PAT = re.compile(sys.argv[0] and os.environ.get("ISA_KERNEL", r"qp_batch_kernelILi2ELi4ELb1ELi0E"))


def stats(seg):
    c = collections.Counter(x.split()[0] for x in seg)
    return dict(n=len(seg), readlane=c["v_readlane_b32"], writelane=c["v_writelane_b32"],
                s_load=sum(v for k, v in c.items() if k.startswith("s_load") or k.startswith("s_buffer_load")),
                ds=sum(v for k, v in c.items() if k.startswith("ds_")),
                waitcnt=c["s_waitcnt"], nop=c["s_nop"],
                vmem=sum(v for k, v in c.items() if k.startswith(("global_", "buffer_"))),
                scratch=sum(v for k, v in c.items() if "scratch" in k))


for lib in sys.argv[1:]:
    isa = disassemble(lib)
    for name, ins in isa.items():
        if not PAT.search(name):
            continue
        L = loops(ins)
        outer = max(L, key=lambda x: x[1] - x[0])
        # the ADMM loop: the largest loop strictly inside the instance loop
        inner = max((l for l in L if l != outer and outer[0] <= l[0] and l[1] <= outer[1]),
                    key=lambda x: x[1] - x[0])
        print(os.path.basename(lib), name[-40:])
        print("  kernel   ", stats([t for _, t, _ in ins]))
        print("  inst loop", stats([t for _, t, _ in ins[outer[0]:outer[1] + 1]]))
        print("  ADMM loop", inner, stats([t for _, t, _ in ins[inner[0]:inner[1] + 1]]))
