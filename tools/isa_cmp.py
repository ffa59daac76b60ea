"""Instruction-level comparison of every kernel in two builds of the library (e.g. before / after a
change confined to diagnostic #ifdefs).  usage: python tools/isa_cmp.py old.so new.so"""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from test_isa_hot_loops import disassemble
a, b = disassemble(sys.argv[1]), disassemble(sys.argv[2])
print("kernels", len(a), len(b), "same names", set(a) == set(b))
diff = [k for k in a if k in b and [t for _, t, _ in a[k]] != [t for _, t, _ in b[k]]]
print("kernels with different instructions:", len(diff))
for k in diff[:10]:
    print("  ", k[-60:], len(a[k]), len(b[k]))
