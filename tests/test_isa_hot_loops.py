"""Build-time ISA guard of the product kernels' hot loops (no GPU needed; round 5).

Two codegen regressions cost measurable throughput this round (Padded schedule tables and
Measured): an SGPR spilled into a VGPR lane and reloaded (`v_readlane` + wait states) on every
solve step of the two-wave kernel (+21 % forward-solve time, −4 % at N = 40), and the ADMM loop
head re-reading the kernel arguments every iteration (an `s_load` whose `lgkmcnt(0)` wait also
drains the LDS queue; −0.5 % at N = 20, −1.7 % at N = 40).  This test disassembles the gfx950
code object inside libmpcqp.so and checks, for the product solve kernels of the reference's
horizons (the one-wave (2, 4) and (4, 8) kernels, the two-wave (2, 4) kernel of N = 40; the
two-wave (1, 2) kernel, selected only for small problems with large LDS images, still reloads a
record descriptor in its step loop):
  * the solve-step loops (the record pipelines: three LDS atomics and five record loads per step)
    contain no `v_readlane` (SGPR-spill reload) and no `s_load` (kernel-argument reload);
  * the first block of the ADMM loop (its header up to the first solve's record prefetch) contains
    no `s_load`;
  * (round 6) an ADMM iteration that neither checks nor adapts rho -- the
    shortest path through the loop, which skips every check block -- reloads no kernel argument
    and at most the spilled SGPRs it reloads today (the checks' own reloads run once per
    check_termination iterations and are not capped here).
"""
import heapq
import os
import re
import subprocess

import pytest

from test_kernel_resources import LIB, LLVM, PRODUCT

BRANCH = re.compile(r"s_(cbranch_\w+|branch)\s.*<([^+>]+)\+0x([0-9a-f]+)>")


def disassemble(lib=LIB, tmp="/tmp"):
    """{kernel symbol: [(address, instruction text, branch target address or None)]}"""
    tools = [os.path.join(LLVM, t) for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-objdump")]
    if not all(os.path.exists(t) for t in tools) or not os.path.exists(lib):
        pytest.skip("ROCm LLVM tools or the library are missing")
    objcopy, bundler, objdump = tools
    fb = os.path.join(tmp, "mpcqp_isa_fatbin_%d.bin" % os.getpid())
    co = os.path.join(tmp, "mpcqp_isa_gfx950_%d.elf" % os.getpid())
    try:
        subprocess.check_call([objcopy, "--dump-section", ".hip_fatbin=" + fb, lib, os.devnull])
        subprocess.check_call([bundler, "--unbundle", "--type=o", "--input=" + fb,
                               "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + co])
        text = subprocess.check_output([objdump, "-d", "--no-show-raw-insn", co], text=True)
    finally:
        for f in (fb, co):
            if os.path.exists(f):
                os.remove(f)
    out, cur, base = {}, None, 0
    for line in text.splitlines():
        m = re.match(r"^([0-9a-f]{16}) <([^>]+)>:", line)
        if m:
            base, cur = int(m.group(1), 16), m.group(2)
            out[cur] = []
            continue
        if cur is None:
            continue
        a = re.search(r"//\s+([0-9A-Fa-f]+):", line)
        if not a:
            continue
        b = BRANCH.search(line)
        out[cur].append((int(a.group(1), 16), line.split("//")[0].strip(),
                         base + int(b.group(3), 16) if b else None))
    return out


def loops(ins):
    """(header index, back-edge index) of every backward branch"""
    idx = {a: i for i, (a, _, _) in enumerate(ins)}
    return sorted({(idx[t], i) for i, (a, _, t) in enumerate(ins) if t is not None and t <= a and t in idx})


HOT = re.compile(r"qp_batch_kernelILi(2ELi4|4ELi8)ELb[01]ELi0E|qp_pair_kernelILi2ELi4ELb[01]ELi2E")


@pytest.fixture(scope="module")
def isa():
    return {k: v for k, v in disassemble().items() if PRODUCT.search(k) and HOT.search(k)}


def test_solve_step_loops_have_no_spill_or_kernarg_reloads(isa):
    assert len(isa) >= 6, sorted(isa)
    for name, ins in isa.items():
        steps = []
        for h, e in loops(ins):
            body = [t for _, t, _ in ins[h:e + 1]]
            if len(body) < 1500 and sum("ds_add" in t for t in body) >= 6 and \
                    sum("buffer_load" in t for t in body) >= 10:
                steps.append((h, e, body))
        assert steps, (name, "no solve-step loop found")
        for h, e, body in steps:
            bad = [t for t in body if t.startswith(("v_readlane", "s_load"))]
            assert not bad, (name, h, e, bad[:4])


def test_admm_loop_head_does_not_reload_kernel_arguments(isa):
    for name, ins in isa.items():
        h, e = max(loops(ins), key=lambda x: x[1] - x[0])  # the ADMM iteration loop
        head = []
        for _, t, _ in ins[h:e]:
            if t.startswith("buffer_load"):  # the forward solve's record prefetch
                break
            head.append(t)
        assert not any(t.startswith("s_load") for t in head), (name, head[:12])


# v_readlane (SGPR-spill reloads) on a non-check iteration, as built in round 6: the N = 20 kernel
# 3 (loop counters at the head), the two-wave N = 40 kernel 0, the (4, 8) one-wave kernel 23
NONCHECK_RELOADS = {"qp_batch_kernelILi2ELi4": 3, "qp_pair_kernelILi2ELi4": 0, "qp_batch_kernelILi4ELi8": 23}


def _succ(ins, i, idx):
    _, t, tgt = ins[i]
    op = t.split()[0]
    if op == "s_branch":
        return [idx[tgt]] if tgt in idx else []
    if op.startswith("s_cbranch"):
        return ([idx[tgt]] if tgt in idx else []) + [i + 1]
    if op in ("s_endpgm", "s_setpc_b64"):
        return []
    return [i + 1]


def _shortest(ins, idx, a, b, lo, hi):
    """instruction indices of a shortest path a -> b inside [lo, hi]"""
    dist, prev, pq = {a: 0}, {}, [(0, a)]
    while pq:
        d, i = heapq.heappop(pq)
        if i == b:
            break
        if d > dist.get(i, 1 << 60):
            continue
        for j in _succ(ins, i, idx):
            if lo <= j <= hi and d + 1 < dist.get(j, 1 << 60):
                dist[j], prev[j] = d + 1, i
                heapq.heappush(pq, (d + 1, j))
    path = [b]
    while path[-1] != a:
        path.append(prev[path[-1]])
    return path[::-1]


def _step_loops(ins):
    return [(h, e) for h, e in loops(ins)
            if e - h < 1500 and sum("ds_add" in t for _, t, _ in ins[h:e + 1]) >= 6
            and sum("buffer_load" in t for _, t, _ in ins[h:e + 1]) >= 10]


def shortest_iteration(ins):
    """instruction texts of the shortest path from the ADMM loop's header to its back edge through
    its first two solve-step loops (the forward and backward solves, each run once): an iteration of
    the solving wave that skips every check block"""
    idx = {a: i for i, (a, _, _) in enumerate(ins)}
    h, e = max(loops(ins), key=lambda x: x[1] - x[0])
    way = [h]
    for sh, se in sorted(l for l in _step_loops(ins) if h < l[0] and l[1] < e)[:2]:  # fwd, bwd
        way += [sh, se]
    way.append(e)
    path = [h]
    for a, b in zip(way, way[1:]):
        path += _shortest(ins, idx, a, b, h, e)[1:]
    return [ins[i][1] for i in path]


def test_non_check_iterations_reload_no_kernel_argument_and_few_spills(isa):
    for name, ins in isa.items():
        cap = next(v for k, v in NONCHECK_RELOADS.items() if k in name)
        path = shortest_iteration(ins)
        assert sum("ds_add_f64" in t for t in path) >= 6, (name, "not a solving path")
        assert not any(t.startswith("s_load") for t in path), name
        reloads = [t for t in path if t.startswith("v_readlane")]
        assert len(reloads) <= cap, (name, len(reloads), reloads[:6])
