"""Build-time register / scratch guard of the product solve kernels (no GPU needed).

The gfx950 code object is taken out of libmpcqp.so (the .hip_fatbin offload bundle) and its
AMDHSA metadata notes are read: every solve kernel that a product handle can launch (one-wave
qp_batch_kernel without matrix prefetch, two-wave qp_pair_kernel with the solves on the first wave)
must allocate at most MPCQP_MAX_KERNEL_REGS registers per lane (arch VGPRs + AGPRs; builds above
~440 computed wrong iterates from a wave's second instance on, DESIGN.md High-register builds) and
at most MPCQP_MAX_KERNEL_SCRATCH bytes of scratch.  mpcqp_create applies the same budget to the
kernel it selects (hipFuncGetAttributes), so a rebuild that crosses it fails here and at run time.
"""
import os
import re
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "mpc_arpo_project_amd", "libmpcqp.so")
LLVM = "/opt/rocm/lib/llvm/bin"
# one-wave kernel mode KM_LDS (engine.hip: 0, the LDS-operand kernel);
# two-wave kernel mode 2 (solves on the first wave)
PRODUCT = re.compile(r"qp_batch_kernelILi\d+ELi\d+ELb[01]ELi0E|qp_pair_kernelILi\d+ELi\d+ELb[01]ELi2E")


def _header_budget(name):
    src = open(os.path.join(REPO, "include", "mpcqp.h")).read()
    return int(re.search(r"#define %s (\d+)" % name, src).group(1))


def kernel_resources(lib=LIB, tmp="/tmp"):
    """{kernel name: {vgpr_count, agpr_count, private_segment_fixed_size, ...}} of the gfx950 code
    object inside `lib`"""
    tools = [os.path.join(LLVM, t) for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-readelf")]
    if not all(os.path.exists(t) for t in tools) or not os.path.exists(lib):
        pytest.skip("ROCm LLVM tools or the library are missing")
    objcopy, bundler, readelf = tools
    fb = os.path.join(tmp, "mpcqp_fatbin_%d.bin" % os.getpid())
    co = os.path.join(tmp, "mpcqp_gfx950_%d.elf" % os.getpid())
    try:
        subprocess.check_call([objcopy, "--dump-section", ".hip_fatbin=" + fb, lib, os.devnull])
        subprocess.check_call([bundler, "--unbundle", "--type=o", "--input=" + fb,
                               "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + co])
        notes = subprocess.check_output([readelf, "--notes", co], text=True)
    finally:
        for f in (fb, co):
            if os.path.exists(f):
                os.remove(f)
    # kernel-level keys sit at one column of the amdhsa.kernels list ("  - .agpr_count: 50" starts
    # an entry, "    .name: ..." continues it); the nested .args entries are indented deeper
    out, cur, col = {}, {}, None
    for line in notes.splitlines():
        m = re.match(r"^(\s*)(-\s+)?\.(\w+):\s*(\S*)", line)
        if not m:
            continue
        c = len(m.group(1)) + len(m.group(2) or "")
        if m.group(2) and m.group(3) == "agpr_count":
            cur, col = {}, c
        if c != col:
            continue
        cur[m.group(3)] = m.group(4)
        if m.group(3) == "name":
            out[m.group(4)] = cur
    return out


def test_product_solve_kernels_within_budget():
    res = kernel_resources()
    regs, scratch = _header_budget("MPCQP_MAX_KERNEL_REGS"), _header_budget("MPCQP_MAX_KERNEL_SCRATCH")
    prod = {k: v for k, v in res.items() if PRODUCT.search(k)}
    assert len(prod) >= 8, sorted(res)  # (2,4) and (4,8) buckets x paired/unpaired x 1/2 waves
    for k, v in prod.items():
        assert int(v["vgpr_count"]) <= regs, (k, v)
        assert int(v["private_segment_fixed_size"]) <= scratch, (k, v)


def test_headline_kernel_has_no_vector_spills():
    """the N = 20 headline kernel (qp_batch_kernel<2,4,paired>) keeps every VGPR in registers"""
    res = kernel_resources()
    k = [v for n, v in res.items() if "qp_batch_kernelILi2ELi4ELb1ELi0E" in n]
    assert k and int(k[0]["vgpr_spill_count"]) == 0, k
