"""SURVEY 5 sanitizer row: the engine's host code -- the planner
(csrc/symbolic.cpp: it packs LDS byte addresses and indices into uint16_t and masked fields), the LDS
layout optimiser (lds_layout.cpp), the CPU interpreter of the compiled device program (emulate.cpp)
and the host entry points of the C ABI (host_abi.cpp) -- built with AddressSanitizer +
UndefinedBehaviorSanitizer (tools/sanitize/Makefile: a host-only library, no GPU code) and driven by
the host tests themselves in a child process with libasan preloaded: the emulated schedules of both
product plans (N = 20 one wave, N = 40 delta-v two waves), the horizons up to the largest bucket,
both step kinds on random structures, the layout optimiser and the host paths of test_abi.py.  Any
ASan report or UBSan runtime error aborts the child (halt_on_error) and fails this test.  The full
tests/test_schedule.py under the sanitizers (55 cases, ~15 min) was run once for the record:
profiles/r05/sanitize_full.log."""
import os
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "build", "sanitize", "libmpcqp_host_asan.so")

# the subset run in the CPU suite (each case re-plans under the sanitizers, 15-40 s apiece; four
# workers)
SELECT = [
    "tests/test_schedule.py::test_emulated_schedule_solves_kkt[20-False-1]",
    "tests/test_schedule.py::test_emulated_schedule_solves_kkt[40-True-3]",
    "tests/test_schedule.py::test_emulated_schedule_solves_kkt[51-False-1]",
    "tests/test_schedule.py::test_layout_optimiser_lowers_modelled_lds_cycles",
    "tests/test_schedule.py::test_emulated_schedule_random_structures[1-0-4-1]",
    "tests/test_schedule.py::test_emulated_schedule_random_structures[2-1-4-2]",
    "tests/test_abi.py::test_host_only_entry_points",
    "tests/test_abi.py::test_symbolic_analysis_matches_oracle_factor",
    "tests/test_abi.py::test_invalid_structure_rejected",
]


def _asan_runtime():
    cxx = shutil.which("g++")
    if not cxx:
        return None
    p = subprocess.check_output([cxx, "-print-file-name=libasan.so"], text=True).strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


def build_sanitized():
    if shutil.which("make") is None or _asan_runtime() is None:
        pytest.skip("g++ / make / libasan not available")
    subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "tools", "sanitize")])
    return LIB


def run_under_sanitizers(tests, timeout=900):
    lib = build_sanitized()
    env = dict(os.environ, LD_PRELOAD=_asan_runtime(), MPCQP_DIAGNOSTICS="1", MPCQP_LIBRARY=lib,
               ASAN_OPTIONS="detect_leaks=0:verify_asan_link_order=0:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        "-n", str(min(4, len(tests))), *tests],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=timeout)
    return r


def test_host_code_clean_under_asan_ubsan():
    r = run_under_sanitizers(SELECT)
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]
    assert f"{len(SELECT)} passed" in out, out[-2000:]


if __name__ == "__main__":  # the full run for the record: python tests/test_sanitize.py
    res = run_under_sanitizers(["tests/test_schedule.py", "tests/test_abi.py::test_horizon_limits"]
                               + SELECT[-3:], timeout=3600)
    print(res.stdout[-3000:], res.stderr[-3000:])
    sys.exit(res.returncode)
