"""ADVICE r04 (engine_pair.inc): the two-wave kernel's instance hand-off relies on both waves
reading the same instance id and making the same number of cross-wave exchanges (so that they
agree on the exchange buffer's phase).  The diagnostic build -DMPCQP_PAIR_CHECKS
(tools/libmpcqp_pair_checks.so, built by __graft_entry__.build()) compares both at every hand-off
and reports a mismatch through the instance's status (-1000).  Here it runs the fixture batch
tiled to B = 8,192 (several instances per workgroup) in every two-wave mode, in a child process
(one library per process), and the product library must give the same bits.  The checks build's
barriers are LDS-counter barriers with a bounded wait: a skipped barrier must be
reported (status -1000), not hang the GPU -- tested by injecting one."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CHECKS_LIB = os.path.join(REPO, "tools", "libmpcqp_pair_checks.so")
MODES = {"auto": {}, "w2_split": {"MPCQP_WAVES": "2"}, "w3": {"MPCQP_WAVES": "3", "MPCQP_W0DIAG": "0"},
         "w3_w0diag": {"MPCQP_WAVES": "3", "MPCQP_W0DIAG": "1"}}


@pytest.mark.parametrize("mode", sorted(MODES))
@pytest.mark.parametrize("Nx,dv,tag", [(20, False, "batch_n20"), (40, True, "batch_n40dv")])
def test_pair_handoff_checks(tmp_path, Nx, dv, tag, mode):
    if not os.path.exists(CHECKS_LIB):
        pytest.skip("tools/libmpcqp_pair_checks.so not built (__graft_entry__.build())")
    if mode == "auto" and Nx == 20:
        pytest.skip("N = 20 runs the one-wave kernel by default")
    outs = {}
    for name, lib in (("checks", CHECKS_LIB), ("product", None)):
        env = dict(os.environ, MPCQP_DIAGNOSTICS="1", **MODES[mode])
        env.pop("MPCQP_LIBRARY", None)
        if lib:
            env["MPCQP_LIBRARY"] = lib
        out = str(tmp_path / f"{name}.npz")
        subprocess.run([sys.executable, os.path.join(HERE, "_pair_checks_run.py"), str(Nx),
                        str(int(dv)), tag, out], env=env, check=True, timeout=240)
        outs[name] = np.load(out)
    a, b = outs["checks"], outs["product"]
    assert int(a["waves_per_instance"]) == 2, "not the two-wave kernel"
    for k in ("status0", "status1"):
        assert not np.any(a[k] == -1000), (k, np.nonzero(a[k] == -1000)[0][:8])
    for k in ("status0", "iter0", "x0", "y0", "status1", "iter1", "x1", "y1"):
        assert np.array_equal(a[k], b[k], equal_nan=True), k


def test_checked_barrier_reports_an_injected_divergence(tmp_path):
    """wave 1 of workgroup 0 skips one barrier in its first instance: the checked barrier's bounded
    wait and the hand-off check turn that into status -1000 on some instance of the first solve
    (instead of a hang), and the next launch, without the skip, is clean again"""
    if not os.path.exists(CHECKS_LIB):
        pytest.skip("tools/libmpcqp_pair_checks.so not built (__graft_entry__.build())")
    env = dict(os.environ, MPCQP_DIAGNOSTICS="1", MPCQP_LIBRARY=CHECKS_LIB)
    out = str(tmp_path / "inject.npz")
    subprocess.run([sys.executable, os.path.join(HERE, "_pair_checks_run.py"), "40", "1",
                    "batch_n40dv", out, "inject"], env=env, check=True, timeout=240)
    a = np.load(out)
    assert int(a["waves_per_instance"]) == 2, "not the two-wave kernel"
    assert np.any(a["status0"] == -1000), "the skipped barrier was not reported"
    assert not np.any(a["status1"] == -1000), np.nonzero(a["status1"] == -1000)[0][:8]
