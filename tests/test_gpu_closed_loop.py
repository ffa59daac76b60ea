"""Device-resident closed loop (mpcqp_cl_* kernels + engine) vs the reference trajectory, and the
GPU-backed restated trajectorySimulate vs the same fixture."""
import numpy as np
import pytest
import torch

from mpc_arpo_project_amd import scenarios
from mpc_arpo_project_amd.closed_loop import BatchClosedLoop
from mpc_arpo_project_amd.simulate import trajectorySimulate

pytestmark = pytest.mark.gpu


def test_trajectory_simulate_on_gpu_matches_reference_loop(golden):
    d = golden("cl_n20")
    sim, mpc, fail, deb = scenarios.radial_scenario(Nx=20)
    run = trajectorySimulate(sim, mpc, fail, deb)  # default solver: the HIP engine
    assert run.i_term == int(d["i_term"])
    assert run.isSuccess == bool(d["isSuccess"])
    assert np.array_equal(run.ctrlr_seq, d["ctrlr_seq"])
    assert np.max(np.abs(run.x_true_pcw - d["x_true_pcw"])) < 1e-6


def test_device_closed_loop_single_chaser(golden, prob20):
    d = golden("cl_n20")
    cl = BatchClosedLoop(prob20, np.array([[100., 10., 0., 0.]]))
    iterm = int(d["i_term"])
    xs = [cl.x_true.cpu().numpy()[0].copy()]
    for i in range(iterm):
        cl.step()
        xs.append(cl.x_true.cpu().numpy()[0].copy())
        assert int(cl.ctrl_seq[0]) == int(d["ctrlr_seq"][i]), i
    xs = np.array(xs).T  # (4, iterm + 1)
    assert np.max(np.abs(xs[:, :iterm] - d["x_true_pcw"])) < 1e-6
    assert np.max(np.abs(cl.ctrl_prev.cpu().numpy()[0] - d["ctrl_hist"][:, iterm])) < 1e-8
    assert int(cl.done[0]) == 1  # the termination test fires where the reference stopped
    cl.close()


def test_shard_invariance(prob20):
    """an instance's result does not depend on its batch neighbours / position (the property the
    multi-GPU sharding relies on)"""
    X = scenarios.sample_estimates(48, seed=5)[:, :4]
    X[:, 2:] = 0.0
    full = BatchClosedLoop(prob20, X, eps_abs=1e-4, eps_rel=1e-4)
    part = BatchClosedLoop(prob20, X[16:32], eps_abs=1e-4, eps_rel=1e-4)
    for _ in range(5):
        rf = full.step()
        rp = part.step()
    torch.cuda.synchronize()
    assert torch.equal(full.x_true[16:32], part.x_true)
    assert torch.equal(rf.iter[16:32], rp.iter)
    full.close()
    part.close()


def test_sharded_closed_loop_matches_single_stream(prob20):
    """two shards on concurrent streams reproduce the one-stream batch bit for bit"""
    from mpc_arpo_project_amd.closed_loop import ShardedClosedLoop

    X = scenarios.sample_estimates(40, seed=11)[:, :4]
    X[:, 2:] = 0.0
    one = BatchClosedLoop(prob20, X, eps_abs=1e-4, eps_rel=1e-4)
    two = ShardedClosedLoop(prob20, X, shards=2, eps_abs=1e-4, eps_rel=1e-4)
    for _ in range(6):
        r1 = one.step()
        r2 = two.step()
    two.synchronize()
    torch.cuda.synchronize()
    assert torch.equal(one.x_true, two.x_true)
    assert torch.equal(r1.iter, torch.cat([r.iter for r in r2]))
    assert torch.equal(one.ctrl_seq, two.ctrl_seq)
    one.close()
    two.close()
