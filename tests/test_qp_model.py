"""Restated QP assembly vs the reference's own construction (bit-exact).

Fixtures: tests/golden/cl_*.npz record the (P, q, A, l, u) the reference's trajectorySimulate
handed to OSQP and every per-step (Ax, l, u) update; batch_*.npz hold the reference's
configureDynamicConstraints outputs for 64 sampled estimates (see tests/golden/gen_fixtures.py).
"""
import numpy as np
import scipy.sparse as sp

from mpc_arpo_project_amd import qp_model, scenarios


def _check_setup(d, prob):
    P = sp.csc_matrix((d["P_data"], d["P_indices"], d["P_indptr"]), shape=tuple(d["P_shape"]))
    assert abs(P - prob.P).max() == 0
    assert np.array_equal(d["q"], prob.q)
    assert np.array_equal(d["A_indices"], prob.A.indices)
    assert np.array_equal(d["A_indptr"], prob.A.indptr)
    assert np.array_equal(d["A_data"], prob.A.data)
    assert np.array_equal(d["l"], prob.l) and np.array_equal(d["u"], prob.u)
    # quirk Q5: the COO data the reference passes is in CSC order
    assert np.array_equal(d["A_data_as_passed"], d["A_data"])


def test_setup_n20_bit_exact(golden, prob20):
    _check_setup(golden("cl_n20"), prob20)
    assert (prob20.n, prob20.m, prob20.nnzA, prob20.P.nnz) == (121, 226, 715, 20 * 4 + 16 + 35 + 2)


def test_setup_n40_deltav_bit_exact(golden, prob40):
    _check_setup(golden("cl_n40dv"), prob40)
    assert (prob40.n, prob40.m, prob40.nnzA) == (201, 406, 1335)


def test_discretization_fingerprint(prob20):
    # SURVEY.md 8(a) A7 fingerprints of the reference's discretization / DARE
    assert abs(prob20.Bd[0, 0] - 0.12499999681) < 1e-10
    assert abs(prob20.Ad[0, 2] - 0.49999997447) < 1e-10
    assert abs(prob20.S[3, 3] - 2.6940145674e6) < 1e-3
    assert abs(prob20.K[1, 3] - 0.91472414295) < 1e-10


def test_batch_configure_bit_exact(golden, prob20, prob40):
    for tag, prob in (("batch_n20", prob20), ("batch_n40dv", prob40)):
        d = golden(tag)
        Ax, l, u = qp_model.configure_batch(prob, d["xest"])
        assert np.array_equal(Ax, d["Ax"])
        assert np.array_equal(l, d["l"]) and np.array_equal(u, d["u"])
        for b in range(0, 64, 9):  # scalar restatement agrees with the batch one
            a1, li, ui = qp_model.configure_dynamic_constraints(prob, d["xest"][b].copy())
            l2, u2 = qp_model.full_bounds(prob, d["xest"][b], li, ui)
            assert np.array_equal(a1, Ax[b]) and np.array_equal(l2, l[b]) and np.array_equal(u2, u[b])


def test_closed_loop_updates_bit_exact(golden, prob20):
    """every (Ax, l, u) update the reference issued along its closed loop is reproduced from the
    recorded state estimate"""
    d = golden("cl_n20")
    xe = d["x_est"]
    for i in range(d["step_Ax"].shape[0]):
        Ax, li, ui = qp_model.configure_dynamic_constraints(prob20, xe[:, i + 1].copy())
        l, u = qp_model.full_bounds(prob20, xe[:, i + 1], li, ui)
        assert np.array_equal(Ax, d["step_Ax"][i])
        assert np.array_equal(l, d["step_l"][i]) and np.array_equal(u, d["step_u"][i])


def test_sampler_in_cone():
    X = scenarios.sample_estimates(1000)
    assert X.shape == (1000, 6)
    assert np.all(X[:, 0] - scenarios.LOS_COT * np.abs(X[:, 1]) >= 1.0)
    assert np.all((X[:, 0] >= 20) & (X[:, 0] <= 110) & (np.abs(X[:, 1]) <= 15))
    assert np.array_equal(X, scenarios.sample_estimates(1000))  # deterministic


def test_in_track_problem_builds():
    sim, mpc, fail, deb = scenarios.in_track_scenario(Nx=20)
    prob = qp_model.build_problem(sim, mpc, fail, deb)
    X = np.array([[-10., 100., 0., 0., 0., 0.], [3., 60., -0.1, -0.2, 0.1, 0.]])
    Ax, l, u = qp_model.configure_batch(prob, X)
    for b in range(2):
        a1, li, ui = qp_model.configure_dynamic_constraints(prob, X[b].copy())
        assert np.array_equal(a1, Ax[b])
        assert np.array_equal(qp_model.full_bounds(prob, X[b], li, ui)[0], l[b])


def _prob_in_track():
    from conftest import _PROBS

    if "intrack40" not in _PROBS:
        sim, mpc, fail, deb = scenarios.in_track_scenario(Nx=40, T_final=100)
        _PROBS["intrack40"] = qp_model.build_problem(sim, mpc, fail, deb)
    return _PROBS["intrack40"]


def test_in_track_setup_and_updates_bit_exact(golden):
    """the in-track approach (reference test/traj_eval_in_track.py, Nx = 40, swap_xy): set-up data
    and every per-step update the reference issued, reproduced bit for bit -- including quirk Q4
    (src/simhelpers.py:69-75: configureDynamicConstraints swaps x / y of the caller's estimate in
    place, so the reference's recorded estimates are the swapped ones)"""
    d = golden("cl_intrack_n40")
    prob = _prob_in_track()
    assert np.array_equal(d["setup_l"], prob.l) and np.array_equal(d["setup_u"], prob.u)
    assert np.array_equal(d["A_data"], prob.A.data)
    xe = d["x_est"]
    for i in range(d["step_Ax"].shape[0]):
        x = xe[:, i + 1].copy()
        x[[0, 1]] = x[[1, 0]]  # undo the in-place swap the reference's call left behind
        Ax, li, ui = qp_model.configure_dynamic_constraints(prob, x, swap_in_place=True)
        assert np.array_equal(x, xe[:, i + 1])  # ... which the restatement reproduces
        l, u = qp_model.full_bounds(prob, xe[:, i + 1][[1, 0, 2, 3, 4, 5]], li, ui)
        assert np.array_equal(Ax, d["step_Ax"][i]), i
        assert np.array_equal(l, d["step_l"][i]) and np.array_equal(u, d["step_u"][i]), i
