"""The reference's Monte-Carlo experiments on the host side (no GPU): the seed-123 noise stream the
sweep driver replays (mpc_arpo_project_amd.sweep.reference_noise) against the noise the reference's
own trajectorySimulate drew in every recorded run (tests/golden/exp_*.npz, gen_experiments.py),
and the fixture's own consistency (the scripts' outputs follow from one run per setting)."""
import numpy as np

from mpc_arpo_project_amd import sweep


def _check_noise(hist, sig, L):
    """hist: the reference's noiseStored[:, :i_term + 1]; column t holds draw t // L"""
    t = np.arange(hist.shape[1])
    w = sweep.reference_noise(sig, t[-1] // int(L) + 1)
    assert np.array_equal(w[t // int(L)].T, hist)


def test_reference_noise_stream_matches_disturb_rej_runs(golden):
    d = golden("exp_disturb_rej")
    for i, L in enumerate(d["noise_lengths"]):
        for j in range(2):
            _check_noise(d[f"noise_{i}_{j}"], (0.7, 0.7), L)


def test_reference_noise_stream_matches_success_rates_run(golden):
    _check_noise(golden("exp_success_rates")["noise"], (0.3, 0.3), 50)


def test_experiment_fixture_outputs():
    from conftest import load_golden

    d = load_golden("exp_disturb_rej")
    # the reference's MC repetitions are identical runs (re-seeded with 123 at every call)
    assert bool(d["mc_repeat_identical"])
    fe = d["final_err"]
    assert np.allclose(d["dist_ratios"], fe[:, :, 1] / fe[:, :, 0], rtol=0, atol=0)
    s = load_golden("exp_success_rates")
    assert int(s["success_count"]) == int(s["mc"]) * int(s["success"][0])


def test_experiment_scenario_defaults():
    assert sweep.SCENARIO_DEFAULTS["radial"] == dict(nx=40, noise="0.75,0.75,50", reject=True,
                                                     tfinal=150.0)
    assert sweep.SCENARIO_DEFAULTS["in_track"]["noise"] == "none"
