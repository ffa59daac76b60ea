#!/bin/bash
# Round-4 evidence on one GPU box: the parity tests with their printouts (calibrated floors,
# reference experiments), the config-5 share at the reference's radial configuration (Nx = 40,
# noise 0.75 held 50 samples, 131,072 scenarios), and the reference's two experiments with the
# reference noise stream.   usage: tools/r4_evidence.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-evidence}"; mkdir -p "$O"; export TMPDIR=/tmp; cd "$R"
[ -n "$EV_SKIP_TESTS" ] || { timeout -k 10 600 python3 -u -m pytest $R/tests/test_gpu_experiments.py "$R/tests/test_gpu_scale_parity.py::test_warm_closed_loop_lockstep" $R/tests/test_gpu_sweep_parity.py -x -v -s --timeout 400 --timeout-method thread > "$O/parity_printouts.log" 2>&1 || { echo "parity tests failed"; tail -30 "$O/parity_printouts.log"; exit 1; }
tail -1 "$O/parity_printouts.log"; }
timeout -k 10 300 python3 -m mpc_arpo_project_amd.sweep --seeds 128 --ics 1024 > "$O/sweep_131k_radial_n40.json" 2> "$O/sweep.err" || { echo "sweep failed"; tail -5 "$O/sweep.err"; exit 1; }
head -c 400 "$O/sweep_131k_radial_n40.json"; echo
timeout -k 10 300 python3 -m mpc_arpo_project_amd.sweep --experiment disturb_rej > "$O/disturb_rej_reference.json" 2> "$O/exp1.err" || { echo "disturb_rej failed"; tail -5 "$O/exp1.err"; exit 1; }
python3 -c "import json;d=json.load(open('$O/disturb_rej_reference.json'));print('disturb_rej', d['dist_ratios'], d['seconds'])"
timeout -k 10 300 python3 -m mpc_arpo_project_amd.sweep --experiment success_rates > "$O/success_rates_reference.json" 2> "$O/exp2.err" || { echo "success_rates failed"; tail -5 "$O/exp2.err"; exit 1; }
python3 -c "import json;d=json.load(open('$O/success_rates_reference.json'));print('success_rates', d['success_count'], d['settings'][0]['mc_runs_identical'], d['seconds'])"
