#!/bin/bash
# round-2 parity characterisation + occupancy scan (GPU box).  usage: tools/r02_parity.sh <tag>
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${1:-par}"; mkdir -p "$O"; cd "$R"
echo "cpus: nproc=$(nproc) affinity=$(python -c 'import os;print(len(os.sched_getaffinity(0)))') quota=$(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"
timeout -k 10 200 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1 || { echo "pytest failed"; tail -40 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
for tag in n20 n40dv; do
  F=""; [ $tag = n40dv ] && F="--nx 40 --dv"
  timeout -k 10 200 python tools/parity_scale.py cold $F > "$O/cold_$tag.json" 2> "$O/cold_$tag.err" || { echo "cold $tag failed"; tail -5 "$O/cold_$tag.err"; exit 1; }
  python -c "import json;d=json.load(open('$O/cold_$tag.json'));d.pop('iter_diff_examples');print(d)"
done
timeout -k 10 300 python tools/parity_scale.py growth --threads 16 > "$O/growth.json" 2> "$O/growth.err" || { echo growth failed; tail -5 "$O/growth.err"; exit 1; }
python -c "import json;d=json.load(open('$O/growth.json'));[print(r) for r in d['rows']]"
for pad in 90000 40000 15600 0; do
  MPCQP_LDS_PAD=$pad timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 3 --split 1 > "$O/occ_$pad.json" 2> "$O/occ_$pad.err" || { echo "occ $pad failed"; tail -5 "$O/occ_$pad.err"; exit 1; }
  python -c "import json;d=json.load(open('$O/occ_$pad.json'));print('pad $pad', d['schedule']['waves_per_cu'], 'solves/s', round(d['value']), 'kernel ms', round(d['roofline']['kernel_ms_per_launch'],2), 'iters', d['admm_iters']['mean'])"
done
timeout -k 10 400 python tools/parity_scale.py warm --batch 16384 --threads 16 > "$O/warm.json" 2> "$O/warm.err" || { echo warm failed; tail -5 "$O/warm.err"; exit 1; }
python -c "
import json;d=json.load(open('$O/warm.json'))
for m in ('free','sync'):
  x=d[m]; print(m, 'status_agree', x['status_agree_mean'], 'iter_agree', x['iter_agree_mean'], 'ever', x['chasers_ever_diverged'], x['first_divergence_hist'])
  for s in x['steps']: print('  ', s['step'], s['status_agree'], s['iter_agree'], s['flips'], s['max_du0_same_iter'], s['max_du0_diff_iter'])
"
