"""Offline schedule simulation of the timed bench window from per-(step, chaser) ADMM iterations
(tools/iters_dump.py): makespan of the 20 timed steps on S slots under (a) one launch per step
(greedy list scheduling in chaser order), (b) one launch for all steps with a chaser's steps run
back to back by one wave (units in chaser order), (c) the same with units longest-first by the
warm-up steps' iterations, (d) a dynamic (chaser, step) queue.  Cost of a solve = iterations + OVH
(the Ruiz passes and the factorization in iteration units).  usage: python tools/sched_sim.py it.npz"""
import heapq
import sys

import numpy as np

d = np.load(sys.argv[1])
it, act = d["iters"].astype(np.float64), d["active"]
W, K, S, OVH = 5, 20, 1024, 33.0
cost = np.where(act, it + OVH, 0.0)
T = cost[W:W + K]                       # [K][B]
B = T.shape[1]


def list_sched(jobs, slots=S):
    h = [0.0] * slots
    heapq.heapify(h)
    for c in jobs:
        t = heapq.heappop(h)
        heapq.heappush(h, t + c)
    return max(h)


per_step = sum(list_sched(T[k][T[k] > 0]) for k in range(K))
units = T.sum(axis=0)
fifo_units = list_sched(units)
pred = cost[1:W].sum(axis=0)
lpt_pred = list_sched(units[np.argsort(-pred, kind="stable")])
lpt_oracle = list_sched(np.sort(units)[::-1])
# dynamic queue: event simulation, FIFO by release time
h = [(0.0, s) for s in range(S)]
heapq.heapify(h)
ready = [(0.0, b, 0) for b in range(B)]  # (release time, chaser, step)
heapq.heapify(ready)
end = 0.0
while ready:
    rt, b, k = heapq.heappop(ready)
    t, s = heapq.heappop(h)
    t0 = max(t, rt)
    t1 = t0 + T[k][b]
    end = max(end, t1)
    heapq.heappush(h, (t1, s))
    if k + 1 < K:
        heapq.heappush(ready, (t1, b, k + 1))
lb = T.sum() / S
print(f"work/S (lower bound) {lb:.0f}")
for name, v in (("per-step launches", per_step), ("fused units, chaser order", fifo_units),
                ("fused units, longest-first by warm-up iters", lpt_pred),
                ("fused units, longest-first (oracle)", lpt_oracle), ("dynamic (chaser, step) queue", end)):
    print(f"{name:45s} {v:12.0f}  idle {1 - lb / v:6.2%}  vs per-step {per_step / v - 1:+6.2%}")
# per-step launches ordered longest-first by the previous step's iterations / by the true ones
prev = sum(list_sched(T[k][np.argsort(-cost[W + k - 1], kind="stable")][T[k][np.argsort(-cost[W + k - 1], kind="stable")] > 0]) for k in range(K))
orc = sum(list_sched(np.sort(T[k][T[k] > 0])[::-1]) for k in range(K))
print(f"{'per-step, longest-first by previous step':45s} {prev:12.0f}  idle {1 - lb / prev:6.2%}  vs per-step {per_step / prev - 1:+6.2%}")
print(f"{'per-step, longest-first (oracle)':45s} {orc:12.0f}  idle {1 - lb / orc:6.2%}  vs per-step {per_step / orc - 1:+6.2%}")
c = np.corrcoef(cost[W:W + K - 1].ravel(), cost[W + 1:W + K].ravel())[0, 1]
print("corr(iters step k, step k+1)", round(c, 3), " share of solves at max_iter", float((it[W:W+K] >= 4000).mean()))
