"""Multi-rank plumbing of the sharded workload on CPU (gloo, world_size 2): every rank builds its
contiguous shard of chasers from the global seed, computes its per-step QP data, and the final
all-gather reproduces the single-process batch exactly (what bench.py relies on for N > 1)."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, B, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from conftest import problem
    from mpc_arpo_project_amd import qp_model

    prob = problem(20, False)
    X = bench.initial_states(world * B, rank, B, 20250328)
    xest = np.hstack([X, np.zeros((B, 2))])
    Ax, l, u = qp_model.configure_batch(prob, xest)
    t = torch.as_tensor(np.hstack([Ax, l, u]))
    g = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(g, t)
    if rank == 0:
        torch.save(torch.cat(g), out_path)
    dist.destroy_process_group()


def test_sharded_gather_matches_single_process(tmp_path):
    world, B = 2, 16
    out = str(tmp_path / "gathered.pt")
    mp.spawn(_worker, args=(world, _free_port(), B, out), nprocs=world, join=True)
    gathered = torch.load(out, weights_only=True).numpy()
    import bench
    from conftest import problem
    from mpc_arpo_project_amd import qp_model

    prob = problem(20, False)
    X = bench.initial_states(world * B, 0, world * B, 20250328)
    Ax, l, u = qp_model.configure_batch(prob, np.hstack([X, np.zeros((world * B, 2))]))
    assert np.array_equal(gathered, np.hstack([Ax, l, u]))


def test_shard_ranges_cover_batch():
    import bench

    world, B = 4, 8
    parts = [bench.initial_states(world * B, r, B, 7) for r in range(world)]
    full = bench.initial_states(world * B, 0, world * B, 7)
    assert np.array_equal(np.vstack(parts), full)


def _summary_rows(G, lo, hi):
    """a deterministic per-scenario summary of global ids [lo, hi): the sweep's initial
    conditions and the restated configure data's row sums (what a rank computes for its shard)"""
    from mpc_arpo_project_amd import sweep

    X = sweep.scenario_states("in_track", 4, G // 4, lo, hi, ic_seed=99)
    g = np.arange(lo, hi, dtype=np.float64)[:, None]
    return torch.as_tensor(np.hstack([g, X, X.sum(axis=1, keepdims=True) * g]))


def _gather_worker(rank, world, port, G, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mpc_arpo_project_amd import launch

    lo, hi = launch.shard_range(G, rank, world)
    full = launch.gather_rows(_summary_rows(G, lo, hi), G, rank, world, dist)
    if rank == 0:
        torch.save(full, out_path)
    dist.destroy_process_group()


def test_summary_gather_matches_single_process(tmp_path):
    """uneven shards (G = 4 x 13 over 3 ranks) gathered with launch.gather_rows equal the
    single-process rows: the sweep's / bench's per-scenario summary path"""
    world, G = 3, 52
    out = str(tmp_path / "summ.pt")
    mp.spawn(_gather_worker, args=(world, _free_port(), G, out), nprocs=world, join=True)
    full = torch.load(out, weights_only=True)
    assert torch.equal(full, _summary_rows(G, 0, G))


def test_sweep_grid_and_in_track_ics():
    from mpc_arpo_project_amd import sweep

    ics = sweep.initial_conditions("in_track", 64, seed=3)
    rad = sweep.initial_conditions("radial", 64, seed=3)
    assert np.array_equal(ics[:, [1, 0, 2, 3]], rad)  # the radial geometry turned on its side
    assert np.all(ics[:, 2:] == 0.0)
    X = sweep.scenario_states("radial", 3, 64, 100, 140, ic_seed=3)
    assert np.array_equal(X, rad[np.arange(100, 140) % 64])


def _traj_rows(G, lo, hi, steps=7):
    """a deterministic stand-in for the closed loops' trajectories of global ids [lo, hi) (initial
    state of each scenario propagated by a fixed linear map, as the device loop records x_true)"""
    from mpc_arpo_project_amd import sweep

    X = torch.as_tensor(sweep.scenario_states("radial", 5, G // 5, lo, hi, ic_seed=11))
    M = torch.tensor([[1.0, 0.0, 0.5, 0.0], [0.0, 1.0, 0.0, 0.5], [0.01, 0.0, 0.99, 0.02],
                      [0.0, -0.01, -0.02, 0.99]], dtype=torch.float64)
    out = [X]
    for _ in range(steps):
        out.append(out[-1] @ M.T)
    return torch.stack(out, dim=1)  # [hi - lo, steps + 1, 4]


def _traj_worker(rank, world, port, G, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mpc_arpo_project_amd import launch, sweep

    lo, hi = launch.shard_range(G, rank, world)
    full = sweep.gather_traj(_traj_rows(G, lo, hi), G, rank, world, dist)
    if rank == 0:
        torch.save(full, out_path)
    else:
        assert full is None
    dist.destroy_process_group()


def test_trajectory_gather_matches_single_process(tmp_path):
    """`sweep --traj`: uneven shards (G = 5 x 11 over 2 and 3 ranks) gathered to rank 0 with
    sweep.gather_traj equal the single-process trajectories, in global scenario order"""
    G = 55
    ref = _traj_rows(G, 0, G)
    for world in (2, 3):
        out = str(tmp_path / f"traj{world}.pt")
        mp.spawn(_traj_worker, args=(world, _free_port(), G, out), nprocs=world, join=True)
        assert torch.equal(torch.load(out, weights_only=True), ref)
