"""One process per GPU: launch helpers shared by bench.py and the sweep driver.

`relaunch(ngpus, argv)` -- when a script is asked for N > 1 GPUs but was not started by
torch.distributed.run, start `python -m torch.distributed.run --nproc-per-node N ...` on the same
script as a CHILD process and return its exit code (the caller exits with it).  It must run
before anything initialises the GPU (no exec: the parent never touched HIP).
`init(backend)` -- rank / world / local rank from the launcher's environment, the rank's device
and the process group (RCCL over xGMI for "nccl"); single-process runs get no group.
`shard_range(G, rank, world)` -- the contiguous block of global ids a rank owns.
`gather_rows(t, G, rank, world, dist)` -- all ranks' [n_rank, F] blocks -> [G, F] (one all-gather
of equal, padded blocks: RCCL needs equal sizes).
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launched() -> bool:
    return "WORLD_SIZE" in os.environ and "RANK" in os.environ


def relaunch(ngpus: int, argv, module: str = None) -> int:
    """Run this program under torch.distributed.run with `ngpus` ranks (child process)."""
    target = ["--module", module] if module else [os.path.abspath(argv[0])]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={ngpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), *target, *argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def init(backend: str = "nccl"):
    """(rank, world, local_rank, device, dist-or-None); sets the rank's current device."""
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend == "nccl":
        if not torch.cuda.is_available():
            raise SystemExit("a ROCm GPU is required")
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    dist = None
    if world > 1:
        import torch.distributed as dist

        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)
    return rank, world, local, device, dist


def shard_range(G: int, rank: int, world: int):
    return G * rank // world, G * (rank + 1) // world


def gather_rows(t, G: int, rank: int, world: int, dist):
    """[hi - lo, F] rows of every rank -> [G, F] in global-id order (every rank gets it)."""
    import torch

    if dist is None or world == 1:
        return t
    per = -(-G // world)
    pad = torch.zeros((per,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[:t.shape[0]] = t
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad)
    rows = [parts[r][:shard_range(G, r, world)[1] - shard_range(G, r, world)[0]]
            for r in range(world)]
    return torch.cat(rows)
