"""Multi-process (world_size 2, gloo, CPU) coverage of the N>1 path: bench.py's replicas
semantics -- each rank tracks its own independent stream (seed 7 + rank), the whole-job
numbers are MAX over rank times and SUM over rank frames (bench.combine_ranks)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    import bench
    from oracle import oracle as O
    from topfusion_amd import synth
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # replica: an independent 80x60 stream per rank through the CPU oracle
        W, H = 80, 60
        fx, fy, cx, cy = synth.intrinsics(W, H)
        frames = synth.orbit_sequence(3, W, H, seed=7 + rank)
        o = O.Oracle(cols=W, rows=H, fx=fx, fy=fy, cx=cx, cy=cy)
        n_ok = sum(bool(o(f)) for f in frames)
        elapsed = 1.0 + rank                  # deterministic stand-in times
        emax, total = bench.combine_ranks(elapsed, len(frames), "cpu", world)
        q.put((rank, emax, total, n_ok, int(frames.astype(np.int64).sum())))
    finally:
        dist.destroy_process_group()


def test_replicas_combine_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    for rank, emax, total, n_ok, _ in res:
        assert emax == 2.0                     # slowest rank
        assert total == 6.0                    # frames of all ranks
        assert n_ok >= 1
    assert res[0][4] != res[1][4]              # independent streams (seed 7 + rank)


def test_single_rank_passthrough():
    sys.path.insert(0, ROOT)
    import bench
    assert bench.combine_ranks(0.5, 10, "cpu", 1) == (0.5, 10.0)


def test_every_bench_config_has_a_runner():
    """Each --config choice of bench.py dispatches to a function the module defines (a config
    whose runner went missing would only fail on the GPU box)."""
    sys.path.insert(0, ROOT)
    import bench
    import inspect
    src = inspect.getsource(bench.main)
    for cfg, fn in (("C3I", "c3_integrate"), ("C3R", "c3_raycast"), ("C5E", "c5e_bench")):
        assert fn in src, (cfg, fn)
        assert callable(getattr(bench, fn, None)), fn
