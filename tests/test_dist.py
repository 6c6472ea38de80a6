"""Multi-process (world_size 2, CPU) coverage of the N>1 path (SURVEY §8e replicas, BASELINE
configs[3]): `bench.py --gpus N` starts its own ranks (topfusion_amd/replicas.launch), or runs as
one rank of a torchrun launch; every rank tracks its own stream (seed 7 + rank) and the job's
numbers are the MAX of the rank times and the SUM of the rank frames.  The CPU runs use the
`--standin` workload (the oracle on an 80x60 stream) and the file collective; the RCCL
collective itself is covered on the GPU (tests/test_gpu_replicas.py)."""
import ctypes
import json
import os
import socket
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "TFUSION_RDZV_DIR", "TFUSION_LAUNCHED"):
        env.pop(k, None)
    return env


def _line(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out                      # rank 0 prints the one line
    return json.loads(lines[0])


def _check_line(d, world):
    m = d["multi_gpu"]
    assert d["n_gpus"] == world and m["world"] == world and m["collective_nranks"] == world
    assert d["config"]["parallelism"] == f"replicas{world}"
    assert len(m["per_rank_frames_per_sec"]) == world
    assert m["per_rank_frames"] == [d["steps"]] * world
    emax = max(m["per_rank_elapsed_s"])
    assert d["value"] == pytest.approx(sum(m["per_rank_frames"]) / emax, rel=1e-3)   # SUM frames / MAX time
    for fps, e, f in zip(m["per_rank_frames_per_sec"], m["per_rank_elapsed_s"], m["per_rank_frames"]):
        assert fps == pytest.approx(f / e, rel=1e-2)
    assert "efficiency" not in json.dumps(d)         # the driver computes scaling itself
    # the line proves itself: every rank's device (distinct) and its own frame verdicts
    assert len(m["per_rank_device"]) == world and m["distinct_devices"] is True
    assert len(set(m["per_rank_device"])) == world
    assert len(m["per_rank_frames_ok"]) == world and all(0 <= v <= d["steps"] for v in m["per_rank_frames_ok"])


def test_bench_launches_its_own_ranks():
    """`python bench.py --gpus 2`: the parent starts two ranks; one line with n_gpus 2."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--standin", "--steps", "2"],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    d = _line(r.stdout)
    _check_line(d, 2)
    assert d["multi_gpu"]["collective"] == "file"


def test_bench_under_torchrun():
    """The driver's torchrun form: each rank started by torch.distributed.run; the ranks meet in
    a directory named after the agent process."""
    port = _free_port()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port),
                        os.path.join(ROOT, "bench.py"), "--gpus", "2", "--standin", "--steps", "2"],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    _check_line(_line(r.stdout), 2)


def test_duplicate_device_exits_nonzero():
    """Two ranks that report the same device: rank 0 prints the line (distinct_devices false, both
    bus ids) and the job exits non-zero -- an N-GPU number must come from N GPUs."""
    env = _env()
    env["TFUSION_STANDIN_SAME_DEVICE"] = "1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--standin", "--steps", "2"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    d = _line(r.stdout)
    assert d["multi_gpu"]["distinct_devices"] is False and "same device" in r.stderr


def test_bus_id_format():
    from topfusion_amd import replicas
    v = replicas.parse_bus_id("0000:c1:00.0")
    assert v == [0, 0xc1, 0, 0] and replicas.format_bus_id(v) == "0000:c1:00.0"


def test_world_mismatch_exits_nonzero():
    env = _env()
    env.update(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--standin"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE 3" in r.stderr


def test_launcher_stops_the_job_when_a_rank_fails(tmp_path):
    """A failing rank ends the job with its status; the other rank (blocked forever) is stopped."""
    from topfusion_amd import replicas
    script = tmp_path / "rank.py"
    script.write_text(textwrap.dedent("""
        import os, sys, time
        if os.environ["RANK"] == "1":
            sys.exit(7)
        time.sleep(600)
    """))
    import time
    t0 = time.monotonic()
    assert replicas.launch(str(script), [], 2) == 7
    assert time.monotonic() - t0 < 60


def _fg_worker(rank, world, path, q):
    sys.path.insert(0, ROOT)
    from topfusion_amd import replicas
    g = replicas.FileGroup(rank, world, path)
    mx = g.allreduce([1.0 + rank, -rank], "max")
    sm = g.allreduce([1.0 + rank, 10.0], "sum")
    ag = g.allgather([rank, rank * 2])
    g.barrier()
    g.close()
    q.put((rank, mx, sm, ag))


def test_file_group_collectives(tmp_path):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_fg_worker, args=(r, 3, str(tmp_path), q)) for r in range(3)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(3))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, mx, sm, ag in res:
        assert mx == [3.0, 0.0]
        assert sm == [6.0, 30.0]
        assert ag == [[0, 0], [1, 2], [2, 4]]


def test_single_rank_passthrough():
    from topfusion_amd import replicas
    rep = replicas.Replicas(0, 0, 1)
    emax, total, multi = rep.summary(0.5, 10)
    assert (emax, total) == (0.5, 10.0) and multi["world"] == 1
    rep.close()


def test_rccl_symbols_present():
    """The RCCL entry points RcclGroup binds exist in /opt/rocm/lib/librccl.so (loaded, not called:
    no GPU here)."""
    from topfusion_amd import replicas
    if not os.path.exists(replicas.RCCL_PATH):
        pytest.skip("no librccl in this image")
    lib = ctypes.CDLL(replicas.RCCL_PATH)
    for f in ("ncclGetUniqueId", "ncclCommInitRank", "ncclAllReduce", "ncclAllGather", "ncclCommCount",
              "ncclCommDestroy", "ncclGetErrorString"):
        assert hasattr(lib, f), f
    assert ctypes.sizeof(replicas._UniqueId) == 128


def test_every_bench_config_has_a_runner():
    """Each --config choice of bench.py dispatches to a function the module defines (a config
    whose runner went missing would only fail on the GPU box)."""
    import bench
    import inspect
    src = inspect.getsource(bench.main)
    for cfg, fn in (("C3I", "c3_integrate"), ("C3R", "c3_raycast"), ("C5E", "c5e_bench")):
        assert fn in src, (cfg, fn)
        assert callable(getattr(bench, fn, None)), fn
