"""GPU coverage of the replicas collective (topfusion_amd/replicas.py): RCCL through ctypes on the
product's HIP runtime.  A one-GPU box runs a one-rank communicator in this process, and (when
RCCL accepts two ranks on one device) the whole `bench.py --gpus 2` launcher path on the C5E
engine workload, whose frames need no co-resident persistent grid."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu


def test_rccl_one_rank(tmp_path):
    from topfusion_amd import replicas
    files = replicas.FileGroup(0, 1, str(tmp_path))
    g = replicas.RcclGroup(0, 1, 0, files)
    try:
        assert g.nranks() == 1
        assert g.allreduce([3.5, -2.0], "max") == [3.5, -2.0]
        assert g.allreduce([1.25], "sum") == [1.25]
        assert g.allgather([7.0, 8.0]) == [[7.0, 8.0]]
        g.barrier()
    finally:
        g.close()


def _two_ranks(collective):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "TFUSION_RDZV_DIR", "TFUSION_LAUNCHED"):
        env.pop(k, None)
    env["TFUSION_RANK_DEVICE_MODULO"] = "1"
    env["TFUSION_RDZV_TIMEOUT"] = "90"
    env["NCCL_DEBUG"] = "WARN"
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "C5E",
                           "--steps", "2", "--warmup", "1", "--frames-per-step", "50", "--collective", collective],
                          cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)


def _check(r, collective):
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    m = d["multi_gpu"]
    assert d["n_gpus"] == 2 and m["collective"] == collective and m["collective_nranks"] == 2
    assert m["per_rank_frames"] == [100, 100]
    assert d["value"] == pytest.approx(200 / max(m["per_rank_elapsed_s"]), rel=1e-3)


def test_bench_two_ranks_one_device_file_collective():
    """`bench.py --gpus 2` on a one-GPU box: the launcher starts two ranks, both on device 0
    (TFUSION_RANK_DEVICE_MODULO, tests only), each fusing its own C5E stream; the numbers are
    combined over the file collective."""
    _check(_two_ranks("file"), "file")


def test_bench_two_ranks_one_device_rccl():
    """The same over RCCL.  RCCL refuses two ranks on one device ("Duplicate GPU detected", an
    invalid-usage error raised after the bootstrap exchange of the unique id succeeded), so on a
    one-GPU box every rank falls back to the file collective and the line says why
    (`rccl_error`); on a node with two devices the numbers go over RCCL."""
    r = _two_ranks("rccl")
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    m = d["multi_gpu"]
    if m["collective"] == "file":
        assert "Duplicate GPU" in m.get("rccl_error", "") or "ncclCommInitRank" in m.get("rccl_error", ""), m
        _check(r, "file")
    else:
        _check(r, "rccl")
