"""Independent streams, one per GPU (SURVEY.md §8e "replicas only"; BASELINE configs[3], C4).

A tfusion stream does not shard: frame k needs frame k-1's pose, TSDF and raycast, and every
ICP iteration needs the previous one.  N GPUs therefore run N independent streams (seed 7 +
rank), and the only communication is the end-of-run aggregation of the per-rank frame counter
and time that the north star asks for ("a RCCL all-reduce over xGMI of the per-rank
frames/sec counter only").  The reference itself is single-GPU (`apps/demo.cpp:151-152`,
`cuda::setDevice(0)`); nothing here has a reference counterpart.

Three pieces, all torch-free so that a GPU process loads exactly one HIP runtime
(/opt/rocm's, the one libtfusion_hip.so links):

* `launch(script, argv, n)` -- the parent of `python bench.py --gpus N`: starts N fresh child
  processes before anything touches a GPU, each with RANK / LOCAL_RANK / WORLD_SIZE set, and
  exits with the first non-zero child status.  Under torchrun (WORLD_SIZE already set) the
  script is a rank itself and no launcher runs.
* `FileGroup` -- a host-side all-gather through files in a rendezvous directory shared by the
  ranks of one node: `TFUSION_RDZV_DIR` (set by `launch`), or under torchrun a directory named
  after the parent agent process (its pid and start time, so a recycled pid cannot meet a stale
  directory).  It carries the RCCL unique id from rank 0 to the others, and is the whole
  collective of the CPU stand-in the tests drive.
* `RcclGroup` -- `/opt/rocm/lib/librccl.so` through ctypes on the product's own HIP runtime:
  `ncclCommInitRank` over the unique id, then `ncclAllReduce` (MAX / SUM, float64) and
  `ncclAllGather` on a small device buffer and a private stream; `ncclCommCount` is reported.
"""
import ctypes
import json
import os
import signal
import subprocess
import sys
import tempfile
import time

RCCL_PATH = "/opt/rocm/lib/librccl.so"
WAIT_S = float(os.environ.get("TFUSION_RDZV_TIMEOUT", "1200"))


def world_from_env():
    """(rank, local_rank, world) from the torchrun / launcher environment."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, local_rank, world


def _proc_start_time(pid):
    """Field 22 of /proc/<pid>/stat (start time in clock ticks since boot), or 0."""
    try:
        with open(f"/proc/{pid}/stat") as f:
            return int(f.read().rsplit(")", 1)[1].split()[19])
    except (OSError, IndexError, ValueError):
        return 0


def rdzv_dir():
    """The directory the ranks of this job share on this node."""
    d = os.environ.get("TFUSION_RDZV_DIR")
    if d:
        return d
    # torchrun: every worker is a child of the same elastic agent
    ppid = os.getppid()
    key = (f"tfusion_rdzv_{ppid}_{_proc_start_time(ppid)}_{os.environ.get('MASTER_PORT', '0')}_"
           f"{os.environ.get('TORCHELASTIC_RESTART_COUNT', '0')}")
    return os.path.join(tempfile.gettempdir(), key)


class FileGroup:
    """All-gather of small JSON values among `world` ranks through files in `path`.  Each call
    writes `<seq>.<rank>.json` (atomically: a temporary file, then rename) and waits, with a
    bounded poll, for the other ranks' files of the same sequence number."""

    def __init__(self, rank, world, path=None, timeout=WAIT_S):
        self.rank, self.world, self.timeout = rank, world, timeout
        self.path = path or rdzv_dir()
        os.makedirs(self.path, exist_ok=True)
        self.seq = 0

    def _name(self, seq, rank):
        return os.path.join(self.path, f"{seq}.{rank}.json")

    def publish(self, value, tag=None):
        seq = self.seq if tag is None else tag
        tmp = self._name(seq, self.rank) + f".tmp{os.getpid()}"
        with open(tmp, "w") as f:
            json.dump(value, f)
        os.replace(tmp, self._name(seq, self.rank))

    def read(self, rank, tag=None):
        """Wait for rank's value of this sequence number (or of `tag`) and return it."""
        seq = self.seq if tag is None else tag
        name = self._name(seq, rank)
        t0 = time.monotonic()
        delay = 1e-4
        while not os.path.exists(name):
            if time.monotonic() - t0 > self.timeout:
                raise TimeoutError(f"rank {self.rank}: rank {rank} never published {name} "
                                   f"({self.timeout:.0f} s)")
            time.sleep(delay)
            delay = min(delay * 2, 0.01)
        with open(name) as f:
            return json.load(f)

    def allgather(self, value):
        self.publish(value)
        out = [self.read(r) for r in range(self.world)]
        self.seq += 1
        return out

    def allreduce(self, values, op):
        vals = self.allgather([float(v) for v in values])
        red = max if op == "max" else sum
        return [red(v[i] for v in vals) for i in range(len(values))]

    def barrier(self):
        self.allgather(None)

    def close(self, remove=False):
        """remove: rank 0 deletes the directory once every rank has closed (torchrun jobs; the
        launcher removes its own directory after the children exit)."""
        self.publish(1, tag="closed")
        if remove and self.rank == 0:
            try:
                for r in range(self.world):
                    self.read(r, tag="closed")
                for n in os.listdir(self.path):
                    os.unlink(os.path.join(self.path, n))
                os.rmdir(self.path)
            except (OSError, TimeoutError):
                pass


# ---------------------------------------------------------------------------------------------
# RCCL over the product's HIP runtime

class _UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]           # NCCL_UNIQUE_ID_BYTES (rccl.h)


NCCL_SUM, NCCL_MAX = 0, 2                                    # ncclRedOp_t
NCCL_FLOAT64 = 8                                             # ncclDataType_t
HIP_H2D, HIP_D2H = 1, 2                                      # hipMemcpyKind


class RcclGroup:
    """One RCCL communicator of `world` ranks, rank `rank` on HIP device `device`.  The unique id
    goes from rank 0 to the others through `files` (a FileGroup).  Needs libtfusion_hip.so's HIP
    runtime loaded first (topfusion_amd._lib.load()) so librccl binds to the same one."""

    def __init__(self, rank, world, device, files):
        from topfusion_amd import _lib
        _lib.load()
        self.rank, self.world, self.device = rank, world, device
        self.hip = ctypes.CDLL("libamdhip64.so.7")              # already loaded: the same handle
        self.nccl = ctypes.CDLL(RCCL_PATH)
        n, h = self.nccl, self.hip
        P, I, S = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
        n.ncclGetUniqueId.argtypes = [ctypes.POINTER(_UniqueId)]
        n.ncclCommInitRank.argtypes = [ctypes.POINTER(P), I, _UniqueId, I]
        n.ncclAllReduce.argtypes = [P, P, S, I, I, P, P]
        n.ncclAllGather.argtypes = [P, P, S, I, P, P]
        n.ncclCommCount.argtypes = [P, ctypes.POINTER(I)]
        n.ncclCommDestroy.argtypes = [P]
        n.ncclGetErrorString.argtypes = [I]
        n.ncclGetErrorString.restype = ctypes.c_char_p
        for f in ("ncclGetUniqueId", "ncclCommInitRank", "ncclAllReduce", "ncclAllGather", "ncclCommCount",
                  "ncclCommDestroy"):
            getattr(n, f).restype = I
        h.hipSetDevice.argtypes = [I]
        h.hipMalloc.argtypes = [ctypes.POINTER(P), S]
        h.hipFree.argtypes = [P]
        h.hipMemcpy.argtypes = [P, P, S, I]
        h.hipStreamCreate.argtypes = [ctypes.POINTER(P)]
        h.hipStreamSynchronize.argtypes = [P]
        h.hipStreamDestroy.argtypes = [P]
        for f in ("hipSetDevice", "hipMalloc", "hipFree", "hipMemcpy", "hipStreamCreate", "hipStreamSynchronize",
                  "hipStreamDestroy"):
            getattr(h, f).restype = I
        self._hip(h.hipSetDevice(device), "hipSetDevice")
        uid = _UniqueId()
        if rank == 0:
            self._nccl(n.ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
            # (the raw 128 bytes: reading the c_char array field would stop at its first NUL)
            files.publish(ctypes.string_at(ctypes.addressof(uid), ctypes.sizeof(uid)).hex(), tag="rccl_uid")
        else:
            raw = bytes.fromhex(files.read(0, tag="rccl_uid"))
            assert len(raw) == ctypes.sizeof(uid)
            ctypes.memmove(ctypes.addressof(uid), raw, len(raw))
        self.comm = P()
        self._nccl(n.ncclCommInitRank(ctypes.byref(self.comm), world, uid, rank), "ncclCommInitRank")
        self.stream = P()
        self._hip(h.hipStreamCreate(ctypes.byref(self.stream)), "hipStreamCreate")
        self.cap = 64 * (world + 1)                              # float64 slots: send + gather buffers
        self.buf = P()
        self._hip(h.hipMalloc(ctypes.byref(self.buf), self.cap * 8), "hipMalloc")

    def _hip(self, rc, what):
        if rc != 0:
            raise RuntimeError(f"rank {self.rank}: {what} failed: hipError {rc}")

    def _nccl(self, rc, what):
        if rc != 0:
            raise RuntimeError(f"rank {self.rank}: {what} failed: {self.nccl.ncclGetErrorString(rc).decode()}")

    def nranks(self):
        c = ctypes.c_int()
        self._nccl(self.nccl.ncclCommCount(self.comm, ctypes.byref(c)), "ncclCommCount")
        return c.value

    def _put(self, values):
        a = (ctypes.c_double * len(values))(*[float(v) for v in values])
        self._hip(self.hip.hipMemcpy(self.buf, a, ctypes.sizeof(a), HIP_H2D), "hipMemcpy H2D")

    def _get(self, n, offset=0):
        a = (ctypes.c_double * n)()
        self._hip(self.hip.hipMemcpy(a, ctypes.c_void_p(self.buf.value + offset * 8), n * 8, HIP_D2H),
                  "hipMemcpy D2H")
        return list(a)

    def allreduce(self, values, op):
        """In-place float64 all-reduce (op "max" or "sum") of a few values."""
        n = len(values)
        assert 0 < n <= 64
        self._put(values)
        self._nccl(self.nccl.ncclAllReduce(self.buf, self.buf, n, NCCL_FLOAT64,
                                           NCCL_MAX if op == "max" else NCCL_SUM, self.comm, self.stream),
                   "ncclAllReduce")
        self._hip(self.hip.hipStreamSynchronize(self.stream), "hipStreamSynchronize")
        return self._get(n)

    def allgather(self, values):
        """float64 all-gather of `values` (the same length on every rank): a list per rank."""
        n = len(values)
        assert 0 < n <= 64
        self._put(values)
        recv = ctypes.c_void_p(self.buf.value + 64 * 8)
        self._nccl(self.nccl.ncclAllGather(self.buf, recv, n, NCCL_FLOAT64, self.comm, self.stream),
                   "ncclAllGather")
        self._hip(self.hip.hipStreamSynchronize(self.stream), "hipStreamSynchronize")
        flat = self._get(n * self.world, offset=64)
        return [flat[r * n:(r + 1) * n] for r in range(self.world)]

    def barrier(self):
        self.allreduce([0.0], "sum")

    def close(self):
        if getattr(self, "comm", None):
            self.hip.hipStreamSynchronize(self.stream)
            self.nccl.ncclCommDestroy(self.comm)
            self.hip.hipFree(self.buf)
            self.hip.hipStreamDestroy(self.stream)
            self.comm = None


def device_identity(device, standin=False):
    """(domain, bus, device, function) of HIP device `device` (hipDeviceGetPCIBusId on the product's
    runtime): what proves that the ranks of a job ran on distinct GPUs.  The CPU stand-in reports
    (-1, rank-free placeholder) -- the caller passes its rank as `device`."""
    if standin:
        return [-1, int(device), 0, 0]
    from topfusion_amd import _lib
    _lib.load()
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipDeviceGetPCIBusId.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
    hip.hipDeviceGetPCIBusId.restype = ctypes.c_int
    buf = ctypes.create_string_buffer(64)
    if hip.hipDeviceGetPCIBusId(buf, 64, int(device)) != 0:
        return [-2, int(device), 0, 0]
    return parse_bus_id(buf.value.decode())


def parse_bus_id(text):
    """"dddd:bb:dd.f" -> [domain, bus, device, function] (hex fields)."""
    dom, bus, rest = text.strip().split(":")
    dev, fn = rest.split(".")
    return [int(dom, 16), int(bus, 16), int(dev, 16), int(fn, 16)]


def format_bus_id(v):
    if v[0] < 0:
        return f"standin:{int(v[1])}" if v[0] == -1 else f"unknown:device{int(v[1])}"
    return f"{int(v[0]):04x}:{int(v[1]):02x}:{int(v[2]):02x}.{int(v[3]):x}"


class Replicas:
    """The collective a bench rank uses: RCCL for the numbers (`kind` "rccl"), the file group for
    the unique id; or the file group alone ("file": the CPU stand-in, or world 1).  If RCCL cannot
    be set up (a missing library, a communicator error) every rank falls back to the file group
    and the line says so (`collective` "file", `rccl_error`)."""

    def __init__(self, rank, local_rank, world, kind="rccl"):
        self.rank, self.local_rank, self.world = rank, local_rank, world
        self.files = FileGroup(rank, world) if world > 1 else None
        self.rccl = None
        self.rccl_error = None
        self.kind = kind if world > 1 else "none"
        if world > 1 and kind == "rccl":
            try:
                self.rccl = RcclGroup(rank, world, local_rank, self.files)
            except (OSError, RuntimeError) as e:
                self.rccl_error = f"rank {rank}: {e}"
            # every rank learns whether every rank has a communicator (over the file group, which
            # works either way); one failure sends all of them to the file group
            errs = self.files.allgather(self.rccl_error)
            bad = [e for e in errs if e]
            if bad:
                if self.rccl is not None:
                    self.rccl.close()
                    self.rccl = None
                self.kind = "file"
                self.rccl_error = bad[0]

    @property
    def group(self):
        return self.rccl or self.files

    def barrier(self):
        if self.world > 1:
            self.group.barrier()

    def nranks(self):
        return self.rccl.nranks() if self.rccl else self.world

    def combine(self, elapsed, frames):
        """Whole-job numbers: the slowest rank's time (MAX), the frames of all ranks (SUM), and
        every rank's own (time, frames) -- three collectives over RCCL (or the file group)."""
        if self.world <= 1:
            return float(elapsed), float(frames), [(float(elapsed), float(frames))]
        g = self.group
        emax = g.allreduce([elapsed], "max")[0]
        total = g.allreduce([frames], "sum")[0]
        per = [tuple(v) for v in g.allgather([float(elapsed), float(frames)])]
        return emax, total, per

    def summary(self, elapsed, frames, identity=None, extra=None):
        """The multi-GPU fields of the bench line (rank 0): world, the communicator's own rank
        count, per-rank frames/s and their spread, and -- so that an N-GPU line proves itself --
        each rank's device (PCI bus id, `identity` = device_identity()) and the per-rank numbers in
        `extra` (name -> number, the same names on every rank, e.g. frames_ok, icp_fallbacks).
        `distinct_devices` is false when two ranks report the same device.  The driver computes
        scaling efficiency itself from the per-N values, so none is reported here."""
        emax, total, per = self.combine(elapsed, frames)
        fps = [f / e if e > 0 else 0.0 for e, f in per]
        keys = sorted(extra or {})
        vec = [float(v) for v in (identity or [-2, self.local_rank, 0, 0])] + [float(extra[k]) for k in keys]
        rows = self.group.allgather(vec) if self.world > 1 else [vec]
        devs = [format_bus_id(r[:4]) for r in rows]
        out = {
            "world": self.world, "collective": self.kind,
            "collective_nranks": self.nranks(),
            "per_rank_frames_per_sec": [round(v, 2) for v in fps],
            "per_rank_elapsed_s": [float(f"{e:.6g}") for e, _ in per],   # (6 significant digits: short runs too)
            "per_rank_frames": [int(f) for _, f in per],
            "rank_spread": round(min(fps) / max(fps), 4) if fps and max(fps) > 0 else None,
            "per_rank_device": devs,
            "distinct_devices": len(set(devs)) == len(devs),
        }
        for i, k in enumerate(keys):
            out[f"per_rank_{k}"] = [int(r[4 + i]) if float(r[4 + i]).is_integer() else r[4 + i] for r in rows]
        if self.rccl_error:
            out["rccl_error"] = self.rccl_error
        return emax, total, out

    def close(self):
        if self.rccl is not None:
            self.rccl.close()
        if self.files is not None:
            self.files.close(remove="TFUSION_RDZV_DIR" not in os.environ)


# ---------------------------------------------------------------------------------------------
# launcher

def launch(script, argv, n, extra_env=None):
    """Run `python script argv` as n ranks (RANK = LOCAL_RANK = r, WORLD_SIZE = n) from this
    process, which touches no GPU.  Children share stdout / stderr (only rank 0 prints the
    line).  Returns the job's exit status: 0, or the first failing rank's (the others are then
    terminated, by the pids started here)."""
    rdzv = tempfile.mkdtemp(prefix="tfusion_rdzv_")
    procs = []
    try:
        for r in range(n):
            env = dict(os.environ)
            env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                       TFUSION_RDZV_DIR=rdzv, TFUSION_LAUNCHED="1")
            env.setdefault("MASTER_ADDR", "127.0.0.1")
            env.update(extra_env or {})
            procs.append(subprocess.Popen([sys.executable, "-u", script] + list(argv), env=env))
        status = 0
        live = list(procs)
        while live:
            for p in list(live):
                rc = p.poll()
                if rc is None:
                    continue
                live.remove(p)
                if rc != 0 and status == 0:
                    status = rc if rc > 0 else 128 - rc
                    sys.stderr.write(f"replicas: rank {procs.index(p)} exited with {rc}; stopping the others\n")
                    for q in live:
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.05)
        return status
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        for name in os.listdir(rdzv):
            try:
                os.unlink(os.path.join(rdzv, name))
            except OSError:
                pass
        try:
            os.rmdir(rdzv)
        except OSError:
            pass
