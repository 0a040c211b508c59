"""Data-parallel gradient reduction on CPU with the gloo backend (world_size 2).

Covers vitmi.dp.GradReducer: buckets over the flat gradient buffer are launched only when
their whole range is inside the finished prefix (backward order), every bucket is reduced
exactly once, and the result is the mean over ranks — the semantics of the reference's
MirroredStrategy cross-replica reduction (old_codes/BayConvT(Par)(Muti).py:16-19)."""
import os
import sys
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from vitmi import dp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
from vitmi.config import ViTConfig


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = {}
        # 1) raw reducer: 10 buckets of 1 KiB (256 floats) over a 2500-element buffer
        n = 2500
        flat = torch.arange(n, dtype=torch.float32) * (rank + 1)
        red = dp.GradReducer(flat, bucket_mb=256 * 4 / (1 << 20))
        red.start()
        red.mark_ready(700)              # only buckets ending <= 700 may launch
        out["early"] = [b for _, b in red.launch_log]
        red.mark_ready(2500)
        red.finish()
        out["flat"] = flat.clone().numpy()
        out["nbuckets"] = len(red.bounds)
        out["launched"] = sorted(b for _, b in red.launch_log)
        # 2) attached to a (CPU-resident) model arena, hooks fired in backward order
        from vitmi.modules import VisionTransformer
        torch.manual_seed(0)
        m = VisionTransformer(ViTConfig(img_size=32, patch_size=8, embed_dim=128, depth=3, num_heads=2,
                                        dtype="fp32"))
        r2 = dp.attach(m, bucket_mb=0.1)
        arena = m.arena()
        arena.grad.copy_(torch.full_like(arena.grad, float(rank + 1)))
        r2.start()
        # AccumulateGrad's post hooks, in backward (= arena) order; one parameter's gradient
        # arrives in a tensor of its own and must be copied into its arena view
        stray = arena.params[3]
        for p in arena.params:
            if p is stray:
                p.grad = torch.full_like(p, float(rank + 1))
            for h in list(p._post_accumulate_grad_hooks.values()):
                h(p)
        out["stray_bound"] = stray.grad.data_ptr() == arena.view(arena.grad, stray).data_ptr()
        r2.finish()
        out["arena_mean"] = arena.grad.clone().numpy()
        out["arena_order"] = [b for _, b in r2.launch_log]
        dp.broadcast_parameters(m)
        out["param0"] = arena.flat[:8].clone().numpy()
        # 3) a model without an arena (the CvT regressor's path in train.fit): parameters and
        #    buffers broadcast from rank 0, then the packed gradients averaged; a parameter
        #    with no gradient on this rank counts as zero
        torch.manual_seed(10 + rank)
        lin = torch.nn.Sequential(torch.nn.Linear(7, 5), torch.nn.BatchNorm1d(5), torch.nn.Linear(5, 3))
        lin[1].running_mean.fill_(float(rank + 1))
        dp.broadcast_module(lin)
        out["lin_w"] = lin[0].weight.detach().clone().numpy()
        out["bn_mean"] = lin[1].running_mean.clone().numpy()
        pr = dp.ParamGradReducer(list(lin.parameters()), bucket_mb=64 * 4 / (1 << 20))
        for i, p in enumerate(lin.parameters()):
            if not (rank == 1 and i == 0):
                p.grad = torch.full_like(p, float(rank + 1) * (i + 1))
        pr.start()
        pr.finish()
        out["lin_grads"] = [p.grad.clone().numpy() for p in lin.parameters()]
        out["lin_buckets"] = len(pr.red.bounds)
        # 4) the RCCL id of the vitmi communicator travels through the job's TCPStore
        out["uid"] = dp.exchange_unique_id(rank, world)
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def _fallback_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # no GPU here: the library's RCCL communicator cannot be created (rank 0 fails to make the
        # id and says so through the store, so rank 1 fails instead of waiting); both ranks agree
        # on the fallback group and the exchange runs there
        comm, group, err = dp.comm_or_fallback(rank, world, make_group=lambda: dist.new_group(backend="gloo"))
        flat = torch.full((1000,), float(rank + 1))
        red = dp.GradReducer(flat, bucket_mb=1000 * 4 / (1 << 20) / 3, group=group)
        red.start()
        red.mark_ready(1000)
        red.finish()
        q.put((rank, {"comm": comm is None, "group": group is not None, "err": err is not None,
                      "mean": float(flat.mean()), "report": dp.comm_report(red)["backend"]}))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_comm_or_fallback_agrees_across_ranks():
    """bench.py's multi-GPU exchange: when the library's RCCL communicator cannot be created, every
    rank falls back to the same torch.distributed group (decided together) and the average still
    comes out right; the report names the backend that ran."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_fallback_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=100) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for r in range(world):
        o = res[r]
        assert o["comm"] and o["group"] and o["err"], o
        assert o["mean"] == 1.5 and o["report"] == "torch.distributed gloo", o


@pytest.mark.timeout(180)
def test_grad_reducer_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=150) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    n = 2500
    expect = torch.arange(n, dtype=torch.float32) * 1.5        # mean of 1x and 2x
    for r in range(world):
        o = {k: torch.from_numpy(v) if hasattr(v, "dtype") else v for k, v in res[r].items()}
        assert torch.allclose(o["flat"], expect)
        # 1 KiB buckets = 256 elements: only buckets [0,256) and [256,512) end <= 700
        assert o["early"] == [0, 1]
        assert o["launched"] == list(range(o["nbuckets"]))
        assert torch.allclose(o["arena_mean"], torch.full_like(o["arena_mean"], 1.5))
        assert o["arena_order"] == sorted(o["arena_order"])    # front-to-back readiness
        assert res[r]["stray_bound"]
        assert (res[r]["param0"] == res[0]["param0"]).all()     # broadcast from rank 0
        assert (res[r]["lin_w"] == res[0]["lin_w"]).all() and (res[r]["bn_mean"] == 1.0).all()
        assert res[r]["lin_buckets"] > 1
        for i, g in enumerate(res[r]["lin_grads"]):
            # rank 0 holds 1*(i+1), rank 1 holds 2*(i+1) (or nothing for parameter 0)
            want = (i + 1) * (0.5 if i == 0 else 1.5)
            assert torch.allclose(torch.from_numpy(g), torch.full(g.shape, want)), i
        assert len(res[r]["uid"]) == dp.UID_BYTES and res[r]["uid"] == res[0]["uid"]


# ------------------------------------------------------------------ abort on timeout
class _Ev:
    def __init__(self, done):
        self.done = done

    def query(self):
        return self.done


def test_watchdog_aborts_a_hung_exchange_and_raises():
    """CommWatchdog: a step's completion event that never fires makes the watchdog call the
    abort (ncclCommAbort through vitmi_comm_destroy(1) in GradReducer.abort) and the training
    thread's next check raises instead of hanging."""
    import time

    from vitmi.dp import CommWatchdog
    aborted = []
    wd = CommWatchdog(0.2, lambda: aborted.append(True), poll_s=0.01)
    try:
        wd.watch(_Ev(True))                  # finished steps are retired
        wd.check()
        wd.watch(_Ev(False))                 # a hung exchange
        t0 = time.monotonic()
        while not aborted and time.monotonic() - t0 < 5:
            time.sleep(0.02)
        assert aborted == [True]
        import pytest
        with pytest.raises(RuntimeError, match="aborted"):
            wd.check()
    finally:
        wd.close()


def test_watchdog_quiet_when_exchanges_finish():
    import time

    from vitmi.dp import CommWatchdog
    aborted = []
    wd = CommWatchdog(0.1, lambda: aborted.append(True), poll_s=0.01)
    try:
        for _ in range(5):
            wd.watch(_Ev(True))
        time.sleep(0.3)
        wd.check()
        assert not aborted
    finally:
        wd.close()


def test_comm_binds_the_rccl_torch_loaded():
    """The library's RCCL leg binds the librccl.so torch already mapped (dladdr of the bound
    ncclAllReduce), so a process holds one RCCL instance (csrc/comm.cpp load_rccl)."""
    import torch  # noqa: F401  (torch maps its RCCL at import)

    from vitmi.dp import VitmiComm
    mapped = sorted({ln.split()[-1] for ln in open("/proc/self/maps") if "librccl" in ln})
    assert mapped, "torch did not map an RCCL"
    bound = VitmiComm.library()
    assert os.path.realpath(bound) in {os.path.realpath(m) for m in mapped}, (bound, mapped)


# ------------------------------------------------------------------ the N>1 bench line's fields
class _FakeComm(dp.VitmiComm):
    """The vitmi communicator's interface with the exchange done by gloo on the host: the RCCL
    id still travels through the job's TCPStore (VitmiComm.from_store), only ncclCommInitRank
    and ncclAllReduce are replaced."""

    def _init(self, rank, world):
        self.calls = 0

    def allreduce_async(self, buf, side, ready=None, op=dp.REDUCE_AVG):
        self.calls += 1
        dist.all_reduce(buf)
        if op == dp.REDUCE_AVG:
            buf.div_(self.world)

    def info(self):
        return self.rank, self.world

    def check(self):
        pass

    @staticmethod
    def library():
        return "fake-rccl"


def _report_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from vitmi.modules import VisionTransformer
        out = {}
        comm = _FakeComm.from_store(rank, world)
        out["uid"] = comm._uid.raw
        torch.manual_seed(0)
        m = VisionTransformer(ViTConfig(img_size=32, patch_size=8, embed_dim=128, depth=4, num_heads=2,
                                        dtype="fp32"))
        red = dp.attach(m, bucket_mb=0.3, comm=comm, timeout_s=0)
        arena = m.arena()
        for step in range(2):
            arena.grad.fill_(float(rank + 1))
            red.start()
            for p in arena.params:              # AccumulateGrad's post hooks, backward order
                for h in list(p._post_accumulate_grad_hooks.values()):
                    h(p)
            in_backward = comm.calls
            red.finish()
        out["mean_ok"] = bool(torch.allclose(arena.grad, torch.full_like(arena.grad, 1.5)))
        out["in_backward"] = in_backward
        out["report"] = dp.comm_report(red)
        out["same"] = dp.replica_report(arena.flat)
        if rank == 1:
            with torch.no_grad():
                arena.flat[7] += 1e-3
        out["diff"] = dp.replica_report(arena.flat)
        cuts = red.bounds
        out["ends"] = [e for _, e in cuts]
        out["block_ends"] = sorted(max(arena.offsets[id(p)] + p.numel() for p in blk.parameters()) for blk in m.blocks)
        out["numel"] = arena.numel
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_multirank_report_fields_gloo_world2():
    """What bench.py adds to its line at N > 1 (dp.comm_report / dp.replica_report), driven
    through GradReducer, the parameters' post-accumulate hooks and VitmiComm.from_store's id
    exchange with a fake communicator: ranks and library as the communicator reports them, the
    block-aligned bucket plan with the tail that finish() launches, and a replica check that
    passes on identical parameters and fails when one rank's parameters differ."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_report_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=150) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert res[0]["uid"] == res[1]["uid"]
    for r in range(world):
        o = res[r]
        rep = o["report"]
        assert o["mean_ok"]
        assert rep["ranks"] == 2 and rep["rank"] == r and rep["library"] == "fake-rccl"
        assert rep["bucket_count"] == len(rep["buckets_mib"]) > 2
        assert rep["tail_buckets"] == [rep["bucket_count"] - 1]      # only the embedding's bucket
        assert rep["tail_bucket_mib"] == rep["buckets_mib"][-1]
        assert o["in_backward"] >= rep["bucket_count"] - 1           # the rest launched from hooks
        assert set(o["block_ends"]) <= set(o["ends"]) and o["ends"][-1] == o["numel"]
        assert o["same"]["replicas_identical"] is True
        assert o["diff"]["replicas_identical"] is False
    assert res[0]["same"]["param_checksum_bits"] == res[1]["same"]["param_checksum_bits"]


_ABORT_CHILD = r"""
import ctypes, os, sys, threading, time
sys.path[:0] = [os.environ["VITMI_PKG"]]
import torch
from vitmi import dp
from vitmi._lib import check

class Never:                      # a HIP event whose all-reduce never completes (a dead peer)
    def query(self):
        return False

comm = dp.VitmiComm(0, 2, bytes(dp.UID_BYTES))   # the stub's ncclCommInitRank
assert dp.VitmiComm.library().endswith("stub_rccl.so"), dp.VitmiComm.library()
red = dp.GradReducer(torch.zeros(256), bucket_mb=0.001, comm=comm, timeout_s=0.3)
red._prev_reserve = 7             # a CU reservation in force (training-thread global)
res = {}

def enqueue():                    # VitmiComm.allreduce_async's library call (host buffer: the stub
    buf = red.flat                # never touches it; the product path asserts a device buffer)
    check(comm._call("vitmi_comm_allreduce_async", buf.data_ptr(), buf.numel(), 0, dp.REDUCE_AVG, None, None),
          "comm_allreduce_async")

def train():                      # the training thread: enqueue blocks inside ncclAllReduce
    try:
        enqueue()
        res["rc"] = "returned"
    except RuntimeError as e:
        res["rc"] = str(e)

t = threading.Thread(target=train, daemon=True)
t0 = time.monotonic()
t.start()
time.sleep(0.1)
red.watchdog.watch(Never())       # what finish() hands the watchdog
t.join(timeout=5)
dt = time.monotonic() - t0
assert not t.is_alive(), "the blocked enqueue was not released by the watchdog's abort"
assert red.watchdog.error and "aborted" in red.watchdog.error, red.watchdog.error
assert "ncclAllReduce" in res["rc"] and "aborted" in res["rc"], res
assert not comm.live and red._prev_reserve == 7
try:
    enqueue()
    raise AssertionError("an all-reduce after the abort must fail")
except RuntimeError as e:
    assert "no communicator" in str(e), e
red.close()
print("ok", round(dt, 3))
"""


def _build_stub(tmp_path):
    import subprocess
    so = tmp_path / "stub_rccl.so"
    subprocess.run(["gcc", "-shared", "-fPIC", "-O1", "-o", str(so), os.path.join(ROOT, "tests", "stub", "stub_rccl.c"),
                    "-lpthread", "-ldl"], check=True)
    return so


@pytest.mark.parametrize("blocking", [False, True], ids=["nonblocking", "blocking"])
def test_watchdog_abort_releases_a_blocked_allreduce(tmp_path, blocking):
    """the watchdog's abort must not wait behind an all-reduce that never
    completes (a peer gone), it must release it, and it must never free the communicator under a
    call in flight.  A stub librccl.so (tests/stub/stub_rccl.c, loaded through VITMI_RCCL_LIB) never
    completes ncclAllReduce until ncclCommAbort.  Non-blocking (the library's default: its config
    init) the enqueue returns ncclInProgress and the library polls; the stub's abort FREES and poisons
    the communicator, so a library call that touched the handle after the abort would fail the check.
    Blocking (the stub refuses the config: the fallback init) the enqueue blocks inside RCCL.  Either
    way the training thread's call returns an error within the watchdog's timeout, the CU reservation
    stays with the training thread, and later calls fail cleanly."""
    import subprocess
    so = _build_stub(tmp_path)
    env = dict(os.environ, VITMI_RCCL_LIB=str(so), VITMI_PKG=os.path.join(ROOT, "transformer-stm_amd"))
    if blocking:
        env["STUB_RCCL_NO_CONFIG"] = "1"
    r = subprocess.run([sys.executable, "-c", _ABORT_CHILD], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout + r.stderr
    assert float(r.stdout.split()[1]) < 3.0


_SHM_CHILD = r"""
import os, sys
sys.path[:0] = [os.environ["VITMI_PKG"]]
import torch
import torch.distributed as dist
from vitmi import dp
from vitmi._lib import check
rank, world = int(sys.argv[1]), 2
dist.init_process_group("gloo", init_method="tcp://127.0.0.1:" + sys.argv[2], rank=rank, world_size=world)
comm = dp.VitmiComm.from_store(rank, world)          # vitmi_comm_init(world = 2) over the stub
assert comm.info() == (rank, world), comm.info()
def call(name, t, *a):
    check(comm._call(name, t.data_ptr(), t.numel(), *a), name)
x = torch.arange(3 * (1 << 20) + 5, dtype=torch.float32) * (rank + 1)       # > one 8 MiB stub slot
call("vitmi_comm_allreduce_async", x, 0, dp.REDUCE_AVG, None, None)
want = torch.arange(x.numel(), dtype=torch.float32) * 1.5
assert torch.equal(x, want), (x[:4], want[:4])
b = torch.full((1000,), float(rank), dtype=torch.bfloat16)
call("vitmi_comm_allreduce_async", b, 1, dp.REDUCE_SUM, None, None)
assert torch.equal(b, torch.full((1000,), 1.0, dtype=torch.bfloat16))
p = torch.randn(777, generator=torch.Generator().manual_seed(rank))
p0 = torch.randn(777, generator=torch.Generator().manual_seed(0))
call("vitmi_comm_broadcast", p, 0, 0, None)
assert torch.equal(p, p0)
comm.check()
comm.destroy()
dist.destroy_process_group()
print("ok", rank)
"""


def test_library_comm_world2_over_functional_stub(tmp_path):
    """The library's own communicator at world 2 (vitmi_comm_init, the non-blocking init poll, the
    enqueue under the comm lock, ncclAvg / ncclSum in fp32 and bf16, broadcast, destroy) between two
    real processes: the stub's shm mode reduces through POSIX shared memory (host buffers here,
    STUB_RCCL_HOST=1; tests/test_gpu_dp.py runs the same stub on device buffers)."""
    import subprocess
    so = _build_stub(tmp_path)
    env = dict(os.environ, VITMI_RCCL_LIB=str(so), VITMI_PKG=os.path.join(ROOT, "transformer-stm_amd"),
               STUB_RCCL_MODE="shm", STUB_RCCL_HOST="1")
    port = str(_free_port())
    procs = [subprocess.Popen([sys.executable, "-c", _SHM_CHILD, str(r), port], env=env, stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True) for r in range(2)]
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=120)[0])
        except subprocess.TimeoutExpired:
            p.kill()
            outs.append(p.communicate()[0])
    for r, (p, o) in enumerate(zip(procs, outs)):
        assert p.returncode == 0 and f"ok {r}" in o, o


def test_reducer_notifies_finished_buckets_in_order_at_world1():
    """GradReducer.listeners (optim.Adam.overlap_with): with nothing to exchange (world 1) every
    bucket is announced once, in order, as soon as the finished prefix covers it; the rest at
    the next step again from the first bucket."""
    flat = torch.zeros(1000)
    red = dp.GradReducer(flat, bucket_mb=256 * 4 / (1 << 20), cuts=[100, 600, 1000])
    assert not red._active
    seen = []
    red.listeners.append(lambda s, e, st: seen.append((s, e, st)))
    for _ in range(2):
        seen.clear()
        red.start()
        red.mark_ready(50)
        assert seen == []
        red.mark_ready(100)
        assert seen == [(0, 100, None)]
        red.mark_ready(700)
        assert [x[:2] for x in seen] == [(0, 100), (100, 356), (356, 600)]
        red.mark_ready(1000)
        red.finish()
        assert [x[:2] for x in seen] == red.bounds
        assert red.bounds[-1][1] == 1000
