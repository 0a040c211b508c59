"""bench.py's multi-rank path, run before the driver's 8-GPU run depends on it: two ranks
launched exactly as the driver launches N > 1 (torch.distributed.run, 127.0.0.1 rendezvous),
sharing the test box's one GPU through the gloo diagnostic leg (--comm gloo).  Bootstrap,
the parameter broadcast, per-rank seeds, the barriers around the timed region, the
max-over-ranks time and teardown all execute; rank 0 prints exactly one JSON line.  The
timing is meaningless (gradients cross the host); the reference's counterpart is
MirroredStrategy, old_codes/BayConvT(Par)(Muti).py:16-19."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
def test_bench_two_ranks_gloo_leg():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--comm", "gloo", "--steps", "2", "--warmup", "1", "--batch", "8",
           "--no-evidence", "--no-cpu-baseline", "--no-secondary"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 16 and out["value"] > 0
    assert out["config"]["parallelism"] == "dp2" and out["scaling"] == "weak"
    assert set(out["phases_ms"]) == {"forward", "backward", "allreduce_wait", "optimizer"}
