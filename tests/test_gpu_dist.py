"""bench.py's multi-GPU branch on a real GPU at world 1: launched by torch.distributed.run with
one rank, it creates the RCCL process group (backend "nccl"), all-reduces the verification
counters and the step time over RCCL, and runs hcdist.gather_encoded (hc_pack_batch on the GPU,
the RCCL all-gather of the encoded sizes) with --gather: the path the driver's N-GPU runs take,
minus the point-to-point sends that need a second GPU."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_world1_rccl(gpu):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--streams", "256", "--steps", "2", "--warmup", "1", "--gather", "--no-configs",
           "--no-cpu-baseline"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    r = json.loads(lines[0])
    assert r["process_group"] == {"backend": "nccl", "world": 1}
    assert r["bit_exact"] is True and r["value"] > 0 and r["n_gpus"] == 1
    g = r["gather"]
    assert g["rank0_spot_check"] is True and g["bytes_to_rank0"] > 0
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "world1_rccl.log"), "w") as f:
        f.write(lines[0] + "\n")
