"""Multi-process path on CPU (gloo, world size 2): stream sharding, counter reduction, size
all-gather and the payload gather into rank 0 reproduce the single-process result exactly.
The encoder here is the oracle (CPU checker) standing in for each rank's GPU encode — the
point is the distributed bookkeeping, which is device-independent."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

W, H, PER_RANK = 48, 40, 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _encode_shard(rank, world):
    import oracle
    import hcdist
    blobs = []
    for k in hcdist.shard(rank, world, PER_RANK):
        st, out = oracle.compress(oracle.synth("photo", k, W, H).tobytes(), True, False, 512)
        assert st == 0
        blobs.append(out)
    cap = max(len(b) for b in blobs) + 16
    buf = torch.zeros(PER_RANK * cap, dtype=torch.uint8)
    for i, b in enumerate(blobs):
        buf[i * cap:i * cap + len(b)] = torch.frombuffer(bytearray(b), dtype=torch.uint8)
    offs = torch.arange(PER_RANK, dtype=torch.int64) * cap
    lens = torch.tensor([len(b) for b in blobs], dtype=torch.int64)
    return buf, offs, lens


def _worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    sys.path[:0] = [os.path.join(root, "huffman-codec_amd", "python"), os.path.join(root, "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import hcdist
    buf, offs, lens = _encode_shard(rank, world)
    total = hcdist.reduce_counters([int(lens.sum()), rank + 1])
    mx = hcdist.reduce_counters([float(rank)], op="max")
    own = hcdist.pack(buf, offs, lens)
    packed, sizes = hcdist.gather_encoded(buf, offs, lens)
    q.put((rank, total.tolist(), mx.tolist(), sizes.tolist(), None if packed is None else packed.numpy().tobytes(),
           own.numel()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_multi_rank_gather_matches_single_process(oracle_mod, world):
    """rank 0 receives every rank's shard (point to point, in stream order); the other ranks
    receive nothing and hold only their own packed shard (no padding to the largest rank)"""
    import hcdist
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=120)
        res[r[0]] = r
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single-process reference of the same 6 streams
    want = []
    for k in range(world * PER_RANK):
        want.append(oracle_mod.compress(oracle_mod.synth("photo", k, W, H).tobytes(), True, False, 512)[1])
    for r in range(world):
        assert res[r][1] == [sum(map(len, want)), world * (world + 1) // 2]
        assert res[r][2] == [float(world - 1)]
        assert res[r][3] == [len(b) for b in want]
        assert res[r][5] == sum(len(b) for b in want[r * PER_RANK:(r + 1) * PER_RANK])
        if r:
            assert res[r][4] is None
    assert res[0][4] == b"".join(want)
    assert list(hcdist.shard(1, 2, 3)) == [3, 4, 5]


def test_pack_single_process():
    import hcdist
    buf = torch.arange(40, dtype=torch.int64).to(torch.uint8)
    offs = torch.tensor([0, 10, 30])
    lens = torch.tensor([3, 0, 5])
    assert hcdist.pack(buf, offs, lens).tolist() == [0, 1, 2, 30, 31, 32, 33, 34]


def _check_dry_line(stdout, world, S, per, weak, N, weak_per):
    import hashlib
    import json
    import sys
    lines = [l for l in stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, stdout
    r = json.loads(lines[0])
    assert r["dry_run"] is True and r["n_gpus"] == world and r["steps"] == 3 and r["warmup"] == 1
    # the launcher's process group exists at world 1 too (the RCCL path on a one-GPU box)
    assert r["process_group"] == {"backend": "gloo", "world": world}
    assert r["config"]["streams_total"] == S and r["config"]["streams_per_gpu"] == per
    assert r["value"] > 0 and r["ms_per_step"] > 0 and r["scaling"] == ("weak" if weak else "strong")
    assert r["bits_per_byte"] == 8.0  # the stand-in copies: encoded = raw bytes
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    sys.path.insert(0, root)
    import bench
    want = torch.cat([bench.stand_in_stream(torch, k, N) for k in range(S)]).numpy().tobytes()
    g = r["gather"]
    assert g["bytes_to_rank0"] == S * N and g["rank0_spot_check"] is True
    assert g["packed_sha256"] == hashlib.sha256(want).hexdigest()
    if world > 1:  # the weak-scaling figure rides beside value, never as it (dry run: --streams per rank)
        w = r["weak_scaling"]
        assert w["scaling"] == "weak" and w["bit_exact"] is True and w["value"] > 0
        assert w["streams_per_gpu"] == weak_per and w["streams_total"] == world * weak_per
    else:
        assert "weak_scaling" not in r
    return r


@pytest.mark.parametrize("world,weak", [(1, False), (2, False), (3, False), (2, True)])
def test_bench_multi_rank_dry_run(world, weak):
    """bench.py's own multi-rank path (shards, barriers, max-over-ranks timing, counter reduction,
    --gather) end to end under the driver's launcher, on CPU: --backend gloo swaps each rank's GPU
    step for a stand-in that copies its streams. Rank 0 prints exactly one JSON line; the gathered
    payload is every rank's shard in global stream order. The headline splits --streams over the
    ranks (strong scaling, C5 as BASELINE defines it); --weak makes it a per-GPU count."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    N = 3000
    S = 2 * world
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
           "--backend", "gloo", "--gpus", str(world), "--steps", "3", "--warmup", "1",
           "--gather", "--dry-stream-bytes", str(N)] + (["--weak", "--streams", "2"] if weak else ["--total-streams", str(S)])
    env = dict(os.environ, OMP_NUM_THREADS="1")
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=root)
    assert p.returncode == 0, p.stderr[-3000:]
    _check_dry_line(p.stdout, world, S, 2, weak, N, 2 if weak else S)


def test_bench_gpus_flag_launches_its_own_ranks():
    """`python bench.py --gpus 2` with NO launcher around it (the form of the driver's bench
    command) starts its two ranks itself: one JSON line with n_gpus 2 from a world-2 process group,
    C5-style split of --total-streams over the ranks"""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    N, S = 2000, 6
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE",
                                                              "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--backend", "gloo", "--gpus", "2", "--steps", "3",
           "--warmup", "1", "--gather", "--dry-stream-bytes", str(N), "--total-streams", str(S)]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=root)
    assert p.returncode == 0, p.stderr[-3000:]
    r = _check_dry_line(p.stdout, 2, S, S // 2, False, N, S)
    assert r["n_gpus"] == 2 and r["process_group"]["world"] == 2


def test_bench_gpus_flag_mismatch_exits_nonzero():
    """under a launcher, --gpus must equal WORLD_SIZE: a mismatch measures nothing and exits
    non-zero (before any process group or device is touched)"""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--backend", "gloo", "--gpus", "3"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=root)
    assert p.returncode != 0
    assert "--gpus 3" in p.stderr and not [l for l in p.stdout.splitlines() if l.startswith("{")]
