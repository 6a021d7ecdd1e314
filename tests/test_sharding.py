"""Multi-rank forward sharding on CPU (gloo, world size 2): each rank runs the
oracle forward on its shard of a global batch; the gathered shards equal the
single-process forward, and the timing reduction is a true max / sum.
(The product kernels need a GPU; the shard arithmetic and reductions that
bench.py uses are what is under test here.)"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import sharding
import golden_util as gu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_shard_bounds_cover_exactly():
    for gb in [0, 1, 5, 256, 2048, 2049]:
        for world in [1, 2, 3, 8]:
            seen = []
            for r in range(world):
                lo, hi = sharding.shard_bounds(gb, world, r)
                assert 0 <= lo <= hi <= gb
                assert hi - lo in (gb // world, gb // world + 1)
                seen.extend(range(lo, hi))
            assert seen == list(range(gb))
    with pytest.raises(ValueError):
        sharding.shard_bounds(8, 2, 2)


def _case_inputs(case):
    """Weights (portable generator over our module tree) and images of a golden case."""
    import model as ours
    meta, arr = gu.load_case(case)
    torch.manual_seed(0)
    m = ours.MainModel.from_dict(**meta["config"])
    sd, x = gu.build_inputs(meta, m)
    return meta, arr, sd, x


def _worker(rank, world, port, case, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sdpnet_oracle as orc
        meta, _, sd, x = _case_inputs(case)
        nr = meta["num_registers"]
        local = sharding.sharded_forward(lambda xs: orc.forward(xs, sd, meta["config"], num_registers=nr), x)
        outs = [None] * world
        dist.all_gather_object(outs, local)
        tmax = sharding.max_over_ranks(float(rank + 1))
        tsum = sharding.sum_over_ranks(float(local.shape[0]))
        if rank == 0:
            q.put((torch.cat(outs).numpy(), tmax, tsum))
    finally:
        dist.destroy_process_group()


def test_two_rank_shards_match_single_process():
    case = "xxs_cf_b4"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, case, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        logits, tmax, tsum = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    import sdpnet_oracle as orc
    meta, arr, sd, x = _case_inputs(case)
    ref = orc.forward(x, sd, meta["config"], num_registers=meta["num_registers"]).numpy()
    assert logits.shape == ref.shape
    assert abs(logits - ref).max() < 1e-5
    assert abs(logits - arr["logits"]).max() < 1e-4   # and the reference's own logits
    assert tmax == 2.0 and tsum == float(ref.shape[0])


def test_bench_launcher_spawns_ranks():
    """bench.py --gpus 2 (outside torch.distributed.run) must start two ranks as a child
    torch.distributed.run and report n_gpus 2; --dry-run swaps the model for a trivial
    CPU step on gloo so the launch / barrier / max-over-ranks path runs here."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1"
    out = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--dry-run",
                          "--steps", "3", "--warmup", "1"], capture_output=True, text=True, env=env, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["comm_world"] == 2 and rec["backend"] == "gloo"
    assert rec["global_batch"] == 512
    assert len({r["pid"] for r in rec["ranks"]}) == 2
    assert [r["shard"] for r in rec["ranks"]] == [[0, 256], [256, 512]]
    # a rank whose WORLD_SIZE disagrees with --gpus refuses to run
    bad = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--dry-run"],
                         capture_output=True, text=True, env=dict(env, WORLD_SIZE="1"), timeout=120)
    assert bad.returncode != 0 and "WORLD_SIZE" in bad.stderr
