"""Data-parallel train step on the GPU: 2 ranks (gloo over CUDA tensors, both
on cuda:0 of the one-GPU box) run graph-replayed steps with their own
cameras; the flat gradient all-reduce keeps the parameters identical, and the
identically seeded density-grid jitter keeps the occupancy grids identical."""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "single-stable-dreamfusion_amd")]
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    import bench
    trainer, data = bench.make_trainer(64, 3, rank, world, True, graph=True)
    for i in range(20):
        trainer.train_iteration(data.collate([i]))
    torch.cuda.synchronize()
    m = trainer.model
    sums = torch.stack([p.detach().double().sum() for p in m.parameters()]
                       + [m.density_grid.double().sum(), m.density_bitfield.double().sum()])
    gathered = [torch.zeros_like(sums.cpu()) for _ in range(world)]
    dist.all_gather(gathered, sums.cpu())
    if rank == 0:
        out.put([g.tolist() for g in gathered])
    dist.destroy_process_group()


def test_two_rank_replicas_stay_identical(gpu):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = q.get(timeout=240)
        for p in procs:
            p.join(timeout=60)
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
                p.join(timeout=30)
    for p in procs:
        assert p.exitcode == 0
    a, b = res
    assert a == b  # bit-identical parameters, density grid and bitfield


def _worker_mean(rank, world, port, out):
    """Each rank's native step writes its own gradient bucket; after the
    exchange (flat_allreduce_, in place on the bucket) every rank holds
    exactly the mean of the per-rank buckets."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "single-stable-dreamfusion_amd")]
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    import bench
    from nerf.utils import _grad_bucket
    trainer, data = bench.make_trainer(64, 3, rank, world, True, graph=True)
    for i in range(4):
        trainer.train_iteration(data.collate([i]))
    params = [p for p in trainer.model.parameters() if p.requires_grad]
    pre = {}

    def hook(g):  # the replay's launches, eagerly, keeping the rank's own bucket
        g.step_timed()
        pre["bucket"] = _grad_bucket(params).clone()
    trainer.step_hook = hook
    trainer.train_iteration(data.collate([5]))
    trainer.step_hook = None
    torch.cuda.synchronize()
    g = next(iter(trainer._graphs.values()))
    reduced = _grad_bucket(params)
    mine = pre["bucket"].cpu()
    both = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(both, mine)
    want = (both[0] + both[1]) / world
    res = {"rank": rank, "eager_exchange": not g.optimizer_in_graph,
           "ranks_differ": not torch.equal(both[0], both[1]),
           "mean_equal": bool(torch.equal(reduced.cpu(), want)),
           "nonzero": bool(mine.abs().sum() > 0)}
    gathered = [None] * world
    dist.all_gather_object(gathered, res)
    if rank == 0:
        out.put(gathered)
    dist.destroy_process_group()


def test_two_rank_reduced_bucket_is_the_mean(gpu):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker_mean, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = q.get(timeout=240)
        for p in procs:
            p.join(timeout=60)
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
                p.join(timeout=30)
    for p in procs:
        assert p.exitcode == 0
    for r in res:
        assert r["eager_exchange"] and r["nonzero"] and r["ranks_differ"], r
        assert r["mean_equal"], r
