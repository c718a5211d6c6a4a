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
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    a, b = res
    assert a == b  # bit-identical parameters, density grid and bitfield
