"""The RCCL (torch.distributed "nccl") gradient exchange on the one GPU of the
box: a 1-rank process group initialised the way bench.py does it
(`init_process_group("nccl", device_id=...)`), a graph-replayed native train
step whose gradients are views of one flat bucket, and `flat_allreduce_`
(reference DDP all-reduce, nerf/utils.py:200-202) run in place on that bucket
through RCCL.  Run in a spawned process so the process group never leaks into
the rest of the session."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(port, out):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "single-stable-dreamfusion_amd")]
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    res = {"backend": dist.get_backend()}
    import bench
    from nerf.utils import _grad_bucket, flat_allreduce_
    trainer, data = bench.make_trainer(64, 3, 0, 1, True, graph=True)
    for i in range(4):
        trainer.train_iteration(data.collate([i]))
    torch.cuda.synchronize()
    params = [p for p in trainer.model.parameters() if p.requires_grad]
    bucket = _grad_bucket(params)
    res["bucket"] = bucket is not None
    if bucket is not None:
        before = bucket.clone()
        ptr = bucket.data_ptr()
        flat_allreduce_(params, 1)  # in place on the bucket, through RCCL
        torch.cuda.synchronize()
        res["in_place"] = _grad_bucket(params) is not None and bucket.data_ptr() == ptr
        res["unchanged"] = bool(torch.equal(before, bucket))
        res["numel"] = bucket.numel()
    x = torch.arange(1024, dtype=torch.float32, device=dev)
    dist.all_reduce(x)
    res["sum_ok"] = bool(torch.equal(x, torch.arange(1024, dtype=torch.float32, device=dev)))
    dist.destroy_process_group()
    out.put(res)


def test_rccl_flat_allreduce_in_place(gpu):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_port(), q))
    p.start()
    try:
        res = q.get(timeout=240)
        p.join(timeout=60)
    finally:
        if p.is_alive():  # hung or dead before reporting: never leave it on the GPU
            p.kill()
            p.join(timeout=30)
    assert p.exitcode == 0
    assert res["backend"] == "nccl"
    assert res["bucket"], "native step gradients are not views of one flat bucket"
    assert res["in_place"] and res["unchanged"]
    assert res["numel"] >= 903480 * 2  # grid table + MLPs, one bucket
    assert res["sum_ok"]


def _worker_in_graph(port, out):
    """The in-graph data-parallel step (RCCL all-reduce + 1/world + Adam
    captured in the native step graph) over a 1-rank nccl group against the
    plain one-GPU graph (no collective): same draws, so bit-identical."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "single-stable-dreamfusion_amd")]
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    import bench

    def run(in_graph):
        tr, dt = bench.make_trainer(64, 5, 0, 1, True, graph=True)
        tr.dp_in_graph = in_graph
        tr.opt.iters = 50  # a moving LR schedule (device learning rates)
        for i in range(20):
            tr.train_iteration(dt.collate([i % 4]))
        torch.cuda.synchronize()
        g = next(iter(tr._graphs.values()))
        return tr, g

    a, ga = run(None)  # auto: the nccl group is up -> collective in the graph
    b, gb = run(False)
    res = {"a_collective": ga.native is not None and ga.native.dp_world == 1,
           "a_opt": bool(ga.optimizer_in_graph),
           "b_plain": gb.native is not None and gb.native.dp_world is None
           and bool(gb.optimizer_in_graph),
           "params_equal": all(bool(torch.equal(pa, pb)) for pa, pb in
                               zip(a.model.parameters(), b.model.parameters())),
           "scale_equal": float(a.scaler.get_scale()) == float(b.scaler.get_scale()),
           "moved": not all(bool(torch.equal(p, q)) for p, q in
                            zip(a.model.parameters(), bench.make_trainer(
                                64, 5, 0, 1, True)[0].model.parameters()))}
    sa, sb = a.optimizer.state_dict()["state"], b.optimizer.state_dict()["state"]
    res["state_equal"] = all(bool(torch.equal(sa[i][k], sb[i][k])) for i in sa
                             for k in ("step", "exp_avg", "exp_avg_sq"))
    dist.destroy_process_group()
    out.put(res)


def test_rccl_all_reduce_captured_in_step_graph(gpu):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker_in_graph, args=(_port(), q))
    p.start()
    try:
        res = q.get(timeout=300)
        p.join(timeout=60)
    finally:
        if p.is_alive():
            p.kill()
            p.join(timeout=30)
    assert p.exitcode == 0
    assert res["a_collective"] and res["a_opt"], res
    assert res["b_plain"], res
    assert res["moved"], res
    assert res["params_equal"] and res["state_equal"] and res["scale_equal"], res


def _worker_two_gpus(rank, world, port, out):
    """One rank per GPU over RCCL, as bench.py --gpus N runs them: the
    in-graph data-parallel native step (all-reduce + 1/world + Adam captured
    in the step graph, replayed every step), per-rank cameras; afterwards
    every rank holds the same replica (bench.replica_check)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "single-stable-dreamfusion_amd")]
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(rank)
    dev = torch.device("cuda", rank)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    import bench
    tr, data = bench.make_trainer(64, 7, rank, world, True, graph=True)
    start = [p.detach().clone() for p in tr.model.parameters()]
    for i in range(12):
        tr.train_iteration(data.collate([i % 4]))
    torch.cuda.synchronize()
    g = next(iter(tr._graphs.values()))
    rows = [(tr.model.local_step - 1 - i) % 16 for i in range(8)]
    samples = float(tr.model.step_counter[rows, 0].float().mean().item())
    identical, per_rank = bench.replica_check(tr, samples, world)
    res = {"in_graph": g.native is not None and g.native.dp_world == world,
           "opt_in_graph": bool(g.optimizer_in_graph), "identical": identical,
           "per_rank": per_rank,
           "moved": not all(bool(torch.equal(a, b)) for a, b in
                            zip(start, tr.model.parameters()))}
    dist.destroy_process_group()
    if rank == 0:
        out.put(res)


def test_two_gpu_in_graph_nccl_step(gpu):
    """bench.py --gpus 2's exchange on two devices (skipped on a one-GPU box):
    every rank replays ONE graph per step holding the RCCL all-reduce, and the
    replicas stay bit-identical while the ranks render different cameras."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker_two_gpus, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = q.get(timeout=300)
        for p in procs:
            p.join(timeout=60)
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
                p.join(timeout=30)
    assert all(p.exitcode == 0 for p in procs)
    assert res["in_graph"] and res["opt_in_graph"], res
    assert res["moved"] and res["identical"], res
    assert len(res["per_rank"]) == 2 and res["per_rank"][0] != res["per_rank"][1], res
