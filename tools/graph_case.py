"""Capture variants of GraphedTrainStep (debugging aid, one variant per process):
    python tools/graph_case.py {plain|eager_default|eager_capture_stream}"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "single-stable-dreamfusion_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402


def main(mode):
    import bench
    from nerf.graph import GraphedTrainStep
    trainer, data = bench.make_trainer(64, 7, 0, 1, True, graph=False)
    batch = data.collate([0])
    for _ in range(3):
        trainer.train_iteration(batch)
    model = trainer.model
    text_z = trainer.text_z[batch["dir"]]
    stream = torch.cuda.Stream()
    if mode != "plain":
        ctx = torch.cuda.stream(stream) if mode == "eager_capture_stream" else None
        if ctx:
            stream.wait_stream(torch.cuda.current_stream())
            ctx.__enter__()
        trainer.optimizer.zero_grad()
        model.device_count_march = True
        with torch.autocast("cuda", dtype=torch.float16):
            loss = trainer.train_step(batch, "albedo", 1.0, text_z)[2]
        trainer.backward_only(loss)
        del loss
        model.device_count_march = False
        if ctx:
            ctx.__exit__(None, None, None)
        torch.cuda.synchronize()
        print("eager ok", flush=True)
    g = GraphedTrainStep(trainer, batch, "albedo", 1.0, text_z, stream)
    g.capture()
    print("captured", flush=True)
    g.load(batch, text_z)
    g.replay()
    torch.cuda.synchronize()
    print(f"{mode} ok", flush=True)


if __name__ == "__main__":
    main(sys.argv[1])
