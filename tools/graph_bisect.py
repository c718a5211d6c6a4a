"""Which part of the train step breaks HIP-graph capture?
    python tools/graph_bisect.py STAGE     (one stage per process)
Stages: march, field, render, sds, backward."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "single-stable-dreamfusion_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402


def main(stage):
    import bench
    import raymarching
    from nerf import field as _field
    trainer, data = bench.make_trainer(64, 0, 0, 1, True, graph=False)
    batch = data.collate([0])
    for _ in range(2):
        trainer.train_iteration(batch)
    model = trainer.model
    text_z = trainer.text_z[batch["dir"]]
    rays_o = batch["rays_o"].clone()
    rays_d = batch["rays_d"].clone()
    model.device_count_march = True
    trainer.optimizer.zero_grad(set_to_none=True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    # warm-up of the exact captured code on the capture stream
    g = torch.cuda.CUDAGraph()

    def body():
        if stage == "march":
            nears, fars = raymarching.near_far_from_aabb(rays_o[0], rays_d[0], model.aabb_train)
            return raymarching.march_rays_train_dev(rays_o[0], rays_d[0], 1.0,
                                                    model.density_bitfield, 1, 128, nears, fars,
                                                    model.step_counter[0], True, 0, 512)
        if stage in ("field", "render"):
            with torch.autocast("cuda", dtype=torch.float16):
                nears, fars = raymarching.near_far_from_aabb(rays_o[0], rays_d[0],
                                                             model.aabb_train)
                x, d, dl, r = raymarching.march_rays_train_dev(
                    rays_o[0], rays_d[0], 1.0, model.density_bitfield, 1, 128, nears, fars,
                    model.step_counter[0], True, 0, 512)
                sig, rgb, _ = model(x, d)
                if stage == "field":
                    return sig
                return raymarching.composite_rays_train(sig, rgb, dl, r, 1e-4)
        with torch.autocast("cuda", dtype=torch.float16):
            _, _, loss = trainer.train_step({"H": 64, "W": 64, "rays_o": rays_o,
                                             "rays_d": rays_d, "dir": None},
                                            "albedo", 1.0, text_z)
        if stage == "backward":
            trainer.backward_only(loss)
        return loss

    with torch.cuda.stream(s):
        body()
        if stage == "backward":
            trainer.optimizer.zero_grad(set_to_none=True)
    torch.cuda.synchronize()
    print("warm-up ok", flush=True)
    with _field.defer_embedding_backward():
        with torch.cuda.graph(g, stream=s):
            out = body()
    print("captured", flush=True)
    g.replay()
    torch.cuda.synchronize()
    print(f"stage {stage} ok", flush=True)


if __name__ == "__main__":
    main(sys.argv[1])
