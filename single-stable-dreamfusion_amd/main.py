"""Command line of the SDS trainer (mirror of reference main.py:12-162, grid
backbone).  Flag names and defaults are the reference's, because the whole
`opt` namespace is forwarded as renderer kwargs (utils.py:363)."""
import argparse
import os
import sys

import numpy as np
import torch


def get_parser():
    p = argparse.ArgumentParser()
    p.add_argument("--text", default=None, help="text prompt")
    p.add_argument("--negative", default="", type=str, help="negative text prompt")
    p.add_argument("-O", action="store_true", help="equals --fp16 --cuda_ray --dir_text")
    p.add_argument("-O2", action="store_true", help="equals --fp16 --dir_text")
    p.add_argument("--test", action="store_true", help="test mode")
    p.add_argument("--save_mesh", action="store_true")
    p.add_argument("--eval_interval", type=int, default=10)
    p.add_argument("--workspace", type=str, default="workspace")
    p.add_argument("--guidance", type=str, default="stable-diffusion",
                   help="stable-diffusion (local weights via DFHIP_SD_PATH) or synthetic")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--iters", type=int, default=10000)
    p.add_argument("--lr", type=float, default=1e-3)
    p.add_argument("--ckpt", type=str, default="latest")
    p.add_argument("--cuda_ray", action="store_true")
    p.add_argument("--max_steps", type=int, default=512)
    p.add_argument("--num_steps", type=int, default=64)
    p.add_argument("--upsample_steps", type=int, default=64)
    p.add_argument("--update_extra_interval", type=int, default=16)
    p.add_argument("--max_ray_batch", type=int, default=4096)
    p.add_argument("--albedo_iters", type=int, default=1000)
    p.add_argument("--uniform_sphere_rate", type=float, default=0.5)
    p.add_argument("--bg_radius", type=float, default=1.4)
    p.add_argument("--density_thresh", type=float, default=10)
    p.add_argument("--fp16", action="store_true")
    # BASELINE configs[4] (C5): bf16 autocast (native bf16 field, no GradScaler)
    # and SD-2.1-base guidance (text dim 1024); not in the reference
    p.add_argument("--bf16", action="store_true")
    p.add_argument("--sd_version", type=str, default="1.5", choices=["1.5", "2.1-base"])
    p.add_argument("--backbone", type=str, default="grid")
    p.add_argument("--w", type=int, default=64)
    p.add_argument("--h", type=int, default=64)
    p.add_argument("--jitter_pose", action="store_true")
    p.add_argument("--bound", type=float, default=1)
    p.add_argument("--dt_gamma", type=float, default=0)
    p.add_argument("--min_near", type=float, default=0.1)
    p.add_argument("--radius_range", type=float, nargs="*", default=[1.0, 1.5])
    p.add_argument("--fovy_range", type=float, nargs="*", default=[40, 70])
    p.add_argument("--dir_text", action="store_true")
    p.add_argument("--suppress_face", action="store_true")
    p.add_argument("--angle_overhead", type=float, default=30)
    p.add_argument("--angle_front", type=float, default=60)
    p.add_argument("--lambda_entropy", type=float, default=1e-4)
    p.add_argument("--lambda_opacity", type=float, default=0)
    p.add_argument("--lambda_orient", type=float, default=1e-2)
    p.add_argument("--lambda_smooth", type=float, default=0)
    p.add_argument("--gui", action="store_true")
    p.add_argument("--W", type=int, default=800)
    p.add_argument("--H", type=int, default=800)
    p.add_argument("--radius", type=float, default=3)
    p.add_argument("--fovy", type=float, default=60)
    p.add_argument("--light_theta", type=float, default=60)
    p.add_argument("--light_phi", type=float, default=0)
    p.add_argument("--max_spp", type=int, default=1)
    return p


def parse_opt(argv=None):
    opt = get_parser().parse_args(argv)
    if opt.O:
        opt.fp16, opt.dir_text, opt.cuda_ray = True, True, True
    elif opt.O2:
        opt.fp16, opt.dir_text = True, True
    if opt.bf16:
        opt.fp16 = False  # -O --bf16: the C5 option replaces fp16 autocast
    return opt


def main(argv=None):
    from nerf.network_grid import NeRFNetwork
    from nerf.provider import NeRFDataset
    from nerf.sd import InjectedSDS, StableDiffusion, SyntheticSDS
    from nerf.utils import Trainer, make_adam, seed_everything

    opt = parse_opt(argv)
    if opt.backbone != "grid":
        raise NotImplementedError(f"--backbone {opt.backbone} is not implemented")
    seed_everything(opt.seed)
    model = NeRFNetwork(opt)
    device = torch.device("cuda")
    if opt.test:
        trainer = Trainer("df", opt, model, None, device=device, workspace=opt.workspace,
                          fp16=opt.fp16, bf16=opt.bf16, use_checkpoint=opt.ckpt)
        loader = NeRFDataset(opt, device=device, type="test", H=opt.H, W=opt.W, size=100).dataloader()
        for data in loader:
            trainer.test_step(data)
        if opt.save_mesh:
            trainer.save_mesh(resolution=256)  # main.py:121-122
        return
    train_loader = NeRFDataset(opt, device=device, type="train", H=opt.h, W=opt.w,
                               size=100).dataloader()
    optimizer = lambda m: make_adam(m.get_params(opt.lr), betas=(0.9, 0.99), eps=1e-15)
    scheduler = lambda o: torch.optim.lr_scheduler.LambdaLR(o, lambda it: 0.1 ** min(it / opt.iters, 1))
    text_dim = 1024 if opt.sd_version == "2.1-base" else 768
    if opt.guidance == "synthetic":
        guidance = InjectedSDS(device, text_dim=text_dim)
    elif opt.guidance == "mock":
        guidance = SyntheticSDS(device, text_dim=text_dim)
    else:
        guidance = StableDiffusion(device, dtype=torch.bfloat16 if opt.bf16 else torch.float16)
    trainer = Trainer("df", opt, model, guidance, device=device, workspace=opt.workspace,
                      optimizer=optimizer, ema_decay=None, fp16=opt.fp16, bf16=opt.bf16,
                      lr_scheduler=scheduler,
                      use_checkpoint=opt.ckpt, eval_interval=opt.eval_interval,
                      scheduler_update_every_step=True)
    max_epoch = int(np.ceil(opt.iters / len(train_loader)))
    trainer.train(train_loader, None, max_epoch)
    if opt.save_mesh:
        trainer.save_mesh(resolution=256)  # main.py:161-162


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    main()
