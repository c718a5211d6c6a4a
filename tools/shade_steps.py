"""Run graph-replayed native train steps of one shading (profiling target):
    python tools/shade_steps.py [textureless|lambertian|albedo] [steps]"""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "single-stable-dreamfusion_amd")):
    sys.path.insert(0, p)
import torch
import bench

kind = sys.argv[1] if len(sys.argv) > 1 else "textureless"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
tr, dat = bench.make_trainer(128, 0, 0, 1, True, graph=True)
tr.pick_shading = lambda: (kind, 0.1 if kind != "albedo" else 1.0)
for _ in range(5):
    tr.train_iteration(dat.collate([0]))
torch.cuda.synchronize()
for _ in range(steps):
    tr.train_iteration(dat.collate([0]))
torch.cuda.synchronize()
print("samples/step", float(tr.model.step_counter[:, 0].float().mean()))
