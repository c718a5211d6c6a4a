"""List the host<->device synchronisations of one train step
(torch.cuda.set_sync_debug_mode): python tools/find_syncs.py"""
import sys
import traceback
import warnings
from collections import Counter
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "single-stable-dreamfusion_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402


def main():
    import bench
    graph = "--eager" not in sys.argv
    trainer, data = bench.make_trainer(128, 0, 0, 1, True, graph=graph)
    for _ in range(3):
        trainer.train_iteration(data.collate([0]))
    torch.cuda.synchronize()
    sites = Counter()

    def hook(message, category, filename, lineno, file=None, line=None):
        stack = [f for f in traceback.extract_stack()[:-1] if "repo" in f.filename]
        key = " <- ".join(f"{Path(f.filename).name}:{f.lineno}" for f in stack[-3:][::-1])
        sites[key] += 1

    warnings.showwarning = hook
    warnings.simplefilter("always")
    torch.cuda.set_sync_debug_mode("warn")
    for _ in range(17):  # crosses one density-grid refresh
        trainer.train_iteration(data.collate([0]))
    torch.cuda.set_sync_debug_mode(0)
    for k, v in sites.most_common():
        print(f"{v:4d}  {k}")


if __name__ == "__main__":
    main()
