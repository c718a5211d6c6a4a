"""Per-kernel instruction census of a disassembly (tools/disasm.sh output):
python tools/kstat.py /tmp/g.s k_grid_bwd_sliced"""
import re
import sys
from collections import Counter


def main(path, pat):
    cur, body = None, {}
    for line in open(path):
        m = re.match(r"^[0-9a-f]+ <(.*)>:", line)
        if m:
            cur = m.group(1)
            body[cur] = []
            continue
        if cur and line.startswith("\t"):
            body[cur].append(line.split()[0])
    for k, ins in body.items():
        if pat not in k:
            continue
        c = Counter(ins)
        vmax = 0
        scratch = sum(v for op, v in c.items() if op.startswith("scratch_"))
        print(k[:90], "instrs", len(ins), "scratch", scratch,
              "ds_add_f64", c["ds_add_f64"], "global_load", sum(v for op, v in c.items() if op.startswith("global_load")),
              "salu", sum(v for op, v in c.items() if op.startswith("s_")))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
