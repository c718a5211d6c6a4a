#!/bin/bash
# A/B: windowed vs slice form of the binned backward, per level and whole.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=${RANGES:-0-0,1-1,2-2,3-3,4-4,5-5,6-6,7-7,8-8,9-9,10-10,11-11,12-12,13-13,14-14,15-15,0-15}
echo "== windowed"; timeout -k 10 200 python tools/grid_bin_case.py --reps 5 --ranges $R || exit 1
echo "== slices"; DFHIP_GRID_NOWIN=1 timeout -k 10 200 python tools/grid_bin_case.py --reps 5 --ranges $R || exit 1
