for r in ${RUNSL:-1 2 4 8 16}; do echo runs $r; DFHIP_WALK_RUNS=$r timeout -k 5 120 python tools/grid_bin_case.py --reps 10 --ranges ${RANGES:-0-15,0-2,3-8,9-15} || exit 1; done
