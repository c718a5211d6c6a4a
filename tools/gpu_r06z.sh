# C4 queue order by line distance (1) vs by occupied cells (2), tiles in
# mirrored halves, R0 / R1 interleaved (tools/infer_case.py)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
for sc in "" "--sphere"; do
  for i in 1 2 3; do
    for v in 1 2; do
      echo "== order$v $sc"; timeout -k 10 180 python -u $R/tools/infer_case.py $sc --order $v | grep res=
    done
  done
done
