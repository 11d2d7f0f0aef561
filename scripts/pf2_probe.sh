# read-back loop (perframe_loop.py), per-frame deferral modes alternated to separate order effects
set -o pipefail
for rep in 1 2 3; do
  for t in "perframe_defer=2" "perframe_defer=0" "perframe_defer_min=1000000000"; do
    timeout -k 10 120 python scripts/perframe_loop.py --tune $t || exit 1
  done
done
