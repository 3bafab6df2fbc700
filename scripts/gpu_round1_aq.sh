#!/bin/bash
# GPU pass aq: k_paths batching sweep (refill_min, dda_budget) on the default workload.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/aq
mkdir -p $O
export PYTHONUNBUFFERED=1
for rm in 24 32 40 48 56; do
  timeout -k 10 120 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --refill-min $rm > $O/rm$rm.log 2>&1 || exit 1
  echo "refill $rm $(grep -o '"value": [0-9.]*' $O/rm$rm.log)"
done
for db in 6 8 16 24; do
  timeout -k 10 120 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --dda-budget $db > $O/db$db.log 2>&1 || exit 1
  echo "budget $db $(grep -o '"value": [0-9.]*' $O/db$db.log)"
done
exit 0
