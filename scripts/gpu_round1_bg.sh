#!/bin/bash
# GPU pass bg: DDA budget / refill sweep on the NanoVDB S-cloud-512 workload.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/bg
mkdir -p $O
export PYTHONUNBUFFERED=1
for db in 8 12 16 24 32; do
  timeout -k 10 200 python bench.py --res 512 --medium nanovdb --steps 6 --warmup 2 --no-cpu-baseline --dda-budget $db > $O/db$db.log 2>&1 || exit 1
  echo "budget $db $(grep -o '"value": [0-9.]*' $O/db$db.log)"
done
for rm in 24 40; do
  timeout -k 10 200 python bench.py --res 512 --medium nanovdb --steps 6 --warmup 2 --no-cpu-baseline --refill-min $rm > $O/rm$rm.log 2>&1 || exit 1
  echo "refill $rm $(grep -o '"value": [0-9.]*' $O/rm$rm.log)"
done
exit 0
