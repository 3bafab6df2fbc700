#!/bin/bash
# round-5 pass j: does staging the NanoVDB majorant in LDS speed up its walk?
# At a 16^3 majorant (fits LDS) the same NanoVDB walk runs with the majorant read through L2
# (in-tree build) and from LDS (variants/vmajlds, -DAVR_VDB_MAJ_LDS), alternating processes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r05/j
mkdir -p $O
export TMPDIR=/tmp
for k in 1 2; do
  timeout -k 10 300 python tools/walk_sweep.py --medium nanovdb --majorant-res 16 --steps 4 --rounds 2 > $O/l2_$k.json 2> $O/l2_$k.err || { tail -5 $O/l2_$k.err; exit 1; }
  AVR_LIB=variants/vmajlds/libavr_hip.so timeout -k 10 300 python tools/walk_sweep.py --medium nanovdb --majorant-res 16 --steps 4 --rounds 2 > $O/lds_$k.json 2> $O/lds_$k.err || { tail -5 $O/lds_$k.err; exit 2; }
done
for f in $O/l2_1.json $O/lds_1.json $O/l2_2.json $O/lds_2.json; do echo "$f $(cut -c1-400 $f)"; done
