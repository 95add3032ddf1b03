#!/bin/bash
# Round-4 GPU probe 4: the split Euler flow's per-layer phases at 1 and 2 members (phase
# build), and the 8-deep ring library against HEAD at 1 / 2 / 4 members.
set -uo pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; cd $R
for m in 2 1; do
FQLPOP_LIB=$R/flow-q-learning_amd/fqlpop/libfqlpop_phase.so FQLPOP_PHASE_PROBE=1 timeout -k 10 120 \
  python -u flow-q-learning_amd/csrc/tools/phase_run.py 30 cube members=$m > $O/r4_phase_m$m.txt 2>&1; rc=$?
echo "members $m rc $rc"; grep -A12 "split Euler" $O/r4_phase_m$m.txt; [ $rc -eq 0 ] || exit $rc
done
S=flow-q-learning_amd/csrc/tools/members_sweep.sh
FQLPOP_LIB=$R/flow-q-learning_amd/fqlpop/libfqlpop_pf8.so bash $S "1 2 4" 1 --diagnostic > $O/r4_sweep4_pf8.txt 2>&1; rc=$?; echo PF8; cat $O/r4_sweep4_pf8.txt; [ $rc -eq 0 ] || exit $rc
bash $S "1 2 4" 1 > $O/r4_sweep4_head.txt 2>&1; rc=$?; echo HEAD; cat $O/r4_sweep4_head.txt
