#!/bin/bash
# Round-4 GPU probe 5 (split launches with wave-uniform tickets: no waterfall loops): split
# bit identity, split Euler phases at 2 / 1 members, per-GPU rate sweep (HEAD, 8-deep ring),
# 2-member step timeline.
set -uo pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -v --timeout 200 --timeout-method thread > $O/r4_split5.txt 2>&1; rc=$?
tail -3 $O/r4_split5.txt; [ $rc -eq 0 ] || exit $rc
for m in 2 1; do
FQLPOP_LIB=$R/flow-q-learning_amd/fqlpop/libfqlpop_phase.so FQLPOP_PHASE_PROBE=1 timeout -k 10 120 \
  python -u flow-q-learning_amd/csrc/tools/phase_run.py 30 cube members=$m > $O/r4_phase5_m$m.txt 2>&1; rc=$?
echo "members $m rc $rc"; grep -A8 "split Euler" $O/r4_phase5_m$m.txt; [ $rc -eq 0 ] || exit $rc
done
S=flow-q-learning_amd/csrc/tools/members_sweep.sh
bash $S "1 2 4 8 16" 1 > $O/r4_sweep5_head.txt 2>&1; rc=$?; echo HEAD; cat $O/r4_sweep5_head.txt; [ $rc -eq 0 ] || exit $rc
FQLPOP_LIB=$R/flow-q-learning_amd/fqlpop/libfqlpop_pf8.so bash $S "1 2 4" 1 --diagnostic > $O/r4_sweep5_pf8.txt 2>&1; rc=$?; echo PF8; cat $O/r4_sweep5_pf8.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tl_m2_s5 -o run -- python3 $R/bench.py --members 2 --steps 60 --warmup 20 --no-cpu-baseline --kernel-iters 1 --no-probe --eval-envs 0 --envmodel-train-steps 0 > $O/tl_m2_s5.log 2>&1 || exit $?
python3 $R/flow-q-learning_amd/csrc/tools/step_timeline.py $O/tl_m2_s5/run_kernel_trace.csv > $O/tl_m2_s5.txt; head -45 $O/tl_m2_s5.txt
