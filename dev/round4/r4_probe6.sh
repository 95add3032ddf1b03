#!/bin/bash
# Round-4 GPU probe 6: per-form split ring depth; split_blocks 256 (default) vs 512.
set -uo pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -v --timeout 200 --timeout-method thread > $O/r4_split6.txt 2>&1; rc=$?
tail -3 $O/r4_split6.txt; [ $rc -eq 0 ] || exit $rc
S=flow-q-learning_amd/csrc/tools/members_sweep.sh
bash $S "1 2 4 8" 1 > $O/r4_sweep6_head.txt 2>&1; rc=$?; echo HEAD; cat $O/r4_sweep6_head.txt; [ $rc -eq 0 ] || exit $rc
bash $S "1 2 4" 1 "--engine-option split_blocks=512" > $O/r4_sweep6_b512.txt 2>&1; rc=$?; echo B512; cat $O/r4_sweep6_b512.txt; [ $rc -eq 0 ] || exit $rc
bash $S "2" 1 > $O/r4_sweep6_head2.txt 2>&1; rc=$?; echo HEAD again; cat $O/r4_sweep6_head2.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for v in 256 512; do
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tl_m2_b$v -o run -- python3 $R/bench.py --members 2 --steps 60 --warmup 20 --no-cpu-baseline --kernel-iters 1 --no-probe --eval-envs 0 --envmodel-train-steps 0 --engine-option split_blocks=$v > $O/tl_m2_b$v.log 2>&1 || exit $?
python3 $R/flow-q-learning_amd/csrc/tools/step_timeline.py $O/tl_m2_b$v/run_kernel_trace.csv > $O/tl_m2_b$v.txt; echo "split_blocks $v"; head -22 $O/tl_m2_b$v.txt
done
