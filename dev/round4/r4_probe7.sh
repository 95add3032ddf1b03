#!/bin/bash
# Round-4 GPU probe 7: default engine options only (split_blocks 256, the configuration that
# never exceeds the probe buffer): split bit identity, per-GPU rate sweep, 2-member timeline.
set -uo pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -v --timeout 200 --timeout-method thread > $O/r4_split7.txt 2>&1; rc=$?
tail -3 $O/r4_split7.txt; [ $rc -eq 0 ] || exit $rc
bash flow-q-learning_amd/csrc/tools/members_sweep.sh "1 2 4 8" 1 > $O/r4_sweep7.txt 2>&1; rc=$?; cat $O/r4_sweep7.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tl_m2_s7 -o run -- python3 $R/bench.py --members 2 --steps 60 --warmup 20 --no-cpu-baseline --kernel-iters 1 --no-probe --eval-envs 0 --envmodel-train-steps 0 > $O/tl_m2_s7.log 2>&1 || exit $?
python3 $R/flow-q-learning_amd/csrc/tools/step_timeline.py $O/tl_m2_s7/run_kernel_trace.csv > $O/tl_m2_s7.txt; head -22 $O/tl_m2_s7.txt
