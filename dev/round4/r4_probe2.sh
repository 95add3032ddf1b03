#!/bin/bash
# Round-4 GPU probe 2: split tests (bounded), members sweep with split on, 2-member step
# timeline, and which step forms survive GPU_MAX_HW_QUEUES=2 (eager, serial graph; the default
# graph last: it crashed in hipGraphLaunch).
set -uo pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -v --timeout 200 --timeout-method thread > $O/r4_split2.txt 2>&1; rc=$?
tail -12 $O/r4_split2.txt; [ $rc -eq 0 ] || exit $rc
bash flow-q-learning_amd/csrc/tools/members_sweep.sh "1 2 4 16" 1 > $O/r4_sweep2.txt 2>&1; rc=$?; cat $O/r4_sweep2.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tl_m2_s2 -o run -- python3 $R/bench.py --members 2 --steps 60 --warmup 20 --no-cpu-baseline --kernel-iters 1 --no-probe --eval-envs 0 --envmodel-train-steps 0 > $O/tl_m2_s2.log 2>&1 || exit $?
python3 $R/flow-q-learning_amd/csrc/tools/step_timeline.py $O/tl_m2_s2/run_kernel_trace.csv > $O/tl_m2_s2.txt; head -45 $O/tl_m2_s2.txt
cd $R
for v in "--no-graph" "--serial"; do
GPU_MAX_HW_QUEUES=2 timeout -k 10 120 python -c "
import ctypes, sys, runpy
ctypes.CDLL('$R/flow-q-learning_amd/csrc/build/crash_bt.so')
sys.argv=['bench.py','--steps','10','--warmup','3','--no-cpu-baseline','--eval-envs','0','--envmodel-train-steps','0','--kernel-iters','2','--preheat-ms','0','$v']
runpy.run_path('bench.py', run_name='__main__')
" > $O/hwq2_$v.json 2> $O/hwq2_$v.err; rc=$?; echo "hwq2 $v rc $rc"; tail -3 $O/hwq2_$v.err; [ $rc -eq 0 ] || exit $rc
done
