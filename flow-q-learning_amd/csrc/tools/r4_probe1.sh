#!/bin/bash
# Round-4 first GPU probe: members-per-GPU sweep, 2-member step timeline, GPU_MAX_HW_QUEUES=2 backtrace.
set -uo pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; cd $R
bash flow-q-learning_amd/csrc/tools/members_sweep.sh "16 1 2 4 8 16" 1 > $O/r4_sweep.txt 2>&1; cat $O/r4_sweep.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tl_m2 -o run -- python3 $R/bench.py --members 2 --steps 60 --warmup 20 --no-cpu-baseline --kernel-iters 1 --no-probe --eval-envs 0 --envmodel-train-steps 0 > $O/tl_m2.log 2>&1 && python3 $R/flow-q-learning_amd/csrc/tools/step_timeline.py $O/tl_m2/run_kernel_trace.csv > $O/tl_m2.txt; head -60 $O/tl_m2.txt
cd $R
GPU_MAX_HW_QUEUES=2 timeout -k 10 120 python -X faulthandler -c "
import ctypes, sys, runpy
ctypes.CDLL('$R/flow-q-learning_amd/csrc/build/crash_bt.so')
sys.argv=['bench.py','--steps','20','--warmup','5','--no-cpu-baseline','--eval-envs','0','--envmodel-train-steps','0','--kernel-iters','2']
runpy.run_path('bench.py', run_name='__main__')
" > $O/hwq2b.json 2> $O/hwq2b.err; echo "hwq2 rc $?"; tail -60 $O/hwq2b.err
