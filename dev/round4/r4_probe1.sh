#!/bin/bash
# Round-4 GPU probe: split-launch tests first (bounded), the GPU suite, members-per-GPU sweeps
# (split off / auto), a 2-member step timeline, and the GPU_MAX_HW_QUEUES=2 run under a
# native backtrace handler (last: it may abort).
set -uo pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; cd $R
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }   # 1 = test failures: the GPU is fine, go on
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -v --timeout 200 --timeout-method thread > $O/r4_split.txt 2>&1; rc=$?
tail -15 $O/r4_split.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/r4_tests.txt 2>&1; rc=$?
tail -15 $O/r4_tests.txt; ok $rc || exit $rc
bash flow-q-learning_amd/csrc/tools/members_sweep.sh "16 1 2 4 8" 1 "--engine-option split=0" > $O/r4_sweep0.txt 2>&1; rc=$?; cat $O/r4_sweep0.txt; [ $rc -eq 0 ] || exit $rc
bash flow-q-learning_amd/csrc/tools/members_sweep.sh "1 2 4" 1 > $O/r4_sweep1.txt 2>&1; rc=$?; cat $O/r4_sweep1.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for sp in 0 1; do
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tl_m2_s$sp -o run -- python3 $R/bench.py --members 2 --steps 60 --warmup 20 --no-cpu-baseline --kernel-iters 1 --no-probe --eval-envs 0 --envmodel-train-steps 0 --engine-option split=$sp > $O/tl_m2_s$sp.log 2>&1 || exit $?
python3 $R/flow-q-learning_amd/csrc/tools/step_timeline.py $O/tl_m2_s$sp/run_kernel_trace.csv > $O/tl_m2_s$sp.txt; head -50 $O/tl_m2_s$sp.txt
done
cd $R
GPU_MAX_HW_QUEUES=2 timeout -k 10 120 python -X faulthandler -c "
import ctypes, sys, runpy
ctypes.CDLL('$R/flow-q-learning_amd/csrc/build/crash_bt.so')
sys.argv=['bench.py','--steps','20','--warmup','5','--no-cpu-baseline','--eval-envs','0','--envmodel-train-steps','0','--kernel-iters','2']
runpy.run_path('bench.py', run_name='__main__')
" > $O/hwq2b.json 2> $O/hwq2b.err; echo "hwq2 rc $?"; tail -60 $O/hwq2b.err
