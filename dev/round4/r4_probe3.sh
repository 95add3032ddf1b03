#!/bin/bash
# Round-4 GPU probe 3: split + small-schedule bit identity, then per-GPU throughput at 1 / 2 /
# 4 / 16 members for: HEAD (deep split ring, small schedule), small schedule off, and the
# 8-deep ring (libfqlpop_pf8.so); a 2-member step timeline; finally the default graph under
# GPU_MAX_HW_QUEUES=2 (round 3: a crash inside hipGraphLaunch), last because it may crash.
set -uo pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -v --timeout 200 --timeout-method thread > $O/r4_split3.txt 2>&1; rc=$?
tail -12 $O/r4_split3.txt; [ $rc -eq 0 ] || exit $rc
S=flow-q-learning_amd/csrc/tools/members_sweep.sh
bash $S "1 2 4 16" 1 > $O/r4_sweep3_head.txt 2>&1; rc=$?; echo HEAD; cat $O/r4_sweep3_head.txt; [ $rc -eq 0 ] || exit $rc
bash $S "1 2" 1 "--engine-option small_sched=0" > $O/r4_sweep3_nosmall.txt 2>&1; rc=$?; echo NOSMALL; cat $O/r4_sweep3_nosmall.txt; [ $rc -eq 0 ] || exit $rc
FQLPOP_LIB=$R/flow-q-learning_amd/fqlpop/libfqlpop_pf8.so bash $S "1 2 4" 1 > $O/r4_sweep3_pf8.txt 2>&1; rc=$?; echo PF8; cat $O/r4_sweep3_pf8.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tl_m2_s3 -o run -- python3 $R/bench.py --members 2 --steps 60 --warmup 20 --no-cpu-baseline --kernel-iters 1 --no-probe --eval-envs 0 --envmodel-train-steps 0 > $O/tl_m2_s3.log 2>&1 || exit $?
python3 $R/flow-q-learning_amd/csrc/tools/step_timeline.py $O/tl_m2_s3/run_kernel_trace.csv > $O/tl_m2_s3.txt; head -45 $O/tl_m2_s3.txt
cd $R
GPU_MAX_HW_QUEUES=2 timeout -k 10 120 python -c "
import ctypes, sys, runpy
ctypes.CDLL('$R/flow-q-learning_amd/csrc/build/crash_bt.so')
sys.argv=['bench.py','--steps','10','--warmup','3','--no-cpu-baseline','--eval-envs','0','--envmodel-train-steps','0','--kernel-iters','2','--preheat-ms','0']
runpy.run_path('bench.py', run_name='__main__')
" > $O/hwq2_graph.json 2> $O/hwq2_graph.err; rc=$?; echo "hwq2 graph rc $rc"; tail -30 $O/hwq2_graph.err
exit 0
