# MFMA-utilisation PMC pass over a short serial-stream bench (run on the GPU box from the repo root):
#   bash flow-q-learning_amd/csrc/tools/pmc_step.sh; python3 flow-q-learning_amd/csrc/tools/pmc_step_summary.py gpurun_out/pmcstep/run_counter_collection.csv
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmcstep -o run -- python3 $R/bench.py --serial --steps 10 --warmup 5 --no-cpu-baseline --kernel-iters 1 --no-probe --eval-envs 0 --envmodel-train-steps 0 > $R/gpurun_out/pmcstep.log 2>&1
echo rc $?
ls $R/gpurun_out/pmcstep
