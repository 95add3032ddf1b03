#!/bin/bash
# Per-kernel counters of the population step at the working tree's HEAD (serial stream, so every
# launch runs uncontended): kernel trace + stats, then one --pmc pass each for the MFMA pipe
# (SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE), FETCH_SIZE and WRITE_SIZE (separate passes: the
# TCC block holds 4 counters, FETCH_SIZE takes 3 and WRITE_SIZE 2).  Summary: pmc_table.py.
#   bash flow-q-learning_amd/csrc/tools/round_pmc.sh <tag> [extra bench args]
set -uo pipefail
TAG=${1:-r}; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
B=(python3 "$R/bench.py" --serial --steps 12 --warmup 4 --no-cpu-baseline --kernel-iters 1 --no-probe --preheat-ms 0
   --eval-envs 0 --envmodel-train-steps 0 "$@")
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- "${B[@]}" \
    > "$O/trace.log" 2>&1 || { echo "trace pass failed"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv \
    -d "$O/mfma" -o run -- "${B[@]}" > "$O/mfma.log" 2>&1 || { echo "mfma pass failed"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/fetch" -o run -- "${B[@]}" \
    > "$O/fetch.log" 2>&1 || { echo "fetch pass failed"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/write" -o run -- "${B[@]}" \
    > "$O/write.log" 2>&1 || { echo "write pass failed"; exit 1; }
python3 "$R/flow-q-learning_amd/csrc/tools/pmc_table.py" "$O" > "$O/table.txt" && cat "$O/table.txt"
