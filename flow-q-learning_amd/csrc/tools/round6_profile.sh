#!/bin/bash
# Round-6 measurement set at the working tree's commit (run from the repo root on the GPU box):
#   1. the driver's exact command, its wall time;
#   2. rocprofv3 --kernel-trace --stats of the same bench without the preheat (every launch of
#      the concurrent 16-member step: in-step averages);
#   3. the serial-stream step: a kernel trace, then one --pmc pass per counter group (MFMA busy,
#      FETCH_SIZE, WRITE_SIZE), pmc_table.py;
#   4. FETCH_SIZE / WRITE_SIZE of the dominant kernel replayed alone (pmc_dominant.json).
# Every GPU step under its own timeout; the script stops at the first failure.
#   FQ_COMMIT=<sha> bash flow-q-learning_amd/csrc/tools/round6_profile.sh <tag>
set -uo pipefail
TAG=${1:-r6}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
T=$R/flow-q-learning_amd/csrc/tools
mkdir -p "$O"
cd "$R"
s0=$(date +%s.%N)
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$O/driver_bench.json" 2> "$O/driver_bench.err" \
    || { echo "driver bench failed"; tail -5 "$O/driver_bench.err"; exit 1; }
s1=$(date +%s.%N)
python3 -c "print(f'wall {${s1} - ${s0}:.2f} s')" > "$O/driver_bench.wall"
cat "$O/driver_bench.wall"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/instep" -o run -- \
    python3 "$R/bench.py" --steps 100 --warmup 20 --no-cpu-baseline --kernel-iters 1 --preheat-ms 0 \
    --envmodel-train-steps 0 --eval-envs 0 > "$O/instep.log" 2>&1 || { echo "in-step trace failed"; exit 1; }
B=(python3 "$R/bench.py" --serial --steps 12 --warmup 4 --no-cpu-baseline --kernel-iters 1 --no-probe --preheat-ms 0
   --eval-envs 0 --envmodel-train-steps 0)
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/pmc/trace" -o run -- "${B[@]}" \
    > "$O/pmc_trace.log" 2>&1 || { echo "serial trace failed"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv \
    -d "$O/pmc/mfma" -o run -- "${B[@]}" > "$O/pmc_mfma.log" 2>&1 || { echo "mfma pass failed"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc/fetch" -o run -- "${B[@]}" \
    > "$O/pmc_fetch.log" 2>&1 || { echo "fetch pass failed"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc/write" -o run -- "${B[@]}" \
    > "$O/pmc_write.log" 2>&1 || { echo "write pass failed"; exit 1; }
python3 "$T/pmc_table.py" "$O/pmc" > "$O/pmc_table_serial.txt" && cat "$O/pmc_table_serial.txt"
K=euler_flow_kernel
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" --output-format csv -d "$O/dom_fetch" -o run -- \
    python3 "$T/profile_dominant.py" 20 > "$O/dom_fetch.log" 2>&1 || { echo "dominant fetch failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" --output-format csv -d "$O/dom_write" -o run -- \
    python3 "$T/profile_dominant.py" 20 > "$O/dom_write.log" 2>&1 || { echo "dominant write failed"; exit 1; }
F=$(ls "$O"/dom_fetch/*counter_collection.csv "$O"/dom_fetch/*/*counter_collection.csv 2>/dev/null | head -1)
W=$(ls "$O"/dom_write/*counter_collection.csv "$O"/dom_write/*/*counter_collection.csv 2>/dev/null | head -1)
python3 "$T/pmc_summary.py" "$F" "$W" "$K" "$O/pmc_dominant.json"
echo "round6_profile $TAG done"
