#!/bin/bash
# Interleaved A/B of the bench preheat kinds on the driver's short command
# (--steps 20 --warmup 5), plus one --steps 500 steady-state reference per kind.
# Usage (repo root, GPU box): bash flow-q-learning_amd/csrc/tools/ab_preheat.sh <tag> [pairs]
set -euo pipefail
TAG=${1:-ph}
PAIRS=${2:-3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
LEGS="--no-cpu-baseline --eval-envs 0 --envmodel-train-steps 0"
for i in $(seq 1 "$PAIRS"); do
    for k in kernel steps; do
        timeout -k 10 240 python "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --preheat-kind $k $LEGS \
            > "$O/${TAG}_${k}_$i.json" 2>> "$O/${TAG}.err"
        python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['preheat'])" \
            "$O/${TAG}_${k}_$i.json" "$k/$i"
    done
done
for k in kernel steps; do
    timeout -k 10 300 python "$R/bench.py" --preheat-kind $k $LEGS > "$O/${TAG}_${k}_500.json" 2>> "$O/${TAG}.err"
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'])" \
        "$O/${TAG}_${k}_500.json" "$k/500"
done
echo "ab_preheat $TAG done"
