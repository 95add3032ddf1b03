#!/bin/bash
# Same-box A/B of the world-model rollout leg (eval_rollout.ms) between the working-tree
# library ("new") and fqlpop/libfqlpop_ref.so, two interleaved pairs (GPU box, repo root).
set -uo pipefail
R=$(pwd); O=$R/gpurun_out
for rep in 1 2; do for f in new ref; do
  if [ $f = new ]; then unset FQLPOP_LIB; else export FQLPOP_LIB=$R/flow-q-learning_amd/csrc/devlib/libfqlpop_$f.so; fi
  timeout -k 5 150 python bench.py --diagnostic --steps 100 --no-cpu-baseline --no-probe --envmodel-train-steps 0 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('$f', d['value'], d['eval_rollout']['ms'])" || exit 1
done; done
