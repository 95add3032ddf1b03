#!/bin/bash
# Same-box A/B of the in-step probe's cost (developer loop, on the GPU box):
#   bash flow-q-learning_amd/csrc/tools/ab_probe.sh [extra bench args]
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
for rep in 1 2 3; do
  for p in "" "--no-probe"; do
    timeout -k 5 120 python bench.py --diagnostic --steps 400 --no-cpu-baseline --eval-envs 0 --envmodel-train-steps 0 $p "$@" \
        2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('probe' if '$p' == '' else 'noprobe', d['value'], d['ms_per_step'])" || exit 1
  done
done
