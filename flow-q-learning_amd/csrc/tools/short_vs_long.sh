#!/bin/bash
# The driver-style short bench (--steps 20 --warmup 5) against a long one, same box:
#   bash flow-q-learning_amd/csrc/tools/short_vs_long.sh
set -uo pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
  timeout -k 5 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --eval-envs 0 --envmodel-train-steps 0 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('20/5', d['value'], d['ms_per_step'])" || exit 1
done
timeout -k 5 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-probe --no-cpu-baseline --eval-envs 0 --envmodel-train-steps 0 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('20/5 no-probe', d['value'], d['ms_per_step'])" || exit 1
timeout -k 5 200 python bench.py --gpus 1 --steps 500 --warmup 50 --no-cpu-baseline --eval-envs 0 --envmodel-train-steps 0 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('500/50', d['value'], d['ms_per_step'])" || exit 1
timeout -k 5 200 python bench.py --gpus 1 --steps 20 --warmup 5 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('20/5 full', d['value'], d['ms_per_step'])" || exit 1
