#!/bin/bash
# Same-box A/B of several builds (developer loop, on the GPU box from the repo root):
#   bash flow-q-learning_amd/csrc/tools/ab_libs.sh new ref opq ...
# "new" is the working-tree library, any other name X is csrc/ablib/libfqlpop_X.so (shipped to the box; csrc/devlib is not) (FQLPOP_LIB);
# the list is run REPS (2) times, interleaved; BENCH_ARGS (e.g. "--members 2") and STEPS (400) as
# in ab_opts.sh.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
for rep in $(seq 1 ${REPS:-2}); do
  for f in "$@"; do
    if [ "$f" = new ]; then unset FQLPOP_LIB; else export FQLPOP_LIB=$R/flow-q-learning_amd/csrc/ablib/libfqlpop_$f.so; fi
    timeout -k 5 120 python bench.py --diagnostic --steps ${STEPS:-400} --no-cpu-baseline --no-probe --eval-envs 0 --envmodel-train-steps 0 \
        ${BENCH_ARGS:-} 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('$f', d['value'], d['ms_per_step'])" || exit 1
  done
done
