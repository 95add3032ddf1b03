set -e
cd $GRAFT_REPO_ROOT
for cfg in "FQLPOP_PRIO=0" "FQLPOP_PRIO=2" "FQLPOP_PRIO=2 FQLPOP_STREAMS=4"; do
  env $cfg timeout -k 10 120 python bench.py --no-cpu-baseline --no-probe --steps 300 > gpurun_out/ab.json 2>/dev/null
  echo "$cfg $(python -c "import json; d=json.load(open('gpurun_out/ab.json')); print(d['value'], d['ms_per_step'])")"
done
