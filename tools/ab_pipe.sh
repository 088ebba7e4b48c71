# A/B of pipelined-runner switches (bench.py default config, nb=100 + the nb=2 detail line;
# BENCHARGS adds bench.py arguments, e.g. --config 1)
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
run() { # name env...
  local n=$1; shift
  env "$@" timeout -k 10 150 python bench.py --steps 20 --warmup 3 --no-cpu --no-roofline --large-nb 2 ${BENCHARGS:-} > gpurun_out/ab_$n.log 2>&1 || return 1
  python3 - "$n" <<'PY'
import json,sys; n=sys.argv[1]
l=[x for x in open("gpurun_out/ab_%s.log" % n) if x.startswith("{")][0]; j=json.loads(l)
lb = j["detail"].get("large_batch") or {}
print(n, round(j["value"]/1e6,2), j["roofline"].get("avg_launch_us"), round(lb.get("value", 0)/1e6,2), lb.get("ms_per_epoch"))
PY
}
# AB: ';'-separated specs "name VAR=value ...", default grouped vs ungrouped applies
IFS=';' read -ra specs <<< "${AB:-grp SKGE_PIPE_GRP=1;nogrp SKGE_PIPE_GRP=0}"
for spec in "${specs[@]}"; do
  run $spec || exit 1
done
