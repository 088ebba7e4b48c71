# A/B of library builds / runtime switches on any bench.py line.
#   AB='name VAR=value ...;name2 ...'  BENCH_ARGS='--config 3 --steps 10'
# prints: name, value (M triples/s), the roofline kernel's avg launch (us), the
# large-batch detail value (M) when present
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
IFS=';' read -ra specs <<< "${AB:-base}"
for spec in "${specs[@]}"; do
  set -- $spec
  n=$1; shift
  env "$@" timeout -k 10 200 python bench.py ${BENCH_ARGS:---steps 20 --warmup 3} --no-cpu \
    > gpurun_out/abb_$n.log 2>&1 || { echo "$n failed"; tail -3 gpurun_out/abb_$n.log; exit 1; }
  python3 - "$n" <<'PY'
import json, sys
n = sys.argv[1]
l = [x for x in open("gpurun_out/abb_%s.log" % n) if x.startswith("{")][0]
j = json.loads(l)
lb = j.get("detail", {}).get("large_batch") or {}
print(n, round(j["value"] / 1e6, 2), j["roofline"].get("avg_launch_us"),
      round(lb["value"] / 1e6, 2) if lb.get("value") else "-", lb.get("ms_per_epoch", "-"))
PY
done
