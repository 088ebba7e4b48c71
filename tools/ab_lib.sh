#!/bin/bash
# A/B of compile-time variants: builds each "name=FLAG" (tools/ablate.sh, on
# the box) and runs one bench line per variant with SKGE_LIB_PATH pointing at
# it.  BENCHARGS: bench.py arguments (e.g. --config 4); BENCHARGS2, if set: a
# second workload, every variant measured on it too.  The default build is
# measured first and last as "base" / "base2".
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 bash tools/ablate.sh "$@" > gpurun_out/ab_lib_build.log 2>&1 || { tail -5 gpurun_out/ab_lib_build.log; exit 1; }
one() {  # name libpath benchargs
  local n=$1 lp=$2 ba=$3
  env ${lp:+SKGE_LIB_PATH=$lp} timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --no-roofline --large-nb 0 $ba > gpurun_out/ablib_$n.log 2>&1 || return 1
  python3 - "$n" "$ba" <<'PY'
import json,sys; n=sys.argv[1]
l=[x for x in open("gpurun_out/ablib_%s.log" % n) if x.startswith("{")][0]; j=json.loads(l)
hp = (j.get("detail") or {}).get("handoff_probe") or {}
print(n, "[%s]" % sys.argv[2], round(j["value"]/1e6,2), j["ms_per_step"], j["roofline"].get("avg_launch_us"), j["roofline"].get("frac"), "hop_us", hp.get("us_per_hop"))
PY
}
sets=("${BENCHARGS:-}")
[ -n "${BENCHARGS2:-}" ] && sets+=("$BENCHARGS2")
k=0
for ba in "${sets[@]}"; do
  k=$((k + 1))
  one base$k "" "$ba" || exit 1
  for v in "$@"; do
    name=${v%%=*}
    one ${name}$k "$PWD/scikit-kge_amd/build_abl/$name/libskgehip.so" "$ba" || exit 1
  done
  one base${k}b "" "$ba" || exit 1
done
