#!/bin/bash
# A/B of compile-time variants: builds each "name=FLAG" (tools/ablate.sh, on
# the box) and runs one bench line per variant with SKGE_LIB_PATH pointing at
# it.  BENCHARGS: bench.py arguments (e.g. --config 4).  The default build is
# measured first as "base".
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 bash tools/ablate.sh "$@" > gpurun_out/ab_lib_build.log 2>&1 || { tail -5 gpurun_out/ab_lib_build.log; exit 1; }
one() {  # name libpath
  local n=$1 lp=$2
  env ${lp:+SKGE_LIB_PATH=$lp} timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --no-roofline --large-nb 0 ${BENCHARGS:-} > gpurun_out/ablib_$n.log 2>&1 || return 1
  python3 - "$n" <<'PY'
import json,sys; n=sys.argv[1]
l=[x for x in open("gpurun_out/ablib_%s.log" % n) if x.startswith("{")][0]; j=json.loads(l)
print(n, round(j["value"]/1e6,2), j["ms_per_step"], j["roofline"].get("avg_launch_us"), j["roofline"].get("frac"))
PY
}
one base "" || exit 1
for v in "$@"; do
  name=${v%%=*}
  one $name "$PWD/scikit-kge_amd/build_abl/$name/libskgehip.so" || exit 1
done
one base2 "" || exit 1
