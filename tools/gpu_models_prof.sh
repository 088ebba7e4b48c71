#!/bin/bash
# Round evidence for the model configs: full GPU tests, smoke, the default
# bench line, configs 3 / 4 with their CPU legs, and rocprofv3 kernel stats of
# the config 3 / 4 benches (gpurun_out/prof_c3_$TAG, prof_c4_$TAG).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG=${TAG:-r02}
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 > gpurun_out/pytest_all.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_all.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_c2_$TAG.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_c2_$TAG.log > gpurun_out/bench_c2_$TAG.json
for c in 3 4; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 > gpurun_out/bench_c${c}_$TAG.log 2>&1 || exit $?
  grep '^{' gpurun_out/bench_c${c}_$TAG.log > gpurun_out/bench_c${c}_$TAG.json
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_c${c}_$TAG -o run -- python3 bench.py --config $c --steps 5 --warmup 1 --no-cpu --large-nb 0 > gpurun_out/prof_c${c}_$TAG.log 2>&1 || exit $?
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/bench_c*_*.json")):
    j = json.load(open(f))
    print(f, j["value"], j["roofline"]["frac"], (j.get("cpu_baseline") or {}).get("value"),
          (j["detail"].get("large_batch") or {}).get("value"))
PY
