#!/bin/bash
# Round-4 check: bench.py --gpus 2 on a one-GPU box (gloo), the normal path and
# the DP-detail watchdog path (limit forced to 2 s).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SKGE_BENCH_ONE_GPU=1 SKGE_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 1 > gpurun_out/bench_g2_b.log 2>&1 || { tail -20 gpurun_out/bench_g2_b.log; exit 1; }
SKGE_BENCH_ONE_GPU=1 SKGE_BENCH_BACKEND=gloo SKGE_BENCH_DP_TIMEOUT=2 timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 1 > gpurun_out/bench_g2_wd.log 2>&1 || { tail -20 gpurun_out/bench_g2_wd.log; exit 1; }
for f in bench_g2_b bench_g2_wd; do
  python3 - "$f" <<'PY'
import json, sys
f = sys.argv[1]
lines = [x for x in open("gpurun_out/%s.log" % f) if x.startswith("{")]
j = json.loads(lines[0])
print(f, "json lines:", len(lines), "n_gpus", j["n_gpus"], "value", j["value"], "cpu", j["cpu_baseline"],
      "dp:", json.dumps(j["detail"]["one_model_dp"])[:160])
PY
done
exit 0
