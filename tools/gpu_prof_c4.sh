#!/bin/bash
# rocprofv3 kernel stats of the RESCAL config-4 bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o run --output-format csv -- python3 bench.py --config 4 --no-cpu --steps 5 --warmup 1 > gpurun_out/prof_c4.log 2>&1 || { tail -5 gpurun_out/prof_c4.log; exit 1; }
f=$(find gpurun_out/prof_c4 -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:12]:
    print("%-60s %6s %10.2f us  %5s%%" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3, r["Percentage"][:5]))
PY
