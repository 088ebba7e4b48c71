set -u
cd $GRAFT_REPO_ROOT
true
run() { # name env... 
  local n=$1; shift
  env "$@" timeout -k 10 150 python bench.py --steps 20 --warmup 3 --no-cpu --no-roofline --large-nb 2 > gpurun_out/ab_$n.log 2>&1 || return 1
  python3 - "$n" <<'PY'
import json,sys; n=sys.argv[1]
l=[x for x in open("gpurun_out/ab_%s.log" % n) if x.startswith("{")][0]; j=json.loads(l)
print(n, round(j["value"]/1e6,2), j["roofline"]["avg_launch_us"], round(j["detail"]["large_batch"]["value"]/1e6,2), j["detail"]["large_batch"]["ms_per_epoch"])
PY
}
run new SKGE_PIPE_E8=1 SKGE_PIPE_OWNMARK=1 || exit 1
run old SKGE_PIPE_E8=0 SKGE_PIPE_OWNMARK=0 || exit 1
run new2 SKGE_PIPE_E8=1 SKGE_PIPE_OWNMARK=1 || exit 1
run old2 SKGE_PIPE_E8=0 SKGE_PIPE_OWNMARK=0 || exit 1
