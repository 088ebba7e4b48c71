"""bench.run_with_watchdog (CPU): the guard around the N > 1 one-model DP
detail -- a detail that does not return prints rank 0's already built line
once, marked, and ends the process with status 0; an exception becomes an
error entry; a normal return passes through."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import sys, time
sys.path.insert(0, %r)
import bench
line = {"value": 1.0, "detail": {"one_model_dp": None}}
mode = sys.argv[1]
if mode == "hang":
    out = bench.run_with_watchdog(lambda: time.sleep(30), line, 0.3)
elif mode == "raise":
    out = bench.run_with_watchdog(lambda: 1 / 0, line, 5.0)
else:
    out = bench.run_with_watchdog(lambda: {"ok": 1}, line, 5.0)
line["detail"]["one_model_dp"] = out
print(bench.json.dumps(line), flush=True)
""" % ROOT


def _run(mode):
    p = subprocess.run([sys.executable, "-c", SCRIPT, mode], capture_output=True, text=True,
                       timeout=120)
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    return p.returncode, [json.loads(x) for x in lines]


def test_watchdog_prints_once_and_exits_zero_on_a_hang():
    rc, lines = _run("hang")
    assert rc == 0 and len(lines) == 1
    assert "not measured" in lines[0]["detail"]["one_model_dp"]["error"]


def test_watchdog_passes_results_and_errors_through():
    rc, lines = _run("ok")
    assert rc == 0 and len(lines) == 1 and lines[0]["detail"]["one_model_dp"] == {"ok": 1}
    rc, lines = _run("raise")
    assert rc == 0 and len(lines) == 1
    assert lines[0]["detail"]["one_model_dp"]["error"].startswith("ZeroDivisionError")
