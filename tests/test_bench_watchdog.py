"""bench.run_with_watchdog (CPU): the guard around every multi-rank
measurement of bench.py -- a measurement that does not return prints rank 0's
line once, the failure marked in it, and ends the process with a NON-zero
status (bench.WATCHDOG_EXIT: a hung collective must not look like a
successful run); an exception becomes an error entry (the caller then exits
non-zero too); a normal return passes through."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import os, sys, time
sys.path.insert(0, %r)
import bench
line = {"value": 1.0, "detail": {}}
mode = sys.argv[1]
if mode == "hang":
    out = bench.run_with_watchdog(lambda: time.sleep(30), line, 0.3, key="details")
elif mode == "hang_main":
    out = bench.run_with_watchdog(lambda: time.sleep(30), line, 0.3)
elif mode == "raise":
    out = bench.run_with_watchdog(lambda: 1 / 0, line, 5.0, key="details")
else:
    out = bench.run_with_watchdog(lambda: {"ok": 1}, line, 5.0, key="details")
if bench.failed(out):
    bench.mark_failure(line, "details", out["error"])
else:
    line["detail"]["details"] = out
print(bench.json.dumps(line), flush=True)
if bench.failed(out):
    os._exit(bench.WATCHDOG_EXIT)
""" % ROOT


def _run(mode):
    p = subprocess.run([sys.executable, "-c", SCRIPT, mode], capture_output=True, text=True,
                       timeout=120)
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    return p.returncode, [json.loads(x) for x in lines]


def test_watchdog_prints_once_and_exits_nonzero_on_a_hang():
    sys.path.insert(0, ROOT)
    import bench
    rc, lines = _run("hang")
    assert rc == bench.WATCHDOG_EXIT != 0 and len(lines) == 1
    assert "not measured" in lines[0]["detail"]["details"]["error"]
    assert lines[0]["value"] == 1.0          # a detail's failure keeps the measured value


def test_watchdog_on_the_main_measurement_nulls_the_value():
    sys.path.insert(0, ROOT)
    import bench
    rc, lines = _run("hang_main")
    assert rc == bench.WATCHDOG_EXIT and len(lines) == 1
    assert lines[0]["value"] is None and "not measured" in lines[0]["error"]


def test_watchdog_passes_results_through_and_errors_exit_nonzero():
    rc, lines = _run("ok")
    assert rc == 0 and len(lines) == 1 and lines[0]["detail"]["details"] == {"ok": 1}
    rc, lines = _run("raise")
    assert rc != 0 and len(lines) == 1
    assert lines[0]["detail"]["details"]["error"].startswith("ZeroDivisionError")
