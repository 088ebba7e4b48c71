import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "scikit-kge_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: longer CPU test")


def pytest_sessionfinish(session, exitstatus):
    """Write the parity headroom records of this session (tests/parity_util.py)
    to gpurun_out/parity_headroom.json: per check, tol / max|err| (>= 1 passes)."""
    try:
        import parity_util
    except Exception:
        return
    if not parity_util.RECORDS:
        return
    import json
    recs = sorted(parity_util.RECORDS, key=lambda r: r[1])
    out = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "parity_headroom.json"), "w") as f:
        json.dump({"checks": len(recs),
                   "min_headroom": recs[0][1] if recs else None,
                   "worst": [{"what": w, "headroom": h, "max_abs_err": e, "n": n}
                             for w, h, e, n in recs[:40]],
                   "all": [[w, h, e, n] for w, h, e, n in recs],
                   # check_step: rows that needed the sign-flip allowance
                   "flip_rows": [[w, k, n, a] for w, k, n, a in parity_util.FLIPS]},
                  f, indent=1, default=lambda x: str(x))
