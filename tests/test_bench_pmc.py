"""bench.py's traffic lookup (host logic, no GPU): the per-launch PMC traffic a
line quotes comes from the SAME round's committed summary (bench.PMC_ROUND;
an older round's is never quoted), and for config 5 from the same epochs the
line times (tools/pmc_epochs.py's per-epoch summary)."""
import json
import os

import bench


def _write(root, rnd, name, data):
    d = os.path.join(root, "profiles", rnd)
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, name), "w") as f:
        json.dump(data, f)


def test_pmc_traffic_epochs_picks_timed_epochs_of_this_round(tmp_path, monkeypatch):
    root = str(tmp_path)
    monkeypatch.setattr(bench, "ROOT", root)
    monkeypatch.setattr(bench, "PMC_ROUND", "r05")
    eps = lambda base: [{"epoch": e, "traffic_bytes_per_launch": base + e} for e in range(4)]
    _write(root, "r04", "pmc_c5_epochs.json", {"k_apply": eps(100)})
    _write(root, "r05", "pmc_c5_epochs.json", {"k_apply": eps(200), "k_other": eps(0)})
    t, src = bench.pmc_traffic_epochs("k_apply", "pmc_c5_epochs.json", 1, 2)
    assert t == (201 + 202) / 2
    assert src.startswith(os.path.join("profiles", "r05")) and src.endswith("epochs 1..2")
    # epochs the summary does not hold -> no number (the caller falls back)
    assert bench.pmc_traffic_epochs("k_apply", "pmc_c5_epochs.json", 3, 2) == (None, None)


def test_pmc_traffic_uses_most_launched_grid(tmp_path, monkeypatch):
    root = str(tmp_path)
    monkeypatch.setattr(bench, "ROOT", root)
    monkeypatch.setattr(bench, "PMC_ROUND", "r05")
    _write(root, "r05", "pmc.json", {"k_pipe_batch": {
        "traffic_bytes_per_launch": 1.0,
        "by_grid": {"453888": {"calls": 4257, "traffic_bytes_per_launch": 14.9e6},
                    "4478464": {"calls": 41, "traffic_bytes_per_launch": 4.6e8}}}})
    t, src = bench.pmc_traffic("k_pipe_batch", "pmc.json")
    assert t == 14.9e6 and src == os.path.join("profiles", "r05", "pmc.json")


def test_pmc_traffic_never_quotes_an_older_round(tmp_path, monkeypatch):
    """A config whose PMC pass this round has not committed gets traffic null,
    not the previous round's number (round 5's config 1, 3 and 4 lines quoted
    r04 summaries)."""
    root = str(tmp_path)
    monkeypatch.setattr(bench, "ROOT", root)
    monkeypatch.setattr(bench, "PMC_ROUND", "r06")
    _write(root, "r05", "pmc_c1.json", {"k_pipe_fused": {"traffic_bytes_per_launch": 9.8e6}})
    assert bench.pmc_traffic("k_pipe_fused", "pmc_c1.json") == (None, None)
    _write(root, "r06", "pmc_c1.json", {"k_pipe_fused": {"traffic_bytes_per_launch": 5.0e6}})
    t, src = bench.pmc_traffic("k_pipe_fused", "pmc_c1.json")
    assert t == 5.0e6 and src == os.path.join("profiles", "r06", "pmc_c1.json")


def test_pmc_round_is_the_current_round():
    """bench.PMC_ROUND names the newest round directory under profiles/ (or
    the one this round is filling)."""
    rounds = sorted(d for d in os.listdir(os.path.join(bench.ROOT, "profiles"))
                    if d.startswith("r") and d[1:].isdigit())
    assert rounds and bench.PMC_ROUND >= rounds[-1]
