"""bench.py's traffic lookup (host logic, no GPU): the per-launch PMC traffic a
line quotes comes from the newest committed round, and for config 5 from the
same epochs the line times (tools/pmc_epochs.py's per-epoch summary)."""
import json
import os

import bench


def _write(root, rnd, name, data):
    d = os.path.join(root, "profiles", rnd)
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, name), "w") as f:
        json.dump(data, f)


def test_pmc_traffic_epochs_picks_timed_epochs_of_newest_round(tmp_path, monkeypatch):
    root = str(tmp_path)
    monkeypatch.setattr(bench, "ROOT", root)
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
    _write(root, "r05", "pmc.json", {"k_pipe_batch": {
        "traffic_bytes_per_launch": 1.0,
        "by_grid": {"453888": {"calls": 4257, "traffic_bytes_per_launch": 14.9e6},
                    "4478464": {"calls": 41, "traffic_bytes_per_launch": 4.6e8}}}})
    t, src = bench.pmc_traffic("k_pipe_batch", "pmc.json")
    assert t == 14.9e6 and src == os.path.join("profiles", "r05", "pmc.json")
