"""Diagnose RESCAL step mismatches vs the oracle (prints offending elements)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "scikit-kge_amd"), os.path.join(ROOT, "tests")]
import numpy as np
import torch
from oracle import skge_oracle as O
from test_gpu_models import _batch, _model


def main():
    n_ent, n_rel, d, P = 400, 18, 200, 700
    m, upd = _model("rescal", n_ent, n_rel, d)
    params = {pid: p.data.cpu().numpy().astype(np.float64) for pid, p in m.params.items()}
    state = {pid: np.zeros_like(v) for pid, v in params.items()}
    rs = np.random.RandomState(5)
    nviol = torch.zeros(1, dtype=torch.int32, device=m.device)
    for b in range(2):
        pos, neg = _batch(rs, n_ent, n_rel, P)
        pre = {k: v.copy() for k, v in params.items()}
        nviol.zero_()
        m._pairwise_step(torch.as_tensor(pos, device=m.device), torch.as_tensor(neg, device=m.device), upd, nviol)
        ps, ns, nv, g = O.pairwise_step("rescal", params, state, pos, neg, 0.1, 0.2, "adagrad", rparam=0.0)
        E = m.params["E"].data.cpu().numpy()
        diff = np.abs(E - params["E"])
        bad = np.argwhere(diff > 1e-5 + 1e-5 * np.abs(params["E"]))
        print("batch", b, "nviol", int(nviol.item()), nv, "bad", len(bad), "max", diff.max())
        rows = sorted(set(bad[:, 0].tolist()))
        print(" bad rows", rows[:20])
        ge, gi = g["E"]
        for r in rows[:5]:
            k = int(np.where(gi == r)[0][0]) if r in gi else -1
            cols = bad[bad[:, 0] == r][:, 1]
            print("  row", r, "ncols", len(cols), "in pos s/o", int((pos[:, 0] == r).sum()), int((pos[:, 1] == r).sum()),
                  "neg s/o", int((neg[:, 0] == r).sum()), int((neg[:, 1] == r).sum()))
            for c in cols[:4]:
                print("    col", c, "got", E[r, c], "want", params["E"][r, c], "pre", pre["E"][r, c],
                      "g", ge[k, c] if k >= 0 else None, "p2", state["E"][r, c])
        # scores comparison
        sc_p = m._pscore.cpu().numpy() if getattr(m, "_pscore", None) is not None else None


if __name__ == "__main__":
    main()
