"""Load golden fixtures (tests/golden/*.npz, made by tools/gen_golden.py)."""
import glob
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def case_names(prefix=""):
    out = []
    for p in sorted(glob.glob(os.path.join(GOLDEN, prefix + "*.npz"))):
        n = os.path.basename(p)[:-4]
        if n != "init_quirks" and not n.startswith(("eval_", "ckpt_")):   # own tests
            out.append(n)
    return out


class Case:
    def __init__(self, name):
        self.name = name
        z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
        self.z = {k: z[k] for k in z.files}
        g = self.z
        self.model = str(g["meta_model"])
        self.mode = str(g["meta_mode"])
        self.opt = str(g["meta_opt"])
        self.d = int(g["d"])
        self.n_ent = int(g["n_ent"])
        self.n_rel = int(g["n_rel"])
        self.lr = float(g["lr"])
        self.margin = float(g["margin"])
        self.l1 = bool(int(g["l1"]))
        self.rparam = float(g["rparam"])
        self.nbatch = int(g["nbatch"])
        self.param_ids = [str(x) for x in g["param_ids"]]
        self.last_update = int(g["last_update_batch"])
        self.hi = self.z["init_" + self.param_ids[0]].dtype == np.float32 and \
            any(v.dtype == np.float64 and v.ndim >= 2 for k, v in self.z.items() if "_after_" in k)

    def init_params(self, dtype=np.float64):
        return {pid: self.z["init_" + pid].astype(dtype) for pid in self.param_ids}

    def has(self, key):
        return key in self.z

    def __getitem__(self, k):
        return self.z[k]

    def batch(self, b):
        pre = "b%d_" % b
        out = {k[len(pre):]: v for k, v in self.z.items() if k.startswith(pre)}
        return out


def tol_for(arr):
    """Fixtures keep float64 outputs for d=8 cases and float32 for larger d."""
    return (1e-9, 1e-10) if arr.dtype == np.float64 else (2e-6, 2e-6)
