"""Loader for the committed golden fixtures (tests/golden/*.npz, made by make_golden.py)."""
import glob
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def names(prefix=""):
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, prefix + "*.npz")))


def load(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        d = {k: z[k] for k in z.files}
    d["meta"] = json.loads(str(d["meta"]))
    return d


def sub(d, prefix, dtype=np.float64):
    return {k[len(prefix):]: (v.astype(dtype) if v.dtype.kind == "f" else v)
            for k, v in d.items() if k.startswith(prefix)}


def close(a, b, tol):
    """max |a-b| <= tol * max(1, max|b|)  (relative to the tensor's scale)."""
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    scale = max(1.0, float(np.abs(b).max()) if b.size else 1.0)
    err = float(np.abs(a - b).max()) if b.size else 0.0
    return err <= tol * scale, err / scale
