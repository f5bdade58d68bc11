"""Determinism probe of the NS trainer (GPU box): the same training run twice from scratch --
eager steps and graph replays -- and the first parameter elements / gradients that differ."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "re-gnn_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)


def main():
    from test_gpu_ns_engine import _mag
    from regnn_hip import ns
    from regnn_hip.ns import NSTrainer
    d = _mag(0.002, seed=8, F=128, hidden=64, classes=13, dropout=0.4)

    def make(**kw):
        return NSTrainer(d["model"](5), None, d["rg"], [6, 4], 100,
                         torch.arange(d["n_paper"], device="cuda"), d["x_dict"], d["edge_type"],
                         d["node_type"], d["local"], d["y"], 7, seed=9, adam=dict(lr=1e-2), **kw)

    def names(tr):
        out, o = [], 0
        for n, p in tr.model.named_parameters():
            out.append((n, o, o + p.numel()))
            o += p.numel()
        return out

    def diff(tag, a, b, tr):
        if torch.equal(a, b):
            print(f"{tag}: bitwise equal")
            return
        dd = (a - b).abs()
        idx = torch.nonzero(dd).flatten().cpu().tolist()
        print(f"{tag}: {len(idx)} elements differ, max {dd.max().item():.3e}")
        for n, lo, hi in names(tr):
            k = [i for i in idx if lo <= i < hi]
            if k:
                print(f"   {n}: {len(k)} of {hi - lo}")

    for pipe in (False, True):
        for mode in ("eager", "graph"):
            runs = []
            for _ in range(2):
                tr = make(pipeline=pipe)
                g = []
                if mode == "graph":
                    tr.capture(warmup=1)
                for i in range(4):
                    (tr.replay if mode == "graph" else tr.step)()
                    torch.cuda.synchronize()
                    g.append((tr.flat.clone(), tr.pflat.clone(), float(tr.loss)))
                runs.append((tr, g))
            (ta, ga), (tb, gb) = runs
            for i in range(4):
                print(f"pipeline={pipe} {mode} step {i}: loss {ga[i][2]!r} {gb[i][2]!r}")
                diff("  grad", ga[i][0], gb[i][0], ta)
                diff("  param", ga[i][1], gb[i][1], ta)


if __name__ == "__main__":
    main()
