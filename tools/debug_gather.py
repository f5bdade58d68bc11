"""Which gather-kernel slab entries differ between two identical fused steps (GPU box)."""
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
    from regnn_hip.ns import NSTrainer
    d = _mag(0.002, seed=8, F=128, hidden=64, classes=13, dropout=0.4)
    C = 13
    hw = (C * 65 + 3 * 64 + 1 + 64 * 64 + 3) & ~3
    outs = []
    for rep in range(6):
        tr = NSTrainer(d["model"](5), None, d["rg"], [6, 4], 100,
                       torch.arange(d["n_paper"], device="cuda"), d["x_dict"], d["edge_type"],
                       d["node_type"], d["local"], d["y"], 7, seed=9, adam=dict(lr=1e-2),
                       pipeline=False)
        tr._forward_backward()
        torch.cuda.synchronize()
        fs = tr.fused
        head_blocks = (tr.sampler.caps[0] + 15) // 16
        g = fs.slab[head_blocks * hw: head_blocks * hw + 512 * 256].view(512, 256).clone()
        s = tr.sampler
        outs.append((g, s.csc[0][1].clone(), s.csc[0][3].clone(), int(s.sizes[1]),
                     tr.model.convs[1].relation_weight.grad.clone()))
    g0 = outs[0]
    for k, o in enumerate(outs[1:], 1):
        print(f"rep {k}: n1 {o[3]} vs {g0[3]}, csc_ptr equal {torch.equal(o[1], g0[1])}, "
              f"long list equal {torch.equal(o[2], g0[2])}, n_long {int(o[2][0])}")
        dd = (o[0] != g0[0]).nonzero().tolist()
        print(f"   slab entries differing: {len(dd)}: {dd[:12]}")
        print(f"   rel1 grad diff: {(o[4] - g0[4]).abs().max().item():.3e}")
        for b, col in dd[:6]:
            print(f"     block {b} col {col}: {g0[0][b, col].item()!r} vs {o[0][b, col].item()!r}")


if __name__ == "__main__":
    main()
