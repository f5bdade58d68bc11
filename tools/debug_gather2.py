"""Which intermediate of the two-layer fused step differs between identical runs (GPU box):
GH (head output), h0 / a0 / stats (agg0), the transposed index (per segment, sorted), G0 and
the gather slab's relation dots."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "re-gnn_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)


def main():
    from test_gpu_ns_engine import _mag
    from regnn_hip.ns import NSTrainer
    d = _mag(0.002, seed=8, F=128, hidden=64, classes=13, dropout=0.4)
    outs = []
    for rep in range(24):
        tr = NSTrainer(d["model"](5), None, d["rg"], [6, 4], 100,
                       torch.arange(d["n_paper"], device="cuda"), d["x_dict"], d["edge_type"],
                       d["node_type"], d["local"], d["y"], 7, seed=9, adam=dict(lr=1e-2),
                       pipeline=False)
        tr._forward_backward()
        torch.cuda.synchronize()
        fs = tr.fused
        by = {t.data_ptr(): t for t in fs.keep if torch.is_tensor(t)}
        W = fs.W
        s = tr.sampler
        n0, n1 = int(s.sizes[0]), int(s.sizes[1])
        cnt, cptr, cent, clong = s.csc[0]
        segs = []
        cp = cptr[:n1 + 1].cpu().tolist()
        ce = cent.cpu()
        for u in range(n1):
            segs.append(sorted(ce[cp[u]:cp[u + 1]].tolist()))
        o = {"GH": by[W.gh1][:n0].clone(), "h0": by[W.xs[1]][:n1].clone(),
             "a0": by[W.a[0]][:n1].clone(), "st0": by[W.stats[0]][:n1].clone(),
             "G0": by[W.ga[0]][:n1].clone(), "segs": segs,
             "blk_idx": s.blocks[0].csr_idx.clone(), "blk_row": s.blocks[0].row.clone(),
             "blk_rel": s.blocks[0].rel.clone(), "rg": tr.model.convs[1].relation_weight.grad.clone(),
             "slab": fs.slab.clone()}
        outs.append(o)
    a = outs[0]
    for k, b in enumerate(outs[1:], 1):
        msg = []
        for key in ("GH", "h0", "a0", "st0", "G0", "blk_idx", "blk_row", "blk_rel", "rg", "slab"):
            if not torch.equal(a[key], b[key]):
                dd = (a[key].double() - b[key].double()).abs()
                nz = torch.nonzero(dd)
                msg.append(f"{key}: {nz.shape[0]} differ (max {dd.max().item():.3e}) first {nz[:4].tolist()}")
        if a["segs"] != b["segs"]:
            bad = [u for u in range(len(a["segs"])) if a["segs"][u] != b["segs"][u]]
            msg.append(f"csc segments differ at rows {bad[:8]}: {a['segs'][bad[0]][:10]} vs {b['segs'][bad[0]][:10]}")
        print(f"rep {k}: " + ("; ".join(msg) if msg else "all equal"))


if __name__ == "__main__":
    main()
