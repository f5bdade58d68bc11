"""Temporary: per-phase wall clocks of the fused NS step's head / agg0 kernels (instrumented
build), one eager step at the bench configuration."""
import argparse, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench

dev = torch.device("cuda:0")
dbg = torch.zeros(2048 * 16, dtype=torch.int64, device=dev)
os.environ["REGNN_NSM_DBG_PTR"] = str(dbg.data_ptr())
args = argparse.Namespace(scale=10, zipf=1.1, hidden=64, dropout=0.5, batch=512, gpus=1)
tr, info = bench.build_ns(args, dev)
for _ in range(3):
    tr.step()
torch.cuda.synchronize()
d = dbg.view(-1, 16).cpu().long()
rate = 100.0  # MHz steady counter
def show(name, rows, nph):
    r = d[rows][:, :nph]
    r = r[r[:, 0] > 0]
    t0 = r[:, 0].min()
    print(f"{name}: {len(r)} blocks, span {(r[:, nph-1].max() - t0).item() / rate:.2f} us")
    print("  block start spread (us):", ((r[:, 0] - t0).float() / rate).quantile(torch.tensor([0., .5, .9, 1.])).tolist())
    for i in range(1, nph):
        dd = (r[:, i] - r[:, i - 1]).float() / rate
        print(f"  phase {i-1}->{i}: mean {dd.mean():.2f} us, max {dd.max():.2f}")

show("agg0", slice(100, 100 + 832), 7)
