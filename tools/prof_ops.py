"""torch.profiler view of the bench step (which aten / HIP ops take device time, with input shapes):
    python tools/prof_ops.py [--dtype bf16] [--scale 10]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "re-gnn_amd"))
import torch  # noqa: E402
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--dtype", default="fp32")
ap.add_argument("--scale", type=float, default=10.0)
a = ap.parse_args()
args = argparse.Namespace(gpus=1, steps=2, warmup=2, workload="mag", scale=a.scale, batch=512,
                          dropout=0.5, graph="off", dtype=a.dtype, no_cpu_baseline=True)
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
w = bench.build_workload(args, dev)
for _ in range(2):
    w["step"]()
torch.cuda.synchronize()
acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
with torch.profiler.profile(activities=acts, record_shapes=True) as prof:
    w["step"]()
    torch.cuda.synchronize()
print(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=40,
                                                         max_name_column_width=60))
