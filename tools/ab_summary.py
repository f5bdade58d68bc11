"""Median / min per variant of tools/ab_steps.sh or ab_env.sh output lines ("[ENV ...] X us ...").
usage: python tools/ab_summary.py LOG"""
import collections
import statistics
import sys

d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    if not line.startswith("[") or line.startswith("[gpurun") or "] " not in line:
        continue
    key, rest = line[1:].split("] ", 1)
    try:
        d[key].append(float(rest.split()[0]))
    except ValueError:
        continue
for k, v in d.items():
    print(f"{k:60s} median {statistics.median(v):6.1f} min {min(v):6.1f} n {len(v)} {v}")
