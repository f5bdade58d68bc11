"""Average idle gap before each model kernel on its queue in a rocprofv3 kernel trace.

usage: trace_gaps.py TRACE_CSV MARKER N
Over the last N steps (a step starts at a dispatch containing MARKER), on MARKER's queue: for each
kernel name, the median gap between the previous kernel's end on that queue and its start, the
mean duration, and the mean step period."""
import csv
import sys
import statistics
from collections import defaultdict


def main():
    path, marker, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]][-n:]
    q = rows[starts[0]]["Queue_Id"]
    win = [r for r in rows[starts[0]:] if r["Queue_Id"] == q]
    gap, dur, cnt = defaultdict(list), defaultdict(float), defaultdict(int)
    prev = None
    for r in win:
        s, e = int(r["Start_Timestamp"]) / 1e3, int(r["End_Timestamp"]) / 1e3
        name = r["Kernel_Name"].split("(")[0][-40:]
        if prev is not None:
            gap[name].append(s - prev)
        dur[name] += e - s
        cnt[name] += 1
        prev = e
    period = (int(rows[starts[-1]]["Start_Timestamp"]) - int(rows[starts[0]]["Start_Timestamp"])) \
        / 1e3 / max(1, n - 1)
    print(f"queue {q}: {len(win)} dispatches over {n} steps, period {period:.1f} us/step")
    for k in dur:
        med = statistics.median(gap[k]) if gap[k] else 0.0
        print(f"  {k:42s} x{cnt[k] / n:4.2f}  gap before (median) {med:6.2f} us  "
              f"dur {dur[k] / cnt[k]:6.2f} us")


if __name__ == "__main__":
    main()
