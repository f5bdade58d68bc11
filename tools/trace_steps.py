"""Per-step timeline of the last run in a rocprofv3 kernel trace (NS step, groups of replays).

usage: trace_steps.py TRACE_CSV FIRST_MARKER LAST_MARKER N
Takes the last N model steps (a step starts at a dispatch whose name contains FIRST_MARKER and
ends at the next LAST_MARKER dispatch) and prints per step: its start relative to the window,
its model span (first start -> last end), the gap since the previous step's end, and every
other-queue (sampler) dispatch that overlaps the step; then the tail after the last step's end.
"""
import csv
import sys


def short(n):
    n = n.split("(")[0].split("<")[0]
    return n.replace("_kernel", "")[:22]


def main():
    path, first, last, n = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]) / 1e3, int(r["End_Timestamp"]) / 1e3
        r["q"] = r.get("Queue_Id", r.get("Stream_Id", "?"))
    starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
    starts = starts[-n:]
    mq = rows[starts[0]]["q"]
    t0 = rows[starts[0]]["s"]
    prev_end = None
    for j, i in enumerate(starts):
        k = i
        while k < len(rows) and last not in rows[k]["Kernel_Name"]:
            k += 1
        s, e = rows[i]["s"], rows[min(k, len(rows) - 1)]["e"]
        nxt = rows[starts[j + 1]]["s"] if j + 1 < len(starts) else e + 400
        side = [r for r in rows if r["q"] != mq and r["e"] > s and r["s"] < nxt]
        gap = "" if prev_end is None else f"{s - prev_end:6.1f}"
        print(f"step {j:3d} start {s - t0:9.1f} span {e - s:6.1f} gap {gap:>6}  side: " +
              " ".join(f"{short(r['Kernel_Name'])}[{r['s'] - s:.0f},{r['e'] - s:.0f}]" for r in side))
        prev_end = e
    tail = [r for r in rows if r["s"] >= prev_end - 1e-3][:12]
    print("after the last step:", " ".join(f"{short(r['Kernel_Name'])}@{r['s'] - prev_end:.0f}"
                                           f"+{r['e'] - r['s']:.0f}" for r in tail))


if __name__ == "__main__":
    main()
