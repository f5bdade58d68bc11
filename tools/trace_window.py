"""Per-step kernel time of the last K steps in a rocprofv3 kernel trace.

usage: trace_window.py TRACE_CSV MARKER K [timeline] [--between]
The timed window starts at the K-th last dispatch whose name contains MARKER (the first kernel of
a step, e.g. ns_batch_kernel) and ends with the last dispatch; --between: the K whole steps from
the (K+1)-th last marker up to the last one (excludes the last step's tail and whatever the
program launches after its timed steps). Prints per-kernel device time per
step, the summed busy time per step and the window's wall time per step (gaps included)."""
import csv
import sys
from collections import defaultdict


def main():
    between = "--between" in sys.argv
    argv = [a for a in sys.argv if a != "--between"]
    path, marker, k = argv[1], argv[2], int(argv[3])
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    if len(starts) < k + (1 if between else 0):
        raise SystemExit(f"only {len(starts)} '{marker}' dispatches")
    win = rows[starts[-k - 1]:starts[-1]] if between else rows[starts[-k]:]
    tot, cnt = defaultdict(float), defaultdict(int)
    for r in win:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        name = r["Kernel_Name"]
        tot[name] += d
        cnt[name] += 1
    busy = sum(tot.values()) / k
    wall = ((int(rows[starts[-1]]["Start_Timestamp"]) if between else int(win[-1]["End_Timestamp"]))
            - int(win[0]["Start_Timestamp"])) / 1e3 / k
    print(f"window: {k} steps, {len(win)} dispatches ({len(win) / k:.1f}/step), "
          f"busy {busy:.1f} us/step, wall {wall:.1f} us/step")
    for name, t in sorted(tot.items(), key=lambda x: -x[1]):
        print(f"{t / k:9.1f} us  x{cnt[name] / k:5.2f}  {name[:140]}")
    if len(argv) > 4:
        # one step's timeline (the second-last step of the window): start / end relative to its
        # first dispatch, and the gap since the latest end before it (queue idle if positive)
        step = rows[starts[-2]:starts[-1]]
        t0 = int(step[0]["Start_Timestamp"])
        last_end = t0
        print("\ntimeline of one step (us): start  end  dur  gap  queue  kernel")
        for r in step:
            s0, e0 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            q = r.get("Queue_Id", r.get("Stream_Id", "?"))
            print(f"{(s0 - t0) / 1e3:8.1f} {(e0 - t0) / 1e3:8.1f} {(e0 - s0) / 1e3:6.1f} "
                  f"{(s0 - last_end) / 1e3:6.1f}  {q:>3}  {r['Kernel_Name'][:70]}")
            last_end = max(last_end, e0)


if __name__ == "__main__":
    main()
