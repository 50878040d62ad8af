#!/usr/bin/env python3
"""tools/timeline.py — per-step kernel timeline of bench.py from a rocprofv3 kernel trace.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl -o tl -- \\
        python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-c3 --no-c4
    python3 tools/timeline.py gpurun_out/tl          # (any directory holding *kernel_trace.csv)

Steps are cut at each sketch_tiles launch; for one step (the median by span) prints every
kernel's start offset, duration and the idle gap before it on its queue, and the step's
busy / idle split (union of kernel intervals over all queues).
"""
import csv
import glob
import os
import sys


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").replace("fpm::", "")[:40]


def main():
    d = sys.argv[1]
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         r.get("Queue_Id", r.get("Stream_Id", "?"))))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if "sketch_tiles_kernel" in r[2]]
    steps = []
    for a, b in zip(starts, starts[1:]):
        steps.append(rows[a:b])
    if not steps:
        print("no steps found")
        return
    spans = sorted(range(len(steps)), key=lambda i: steps[i][-1][1] - steps[i][0][0])
    s = steps[spans[len(spans) // 2]]
    t0 = s[0][0]
    last_end = {}
    print(f"{len(steps)} steps; median step: {len(s)} launches")
    for st, en, nm, q in s:
        gap = st - last_end.get(q, st)
        last_end[q] = en
        print(f"  q{q:>3} +{(st - t0) / 1e3:8.1f} us  {(en - st) / 1e3:8.1f} us  gap {gap / 1e3:6.1f}  {short(nm)}")
    iv = sorted((st, en) for st, en, _, _ in s)
    busy, cur_s, cur_e = 0, iv[0][0], iv[0][1]
    for st, en in iv[1:]:
        if st > cur_e:
            busy += cur_e - cur_s
            cur_s, cur_e = st, en
        else:
            cur_e = max(cur_e, en)
    busy += cur_e - cur_s
    span = s[-1][1] - t0
    print(f"span {span / 1e3:.1f} us (to the last kernel's end), busy {busy / 1e3:.1f} us, "
          f"idle {(span - busy) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
