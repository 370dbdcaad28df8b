#!/usr/bin/env python3
"""The concurrent rest-of-round launches (fwh_update_kernel<true, 4>, one per update stream) in a
rocprofv3 kernel trace: per-launch durations, the span of each pair, and the period per pair over
a build, (last end - first start) / pairs, which is the unit bench.py times with HIP events on
one GPU (dist_enc 5). Builds are separated by gaps longer than 10 ms.
usage: tools/pair_spans.py <run_kernel_trace.csv> [kernel-substring]"""
import csv
import sys

path = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else "fwh_update_kernel<true, 4>"
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(path))
             if sub in r["Kernel_Name"]))
spans = [max(a[1], b[1]) - min(a[0], b[0]) for a, b in zip(ks[0::2], ks[1::2])]
per = [b - a for a, b in ks]
print(f"launches {len(ks)}  pairs {len(spans)}")
print(f"per-launch average {sum(per) / len(per) / 1e6:.4f} ms")
print(f"pair span average  {sum(spans) / len(spans) / 1e6:.4f} ms  (min {min(spans) / 1e6:.4f}, "
      f"max {max(spans) / 1e6:.4f})")
builds, cur = [], [ks[0]]
for a, b in zip(ks, ks[1:]):
    if b[0] - a[1] > 10_000_000:
        builds.append(cur)
        cur = []
    cur.append(b)
builds.append(cur)
per_build = [((max(x[1] for x in bl) - min(x[0] for x in bl)) / (len(bl) // 2)) / 1e6 for bl in builds]
print("period per pair, per build: " + ", ".join(f"{v:.4f}" for v in per_build) + " ms")
print(f"start offset within a pair, average {sum(abs(a[0] - b[0]) for a, b in zip(ks[0::2], ks[1::2])) / len(spans) / 1e3:.1f} us")
