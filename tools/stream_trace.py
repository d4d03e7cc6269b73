"""The streamed leg (configs[4]) of a rocprofv3 kernel trace of bench.py: the window from the first to
the last lean graph build (graph_build_kernel under 30 us), GPU busy fraction (union of kernel intervals),
the largest idle gaps, per-kernel totals and the lean build's duration.
Usage: python tools/stream_trace.py run_kernel_trace.csv"""
import collections
import csv
import re
import sys

rows = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']),
               re.sub(r'\(.*', '', r['Kernel_Name']).replace('void ', '').replace('wd::', '')[:44])
              for r in csv.DictReader(open(sys.argv[1])))
lean = [r for r in rows if r[2].startswith('graph_build_kernel') and r[1] - r[0] < 30000]
t0, t1 = lean[0][0], lean[-1][1]
win = [r for r in rows if r[0] >= t0 and r[1] <= t1]
busy, gaps, end = 0, [], t0
for s, e, _ in win:
    if s > end:
        gaps.append(s - end)
    busy += max(0, e - max(s, end))
    end = max(end, e)
tot = collections.defaultdict(lambda: [0, 0])
for s, e, n in win:
    tot[n][0] += 1
    tot[n][1] += e - s
span = t1 - t0
print(f'streamed leg: {span / 1e3:.1f} us, GPU busy {busy / 1e3:.1f} us ({busy / span:.2f}), {len(gaps)} idle gaps, '
      f'largest {sorted(gaps)[-5:] and [round(g / 1e3, 1) for g in sorted(gaps)[-5:]]} us, '
      f'median gap {sorted(gaps)[len(gaps) // 2] / 1e3 if gaps else 0:.2f} us')
print(f'lean graph builds: {len(lean)}, median {sorted(r[1] - r[0] for r in lean)[len(lean) // 2] / 1e3:.1f} us')
for n, (c, t) in sorted(tot.items(), key=lambda x: -x[1][1]):
    print(f'  {n:44s} {c:6d} x {t / c / 1e3:7.2f} us = {t / 1e3:9.1f} us')
