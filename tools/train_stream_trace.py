"""Resident against streamed training steps in a rocprofv3 kernel trace of tools/train_stream_host.py:
step period (adam_kernel to adam_kernel), per-kernel median durations in each phase, and the feed's
graph builds.  Phases split at the largest gap between Adam steps (the feed's start-up).
Usage: python tools/train_stream_trace.py run_kernel_trace.csv"""
import collections
import csv
import re
import statistics
import sys

rows = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']),
               re.sub(r'\(.*', '', r['Kernel_Name']).replace('void ', '').replace('wd::', '')[:44])
              for r in csv.DictReader(open(sys.argv[1])))
adam = [r for r in rows if r[2].startswith('adam_kernel')]
gaps = [(adam[i + 1][0] - adam[i][0], i) for i in range(len(adam) - 1)]
cut = max(gaps)[1]  # the resident phase ends at adam[cut]; warm-up of the feed follows
phases = {'resident': (adam[max(0, cut - 300)][0], adam[cut][1]), 'streamed': (adam[-300][0], adam[-1][1])}
for name, (t0, t1) in phases.items():
    a = [r for r in adam if t0 <= r[0] <= t1]
    per = [(a[i + 1][0] - a[i][0]) / 1e3 for i in range(len(a) - 1)]
    win = [r for r in rows if t0 <= r[0] and r[1] <= t1]
    d = collections.defaultdict(list)
    for s, e, n in win:
        d[n].append((e - s) / 1e3)
    busy, end = 0, t0
    for s, e, _ in win:
        busy += max(0, e - max(s, end))
        end = max(end, e)
    print(f'{name}: {len(per)} steps, median period {statistics.median(per):.1f} us, GPU busy {busy / (t1 - t0):.2f}')
    for n, v in sorted(d.items(), key=lambda x: -sum(x[1])):
        print(f'   {n:44s} {len(v):6d} x median {statistics.median(v):7.2f} us (sum per step {sum(v) / max(1, len(per)):7.2f})')
