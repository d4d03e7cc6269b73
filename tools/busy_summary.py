"""GPU busy / idle over the last part of a rocprofv3 kernel trace (any kernels, any streams): union of the
kernel intervals vs the wall span, the largest idle gaps, and per-kernel totals.
Usage: python tools/busy_summary.py run_kernel_trace.csv [fraction of the trace at the end, default 0.5]"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
iv = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']),
             re.sub(r'\(.*', '', r['Kernel_Name']).replace('void ', '').replace('wd::', '')[:40]) for r in rows)
t_end = max(e for _, e, _ in iv)
t0 = iv[0][0] + (1 - frac) * (t_end - iv[0][0])
iv = [x for x in iv if x[0] >= t0]
busy, cur_s, cur_e, gaps = 0, iv[0][0], iv[0][1], []
for s, e, _ in iv[1:]:
    if s > cur_e:
        busy += cur_e - cur_s
        gaps.append((s - cur_e, cur_e))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = cur_e - iv[0][0]
tot = collections.Counter()
cnt = collections.Counter()
for s, e, n in iv:
    tot[n] += e - s
    cnt[n] += 1
print(f'window {span / 1e3:.1f} us: busy {busy / 1e3:.1f} us ({100 * busy / span:.1f} %), {len(gaps)} gaps, '
      f'idle {sum(g for g, _ in gaps) / 1e3:.1f} us; largest: {[round(g / 1e3, 1) for g, _ in sorted(gaps)[-8:]]}')
for n, t in tot.most_common(8):
    print(f'  {n:40s} {cnt[n]:6d} x {t / cnt[n] / 1e3:8.2f} us = {t / 1e3:9.1f} us')
