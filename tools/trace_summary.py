"""Summarise a rocprofv3 kernel trace: per-forward kernel sequence with durations (median over
forwards).  Usage: python tools/trace_summary.py gpurun_out/rocprof/run_kernel_trace.csv [period]"""
import csv
import re
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
period = int(sys.argv[2]) if len(sys.argv) > 2 else None
names = [re.sub(r'\(.*', '', r['Kernel_Name']).replace('void ', '').replace('(anonymous namespace)::', '').replace('wd::', '')[:48]
         for r in rows]
dur = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000 for r in rows]
start = [int(r['Start_Timestamp']) / 1000 for r in rows]
# a forward ends with its readout: readout_kernel (unblocked path) or wo_readout_kernel (fused path)
END = 'wo_readout_kernel' if any(n.startswith('wo_readout_kernel') for n in names) else 'readout_kernel'
if period is None:  # period = distance between readout launches
    ro = [i for i, n in enumerate(names) if n.startswith(END)]
    period = ro[-1] - ro[-2]
last = max(i for i, n in enumerate(names) if n.startswith(END))
seqs = []
i = last
while i - period + 1 >= 0 and names[i].startswith(END):
    seqs.append(list(range(i - period + 1, i + 1)))
    i -= period
print(f'{len(seqs)} forwards x {period} kernels')
tot = 0.0
for k in range(period):
    ds = [dur[s[k]] for s in seqs]
    gaps = [start[s[k]] - (start[s[k] - 1] + dur[s[k] - 1]) for s in seqs if s[k] > 0]
    med = statistics.median(ds)
    tot += med
    print(f'{names[seqs[0][k]]:48s} {med:8.2f} us   gap-before {statistics.median(gaps):6.2f} us')
span = [start[s[-1]] + dur[s[-1]] - start[s[0]] for s in seqs]
print(f'sum of kernel medians {tot:.2f} us; first-start..last-end median {statistics.median(span):.2f} us')
