"""Group a kernel trace of tools/size_sweep.py by (kernel, grid) and print median durations."""
import collections
import csv
import re
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    n = re.sub(r'\(.*', '', r['Kernel_Name']).replace('void ', '').replace('wd::', '')
    d[(n, int(r['Grid_Size_X']))].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000)
for (n, gsz), v in sorted(d.items(), key=lambda x: (x[0][0], x[0][1])):
    if len(v) >= 20:
        print(f'{n:42s} grid {gsz:8d} x{len(v):4d}  median {statistics.median(v):8.2f} us')
