"""Per-kernel averages of rocprofv3 counter CSVs (one row per dispatch x counter).
Usage: python tools/pmc_summary.py gpurun_out/pmc"""
import collections
import csv
import glob
import os
import re
import sys

root = sys.argv[1]
data = collections.defaultdict(lambda: collections.defaultdict(list))
grid = {}
for f in glob.glob(os.path.join(root, '*', '*counter_collection.csv')):
    for r in csv.DictReader(open(f)):
        name = re.sub(r'\(.*', '', r['Kernel_Name']).replace('void ', '').replace('wd::', '')
        key = (name, r.get('Grid_Size', r.get('Grid_Size_X', '')))
        data[key][r['Counter_Name']].append(float(r['Counter_Value']))
for key in sorted(data):
    c = data[key]
    n = max(len(v) for v in c.values())
    if n < 3:
        continue
    avg = {k: sum(v) / len(v) for k, v in c.items()}
    print(f'{key[0]:40s} grid={key[1]:>8s} dispatches={n}')
    for k in sorted(avg):
        print(f'    {k:28s} {avg[k]:16.1f}')
