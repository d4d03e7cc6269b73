"""Per-kernel averages of rocprofv3 counter CSVs (one row per dispatch x counter).
Usage: python tools/pmc_summary.py gpurun_out/pmc [traffic.json]

With a second argument, also writes per-kernel HBM-side bytes per launch as JSON (read by bench.py
for roofline.traffic): FETCH_SIZE (KB) x 2 — on gfx950 FETCH_SIZE reports half the bytes of wide
16-B-per-lane reads (MI355X_MICROARCH.md §HBM), and every load of these kernels is 16 B per lane
(LDS-DMA / float4) — plus WRITE_SIZE (KB, exact for 16-B stores).  Both count Infinity-Cache hits."""
import collections
import csv
import json
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

if len(sys.argv) > 2:
    traffic = {}
    by_name = collections.defaultdict(list)
    for key in data:
        c = data[key]
        if 'FETCH_SIZE' in c and 'WRITE_SIZE' in c and len(c['FETCH_SIZE']) >= 3:
            by_name[key[0]].append(key)
    for name, keys in by_name.items():
        f = [v for k in keys for v in data[k]['FETCH_SIZE']]
        w = [v for k in keys for v in data[k]['WRITE_SIZE']]
        fetch = 2.0 * 1024 * sum(f) / len(f)
        write = 1024.0 * sum(w) / len(w)
        traffic[name] = {'fetch_bytes': fetch, 'write_bytes': write, 'traffic_bytes': fetch + write,
                         'dispatches': len(f)}
    traffic['_note'] = ('HBM-side bytes per launch from rocprofv3 --pmc FETCH_SIZE (x2, gfx950 wide-read '
                        'correction) and WRITE_SIZE, separate passes (tools/pmc.sh); includes Infinity-Cache hits')
    json.dump(traffic, open(sys.argv[2], 'w'), indent=1, sort_keys=True)
