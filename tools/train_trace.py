"""One training step's kernel sequence from a rocprofv3 kernel trace of tools/train_bench.py: the
kernels from the last weight pack (pack_kernel, the first launch of a training forward) to the end.
Usage: python tools/train_trace.py gpurun_out/rocprof_train/run_kernel_trace.csv"""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
first = max(i for i, r in enumerate(rows) if 'pack_kernel' in r['Kernel_Name'])
t0 = int(rows[first]['Start_Timestamp'])
print('One training step (B=128 polymer, depth 3, hidden 300, MoleculeModel + MSE + fused Adam), '
      'rocprofv3 --kernel-trace of tools/train_bench.py')
print('start_us  dur_us  kernel')
busy = 0.0
for r in rows[first:]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    busy += (e - s) / 1e3
    name = re.sub(r'\(.*', '', r['Kernel_Name']).replace('void ', '')[:70]
    print(f'{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.2f}  {name}')
print(f'kernel time {busy:.1f} us; first start .. last end {(int(rows[-1]["End_Timestamp"]) - t0) / 1e3:.1f} us')
