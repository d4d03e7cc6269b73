"""One training step's kernel sequence from a rocprofv3 --kernel-trace database (results.db) of
tools/train_bench.py: the last step's kernels (its weight pack when the optimizer did not repack, the
training forward, backward and the optimizer).  Usage: python tools/train_trace_db.py gpurun_out/rocprof_train/run_results.db"""
import re
import sqlite3
import sys

con = sqlite3.connect(sys.argv[1])
rows = con.execute('select d.start, d.end, s.kernel_name from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s '
                   'on d.kernel_id = s.id order by d.start').fetchall()
# the last step: from the last embed_kernel (the training forward's first layer), back over the weight pack
# launches that precede it when the optimizer did not repack
first = max(i for i, r in enumerate(rows) if 'embed_kernel' in r[2])
while first > 0 and any(k in rows[first - 1][2] for k in ('pack_kernel', 'split_tiles_batch', 'split_h2_kernel')) and \
        'adam_kernel' not in rows[first - 1][2]:
    first -= 1
t0 = rows[first][0]
print('One training step (B=128 polymer, depth 3, hidden 300, MoleculeModel + MSE + fused Adam), '
      'rocprofv3 --kernel-trace of tools/train_bench.py')
print('start_us  dur_us  kernel')
busy = 0.0
for s, e, name in rows[first:]:
    busy += (e - s) / 1e3
    name = re.sub(r'\(.*', '', name).replace('void ', '')[:70]
    print(f'{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.2f}  {name}')
print(f'kernel time {busy:.1f} us; first start .. last end {(rows[-1][1] - t0) / 1e3:.1f} us')
