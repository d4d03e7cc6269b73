# round 6: the driver's bench command (20/5, 200/20) and the two-CPU run again, after the profiles the bench cites were refreshed
set -e
export TMPDIR=/tmp
D=gpurun_out/r6y
mkdir -p $D
{ echo '$ python3 bench.py --gpus 1 --steps 20 --warmup 5'; timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5;
  echo '$ python3 bench.py --gpus 1 --steps 200 --warmup 20'; timeout -k 10 400 python3 bench.py --gpus 1 --steps 200 --warmup 20; } > $D/bench_driver_cmd.log 2>&1
{ echo '$ python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpus 2 --no-cpu'; timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpus 2 --no-cpu; } > $D/cpus2.log 2>&1
nproc > $D/nproc.txt; python3 -c "import os; print(sorted(os.sched_getaffinity(0))[:8], len(os.sched_getaffinity(0)))" >> $D/nproc.txt; uptime >> $D/nproc.txt
