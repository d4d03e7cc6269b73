# round 6: first-use host costs (tools/first_use.py) and the driver's bench command with the resident batches
# registered on the bench's streams in setup
set -e
export TMPDIR=/tmp
D=gpurun_out/r6x
mkdir -p $D
timeout -k 10 300 python3 -u tools/first_use.py > $D/first_use.log 2>&1
{ echo '$ python3 bench.py --gpus 1 --steps 20 --warmup 5'; timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu;
  echo '$ python3 bench.py --gpus 1 --steps 200 --warmup 20'; timeout -k 10 400 python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu; } > $D/bench_driver_cmd.log 2>&1
