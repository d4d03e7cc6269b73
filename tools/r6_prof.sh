# round 6 profiles of the final tree: rocprofv3 kernel statistics of the headline workload with one batch in
# flight and with the bench's three streams, the PMC passes for HBM traffic (tools/pmc.sh), one training
# step's kernel trace
set -e
export TMPDIR=/tmp
D=gpurun_out/r6e
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof1 -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu --no-secondary --streams 1 --many 0 --stream-graphs 0 --stream-train-graphs 0 > $D/prof1.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof3 -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu --no-secondary --many 0 --stream-graphs 0 --stream-train-graphs 0 > $D/prof3.log 2>&1
PMC_PASSES="fetch write waves" bash tools/pmc.sh > $D/pmc.log 2>&1
STEPS=20 timeout -k 10 200 rocprofv3 --kernel-trace -d $D/train -o run -- python3 tools/train_bench.py > $D/train_prof.log 2>&1
