set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local n=$1; shift; echo "== $n $(date +%T)"; timeout -k 10 150 "$@" > gpurun_out/diag_$n.log 2>&1; local rc=$?; echo "== $n rc=$rc $(date +%T)"; tail -c 300 gpurun_out/diag_$n.log; echo; if [ $rc -ne 0 ]; then exit $rc; fi; }
run main python bench.py --steps 200 --warmup 20 --no-cpu --no-secondary --stream-graphs 0 --stream-train-graphs 0
run stream python bench.py --steps 20 --warmup 5 --no-cpu --no-secondary --stream-graphs 200000 --stream-train-graphs 0
run strain python bench.py --steps 20 --warmup 5 --no-cpu --no-secondary --stream-graphs 0 --stream-train-graphs 32768
run secondary python bench.py --steps 20 --warmup 5 --no-cpu --stream-graphs 0 --stream-train-graphs 0
