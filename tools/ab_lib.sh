set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
B="python bench.py --steps 300 --warmup 20 --no-cpu --stream-graphs 0 --stream-train-graphs 0 --no-secondary --many 0"
for v in new base new base; do
  if [ $v = base ]; then export WDMPNN_LIB=$PWD/exp/libwdmpnn_base.so; else unset WDMPNN_LIB; fi
  timeout -k 10 200 $B > gpurun_out/ab_$v.log 2>&1 || exit $?
  python - "$v" <<'PY'
import json,sys
l=[x for x in open(f'gpurun_out/ab_{sys.argv[1]}.log') if x.startswith('{')][-1]; d=json.loads(l)
print(sys.argv[1], round(d['value']/1e6,2), 'single', round(d['single_stream']['value']/1e6,2), 'layer us', round(d['roofline']['avg_launch_us'],2))
PY
done
unset WDMPNN_LIB
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/rocprof_ab -o run --output-format csv -- python bench.py --steps 100 --warmup 10 --no-cpu --no-secondary --streams 1 --stream-graphs 0 --stream-train-graphs 0 > gpurun_out/rocprof_ab.log 2>&1 && python tools/kstats.py gpurun_out/rocprof_ab/run_kernel_stats.csv 5
