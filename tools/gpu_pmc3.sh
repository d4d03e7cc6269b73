# L2 hit/miss and HBM-side fetch of the single-stream bench for each experiment library named
set -o pipefail
for LIB in "$@"; do
  rm -rf gpurun_out/pmc3_$LIB; mkdir -p gpurun_out/pmc3_$LIB
  for pass in "tcc:TCC_HIT_sum TCC_MISS_sum" "fetch:FETCH_SIZE" "write:WRITE_SIZE" "tcp:TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
    name=${pass%%:*}; ctrs=${pass#*:}
    WDMPNN_LIB=$PWD/exp/libwdmpnn_$LIB.so timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/pmc3_$LIB/$name -o run -- \
      python bench.py --steps 20 --warmup 3 --no-cpu --no-secondary --streams 1 --many 0 --stream-graphs 0 --stream-train-graphs 0 > gpurun_out/pmc3_$LIB/$name.log 2>&1 || { echo "pass $name failed"; tail -3 gpurun_out/pmc3_$LIB/$name.log; }
  done
  echo "== $LIB"; python tools/pmc_summary.py gpurun_out/pmc3_$LIB | grep -A6 "mp_layer\|embed\|wo_readout" | head -40
done
