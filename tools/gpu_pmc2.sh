# PMC passes (waves, lds) of the single-stream bench for each experiment library named
set -o pipefail
for LIB in "$@"; do
  rm -rf gpurun_out/pmc_$LIB; mkdir -p gpurun_out/pmc_$LIB
  for pass in "waves:SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
              "lds:SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_ACTIVE_INST_VALU"; do
    name=${pass%%:*}; ctrs=${pass#*:}
    WDMPNN_LIB=$PWD/exp/libwdmpnn_$LIB.so timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/pmc_$LIB/$name -o run -- \
      python bench.py --steps 20 --warmup 3 --no-cpu --no-secondary --streams 1 --many 0 --stream-graphs 0 --stream-train-graphs 0 > gpurun_out/pmc_$LIB/$name.log 2>&1 || { tail gpurun_out/pmc_$LIB/$name.log; exit 1; }
  done
  echo "== $LIB"; python tools/pmc_summary.py gpurun_out/pmc_$LIB | grep -A12 mp_layer | head -40
done
