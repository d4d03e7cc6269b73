#!/bin/bash
# PMC passes over a short bench run (each pass its own rocprofv3 invocation: counters only, no
# sys/runtime traces).  Output: gpurun_out/pmc/<pass>/...counter_collection.csv
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
run() {
  local name=$1; shift
  echo "== pmc $name: $*"
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc/$name -o run -- \
      python bench.py --steps 20 --warmup 3 --no-cpu --no-secondary --streams 1 --many 0 --stream-graphs 0 --stream-train-graphs 0 ${PMC_BENCH_ARGS:-} > gpurun_out/pmc/$name.log 2>&1
  local rc=$?
  echo "== pmc $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/pmc/$name.log; exit $rc; fi
}
PASSES=${PMC_PASSES:-"waves lds fetch write tcc"}
want() { case " $PASSES " in *" $1 "*) return 0 ;; *) return 1 ;; esac; }
want waves && run waves SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE
want lds && run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_ACTIVE_INST_VALU
want fetch && run fetch FETCH_SIZE
want write && run write WRITE_SIZE
want tcc && run tcc TCC_HIT_sum TCC_MISS_sum
# (TA_* counters: a pass with them did not finish within 300 s on the box; not collected)
exit 0
