set -o pipefail
# r1ak: hardware counters of the LDS-DMA conv kernel on the four stages' 3x3 convs.
OUT=gpurun_out/r1ak; mkdir -p $OUT; export TMPDIR=/tmp
run() {  # name counters...
  local n=$1; shift
  echo "pass $n: $*"
  timeout -s KILL 180 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $OUT/$n -o $n -- \
    python3 benchmarks/kernel_pmc.py --set conv3x3 > $OUT/$n.log 2>&1 || { tail -5 $OUT/$n.log; exit 3; }
}
run p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES
run p2 SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE
run p3 FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT
python3 tools/pmc_summary.py --all-counters "stalls=$OUT/p1/**/*counter_collection.csv" \
  "instructions=$OUT/p2/**/*counter_collection.csv" "fetch=$OUT/p3/**/*counter_collection.csv" \
  --title "LDS-DMA conv kernel, 3x3 convs of stages 1-4: per-dispatch counters (r1ak)" \
  -o $OUT/kernel_pmc.md > /dev/null
cut -c1-600 $OUT/kernel_pmc.md
