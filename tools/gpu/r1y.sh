set -o pipefail
# r1y: per-kernel hardware counters of the hand-written kernels (stall / instruction mix /
# LDS conflicts / HBM bytes), one rocprofv3 --pmc pass per counter group.
OUT=gpurun_out/r1y; mkdir -p $OUT; export TMPDIR=/tmp
make -C native -j16 > $OUT/build.log 2>&1 || exit 1
run() {  # name counters...
  local n=$1; shift
  echo "pass $n: $*"
  timeout -s KILL 180 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $OUT/$n -o $n -- \
    python3 benchmarks/kernel_pmc.py > $OUT/$n.log 2>&1 || { tail -5 $OUT/$n.log; exit 3; }
}
run p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES
run p2 SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES SQ_INSTS_SALU SQ_INST_LEVEL_VMEM
run p3 FETCH_SIZE
run p4 WRITE_SIZE
python3 tools/pmc_summary.py --all-counters "stalls=$OUT/p1/**/*counter_collection.csv" \
  "instructions=$OUT/p2/**/*counter_collection.csv" "fetch=$OUT/p3/**/*counter_collection.csv" \
  "write=$OUT/p4/**/*counter_collection.csv" --title "Hand-written gfx950 kernels: per-dispatch counters (r1y)" \
  -o $OUT/kernel_pmc.md > /dev/null
cut -c1-400 $OUT/kernel_pmc.md
