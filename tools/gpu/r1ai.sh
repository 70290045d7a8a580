set -o pipefail
# r1ai: per-kernel profile of the headline step (ResNet-V2-50 inference in a vGPU) after r1ah.
OUT=gpurun_out/r1ai; mkdir -p $OUT; export TMPDIR=/tmp
make -C native -j16 > $OUT/build.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench -- python3 bench.py --steps 60 --warmup 10 \
  --modes vgpu > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 10; }
python3 tools/prof_summary.py "$OUT/prof/**/*results.db" --top 30 -o $OUT/prof_summary.md \
  --title "ResNet-V2-50 inference b=50 346x346 bf16 in a vGPU, 60 timed steps (r1ai)" > /dev/null || true
head -45 $OUT/prof_summary.md
