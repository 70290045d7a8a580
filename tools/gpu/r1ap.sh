set -o pipefail
# r1ap: per-kernel steady-state profile of the headline step after the dual-source conv (r1ao).
OUT=gpurun_out/r1ap; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench -- python3 bench.py --steps 60 --warmup 10 \
  --modes vgpu > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 10; }
python3 tools/prof_summary.py "$OUT/prof/**/*results.db" --last-ms 120 --top 30 -o $OUT/prof_steady.md \
  --title "ResNet-V2-50 inference b=50 346x346 bf16 in a vGPU: steady state (last 120 ms), r1ap" > /dev/null
cut -c1-160 $OUT/prof_steady.md | head -45
