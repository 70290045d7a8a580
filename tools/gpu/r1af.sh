set -o pipefail
# r1af: eager training cases, more ABBA repeats; with and without the launch hooks.
OUT=gpurun_out/r1af; mkdir -p $OUT; export TMPDIR=/tmp
make -C native -j16 > $OUT/build.log 2>&1 || exit 1
timeout -k 10 900 python benchmarks/aibench_suite.py --cases resnet50-train,deeplab-train --steps 30 --warmup 10 \
  --repeats 4 --modes native,vgpu --md-out $OUT/train.md --json-out $OUT/train.json > $OUT/train.log 2>&1 || { tail -20 $OUT/train.log; exit 2; }
cat $OUT/train.md
VGPU_HOOK_LAUNCH=0 timeout -k 10 900 python benchmarks/aibench_suite.py --cases resnet50-train,deeplab-train --steps 30 --warmup 10 \
  --repeats 4 --modes native,vgpu --md-out $OUT/train_nohook.md > $OUT/train_nohook.log 2>&1 || { tail -20 $OUT/train_nohook.log; exit 3; }
cat $OUT/train_nohook.md
