#!/bin/bash
# Mix with priority classes + CU reservation (r3f), then the many-pod study (r3e).
mkdir -p gpurun_out/r3f
timeout -k 10 560 python -u benchmarks/mix.py --seconds 8 \
  --priority "resnet50-inf:1:lat=0,vgg16-train=2,lstm-train=2,deeplab-inf=2" \
  --json-out gpurun_out/r3f/mix.json --md-out gpurun_out/r3f/mix.md > gpurun_out/r3f/mix.log 2>&1 || exit $?
bash tools/gpu/r3_many.sh gpurun_out/r3e base,conc
