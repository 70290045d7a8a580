#!/bin/bash
# The latency class at HEAD: the r3t mix - a b=1 ResNet-50 service at
# 100 req/s (priority 0) next to VGG-16 training, LSTM training and DeepLab inference
# (priority 2), split 4, default policy (strict preemption: hold 3 ms + depth 4; polled waits
# on a crowded GPU, which the latency class is exempt from) - ABAB x3 against no classes.
set -o pipefail
OUT=gpurun_out/${1:-r6h}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u benchmarks/mix.py --seconds 8 --ab ${2:-3} \
  --priority "resnet50-inf:1:lat=0,vgg16-train=2,lstm-train=2,deeplab-inf=2" \
  --json-out $OUT/mix.json --md-out $OUT/mix.md > $OUT/mix.log 2>&1
rc=$?; tail -12 $OUT/mix.md 2>/dev/null; exit $rc
