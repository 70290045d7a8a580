#!/bin/bash
# Round-3 mix, ABAB: default / priority classes / priority classes with the background
# pods' kernels serialised (AMD_SERIALIZE_KERNEL=3: their in-flight queue bounded to one
# kernel), to see whether the latency pod's remaining delay is the trainers' queued work.
out=${1:-gpurun_out/r3j}
reps=${2:-3}
mkdir -p "$out"
timeout -k 10 1000 python -u benchmarks/mix.py --seconds 8 --ab "$reps" \
  --priority "resnet50-inf:1:lat=0,vgg16-train=2,lstm-train=2,deeplab-inf=2" --bg-env AMD_SERIALIZE_KERNEL=3 \
  --json-out "$out/mixab.json" --md-out "$out/mixab.md" > "$out/mixab.log" 2>&1
