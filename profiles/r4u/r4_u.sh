#!/bin/bash
# Round-4 GPU study (profiles/r4u): the two suite cases whose overhead median sat above the
# reference's figure within noise (DeepLab training b=1, ResNet-50 inference), 8 ABBA repeats.
out=${1:-gpurun_out/r4u}
mkdir -p "$out"
timeout -k 10 1000 python -u benchmarks/aibench_suite.py --cases deeplab-train,resnet50-inf --repeats 8 --vdm 0 \
  --json-out "$out/suite.json" --md-out "$out/suite.md" > "$out/suite.log" 2>&1
echo "suite_rc=$?" >> "$out/suite.log"
