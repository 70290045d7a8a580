#!/bin/bash
# Round-3 limiter study on one MI355X (profiles/r3*):
#   mix       heterogeneous pods (benchmarks/mix.py): isolation + inference P50/P99
#   light     4 concurrent light tenants (ResNet-50 b=4) at 25 % temporal, charge
#             model share vs progress (benchmarks/temporal_accuracy.py)
# Each step has its own time limit; steps chained with && (a failure ends the script).
out=${1:-gpurun_out/r3s}
what=${2:-mix,light}
mkdir -p "$out"
ok=0
if [[ $what == *mix* ]]; then
  timeout -k 10 420 python -u benchmarks/mix.py --seconds 8 --json-out "$out/mix.json" --md-out "$out/mix.md" \
    > "$out/mix.log" 2>&1 || exit $?
fi
if [[ $what == *light* ]]; then
  for model in share progress; do
    timeout -k 10 300 python -u benchmarks/temporal_accuracy.py --workload resnet50 --batch 4 --tenants 1,4 \
      --limits 25 --seconds 5 --extra VGPU_CHARGE_MODEL=$model --json-out "$out/light_$model.json" \
      --md-out "$out/light_$model.md" > "$out/light_$model.log" 2>&1 || exit $?
  done
fi
exit $ok
