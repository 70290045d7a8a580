#!/bin/bash
# Round-3: strict preemption of the background class. The r3j mix (b=1 ResNet-50 service
# at 100 req/s, priority 0, next to VGG-16 training, LSTM training, DeepLab inference at
# priority 2), ABAB: soft yield (shipped) / held while the service is busy
# (VGPU_PREEMPT_HOLD_MS) / held + at most 4 packets in flight per trainer process
# (VGPU_PREEMPT_DEPTH).
out=${1:-gpurun_out/r3q}
reps=${2:-3}
mkdir -p "$out"
[ -n "$SKIP_TESTS" ] || timeout -k 10 300 python -u -m pytest -v -rfE --timeout 240 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_limits.py -k "depth_bound or yields_to_a_busy" > "$out/pytest.log" 2>&1
rc=$?
echo "pytest_rc=$rc" >> "$out/pytest.log"
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 960 python -u benchmarks/mix.py --seconds 8 --ab "$reps" --skip-default \
  --priority "resnet50-inf:1:lat=0,vgg16-train=2,lstm-train=2,deeplab-inf=2" \
  ${ARMS:---bg-env VGPU_PREEMPT_HOLD_MS=20 --bg-env VGPU_PREEMPT_HOLD_MS=20,VGPU_PREEMPT_DEPTH=4} \
  --json-out "$out/mix.json" --md-out "$out/mix.md" > "$out/mix.log" 2>&1
