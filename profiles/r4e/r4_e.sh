#!/bin/bash
# Round-4 re-measurement at HEAD (profiles/r4e):
#   cfg3   BASELINE config 3: two VGG-16 training pods at 50 % (split 2, default auto policy)
#   cfg4   BASELINE config 4: a 322 GiB vGPU on 288 GiB HBM, LSTM training on a 300 GiB dataset
#   prof   rocprofv3 steady state of the headline tenant (native / quota-only / 25 % temporal):
#          find-db filled first, kernels counted inside the timed roctx window only
#   pmc    SQ busy-CU counters of a 25 % pod, CU mask vs GPU-time limiter
out=${1:-gpurun_out/r4e}
what=${2:-cfg3,cfg4,prof,pmc}
mkdir -p "$out"
export TMPDIR=/tmp
if [[ $what == *cfg3* ]]; then
  timeout -k 10 300 python -u benchmarks/vgpu_scaling.py --case vgg16-train --tenants 1,2 --policy default \
    --seconds 8 --json-out "$out/cfg3.json" --md-out "$out/cfg3.md" > "$out/cfg3.log" 2>&1 || exit $?
fi
if [[ $what == *cfg4* ]]; then
  timeout -k 10 400 python -u benchmarks/oversubscribe.py --modes resident,vdm --json-out "$out/cfg4.json" \
    --md-out "$out/cfg4.md" > "$out/cfg4.log" 2>&1 || exit $?
fi
if [[ $what == *prof* ]]; then
  timeout -k 10 500 python -u tools/probe/prof_tenant.py --out "$out/prof" --steps 30 > "$out/prof.log" 2>&1 || exit $?
fi
if [[ $what == *pmc* ]]; then
  for m in spatial temporal; do
    timeout -s KILL 120 rocprofv3 --pmc SIMD_UTILIZATION SQ_WAVES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --kernel-trace \
      --output-format csv -d "$out/pmc_$m" -o "t25_$m" -- python3 benchmarks/cu_occupancy.py --cu-limit 25 \
      --cu-mode $m --workload resnet --iters 20 > "$out/pmc_$m.log" 2>&1 || exit $?
  done
  python tools/pmc_summary.py "spatial25=$out/pmc_spatial/**/*counter_collection.csv" \
    "temporal25=$out/pmc_temporal/**/*counter_collection.csv" --title "ResNet-50 b=50 in a 25 % vGPU: CU mask vs GPU-time limiter" -o "$out/pmc.md" > "$out/pmc_summary.log" 2>&1
  find "$out" -name "*counter_collection.csv" -size +20M -delete
fi
