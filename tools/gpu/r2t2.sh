#!/bin/bash
out=gpurun_out/r2t2; mkdir -p $out
export VGPU_DEVICE_MEMORY_LIMIT=8g VGPU_DEVICE_CU_LIMIT=25 VGPU_CU_MODE=spatial VGPU_SHARED_CACHE=/tmp/cuprobe.cache VGPU_LOG_LEVEL=4
LIB=$(python -c "from amdvgpu.shim.native import shim_path; print(shim_path())")
LD_PRELOAD=$LIB timeout -k 5 120 python -c "import torch; print('CUS', torch.cuda.get_device_properties(0).multi_processor_count)" > $out/dbg.log 2>&1
echo "rc=$?" >> $out/steps.txt
grep -E "CU count|CUS|phase|init|mask" $out/dbg.log | head -60 > $out/dbg_cu.txt
