set -o pipefail
OUT=gpurun_out/diag; mkdir -p $OUT; export TMPDIR=/tmp
make -C native -j16 > $OUT/build.log 2>&1 || exit 1
L=4paradigm-k8s-device-plugin_amd/lib
PRE="${LD_PRELOAD:+$LD_PRELOAD:}$PWD/$L/libvgpu_hip.so"
for k in malloc managed; do
  echo "== $k"
  VGPU_DEVICE_MEMORY_LIMIT=2048m VGPU_SHARED_CACHE=/tmp/diag-$k.cache VGPU_LOG_LEVEL=3 VGPU_STATS=1 LD_PRELOAD="$PRE" \
    timeout -k 5 60 $L/hip_alloc_probe $k > $OUT/probe_$k.log 2>&1; echo rc=$?
  grep -v "agent_get_info\|pool_get_info" $OUT/probe_$k.log | tail -25
done
echo "== amdsmi under shim with configured region"
VGPU_DEVICE_MEMORY_LIMIT=24g VGPU_SHARED_CACHE=/tmp/diag-smi.cache LD_PRELOAD="$PRE" timeout -k 5 60 python -c "import torch; torch.cuda.mem_get_info(0)" 
VGPU_DEVICE_MEMORY_LIMIT=24g VGPU_SHARED_CACHE=/tmp/diag-smi.cache VGPU_LOG_LEVEL=3 LD_PRELOAD="$PRE" timeout -k 5 60 python -c "
import amdsmi, traceback
try:
    amdsmi.amdsmi_init(); print('init ok')
    h = amdsmi.amdsmi_get_processor_handles()[0]; print('handles ok')
    print('total', amdsmi.amdsmi_get_gpu_memory_total(h, amdsmi.AmdSmiMemoryType.VRAM))
except Exception:
    traceback.print_exc()
" > $OUT/amdsmi.log 2>&1; tail -20 $OUT/amdsmi.log
grep -o "amdsmi[a-z_]*\.so[.0-9]*\|libamd_smi[.a-z0-9]*" /proc/self/maps | head -2
python -c "import amdsmi.amdsmi_wrapper as w; print(w.__file__)" 2>&1 | tail -1
