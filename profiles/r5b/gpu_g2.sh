set -o pipefail
cd $GRAFT_REPO_ROOT
P=4paradigm-k8s-device-plugin_amd/lib/escape_probe
echo "== no shim" > gpurun_out/g2.log
timeout -k 5 60 $P svm 8192 2048 >> gpurun_out/g2.log 2>&1
echo "== shim 4g" >> gpurun_out/g2.log
VGPU_DEVICE_MEMORY_LIMIT=4g VGPU_SHARED_CACHE=/tmp/g2.cache LD_PRELOAD=$PWD/4paradigm-k8s-device-plugin_amd/lib/libvgpu_hip.so VGPU_LOG_LEVEL=3 timeout -k 5 60 $P svm 8192 2048 >> gpurun_out/g2.log 2>&1
echo "== host" >> gpurun_out/g2.log
VGPU_DEVICE_MEMORY_LIMIT=4g VGPU_HOST_MEMORY_LIMIT=1g VGPU_SHARED_CACHE=/tmp/g2b.cache LD_PRELOAD=$PWD/4paradigm-k8s-device-plugin_amd/lib/libvgpu_hip.so timeout -k 5 60 $P host 600 >> gpurun_out/g2.log 2>&1
cat gpurun_out/g2.log | grep -v "^\[vGPU DEBUG" | tail -40
