set -o pipefail
OUT=gpurun_out/r1w; mkdir -p $OUT; export TMPDIR=/tmp
make -C native -j16 > $OUT/build.log 2>&1 || exit 1
P=4paradigm-k8s-device-plugin_amd/lib
VGPU_LOG_LEVEL=4 VGPU_DEVICE_MEMORY_LIMIT=2048m VGPU_SHARED_CACHE=/tmp/probe-a.cache LD_PRELOAD=$PWD/$P/libvgpu_hip.so \
  timeout -k 10 60 $P/hip_alloc_probe async > $OUT/shim_async.log 2>&1; echo "rc=$?"; grep -v "launch\|memcpy" $OUT/shim_async.log | tail -40 | cut -c1-200
rm -f /tmp/probe-a.cache
true
