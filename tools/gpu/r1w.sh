set -o pipefail
OUT=gpurun_out/r1w; mkdir -p $OUT; export TMPDIR=/tmp
make -C native -j16 > $OUT/build.log 2>&1 || exit 1
for k in malloc managed pitch 3d ext async vmm; do
  VGPU_DEVICE_MEMORY_LIMIT=2048m VGPU_SHARED_CACHE=/tmp/probe-$k.cache LD_PRELOAD=$PWD/4paradigm-k8s-device-plugin_amd/lib/libvgpu_hip.so \
    timeout -k 10 60 4paradigm-k8s-device-plugin_amd/lib/hip_alloc_probe $k 2>&1 | tail -1 || exit 2
  rm -f /tmp/probe-$k.cache
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_shim.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "allocations_are_accounted" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 6; }
tail -1 $OUT/pytest.log
