#!/bin/bash
set -o pipefail
cd "$(dirname "$0")"
mkdir -p ../../gpurun_out/probe
O=../../gpurun_out/probe
sh -c "ls -la /sys/class/kfd/kfd/proc/*/stats_*/ | head -20; cat /sys/class/kfd/kfd/proc/*/stats_*/* 2>&1 | head -20; cat /sys/class/kfd/kfd/topology/nodes/4/properties" > $O/kfd.txt 2>&1
echo "env done"
PRE="${LD_PRELOAD:+$LD_PRELOAD:}$PWD/hsa_probe.so"
timeout -k 10 300 python torch_probe.py > $O/torch_native.txt 2>&1 || exit 1
LD_PRELOAD="$PRE" timeout -k 10 300 python torch_probe.py > $O/torch_probe.txt 2>&1 || exit 1
LD_PRELOAD="$PRE" PROBE_CU_MASK=64 timeout -k 10 300 python torch_probe.py > $O/torch_probe_mask64.txt 2>&1 || exit 1
echo "torch done"
timeout -k 10 300 ./cu_map 256 > $O/cu_map.txt 2>&1 || exit 1
echo "all done"
