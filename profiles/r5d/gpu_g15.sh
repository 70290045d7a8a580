# Round-5 GPU check (profiles/r5d, part 7): the suite's VDM column (two concurrent pods of a
# split-2 plugin, the reference's "virtual device memory" pods) for launch-bound cases, placed
# by the product (--numa-spread auto: the two vGPUs get different CPU nodes, the shim keeps
# each pod there) and as round 4 had it (both pods pinned to the GPU's NUMA node).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5d
mkdir -p $O
for pl in product local; do
  timeout -k 10 500 python -u benchmarks/aibench_suite.py --cases lstm-inf,resnet152-inf,deeplab-inf \
    --modes native,vgpu --repeats 1 --vdm 1 --vdm-seconds 6 --vdm-placement $pl \
    --json-out $O/vdm_$pl.json --md-out $O/vdm_$pl.md > $O/vdm_$pl.log 2>&1 || exit $?
  tail -8 $O/vdm_$pl.md
done
