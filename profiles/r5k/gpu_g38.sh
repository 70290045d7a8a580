# Round-5 GPU study (profiles/r5k, part 7): tiny kernels from 1/2/4 processes, two per socket
# from 3 on - which wait carries the per-socket effect? torch's synchronize (HIP spins on the
# completion signal), a blocking event wait, no wait for 4096 launches, and the shim's
# polling wait (VGPU_SYNC_WAIT=poll).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/r5k
mkdir -p $out
T="timeout -k 10 200 python3 -u tools/probe/tiny_kernels.py --procs 1,2,4 --nblocks 8 --us 5"
{
$T --wait spin &&
$T --wait block &&
$T --sync-every 4096 &&
$T --shim --env VGPU_SYNC_WAIT=poll &&
$T --shim --env VGPU_SYNC_WAIT=native
} > $out/tiny_waits.jsonl 2> $out/tiny_waits.err
rc=$?
cat $out/tiny_waits.jsonl
exit $rc
