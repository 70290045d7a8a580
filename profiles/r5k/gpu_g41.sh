# Round-5 GPU check (profiles/r5k, part 9): tiny kernels from 1/2/4 processes in quota-only
# vGPUs with the shim's default wait (auto: polled once two other processes keep the GPU busy).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/r5k
mkdir -p $out
timeout -k 10 200 python3 -u tools/probe/tiny_kernels.py --procs 1,2,4 --nblocks 8 --us 5 --shim --seconds 5 \
  > $out/tiny_auto.jsonl 2> $out/tiny_auto.err
rc=$?
cat $out/tiny_auto.jsonl
exit $rc
