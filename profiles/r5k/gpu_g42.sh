# Round-5 GPU check (profiles/r5k, part 10): tiny kernels from 1/2/4 processes in split-4-like
# vGPUs (25 % share, auto mode: the crowd count runs) with the shim's default wait.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/r5k
mkdir -p $out
timeout -k 10 200 python3 -u tools/probe/tiny_kernels.py --procs 1,2,4 --nblocks 8 --us 5 --shim --cu-limit 25 \
  --seconds 6 > $out/tiny_auto25.jsonl 2> $out/tiny_auto25.err
rc=$?
cat $out/tiny_auto25.jsonl
exit $rc
