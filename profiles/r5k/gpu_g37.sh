# Round-5 GPU study (profiles/r5k, part 6): tiny kernels from 1/2/3/4/8 processes (one
# socket each, two per socket from 3 on) - the GPU's handling of several processes' queues
# without PyTorch's host path. 8 one-wave-per-CU blocks of 5 us, and 64 blocks of 20 us.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/r5k
mkdir -p $out
timeout -k 10 300 python3 -u tools/probe/tiny_kernels.py --procs 1,2,3,4,8 --nblocks 8 --us 5 > $out/tiny_8x5.jsonl 2> $out/tiny_8x5.err &&
cat $out/tiny_8x5.jsonl &&
timeout -k 10 300 python3 -u tools/probe/tiny_kernels.py --procs 1,2,3,4,8 --nblocks 64 --us 20 > $out/tiny_64x20.jsonl 2> $out/tiny_64x20.err &&
cat $out/tiny_64x20.jsonl
