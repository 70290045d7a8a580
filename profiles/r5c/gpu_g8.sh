# Round-5 GPU study (profiles/r5c): the 16-pod point with stock waits - every sweep pod calls
# torch's synchronize (VGPU_BENCH_SYNC=spin, the bench's default now) and the shim polls the
# waits of pods on a crowded GPU - ten times over two bench runs.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/r5c
mkdir -p $out
for run in 1 2; do
  timeout -k 10 560 python -u bench.py --modes native --sweep on --sweep-tenants 1,16,16,16,16,16 --rccl-probe 0 \
    --time-budget 520 --json-out "$out/spin$run.json" > "$out/spin$run.log" 2>&1
  rc=$?
  echo "bench_rc=$rc" >> "$out/spin$run.log"
  tail -2 "$out/spin$run.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
done
