# Round-5 GPU study (profiles/r5d, part 5): the launch cost of an empty kernel from C++
# (native/tests/hip_launch_probe.hip), alone and with a second launcher on the same socket or
# on the other one, to separate HIP's launch path from PyTorch.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5d
mkdir -p $O
L=4paradigm-k8s-device-plugin_amd/lib/hip_launch_probe
read LOCAL REMOTE < <(python3 - <<'PY'
import sys; sys.path.insert(0, "tools/probe"); sys.path.insert(0, ".")
import cotenancy as c
n, g = c._numa_nodes(), c._gpu_node()
loc = n.get(g, [])
rem = [x for k, cs in sorted(n.items()) if k != g for x in cs]
print(loc[0], rem[0])
PY
)
L2=$((LOCAL + 4)); R2=$((REMOTE + 4))
echo "gpu-local cpu $LOCAL, remote cpu $REMOTE" | tee $O/launch_probe.txt
one() { timeout -k 5 120 taskset -c $1 $L 400000 1000; }
pair() { one $1 > /tmp/p1.txt & a=$!; one $2 > /tmp/p2.txt & b=$!; wait $a && wait $b && echo "$(cat /tmp/p1.txt) $(cat /tmp/p2.txt)"; }
{
echo "alone local: $(one $LOCAL)" &&
echo "alone remote: $(one $REMOTE)" &&
echo "pair local+local: $(pair $LOCAL $L2)" &&
echo "pair remote+remote: $(pair $REMOTE $R2)" &&
echo "pair local+remote: $(pair $LOCAL $REMOTE)" &&
export GPU_MAX_HW_QUEUES=1 &&
echo "hwq1 pair local+local: $(pair $LOCAL $L2)" &&
unset GPU_MAX_HW_QUEUES &&
export HSA_ENABLE_INTERRUPT=0 &&
echo "nointr pair local+local: $(pair $LOCAL $L2)"
} 2>&1 | tee -a $O/launch_probe.txt
# CPU placement vs host-memory placement, for the PyTorch LSTM pair
C="timeout -k 10 240 python3 -u tools/probe/cotenancy.py --seconds 4 --case lstm-inf --procs 2"
for v in "local split" "remote split" "split local" "split remote" "local local"; do
  set -- $v
  $C --placement $1 --mem $2 > $O/mem_$1_$2.json 2> $O/mem_$1_$2.err || exit $?
  tail -1 $O/mem_$1_$2.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('cpus $1 mem $2', d['aggregate_items_per_s'], [t['items_per_s'] for t in d['tenants']])" | tee -a $O/launch_probe.txt
done
