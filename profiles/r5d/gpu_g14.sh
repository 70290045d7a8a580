# Round-5 GPU study (profiles/r5d, part 6): is the same-socket serialisation of two PyTorch
# launch-bound tenants a per-socket or a per-L3 (CCD) effect? Pairs pinned within one L3
# domain, on two L3 domains of the GPU's socket, and on SMT siblings.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5d
mkdir -p $O
python3 tools/probe/cotenancy.py --l3 | tee $O/l3_domains.json
eval "$(python3 - <<'PY'
import json, os, sys
sys.path.insert(0, "tools/probe"); sys.path.insert(0, ".")
import cotenancy as c
def parse(t):
    out = []
    for part in t.strip().split(","):
        lo, _, hi = part.partition("-")
        out += list(range(int(lo), int(hi or lo) + 1))
    return out
n, g = c._numa_nodes(), c._gpu_node()
local = set(n.get(g, []))
doms = []
for cpu in sorted(local):
    d = tuple(parse(open(f"/sys/devices/system/cpu/cpu{cpu}/cache/index3/shared_cpu_list").read()))
    if d not in doms:
        doms.append(d)
def phys(d):   # one thread per core, in order
    seen, out = set(), []
    for cpu in d:
        sib = tuple(parse(open(f"/sys/devices/system/cpu/cpu{cpu}/topology/thread_siblings_list").read()))
        if sib not in seen:
            seen.add(sib); out.append(cpu)
    return out
d0, d1 = phys(doms[0]), phys(doms[1])
sib = parse(open(f"/sys/devices/system/cpu/cpu{d0[0]}/topology/thread_siblings_list").read())
fmt = lambda xs: ",".join(map(str, xs))
print(f'SAME_L3="{fmt(d0[0:4])};{fmt(d0[4:8])}"')
print(f'TWO_L3="{fmt(d0[0:4])};{fmt(d1[0:4])}"')
print(f'SMT="{sib[0]};{sib[-1]}"')
print(f'ONE_EACH_L3="{d0[0]};{d1[0]}"')
print(f'ONE_SAME_L3="{d0[0]};{d0[1]}"')
PY
)"
echo "same L3: $SAME_L3 | two L3: $TWO_L3 | SMT: $SMT" | tee $O/l3_pairs.txt
C="timeout -k 10 240 python3 -u tools/probe/cotenancy.py --seconds 4 --procs 2"
for c in lstm-inf resnet152-inf; do
  for v in SAME_L3 TWO_L3 SMT ONE_EACH_L3 ONE_SAME_L3; do
    $C --case $c --cpu-lists "${!v}" > $O/l3_${c}_$v.json 2> $O/l3_${c}_$v.err || exit $?
    tail -1 $O/l3_${c}_$v.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('$c $v ${!v}', d['aggregate_items_per_s'], [t['items_per_s'] for t in d['tenants']])" | tee -a $O/l3_pairs.txt
  done
done
