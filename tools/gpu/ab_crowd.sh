#!/bin/bash
# A/B of the 4-pod crowded point: round-5 tree vs HEAD, and HEAD with single features off.
set -o pipefail
OUT=gpurun_out/r6c; mkdir -p $OUT
export TMPDIR=/tmp
run() { # tag dir extra-args...
  local tag=$1 dir=$2; shift 2
  echo "== $tag $(date +%T)"
  (cd $dir && timeout -k 10 200 python bench.py --gpus 1 --steps 10 --warmup 3 --modes native --sweep on \
     --sweep-tenants 1,4 --sweep-seconds 5 --time-budget 180 --json-out /root/repo/$OUT/$tag.json "$@" \
     > /root/repo/$OUT/$tag.log 2>&1) || { echo "$tag failed rc=$?"; tail -5 $OUT/$tag.log; return 1; }
  python - $OUT/$tag.json <<'PY'
import json,sys
d=json.load(open(sys.argv[1]))
for r in d["sweep"]:
    if r["tenants"]==4: print({k:r.get(k) for k in ("aggregate_vs_one","min_tenant_vs_entitlement","cpus_busy","granted_pct","throttled_pct")})
PY
}
run r5 ab_r5 && run head . && run head_nospread . --sweep-pod-env VGPU_CPU_SPREAD=0 && run head_nodlsym . --sweep-pod-env VGPU_HOOK_DLSYM=0 && run r5_again ab_r5
