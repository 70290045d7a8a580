#!/bin/bash
# Round-3: pod warm-up under a crowded GPU is MIOpen's find (cudnn.benchmark) run by every
# pod on its 1/N of the GPU. With one find-db shared by the pods (filled by the lone
# reference pod first), do 12 and 16 pods warm up faster, and is the spread between pods
# (different pods picking different conv algorithms under contention?) narrower?
# MIOpen keys its find-db by the CU count the device reports (gfx950_<CUs>), and a split-N
# pod reports its slice: with [split] set, the lone pod is a split-N pod too, so it fills
# the very db entries the N pods look up.
#   bash profiles/r3q/r3_finddb.sh <out> <tenants> [split]
out=${1:-gpurun_out/r3o}
tenants=${2:-1,12,16}
split=${3:+--split $3}
mkdir -p "$out"
{
  echo "HOME=$HOME"
  ls -la "$HOME/.config/miopen" "$HOME/.cache/miopen" 2>&1
} > "$out/env.txt"
db=$(mktemp -d /tmp/miopen-db.XXXXXX)
export MIOPEN_USER_DB_PATH="$db/db" MIOPEN_CUSTOM_CACHE_DIR="$db/cache"
mkdir -p "$MIOPEN_USER_DB_PATH" "$MIOPEN_CUSTOM_CACHE_DIR"
timeout -k 10 1000 python -u benchmarks/vgpu_scaling.py --policy default --seconds 10 --tenants "$tenants" $split \
  --json-out "$out/finddb.json" --md-out "$out/finddb.md" > "$out/finddb.log" 2>&1
rc=$?
ls -la "$MIOPEN_USER_DB_PATH" >> "$out/env.txt" 2>&1
exit $rc
