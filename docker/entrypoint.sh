#!/bin/bash
# Installs the data plane onto the host (hostPath /usr/local/vgpu) and starts the plugin.
# Reference: entrypoint.sh:1-3 (cp -f /etc/vgpu/* /usr/local/vgpu/ ; exec plugin).
set -euo pipefail
SRC=${VGPU_LIB_DIR:-/opt/amd-vgpu/4paradigm-k8s-device-plugin_amd/lib}
DEST=${VGPU_DIR:-/usr/local/vgpu}
mkdir -p "$DEST" "$DEST/shared" "$DEST/allowlist/containers" "$DEST/lock" "$DEST/board"
chmod 0755 "$DEST/board"   # node-wide board: each container writes only its own slot
# Host-PID discovery lock: root-owned and mounted read-only into every container (flock
# works on a read-only descriptor; tenants cannot unlink or replace it).
[ -e "$DEST/lock/hostpid.lock" ] || : > "$DEST/lock/hostpid.lock"
chmod 0755 "$DEST/lock"
chmod 0644 "$DEST/lock/hostpid.lock"
# Atomic replace: containers that already mapped the old shim keep their inode.
for f in libvgpu_hip.so libvgpu_region.so vgpu-validate vgpuctl ld.so.preload; do
  install -m 0755 "$SRC/$f" "$DEST/.$f.new" && mv -f "$DEST/.$f.new" "$DEST/$f"
done
chmod 0644 "$DEST/ld.so.preload"
# Node-wide allow-list (fallback when a per-container list cannot be written): ROCr UUIDs
# of this node's GPUs. The plugin writes each container's own list under containers/.
python3 -c 'import sys; sys.path.insert(0, "/opt/amd-vgpu")
from amdvgpu.plugin.devices import SysfsBackend
print("\n".join(d.uuid for d in SysfsBackend().devices()))' > "$DEST/allowlist/allowlist" || true
exec python3 -m amdvgpu.plugin.main "$@"
