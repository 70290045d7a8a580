#!/bin/bash
# Installs the data plane onto the host (hostPath /usr/local/vgpu) and starts the plugin.
# Reference: entrypoint.sh:1-3 (cp -f /etc/vgpu/* /usr/local/vgpu/ ; exec plugin).
set -euo pipefail
DEST=${VGPU_DIR:-/usr/local/vgpu}
mkdir -p "$DEST" "$DEST/shared" "$DEST/allowlist"
# Atomic replace: containers that already mapped the old shim keep their inode.
for f in libvgpu_hip.so libvgpu_region.so vgpu-validate vgpuctl ld.so.preload; do
  install -m 0755 "/opt/amd-vgpu/lib/$f" "$DEST/.$f.new" && mv -f "$DEST/.$f.new" "$DEST/$f"
done
chmod 0644 "$DEST/ld.so.preload"
# Device allow-list for vgpu-validate (ROCr UUIDs of this node's GPUs).
python3 -c 'import sys; sys.path.insert(0, "/opt/amd-vgpu")
from amdvgpu.plugin.devices import SysfsBackend
print("\n".join(d.uuid for d in SysfsBackend().devices()))' > "$DEST/allowlist/allowlist" || true
exec python3 -m amdvgpu.plugin.main "$@"
