// vGPU index map (VGPU_DEVICE_MAP = "0:<uuid> 1:<uuid> ...").
//
// Reference: libvgpu.so src/nvml/util.c parser@0x28a39 [230-271],
// initial_virtual_devices@0x27f0d [135-162] (max 16 entries, duplicate physical
// device detection "device index %d and %d are the same physical device").
//
// The reference then fabricates duplicate virtual devices. On MI355X the shim
// instead resolves the map onto the real visible GPU agents (matched by ROCr UUID
// "GPU-<hex>") and, when two vGPUs land on one physical GPU, merges their quotas
// and CU shares into that one device (no fake duplicate devices that would break
// cooperative launch or RCCL peer setup).
#pragma once

#include "vgpu/config.h"

namespace vgpu {

struct DeviceMapEntry {
  int vidx = -1;
  char uuid[64] = {0};
};

struct DeviceMap {
  int n = 0;
  DeviceMapEntry e[kMaxDevices];
  int duplicates = 0;  // entries whose UUID repeats an earlier one
};

// Returns false on malformed input or more than kMaxDevices entries.
bool parse_device_map(const char* s, DeviceMap* out);

// Normalises a UUID for comparison: lower-case, strips a "GPU-" prefix.
void normalize_uuid(const char* in, char* out, int outlen);

// Resolves per-agent (HIP ordinal) device configs. `agent_uuids[k]` is the ROCr
// UUID of visible GPU agent k. Positional fallback (config index == ordinal) when
// the map is empty or a UUID is not found. Returns the number of resolved agents.
int resolve_devices(const Config& cfg, const DeviceMap& map, const char* const* agent_uuids,
                    int n_agents, DeviceConfig* out);

}  // namespace vgpu
