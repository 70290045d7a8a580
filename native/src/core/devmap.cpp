#include "vgpu/devmap.h"

#include <cctype>
#include <cstdio>
#include <cstring>

#include "vgpu/log.h"

namespace vgpu {

void normalize_uuid(const char* in, char* out, int outlen) {
  if (!in) in = "";
  if (!strncasecmp(in, "GPU-", 4)) in += 4;
  int i = 0;
  for (; in[i] && i < outlen - 1; i++) out[i] = (char)tolower((unsigned char)in[i]);
  out[i] = 0;
}

bool parse_device_map(const char* s, DeviceMap* out) {
  *out = DeviceMap();
  if (!s) return true;
  const char* p = s;
  while (*p) {
    while (*p == ' ' || *p == ',' || *p == ';') p++;
    if (!*p) break;
    const char* tok = p;
    while (*p && *p != ' ' && *p != ',' && *p != ';') p++;
    size_t len = (size_t)(p - tok);
    char buf[128];
    if (len >= sizeof(buf)) return false;
    memcpy(buf, tok, len);
    buf[len] = 0;
    char* colon = strchr(buf, ':');
    if (!colon) return false;
    *colon = 0;
    char* end = nullptr;
    long v = strtol(buf, &end, 10);
    if (end == buf || *end || v < 0 || v >= kMaxDevices) return false;
    if (out->n >= kMaxDevices) {
      VLOG_ERROR("Max GPUs per node can't exceed %d", kMaxDevices);
      return false;
    }
    DeviceMapEntry& e = out->e[out->n];
    e.vidx = (int)v;
    snprintf(e.uuid, sizeof(e.uuid), "%s", colon + 1);
    for (int j = 0; j < out->n; j++) {
      char a[64], b[64];
      normalize_uuid(out->e[j].uuid, a, sizeof(a));
      normalize_uuid(e.uuid, b, sizeof(b));
      if (!strcmp(a, b)) {
        VLOG_WARN("device index %d and %d are the same physical device", out->e[j].vidx, e.vidx);
        out->duplicates++;
        break;
      }
    }
    out->n++;
  }
  return true;
}

int resolve_devices(const Config& cfg, const DeviceMap& map, const char* const* agent_uuids,
                    int n_agents, DeviceConfig* out) {
  if (n_agents > kMaxDevices) n_agents = kMaxDevices;
  for (int k = 0; k < n_agents; k++) {
    out[k] = DeviceConfig();
    char au[64];
    normalize_uuid(agent_uuids ? agent_uuids[k] : "", au, sizeof(au));
    bool matched = false;
    if (au[0]) {
      for (int j = 0; j < map.n; j++) {
        char mu[64];
        normalize_uuid(map.e[j].uuid, mu, sizeof(mu));
        if (strcmp(mu, au)) continue;
        const DeviceConfig& c = cfg.dev[map.e[j].vidx];
        if (!matched) {
          out[k] = c;
          matched = true;
        } else if (cfg.duplicate_merge) {
          // Second vGPU of the same physical GPU: merge quota and CU share.
          if (out[k].mem_limit && c.mem_limit) out[k].mem_limit += c.mem_limit;
          else out[k].mem_limit = 0;
          if (out[k].hbm_limit && c.hbm_limit) out[k].hbm_limit += c.hbm_limit;
          else out[k].hbm_limit = 0;
          int pct = out[k].cu_limit_pct + c.cu_limit_pct;
          out[k].cu_limit_pct = (out[k].cu_limit_pct && c.cu_limit_pct && pct < 100) ? pct : 0;
          // Adjacent CU ranges from the plugin collapse into one; anything else falls
          // back to the merged percentage.
          if (out[k].cu_range_begin >= 0 && c.cu_range_begin >= 0 &&
              (out[k].cu_range_end == c.cu_range_begin || c.cu_range_end == out[k].cu_range_begin)) {
            int b = out[k].cu_range_begin < c.cu_range_begin ? out[k].cu_range_begin : c.cu_range_begin;
            int e = out[k].cu_range_end > c.cu_range_end ? out[k].cu_range_end : c.cu_range_end;
            out[k].cu_range_begin = b;
            out[k].cu_range_end = e;
          } else {
            out[k].cu_range_begin = out[k].cu_range_end = -1;
          }
        }
      }
    }
    // No map: positional. With a map, an agent it does not name is not one of the
    // container's vGPUs (only reachable if visibility was widened inside the container).
    if (!matched && map.n == 0) out[k] = cfg.dev[k];
    if (!matched && map.n > 0) out[k].unmapped = true;
    if (agent_uuids && agent_uuids[k]) snprintf(out[k].uuid, sizeof(out[k].uuid), "%s", agent_uuids[k]);
  }
  return n_agents;
}

}  // namespace vgpu
