// vgpu-validate: device-authorisation check for a vGPU container.
//
// Reference: vgpu/vgpuvalidator [validator.c:10-111] decrypts /vgpu/license and
// checks each visible device UUID against an authorised pool ("device %s
// authorized" / "uuid %s UNAUTHORIZED"); `--decode` dumps the list. The MI355X build
// keeps the authorisation capability and drops the commercial AES licensing: the
// plugin writes a plain allow-list of ROCr UUIDs (one per line) and this tool checks
// the GPUs ROCr exposes to the container against it. ROCr is loaded with dlopen so
// the tool has no build-time GPU dependency.
//
//   vgpu-validate [--allowlist FILE]   exit 0 iff every visible GPU is authorised
//   vgpu-validate --decode [FILE]      print the allow-list
//   vgpu-validate --list               print the visible GPU UUIDs
#include <dlfcn.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <cctype>
#include <cstdio>
#include <cstring>
#include <set>
#include <string>
#include <vector>

static std::string norm(std::string s) {
  while (!s.empty() && isspace((unsigned char)s.back())) s.pop_back();
  size_t i = 0;
  while (i < s.size() && isspace((unsigned char)s[i])) i++;
  s = s.substr(i);
  if (s.size() >= 4 && !strncasecmp(s.c_str(), "GPU-", 4)) s = s.substr(4);
  for (auto& c : s) c = (char)tolower((unsigned char)c);
  return s;
}

static bool read_allowlist(const char* path, std::vector<std::string>* out) {
  FILE* f = fopen(path, "r");
  if (!f) return false;
  char line[256];
  while (fgets(line, sizeof(line), f)) {
    std::string s = line;
    if (s.empty() || s[0] == '#') continue;
    s = norm(s);
    if (!s.empty()) out->push_back(s);
  }
  fclose(f);
  return true;
}

using init_fn = hsa_status_t (*)();
using iter_fn = hsa_status_t (*)(hsa_status_t (*)(hsa_agent_t, void*), void*);
using info_fn = hsa_status_t (*)(hsa_agent_t, hsa_agent_info_t, void*);
static info_fn g_info;

static hsa_status_t agent_cb(hsa_agent_t a, void* data) {
  hsa_device_type_t t;
  if (g_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS || t != HSA_DEVICE_TYPE_GPU) return HSA_STATUS_SUCCESS;
  char uuid[64] = {0};
  g_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_UUID, uuid);
  static_cast<std::vector<std::string>*>(data)->push_back(uuid);
  return HSA_STATUS_SUCCESS;
}

static bool visible_gpus(std::vector<std::string>* out) {
  void* h = dlopen("libhsa-runtime64.so.1", RTLD_NOW | RTLD_LOCAL);
  if (!h) h = dlopen("/opt/rocm/lib/libhsa-runtime64.so.1", RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    fprintf(stderr, "vgpu-validate: cannot load ROCr: %s\n", dlerror());
    return false;
  }
  auto init = (init_fn)dlsym(h, "hsa_init");
  auto iter = (iter_fn)dlsym(h, "hsa_iterate_agents");
  g_info = (info_fn)dlsym(h, "hsa_agent_get_info");
  if (!init || !iter || !g_info || init() != HSA_STATUS_SUCCESS) {
    fprintf(stderr, "vgpu-validate: ROCr initialisation failed\n");
    return false;
  }
  iter(agent_cb, out);
  return true;
}

int main(int argc, char** argv) {
  const char* allow = "/vgpu/allowlist";
  bool decode = false, list = false;
  for (int i = 1; i < argc; i++) {
    if (!strcmp(argv[i], "--decode")) {
      decode = true;
      if (i + 1 < argc && argv[i + 1][0] != '-') allow = argv[++i];
    } else if (!strcmp(argv[i], "--allowlist") && i + 1 < argc) {
      allow = argv[++i];
    } else if (!strcmp(argv[i], "--list")) {
      list = true;
    } else {
      fprintf(stderr, "usage: vgpu-validate [--allowlist FILE] | --decode [FILE] | --list\n");
      return 2;
    }
  }
  std::vector<std::string> allowed;
  if (decode) {
    if (!read_allowlist(allow, &allowed)) {
      fprintf(stderr, "vgpu-validate: cannot read %s\n", allow);
      return 1;
    }
    for (auto& a : allowed) printf("GPU-%s\n", a.c_str());
    return 0;
  }
  std::vector<std::string> gpus;
  if (!visible_gpus(&gpus)) return 1;
  if (list) {
    for (auto& g : gpus) printf("%s\n", g.c_str());
    return 0;
  }
  if (!read_allowlist(allow, &allowed)) {
    fprintf(stderr, "vgpu-validate: cannot read allow-list %s\n", allow);
    return 1;
  }
  std::set<std::string> ok(allowed.begin(), allowed.end());
  int bad = 0;
  for (auto& g : gpus) {
    if (ok.count(norm(g))) {
      printf("device %s authorized\n", g.c_str());
    } else {
      printf("uuid %s UNAUTHORIZED\n", g.c_str());
      bad++;
    }
  }
  return bad ? 1 : 0;
}
