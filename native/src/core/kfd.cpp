#include "vgpu/kfd.h"

#include <dirent.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

namespace vgpu {

const char* g_kfd_proc_root = "/sys/class/kfd/kfd/proc";

std::vector<int> kfd_list_pids() {
  std::vector<int> v;
  DIR* d = opendir(g_kfd_proc_root);
  if (!d) return v;
  while (struct dirent* e = readdir(d)) {
    char* end = nullptr;
    long p = strtol(e->d_name, &end, 10);
    if (end != e->d_name && !*end && p > 0) v.push_back((int)p);
  }
  closedir(d);
  std::sort(v.begin(), v.end());
  return v;
}

pid_t kfd_diff_pid(const std::vector<int>& before, const std::vector<int>& after) {
  pid_t found = 0;
  int n = 0;
  for (int p : after) {
    if (!std::binary_search(before.begin(), before.end(), p)) {
      found = p;
      n++;
    }
  }
  return n == 1 ? found : 0;
}

static int64_t read_i64(const char* path) {
  FILE* f = fopen(path, "r");
  if (!f) return -1;
  long long v = -1;
  if (fscanf(f, "%lld", &v) != 1) v = -1;
  fclose(f);
  return v;
}

int64_t kfd_cu_occupancy(pid_t hostpid, uint32_t gpu_id) {
  char path[256];
  snprintf(path, sizeof(path), "%s/%d/stats_%u/cu_occupancy", g_kfd_proc_root, (int)hostpid, gpu_id);
  return read_i64(path);
}

int64_t kfd_vram_usage(pid_t hostpid, uint32_t gpu_id) {
  char path[256];
  snprintf(path, sizeof(path), "%s/%d/vram_%u", g_kfd_proc_root, (int)hostpid, gpu_id);
  return read_i64(path);
}

}  // namespace vgpu
