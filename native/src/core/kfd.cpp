#include "vgpu/kfd.h"

#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <sys/file.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "vgpu/log.h"

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
  int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return -1;
  char buf[32];
  ssize_t n = read(fd, buf, sizeof(buf) - 1);
  close(fd);
  if (n <= 0) return -1;
  buf[n] = 0;
  char* end = nullptr;
  long long v = strtoll(buf, &end, 10);
  return end == buf ? -1 : v;
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

std::vector<int> kfd_pids_on_gpu(uint32_t gpu_id) {
  std::vector<int> out;
  char path[256];
  for (int p : kfd_list_pids()) {
    snprintf(path, sizeof(path), "%s/%d/stats_%u", g_kfd_proc_root, p, gpu_id);
    if (access(path, F_OK) == 0) out.push_back(p);  // not stat (GLIBC_2.33, glibc_compat.h)
  }
  return out;
}

int kfd_lock(const char* path, int timeout_ms) {
  if (!path || !*path) return kLockUnavailable;
  // In a pod the plugin bind-mounts a lock file it created, read-only: tenants can take
  // the lock (flock works on a read-only descriptor) but cannot unlink or replace it.
  int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) {
    // Outside a pod: create it, world-accessible (processes of one container may run as
    // different users). The process umask is left alone - it is shared with the
    // application's threads - and the modes are set explicitly on what this call created.
    std::string dir(path);
    size_t slash = dir.rfind('/');
    if (slash != std::string::npos && slash > 0) {
      dir.resize(slash);
      if (mkdir(dir.c_str(), 0700) == 0) chmod(dir.c_str(), 01777);
    }
    fd = open(path, O_RDWR | O_CREAT | O_EXCL | O_CLOEXEC, 0600);
    if (fd >= 0) fchmod(fd, 0666);
    else fd = open(path, O_RDONLY | O_CLOEXEC);  // created by someone else meanwhile
  }
  if (fd < 0) return kLockUnavailable;
  // flock is released by the kernel when the holder dies: no expiry heuristic needed
  // (the reference's lock file carries a timestamp and is broken after a timeout).
  for (int waited = 0;; waited++) {
    if (flock(fd, LOCK_EX | LOCK_NB) == 0) return fd;
    if (errno != EWOULDBLOCK || waited >= timeout_ms) break;
    struct timespec ts = {0, 1000000};
    nanosleep(&ts, nullptr);
  }
  close(fd);
  return kLockBusy;
}

void kfd_unlock(int fd) {
  if (fd < 0) return;
  flock(fd, LOCK_UN);
  close(fd);
}

pid_t kfd_resolve_hostpid(uint32_t gpu_id, VramProbe probe, void* ctx, const char* lock_path, int lock_timeout_ms,
                          unsigned seed) {
  const pid_t self = getpid();
  std::vector<int> pids = kfd_list_pids();
  if (std::binary_search(pids.begin(), pids.end(), (int)self)) return self;
  if (!probe || !gpu_id) return 0;
  // The lock only keeps concurrent probes from blurring each other's signatures; a
  // holder that never lets go (any tenant can flock the node-wide file) must not stop
  // this process from resolving its host PID, so after the wait the search runs
  // unlocked: each candidate must match two different random sizes, which another
  // process's concurrent probe does not.
  int lock = lock_path && *lock_path ? kfd_lock(lock_path, lock_timeout_ms) : kLockUnavailable;
  if (lock == kLockBusy) VLOG_INFO("host-PID discovery: lock %s still busy after %d ms, probing unlocked", lock_path,
                                   lock_timeout_ms);
  std::vector<int> cand;
  for (int p : pids)
    if (kfd_vram_usage(p, gpu_id) >= 0) cand.push_back(p);
  constexpr uint64_t kUnit = 2ull << 20;  // KFD/ROCr VRAM granularity for large buffers
  unsigned rng = seed ? seed : (unsigned)self * 2654435761u;
  uint64_t prev = 0;
  pid_t found = 0;
  for (int round = 0; round < 4 && !cand.empty(); round++) {
    rng = rng * 1103515245u + 12345u;
    uint64_t size = kUnit * (3 + (rng >> 8) % 61);  // 6..126 MiB, unlikely to match anyone else
    if (size == prev) size += kUnit;
    prev = size;
    std::vector<int64_t> before(cand.size());
    for (size_t i = 0; i < cand.size(); i++) before[i] = kfd_vram_usage(cand[i], gpu_id);
    if (!probe(ctx, size, true)) break;
    std::vector<int> keep;
    for (size_t i = 0; i < cand.size(); i++) {
      int64_t after = kfd_vram_usage(cand[i], gpu_id);
      if (before[i] >= 0 && after >= 0 && (uint64_t)(after - before[i]) >= size &&
          (uint64_t)(after - before[i]) < size + kUnit)
        keep.push_back(cand[i]);
    }
    probe(ctx, size, false);
    cand.swap(keep);
    // One survivor confirmed by at least two different sizes.
    if (cand.size() == 1 && round >= 1) {
      found = cand[0];
      break;
    }
  }
  kfd_unlock(lock);
  if (found) VLOG_INFO("host PID %d (VRAM signature on gpu_id %u)", (int)found, gpu_id);
  return found;
}

}  // namespace vgpu
