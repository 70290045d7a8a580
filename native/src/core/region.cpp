// Shared accounting region. Behavioural parity target: libvgpu.so
// src/multiprocess/multiprocess_memory_limit.c (try_create_shrreg [645-741],
// lock_shrreg [516-540], init_proc_slot_withlock, exit_handler [475-494],
// add/rm_gpu_device_memory_usage [359-382], rm_quitted_process [234-248]).
// Design notes are in vgpu/region.h.
#include "vgpu/region.h"

#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <sys/file.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>

#include "vgpu/cumask.h"
#include "vgpu/log.h"

namespace vgpu {

uint64_t proc_start_time(pid_t pid) {
  char path[64];
  snprintf(path, sizeof(path), "/proc/%d/stat", (int)pid);
  FILE* f = fopen(path, "r");
  if (!f) return 0;
  char buf[1024];
  size_t n = fread(buf, 1, sizeof(buf) - 1, f);
  fclose(f);
  buf[n] = 0;
  // comm may contain spaces/parens: fields restart after the last ')'.
  char* p = strrchr(buf, ')');
  if (!p) return 0;
  p++;
  // After ')' come fields 3.. ; start time is field 22 -> 20th token after ')'.
  int field = 2;
  char* save = nullptr;
  for (char* tok = strtok_r(p, " ", &save); tok; tok = strtok_r(nullptr, " ", &save)) {
    field++;
    if (field == 22) return strtoull(tok, nullptr, 10);
  }
  return 0;
}

bool proc_alive(pid_t pid, uint64_t start_time) {
  if (pid <= 0) return false;
  if (kill(pid, 0) != 0 && errno == ESRCH) return false;
  if (start_time) {
    uint64_t st = proc_start_time(pid);
    if (st && st != start_time) return false;  // PID was reused
  }
  return true;
}

uint64_t self_pidns() {
  static const uint64_t ns = [] {
    char buf[64];
    ssize_t n = readlink("/proc/self/ns/pid", buf, sizeof(buf) - 1);
    if (n <= 0) return (uint64_t)0;
    buf[n] = 0;
    const char* p = strchr(buf, '[');
    return p ? (uint64_t)strtoull(p + 1, nullptr, 10) : (uint64_t)0;
  }();
  return ns;
}

namespace {

// Whether a slot's process has exited, judged from the caller's PID namespace. A slot
// records the PID in its own (container) namespace; a caller in another namespace (the
// node monitor, vgpuctl on the host) must not look that PID up in its own /proc, where
// it names an unrelated process or none (the slot of a live tenant would be freed and
// its charges dropped). From the host namespace the slot's host PID is checked; from any
// other namespace the slot is kept.
bool slot_exited(const ProcSlot& s) {
  const int32_t pid = s.pid.load();
  const uint64_t me = self_pidns();
  if (!s.pidns || !me || s.pidns == me) return !proc_alive(pid, s.start_time);
  const int32_t hp = s.hostpid.load();
  if (me == kInitPidNs && hp > 0) return !proc_alive(hp, s.start_time);  // start time is namespace-independent
  return false;
}

}  // namespace

SharedRegion::~SharedRegion() { detach(); }

void SharedRegion::init_mutex(pthread_mutex_t* m) {
  pthread_mutexattr_t a;
  pthread_mutexattr_init(&a);
  pthread_mutexattr_setpshared(&a, PTHREAD_PROCESS_SHARED);
  pthread_mutexattr_setrobust(&a, PTHREAD_MUTEX_ROBUST);
  pthread_mutex_init(m, &a);
  pthread_mutexattr_destroy(&a);
}

int SharedRegion::attach(const char* path, const Config* cfg, bool create) {
  detach();
  snprintf(path_, sizeof(path_), "%s", path);
  mode_t old = umask(0);
  int fd = open(path, O_RDWR | (create ? O_CREAT : 0) | O_CLOEXEC, 0666);
  umask(old);
  if (fd < 0) return -errno;
  // Serialise creation/initialisation with an advisory file lock (reference: lockf).
  if (flock(fd, LOCK_EX) != 0) {
    int e = errno;
    close(fd);
    return -e;
  }
  // File size by lseek, not fstat: fstat is a GLIBC_2.33 symbol, and this code runs in
  // tenant images with older C libraries (glibc_compat.h).
  const off_t fsize = lseek(fd, 0, SEEK_END);
  if (fsize < 0) {
    int e = errno;
    flock(fd, LOCK_UN);
    close(fd);
    return -e;
  }
  // A file shorter than the layout was never fully initialised or was cut short: its
  // header may still look valid while the limits behind it read as 0 (= unlimited), so it
  // is rebuilt from the environment rather than trusted.
  const bool short_file = (size_t)fsize < sizeof(Region);
  if (short_file) {
    if (!create || ftruncate(fd, sizeof(Region)) != 0) {
      int e = create ? errno : EINVAL;
      flock(fd, LOCK_UN);
      close(fd);
      return -e;
    }
  }
  void* p = mmap(nullptr, sizeof(Region), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (p == MAP_FAILED) {
    int e = errno;
    flock(fd, LOCK_UN);
    close(fd);
    return -e;
  }
  r_ = static_cast<Region*>(p);
  fd_ = fd;
  if (r_->hdr.magic != kRegionMagic || short_file) {
    if (!create) {
      munmap(p, sizeof(Region));
      r_ = nullptr;
      flock(fd, LOCK_UN);
      close(fd);
      fd_ = -1;
      return -EINVAL;
    }
    init_fresh(cfg);
  } else if (r_->hdr.version != kRegionVersion || r_->hdr.region_size != sizeof(Region)) {
    VLOG_ERROR("shared region %s has layout v%u/%lu, this shim expects v%u/%zu", path,
               r_->hdr.version, (unsigned long)r_->hdr.region_size, kRegionVersion, sizeof(Region));
    munmap(p, sizeof(Region));
    r_ = nullptr;
    flock(fd, LOCK_UN);
    close(fd);
    fd_ = -1;
    return -EPROTO;
  } else if (cfg) {
    check_consistency(cfg);
  }
  flock(fd, LOCK_UN);
  return 0;
}

void SharedRegion::detach() {
  if (r_) munmap(r_, sizeof(Region));
  if (fd_ >= 0) close(fd_);
  r_ = nullptr;
  fd_ = -1;
}

void SharedRegion::init_fresh(const Config* cfg) {
  memset(static_cast<void*>(r_), 0, sizeof(Region));
  r_->hdr.version = kRegionVersion;
  r_->hdr.region_size = sizeof(Region);
  init_mutex(&r_->hdr.mutex);
  r_->hdr.utilization_switch.store(1);
  r_->hdr.recent_kernel.store(2);
  r_->hdr.priority.store(cfg ? cfg->priority : 1);
  uint32_t flags = 0;
  if (cfg && cfg->oversubscribe) flags |= kFlagOversubscribe;
  if (cfg && cfg->active_oom_killer) flags |= kFlagActiveOomKiller;
  r_->hdr.flags = flags;
  r_->hdr.host_limit = cfg ? cfg->host_mem_limit : 0;
  int n = 0;
  if (cfg) {
    for (int i = 0; i < kMaxDevices; i++) {
      DeviceState& d = r_->dev[i];
      d.mem_limit = cfg->dev[i].mem_limit;
      d.hbm_limit = cfg->dev[i].hbm_limit;
      d.cu_limit_pct = cfg->dev[i].cu_limit_pct;
      d.cu_share_bp = cfg->dev[i].cu_share_bp;
      d.cu_range_begin = cfg->dev[i].cu_range_begin;
      d.cu_range_end = cfg->dev[i].cu_range_end;
      memcpy(d.uuid, cfg->dev[i].uuid, sizeof(d.uuid));
      d.uuid[sizeof(d.uuid) - 1] = 0;
      d.crowd.store(-1);
    }
    n = cfg->num_devices;
  } else {
    for (int i = 0; i < kMaxDevices; i++) {
      r_->dev[i].cu_range_begin = r_->dev[i].cu_range_end = -1;
      r_->dev[i].crowd.store(-1);
    }
  }
  r_->hdr.num_devices = n;
  {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    uint64_t e = ((uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec) ^ ((uint64_t)getpid() << 40) ^
                 (uint64_t)(uintptr_t)this;
    e ^= e >> 29;
    e *= 0xbf58476d1ce4e5b9ull;
    r_->hdr.epoch = e ^ (e >> 32);
  }
  r_->hdr.initialized.store(1);
  std::atomic_thread_fence(std::memory_order_release);
  r_->hdr.magic = kRegionMagic;  // published last
}

void SharedRegion::check_consistency(const Config* cfg) {
  // Only devices the region actually describes: a GPU process records the visible agents,
  // while an attach-only process (e.g. amd-smi) carries the raw env for all 16 slots.
  const int n = r_->hdr.num_devices > 0 ? r_->hdr.num_devices : kMaxDevices;
  for (int i = 0; i < n && i < kMaxDevices; i++) {
    uint64_t have = r_->dev[i].mem_limit;
    uint64_t want = cfg->dev[i].mem_limit;
    if (want && have != want) {
      VLOG_WARN("limit inconsistency on device %d: region=%lu env=%lu (region wins)", i,
                (unsigned long)have, (unsigned long)want);
    }
    if (cfg->dev[i].cu_limit_pct && r_->dev[i].cu_limit_pct != cfg->dev[i].cu_limit_pct) {
      VLOG_WARN("CU limit inconsistency on device %d: region=%d env=%d (region wins)", i,
                r_->dev[i].cu_limit_pct, cfg->dev[i].cu_limit_pct);
    }
  }
  if (cfg->host_mem_limit && r_->hdr.host_limit != cfg->host_mem_limit)
    VLOG_WARN("host memory limit inconsistency: region=%lu env=%lu (region wins)",
              (unsigned long)r_->hdr.host_limit, (unsigned long)cfg->host_mem_limit);
  if (cfg->num_devices > r_->hdr.num_devices) r_->hdr.num_devices = cfg->num_devices;
}

bool SharedRegion::lock() {
  int rc = pthread_mutex_lock(&r_->hdr.mutex);
  if (rc == EOWNERDEAD) {
    // The previous owner died inside the critical section. State it protects is
    // either consistent (all updates are single atomics) or repaired by reclaim.
    VLOG_WARN("shared region lock owner died; recovering");
    pthread_mutex_consistent(&r_->hdr.mutex);
    return true;
  }
  if (rc == ENOTRECOVERABLE) {
    VLOG_ERROR("shared region mutex is not recoverable");
    return false;
  }
  return rc == 0;
}

bool SharedRegion::lock_for(int timeout_ms) {
  struct timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);  // pthread_mutex_timedlock's clock
  ts.tv_sec += timeout_ms / 1000;
  ts.tv_nsec += (long)(timeout_ms % 1000) * 1000000L;
  if (ts.tv_nsec >= 1000000000L) {
    ts.tv_sec++;
    ts.tv_nsec -= 1000000000L;
  }
  int rc = pthread_mutex_timedlock(&r_->hdr.mutex, &ts);
  if (rc == EOWNERDEAD) {
    VLOG_WARN("shared region lock owner died; recovering");
    pthread_mutex_consistent(&r_->hdr.mutex);
    return true;
  }
  if (rc == ETIMEDOUT) {
    VLOG_WARN("shared region lock still held after %d ms (holder stopped?); going on without it", timeout_ms);
    return false;
  }
  return rc == 0;
}

void SharedRegion::unlock() { pthread_mutex_unlock(&r_->hdr.mutex); }

int SharedRegion::num_devices() const { return r_ ? r_->hdr.num_devices : 0; }

int SharedRegion::find_slot(pid_t pid) const {
  for (int i = 0; i < kMaxProcs; i++)
    if (r_->procs[i].pid.load(std::memory_order_relaxed) == pid) return i;
  return -1;
}

int SharedRegion::register_process(pid_t pid, pid_t hostpid, int priority) {
  if (!lock()) return -1;
  int slot = -1;
  for (int attempt = 0; attempt < 2 && slot < 0; attempt++) {
    for (int i = 0; i < kMaxProcs; i++) {
      int32_t cur = r_->procs[i].pid.load(std::memory_order_relaxed);
      if (cur == pid) {  // stale slot of a previous process with our PID
        clear_slot_locked(i);
        cur = 0;
      }
      if (cur == 0) {
        slot = i;
        break;
      }
    }
    if (slot < 0) {
      unlock();
      reclaim_dead();
      if (!lock()) return -1;
    }
  }
  if (slot >= 0) {
    ProcSlot& s = r_->procs[slot];
    memset(static_cast<void*>(&s.used), 0, sizeof(s.used));
    s.host_used.store(0);
    s.host_peak.store(0);
    s.launches.store(0);
    s.throttle_ns.store(0);
    s.suspend_ns.store(0);
    s.oom_events.store(0);
    s.priority = priority;
    s.start_time = proc_start_time(pid);
    s.pidns = pid == getpid() ? self_pidns() : 0;  // registered by someone else: unknown
    s.hostpid.store(hostpid);
    s.status.store(r_->hdr.suspend_all.load() ? kProcSuspended : kProcRunning);
    s.pid.store(pid, std::memory_order_release);
    r_->hdr.proc_num.fetch_add(1);
  } else {
    VLOG_ERROR("no free process slot in shared region (%d in use)", kMaxProcs);
  }
  unlock();
  return slot;
}

void SharedRegion::clear_slot_locked(int slot) {
  ProcSlot& s = r_->procs[slot];
  if (s.pid.load() == 0) return;
  for (int d = 0; d < kMaxDevices; d++) {
    uint64_t t = s.used[d].total.exchange(0);
    uint64_t sp = s.used[d].kind[kMemSpill].load();
    for (int k = 0; k < kMemKinds; k++) s.used[d].kind[k].store(0);
    s.used[d].svm_vram.store(0);
    if (t) r_->dev[d].used.fetch_sub(t);
    if (sp) r_->dev[d].spilled.fetch_sub(sp);
  }
  if (uint64_t h = s.host_used.exchange(0)) r_->hdr.host_used.fetch_sub(h);
  s.status.store(kProcFree);
  s.hostpid.store(0);
  s.pid.store(0, std::memory_order_release);
  r_->hdr.proc_num.fetch_sub(1);
}

void SharedRegion::unregister_process(int slot) {
  if (!r_ || slot < 0 || slot >= kMaxProcs) return;
  if (!lock()) return;
  clear_slot_locked(slot);
  unlock();
}

int SharedRegion::reclaim_dead() {
  if (!r_) return 0;
  // Reached from the allocation path (charge over the limit): a stopped lock holder must
  // turn into an OOM for the caller, not a hang.
  if (!lock_for(kLockTimeoutMs)) return 0;
  int n = 0;
  for (int i = 0; i < kMaxProcs; i++) {
    ProcSlot& s = r_->procs[i];
    int32_t pid = s.pid.load();
    if (pid == 0) continue;
    if (slot_exited(s)) {
      VLOG_INFO("reclaiming slot %d of exited pid %d", i, pid);
      clear_slot_locked(i);
      n++;
    }
  }
  unlock();
  return n;
}

namespace {
uint64_t lower_limit(uint64_t lim, uint64_t ceil) {  // 0 = unlimited on either side
  if (!ceil) return lim;
  return lim && lim < ceil ? lim : ceil;
}
}  // namespace

Charge SharedRegion::charge(int slot, int dev, uint64_t bytes, MemKind kind) {
  DeviceState& d = r_->dev[dev];
  for (int attempt = 0; attempt < 2; attempt++) {
    uint64_t lim = lower_limit(d.mem_limit, ceil_mem_[dev]);
    uint64_t cur = d.used.load(std::memory_order_relaxed);
    bool admitted = false;
    while (true) {
      if (lim && (bytes > lim || cur > lim - bytes)) break;  // overflow-safe cur + bytes > lim
      if (d.used.compare_exchange_weak(cur, cur + bytes, std::memory_order_acq_rel)) {
        admitted = true;
        break;
      }
    }
    if (admitted) {
      if (slot >= 0) {
        DeviceUsage& u = r_->procs[slot].used[dev];
        uint64_t t = u.total.fetch_add(bytes) + bytes;
        u.kind[kind].fetch_add(bytes);
        uint64_t pk = u.peak.load();
        while (t > pk && !u.peak.compare_exchange_weak(pk, t)) {
        }
      }
      if (kind == kMemSpill) d.spilled.fetch_add(bytes);
      return Charge::kOk;
    }
    // Over the limit: memory of exited processes may still be charged. Reclaim once
    // and retry (reference oom_check → rm_quitted_process → retry).
    if (attempt == 0 && reclaim_dead() == 0) break;
  }
  if (slot >= 0) r_->procs[slot].oom_events.fetch_add(1);
  return Charge::kOverLimit;
}

void SharedRegion::force_charge(int slot, int dev, uint64_t bytes, MemKind kind) {
  r_->dev[dev].used.fetch_add(bytes);
  if (kind == kMemSpill) r_->dev[dev].spilled.fetch_add(bytes);
  if (slot >= 0) {
    r_->procs[slot].used[dev].total.fetch_add(bytes);
    r_->procs[slot].used[dev].kind[kind].fetch_add(bytes);
  }
}

void SharedRegion::uncharge(int slot, int dev, uint64_t bytes, MemKind kind) {
  DeviceState& d = r_->dev[dev];
  // Saturating subtraction: a slot reclaimed concurrently must not underflow.
  auto sat_sub = [](std::atomic<uint64_t>& a, uint64_t v) {
    uint64_t cur = a.load(std::memory_order_relaxed);
    while (!a.compare_exchange_weak(cur, cur > v ? cur - v : 0)) {
    }
  };
  if (slot >= 0) {
    DeviceUsage& u = r_->procs[slot].used[dev];
    uint64_t have = u.total.load();
    if (have < bytes) bytes = have;  // slot already reclaimed/cleared
    sat_sub(u.total, bytes);
    sat_sub(u.kind[kind], bytes);
  }
  sat_sub(d.used, bytes);
  if (kind == kMemSpill) sat_sub(d.spilled, bytes);
}

uint64_t SharedRegion::usage(int dev) const { return r_->dev[dev].used.load(std::memory_order_relaxed); }
uint64_t SharedRegion::limit(int dev) const { return lower_limit(r_->dev[dev].mem_limit, ceil_mem_[dev]); }
uint64_t SharedRegion::hbm_limit(int dev) const { return lower_limit(r_->dev[dev].hbm_limit, ceil_hbm_[dev]); }
void SharedRegion::set_svm_vram(int slot, int dev, uint64_t bytes) {
  if (!r_ || slot < 0 || slot >= kMaxProcs || dev < 0 || dev >= kMaxDevices) return;
  r_->procs[slot].used[dev].svm_vram.store(bytes, std::memory_order_relaxed);
}

uint64_t SharedRegion::svm_vram(int dev) const {
  if (!r_ || dev < 0 || dev >= kMaxDevices) return 0;
  uint64_t n = 0;
  for (int i = 0; i < kMaxProcs; i++)
    if (r_->procs[i].pid.load(std::memory_order_relaxed)) n += r_->procs[i].used[dev].svm_vram.load(std::memory_order_relaxed);
  return n;
}

uint64_t SharedRegion::resident(int dev) const {
  // Sequentially consistent: pairs with promote_spill (an allocator charges `used`, then reads
  // `spilled`; a promotion lowers `spilled`, then reads `used` - one of them sees the other).
  uint64_t u = r_->dev[dev].used.load(std::memory_order_seq_cst);
  uint64_t s = r_->dev[dev].spilled.load(std::memory_order_seq_cst);
  return u > s ? u - s : 0;
}

bool SharedRegion::promote_spill(int slot, int dev, uint64_t bytes, uint64_t cap) {
  DeviceState& d = r_->dev[dev];
  // Lower `spilled` first, then check the resident bytes it implies: an allocation charging
  // `used` concurrently either sees this move (and spills itself) or is seen here (and the
  // move is undone), so the two cannot jointly push the container past its HBM share.
  uint64_t cur = d.spilled.load(std::memory_order_seq_cst);
  do {
    if (cur < bytes) return false;
  } while (!d.spilled.compare_exchange_weak(cur, cur - bytes, std::memory_order_seq_cst));
  if (cap) {
    const uint64_t u = d.used.load(std::memory_order_seq_cst);
    const uint64_t sp = d.spilled.load(std::memory_order_seq_cst);
    if ((u > sp ? u - sp : 0) > cap) {
      d.spilled.fetch_add(bytes, std::memory_order_seq_cst);
      return false;
    }
  }
  if (slot >= 0) {
    DeviceUsage& u = r_->procs[slot].used[dev];
    uint64_t have = u.kind[kMemSpill].load();
    uint64_t moved = have < bytes ? have : bytes;
    u.kind[kMemSpill].fetch_sub(moved);
    u.kind[kMemData].fetch_add(moved);
  }
  return true;
}

void SharedRegion::demote_to_spill(int slot, int dev, uint64_t bytes) {
  r_->dev[dev].spilled.fetch_add(bytes, std::memory_order_seq_cst);
  if (slot >= 0) {
    DeviceUsage& u = r_->procs[slot].used[dev];
    uint64_t have = u.kind[kMemData].load();
    uint64_t moved = have < bytes ? have : bytes;
    u.kind[kMemData].fetch_sub(moved);
    u.kind[kMemSpill].fetch_add(moved);
  }
}
uint64_t SharedRegion::proc_usage(int slot, int dev) const { return r_->procs[slot].used[dev].total.load(); }

Charge SharedRegion::charge_host(int slot, uint64_t bytes) {
  RegionHeader& h = r_->hdr;
  for (int attempt = 0; attempt < 2; attempt++) {
    const uint64_t lim = lower_limit(h.host_limit, ceil_host_);
    uint64_t cur = h.host_used.load(std::memory_order_relaxed);
    bool admitted = false;
    while (true) {
      if (lim && (bytes > lim || cur > lim - bytes)) break;
      if (h.host_used.compare_exchange_weak(cur, cur + bytes, std::memory_order_acq_rel)) {
        admitted = true;
        break;
      }
    }
    if (admitted) {
      if (slot >= 0) {
        ProcSlot& p = r_->procs[slot];
        uint64_t t = p.host_used.fetch_add(bytes) + bytes;
        uint64_t pk = p.host_peak.load();
        while (t > pk && !p.host_peak.compare_exchange_weak(pk, t)) {
        }
      }
      return Charge::kOk;
    }
    if (attempt == 0 && reclaim_dead() == 0) break;
  }
  if (slot >= 0) r_->procs[slot].oom_events.fetch_add(1);
  return Charge::kOverLimit;
}

void SharedRegion::uncharge_host(int slot, uint64_t bytes) {
  auto sat_sub = [](std::atomic<uint64_t>& a, uint64_t v) {
    uint64_t cur = a.load(std::memory_order_relaxed);
    while (!a.compare_exchange_weak(cur, cur > v ? cur - v : 0)) {
    }
  };
  if (slot >= 0) {
    ProcSlot& p = r_->procs[slot];
    const uint64_t have = p.host_used.load();
    if (have < bytes) bytes = have;  // slot already reclaimed/cleared
    sat_sub(p.host_used, bytes);
  }
  sat_sub(r_->hdr.host_used, bytes);
}

uint64_t SharedRegion::host_usage() const { return r_->hdr.host_used.load(std::memory_order_relaxed); }
uint64_t SharedRegion::host_limit() const { return lower_limit(r_->hdr.host_limit, ceil_host_); }
void SharedRegion::set_host_limit(uint64_t bytes) {
  r_->hdr.host_limit = lower_limit(bytes, ceil_host_);
  r_->hdr.generation.fetch_add(1);
}

void SharedRegion::set_ceiling(int dev, uint64_t mem_bytes) {
  if (dev >= 0 && dev < kMaxDevices) ceil_mem_[dev] = mem_bytes;
}

void SharedRegion::set_hbm_ceiling(int dev, uint64_t bytes) {
  if (dev >= 0 && dev < kMaxDevices) ceil_hbm_[dev] = bytes;
}

void SharedRegion::set_host_ceiling(uint64_t bytes) { ceil_host_ = bytes; }

uint64_t SharedRegion::inode() const {
  if (fd_ < 0) return 0;
  struct stat st;
  // By system call: fstat is a GLIBC_2.33 symbol (glibc_compat.h).
  if (syscall(SYS_fstat, fd_, &st) != 0) return 0;
  return (uint64_t)st.st_ino;
}

void SharedRegion::touch() {
  if (fd_ >= 0) (void)futimens(fd_, nullptr);
}

bool SharedRegion::reinit_if_invalid(const Config* cfg) {
  if (!r_ || fd_ < 0) return false;
  if (r_->hdr.magic == kRegionMagic && r_->hdr.version == kRegionVersion && r_->hdr.region_size == sizeof(Region))
    return false;
  if (flock(fd_, LOCK_EX) != 0) return false;
  bool done = false;
  if (r_->hdr.magic != kRegionMagic || r_->hdr.version != kRegionVersion || r_->hdr.region_size != sizeof(Region)) {
    VLOG_ERROR("shared region %s was overwritten; re-initialising it", path_);
    init_fresh(cfg);
    done = true;
  }
  flock(fd_, LOCK_UN);
  return done;
}

void SharedRegion::set_limit(int dev, uint64_t bytes) {
  r_->dev[dev].mem_limit = lower_limit(bytes, ceil_mem_[dev]);
  if (dev >= r_->hdr.num_devices) r_->hdr.num_devices = dev + 1;
  r_->hdr.generation.fetch_add(1);
}

void SharedRegion::set_cu_limit(int dev, int pct) {
  DeviceState& d = r_->dev[dev];
  bool locked = lock_for(kLockTimeoutMs);  // node tools must not hang behind a stopped tenant
  d.cu_limit_pct = pct;
  d.cu_share_bp = 0;  // a live share is a whole percent
  if (d.configured && d.cu_count > 0) {
    // Keep the vGPU's anchor (the start of the slice the plugin assigned) and resize the
    // slice to the new share, shifted left when it would run past the last CU.
    const int xcc = d.num_xcc > 0 ? d.num_xcc : 1;
    int want = cu_share_count(d.cu_count, xcc, pct);
    int b = d.cu_range_begin >= 0 ? d.cu_range_begin / xcc * xcc : 0;
    if (b + want > d.cu_count) b = (d.cu_count - want) / xcc * xcc;
    CuMask m = cu_mask_range(d.cu_count, xcc, b, b + want, d.num_se > 0 ? d.num_se : 1);
    memcpy(d.cu_mask, m.words, sizeof(d.cu_mask));
    d.cu_mask_bits = m.nbits;
  }
  if (dev >= r_->hdr.num_devices) r_->hdr.num_devices = dev + 1;
  if (locked) unlock();
  r_->hdr.generation.fetch_add(1);
}

void SharedRegion::suspend_all() {
  r_->hdr.suspend_all.store(1);
  for (int i = 0; i < kMaxProcs; i++)
    if (r_->procs[i].pid.load()) r_->procs[i].status.store(kProcSuspended);
  r_->hdr.generation.fetch_add(1);
}

void SharedRegion::resume_all() {
  r_->hdr.suspend_all.store(0);
  for (int i = 0; i < kMaxProcs; i++)
    if (r_->procs[i].pid.load()) r_->procs[i].status.store(kProcRunning);
  r_->hdr.generation.fetch_add(1);
}

void SharedRegion::set_proc_status(int slot, int status) {
  if (slot >= 0 && slot < kMaxProcs) r_->procs[slot].status.store(status);
}

}  // namespace vgpu
