// Node-wide GPU-time ledger, read side (see vgpu/ledger.h). The writer is the
// vgpu-ledger daemon (src/tools/vgpu_ledger.cpp).
#include "vgpu/ledger.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

namespace vgpu {

std::string ledger_path(const std::string& dir, uint32_t gpu_id) {
  return dir + "/ledger." + std::to_string(gpu_id);
}

LedgerReader::~LedgerReader() { close(); }

void LedgerReader::close() {
  if (f_) munmap(const_cast<LedgerFile*>(f_), sizeof(LedgerFile));
  f_ = nullptr;
}

bool LedgerReader::open(const std::string& dir, uint32_t gpu_id) {
  if (f_ && gpu_id_ == gpu_id) return true;
  if (f_) {
    munmap(const_cast<LedgerFile*>(f_), sizeof(LedgerFile));
    f_ = nullptr;
  }
  if (dir.empty() || !gpu_id) return false;
  int fd = ::open(ledger_path(dir, gpu_id).c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return false;
  // Size by lseek (fstat is GLIBC_2.33, glibc_compat.h): a short file is not a ledger yet.
  const off_t size = lseek(fd, 0, SEEK_END);
  void* p = size >= (off_t)sizeof(LedgerFile) ? mmap(nullptr, sizeof(LedgerFile), PROT_READ, MAP_SHARED, fd, 0)
                                              : MAP_FAILED;
  ::close(fd);
  if (p == MAP_FAILED) return false;
  const LedgerFile* f = static_cast<const LedgerFile*>(p);
  if (f->magic != kLedgerMagic || f->version != kLedgerVersion || f->gpu_id != gpu_id) {
    munmap(p, sizeof(LedgerFile));
    return false;
  }
  f_ = f;
  gpu_id_ = gpu_id;
  return true;
}

bool LedgerReader::fresh(uint64_t now) const {
  if (!f_) return false;
  const uint64_t hb = f_->heartbeat_ns.load(std::memory_order_acquire);
  // A few of the daemon's own periods (it reads every GPU of the node in turn, so its
  // period stretches with the processes on the node), never less than kLedgerStaleNs.
  const uint64_t period = f_->period_ns.load(std::memory_order_relaxed);
  const uint64_t stale = period < kLedgerStaleNs / kLedgerStalePeriods ? kLedgerStaleNs : period * kLedgerStalePeriods;
  // A heartbeat newer than `now` (written after the caller read its clock) is fresh.
  return hb && hb <= now + stale && (hb >= now || now - hb <= stale);
}

const LedgerEntry* LedgerReader::find(int pid) const {
  if (!f_ || pid <= 0) return nullptr;
  int n = f_->n.load(std::memory_order_acquire);
  if (n > kLedgerMaxPids) n = kLedgerMaxPids;
  for (int i = 0; i < n; i++)
    if (f_->e[i].pid.load(std::memory_order_relaxed) == pid) return &f_->e[i];
  return nullptr;
}

}  // namespace vgpu
