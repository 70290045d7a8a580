// Node-wide GPU-time ledger: one occupancy sampler per node instead of one per container.
//
// Without it every limited container's sampler reads the KFD cu_occupancy of its own
// processes and of every other process on its GPU (ratelimit.h): with n containers the
// node makes n² reads per period, every read costs the GPU (a read walks the GPU's wave
// slots; sampling 12 pods every 1 ms cost 14 % of the GPU, profiles/r2ae), so the period
// stretches to base·n²/32 - 8 ms at 16 pods - and each container charges itself from its
// own, unsynchronised snapshots. The reference samples NVML per container too
// (utilization_watcher [multiprocess_utilization_watcher.c:195-216]).
//
// The ledger daemon (vgpu-ledger, started by the device plugin as root with --ledger) reads each
// process on a GPU once per period - n reads for n processes - and integrates, from one
// consistent snapshot per period, each process's processor-sharing charge
//     charged_ns += dt · occ(pid) / Σ occ          (trapezoid over the period)
// into <board>/ledger.<gpu_id>. Containers read it through the board directory (mounted
// read-only; the daemon's files are root-owned 0644), so no tenant can alter another's
// charge: a container's limiter takes the growth of its processes' cumulative charges as
// its charge, and the last occupancy of every process on the GPU for crowd and class
// decisions. A stale or missing ledger (daemon not running, old plugin) leaves the
// container sampling by itself as before.
#pragma once

#include <sys/types.h>

#include <atomic>
#include <cstdint>
#include <string>

namespace vgpu {

constexpr uint32_t kLedgerMagic = 0x56474c31u;  // "VGL1"
constexpr uint32_t kLedgerVersion = 1;
constexpr int kLedgerMaxPids = 1024;
// A ledger whose heartbeat is older than max(kLedgerStaleNs, kLedgerStalePeriods x its own
// sampling period) is ignored (containers sample by themselves).
constexpr uint64_t kLedgerStaleNs = 50'000'000ull;
constexpr uint64_t kLedgerStalePeriods = 4;

struct alignas(32) LedgerEntry {
  std::atomic<int32_t> pid;          // host PID, 0 = free entry
  std::atomic<int32_t> occ;          // cu_occupancy at the last sample
  std::atomic<uint64_t> charged_ns;  // cumulative processor-sharing charge
  std::atomic<uint64_t> busy_ns;     // CLOCK_MONOTONIC of the last sample with resident waves
  std::atomic<uint64_t> seen_ns;     // first sample of this PID in this entry (reuse guard)
};

struct LedgerFile {
  uint32_t magic;
  uint32_t version;
  uint32_t gpu_id;
  std::atomic<int32_t> n;              // high-water mark of used entries
  std::atomic<uint64_t> heartbeat_ns;  // CLOCK_MONOTONIC of the last sample
  std::atomic<uint64_t> samples;
  std::atomic<uint64_t> period_ns;     // current sampling period
  std::atomic<int64_t> total_occ;      // Σ occ at the last sample
  std::atomic<uint64_t> reads;         // cu_occupancy reads so far (overhead accounting)
  uint64_t reserved[9];
  LedgerEntry e[kLedgerMaxPids];
};

// Path of the ledger of KFD gpu_id under `dir`.
std::string ledger_path(const std::string& dir, uint32_t gpu_id);

// Read side (containers): maps <dir>/ledger.<gpu_id> read-only when it exists.
class LedgerReader {
 public:
  LedgerReader() = default;
  ~LedgerReader();
  LedgerReader(const LedgerReader&) = delete;
  LedgerReader& operator=(const LedgerReader&) = delete;

  // (Re)maps the file; false when it is absent or foreign. Cheap to call again.
  bool open(const std::string& dir, uint32_t gpu_id);
  bool attached() const { return f_ != nullptr; }
  void close();
  // Attached and sampled within kLedgerStaleNs of `now`.
  bool fresh(uint64_t now) const;
  const LedgerFile* file() const { return f_; }
  // The entry of `pid`, or null.
  const LedgerEntry* find(int pid) const;

 private:
  const LedgerFile* f_ = nullptr;
  uint32_t gpu_id_ = 0;
};

}  // namespace vgpu
