// Node-wide GPU board: what the vGPU containers of a node tell each other.
//
// The reference has no cross-container channel: every container's limiter works alone,
// and its CUDA_TASK_PRIORITY is stored but never acted on. Scheduling
// classes need one: a background container must know which busy processes on its GPU
// belong to higher-priority containers in order to yield to them, and not to its peers.
//
// Layout on the node: the plugin creates <vgpu_dir>/board/ (root, 0755) and, per
// container, one slot file <id>.slot in it. The container gets the directory read-only
// and its own slot file read-write on top (docs/ABI.md): every container reads every
// slot, and writes only its own - no tenant can alter what another one publishes. A
// slot is written by the container's sampler (lease holder) and is only advice to the
// containers that opt into yielding (background class): a tenant lying in its own slot
// cannot take anything from a container that does not yield.
#pragma once

#include <sys/types.h>

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "vgpu/config.h"

namespace vgpu {

constexpr uint32_t kBoardMagic = 0x56424431u;  // "VBD1"
constexpr uint32_t kBoardVersion = 1;
constexpr int kBoardMaxPids = 256;

// Scheduling classes from VGPU_TASK_PRIORITY (0 high, 1 normal, >= 2 low).
constexpr int kPrioLatency = 0;     // <= 0: never duty-cycled by auto mode; HW queues high
constexpr int kPrioNormal = 1;
constexpr int kPrioBackground = 2;  // >= 2: yields GPU time to busy higher-priority tenants

struct alignas(64) BoardSlot {
  uint32_t magic;
  uint32_t version;
  std::atomic<uint64_t> heartbeat_ns;     // CLOCK_MONOTONIC of the last update (0 = left)
  std::atomic<int32_t> priority;
  int32_t ndev;
  uint32_t gpu_id[kMaxDevices];           // KFD gpu_id of the container's devices
  uint32_t cu_mask[kMaxDevices][kCuMaskWords];  // the spatial mask its queues use (0 = all CUs)
  std::atomic<int32_t> gate[kMaxDevices];       // GPU-time gate open at the last sample
  std::atomic<uint64_t> want_since[kMaxDevices];  // waiting for admission since (0 = not waiting)
  std::atomic<int32_t> npids;
  std::atomic<int32_t> hostpids[kBoardMaxPids];
  // Appended after the version-1 fields (a reader accepts a version-1 slot that ends here and
  // reads them as 0): virtual device memory made visible node-wide.
  std::atomic<uint64_t> svm_vram[kMaxDevices];     // the container's SVM bytes in each GPU's VRAM
  std::atomic<uint64_t> hbm_want[kMaxDevices];     // refused HBM within its share: bytes wanted ...
  std::atomic<uint64_t> hbm_want_ns[kMaxDevices];  // ... since (CLOCK_MONOTONIC; 0 = none)
  // Appended (round 6): the CPU node the container's processes run on (VGPU_CPU_NODE), plus
  // one (0 = unknown, as an older slot reads): the concurrency admission pairs containers of
  // different CPU sockets.
  std::atomic<int32_t> cpu_node1;
  std::atomic<uint32_t> launch_rate;  // the container's kernel launches per second (EWMA)
  std::atomic<int32_t> steady1;       // 0 unknown, 1 bursty (idles between launches), 2 steady
};
constexpr size_t kBoardSlotV1Size = offsetof(BoardSlot, svm_vram);

// An HBM request older than this is over (the requester gave up or was served).
constexpr uint64_t kBoardWantNs = 3'000'000'000ull;
// Slot staleness: a slot whose heartbeat is older than this is ignored.
constexpr uint64_t kBoardStaleNs = 2'000'000'000ull;
// A publishing container touches its slot file's mtime every kBoardTouchS; readers skip,
// without opening them, slots untouched for kBoardSkipAgeS (the plugin removes slots
// untouched for an hour: contract.py BOARD_MAX_AGE_S).
constexpr int64_t kBoardTouchS = 10;
constexpr int64_t kBoardSkipAgeS = 60;

// Another container as read from its slot.
struct BoardPeer {
  std::string name;                          // its slot file's name without ".slot" (the container)
  int priority = kPrioNormal;
  std::vector<uint32_t> gpu_ids;
  std::vector<std::vector<uint32_t>> masks;  // per device, kCuMaskWords words (all 0 = no mask)
  std::vector<int> gate;                     // per device
  std::vector<uint64_t> want_since;          // per device
  std::vector<int> hostpids;
  std::vector<uint64_t> svm_vram;            // per device
  std::vector<uint64_t> hbm_want;            // per device (0 = none, or stale)
  std::vector<uint64_t> hbm_want_ns;         // per device: when it was (re-)published
  int cpu_node = -1;                         // VGPU_CPU_NODE (-1 = unknown)
  uint32_t launch_rate = 0;                  // kernel launches per second
  int steady = -1;                           // -1 unknown, 0 bursty, 1 steady
};

// Automatic pair turns (VGPU_GPU_CONCURRENCY=auto): below VGPU_PAIRS_OFF_RATE launches/s of
// all the containers of a GPU for this long, they stop taking turns.
constexpr uint64_t kPairsOffNs = 2'000'000'000ull;

// A container's view of the board directory: its own slot (read-write) and the others.
class Board {
 public:
  Board() = default;
  ~Board();
  Board(const Board&) = delete;
  Board& operator=(const Board&) = delete;

  // Maps `dir`/`self_name` read-write (created if missing and the directory allows it).
  // Returns 0 or -errno; without a board every query answers "no peers".
  int open(const char* dir, const char* self_name);
  // Reads the directory without a slot of its own (the ledger daemon).
  int open_readonly(const char* dir);
  bool attached() const { return self_ != nullptr; }
  BoardSlot* self() { return self_; }

  // Publishes this container's state (the sampler calls it every period).
  // `masks`: ndev x kCuMaskWords words, or null.
  void publish(int priority, const uint32_t* gpu_ids, int ndev, const std::vector<int>& hostpids, uint64_t now,
               const uint32_t (*masks)[kCuMaskWords] = nullptr);
  void leave();
  // Gate state of device `dev` for the concurrency admission (every sample).
  void publish_gate(int dev, bool open, uint64_t want_since);
  // The CPU node the container's processes run on (-1 = none / unknown).
  void publish_cpu_node(int node);
  // The container's kernel launches per second.
  void publish_launch_rate(uint32_t per_s);
  // Sum of the live peers' launch rates on GPU `gpu_id`.
  uint64_t peers_launch_rate(uint32_t gpu_id) const;
  // Whether the container launches steadily (a batch pod) or in bursts (a serving pod).
  void publish_steady(bool steady);
  // Whether a live peer on GPU `gpu_id` launching at least `min_rate` kernels/s is bursty.
  bool bursty_peer_on(uint32_t gpu_id, uint32_t min_rate) const;
  // Virtual device memory of device `dev`: the container's SVM bytes in VRAM, and HBM it was
  // refused within its share (0 = none) since `want_ns`.
  void publish_memory(int dev, uint64_t svm_vram, uint64_t hbm_want, uint64_t want_ns);
  // Sum over live peers of their SVM bytes in GPU `gpu_id`'s VRAM, and the largest HBM a
  // peer there is waiting for (requests older than kBoardWantNs are dropped).
  uint64_t peers_svm_vram(uint32_t gpu_id) const;
  uint64_t peers_hbm_want(uint32_t gpu_id, uint64_t* newest_ns = nullptr) const;

  // Concurrency admission (VGPU_GPU_CONCURRENCY = k): may this container open its gate on
  // GPU `gpu_id`, given it has wanted to since `want_since`? Yes while fewer than k
  // peers hold their gates open there and fewer than (k - open) peers that could be admitted
  // have been waiting longer. CPU-socket aware: when the GPU's containers run on D > 1
  // CPU nodes (`node`, the peers' published ones), at most ceil(k / D) holders per node -
  // two launch-bound processes on one socket run no faster together than one alone
  // (profiles/r5d), so k = 2 takes turns in cross-socket pairs. Peers as of the last refresh().
  bool admit(uint32_t gpu_id, int k, uint64_t want_since, int node = -1) const;
  // Whether a peer on GPU `gpu_id` waits for admission that this container's turn (k places,
  // this container on CPU node `node`) stands in the way of: any waiting peer when nodes are
  // unknown; with nodes, one of its own node, any when this node holds more than its share of
  // the places, or one whose node has room when all k places are taken.
  bool waiting(uint32_t gpu_id, int k = 0, int node = -1) const;

  // Re-reads the other slots (live ones only). Cheap enough for every 100 ms.
  const std::vector<BoardPeer>& refresh(uint64_t now);
  const std::vector<BoardPeer>& peers() const { return peers_; }

  // Priority of the container owning host PID `pid` on GPU `gpu_id` (kPrioNormal for a
  // process no live slot lists: an unmanaged process counts as a normal tenant).
  int priority_of(int pid, uint32_t gpu_id) const;
  // Whether a live peer of priority < `priority` has GPU `gpu_id` (as of the last refresh).
  bool better_on(uint32_t gpu_id, int priority) const;

  // OR of the CU masks that tenants of priority <= `max_priority` use on GPU `gpu_id`
  // (the CUs a background tenant leaves to the latency class).
  void reserved_mask(uint32_t gpu_id, int max_priority, uint32_t* out_words) const;

 private:
  std::string dir_, self_name_;
  BoardSlot* self_ = nullptr;
  int fd_ = -1;
  int64_t touched_s_ = 0;  // CLOCK_REALTIME seconds of the last mtime touch
  std::vector<BoardPeer> peers_;
};

}  // namespace vgpu
