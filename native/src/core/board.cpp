// Node-wide GPU board (see vgpu/board.h).
#include "vgpu/board.h"

#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <map>
#include <set>

#include "vgpu/log.h"

namespace vgpu {

namespace {

// Modification time of `path` in seconds (CLOCK_REALTIME), -1 if unknown. By system call:
// stat/fstat are GLIBC_2.33 symbols, which the preloaded shim must not need (glibc_compat.h);
// on x86-64 the kernel's struct stat is glibc's.
int64_t file_mtime(const char* path) {
  struct stat st;
  if (syscall(SYS_newfstatat, AT_FDCWD, path, &st, 0) != 0) return -1;
  return (int64_t)st.st_mtim.tv_sec;
}

int64_t wall_seconds() {
  struct timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return (int64_t)ts.tv_sec;
}

}  // namespace

Board::~Board() {
  if (self_) munmap(self_, sizeof(BoardSlot));
  if (fd_ >= 0) close(fd_);
}

int Board::open(const char* dir, const char* self_name) {
  if (!dir || !*dir || !self_name || !*self_name || strchr(self_name, '/')) return -EINVAL;
  dir_ = dir;
  self_name_ = self_name;
  const std::string path = dir_ + "/" + self_name_;
  int fd = ::open(path.c_str(), O_RDWR | O_CLOEXEC);
  if (fd < 0 && errno == ENOENT) fd = ::open(path.c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0644);
  if (fd < 0) return -errno;
  // Size by lseek (fstat is GLIBC_2.33, glibc_compat.h); a short slot is extended.
  const off_t size = lseek(fd, 0, SEEK_END);
  if (size < (off_t)sizeof(BoardSlot) && ftruncate(fd, sizeof(BoardSlot)) != 0) {
    int e = errno;
    ::close(fd);
    return -e;
  }
  void* p = mmap(nullptr, sizeof(BoardSlot), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (p == MAP_FAILED) {
    int e = errno;
    ::close(fd);
    return -e;
  }
  self_ = static_cast<BoardSlot*>(p);
  fd_ = fd;
  if (self_->magic != kBoardMagic || self_->version != kBoardVersion) {
    memset(static_cast<void*>(self_), 0, sizeof(BoardSlot));
    self_->version = kBoardVersion;
    std::atomic_thread_fence(std::memory_order_release);
    self_->magic = kBoardMagic;
  }
  return 0;
}

int Board::open_readonly(const char* dir) {
  if (!dir || !*dir) return -EINVAL;
  dir_ = dir;
  self_name_.clear();
  return 0;
}

void Board::publish(int priority, const uint32_t* gpu_ids, int ndev, const std::vector<int>& hostpids, uint64_t now,
                    const uint32_t (*masks)[kCuMaskWords]) {
  if (!self_) return;
  self_->priority.store(priority, std::memory_order_relaxed);
  ndev = std::max(0, std::min(ndev, kMaxDevices));
  for (int i = 0; i < ndev; i++) {
    self_->gpu_id[i] = gpu_ids[i];
    for (int w = 0; w < kCuMaskWords; w++) self_->cu_mask[i][w] = masks ? masks[i][w] : 0;
  }
  self_->ndev = ndev;
  const int n = std::min((int)hostpids.size(), kBoardMaxPids);
  for (int i = 0; i < n; i++) self_->hostpids[i].store(hostpids[i], std::memory_order_relaxed);
  self_->npids.store(n, std::memory_order_release);
  self_->heartbeat_ns.store(now, std::memory_order_release);
  // Writes through the mapping need not touch the file's mtime (tmpfs never does): it is
  // touched explicitly, so readers - and the plugin's clean-up of departed containers'
  // slots - can tell a live slot from a dead one without reading it.
  const int64_t wall = wall_seconds();
  if (wall - touched_s_ >= kBoardTouchS && futimens(fd_, nullptr) == 0) touched_s_ = wall;
}

void Board::leave() {
  if (self_) self_->heartbeat_ns.store(0, std::memory_order_release);
}

void Board::publish_gate(int dev, bool open, uint64_t want_since) {
  if (!self_ || dev < 0 || dev >= kMaxDevices) return;
  self_->gate[dev].store(open ? 1 : 0, std::memory_order_relaxed);
  self_->want_since[dev].store(want_since, std::memory_order_relaxed);
}

void Board::publish_cpu_node(int node) {
  if (self_) self_->cpu_node1.store(node >= 0 ? node + 1 : 0, std::memory_order_relaxed);
}

void Board::publish_launch_rate(uint32_t per_s) {
  if (self_) self_->launch_rate.store(per_s, std::memory_order_relaxed);
}

uint64_t Board::peers_launch_rate(uint32_t gpu_id) const {
  uint64_t n = 0;
  for (const BoardPeer& p : peers_)
    if (std::find(p.gpu_ids.begin(), p.gpu_ids.end(), gpu_id) != p.gpu_ids.end()) n += p.launch_rate;
  return n;
}

void Board::publish_steady(bool steady) {
  if (self_) self_->steady1.store(steady ? 2 : 1, std::memory_order_relaxed);
}

bool Board::bursty_peer_on(uint32_t gpu_id, uint32_t min_rate) const {
  for (const BoardPeer& p : peers_)
    if (p.steady == 0 && p.launch_rate >= min_rate &&
        std::find(p.gpu_ids.begin(), p.gpu_ids.end(), gpu_id) != p.gpu_ids.end())
      return true;
  return false;
}

void Board::publish_memory(int dev, uint64_t svm_vram, uint64_t hbm_want, uint64_t want_ns) {
  if (!self_ || dev < 0 || dev >= kMaxDevices) return;
  self_->svm_vram[dev].store(svm_vram, std::memory_order_relaxed);
  self_->hbm_want_ns[dev].store(hbm_want ? want_ns : 0, std::memory_order_relaxed);
  self_->hbm_want[dev].store(hbm_want, std::memory_order_relaxed);
}

uint64_t Board::peers_svm_vram(uint32_t gpu_id) const {
  uint64_t n = 0;
  for (const BoardPeer& p : peers_)
    for (size_t i = 0; i < p.gpu_ids.size() && i < p.svm_vram.size(); i++)
      if (p.gpu_ids[i] == gpu_id) n += p.svm_vram[i];
  return n;
}

uint64_t Board::peers_hbm_want(uint32_t gpu_id, uint64_t* newest_ns) const {
  uint64_t n = 0, newest = 0;
  for (const BoardPeer& p : peers_)
    for (size_t i = 0; i < p.gpu_ids.size() && i < p.hbm_want.size() && i < p.hbm_want_ns.size(); i++)
      if (p.gpu_ids[i] == gpu_id && p.hbm_want[i]) {
        n = std::max(n, p.hbm_want[i]);
        newest = std::max(newest, p.hbm_want_ns[i]);
      }
  if (newest_ns) *newest_ns = newest;
  return n;
}

namespace {

// Holders per CPU node and the distinct nodes of the containers on `gpu_id` (this one's
// `node` included); the per-node cap of k holders (k when the nodes are unknown or one).
struct NodeLoad {
  std::map<int, int> held;
  std::set<int> nodes;
  int cap = 0;
  bool room(int n) const {
    if (n < 0 || nodes.size() <= 1) return true;
    auto it = held.find(n);
    return (it == held.end() ? 0 : it->second) < cap;
  }
};

NodeLoad node_load(const std::vector<BoardPeer>& peers, uint32_t gpu_id, int k, int node) {
  NodeLoad l;
  if (node >= 0) l.nodes.insert(node);
  for (const BoardPeer& p : peers)
    for (size_t i = 0; i < p.gpu_ids.size() && i < p.gate.size(); i++) {
      if (p.gpu_ids[i] != gpu_id) continue;
      if (p.cpu_node >= 0) l.nodes.insert(p.cpu_node);
      if (p.gate[i] && p.cpu_node >= 0) l.held[p.cpu_node]++;
    }
  // Socket awareness needs this container's node too: without it every node counts alike.
  if (node < 0) l.nodes.clear();
  const int d = (int)l.nodes.size();
  l.cap = d > 1 ? (k + d - 1) / d : k;
  return l;
}

}  // namespace

bool Board::waiting(uint32_t gpu_id, int k, int node) const {
  // This container holds a turn on `gpu_id` (CPU node `node`). A waiter is in its way when
  // nodes are unknown (plain round robin), when it is of the same node, when this node holds
  // more than its cap (peers' nodes were not known yet when it was admitted), or when all k
  // places are taken and the waiter's node has room.
  const NodeLoad load = node_load(peers_, gpu_id, k, node);
  int open = 1;  // this container
  bool any = false, blocked_by_total = false, same = false;
  for (const BoardPeer& p : peers_)
    for (size_t i = 0; i < p.gpu_ids.size() && i < p.want_since.size() && i < p.gate.size(); i++) {
      if (p.gpu_ids[i] != gpu_id) continue;
      if (p.gate[i]) {
        open++;
        continue;
      }
      if (!p.want_since[i]) continue;
      any = true;
      if (node < 0 || p.cpu_node < 0 || load.nodes.size() <= 1 || p.cpu_node == node) same = true;
      else if (load.room(p.cpu_node)) blocked_by_total = true;
    }
  if (!any) return false;
  if (same) return true;
  auto it = load.held.find(node);
  const int mine = 1 + (it == load.held.end() ? 0 : it->second);
  return mine > load.cap || (blocked_by_total && open >= k);
}

bool Board::admit(uint32_t gpu_id, int k, uint64_t want_since, int node) const {
  if (k <= 0) return true;
  const NodeLoad load = node_load(peers_, gpu_id, k, node);
  int open = 0, ahead = 0;
  for (const BoardPeer& p : peers_) {
    for (size_t i = 0; i < p.gpu_ids.size() && i < p.gate.size(); i++) {
      if (p.gpu_ids[i] != gpu_id) continue;
      if (p.gate[i]) open++;
      else if (p.want_since[i] && p.want_since[i] < want_since && load.room(p.cpu_node)) ahead++;
    }
  }
  return open < k && ahead < k - open && load.room(node);
}

const std::vector<BoardPeer>& Board::refresh(uint64_t now) {
  peers_.clear();
  if (dir_.empty()) return peers_;
  DIR* d = opendir(dir_.c_str());
  if (!d) return peers_;
  const int64_t wall = wall_seconds();
  while (struct dirent* e = readdir(d)) {
    const size_t len = strlen(e->d_name);
    if (len < 6 || strcmp(e->d_name + len - 5, ".slot") != 0 || self_name_ == e->d_name) continue;
    const std::string path = dir_ + "/" + e->d_name;
    // A slot nobody has touched for a while belongs to a container without a live GPU
    // process (or one long gone): skipped without opening it, so departed containers'
    // slots cost one stat each until the plugin removes them.
    const int64_t mt = file_mtime(path.c_str());
    if (mt >= 0 && wall - mt > kBoardSkipAgeS) continue;
    int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0) continue;
    BoardSlot s;
    memset(static_cast<void*>(&s), 0, sizeof(s));
    // A plain read of a slot another container keeps rewriting: fields may be torn, so
    // every value is bounds-checked and the heartbeat decides liveness. A slot of an older
    // shim ends after the version-1 fields: the appended ones read as 0.
    const ssize_t got = pread(fd, static_cast<void*>(&s), sizeof(s), 0);
    ::close(fd);
    if (got < (ssize_t)kBoardSlotV1Size || s.magic != kBoardMagic || s.version != kBoardVersion) continue;
    const uint64_t hb = s.heartbeat_ns.load(std::memory_order_relaxed);
    // A heartbeat newer than `now` (the peer published after the caller read its clock) is
    // fresh: `now - hb` would wrap and drop a live peer at random.
    if (!hb || hb > now + kBoardStaleNs || (hb < now && now - hb > kBoardStaleNs)) continue;
    BoardPeer p;
    p.name.assign(e->d_name, len - 5);
    p.priority = s.priority.load(std::memory_order_relaxed);
    const int ndev = std::max(0, std::min(s.ndev, kMaxDevices));
    p.gpu_ids.assign(s.gpu_id, s.gpu_id + ndev);
    for (int i = 0; i < ndev; i++) {
      p.masks.emplace_back(s.cu_mask[i], s.cu_mask[i] + kCuMaskWords);
      p.gate.push_back(s.gate[i].load(std::memory_order_relaxed));
      p.want_since.push_back(s.want_since[i].load(std::memory_order_relaxed));
      p.svm_vram.push_back(s.svm_vram[i].load(std::memory_order_relaxed));
      const uint64_t wn = s.hbm_want_ns[i].load(std::memory_order_relaxed);
      const bool fresh = wn && wn <= now + kBoardStaleNs && (wn >= now || now - wn < kBoardWantNs);
      p.hbm_want.push_back(fresh ? s.hbm_want[i].load(std::memory_order_relaxed) : 0);
      p.hbm_want_ns.push_back(fresh ? wn : 0);
    }
    const int32_t cn = got >= (ssize_t)sizeof(BoardSlot) ? s.cpu_node1.load(std::memory_order_relaxed) : 0;
    p.cpu_node = cn > 0 && cn <= 64 ? cn - 1 : -1;
    if (got >= (ssize_t)sizeof(BoardSlot)) {
      p.launch_rate = std::min<uint32_t>(s.launch_rate.load(std::memory_order_relaxed), 10'000'000u);
      const int32_t st = s.steady1.load(std::memory_order_relaxed);
      p.steady = st == 1 ? 0 : st == 2 ? 1 : -1;
    }
    const int n = std::max(0, std::min(s.npids.load(std::memory_order_relaxed), kBoardMaxPids));
    for (int i = 0; i < n; i++) {
      const int pid = s.hostpids[i].load(std::memory_order_relaxed);
      if (pid > 0) p.hostpids.push_back(pid);
    }
    peers_.push_back(std::move(p));
  }
  closedir(d);
  return peers_;
}

void Board::reserved_mask(uint32_t gpu_id, int max_priority, uint32_t* out_words) const {
  for (int w = 0; w < kCuMaskWords; w++) out_words[w] = 0;
  for (const BoardPeer& p : peers_) {
    if (p.priority > max_priority) continue;
    for (size_t i = 0; i < p.gpu_ids.size() && i < p.masks.size(); i++)
      if (p.gpu_ids[i] == gpu_id)
        for (int w = 0; w < kCuMaskWords; w++) out_words[w] |= p.masks[i][w];
  }
}

int Board::priority_of(int pid, uint32_t gpu_id) const {
  for (const BoardPeer& p : peers_) {
    if (std::find(p.gpu_ids.begin(), p.gpu_ids.end(), gpu_id) == p.gpu_ids.end()) continue;
    if (std::find(p.hostpids.begin(), p.hostpids.end(), pid) != p.hostpids.end()) return p.priority;
  }
  return kPrioNormal;
}

bool Board::better_on(uint32_t gpu_id, int priority) const {
  for (const BoardPeer& p : peers_)
    if (p.priority < priority && std::find(p.gpu_ids.begin(), p.gpu_ids.end(), gpu_id) != p.gpu_ids.end())
      return true;
  return false;
}

}  // namespace vgpu
