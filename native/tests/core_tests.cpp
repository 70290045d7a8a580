// Native unit tests of the shim core (no GPU). Driven by tests/test_native_core.py;
// run one case with `vgpu_core_tests <name>` or all with no argument.
// Built plain and with -fsanitize=thread / address (make SAN=thread|address).
#include <fcntl.h>
#include <signal.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "vgpu/board.h"
#include "vgpu/config.h"
#include "vgpu/cumask.h"
#include "vgpu/devmap.h"
#include "vgpu/kfd.h"
#include "vgpu/ledger.h"
#include "vgpu/ratelimit.h"
#include "vgpu/region.h"

using namespace vgpu;

static int g_failures = 0;
#define CHECK(cond)                                                              \
  do {                                                                           \
    if (!(cond)) {                                                               \
      fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond);    \
      g_failures++;                                                              \
    }                                                                            \
  } while (0)
#define CHECK_EQ(a, b)                                                                              \
  do {                                                                                              \
    auto _a = (a);                                                                                  \
    auto _b = (b);                                                                                  \
    if (!(_a == _b)) {                                                                              \
      fprintf(stderr, "CHECK_EQ failed %s:%d: %s (%lld) != %s (%lld)\n", __FILE__, __LINE__, #a,    \
              (long long)_a, #b, (long long)_b);                                                    \
      g_failures++;                                                                                 \
    }                                                                                               \
  } while (0)

static std::string tmp_region(const char* tag) {
  char buf[256];
  snprintf(buf, sizeof(buf), "/tmp/vgpu_core_test_%s_%d.cache", tag, (int)getpid());
  unlink(buf);
  return buf;
}

static std::map<std::string, const char*> g_env;
static const char* fake_getenv(const char* k) {
  auto it = g_env.find(k);
  return it == g_env.end() ? nullptr : it->second;
}

static void test_parse_size() {
  uint64_t v = 0;
  CHECK(parse_size("1024", &v) && v == 1024);
  CHECK(parse_size("73728m", &v) && v == 73728ull << 20);
  CHECK(parse_size("16G", &v) && v == 16ull << 30);
  CHECK(parse_size("4k", &v) && v == 4096);
  CHECK(parse_size("2GiB", &v) && v == 2ull << 30);
  CHECK(parse_size("10MB", &v) && v == 10ull << 20);
  CHECK(!parse_size("", &v));
  CHECK(!parse_size("-5m", &v));
  CHECK(!parse_size("12x", &v));
  CHECK(!parse_size("99999999999999999999", &v));
  CHECK(!parse_size("17179869184T", &v));  // overflow after shift
}

static void test_parse_range() {
  int b = 0, e = 0;
  CHECK(parse_range("64-128", &b, &e) && b == 64 && e == 128);
  CHECK(parse_range("32:64", &b, &e) && b == 32 && e == 96);
  CHECK(!parse_range("128-64", &b, &e));
  CHECK(!parse_range("0-300", &b, &e));
  CHECK(!parse_range("abc", &b, &e));
}

static void test_config() {
  g_env.clear();
  g_env["VGPU_DEVICE_MEMORY_LIMIT_0"] = "73728m";
  g_env["VGPU_DEVICE_MEMORY_LIMIT_1"] = "36864m";
  g_env["VGPU_DEVICE_CU_LIMIT"] = "25";
  g_env["VGPU_DEVICE_CU_RANGE_1"] = "64-128";
  g_env["VGPU_SHARED_CACHE"] = "/tmp/x.cache";
  g_env["VGPU_OVERSUBSCRIBE"] = "true";
  g_env["VGPU_TASK_PRIORITY"] = "3";
  g_env["VGPU_CU_MODE"] = "temporal";
  g_env["VGPU_CU_POLICY"] = "FORCE";
  g_env["VGPU_ACTIVE_OOM_KILLER"] = "1";
  Config c;
  load_config(&c, fake_getenv);
  CHECK_EQ(c.num_devices, 2);
  CHECK_EQ(c.dev[0].mem_limit, 73728ull << 20);
  CHECK_EQ(c.dev[1].mem_limit, 36864ull << 20);
  CHECK_EQ(c.dev[0].cu_limit_pct, 25);
  CHECK_EQ(c.dev[1].cu_range_begin, 64);
  CHECK_EQ(c.dev[1].cu_range_end, 128);
  CHECK(c.shared_cache == "/tmp/x.cache");
  CHECK(c.oversubscribe);
  CHECK_EQ(c.priority, 3);
  CHECK(c.cu_mode == CuMode::kTemporal);
  CHECK(c.cu_policy == CuPolicy::kForce);
  CHECK(c.active_oom_killer);
  CHECK(c.any_memory_limit() && c.any_cu_limit());
  // Global fallback and invalid values.
  g_env.clear();
  g_env["VGPU_DEVICE_MEMORY_LIMIT"] = "1g";
  g_env["VGPU_DEVICE_MEMORY_LIMIT_3"] = "garbage";
  g_env["VGPU_DEVICE_CU_LIMIT"] = "150";
  load_config(&c, fake_getenv);
  CHECK_EQ(c.dev[3].mem_limit, 1ull << 30);
  CHECK_EQ(c.dev[7].mem_limit, 1ull << 30);
  CHECK_EQ(c.dev[0].cu_limit_pct, 0);
  CHECK(!c.oversubscribe);
  CHECK(c.cu_mode == CuMode::kAuto);
}

static void test_spill_config() {
  g_env.clear();
  Config c;
  load_config(&c, fake_getenv);
  CHECK(c.spill_policy == SpillPolicy::kLargeFirst);
  CHECK_EQ(c.spill_large_bytes, 256ull << 20);
  CHECK_EQ(spill_reserve(c, 288ull << 30), 18ull << 30);
  CHECK_EQ(spill_reserve(c, 2ull << 30), 512ull << 20);
  CHECK_EQ(spill_reserve(c, 64ull << 30), 4ull << 30);
  g_env["VGPU_SPILL_POLICY"] = "first-come";
  g_env["VGPU_SPILL_LARGE"] = "1g";
  g_env["VGPU_SPILL_RESERVE"] = "3g";
  Config d;
  load_config(&d, fake_getenv);
  CHECK(d.spill_policy == SpillPolicy::kFirstCome);
  CHECK_EQ(d.spill_large_bytes, 1ull << 30);
  CHECK_EQ(spill_reserve(d, 288ull << 30), 3ull << 30);
  g_env.clear();
}

static const char* legacy_env(const char* k) {
  static const std::map<std::string, std::string> m = {
      {"CUDA_DEVICE_MEMORY_LIMIT", "4g"}, {"CUDA_DEVICE_MEMORY_LIMIT_1", "2048m"},
      {"CUDA_DEVICE_SM_LIMIT", "30"},     {"VGPU_DEVICE_MEMORY_LIMIT_2", "1g"},
      {"CUDA_DEVICE_MEMORY_LIMIT_2", "9g"}, {"CUDA_TASK_PRIORITY", "0"},
      {"GPU_CORE_UTILIZATION_POLICY", "FORCE"}, {"CUDA_OVERSUBSCRIBE", "true"}};
  auto it = m.find(k);
  return it == m.end() ? nullptr : it->second.c_str();
}

static void test_legacy_env_names() {
  Config c;
  load_config(&c, legacy_env);
  CHECK_EQ(c.dev[0].mem_limit, 4ull << 30);
  CHECK_EQ(c.dev[1].mem_limit, 2048ull << 20);
  CHECK_EQ(c.dev[2].mem_limit, 1ull << 30);  // the VGPU_* name wins over the legacy one
  CHECK_EQ(c.dev[0].cu_limit_pct, 30);
  CHECK_EQ(c.priority, 0);
  CHECK(c.cu_policy == CuPolicy::kForce);
  CHECK(c.oversubscribe);
}

static void test_override_file() {
  std::string p = tmp_region("override");
  FILE* f = fopen(p.c_str(), "w");
  fprintf(f, "# comment\nVGPU_TEST_OVR_A=1\nexport VGPU_TEST_OVR_B=hello world\n\nbad line\n");
  fclose(f);
  CHECK_EQ(apply_override_env_file(p.c_str()), 2);
  CHECK(!strcmp(getenv("VGPU_TEST_OVR_A"), "1"));
  CHECK(!strcmp(getenv("VGPU_TEST_OVR_B"), "hello world"));
  CHECK_EQ(apply_override_env_file("/nonexistent/file"), 0);
  unlink(p.c_str());
}

static Config limits_cfg(uint64_t lim0) {
  Config c;
  c.dev[0].mem_limit = lim0;
  c.num_devices = 1;
  return c;
}

static void test_region_basic() {
  std::string p = tmp_region("basic");
  Config c = limits_cfg(1000);
  SharedRegion r;
  CHECK_EQ(r.attach(p.c_str(), &c, true), 0);
  CHECK_EQ(r.limit(0), 1000u);
  int s = r.register_process(getpid(), getpid(), 1);
  CHECK(s >= 0);
  CHECK(r.charge(s, 0, 600, kMemData) == Charge::kOk);
  CHECK(r.charge(s, 0, 500, kMemData) == Charge::kOverLimit);
  CHECK(r.charge(s, 0, 400, kMemData) == Charge::kOk);
  CHECK_EQ(r.usage(0), 1000u);
  r.uncharge(s, 0, 600, kMemData);
  CHECK_EQ(r.usage(0), 400u);
  CHECK_EQ(r.proc_usage(s, 0), 400u);
  CHECK_EQ(r.raw()->procs[s].used[0].peak.load(), 1000u);
  CHECK_EQ(r.raw()->procs[s].oom_events.load(), 1u);
  // A second attach sees the same state; env limits do not override stored ones.
  Config c2 = limits_cfg(5000);
  SharedRegion r2;
  CHECK_EQ(r2.attach(p.c_str(), &c2, true), 0);
  CHECK_EQ(r2.limit(0), 1000u);
  CHECK_EQ(r2.usage(0), 400u);
  // Unregister releases the slot's charges.
  r.unregister_process(s);
  CHECK_EQ(r2.usage(0), 0u);
  CHECK_EQ(r2.raw()->hdr.proc_num.load(), 0);
  // Control API.
  r2.set_limit(0, 2000);
  CHECK_EQ(r.limit(0), 2000u);
  r2.suspend_all();
  CHECK_EQ(r.raw()->hdr.suspend_all.load(), 1);
  r2.resume_all();
  CHECK_EQ(r.raw()->hdr.suspend_all.load(), 0);
  // Attach without create to a missing file fails.
  SharedRegion r3;
  CHECK(r3.attach("/tmp/vgpu_core_test_missing.cache", nullptr, false) < 0);
  unlink(p.c_str());
}

static void test_region_unlimited_and_kinds() {
  std::string p = tmp_region("kinds");
  Config c = limits_cfg(0);
  SharedRegion r;
  CHECK_EQ(r.attach(p.c_str(), &c, true), 0);
  int s = r.register_process(getpid(), 0, 1);
  CHECK(r.charge(s, 0, 1ull << 40, kMemData) == Charge::kOk);
  r.force_charge(s, 0, 100, kMemSpill);
  CHECK_EQ(r.raw()->dev[0].spilled.load(), 100u);
  r.uncharge(s, 0, 100, kMemSpill);
  CHECK_EQ(r.raw()->dev[0].spilled.load(), 0u);
  // Uncharging more than charged saturates instead of wrapping.
  r.uncharge(s, 0, (1ull << 40) + 12345, kMemData);
  CHECK_EQ(r.usage(0), 0u);
  r.unregister_process(s);
  unlink(p.c_str());
}

static void test_region_threads_never_overshoot() {
  std::string p = tmp_region("threads");
  const uint64_t limit = 1000000;
  Config c = limits_cfg(limit);
  SharedRegion r;
  CHECK_EQ(r.attach(p.c_str(), &c, true), 0);
  int s = r.register_process(getpid(), 0, 1);
  std::atomic<uint64_t> granted{0};
  std::vector<std::thread> th;
  for (int t = 0; t < 8; t++) {
    th.emplace_back([&] {
      for (int i = 0; i < 20000; i++) {
        if (r.charge(s, 0, 7, kMemData) == Charge::kOk) {
          granted.fetch_add(7);
          if (i % 3 == 0) {
            r.uncharge(s, 0, 7, kMemData);
            granted.fetch_sub(7);
          }
        }
        CHECK(r.usage(0) <= limit);
      }
    });
  }
  for (auto& t : th) t.join();
  CHECK_EQ(r.usage(0), granted.load());
  CHECK(r.usage(0) <= limit);
  r.unregister_process(s);
  unlink(p.c_str());
}

static void test_region_multiprocess_and_reclaim() {
  std::string p = tmp_region("mp");
  Config c = limits_cfg(1000);
  SharedRegion r;
  CHECK_EQ(r.attach(p.c_str(), &c, true), 0);
  // Children charge and exit without unregistering (crash): reclaim must free it.
  for (int k = 0; k < 4; k++) {
    pid_t pid = fork();
    if (pid == 0) {
      SharedRegion rc;
      if (rc.attach(p.c_str(), nullptr, false) != 0) _exit(2);
      int s = rc.register_process(getpid(), 0, 1);
      if (s < 0) _exit(3);
      _exit(rc.charge(s, 0, 200, kMemData) == Charge::kOk ? 0 : 4);
    }
    int st = 0;
    waitpid(pid, &st, 0);
    CHECK(WIFEXITED(st) && WEXITSTATUS(st) == 0);
  }
  CHECK_EQ(r.usage(0), 800u);
  CHECK_EQ(r.raw()->hdr.proc_num.load(), 4);
  // Over the limit: charge() reclaims the dead slots and retries (reference oom_check).
  int s = r.register_process(getpid(), 0, 1);
  CHECK(r.charge(s, 0, 900, kMemData) == Charge::kOk);
  CHECK_EQ(r.usage(0), 900u);
  CHECK_EQ(r.raw()->hdr.proc_num.load(), 1);
  CHECK_EQ(r.reclaim_dead(), 0);
  r.unregister_process(s);
  unlink(p.c_str());
}

static void test_region_robust_lock() {
  std::string p = tmp_region("robust");
  Config c = limits_cfg(1000);
  SharedRegion r;
  CHECK_EQ(r.attach(p.c_str(), &c, true), 0);
  pid_t pid = fork();
  if (pid == 0) {
    SharedRegion rc;
    if (rc.attach(p.c_str(), nullptr, false) != 0) _exit(2);
    rc.lock();
    _exit(0);  // dies holding the lock
  }
  int st = 0;
  waitpid(pid, &st, 0);
  CHECK(r.lock());  // EOWNERDEAD → consistent
  r.unlock();
  CHECK(r.lock());
  r.unlock();
  unlink(p.c_str());
}

// Fault injection (SURVEY §5 "SIGSTOP the lock owner"): a process stopped while it holds
// the region lock. Charges under the limit never take the lock; an over-limit charge (its
// reclaim pass wants the lock) turns into an OOM within the bound instead of hanging, and
// set_cu_limit (vgpuctl, the monitor) completes too. Once the holder dies the robust
// mutex recovers.
static void test_region_stopped_lock_owner() {
  std::string p = tmp_region("stopped");
  Config c = limits_cfg(1000);
  SharedRegion r;
  CHECK_EQ(r.attach(p.c_str(), &c, true), 0);
  int s = r.register_process(getpid(), getpid(), 1);
  pid_t pid = fork();
  if (pid == 0) {
    SharedRegion rc;
    if (rc.attach(p.c_str(), nullptr, false) != 0) _exit(2);
    rc.lock();
    raise(SIGSTOP);
    _exit(0);
  }
  int st = 0;
  CHECK_EQ(waitpid(pid, &st, WUNTRACED), pid);
  CHECK(WIFSTOPPED(st));
  uint64_t t0 = now_ns();
  CHECK(r.charge(s, 0, 600, kMemData) == Charge::kOk);         // lock-free admission
  CHECK(now_ns() - t0 < 100'000'000ull);
  t0 = now_ns();
  CHECK(r.charge(s, 0, 600, kMemData) == Charge::kOverLimit);  // reclaim gives up: OOM
  uint64_t waited = now_ns() - t0;
  CHECK(waited >= (uint64_t)kLockTimeoutMs * 900000ull && waited < (uint64_t)kLockTimeoutMs * 3000000ull);
  t0 = now_ns();
  r.set_cu_limit(0, 25);
  CHECK(now_ns() - t0 < (uint64_t)kLockTimeoutMs * 3000000ull);
  CHECK_EQ(r.raw()->dev[0].cu_limit_pct, 25);
  kill(pid, SIGKILL);
  waitpid(pid, &st, 0);
  CHECK(r.lock());  // EOWNERDEAD -> consistent
  r.unlock();
  r.uncharge(s, 0, 600, kMemData);
  r.unregister_process(s);
  unlink(p.c_str());
}

// Node-side reclaim (monitor, vgpuctl) runs outside the tenant's PID namespace: a slot
// whose PID belongs to another namespace is never judged by the caller's /proc.
static void test_region_reclaim_namespaces() {
  std::string p = tmp_region("pidns");
  Config c = limits_cfg(1000);
  SharedRegion r;
  CHECK_EQ(r.attach(p.c_str(), &c, true), 0);
  CHECK(self_pidns() != 0);
  for (int foreign = 0; foreign < 2; foreign++) {
    pid_t pid = fork();
    if (pid == 0) {
      SharedRegion rc;
      if (rc.attach(p.c_str(), nullptr, false) != 0) _exit(2);
      int s = rc.register_process(getpid(), 0, 1);
      if (s < 0 || rc.raw()->procs[s].pidns != self_pidns()) _exit(3);
      if (foreign) rc.raw()->procs[s].pidns = 12345;  // as if registered in another namespace
      rc.charge(s, 0, 100, kMemData);
      _exit(0);  // dies without unregistering
    }
    int st = 0;
    waitpid(pid, &st, 0);
    CHECK(WIFEXITED(st) && WEXITSTATUS(st) == 0);
    CHECK_EQ(r.usage(0), 100u);
    CHECK_EQ(r.reclaim_dead(), foreign ? 0 : 1);  // same namespace: reclaimed; foreign: kept
    CHECK_EQ(r.usage(0), foreign ? 100u : 0u);
  }
  unlink(p.c_str());
}

static void test_region_version_guard() {
  std::string p = tmp_region("ver");
  Config c = limits_cfg(1);
  {
    SharedRegion r;
    CHECK_EQ(r.attach(p.c_str(), &c, true), 0);
    r.raw()->hdr.version = 999;
  }
  SharedRegion r2;
  CHECK(r2.attach(p.c_str(), &c, true) < 0);
  unlink(p.c_str());
}

// Fault injection: a region file whose header was overwritten, and one cut short, are
// re-initialised by a creating attach (the tenant keeps running with its env limits) and
// refused by a read-only attach (vgpuctl / the monitor never act on garbage).
static void test_region_corruption() {
  std::string p = tmp_region("corrupt");
  Config c = limits_cfg(4096);
  {
    SharedRegion r;
    CHECK_EQ(r.attach(p.c_str(), &c, true), 0);
    int slot = r.register_process(getpid(), 0, 1);
    CHECK(slot >= 0);
    CHECK(r.charge(slot, 0, 100, kMemData) == Charge::kOk);
  }
  {
    int fd = open(p.c_str(), O_WRONLY);
    CHECK(fd >= 0);
    char junk[256];
    for (size_t i = 0; i < sizeof(junk); i++) junk[i] = (char)(0x5a ^ i);
    CHECK(pwrite(fd, junk, sizeof(junk), 0) == (ssize_t)sizeof(junk));
    close(fd);
  }
  {
    SharedRegion ro;
    CHECK_EQ(ro.attach(p.c_str(), nullptr, false), -EINVAL);
    SharedRegion r;
    CHECK_EQ(r.attach(p.c_str(), &c, true), 0);
    CHECK_EQ(r.limit(0), (uint64_t)4096);
    CHECK_EQ(r.usage(0), (uint64_t)0);
    CHECK(r.lock());
    r.unlock();
  }
  CHECK(truncate(p.c_str(), 100) == 0);
  {
    SharedRegion ro;
    CHECK(ro.attach(p.c_str(), nullptr, false) < 0);
    SharedRegion r;
    CHECK_EQ(r.attach(p.c_str(), &c, true), 0);
    CHECK_EQ(r.limit(0), (uint64_t)4096);
  }
  unlink(p.c_str());
}

static void test_proc_alive() {
  CHECK(proc_alive(getpid(), proc_start_time(getpid())));
  CHECK(!proc_alive(getpid(), proc_start_time(getpid()) + 1));
  pid_t pid = fork();
  if (pid == 0) _exit(0);
  int st;
  waitpid(pid, &st, 0);
  CHECK(!proc_alive(pid, 0));
}

static void test_cumask() {
  CHECK_EQ(cu_share_count(256, 8, 25), 64);
  CHECK_EQ(cu_share_count(256, 8, 50), 128);
  CHECK_EQ(cu_share_count(256, 8, 33), 80);    // 84.48 → 80 (multiple of 8)
  CHECK_EQ(cu_share_count(256, 8, 1), 8);      // at least one CU per XCC
  CHECK_EQ(cu_share_count(256, 8, 0), 256);
  CHECK_EQ(cu_share_count(256, 8, 100), 256);
  CuMask m = cu_mask_for(256, 8, 25, -1, -1);
  CHECK_EQ(m.count(), 64);
  CHECK(m.test(0) && m.test(63) && !m.test(64));
  CHECK(cu_mask_balanced(m, 8));
  CuMask r = cu_mask_range(256, 8, 3, 61);  // snapped to [0,64)
  CHECK_EQ(r.count(), 64);
  // Partition 256 CUs among 3 tenants: 88/88/80, disjoint, covering.
  int b[3], e[3];
  for (int i = 0; i < 3; i++) cu_partition_range(256, 8, 3, i, &b[i], &e[i]);
  CHECK_EQ(b[0], 0);
  CHECK_EQ(e[0] - b[0], 88);
  CHECK_EQ(b[1], e[0]);
  CHECK_EQ(e[1] - b[1], 88);
  CHECK_EQ(b[2], e[1]);
  CHECK_EQ(e[2], 256);
  for (int split = 1; split <= 32; split++) {
    int covered = 0, prev_end = 0;
    for (int i = 0; i < split; i++) {
      int bb, ee;
      cu_partition_range(256, 8, split, i, &bb, &ee);
      CHECK_EQ(bb, prev_end);
      CHECK(ee > bb);
      CHECK_EQ((ee - bb) % 8, 0);
      CHECK(cu_mask_balanced(cu_mask_range(256, 8, bb, ee), 8));
      covered += ee - bb;
      prev_end = ee;
    }
    CHECK_EQ(covered, 256);
  }
  // Unbalanced masks.
  CuMask u;
  u.nbits = 256;
  u.set(0);
  CHECK(!cu_mask_balanced(u, 8));
  // Intersection: a user mask cannot escape the vGPU; an unbalanced result falls back.
  CuMask vg = cu_mask_range(256, 8, 64, 128);
  CuMask user = cu_mask_range(256, 8, 0, 96);
  CuMask x = cu_mask_intersect(user, vg, 8);
  CHECK_EQ(x.count(), 32);
  CHECK(x.test(64) && !x.test(96) && !x.test(0));
  CuMask bad = cu_mask_intersect(u, vg, 8);
  CHECK_EQ(bad.count(), 64);
}

static void test_cumask_se_layout() {
  // Bijection over the chip.
  std::vector<int> seen(256, 0);
  for (int L = 0; L < 256; L++) seen[cu_logical_to_bit(256, 8, 4, L)]++;
  for (int b = 0; b < 256; b++) CHECK_EQ(seen[b], 1);
  // N = 4 tenants: each gets one whole SE on every XCC, disjoint between tenants.
  for (int slot = 0; slot < 4; slot++) {
    CuMask m = cu_mask_range(256, 8, slot * 64, slot * 64 + 64, 4);
    CHECK_EQ(m.count(), 64);
    CHECK(cu_mask_balanced(m, 8));
    for (int b = 0; b < 256; b++)
      if (m.test(b)) CHECK_EQ((b / 8) % 4, slot);  // KFD: SE = local index % num_se
  }
  // N = 8: half an SE each; N = 2: two SEs each.
  CuMask h = cu_mask_range(256, 8, 32, 64, 4);
  for (int b = 0; b < 256; b++)
    if (h.test(b)) CHECK_EQ((b / 8) % 4, 0);
  CuMask two = cu_mask_range(256, 8, 128, 256, 4);
  for (int b = 0; b < 256; b++)
    if (two.test(b)) CHECK((b / 8) % 4 >= 2);
  // num_se = 1 is the identity (interleaved layout).
  for (int L = 0; L < 256; L++) CHECK_EQ(cu_logical_to_bit(256, 8, 1, L), L);
}

static void test_devmap() {
  DeviceMap m;
  CHECK(parse_device_map("0:GPU-aaaa 1:GPU-bbbb", &m));
  CHECK_EQ(m.n, 2);
  CHECK_EQ(m.duplicates, 0);
  CHECK(parse_device_map("0:GPU-aaaa 1:gpu-AAAA", &m));
  CHECK_EQ(m.duplicates, 1);
  CHECK(!parse_device_map("0-GPU", &m));
  CHECK(!parse_device_map("99:GPU-x", &m));
  CHECK(parse_device_map("", &m) && m.n == 0);
  CHECK(parse_device_map(nullptr, &m) && m.n == 0);
  char u[64];
  normalize_uuid("GPU-98139BA16298D729", u, sizeof(u));
  CHECK(!strcmp(u, "98139ba16298d729"));

  Config c;
  c.dev[0].mem_limit = 100;
  c.dev[0].cu_limit_pct = 25;
  c.dev[0].cu_range_begin = 0;
  c.dev[0].cu_range_end = 64;
  c.dev[1].mem_limit = 200;
  c.dev[1].cu_limit_pct = 25;
  c.dev[1].cu_range_begin = 64;
  c.dev[1].cu_range_end = 128;
  c.dev[2].mem_limit = 300;
  // Map order differs from agent order; vGPUs 0 and 1 share physical GPU bbbb.
  CHECK(parse_device_map("0:GPU-bbbb 1:GPU-bbbb 2:GPU-aaaa", &m));
  const char* agents[2] = {"GPU-aaaa", "GPU-bbbb"};
  DeviceConfig out[kMaxDevices];
  CHECK_EQ(resolve_devices(c, m, agents, 2, out), 2);
  CHECK_EQ(out[0].mem_limit, 300u);
  CHECK_EQ(out[1].mem_limit, 300u);  // 100 + 200 merged
  CHECK_EQ(out[1].cu_limit_pct, 50);
  CHECK_EQ(out[1].cu_range_begin, 0);
  CHECK_EQ(out[1].cu_range_end, 128);
  // No map: positional.
  DeviceMap empty;
  resolve_devices(c, empty, agents, 2, out);
  CHECK_EQ(out[0].mem_limit, 100u);
  CHECK_EQ(out[1].mem_limit, 200u);
}

// Closed-loop simulation of the temporal limiter against a GPU model: each tenant's
// host enqueues 300 µs kernels every 20 µs while its gate is open (queue depth 64, so
// the GPU runs far behind the host), the GPU serves the busy tenants processor-sharing
// (k busy tenants progress at 1/k each), and the sampler charges each tenant its
// occupancy share every ~1 ms (±25 % jitter), as watcher.cpp does. Returns each
// tenant's achieved throughput as a fraction of the whole GPU.
static std::vector<double> simulate_limiter(const std::vector<int>& limits, double seconds, int sample_us = 1000) {
  const int n = (int)limits.size();
  const int64_t step_ns = 10'000, kernel_ns = 300'000, launch_ns = 20'000, depth = 64;
  std::vector<DeviceState> dev(n);
  std::vector<TimeShareParams> par(n);
  std::vector<int64_t> backlog(n, 0), next_launch(n, 0);
  std::vector<double> done(n, 0);
  std::vector<int> prev_pm(n, 0);
  std::vector<bool> opened(n, false);
  for (int i = 0; i < n; i++) {
    par[i] = timeshare_params(limits[i]);
    dev[i].credit_ns.store(par[i].burst_ns);
    dev[i].gate_open.store(1);
  }
  unsigned rng = 12345;
  int64_t next_sample = sample_us * 1000, last_sample = 0;
  const int64_t end = (int64_t)(seconds * 1e9);
  for (int64_t t = 0; t < end; t += step_ns) {
    for (int i = 0; i < n; i++) {  // host side: gate + enqueue
      if (t >= next_launch[i] && dev[i].gate_open.load() && backlog[i] < depth * kernel_ns) {
        backlog[i] += kernel_ns;
        next_launch[i] = t + launch_ns;
      }
    }
    int k = 0;
    for (int i = 0; i < n; i++) k += backlog[i] > 0;
    for (int i = 0; i < n; i++) {  // GPU side: processor sharing
      if (backlog[i] <= 0) continue;
      int64_t prog = std::min<int64_t>(backlog[i], step_ns / k);
      backlog[i] -= prog;
      done[i] += (double)prog;
    }
    if (t >= next_sample) {  // sampler: occupancy share at the sample instant
      int64_t dt = t - last_sample;
      last_sample = t;
      int busy = 0;
      for (int i = 0; i < n; i++) busy += backlog[i] > 0;
      for (int i = 0; i < n; i++) {
        int pm = (int)timeshare_charge(1000, backlog[i] > 0 ? 32 : 0, 32 * (int64_t)busy);
        int64_t charge = timeshare_interval(dt, prev_pm[i], pm, opened[i]);
        bool was_closed = !dev[i].gate_open.load();
        timeshare_apply(dev[i], par[i], dt, charge);
        opened[i] = was_closed && dev[i].gate_open.load();
        prev_pm[i] = pm;
      }
      rng = rng * 1103515245u + 12345u;
      next_sample = t + sample_us * 750 + (int64_t)((rng >> 8) % (uint32_t)(sample_us * 500));
    }
  }
  std::vector<double> frac(n);
  for (int i = 0; i < n; i++) frac[i] = done[i] / (double)end;
  return frac;
}

static void test_ratelimit() {
  // Charging: busy time weighted by the container's share of resident waves.
  CHECK_EQ(timeshare_charge(1000000, 0, 100), 0);
  CHECK_EQ(timeshare_charge(1000000, 64, 64), 1000000);
  CHECK_EQ(timeshare_charge(900000, 10, 30), 300000);
  CHECK_EQ(timeshare_charge(1000000, 50, 10), 1000000);  // total below mine: alone
  // Progress floor: co-running at full own occupancy pays what it would alone; crowded
  // down to a third of its peak it pays the share (here larger); no reference: the share.
  CHECK_EQ(timeshare_progress_pm(500, 40, 40), 1000);
  CHECK_EQ(timeshare_progress_pm(500, 30, 40), 750);
  CHECK_EQ(timeshare_progress_pm(400, 10, 30), 400);
  CHECK_EQ(timeshare_progress_pm(400, 10, 0), 400);
  CHECK_EQ(timeshare_progress_pm(0, 0, 40), 0);
  // The occupancy reference follows peaks at once and decays slowly (1/2048 per sample).
  CHECK_EQ(occupancy_ref_update(0, 64), 64);
  CHECK_EQ(occupancy_ref_update(4096, 0), 4094);
  CHECK_EQ(occupancy_ref_update(4096, 5000), 5000);
  // Credit arithmetic and clamps.
  TimeShareParams p = timeshare_params(25);
  CHECK_EQ(p.burst_ns, 10000000);
  CHECK_EQ(p.reopen_ns, 5000000);
  CHECK_EQ(timeshare_params(5).burst_ns, 4000000);
  CHECK(timeshare_gate(true, 1, p) && !timeshare_gate(true, 0, p));
  CHECK(!timeshare_gate(false, p.reopen_ns - 1, p) && timeshare_gate(false, p.reopen_ns, p));
  CHECK_EQ(timeshare_step(0, p, 1000000, 1000000), -750000);
  CHECK_EQ(timeshare_step(0, p, 1000000, 0), 250000);
  CHECK_EQ(timeshare_step(p.burst_ns, p, 1000000, 0), p.burst_ns);
  CHECK_EQ(timeshare_step(-p.debt_ns, p, 1000000, 1000000), -p.debt_ns);
  // Unlimited: grants the whole interval.
  CHECK_EQ(timeshare_step(0, timeshare_params(0), 1000000, 1000000), 0);
  // Exact share (basis points) next to the rounded-up whole percent: split 16 = 6.25 %.
  TimeShareParams q = timeshare_params(7, 40, 625);
  CHECK_EQ(q.limit_bp, 625);
  CHECK_EQ(timeshare_step(0, q, 1000000, 0), 62500);
  CHECK_EQ(timeshare_step(0, timeshare_params(7), 1000000, 0), 70000);
  CHECK_EQ(timeshare_params(0, 40, 625).limit_bp, 0);  // unlimited stays unlimited
  // Sampling periods: base while the node-wide reads fit the budget, then proportional.
  CHECK_EQ(sample_period_ns(1000000, 1, 32, 10000000), 1000000);
  CHECK_EQ(sample_period_ns(1000000, 5 * 5, 32, 10000000), 1000000);   // 5 processes: base
  CHECK_EQ(sample_period_ns(1000000, 8 * 8, 32, 10000000), 2000000);
  CHECK_EQ(sample_period_ns(1000000, 12 * 12, 32, 10000000), 4500000);  // 12 pods
  CHECK_EQ(sample_period_ns(1000000, 64 * 64, 32, 10000000), 10000000);
  CHECK_EQ(sample_period_ns(1000000, 64 * 64, 0, 10000000), 1000000);   // budget 0: fixed
  CHECK_EQ(sample_period_ns(20000000, 64 * 64, 32, 10000000), 20000000);  // never below base

  // Closed loop, one tenant: achieved share within 2 points of every limit.
  for (int lim : {10, 25, 50, 75, 90}) {
    double got = simulate_limiter({lim}, 4.0)[0] * 100.0;
    if (getenv("VGPU_SIM_VERBOSE") || got < lim - 2.0 || got > lim + 2.0) fprintf(stderr, "limit %d: achieved %.2f %%\n", lim, got);
    CHECK(got >= lim - 2.0 && got <= lim + 2.0);
  }
  // Two concurrent tenants: each gets its limit of the GPU's throughput; when both
  // limits sum to more than the GPU, each gets its processor share instead.
  for (int lim : {10, 25, 40}) {
    std::vector<double> got = simulate_limiter({lim, lim}, 4.0);
    for (double g : got) {
      if (getenv("VGPU_SIM_VERBOSE") || g * 100 < lim - 2.0 || g * 100 > lim + 2.0) fprintf(stderr, "2x%d: achieved %.2f %%\n", lim, g * 100);
      CHECK(g * 100 >= lim - 2.0 && g * 100 <= lim + 2.0);
    }
  }
  {
    std::vector<double> got = simulate_limiter({75, 75}, 4.0);
    CHECK(got[0] > 0.46 && got[1] > 0.46 && got[0] + got[1] > 0.97);
    std::vector<double> mixed = simulate_limiter({20, 100}, 4.0);  // limited next to an unlimited one
    CHECK(mixed[0] * 100 >= 18.0 && mixed[0] * 100 <= 22.0);
    CHECK(mixed[0] + mixed[1] > 0.97);  // the GPU stays busy
  }

  // The launch-side gate.
  std::string path = tmp_region("rl");
  Config c = limits_cfg(0);
  SharedRegion r;
  CHECK_EQ(r.attach(path.c_str(), &c, true), 0);
  DeviceState& d = r.raw()->dev[0];
  RegionHeader& h = r.raw()->hdr;
  d.credit_ns.store(1000);
  d.gate_open.store(1);
  d.cu_mode.store(2);  // on the GPU-time limiter
  h.watcher_heartbeat.store(now_ns());
  CHECK(!limiter_would_block(h, d, true));
  CHECK_EQ(limiter_acquire(h, d, true), 0u);
  // Exhausted credit blocks until the sampler grants more.
  d.credit_ns.store(-1);
  d.gate_open.store(0);
  CHECK(limiter_would_block(h, d, true));
  CHECK(!limiter_would_block(h, d, false));  // not limited: credit ignored
  std::thread refill([&] {
    usleep(30000);
    h.watcher_heartbeat.store(now_ns());
    d.credit_ns.store(500);
    d.gate_open.store(1);
  });
  uint64_t waited = limiter_acquire(h, d, true);
  refill.join();
  CHECK(waited >= 20000000u);
  // A launch blocked on the credit is released when the device leaves the GPU-time limiter
  // (auto mode back on the CU mask): nobody would re-open the gate (profiles/r3g).
  d.credit_ns.store(-100000);
  d.gate_open.store(0);
  std::atomic<bool> stop_hb{false};
  std::thread hb([&] {
    while (!stop_hb) {
      h.watcher_heartbeat.store(now_ns());  // the maintenance thread stays alive
      usleep(1000);
    }
  });
  std::thread leave([&] {
    usleep(30000);
    d.cu_mode.store(1);
  });
  waited = limiter_acquire(h, d, true);
  leave.join();
  stop_hb = true;
  hb.join();
  CHECK(waited >= 20000000u && waited < 500000000u);
  d.cu_mode.store(2);
  // A dead sampler (stale heartbeat) never blocks launches forever.
  d.credit_ns.store(-100000);
  d.gate_open.store(0);
  h.watcher_heartbeat.store(now_ns() - 5'000'000'000ull);
  CHECK(limiter_acquire(h, d, true) < 100'000'000u);
  // The external launch block holds every mode, limited or not.
  h.recent_kernel.store(-1);
  CHECK(limiter_would_block(h, d, false));
  std::thread unblock([&] {
    usleep(30000);
    h.recent_kernel.store(2);
  });
  waited = limiter_acquire(h, d, false);
  unblock.join();
  CHECK(waited >= 20000000u);
  // Sampler bookkeeping.
  d.credit_ns.store(0);
  timeshare_apply(d, timeshare_params(50), 100'000'000, 100'000'000);
  CHECK_EQ(d.credit_ns.load(), -50'000'000);
  CHECK_EQ(d.gate_open.load(), 0);
  CHECK_EQ(d.charged_ns.load(), 100'000'000u);
  CHECK_EQ(d.util_pm.load(), 1000);
  unlink(path.c_str());
}

static void test_auto_mode_and_live_cu() {
  CHECK(effective_cu_mode(CuMode::kAuto, 50) == CuMode::kSpatial);
  CHECK(effective_cu_mode(CuMode::kAuto, 100) == CuMode::kSpatial);
  CHECK(effective_cu_mode(CuMode::kAuto, 25) == CuMode::kTemporal);      // crowd not assessed yet
  CHECK(effective_cu_mode(CuMode::kAuto, 12) == CuMode::kTemporal);
  CHECK(effective_cu_mode(CuMode::kAuto, 25, 0) == CuMode::kSpatial);    // alone: keep the CU mask
  CHECK(effective_cu_mode(CuMode::kAuto, 25, 1) == CuMode::kSpatial);    // one other busy tenant
  CHECK(effective_cu_mode(CuMode::kAuto, 25, 2) == CuMode::kTemporal);   // crowded: GPU-time limiter
  CHECK(effective_cu_mode(CuMode::kAuto, 60, 7) == CuMode::kSpatial);    // large shares always masked
  CHECK(effective_cu_mode(CuMode::kTemporal, 25, 0) == CuMode::kTemporal);
  CHECK(effective_cu_mode(CuMode::kTemporal, 75) == CuMode::kTemporal);
  CHECK(effective_cu_mode(CuMode::kSpatial, 10) == CuMode::kSpatial);
  // set_cu_limit recomputes the mask around the vGPU's anchor and bumps the generation.
  std::string p = tmp_region("livecu");
  Config c = limits_cfg(0);
  c.dev[0].cu_limit_pct = 50;
  c.dev[0].cu_range_begin = 128;
  c.dev[0].cu_range_end = 256;
  SharedRegion r;
  CHECK_EQ(r.attach(p.c_str(), &c, true), 0);
  DeviceState& d = r.raw()->dev[0];
  d.cu_count = 256;
  d.num_xcc = 8;
  d.num_se = 4;
  d.configured = 1;
  uint64_t g0 = r.raw()->hdr.generation.load();
  r.set_cu_limit(0, 25);
  CHECK(r.raw()->hdr.generation.load() > g0);
  CuMask m;
  memcpy(m.words, d.cu_mask, sizeof(m.words));
  m.nbits = 256;
  CHECK_EQ(m.count(), 64);
  CHECK(cu_mask_balanced(m, 8));
  for (int b = 0; b < 256; b++)
    if (m.test(b)) CHECK_EQ((b / 8) % 4, 2);  // logical [128,192) = SE 2 of every XCC
  r.set_cu_limit(0, 75);  // would run past the end: shifted left to [64, 256)
  memcpy(m.words, d.cu_mask, sizeof(m.words));
  CHECK_EQ(m.count(), 192);
  CHECK_EQ(d.cu_range_begin, 128);  // the anchor is kept
  unlink(p.c_str());
}

static void test_charge_overflow() {
  std::string p = tmp_region("ovf");
  Config c = limits_cfg(1ull << 30);
  SharedRegion r;
  CHECK_EQ(r.attach(p.c_str(), &c, true), 0);
  int s = r.register_process(getpid(), 0, 1);
  CHECK(r.charge(s, 0, 1ull << 29, kMemData) == Charge::kOk);
  // cur + bytes wraps past 2^64: must be refused, not admitted.
  CHECK(r.charge(s, 0, ~0ull - 100, kMemData) == Charge::kOverLimit);
  CHECK(r.charge(s, 0, ~0ull, kMemData) == Charge::kOverLimit);
  CHECK_EQ(r.usage(0), 1ull << 29);
  r.unregister_process(s);
  unlink(p.c_str());
}

// Fake KFD tree + fake VRAM probe for host-PID discovery.
struct FakeKfd {
  std::string root;
  uint32_t gid = 7;
  void write(int pid, int64_t v) {
    FILE* f = fopen((root + "/" + std::to_string(pid) + "/vram_" + std::to_string(gid)).c_str(), "w");
    if (f) {
      fprintf(f, "%lld\n", (long long)v);
      fclose(f);
    }
  }
  void add(int pid, int64_t v) {
    CHECK(system(("mkdir -p " + root + "/" + std::to_string(pid) + "/stats_" + std::to_string(gid)).c_str()) == 0);
    write(pid, v);
  }
  void bump(int pid, int64_t delta) {
    int64_t v = kfd_vram_usage(pid, gid);
    write(pid, v + delta);
  }
};

struct ProbeCtx {
  FakeKfd* k;
  int self;
  int mimic = -1;     // a foreign process that happens to allocate the same size once
  int mimic_left = 0;
  int noisy = -1;     // a foreign process allocating 4 MiB on every probe
};

static bool fake_probe(void* vctx, uint64_t bytes, bool alloc) {
  ProbeCtx* c = static_cast<ProbeCtx*>(vctx);
  int64_t d = alloc ? (int64_t)bytes : -(int64_t)bytes;
  c->k->bump(c->self, d);
  if (alloc && c->mimic >= 0 && c->mimic_left > 0) {
    c->k->bump(c->mimic, (int64_t)bytes);
    c->mimic_left--;
  }
  if (alloc && c->noisy >= 0) c->k->bump(c->noisy, 4 << 20);
  return true;
}

static void test_hostpid_resolution() {
  char dir[] = "/tmp/vgpu_kfdpid_XXXXXX";
  CHECK(mkdtemp(dir) != nullptr);
  static std::string kroot;
  kroot = dir;
  FakeKfd k{kroot};
  g_kfd_proc_root = kroot.c_str();
  std::string lock = kroot + "/lockdir/lock";
  for (int p : {100, 200, 300, 400}) k.add(p, 64ll << 20);
  // A namespaced process is found by its VRAM signature despite a mimic and noise.
  ProbeCtx ctx{&k, 200, 300, 1, 100};
  CHECK_EQ(kfd_resolve_hostpid(k.gid, fake_probe, &ctx, lock.c_str(), 100, 42), 200);
  CHECK_EQ(kfd_vram_usage(200, k.gid), 64ll << 20);  // every probe freed again
  // A failing probe allocation resolves nothing.
  CHECK_EQ(kfd_resolve_hostpid(k.gid, [](void*, uint64_t, bool) { return false; }, nullptr, nullptr, 0, 1), 0);
  // No probe: unresolved, unless KFD lists our own PID (no PID namespace).
  CHECK_EQ(kfd_resolve_hostpid(k.gid, nullptr, nullptr, nullptr, 0, 1), 0);
  k.add(getpid(), 0);
  CHECK_EQ(kfd_resolve_hostpid(k.gid, nullptr, nullptr, nullptr, 0, 1), getpid());
  CHECK(system(("rm -rf " + kroot + "/" + std::to_string(getpid())).c_str()) == 0);
  // A lock somebody holds forever (any tenant can flock the node-wide file) delays the
  // search by the wait only: it then runs unlocked and still resolves. Creating the lock
  // leaves the process umask alone.
  const mode_t um = umask(022);
  int held = kfd_lock(lock.c_str(), 0);
  CHECK(held >= 0);
  CHECK_EQ((int)umask(022), 022);
  umask(um);
  CHECK_EQ(kfd_lock(lock.c_str(), 5), kLockBusy);
  ProbeCtx c2{&k, 400};
  CHECK_EQ(kfd_resolve_hostpid(k.gid, fake_probe, &c2, lock.c_str(), 20, 7), 400);
  kfd_unlock(held);
  CHECK_EQ(kfd_resolve_hostpid(k.gid, fake_probe, &c2, lock.c_str(), 20, 7), 400);
  // The plugin's lock is a read-only file: flock works on it all the same.
  CHECK(chmod(lock.c_str(), 0444) == 0);
  int ro = kfd_lock(lock.c_str(), 0);
  CHECK(ro >= 0);
  kfd_unlock(ro);
  CHECK_EQ(kfd_lock((kroot + "/no/such/dir/lock").c_str(), 0), kLockUnavailable);

  // 16 processes of one container start together while foreign processes come and go
  // and allocate: every one resolves its own host PID (serialised by the lock).
  const int kStarters = 16;
  for (int i = 0; i < kStarters; i++) k.add(1000 + i, (int64_t)(i + 1) << 21);
  // The noise process stops cooperatively (a stop file): killing it could orphan one of
  // its `mkdir -p` helpers, which then races the final rm -rf.
  const std::string stop_file = kroot + "/stop";
  pid_t noise = fork();
  if (noise == 0) {
    unsigned rng = 99;
    for (int it = 0; it < 4000 && access(stop_file.c_str(), F_OK) != 0; it++) {
      rng = rng * 1103515245u + 12345u;
      int p = 5000 + (int)((rng >> 8) % 64);
      if ((rng >> 20) % 3 == 0) k.add(p, 0);
      else k.bump(p, (int64_t)(2 + (rng >> 12) % 40) << 21);
      usleep(200);
    }
    _exit(0);
  }
  std::vector<pid_t> kids;
  for (int i = 0; i < kStarters; i++) {
    pid_t c = fork();
    if (c == 0) {
      ProbeCtx pc{&k, 1000 + i};
      pid_t got = kfd_resolve_hostpid(k.gid, fake_probe, &pc, lock.c_str(), 20000, (unsigned)(i * 7919 + 1));
      _exit(got == 1000 + i ? 0 : 1);
    }
    kids.push_back(c);
  }
  int ok = 0;
  for (pid_t c : kids) {
    int st = 0;
    waitpid(c, &st, 0);
    ok += WIFEXITED(st) && WEXITSTATUS(st) == 0;
  }
  FILE* sf = fopen(stop_file.c_str(), "w");
  if (sf) fclose(sf);
  waitpid(noise, nullptr, 0);
  CHECK_EQ(ok, kStarters);
  CHECK(system(("rm -rf " + kroot).c_str()) == 0);
  g_kfd_proc_root = "/sys/class/kfd/kfd/proc";
}

static void test_board() {
  char dir[] = "/tmp/vgpu_board_XXXXXX";
  CHECK(mkdtemp(dir) != nullptr);
  Board a, b;
  CHECK_EQ(a.open(dir, "a.slot"), 0);
  CHECK_EQ(b.open(dir, "b.slot"), 0);
  CHECK_EQ(a.open(dir, "../escape.slot"), -EINVAL);
  const uint64_t now = now_ns();
  const uint32_t gpus_a[2] = {1000, 1001}, gpus_b[1] = {1001};
  a.publish(kPrioNormal, gpus_a, 2, {4242, 4243}, now);
  b.publish(kPrioBackground, gpus_b, 1, {5151}, now);
  // Each sees the other, never itself.
  CHECK_EQ((int)b.refresh(now).size(), 1);
  CHECK_EQ(b.priority_of(4243, 1001), kPrioNormal);
  CHECK_EQ(a.refresh(now).size(), 1u);
  CHECK_EQ(a.priority_of(5151, 1001), kPrioBackground);
  CHECK_EQ(a.priority_of(5151, 1000), kPrioNormal);  // not on that GPU: unknown = normal
  CHECK_EQ(a.priority_of(9999, 1001), kPrioNormal);  // on no slot
  // A slot file untouched for longer than kBoardSkipAgeS is skipped unread (its container
  // has no live publisher), whatever its heartbeat says; publishing touches it again.
  {
    const std::string bpath = std::string(dir) + "/b.slot";
    struct timespec old[2] = {{time(nullptr) - kBoardSkipAgeS - 5, 0}, {time(nullptr) - kBoardSkipAgeS - 5, 0}};
    CHECK_EQ(utimensat(AT_FDCWD, bpath.c_str(), old, 0), 0);
    CHECK_EQ(a.refresh(now).size(), 0u);
    Board b2;
    CHECK_EQ(b2.open(dir, "b.slot"), 0);
    b2.publish(kPrioBackground, gpus_b, 1, {5151}, now);
    CHECK_EQ(a.refresh(now).size(), 1u);
  }
  // Concurrency admission across CPU sockets (k = 2, nodes published): a holder on node 0,
  // a waiter of node 0 that came first and one of node 1 - the node-1 one is admitted next to
  // the holder, the node-0 one waits for the holder's turn to end.
  {
    Board h, w0, w1;
    CHECK_EQ(h.open(dir, "h.slot"), 0);
    CHECK_EQ(w0.open(dir, "w0.slot"), 0);
    CHECK_EQ(w1.open(dir, "w1.slot"), 0);
    const uint32_t g[1] = {7000};
    for (Board* x : {&h, &w0, &w1}) x->publish(kPrioNormal, g, 1, {}, now);
    h.publish_cpu_node(0);
    w0.publish_cpu_node(0);
    w1.publish_cpu_node(1);
    h.publish_gate(0, true, 0);
    w0.publish_gate(0, false, now - 2000);
    w1.publish_gate(0, false, now - 1000);
    w1.refresh(now);
    w0.refresh(now);
    h.refresh(now);
    CHECK(w1.admit(7000, 2, now - 1000, 1));   // node 1 is free: the earlier node-0 waiter is not ahead
    CHECK(!w0.admit(7000, 2, now - 2000, 0));  // node 0 holds its one place
    CHECK(h.waiting(7000, 2, 0));              // the holder's turn stands in w0's way
    CHECK(!w1.waiting(7000, 2, 1));            // nobody of node 1 waits behind w1
    // Two holders of node 0 (admitted before the nodes were known) and a node-1 waiter: all
    // places are taken and node 0 is over its share, so its holders yield after their turn.
    {
      Board h2;
      CHECK_EQ(h2.open(dir, "h2.slot"), 0);
      h2.publish(kPrioNormal, g, 1, {}, now);
      h2.publish_cpu_node(0);
      h2.publish_gate(0, true, 0);
      w0.publish_gate(0, false, 0);  // w0 not waiting now
      h.refresh(now);
      CHECK(h.waiting(7000, 2, 0));   // over node 0's share, and w1 (node 1, room) is blocked by the total
      w1.publish_gate(0, false, 0);   // nobody waits: nobody yields
      h.refresh(now);
      CHECK(!h.waiting(7000, 2, 0));
      h2.leave();
      w0.publish_gate(0, false, now - 2000);
      w1.publish_gate(0, false, now - 1000);
      w0.refresh(now);
      w1.refresh(now);
      h.refresh(now);
    }
    // Launch rates and steadiness (auto pair turns): a bursty peer busy on the GPU is seen.
    w1.publish_launch_rate(2500);
    w1.publish_steady(false);
    h.refresh(now);
    CHECK_EQ(h.peers_launch_rate(7000), 2500u);
    CHECK(h.bursty_peer_on(7000, 500));
    CHECK(!h.bursty_peer_on(7000, 5000));   // below the rate that counts as busy
    w1.publish_steady(true);
    h.refresh(now);
    CHECK(!h.bursty_peer_on(7000, 500));
    // Without nodes (a container that does not publish one): plain first-come admission.
    CHECK(!w1.admit(7000, 2, now - 1000, -1));  // w0 came first and one place is left
    CHECK(w0.admit(7000, 2, now - 2000, -1));
    // Every container on one node: the cap is k, as without nodes.
    w1.publish_cpu_node(0);
    w0.refresh(now);
    CHECK(w0.admit(7000, 2, now - 2000, 0));
    for (Board* x : {&h, &w0, &w1}) x->leave();
  }
  // A heartbeat written after the reader took its clock is fresh, not "stale by 2^64 ns":
  // peers used to drop out of refresh() at random this way.
  CHECK_EQ(a.refresh(now - 1000).size(), 1u);
  // A stale heartbeat (the container is gone) or a departed slot is ignored.
  CHECK_EQ(a.refresh(now + kBoardStaleNs + 1).size(), 0u);
  b.leave();
  CHECK_EQ(a.refresh(now).size(), 0u);
  // Garbage in a slot file (a tenant writing nonsense into its own slot) is ignored.
  FILE* f = fopen((std::string(dir) + "/junk.slot").c_str(), "w");
  CHECK(f != nullptr);
  fputs("not a slot", f);
  fclose(f);
  CHECK_EQ(a.refresh(now).size(), 0u);
  CHECK(system((std::string("rm -rf ") + dir).c_str()) == 0);
}

static void test_ledger_fresh() {
  char dir[] = "/tmp/vgpu_ledger_XXXXXX";
  CHECK(mkdtemp(dir) != nullptr);
  const uint32_t gid = 4242;
  LedgerFile* lf = new LedgerFile();
  memset(static_cast<void*>(lf), 0, sizeof(LedgerFile));
  lf->magic = kLedgerMagic;
  lf->version = kLedgerVersion;
  lf->gpu_id = gid;
  const uint64_t now = now_ns();
  lf->heartbeat_ns.store(now);
  lf->period_ns.store(1'000'000);
  std::string path = ledger_path(dir, gid);
  FILE* f = fopen(path.c_str(), "w");
  CHECK(f != nullptr);
  CHECK_EQ(fwrite(lf, sizeof(LedgerFile), 1, f), 1u);
  fclose(f);
  LedgerReader r;
  CHECK(r.open(dir, gid));
  CHECK(r.fresh(now + 10'000'000));
  CHECK(r.fresh(now - 1000));                      // written after the reader took its clock
  CHECK(!r.fresh(now + kLedgerStaleNs + 1));       // short period: the fixed floor applies
  // A daemon whose period stretched (every GPU of a busy node read in turn): stale only after
  // a few of its own periods, not after the fixed 50 ms.
  int fd = open(path.c_str(), O_WRONLY);
  CHECK(fd >= 0);
  const uint64_t period = 40'000'000;
  CHECK_EQ(pwrite(fd, &period, sizeof(period), offsetof(LedgerFile, period_ns)), (ssize_t)sizeof(period));
  close(fd);
  CHECK(r.fresh(now + 100'000'000));
  CHECK(!r.fresh(now + kLedgerStalePeriods * period + 1));
  delete lf;
  CHECK(system((std::string("rm -rf ") + dir).c_str()) == 0);
}

static void test_kfd() {
  char dir[] = "/tmp/vgpu_kfd_XXXXXX";
  CHECK(mkdtemp(dir) != nullptr);
  std::string root = dir;
  auto mk = [&](const std::string& s) { CHECK(system(("mkdir -p " + root + "/" + s).c_str()) == 0); };
  mk("100/stats_7");
  mk("200");
  FILE* f = fopen((root + "/100/stats_7/cu_occupancy").c_str(), "w");
  fprintf(f, "64\n");
  fclose(f);
  f = fopen((root + "/100/vram_7").c_str(), "w");
  fprintf(f, "4096\n");
  fclose(f);
  static std::string kfd_root;  // outlives the test: g_kfd_proc_root keeps a pointer
  kfd_root = root;
  g_kfd_proc_root = kfd_root.c_str();
  std::vector<int> before = kfd_list_pids();
  CHECK_EQ(before.size(), 2u);
  mk("300");
  std::vector<int> after = kfd_list_pids();
  CHECK_EQ(kfd_diff_pid(before, after), 300);
  mk("400");
  CHECK_EQ(kfd_diff_pid(before, kfd_list_pids()), 0);  // ambiguous → unknown
  CHECK_EQ(kfd_cu_occupancy(100, 7), 64);
  CHECK_EQ(kfd_vram_usage(100, 7), 4096);
  CHECK_EQ(kfd_cu_occupancy(100, 8), -1);
  CHECK(system(("rm -rf " + root).c_str()) == 0);
  g_kfd_proc_root = "/sys/class/kfd/kfd/proc";
}

int main(int argc, char** argv) {
  std::vector<std::pair<const char*, std::function<void()>>> tests = {
      {"parse_size", test_parse_size},
      {"parse_range", test_parse_range},
      {"config", test_config},
      {"legacy_env_names", test_legacy_env_names},
      {"spill_config", test_spill_config},
      {"override_file", test_override_file},
      {"region_basic", test_region_basic},
      {"region_kinds", test_region_unlimited_and_kinds},
      {"region_threads", test_region_threads_never_overshoot},
      {"region_multiprocess", test_region_multiprocess_and_reclaim},
      {"region_robust_lock", test_region_robust_lock},
      {"region_version_guard", test_region_version_guard},
      {"region_corruption", test_region_corruption},
      {"proc_alive", test_proc_alive},
      {"cumask", test_cumask},
      {"cumask_se_layout", test_cumask_se_layout},
      {"devmap", test_devmap},
      {"ratelimit", test_ratelimit},
      {"region_stopped_lock_owner", test_region_stopped_lock_owner},
      {"region_reclaim_namespaces", test_region_reclaim_namespaces},
      {"auto_mode_live_cu", test_auto_mode_and_live_cu},
      {"charge_overflow", test_charge_overflow},
      {"kfd", test_kfd},
      {"hostpid_resolution", test_hostpid_resolution},
      {"board", test_board},
      {"ledger_fresh", test_ledger_fresh},
  };
  if (argc > 1 && !strcmp(argv[1], "--list")) {
    for (auto& t : tests) printf("%s\n", t.first);
    return 0;
  }
  int ran = 0;
  for (auto& t : tests) {
    if (argc > 1 && strcmp(argv[1], t.first)) continue;
    int before = g_failures;
    t.second();
    printf("%s %s\n", g_failures == before ? "PASS" : "FAIL", t.first);
    ran++;
  }
  if (!ran) {
    fprintf(stderr, "no such test\n");
    return 2;
  }
  return g_failures ? 1 : 0;
}
