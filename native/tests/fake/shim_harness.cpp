// Driver for CPU-only shim tests: a "HIP application" linked against the fake HIP/ROCr
// (fake_hip.cpp, fake_hsa.cpp) and run with libvgpu_hip.so preloaded, exactly like a
// PyTorch process under the vGPU contract. It executes a small script given on the
// command line and prints one JSON object per step (tests/test_shim_fake.py):
//
//   dev=N            hipSetDevice(N)
//   malloc=SIZE      hipMalloc (K/M/G suffixes) -> {"malloc": "ok"|"oom"}
//   free             hipFree of the most recent successful allocation
//   meminfo          hipMemGetInfo -> {"free": .., "total": ..}
//   count            hipGetDeviceCount and hipGetDevice -> {"count": n, "current": d}
//   props=D          hipGetDeviceProperties / hipDeviceTotalMem / the TotalGlobalMem attribute of device D
//                    -> {"total": .., "totalmem": .., "attrmem": ..}
//   canpeer=A,B      hipDeviceCanAccessPeer(A, B), then hipDeviceEnablePeerAccess(B) from the current device
//   stream           hipStreamCreate on the current device (becomes the current stream)
//   usestream=I      the I-th stream created so far becomes the current stream (the current
//                    device stays: a stream of another device used from this thread)
//   launch=US,N      N launches of a US-microsecond kernel, then synchronize
//   run=US,SECS      back-to-back US-microsecond kernels for SECS seconds (sync every 8):
//                    {"busy_frac": GPU time executed / wall, ...}
//   graph=US,SECS    like run, with hipGraphLaunch of a US-microsecond "graph"
//   internal=SIZE    runtime-internal device memory (bypasses every hook; negative frees)
//   queues           CU-mask bit count, mask changes and priority of every created stream
//   cus              the current device's CU count as the runtime sees it
//   curlimit         the shim's vgpu_get_current_device_memory_limit (the current HIP
//                    device mapped to its agent): {"dev": N, "limit": bytes}
//   burst=US,N       N launches of a US-microsecond kernel on the current stream without
//                    waiting, then synchronize: {"burst": N, "max_depth": most packets seen
//                    queued on the stream's HSA queue right after a launch, "wall": s}
//   setlimit=SIZE / setcu=PCT  the in-container setters -> {"setlimit": rc} / {"setcu": rc}
//   mark=TEXT        prints {"mark": TEXT} (a point the test waits for before acting)
//   sleep=SECS
//   forkmalloc=SIZE  fork; the child hipMallocs SIZE and exits normally:
//                    {"child_malloc": "ok"|"oom"|"crash"}
//   forkstorm=N      while a second thread allocates and frees 1 MiB in a loop, fork N
//                    CPU-only children that exit normally: {"forkstorm": ok_children}
//   gates=MODE       for every name in $FAKE_GATE_NAMES (comma-separated): resolve it as
//                    an application would - MODE direct (the global scope, i.e. a linked
//                    call), dlsym (dlsym on a libamdhip64 handle), procaddr (dlsym of
//                    hipGetProcAddress on that handle, then hipGetProcAddress: Triton's
//                    way) - and call it while the container is suspended (resumed after
//                    40 ms by a second thread): {"unrouted": names whose pointer is not the
//                    shim's, "ungated": names that did not block, "unreached": names whose
//                    call never reached the runtime}
//   hostmalloc=SIZE  hipHostMalloc -> {"hostmalloc": "ok"|"oom"}; hostfree frees the last one
//                    (hostfree_hipfree: through hipFree, which releases pinned memory too)
//   freeidx=I        hipFree of the I-th successful allocation (of all made so far)
//   fill=B / check=B the CPU writes byte B into / checks byte B in every byte of the most
//                    recent allocation (spilled SVM memory only: the fake's HBM is not
//                    mapped) -> {"check": "ok"|"bad"}
//   where            where the most recent allocation lives: {"where": gpu ordinal, -1 = host
//                    memory (an SVM range), -2 = not an SVM range}
//   spilled          the shim's vgpu_get_current_device_spilled: {"spilled": bytes}
//   peer=D           hsa_amd_agents_allow_access for GPU D on the most recent allocation (what
//                    HIP does for peer devices): {"peer": status, "svm_access": whether the
//                    fake's SVM range now lists that agent}
//   hostregister=SIZE  hipHostRegister of a fresh heap buffer -> {"hostregister": "ok"|"oom"};
//                    hostunregister unregisters (and frees) the last one
//   hsahost=SIZE     hsa_amd_memory_pool_allocate on the CPU pool, as a direct ROCr caller
//                    (ctypes) would: {"hsahost": status}; hsahostfree frees the last one
//   hsalock=SIZE     hsa_amd_memory_lock of a fresh heap buffer: {"hsalock": status};
//                    hsaunlock unlocks (and frees) the last one; relock=SIZE locks the last
//                    locked buffer again with its own size
//   hostusage        the container's pinned host memory: {"hostusage": bytes}
//   hsamemfree       hsa_memory_free of the most recent allocation: {"hsamemfree": status}
//   waitsig=MS       a blocking hsa_signal_wait_scacquire on a signal another thread completes
//                    after MS ms: {"waitsig": wall ms, "cpu_ms": the waiting thread's CPU ms};
//                    waitspin=MS the same as an active (spin) wait with no time-out
//   usage            the current device's charged bytes: {"usage": bytes}
//   svmmap=SIZE      mmap SIZE bytes of ordinary memory and give the current device access
//                    (SVM attributes, no placement): {"svmmap": status}
//   svmprefetch=D    hsa_amd_svm_prefetch_async of the last range to GPU D (-1 = the CPU):
//                    {"svmprefetch": status}
//   svmpref=D        HSA_AMD_SVM_ATTRIB_PREFERRED_LOCATION of the last range: {"svmpref": status}
//   hipprefetch=D / hipadvise=D  hipMemPrefetchAsync / hipMemAdvise(SetPreferredLocation) of
//                    the last range: {"hipprefetch": rc} / {"hipadvise": rc}
//   svmunmap         munmap of the last range: {"svmunmap": true}
//   ipcexport        hipIpcGetMemHandle of the most recent allocation: {"ipcexport": rc}
//   affinity         the CPUs this process may run on: {"affinity": [cpu, ...]}
#define __HIP_PLATFORM_AMD__ 1
#include <dlfcn.h>
#include <sched.h>
#include <hip/hip_runtime_api.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <sys/mman.h>
#include <time.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

extern "C" {
uint64_t fake_hip_busy_us(int dev, uint64_t* kernels);
hsa_queue_t* fake_hip_stream_queue(hipStream_t stream);
int fake_rocr_queue_state(const hsa_queue_t* queue, uint32_t* mask_words8, int* priority, int* device);
int fake_rocr_internal_alloc(int dev, int64_t bytes);
int fake_rocr_host_pid();
int fake_hip_device_cus(int dev);
const char* fake_hip_last_call();
int fake_rocr_svm_location(const void* ptr);
int fake_rocr_svm_has_access(const void* ptr, uint64_t agent);
void fake_rocr_svm_gc();
}

namespace {

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

long long parse_size(const char* s) {
  char* end = nullptr;
  long long v = strtoll(s, &end, 10);
  switch (end && *end ? *end : 0) {
    case 'k': case 'K': v <<= 10; break;
    case 'm': case 'M': v <<= 20; break;
    case 'g': case 'G': v <<= 30; break;
    default: break;
  }
  return v;
}

std::vector<std::string> split_names(const char* s) {
  std::vector<std::string> out;
  std::string cur;
  for (const char* p = s ? s : ""; ; p++) {
    if (*p == ',' || *p == 0) {
      if (!cur.empty()) out.push_back(cur);
      cur.clear();
      if (!*p) break;
    } else {
      cur += *p;
    }
  }
  return out;
}

void json_list(const char* key, const std::vector<std::string>& v, bool last) {
  printf("\"%s\": [", key);
  for (size_t i = 0; i < v.size(); i++) printf("%s\"%s\"", i ? ", " : "", v[i].c_str());
  printf("]%s", last ? "" : ", ");
}

void gates(const std::string& mode) {
  using Ctl = int (*)();
  using ProcAddr = hipError_t (*)(const char*, void**, int, uint64_t, hipDriverProcAddressQueryResult*);
  auto suspend = reinterpret_cast<Ctl>(dlsym(RTLD_DEFAULT, "vgpu_suspend_all"));
  auto resume = reinterpret_cast<Ctl>(dlsym(RTLD_DEFAULT, "vgpu_resume_all"));
  void* h = dlopen("libamdhip64.so", RTLD_NOLOAD | RTLD_LAZY);
  ProcAddr gpa = h ? reinterpret_cast<ProcAddr>(dlsym(h, "hipGetProcAddress")) : nullptr;
  std::vector<std::string> names = split_names(getenv("FAKE_GATE_NAMES")), unrouted, ungated, unreached;
  for (const std::string& n : names) {
    void* shim_fn = dlsym(RTLD_DEFAULT, n.c_str());
    void* p = nullptr;
    if (mode == "direct") p = shim_fn;
    else if (mode == "dlsym") p = h ? dlsym(h, n.c_str()) : nullptr;
    else if (gpa) (void)gpa(n.c_str(), &p, 0, 0, nullptr);
    if (!p || p != shim_fn) {
      unrouted.push_back(n);
      if (!p) continue;
    }
    if (!suspend || !resume || suspend() != 0) {
      ungated.push_back(n);
      continue;
    }
    std::thread t([&] {
      std::this_thread::sleep_for(std::chrono::milliseconds(40));
      resume();
    });
    double t0 = now_s();
    (void)reinterpret_cast<int (*)()>(p)();
    double dt = now_s() - t0;
    t.join();
    if (dt < 0.030) ungated.push_back(n);
    if (n != fake_hip_last_call()) unreached.push_back(n);
  }
  printf("{\"gates\": \"%s\", \"n\": %zu, ", mode.c_str(), names.size());
  json_list("unrouted", unrouted, false);
  json_list("ungated", ungated, false);
  json_list("unreached", unreached, true);
  printf("}\n");
}

}  // namespace

int main(int argc, char** argv) {
  // HARNESS_LAZY_INIT=1: no hipInit and no agent scan up front, so the first command is the
  // program's first HIP call (e.g. hipSetDevice(1) before anything else)
  const bool lazy = getenv("HARNESS_LAZY_INIT") != nullptr;
  if (!lazy && hipInit(0) != hipSuccess) return 1;
  int dev = 0;
  hipStream_t stream = nullptr;
  std::vector<void*> ptrs, all_ptrs;
  std::vector<size_t> sizes;
  std::vector<hipStream_t> streams;
  std::vector<void*> host_ptrs, registered, hsa_host, hsa_locked;
  std::vector<std::pair<void*, size_t>> svm_ranges;
  hsa_agent_t cpu_agent{0};
  std::vector<hsa_agent_t> gpu_agents;
  hsa_amd_memory_pool_t cpu_pool{0};
  if (!lazy)
  (void)hsa_iterate_agents(
      [](hsa_agent_t a, void* d) {
        hsa_device_type_t t;
        hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
        auto* v = static_cast<std::pair<hsa_agent_t*, std::vector<hsa_agent_t>*>*>(d);
        if (t == HSA_DEVICE_TYPE_CPU && !v->first->handle) *v->first = a;
        if (t == HSA_DEVICE_TYPE_GPU) v->second->push_back(a);
        return HSA_STATUS_SUCCESS;
      },
      new std::pair<hsa_agent_t*, std::vector<hsa_agent_t>*>(&cpu_agent, &gpu_agents));
  if (cpu_agent.handle)
    (void)hsa_amd_agent_iterate_memory_pools(
        cpu_agent,
        [](hsa_amd_memory_pool_t p, void* d) {
          *static_cast<hsa_amd_memory_pool_t*>(d) = p;
          return HSA_STATUS_SUCCESS;
        },
        &cpu_pool);
  auto agent_for = [&](int d) { return d >= 0 && d < (int)gpu_agents.size() ? gpu_agents[d] : cpu_agent; };
  auto api_u64 = [](const char* name) {
    using Get = uint64_t (*)();
    auto f = reinterpret_cast<Get>(dlsym(RTLD_DEFAULT, name));
    return f ? (unsigned long long)f() : 0ull;
  };
  static uint32_t kernel_us[64];
  int kslot = 0;
  printf("{\"pid\": %d, \"fake_hostpid\": %d}\n", (int)getpid(), fake_rocr_host_pid());
  for (int i = 1; i < argc; i++) {
    std::string op(argv[i]);
    std::string key = op.substr(0, op.find('='));
    std::string val = op.find('=') == std::string::npos ? "" : op.substr(op.find('=') + 1);
    if (key == "dev") {
      dev = atoi(val.c_str());
      printf("{\"dev\": %d, \"rc\": %d}\n", dev, (int)hipSetDevice(dev));
      stream = nullptr;
    } else if (key == "malloc") {
      void* p = nullptr;
      hipError_t e = hipMalloc(&p, (size_t)parse_size(val.c_str()));
      if (e == hipSuccess) {
        ptrs.push_back(p);
        all_ptrs.push_back(p);
        sizes.push_back((size_t)parse_size(val.c_str()));
      }
      printf("{\"malloc\": \"%s\", \"bytes\": %lld}\n", e == hipSuccess ? "ok" : "oom", parse_size(val.c_str()));
    } else if (key == "free") {
      if (!ptrs.empty()) {
        (void)hipFree(ptrs.back());
        std::replace(all_ptrs.begin(), all_ptrs.end(), ptrs.back(), static_cast<void*>(nullptr));
        ptrs.pop_back();
      }
      printf("{\"free\": true}\n");
    } else if (key == "freeidx") {
      const size_t i = (size_t)atoi(val.c_str());
      if (i < all_ptrs.size() && all_ptrs[i]) {
        (void)hipFree(all_ptrs[i]);
        for (size_t j = 0; j < ptrs.size(); j++)
          if (ptrs[j] == all_ptrs[i]) ptrs.erase(ptrs.begin() + (long)j);
        all_ptrs[i] = nullptr;
      }
      printf("{\"freeidx\": %zu}\n", i);
    } else if (key == "fill" || key == "check") {
      const int b = atoi(val.c_str());
      size_t bad = 0;
      if (!ptrs.empty()) {
        unsigned char* p = static_cast<unsigned char*>(ptrs.back());
        const size_t n = sizes[std::find(all_ptrs.begin(), all_ptrs.end(), ptrs.back()) - all_ptrs.begin()];
        if (key == "fill") memset(p, b, n);
        else
          for (size_t j = 0; j < n; j++) bad += p[j] != (unsigned char)b;
      }
      if (key == "fill") printf("{\"fill\": %d}\n", b);
      else printf("{\"check\": \"%s\", \"bad\": %zu}\n", bad || ptrs.empty() ? "bad" : "ok", bad);
    } else if (key == "where") {
      printf("{\"where\": %d}\n", ptrs.empty() ? -2 : fake_rocr_svm_location(ptrs.back()));
    } else if (key == "peer") {
      const uint64_t agent = (uint64_t)atoi(val.c_str()) + 1;  // the fake's GPU agent handles are 1..n
      hsa_agent_t a{agent};
      int st = ptrs.empty() ? -1 : (int)hsa_amd_agents_allow_access(1, &a, nullptr, ptrs.back());
      printf("{\"peer\": %d, \"svm_access\": %d}\n", st, ptrs.empty() ? 0 : fake_rocr_svm_has_access(ptrs.back(), agent));
    } else if (key == "spilled") {
      using Get = uint64_t (*)();
      auto f = reinterpret_cast<Get>(dlsym(RTLD_DEFAULT, "vgpu_get_current_device_spilled"));
      printf("{\"spilled\": %llu}\n", f ? (unsigned long long)f() : 0ull);
    } else if (key == "affinity") {
      cpu_set_t set;
      CPU_ZERO(&set);
      sched_getaffinity(0, sizeof(set), &set);
      printf("{\"affinity\": [");
      bool first = true;
      for (int c = 0; c < CPU_SETSIZE; c++)
        if (CPU_ISSET(c, &set)) {
          printf("%s%d", first ? "" : ", ", c);
          first = false;
        }
      printf("]}\n");
    } else if (key == "count") {
      int n = -1;
      hipError_t e = hipGetDeviceCount(&n);
      int cur = -1;
      (void)hipGetDevice(&cur);
      printf("{\"count\": %d, \"rc\": %d, \"current\": %d}\n", n, (int)e, cur);
    } else if (key == "props") {
      hipDeviceProp_t p;
      const int d = atoi(val.c_str());
      hipError_t e = hipGetDeviceProperties(&p, d);
      size_t tm = 0;
      hipError_t e2 = hipDeviceTotalMem(&tm, d);
      int am = -1;
      hipError_t e3 = hipDeviceGetAttribute(&am, hipDeviceAttributeTotalGlobalMem, d);
      printf("{\"props\": %d, \"rc\": %d, \"total\": %zu, \"totalmem\": %zu, \"rc2\": %d, \"attrmem\": %d, "
             "\"rc3\": %d}\n", d, (int)e, e == hipSuccess ? (size_t)p.totalGlobalMem : 0, tm, (int)e2, am, (int)e3);
    } else if (key == "canpeer") {
      const int a = atoi(val.c_str()), b = atoi(val.substr(val.find(',') + 1).c_str());
      int can = -1;
      hipError_t e = hipDeviceCanAccessPeer(&can, a, b);
      hipError_t e2 = hipDeviceEnablePeerAccess(b, 0);
      printf("{\"canpeer\": %d, \"rc\": %d, \"enable\": %d}\n", can, (int)e, (int)e2);
    } else if (key == "meminfo") {
      size_t f = 0, t = 0;
      (void)hipMemGetInfo(&f, &t);
      printf("{\"dev\": %d, \"free\": %zu, \"total\": %zu}\n", dev, f, t);
    } else if (key == "stream") {
      (void)hipStreamCreate(&stream);
      streams.push_back(stream);
      printf("{\"stream\": %zu}\n", streams.size() - 1);
    } else if (key == "usestream") {
      // a stream created earlier (on whichever device), without changing the current device
      const size_t i = (size_t)atoi(val.c_str());
      stream = i < streams.size() ? streams[i] : nullptr;
      printf("{\"usestream\": %zu}\n", i);
    } else if (key == "launch" || key == "graph" || key == "run") {
      unsigned us = (unsigned)atoi(val.c_str());
      double amount = atof(val.substr(val.find(',') + 1).c_str());
      uint32_t* k = &kernel_us[kslot++ % 64];
      *k = us;
      int sdev = dev;  // the device the stream's kernels run on
      if (stream) (void)hipStreamGetDevice(stream, &sdev);
      uint64_t k0 = 0, b0 = fake_hip_busy_us(sdev, &k0);
      double t0 = now_s();
      long n = 0;
      for (;; n++) {
        const bool timed = key != "launch";
        if (timed ? now_s() - t0 >= amount : n >= (long)amount) break;
        if (key == "graph") (void)hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(k), stream);
        else (void)hipLaunchKernel(k, dim3(1), dim3(64), nullptr, 0, stream);
        if (timed && n % 8 == 7) (void)hipStreamSynchronize(stream);
      }
      (void)hipStreamSynchronize(stream);
      double wall = now_s() - t0;
      uint64_t k1 = 0, b1 = fake_hip_busy_us(sdev, &k1);
      printf("{\"%s\": %ld, \"wall\": %.6f, \"busy_us\": %llu, \"busy_frac\": %.4f}\n", key.c_str(), n, wall,
             (unsigned long long)(b1 - b0), (b1 - b0) / 1e6 / wall);
    } else if (key == "burst") {
      unsigned us = (unsigned)atoi(val.c_str());
      long n = atol(val.substr(val.find(',') + 1).c_str());
      uint32_t* k = &kernel_us[kslot++ % 64];
      *k = us;
      hsa_queue_t* q = stream ? fake_hip_stream_queue(stream) : nullptr;
      uint64_t max_depth = 0;
      double t0 = now_s();
      for (long i = 0; i < n; i++) {
        (void)hipLaunchKernel(k, dim3(1), dim3(64), nullptr, 0, stream);
        if (q) {
          uint64_t d = hsa_queue_load_write_index_relaxed(q) - hsa_queue_load_read_index_relaxed(q);
          if (d > max_depth) max_depth = d;
        }
      }
      (void)hipStreamSynchronize(stream);
      printf("{\"burst\": %ld, \"max_depth\": %llu, \"wall\": %.6f}\n", n, (unsigned long long)max_depth,
             now_s() - t0);
    } else if (key == "internal") {
      fake_rocr_internal_alloc(dev, parse_size(val.c_str()));
      printf("{\"internal\": %lld}\n", parse_size(val.c_str()));
    } else if (key == "queues") {
      printf("{\"queues\": [");
      for (size_t q = 0; q < streams.size(); q++) {
        uint32_t m[8];
        int prio = 0, d = 0;
        int sets = fake_rocr_queue_state(fake_hip_stream_queue(streams[q]), m, &prio, &d);
        int bits = 0;
        for (uint32_t w : m) bits += __builtin_popcount(w);
        printf("%s{\"dev\": %d, \"cus\": %d, \"sets\": %d, \"priority\": %d, \"mask0\": %u}", q ? ", " : "", d, bits,
               sets, prio, m[0]);
      }
      printf("]}\n");
    } else if (key == "cus") {
      printf("{\"dev\": %d, \"cus\": %d}\n", dev, fake_hip_device_cus(dev));
    } else if (key == "forkmalloc") {
      fflush(stdout);
      pid_t c = fork();
      if (c == 0) {
        void* p = nullptr;
        hipError_t e = hipMalloc(&p, (size_t)parse_size(val.c_str()));
        exit(e == hipSuccess ? 0 : 3);  // normal exit: the shim's exit handler releases the slot
      }
      int st = 0;
      waitpid(c, &st, 0);
      const char* r = WIFEXITED(st) ? (WEXITSTATUS(st) == 0 ? "ok" : "oom") : "crash";
      printf("{\"child_malloc\": \"%s\"}\n", r);
    } else if (key == "forkstorm") {
      std::atomic<bool> stop{false};
      std::thread churn([&] {
        while (!stop.load()) {
          void* p = nullptr;
          if (hipMalloc(&p, 1 << 20) == hipSuccess) (void)hipFree(p);
        }
      });
      int ok = 0, n = atoi(val.c_str());
      fflush(stdout);
      for (int k = 0; k < n; k++) {
        pid_t c = fork();
        if (c == 0) exit(0);  // CPU-only child, like a DataLoader worker (HIP is not fork-safe)
        int st = 0;
        waitpid(c, &st, 0);
        ok += WIFEXITED(st) && WEXITSTATUS(st) == 0;
      }
      stop = true;
      churn.join();
      printf("{\"forkstorm\": %d}\n", ok);
    } else if (key == "curlimit") {
      using Lim = uint64_t (*)();
      auto f = reinterpret_cast<Lim>(dlsym(RTLD_DEFAULT, "vgpu_get_current_device_memory_limit"));
      printf("{\"dev\": %d, \"limit\": %llu}\n", dev, f ? (unsigned long long)f() : 0ull);
    } else if (key == "gates") {
      gates(val);
    } else if (key == "hostmalloc") {
      void* p = nullptr;
      hipError_t e = hipHostMalloc(&p, (size_t)parse_size(val.c_str()), 0);
      if (e == hipSuccess) host_ptrs.push_back(p);
      printf("{\"hostmalloc\": \"%s\"}\n", e == hipSuccess ? "ok" : "oom");
    } else if (key == "hostfree") {
      if (!host_ptrs.empty()) {
        (void)hipHostFree(host_ptrs.back());
        host_ptrs.pop_back();
      }
      printf("{\"hostfree\": true}\n");
    } else if (key == "hostfree_hipfree") {
      if (!host_ptrs.empty()) {
        (void)hipFree(host_ptrs.back());
        host_ptrs.pop_back();
      }
      printf("{\"hostfree\": true}\n");
    } else if (key == "hostregister") {
      size_t n = (size_t)parse_size(val.c_str());
      void* p = malloc(n ? n : 1);
      hipError_t e = hipHostRegister(p, n, 0);
      if (e == hipSuccess) registered.push_back(p);
      else free(p);
      printf("{\"hostregister\": \"%s\"}\n", e == hipSuccess ? "ok" : "oom");
    } else if (key == "hostunregister") {
      if (!registered.empty()) {
        (void)hipHostUnregister(registered.back());
        free(registered.back());
        registered.pop_back();
      }
      printf("{\"hostunregister\": true}\n");
    } else if (key == "waitsig" || key == "waitspin") {
      // A blocking ROCr wait on a signal another thread completes after MS milliseconds (a
      // kernel finishing): {"waitsig": wall ms, "cpu_ms": this thread's CPU time in the wait}
      const int ms = atoi(val.c_str());
      hsa_signal_t sig;
      hsa_signal_create(1, 0, nullptr, &sig);
      std::thread done([&] {
        std::this_thread::sleep_for(std::chrono::milliseconds(ms));
        hsa_signal_store_relaxed(sig, 0);
      });
      struct timespec c0, c1;
      clock_gettime(CLOCK_THREAD_CPUTIME_ID, &c0);
      const double t0 = now_s();
      hsa_signal_value_t v = hsa_signal_wait_scacquire(
          sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, key == "waitsig" ? HSA_WAIT_STATE_BLOCKED : HSA_WAIT_STATE_ACTIVE);
      const double wall = now_s() - t0;
      clock_gettime(CLOCK_THREAD_CPUTIME_ID, &c1);
      done.join();
      hsa_signal_destroy(sig);
      printf("{\"%s\": %.3f, \"cpu_ms\": %.3f, \"value\": %ld}\n", key.c_str(), wall * 1e3,
             (c1.tv_sec - c0.tv_sec) * 1e3 + (c1.tv_nsec - c0.tv_nsec) / 1e6, (long)v);
    } else if (key == "hsamemfree") {
      // the most recent device allocation, freed through ROCr's legacy entry point
      int st = -1;
      if (!ptrs.empty()) {
        st = (int)hsa_memory_free(ptrs.back());
        std::replace(all_ptrs.begin(), all_ptrs.end(), ptrs.back(), static_cast<void*>(nullptr));
        ptrs.pop_back();
      }
      printf("{\"hsamemfree\": %d}\n", st);
    } else if (key == "hsahost") {
      void* p = nullptr;
      int st = (int)hsa_amd_memory_pool_allocate(cpu_pool, (size_t)parse_size(val.c_str()), 0, &p);
      if (st == 0) hsa_host.push_back(p);
      printf("{\"hsahost\": %d}\n", st);
    } else if (key == "hsahostfree") {
      int st = -1;
      if (!hsa_host.empty()) {
        st = (int)hsa_amd_memory_pool_free(hsa_host.back());
        hsa_host.pop_back();
      }
      printf("{\"hsahostfree\": %d}\n", st);
    } else if (key == "hsalock") {
      size_t n = (size_t)parse_size(val.c_str());
      void* p = malloc(n ? n : 1);
      void* agent_ptr = nullptr;
      int st = (int)hsa_amd_memory_lock(p, n, nullptr, 0, &agent_ptr);
      if (st == 0) hsa_locked.push_back(p);
      else free(p);
      printf("{\"hsalock\": %d}\n", st);
    } else if (key == "relock") {
      // the last locked buffer locked once more, with a size of its own
      int st = -1;
      void* agent_ptr = nullptr;
      if (!hsa_locked.empty()) {
        st = (int)hsa_amd_memory_lock(hsa_locked.back(), (size_t)parse_size(val.c_str()), nullptr, 0, &agent_ptr);
        if (st == 0) hsa_locked.push_back(hsa_locked.back());
      }
      printf("{\"relock\": %d}\n", st);
    } else if (key == "hsaunlock") {
      int st = -1;
      if (!hsa_locked.empty()) {
        void* p = hsa_locked.back();
        st = (int)hsa_amd_memory_unlock(p);
        hsa_locked.pop_back();
        if (std::find(hsa_locked.begin(), hsa_locked.end(), p) == hsa_locked.end()) free(p);  // its last lock
      }
      printf("{\"hsaunlock\": %d}\n", st);
    } else if (key == "hostusage") {
      printf("{\"hostusage\": %llu}\n", api_u64("vgpu_get_host_memory_usage"));
    } else if (key == "usage") {
      printf("{\"usage\": %llu}\n", api_u64("vgpu_get_current_device_memory_usage"));
    } else if (key == "ipcexport") {
      hipIpcMemHandle_t h;
      int rc = ptrs.empty() ? -1 : (int)hipIpcGetMemHandle(&h, ptrs.back());
      printf("{\"ipcexport\": %d}\n", rc);
    } else if (key == "svmmap") {
      size_t n = (size_t)parse_size(val.c_str());
      void* p = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
      hsa_amd_svm_attribute_pair_t a{HSA_AMD_SVM_ATTRIB_AGENT_ACCESSIBLE_IN_PLACE, agent_for(dev).handle};
      int st = p == MAP_FAILED ? -1 : (int)hsa_amd_svm_attributes_set(p, n, &a, 1);
      if (p != MAP_FAILED) svm_ranges.emplace_back(p, n);
      printf("{\"svmmap\": %d}\n", st);
    } else if (key == "svmprefetch" || key == "svmpref") {
      int st = -1;
      if (!svm_ranges.empty()) {
        const hsa_agent_t a = agent_for(atoi(val.c_str()));
        if (key == "svmpref") {
          hsa_amd_svm_attribute_pair_t at{HSA_AMD_SVM_ATTRIB_PREFERRED_LOCATION, a.handle};
          st = (int)hsa_amd_svm_attributes_set(svm_ranges.back().first, svm_ranges.back().second, &at, 1);
        } else {
          hsa_signal_t sig;
          hsa_signal_create(1, 0, nullptr, &sig);
          st = (int)hsa_amd_svm_prefetch_async(svm_ranges.back().first, svm_ranges.back().second, a, 0, nullptr, sig);
          hsa_signal_destroy(sig);
        }
      }
      printf("{\"%s\": %d}\n", key.c_str(), st);
    } else if (key == "hipprefetch" || key == "hipadvise") {
      int rc = -1;
      if (!svm_ranges.empty()) {
        const int d = atoi(val.c_str());
        rc = key == "hipprefetch"
                 ? (int)hipMemPrefetchAsync(svm_ranges.back().first, svm_ranges.back().second, d, stream)
                 : (int)hipMemAdvise(svm_ranges.back().first, svm_ranges.back().second, hipMemAdviseSetPreferredLocation, d);
      }
      printf("{\"%s\": %d}\n", key.c_str(), rc);
    } else if (key == "svmunmap") {
      if (!svm_ranges.empty()) {
        munmap(svm_ranges.back().first, svm_ranges.back().second);
        fake_rocr_svm_gc();  // the driver drops the range at once (MMU notifier)
        svm_ranges.pop_back();
      }
      printf("{\"svmunmap\": true}\n");
    } else if (key == "setlimit" || key == "setcu") {
      // The in-container control API (reference set_current_device_memory_limit /
      // set_current_device_sm_limit_scale): {"setlimit": rc} / {"setcu": rc}
      int rc = -2;
      if (key == "setlimit") {
        using Set = int (*)(uint64_t);
        auto f = reinterpret_cast<Set>(dlsym(RTLD_DEFAULT, "vgpu_set_current_device_memory_limit"));
        if (f) rc = f((uint64_t)parse_size(val.c_str()));
      } else {
        using Set = int (*)(int);
        auto f = reinterpret_cast<Set>(dlsym(RTLD_DEFAULT, "vgpu_set_current_device_cu_limit"));
        if (f) rc = f(atoi(val.c_str()));
      }
      printf("{\"%s\": %d}\n", key.c_str(), rc);
    } else if (key == "mark") {
      printf("{\"mark\": \"%s\"}\n", val.c_str());
    } else if (key == "sleep") {
      std::this_thread::sleep_for(std::chrono::duration<double>(atof(val.c_str())));
      printf("{\"slept\": %s}\n", val.c_str());
    } else {
      fprintf(stderr, "unknown op %s\n", op.c_str());
      return 2;
    }
    fflush(stdout);
  }
  return 0;
}
