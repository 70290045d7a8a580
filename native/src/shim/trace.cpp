// roctx ranges around the shim's blocking waits (SURVEY.md §5 tracing plan).
//
// The reference only logs at debug level ([4pdvGPU Debug...] at every hook). Here a
// launch that the temporal limiter or the external block holds back, and any call held
// by a suspend, is bracketed by a roctx range ("vgpu:throttle", "vgpu:suspended"), so
// `rocprofv3 --marker-trace` shows the stall on the timeline next to the tenant's kernels;
// the same waits are summed per process in the region (throttle_ns / suspend_ns → the
// monitor's vgpu_process_{throttle,suspend}_seconds_total). Off unless VGPU_TRACE=1: the
// roctx library is then dlopen'ed once and only blocking waits pay for a range.
#include <dlfcn.h>

#include <atomic>
#include <cstdlib>

#include "real.h"
#include "shim.h"

namespace vgpu {

namespace {

using PushFn = int (*)(const char*);
using PopFn = int (*)();

std::atomic<int> g_state{0};  // 0 = not resolved, 1 = on, 2 = off
PushFn g_push = nullptr;
PopFn g_pop = nullptr;

bool resolve() {
  int s = g_state.load(std::memory_order_acquire);
  if (__builtin_expect(s != 0, 1)) return s == 1;
  const char* e = getenv("VGPU_TRACE");
  bool on = e && *e && *e != '0';
  if (on) {
    void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_GLOBAL | RTLD_NOLOAD);
    if (!h) h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("libroctx64.so.4", RTLD_NOW | RTLD_GLOBAL);
    if (h) {
      g_push = reinterpret_cast<PushFn>(real_dlsym(h, "roctxRangePushA"));
      g_pop = reinterpret_cast<PopFn>(real_dlsym(h, "roctxRangePop"));
    }
    on = g_push && g_pop;
  }
  g_state.store(on ? 1 : 2, std::memory_order_release);
  return on;
}

}  // namespace

void trace_push(const char* name) {
  if (resolve()) g_push(name);
}

void trace_pop() {
  if (g_state.load(std::memory_order_relaxed) == 1) g_pop();
}

}  // namespace vgpu
