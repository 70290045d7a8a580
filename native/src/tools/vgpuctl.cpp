// vgpuctl: inspect and control a container's shared region from the node.
//
// The reference exposes this control surface only as symbols of libvgpu.so
// (suspend_all, resume_all, set_current_device_sm_limit_scale, ...) for an
// out-of-tree monitor (observability). This is the in-tree tool.
//
//   vgpuctl <region> show                 JSON dump (devices + processes)
//   vgpuctl <region> suspend|resume       block / unblock every gate
//   vgpuctl <region> block|unblock        launch block (recent_kernel < 0)
//   vgpuctl <region> set-limit <dev> <size>
//   vgpuctl <region> set-cu <dev> <pct>
//   vgpuctl <region> set-host-limit <size>  pinned host memory budget (0 = unlimited)
//   vgpuctl <region> priority <n>
//   vgpuctl <region> reclaim              free slots of exited processes
//   vgpuctl ledger <board-dir>            the node GPU-time ledgers (vgpu/ledger.h), JSON
//   vgpuctl board <board-dir>             the live containers on the node board (vgpu/board.h):
//                                         class, CPU node, launch rate and steadiness, and per
//                                         GPU whether it holds a turn or waits for one, JSON
#include <dirent.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "vgpu/board.h"
#include "vgpu/ledger.h"
#include "vgpu/ratelimit.h"
#include "vgpu/region_api.h"

// Every <board>/ledger.<gpu_id>: sampling state and each process's charged GPU time.
static int show_ledgers(const char* dir) {
  DIR* d = opendir(dir);
  if (!d) {
    fprintf(stderr, "vgpuctl: cannot open %s\n", dir);
    return 1;
  }
  printf("{\"ledgers\": [");
  int n = 0;
  const uint64_t now = vgpu::now_ns();
  while (struct dirent* e = readdir(d)) {
    if (strncmp(e->d_name, "ledger.", 7) != 0) continue;
    char* end = nullptr;
    const unsigned long id = strtoul(e->d_name + 7, &end, 10);
    if (end == e->d_name + 7 || *end) continue;
    vgpu::LedgerReader l;
    if (!l.open(dir, (uint32_t)id)) continue;
    const vgpu::LedgerFile* f = l.file();
    const uint64_t hb = f->heartbeat_ns.load();
    printf("%s\n  {\"gpu_id\": %lu, \"fresh\": %s, \"age_ms\": %.1f, \"samples\": %llu, \"reads\": %llu, "
           "\"period_us\": %llu, \"total_occ\": %lld, \"procs\": [",
           n++ ? "," : "", id, l.fresh(now) ? "true" : "false", hb && now > hb ? (now - hb) / 1e6 : 0.0,
           (unsigned long long)f->samples.load(), (unsigned long long)f->reads.load(),
           (unsigned long long)f->period_ns.load() / 1000, (long long)f->total_occ.load());
    int m = 0;
    const int k = f->n.load() < vgpu::kLedgerMaxPids ? f->n.load() : vgpu::kLedgerMaxPids;
    for (int i = 0; i < k; i++) {
      const int pid = f->e[i].pid.load();
      if (pid <= 0) continue;
      printf("%s{\"hostpid\": %d, \"occ\": %d, \"charged_ms\": %.3f}", m++ ? ", " : "", pid, f->e[i].occ.load(),
             f->e[i].charged_ns.load() / 1e6);
    }
    printf("]}");
  }
  closedir(d);
  printf("]}\n");
  return 0;
}

// The live slots of <board>: what the containers of the node tell each other.
static int show_board(const char* dir) {
  vgpu::Board b;
  DIR* probe = opendir(dir);
  if (probe) closedir(probe);
  if (!probe || b.open_readonly(dir) != 0) {
    fprintf(stderr, "vgpuctl: cannot open %s\n", dir);
    return 1;
  }
  const uint64_t now = vgpu::now_ns();
  const auto& peers = b.refresh(now);
  printf("{\"containers\": [");
  int n = 0;
  for (const vgpu::BoardPeer& p : peers) {
    printf("%s\n  {\"container\": \"%s\", \"priority\": %d, \"cpu_node\": %d, \"launches_per_s\": %u, "
           "\"steady\": %s, \"hostpids\": [",
           n++ ? "," : "", p.name.c_str(), p.priority, p.cpu_node, p.launch_rate,
           p.steady < 0 ? "null" : p.steady ? "true" : "false");
    for (size_t i = 0; i < p.hostpids.size(); i++) printf("%s%d", i ? ", " : "", p.hostpids[i]);
    printf("], \"gpus\": [");
    for (size_t i = 0; i < p.gpu_ids.size(); i++) {
      const uint64_t want = i < p.want_since.size() ? p.want_since[i] : 0;
      printf("%s{\"gpu_id\": %u, \"holds_turn\": %s, \"waiting_ms\": ", i ? ", " : "", p.gpu_ids[i],
             i < p.gate.size() && p.gate[i] ? "true" : "false");
      if (want && now > want) printf("%.1f", (now - want) / 1e6);
      else printf("null");
      printf(", \"svm_vram\": %llu}", (unsigned long long)(i < p.svm_vram.size() ? p.svm_vram[i] : 0));
    }
    printf("]}");
  }
  printf("]}\n");
  return 0;
}

static int usage() {
  fprintf(stderr,
          "usage: vgpuctl <region-file> show|suspend|resume|block|unblock|reclaim|"
          "set-limit <dev> <size>|set-cu <dev> <pct>|set-host-limit <size>|priority <n>\n"
          "       vgpuctl ledger <board-dir>\n"
          "       vgpuctl board <board-dir>\n");
  return 2;
}

static void show(vgpu_region* r) {
  uint64_t host_limit = 0, host_used = 0;
  vgpu_region_host_info(r, &host_limit, &host_used);
  printf("{\"version\": %u, \"num_devices\": %d, \"suspended\": %d, \"priority\": %d, \"recent_kernel\": %d, "
         "\"samples\": %llu, \"other_refreshes\": %llu, \"host_limit\": %llu, \"host_used\": %llu,\n",
         vgpu_region_version(), vgpu_region_num_devices(r), vgpu_region_suspended(r), vgpu_region_get_priority(r),
         vgpu_region_get_recent_kernel(r), (unsigned long long)vgpu_region_samples(r),
         (unsigned long long)vgpu_region_other_refreshes(r), (unsigned long long)host_limit,
         (unsigned long long)host_used);
  printf(" \"devices\": [");
  int nd = vgpu_region_num_devices(r);
  for (int d = 0; d < nd; d++) {
    vgpu_device_info di;
    vgpu_region_device_info(r, d, &di);
    printf("%s\n  {\"index\": %d, \"uuid\": \"%s\", \"mem_limit\": %llu, \"phys_total\": %llu, \"used\": %llu, "
           "\"spilled\": %llu, \"monitor_used\": %llu, \"cu_limit_pct\": %d, \"cu_count\": %d, \"cu_mask_count\": %d, "
           "\"util_pct\": %d, \"cu_mode\": %d, \"crowd\": %d, \"credit_ns\": %lld, \"charged_ns\": %llu, "
           "\"wall_ns\": %llu, \"preempt\": %d, \"depth_cap\": %d}",
           d ? "," : "", d, di.uuid, (unsigned long long)di.mem_limit, (unsigned long long)di.phys_total,
           (unsigned long long)di.used, (unsigned long long)di.spilled, (unsigned long long)di.monitor_used,
           di.cu_limit_pct, di.cu_count, di.cu_mask_count, di.util_pct, di.cu_mode, di.crowd, (long long)di.credit_ns,
           (unsigned long long)di.charged_ns, (unsigned long long)di.wall_ns, di.preempt, di.depth_cap);
  }
  printf("],\n \"processes\": [");
  static vgpu_proc_info procs[1024];
  int np = vgpu_region_procs(r, procs, 1024);
  for (int i = 0; i < np; i++) {
    const vgpu_proc_info& p = procs[i];
    printf("%s\n  {\"pid\": %d, \"hostpid\": %d, \"status\": %d, \"launches\": %llu, \"throttle_ns\": %llu, "
           "\"suspend_ns\": %llu, \"oom_events\": %llu, \"host_used\": %llu, \"used\": [",
           i ? "," : "", p.pid, p.hostpid, p.status, (unsigned long long)p.launches,
           (unsigned long long)p.throttle_ns, (unsigned long long)p.suspend_ns, (unsigned long long)p.oom_events,
           (unsigned long long)p.host_used);
    for (int d = 0; d < (nd ? nd : 1); d++) printf("%s%llu", d ? ", " : "", (unsigned long long)p.used[d]);
    printf("]}");
  }
  printf("]}\n");
}

int main(int argc, char** argv) {
  if (argc < 3) return usage();
  if (!strcmp(argv[1], "ledger")) return show_ledgers(argv[2]);
  if (!strcmp(argv[1], "board")) return show_board(argv[2]);
  int err = 0;
  vgpu_region* r = vgpu_region_open(argv[1], 0, &err);
  if (!r) {
    fprintf(stderr, "vgpuctl: cannot open region %s: %s\n", argv[1], strerror(-err));
    return 1;
  }
  const char* cmd = argv[2];
  int rc = 0;
  if (!strcmp(cmd, "show")) show(r);
  else if (!strcmp(cmd, "suspend")) rc = vgpu_region_suspend_all(r);
  else if (!strcmp(cmd, "resume")) rc = vgpu_region_resume_all(r);
  else if (!strcmp(cmd, "block")) rc = vgpu_region_set_recent_kernel(r, -1);
  else if (!strcmp(cmd, "unblock")) rc = vgpu_region_set_recent_kernel(r, 2);
  else if (!strcmp(cmd, "reclaim")) printf("%d\n", vgpu_region_reclaim(r));
  else if (!strcmp(cmd, "set-limit") && argc == 5) {
    int64_t v = vgpu_parse_size(argv[4]);
    rc = v < 0 ? -1 : vgpu_region_set_memory_limit(r, atoi(argv[3]), (uint64_t)v);
  } else if (!strcmp(cmd, "set-cu") && argc == 5) {
    rc = vgpu_region_set_cu_limit(r, atoi(argv[3]), atoi(argv[4]));
  } else if (!strcmp(cmd, "set-host-limit") && argc == 4) {
    int64_t v = vgpu_parse_size(argv[3]);
    rc = v < 0 ? -1 : vgpu_region_set_host_limit(r, (uint64_t)v);
  }
  else if (!strcmp(cmd, "priority") && argc == 4) rc = vgpu_region_set_priority(r, atoi(argv[3]));
  else rc = usage();
  vgpu_region_close(r);
  return rc == 0 ? 0 : 1;
}
