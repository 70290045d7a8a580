// dlsym / dlvsym interposition: lookups made on a library handle never consult the
// preloaded shim, so hooked names are routed back into it here.
//
// Reference: libvgpu.so overrides dlsym [src/libvgpu.c:109-124] (__dlsym_hook_section routes
// 199 hooked driver names) so that runtimes that dlopen the driver still reach the hooks.
// On MI355X the lookups that need it:
//   * ROCr entry points looked up on a libhsa-runtime64 handle (ctypes.CDLL(libhsa...),
//     dlsym(dlopen("libhsa-runtime64.so.1"), "hsa_amd_memory_pool_allocate")): the HSA
//     layer is where the quota, the CU mask and the shim's own initialisation live, so a
//     lookup that found ROCr's definition of a name the shim exports under ROCR_1 gets the
//     shim's (hsa_hooks.cpp), for callers outside ROCr and the shim - hsa_init included,
//     so a ctypes-only HSA program initialises the shim;
//   * HIP runtimes loaded by handle: Triton (every torch.compile tenant) dlopens
//     libamdhip64 and resolves hipGetProcAddress with dlsym(handle, ...), then its launch
//     entry points through it. Names starting with "hip" that the shim gates
//     (hip_gates.def) and that resolve to the very entry point the gate forwards to are
//     redirected to the shim's definition (gates.cpp: hip_hook_for_name), for callers
//     outside libamdhip64;
//   * the in-container SMI tools: Python (ctypes over libamd_smi.so / librocm_smi64.so)
//     resolves every entry point with dlsym(handle, name). Only names starting with
//     "amdsmi_" / "rsmi_" that resolve into an SMI library and have a virtualising hook
//     are redirected (to smi_hooks.cpp), and only for callers outside the SMI libraries
//     (libamd_smi embeds and calls rocm_smi itself, with node indices);
//   * the lookup functions themselves: dlsym(libc, "dlsym") or dlvsym(.., "dlvsym", ..)
//     would hand out glibc's and skip all of the above, so those names get the shim's.
// dlvsym is interposed as well, with the same routing (versions must match: ROCR_1 for
// ROCr, the gate's version for HIP). Every lookup that is not routed is a guaranteed tail
// call ([[clang::musttail]]) into glibc, so RTLD_NEXT keeps resolving relative to the
// *original* caller - other interposers preloaded alongside the shim are unaffected.
// glibc's own dlsym / dlvsym are found by reading the C library's dynamic symbol table
// (dl_iterate_phdr): the shim cannot ask dlvsym for them once it interposes dlvsym.
// Both glibc symbol versions are provided (GLIBC_2.2.5 for old binaries and C libraries,
// GLIBC_2.34 for current ones). This file is compiled with clang (musttail).
#include <dlfcn.h>
#include <elf.h>
#include <link.h>
#include <sys/mman.h>
#include <unistd.h>

#include <atomic>
#include <cstdlib>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include <amd_smi/amdsmi.h>
#include <rocm_smi/rocm_smi.h>

#include "real.h"
#include "vgpu/config.h"
#include "vgpu/log.h"

extern "C" {
amdsmi_status_t amdsmi_get_gpu_memory_total(amdsmi_processor_handle, amdsmi_memory_type_t, uint64_t*);
amdsmi_status_t amdsmi_get_gpu_memory_usage(amdsmi_processor_handle, amdsmi_memory_type_t, uint64_t*);
amdsmi_status_t amdsmi_get_gpu_vram_usage(amdsmi_processor_handle, amdsmi_vram_usage_t*);
amdsmi_status_t amdsmi_get_processor_handles(amdsmi_socket_handle, uint32_t*, amdsmi_processor_handle*);
amdsmi_status_t amdsmi_get_gpu_process_list(amdsmi_processor_handle, uint32_t*, amdsmi_proc_info_t*);
rsmi_status_t rsmi_dev_memory_total_get(uint32_t, rsmi_memory_type_t, uint64_t*);
rsmi_status_t rsmi_dev_memory_usage_get(uint32_t, rsmi_memory_type_t, uint64_t*);
rsmi_status_t rsmi_compute_process_info_get(rsmi_process_info_t*, uint32_t*);
rsmi_status_t rsmi_compute_process_info_by_pid_get(uint32_t, rsmi_process_info_t*);
rsmi_status_t rsmi_num_monitor_devices(uint32_t*);
rsmi_status_t rsmi_compute_process_gpus_get(uint32_t, uint32_t*, uint32_t*);
void* shim_dlsym_v234(void* handle, const char* name);
void* shim_dlsym_v225(void* handle, const char* name);
void* shim_dlvsym_v234(void* handle, const char* name, const char* version);
void* shim_dlvsym_v225(void* handle, const char* name, const char* version);
void* shim_dlopen_v234(const char* file, int mode);
void* shim_dlopen_v225(const char* file, int mode);
void* shim_dlmopen_v234(Lmid_t lmid, const char* file, int mode);
void* shim_dlmopen_v234_compat(Lmid_t lmid, const char* file, int mode);
}

namespace vgpu {
void* rsmi_remap_hook(const char* name);  // smi_hooks.cpp (generated index remapping)
}

namespace {

using DlsymFn = void* (*)(void*, const char*);
using DlvsymFn = void* (*)(void*, const char*, const char*);

// VGPU_HOOK_DLSYM=0 turns the redirection off (read once when the shim is loaded).
bool g_dlsym_hook_on = true;
__attribute__((constructor)) void dlsym_hook_ctor() {
  if (vgpu::ceiling_present()) return;  // not a tenant's switch where the plugin set limits
  const char* s = getenv("VGPU_HOOK_DLSYM");
  if (s && (*s == '0' || *s == 'f' || *s == 'F' || *s == 'n' || *s == 'N')) g_dlsym_hook_on = false;
}

// ---------------------------------------------------------------- glibc's lookup functions

// Looks `name`@`version` up in the dynamic symbol table of the loaded C library (libc.so.6,
// or libdl.so.2 where glibc < 2.34 keeps the dl functions).
struct ElfQuery {
  const char* name;
  const char* version;
  void* found;
};

// Number of dynamic symbols from a DT_GNU_HASH table: past the highest bucket's chain end.
size_t gnu_hash_count(const uint32_t* gh) {
  const uint32_t nbuckets = gh[0], symoffset = gh[1], bloom_size = gh[2];
  const uint32_t* buckets = reinterpret_cast<const uint32_t*>(reinterpret_cast<const ElfW(Addr)*>(gh + 4) + bloom_size);
  const uint32_t* chain = buckets + nbuckets;
  uint32_t last = 0;
  for (uint32_t i = 0; i < nbuckets; i++)
    if (buckets[i] > last) last = buckets[i];
  if (last < symoffset) return symoffset;
  while (!(chain[last - symoffset] & 1u)) last++;
  return (size_t)last + 1;
}

int elf_lookup_cb(struct dl_phdr_info* info, size_t, void* data) {
  ElfQuery* q = static_cast<ElfQuery*>(data);
  const char* fn = info->dlpi_name;
  if (!fn || !*fn) return 0;
  const char* base_name = strrchr(fn, '/');
  base_name = base_name ? base_name + 1 : fn;
  if (strncmp(base_name, "libc.so.", 8) != 0 && strncmp(base_name, "libdl.so.", 9) != 0) return 0;
  const ElfW(Addr) base = info->dlpi_addr;
  const ElfW(Dyn)* dyn = nullptr;
  for (int i = 0; i < info->dlpi_phnum; i++)
    if (info->dlpi_phdr[i].p_type == PT_DYNAMIC) dyn = reinterpret_cast<const ElfW(Dyn)*>(base + info->dlpi_phdr[i].p_vaddr);
  if (!dyn) return 0;
  const ElfW(Sym)* symtab = nullptr;
  const char* strtab = nullptr;
  const ElfW(Half)* versym = nullptr;
  const char* verdef = nullptr;
  const uint32_t* hash = nullptr;
  const uint32_t* gnu_hash = nullptr;
  // ld.so relocates these d_ptr values in place on x86-64; a value below the load base is
  // still an offset.
  auto at = [base](ElfW(Addr) a) { return a < base ? a + base : a; };
  for (const ElfW(Dyn)* d = dyn; d->d_tag != DT_NULL; d++) {
    switch (d->d_tag) {
      case DT_SYMTAB: symtab = reinterpret_cast<const ElfW(Sym)*>(at(d->d_un.d_ptr)); break;
      case DT_STRTAB: strtab = reinterpret_cast<const char*>(at(d->d_un.d_ptr)); break;
      case DT_VERSYM: versym = reinterpret_cast<const ElfW(Half)*>(at(d->d_un.d_ptr)); break;
      case DT_VERDEF: verdef = reinterpret_cast<const char*>(at(d->d_un.d_ptr)); break;
      case DT_HASH: hash = reinterpret_cast<const uint32_t*>(at(d->d_un.d_ptr)); break;
      case DT_GNU_HASH: gnu_hash = reinterpret_cast<const uint32_t*>(at(d->d_un.d_ptr)); break;
      default: break;
    }
  }
  if (!symtab || !strtab || !versym || !verdef || (!hash && !gnu_hash)) return 0;
  const size_t nsyms = hash ? hash[1] : gnu_hash_count(gnu_hash);
  for (size_t i = 0; i < nsyms; i++) {
    const ElfW(Sym)& s = symtab[i];
    if (s.st_shndx == SHN_UNDEF || !s.st_value || strcmp(strtab + s.st_name, q->name) != 0) continue;
    const ElfW(Half) ndx = versym[i] & 0x7fff;
    for (const char* v = verdef;;) {
      const ElfW(Verdef)* vd = reinterpret_cast<const ElfW(Verdef)*>(v);
      if (vd->vd_ndx == ndx && vd->vd_cnt > 0) {
        const ElfW(Verdaux)* aux = reinterpret_cast<const ElfW(Verdaux)*>(v + vd->vd_aux);
        if (strcmp(strtab + aux->vda_name, q->version) == 0) {
          q->found = reinterpret_cast<void*>(base + s.st_value);
          return 1;
        }
        break;
      }
      if (!vd->vd_next) break;
      v += vd->vd_next;
    }
  }
  return 0;
}

void* libc_symbol(const char* name, const char* version) {
  ElfQuery q{name, version, nullptr};
  dl_iterate_phdr(elf_lookup_cb, &q);
  return q.found;
}

std::atomic<DlsymFn> g_real_234{nullptr};
std::atomic<DlsymFn> g_real_225{nullptr};
std::atomic<DlvsymFn> g_realv_234{nullptr};
std::atomic<DlvsymFn> g_realv_225{nullptr};

// glibc's definition of `name` for symbol version `ver`, or its other version when the C
// library predates it (glibc < 2.34 has only GLIBC_2.2.5).
template <typename Fn>
Fn load_real(std::atomic<Fn>& slot, const char* name, const char* ver) {
  Fn f = slot.load(std::memory_order_acquire);
  if (__builtin_expect(f != nullptr, 1)) return f;
  f = reinterpret_cast<Fn>(libc_symbol(name, ver));
  if (!f) f = reinterpret_cast<Fn>(libc_symbol(name, ver[7] == '3' ? "GLIBC_2.2.5" : "GLIBC_2.34"));
  slot.store(f, std::memory_order_release);
  return f;
}

using DlopenFn = void* (*)(const char*, int);
using DlmopenFn = void* (*)(Lmid_t, const char*, int);
using DlinfoFn = int (*)(void*, int, void*);
std::atomic<DlopenFn> g_open_234{nullptr};
std::atomic<DlopenFn> g_open_225{nullptr};
std::atomic<DlmopenFn> g_mopen_234{nullptr};
std::atomic<DlmopenFn> g_mopen_234c{nullptr};
std::atomic<DlinfoFn> g_info{nullptr};
DlopenFn real_dlopen_234() { return load_real(g_open_234, "dlopen", "GLIBC_2.34"); }
DlopenFn real_dlopen_225() { return load_real(g_open_225, "dlopen", "GLIBC_2.2.5"); }
// dlmopen's first version is GLIBC_2.3.4 (load_real's fallback covers glibc < 2.34 through it).
DlmopenFn real_dlmopen_234() {
  DlmopenFn f = g_mopen_234.load(std::memory_order_acquire);
  if (__builtin_expect(f != nullptr, 1)) return f;
  f = reinterpret_cast<DlmopenFn>(libc_symbol("dlmopen", "GLIBC_2.34"));
  if (!f) f = reinterpret_cast<DlmopenFn>(libc_symbol("dlmopen", "GLIBC_2.3.4"));
  g_mopen_234.store(f, std::memory_order_release);
  return f;
}
DlmopenFn real_dlmopen_compat() {
  DlmopenFn f = g_mopen_234c.load(std::memory_order_acquire);
  if (__builtin_expect(f != nullptr, 1)) return f;
  f = reinterpret_cast<DlmopenFn>(libc_symbol("dlmopen", "GLIBC_2.3.4"));
  if (!f) f = reinterpret_cast<DlmopenFn>(libc_symbol("dlmopen", "GLIBC_2.34"));
  g_mopen_234c.store(f, std::memory_order_release);
  return f;
}
DlinfoFn real_dlinfo() {
  DlinfoFn f = g_info.load(std::memory_order_acquire);
  if (__builtin_expect(f != nullptr, 1)) return f;
  f = reinterpret_cast<DlinfoFn>(libc_symbol("dlinfo", "GLIBC_2.3.3"));
  if (!f) f = reinterpret_cast<DlinfoFn>(libc_symbol("dlinfo", "GLIBC_2.34"));
  g_info.store(f, std::memory_order_release);
  return f;
}

DlsymFn real_dlsym_234() { return load_real(g_real_234, "dlsym", "GLIBC_2.34"); }
DlsymFn real_dlsym_225() { return load_real(g_real_225, "dlsym", "GLIBC_2.2.5"); }
DlvsymFn real_dlvsym_234() { return load_real(g_realv_234, "dlvsym", "GLIBC_2.34"); }
DlvsymFn real_dlvsym_225() { return load_real(g_realv_225, "dlvsym", "GLIBC_2.2.5"); }

// ---------------------------------------------------------------- where an address lives

const char* object_of(const void* addr) {
  Dl_info info;
  if (!addr || !dladdr(addr, &info) || !info.dli_fname) return nullptr;
  return info.dli_fname;
}

bool in_library(const void* addr, const char* soname_part) {
  const char* f = object_of(addr);
  return f && strstr(f, soname_part) && !strstr(f, "vgpu");
}

bool in_hip_library(const void* addr) { return in_library(addr, "libamdhip64"); }
bool in_hsa_library(const void* addr) { return in_library(addr, "libhsa-runtime64"); }

bool in_smi_library(const void* addr) {
  const char* f = object_of(addr);
  return f && (strstr(f, "amd_smi") || strstr(f, "rocm_smi")) && !strstr(f, "vgpu");
}

bool in_libc(const void* addr) {
  const char* f = object_of(addr);
  if (!f) return false;
  const char* b = strrchr(f, '/');
  b = b ? b + 1 : f;
  return strncmp(b, "libc.so.", 8) == 0 || strncmp(b, "libdl.so.", 9) == 0;
}

bool in_shim(const void* addr) {
  Dl_info a, self;
  return addr && dladdr(addr, &a) && dladdr(reinterpret_cast<const void*>(&in_shim), &self) &&
         a.dli_fbase == self.dli_fbase;
}

// ---------------------------------------------------------------- routing tables

struct Hook {
  const char* name;
  void* fn;
};

const Hook kSmiHooks[] = {
    {"amdsmi_get_gpu_memory_total", reinterpret_cast<void*>(&amdsmi_get_gpu_memory_total)},
    {"amdsmi_get_gpu_memory_usage", reinterpret_cast<void*>(&amdsmi_get_gpu_memory_usage)},
    {"amdsmi_get_gpu_vram_usage", reinterpret_cast<void*>(&amdsmi_get_gpu_vram_usage)},
    {"amdsmi_get_processor_handles", reinterpret_cast<void*>(&amdsmi_get_processor_handles)},
    {"amdsmi_get_gpu_process_list", reinterpret_cast<void*>(&amdsmi_get_gpu_process_list)},
    {"rsmi_dev_memory_total_get", reinterpret_cast<void*>(&rsmi_dev_memory_total_get)},
    {"rsmi_dev_memory_usage_get", reinterpret_cast<void*>(&rsmi_dev_memory_usage_get)},
    {"rsmi_compute_process_info_get", reinterpret_cast<void*>(&rsmi_compute_process_info_get)},
    {"rsmi_compute_process_info_by_pid_get", reinterpret_cast<void*>(&rsmi_compute_process_info_by_pid_get)},
    {"rsmi_num_monitor_devices", reinterpret_cast<void*>(&rsmi_num_monitor_devices)},
    {"rsmi_compute_process_gpus_get", reinterpret_cast<void*>(&rsmi_compute_process_gpus_get)},
};

// hsa* lookups on a library handle: the shim's definition (exported as name@ROCR_1) when
// the lookup found ROCr's entry point of that name.
__attribute__((noinline)) void* maybe_hook_hsa(const char* name, const char* version, void* found,
                                               const void* caller) {
  if (!found || (version && strcmp(version, "ROCR_1") != 0)) return nullptr;
  if (!in_hsa_library(found) || in_hsa_library(caller) || in_shim(caller)) return nullptr;
  return vgpu::hsa_hook_for_name(name);
}

// hip* lookups on a library handle: the shim's gate when the lookup found the runtime's
// entry point that gate forwards to.
__attribute__((noinline)) void* maybe_hook_hip(const char* name, const char* version, void* found,
                                               const void* caller) {
  if (!found || !in_hip_library(found)) return nullptr;
  if (in_hip_library(caller) || in_shim(caller)) return nullptr;
  return vgpu::hip_hook_for_name(name, version, found);
}

__attribute__((noinline)) void* maybe_hook_smi(const char* name, void* found, const void* caller) {
  void* hook = nullptr;
  for (const Hook& h : kSmiHooks)
    if (strcmp(name, h.name) == 0) hook = h.fn;
  if (!hook && name[0] == 'r') hook = vgpu::rsmi_remap_hook(name);
  if (!hook || in_smi_library(caller)) return nullptr;
  return found && in_smi_library(found) ? hook : nullptr;
}

// dlsym / dlvsym themselves, found in the C library: the shim's interposer of the same
// symbol version (so a tenant cannot fetch glibc's and look ROCr up unrouted).
__attribute__((noinline)) void* maybe_hook_lookup(const char* name, void* found, const void* caller) {
  if (!found || in_shim(caller) || !in_libc(found)) return nullptr;
  if (strcmp(name, "dlsym") == 0)
    return found == reinterpret_cast<void*>(real_dlsym_225()) && found != reinterpret_cast<void*>(real_dlsym_234())
               ? reinterpret_cast<void*>(&shim_dlsym_v225)
               : reinterpret_cast<void*>(&shim_dlsym_v234);
  if (strcmp(name, "dlvsym") == 0)
    return found == reinterpret_cast<void*>(real_dlvsym_225()) && found != reinterpret_cast<void*>(real_dlvsym_234())
               ? reinterpret_cast<void*>(&shim_dlvsym_v225)
               : reinterpret_cast<void*>(&shim_dlvsym_v234);
  return nullptr;
}

// Whether a looked-up name may be routed at all (cheap first-character filter: every other
// lookup goes straight to glibc).
inline bool routable(const char* name) {
  switch (name[0]) {
    case 'h': return name[1] == 'i' || (name[1] == 's' && name[2] == 'a' && name[3] == '_');
    case 'a': return strncmp(name, "amdsmi_", 7) == 0;
    case 'r': return strncmp(name, "rsmi_", 5) == 0;
    case 'd': return name[1] == 'l' && (strcmp(name, "dlsym") == 0 || strcmp(name, "dlvsym") == 0 ||
                                        strcmp(name, "dlopen") == 0 || strcmp(name, "dlmopen") == 0);
    default: return false;
  }
}

// The routed answer for a lookup that found `found`, or null to keep it.
void* route(const char* name, const char* version, void* found, const void* caller) {
  switch (name[0]) {
    case 'h': return name[1] == 'i' ? maybe_hook_hip(name, version, found, caller)
                                    : maybe_hook_hsa(name, version, found, caller);
    case 'a':
    case 'r': return maybe_hook_smi(name, found, caller);
    case 'd': return maybe_hook_lookup(name, found, caller);
    default: return nullptr;
  }
}

// ---------------------------------------------------------------- loader-level bypasses
//
// RTLD_DEEPBIND puts a loaded object's own dependency scope ahead of the global scope, where
// the preloaded shim is: a HIP runtime loaded that way binds its hsa_* imports straight to
// ROCr (no quota, no CU mask), and an application object loaded that way binds its hip*
// imports straight to HIP (no launch gate). PyTorch imported afterwards reuses the HIP
// already loaded, so one flag would lift every limit. dlmopen(LM_ID_NEWLM) goes further: a
// second link-map namespace, with its own ROCr, that never saw the preload.
//
//   * dlopen of the ROCm runtime itself (libamdhip64 / libhsa-runtime64) with RTLD_DEEPBIND:
//     the flag is dropped (a guaranteed tail call, so the caller's RUNPATH still applies).
//   * any other RTLD_DEEPBIND dlopen: it may pull ROCr in as a dependency, or - ROCm already
//     loaded, the usual case once torch is imported - bind a tenant module's hip* imports to
//     the HIP runtime ahead of the shim (its launches would skip the GPU-time limiter). After
//     the load, every object it brought in has its GOT entries for the names the shim hooks
//     rewritten to the shim's definitions - what binding through the global scope would have
//     given. The load itself is then a plain call: a bare file name the loader does not find
//     from the shim's position (LD_LIBRARY_PATH, the executable's RUNPATH, ld.so.cache, the
//     default directories) is tried in the calling object's own DT_RUNPATH / DT_RPATH
//     directories ($ORIGIN expanded), as the caller's own dlopen would.
//   * dlmopen of anything into a namespace other than the base one that ends up holding the
//     ROCm runtime is refused (logged; NULL returned) in a vGPU container - limits configured
//     in the environment or by a plugin limits file - and only logged elsewhere.
// The raw KFD ioctl interface remains outside any interposer; the KFD-measured OOM killer
// (watcher.cpp) is the backstop for it.

bool rocm_runtime_path(const char* f) {
  const char* b = strrchr(f, '/');
  b = b ? b + 1 : f;
  return strstr(b, "libamdhip64") || strstr(b, "libhsa-runtime64");
}

int rocm_loaded_cb(struct dl_phdr_info* info, size_t, void*) {
  const char* n = info->dlpi_name;
  return n && *n && !strstr(n, "vgpu") && (strstr(n, "libhsa-runtime64") || strstr(n, "libamdhip64")) ? 1 : 0;
}

bool rocm_loaded() { return dl_iterate_phdr(rocm_loaded_cb, nullptr) != 0; }

using Loaded = std::vector<std::pair<ElfW(Addr), const ElfW(Phdr)*>>;

int snapshot_cb(struct dl_phdr_info* info, size_t, void* data) {
  static_cast<Loaded*>(data)->emplace_back(info->dlpi_addr, info->dlpi_phdr);
  return 0;
}

bool vgpu_container_env() {
  if (vgpu::ceiling_present()) return true;
  for (char** e = environ; e && *e; e++)
    if (!strncmp(*e, "VGPU_DEVICE_MEMORY_LIMIT", 24) || !strncmp(*e, "VGPU_DEVICE_CU_LIMIT", 20)) return true;
  return false;
}

// Points `slot` (a GOT entry inside a RELRO range when `relro`) at `target`.
void write_got(void** slot, void* target, bool relro) {
  if (*slot == target) return;
  const uintptr_t pg = (uintptr_t)sysconf(_SC_PAGESIZE);
  void* page = reinterpret_cast<void*>(reinterpret_cast<uintptr_t>(slot) & ~(pg - 1));
  if (relro && mprotect(page, pg, PROT_READ | PROT_WRITE) != 0) return;
  *slot = target;
  if (relro) mprotect(page, pg, PROT_READ);
}

struct Rebind {
  ElfW(Addr) base;
  const ElfW(Phdr)* phdr;
  int phnum;
  const char* name;
  int patched;
};

// Rewrites the GOT entries of one object for the names the shim hooks (ROCr entry points:
// hsa_hook_for_name; gated HIP entry points: hip_hook_for_name).
int rebind_object(const Rebind& o) {
  const ElfW(Dyn)* dyn = nullptr;
  uintptr_t relro_lo = 0, relro_hi = 0;
  for (int i = 0; i < o.phnum; i++) {
    if (o.phdr[i].p_type == PT_DYNAMIC) dyn = reinterpret_cast<const ElfW(Dyn)*>(o.base + o.phdr[i].p_vaddr);
    if (o.phdr[i].p_type == PT_GNU_RELRO) {
      relro_lo = o.base + o.phdr[i].p_vaddr;
      relro_hi = relro_lo + o.phdr[i].p_memsz;
    }
  }
  if (!dyn) return 0;
  const ElfW(Sym)* symtab = nullptr;
  const char* strtab = nullptr;
  const ElfW(Rela)* rela = nullptr;
  const ElfW(Rela)* jmprel = nullptr;
  size_t relasz = 0, pltrelsz = 0;
  auto at = [&o](ElfW(Addr) a) { return a < o.base ? a + o.base : a; };
  for (const ElfW(Dyn)* d = dyn; d->d_tag != DT_NULL; d++) {
    switch (d->d_tag) {
      case DT_SYMTAB: symtab = reinterpret_cast<const ElfW(Sym)*>(at(d->d_un.d_ptr)); break;
      case DT_STRTAB: strtab = reinterpret_cast<const char*>(at(d->d_un.d_ptr)); break;
      case DT_RELA: rela = reinterpret_cast<const ElfW(Rela)*>(at(d->d_un.d_ptr)); break;
      case DT_RELASZ: relasz = d->d_un.d_val; break;
      case DT_JMPREL: jmprel = reinterpret_cast<const ElfW(Rela)*>(at(d->d_un.d_ptr)); break;
      case DT_PLTRELSZ: pltrelsz = d->d_un.d_val; break;
      default: break;
    }
  }
  if (!symtab || !strtab) return 0;
  int n = 0;
  auto visit = [&](const ElfW(Rela)* r, size_t bytes) {
    for (size_t i = 0; r && i < bytes / sizeof(ElfW(Rela)); i++) {
      const unsigned type = ELF64_R_TYPE(r[i].r_info);
      if (type != R_X86_64_JUMP_SLOT && type != R_X86_64_GLOB_DAT) continue;
      const ElfW(Sym)& sym = symtab[ELF64_R_SYM(r[i].r_info)];
      if (sym.st_shndx != SHN_UNDEF) continue;
      const char* name = strtab + sym.st_name;
      void* hook = nullptr;
      if (name[0] == 'h' && name[1] == 's' && name[2] == 'a' && name[3] == '_') {
        hook = vgpu::hsa_hook_for_name(name);
      } else if (name[0] == 'h' && name[1] == 'i' && name[2] == 'p') {
        void* real = vgpu::resolve_real("libamdhip64", name, nullptr, true);
        if (real) hook = vgpu::hip_hook_for_name(name, nullptr, real);
      }
      if (!hook) continue;
      void** slot = reinterpret_cast<void**>(o.base + r[i].r_offset);
      const uintptr_t a = reinterpret_cast<uintptr_t>(slot);
      write_got(slot, hook, a >= relro_lo && a < relro_hi);
      n++;
    }
  };
  visit(rela, relasz);
  visit(jmprel, pltrelsz);
  return n;
}

struct NewObjects {
  const Loaded* before;
  std::vector<Rebind> out;
};

int new_objects_cb(struct dl_phdr_info* info, size_t, void* data) {
  NewObjects* n = static_cast<NewObjects*>(data);
  for (const auto& b : *n->before)
    if (b.first == info->dlpi_addr && b.second == info->dlpi_phdr) return 0;
  const char* nm = info->dlpi_name ? info->dlpi_name : "";
  const char* b = strrchr(nm, '/');
  b = b ? b + 1 : nm;
  // ROCr's own calls stay inside ROCr; the shim and the C library are never rebound.
  if (strstr(nm, "vgpu") || strstr(b, "libhsa-runtime64") || !strncmp(b, "libc.so", 7) || !strncmp(b, "ld-linux", 8))
    return 0;
  n->out.push_back(Rebind{info->dlpi_addr, info->dlpi_phdr, info->dlpi_phnum, nm, 0});
  return 0;
}

void rebind_new_objects(const Loaded& before, const char* file) {
  NewObjects n{&before, {}};
  dl_iterate_phdr(new_objects_cb, &n);
  int total = 0;
  for (Rebind& o : n.out) total += rebind_object(o);
  if (total)
    VLOG_WARN("dlopen(%s, RTLD_DEEPBIND): %d GOT entries of %zu new object(s) bound to the vGPU shim", file, total,
              n.out.size());
}

// The namespace of `h` holds the ROCm runtime.
bool namespace_has_rocm(void* h) {
  DlinfoFn info = real_dlinfo();
  struct link_map* lm = nullptr;
  if (!info || info(h, RTLD_DI_LINKMAP, &lm) != 0 || !lm) return false;
  while (lm->l_prev) lm = lm->l_prev;
  for (; lm; lm = lm->l_next)
    if (lm->l_name && rocm_runtime_path(lm->l_name)) return true;
  return false;
}

}  // namespace

namespace vgpu {
// The shim's own lookups must bypass the interposers (they want the real symbols). Called
// from the shim, RTLD_NEXT stays relative to the shim.
void* real_dlsym(void* handle, const char* name) { return real_dlsym_234()(handle, name); }
void* real_dlvsym(void* handle, const char* name, const char* version) {
  return real_dlvsym_234()(handle, name, version);
}
}  // namespace vgpu

namespace {

// A loader entry point looked up on a handle of a namespace other than the base one: that
// namespace's own dlopen / dlmopen / dlsym never saw the preload, so a tenant that dlmopen'ed
// something harmless (libc) could load the ROCm runtime through it. Refused (NULL) in a vGPU
// container. Best effort - code running inside such a namespace can still reach its loader
// (a constructor that dlopens); checked_dlmopen refuses a namespace found holding ROCm when
// dlmopen returns, and the KFD-measured OOM killer (watcher.cpp) is the backstop.
__attribute__((noinline)) bool foreign_loader_lookup(void* handle, const char* name) {
  if (name[0] != 'd' || name[1] != 'l') return false;
  DlinfoFn info = real_dlinfo();
  Lmid_t lmid = LM_ID_BASE;
  if (!info || info(handle, RTLD_DI_LMID, &lmid) != 0 || lmid == LM_ID_BASE) return false;
  if (!vgpu_container_env()) return false;
  VLOG_ERROR("dlsym(%s) on a handle of link-map namespace %ld refused: its loader bypasses the vGPU shim", name,
             (long)lmid);
  return true;
}

}  // namespace

extern "C" {

// A routable lookup on a library handle is resolved first (a plain call: the handle names
// the library, so the result does not depend on the caller) and replaced by the shim's
// definition when it is one; every other lookup is a guaranteed tail call so RTLD_NEXT
// stays relative to the caller.
#define VGPU_DLSYM_BODY(realfn)                                                           \
  DlsymFn real = realfn();                                                                \
  if (__builtin_expect(g_dlsym_hook_on && name != nullptr, 1) && handle != RTLD_NEXT &&   \
      handle != RTLD_DEFAULT && routable(name)) {                                         \
    if (__builtin_expect(foreign_loader_lookup(handle, name), 0)) return nullptr;          \
    void* p = real(handle, name);                                                         \
    void* h = route(name, nullptr, p, __builtin_return_address(0));                       \
    return h ? h : p;                                                                     \
  }                                                                                       \
  [[clang::musttail]] return real(handle, name);

#define VGPU_DLVSYM_BODY(realfn)                                                          \
  DlvsymFn real = realfn();                                                               \
  if (__builtin_expect(g_dlsym_hook_on && name != nullptr, 1) && handle != RTLD_NEXT &&   \
      handle != RTLD_DEFAULT && routable(name)) {                                         \
    if (__builtin_expect(foreign_loader_lookup(handle, name), 0)) return nullptr;          \
    void* p = real(handle, name, version);                                                \
    void* h = route(name, version, p, __builtin_return_address(0));                       \
    return h ? h : p;                                                                     \
  }                                                                                       \
  [[clang::musttail]] return real(handle, name, version);

__attribute__((visibility("default"))) void* shim_dlsym_v234(void* handle, const char* name) {
  VGPU_DLSYM_BODY(real_dlsym_234)
}

__attribute__((visibility("default"))) void* shim_dlsym_v225(void* handle, const char* name) {
  VGPU_DLSYM_BODY(real_dlsym_225)
}

__attribute__((visibility("default"))) void* shim_dlvsym_v234(void* handle, const char* name, const char* version) {
  VGPU_DLVSYM_BODY(real_dlvsym_234)
}

__attribute__((visibility("default"))) void* shim_dlvsym_v225(void* handle, const char* name, const char* version) {
  VGPU_DLVSYM_BODY(real_dlvsym_225)
}

// dlopen: see "loader-level bypasses" above.
#define VGPU_DLOPEN_BODY(realfn)                                                          \
  DlopenFn real = realfn();                                                               \
  if (__builtin_expect(!g_dlsym_hook_on || !file || !(mode & RTLD_DEEPBIND), 1))          \
    [[clang::musttail]] return real(file, mode);                                          \
  if (rocm_runtime_path(file)) {                                                          \
    VLOG_WARN("dlopen(%s): RTLD_DEEPBIND dropped (the ROCm runtime binds through the vGPU shim)", file); \
    [[clang::musttail]] return real(file, mode & ~RTLD_DEEPBIND);                         \
  }                                                                                       \
  return deepbind_open(real, file, mode, __builtin_return_address(0));

// The directories of the calling object's DT_RUNPATH (or DT_RPATH), $ORIGIN expanded. The
// object is found by address with dl_iterate_phdr (dladdr1 is a GLIBC_2.34 symbol, which the
// shim must not need: test_native_core.py).
struct CallerObject {
  uintptr_t addr;
  ElfW(Addr) base = 0;
  const ElfW(Dyn)* dyn = nullptr;
  std::string name;
};

static int caller_object_cb(struct dl_phdr_info* info, size_t, void* data) {
  CallerObject* c = static_cast<CallerObject*>(data);
  bool inside = false;
  const ElfW(Dyn)* dyn = nullptr;
  for (int i = 0; i < info->dlpi_phnum; i++) {
    const ElfW(Phdr)& ph = info->dlpi_phdr[i];
    const uintptr_t lo = info->dlpi_addr + ph.p_vaddr;
    if (ph.p_type == PT_LOAD && c->addr >= lo && c->addr < lo + ph.p_memsz) inside = true;
    if (ph.p_type == PT_DYNAMIC) dyn = reinterpret_cast<const ElfW(Dyn)*>(lo);
  }
  if (!inside) return 0;
  c->base = info->dlpi_addr;
  c->dyn = dyn;
  c->name = info->dlpi_name ? info->dlpi_name : "";
  return 1;
}

static std::vector<std::string> caller_search_dirs(const void* caller) {
  std::vector<std::string> dirs;
  CallerObject c;
  c.addr = reinterpret_cast<uintptr_t>(caller);
  if (!caller || !dl_iterate_phdr(caller_object_cb, &c) || !c.dyn) return dirs;
  const char* strtab = nullptr;
  ElfW(Addr) runpath = 0, rpath = 0;
  bool has_runpath = false, has_rpath = false;
  for (const ElfW(Dyn)* d = c.dyn; d->d_tag != DT_NULL; d++) {
    if (d->d_tag == DT_STRTAB)
      strtab = reinterpret_cast<const char*>(d->d_un.d_ptr < c.base ? d->d_un.d_ptr + c.base : d->d_un.d_ptr);
    if (d->d_tag == DT_RUNPATH) {
      runpath = d->d_un.d_val;
      has_runpath = true;
    }
    if (d->d_tag == DT_RPATH) {
      rpath = d->d_un.d_val;
      has_rpath = true;
    }
  }
  if (!strtab || (!has_runpath && !has_rpath)) return dirs;
  // The main program's name is empty in the list: /proc/self/exe's directory is its origin.
  std::string origin = c.name;
  if (origin.empty()) {
    char exe[4096];
    const ssize_t n = readlink("/proc/self/exe", exe, sizeof(exe) - 1);
    origin = n > 0 ? std::string(exe, (size_t)n) : ".";
  }
  origin = origin.find('/') == std::string::npos ? "." : origin.substr(0, origin.rfind('/'));
  std::string list = strtab + (has_runpath ? runpath : rpath), cur;
  for (size_t i = 0; i <= list.size(); i++) {
    if (i == list.size() || list[i] == ':') {
      for (const char* tok : {"$ORIGIN", "${ORIGIN}"})
        for (size_t at; (at = cur.find(tok)) != std::string::npos;) cur.replace(at, strlen(tok), origin);
      if (!cur.empty()) dirs.push_back(cur);
      cur.clear();
    } else {
      cur += list[i];
    }
  }
  return dirs;
}

__attribute__((noinline)) static void* deepbind_open(DlopenFn real, const char* file, int mode, const void* caller) {
  Loaded before;
  dl_iterate_phdr(snapshot_cb, &before);
  void* h = real(file, mode);
  if (!h && !strchr(file, '/'))
    for (const std::string& d : caller_search_dirs(caller))
      if ((h = real((d + "/" + file).c_str(), mode))) break;
  if (h && rocm_loaded()) rebind_new_objects(before, file);
  return h;
}

__attribute__((visibility("default"))) void* shim_dlopen_v234(const char* file, int mode) {
  VGPU_DLOPEN_BODY(real_dlopen_234)
}

__attribute__((visibility("default"))) void* shim_dlopen_v225(const char* file, int mode) {
  VGPU_DLOPEN_BODY(real_dlopen_225)
}

// dlmopen: a namespace other than the base one never saw the preloaded shim.
__attribute__((noinline)) static void* checked_dlmopen(DlmopenFn real, Lmid_t lmid, const char* file, int mode) {
  void* h = real(lmid, file, mode);
  if (!h || !namespace_has_rocm(h)) return h;
  if (!vgpu_container_env()) {
    VLOG_WARN("dlmopen(%s): the ROCm runtime was loaded into a separate namespace, outside the vGPU shim", file);
    return h;
  }
  VLOG_ERROR("dlmopen(%s): refused - a second link-map namespace would hold a ROCm runtime outside the vGPU "
             "limits", file);
  dlclose(h);
  return nullptr;
}

#define VGPU_DLMOPEN_BODY(realfn)                                                         \
  DlmopenFn real = realfn();                                                              \
  if (__builtin_expect(!g_dlsym_hook_on || !file || lmid == LM_ID_BASE, 1))               \
    [[clang::musttail]] return real(lmid, file, mode);                                    \
  return checked_dlmopen(real, lmid, file, mode);

__attribute__((visibility("default"))) void* shim_dlmopen_v234(Lmid_t lmid, const char* file, int mode) {
  VGPU_DLMOPEN_BODY(real_dlmopen_234)
}

__attribute__((visibility("default"))) void* shim_dlmopen_v234_compat(Lmid_t lmid, const char* file, int mode) {
  VGPU_DLMOPEN_BODY(real_dlmopen_compat)
}

}  // extern "C"

__asm__(".symver shim_dlopen_v234, dlopen@@GLIBC_2.34");
__asm__(".symver shim_dlopen_v225, dlopen@GLIBC_2.2.5");
__asm__(".symver shim_dlmopen_v234, dlmopen@@GLIBC_2.34");
__asm__(".symver shim_dlmopen_v234_compat, dlmopen@GLIBC_2.3.4");
__asm__(".symver shim_dlsym_v234, dlsym@@GLIBC_2.34");
__asm__(".symver shim_dlsym_v225, dlsym@GLIBC_2.2.5");
__asm__(".symver shim_dlvsym_v234, dlvsym@@GLIBC_2.34");
__asm__(".symver shim_dlvsym_v225, dlvsym@GLIBC_2.2.5");
