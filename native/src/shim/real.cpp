#include "real.h"

#include <dlfcn.h>
#include <link.h>

#include <cstring>

#include "vgpu/log.h"

namespace vgpu {

namespace {
struct Find {
  const char* substr;
  void* self_base;
  const char* path;
};

// Any loaded object (other than the shim) that defines `name`: the SMI entry points may
// live in librocm_smi64 or be statically linked into, and re-exported by, libamd_smi.
struct FindSym {
  const char* name;
  void* self_base;
  void* found;
};

int find_sym_cb(struct dl_phdr_info* info, size_t, void* data) {
  FindSym* f = static_cast<FindSym*>(data);
  if (!info->dlpi_name || !info->dlpi_name[0] || (void*)info->dlpi_addr == f->self_base) return 0;
  if (strstr(info->dlpi_name, "vgpu")) return 0;
  void* h = dlopen(info->dlpi_name, RTLD_NOLOAD | RTLD_LAZY);
  if (!h) return 0;
  void* p = real_dlsym(h, f->name);
  dlclose(h);
  if (!p) return 0;
  Dl_info di;
  // dlsym on a handle also searches the object's dependencies: accept only a definition
  // that does not resolve back into the shim.
  if (dladdr(p, &di) && di.dli_fbase == f->self_base) return 0;
  f->found = p;
  return 1;
}

int find_cb(struct dl_phdr_info* info, size_t, void* data) {
  Find* f = static_cast<Find*>(data);
  if (!info->dlpi_name || !info->dlpi_name[0]) return 0;
  if ((void*)info->dlpi_addr == f->self_base) return 0;
  if (strstr(info->dlpi_name, f->substr) && !strstr(info->dlpi_name, "vgpu")) {
    f->path = info->dlpi_name;
    return 1;
  }
  return 0;
}
}  // namespace

void* resolve_real(const char* lib_substr, const char* name, const char* ver, bool quiet) {
  Dl_info self;
  void* self_base = nullptr;
  if (dladdr(reinterpret_cast<void*>(&resolve_real), &self)) self_base = self.dli_fbase;
  Find f{lib_substr, self_base, nullptr};
  dl_iterate_phdr(find_cb, &f);
  void* p = nullptr;
  if (f.path) {
    void* h = dlopen(f.path, RTLD_NOLOAD | RTLD_LAZY);
    if (h) {
      p = ver ? real_dlvsym(h, name, ver) : nullptr;
      if (!p) p = real_dlsym(h, name);
      // dlopen(RTLD_NOLOAD) took a reference; the object stays loaded regardless.
      dlclose(h);
    }
  }
  if (!p) p = ver ? real_dlvsym(RTLD_NEXT, name, ver) : nullptr;
  if (!p) p = real_dlsym(RTLD_NEXT, name);
  if (!p) {
    FindSym fs{name, self_base, nullptr};
    dl_iterate_phdr(find_sym_cb, &fs);
    p = fs.found;
  }
  if (!p && !quiet) VLOG_ERROR("cannot resolve real %s in %s", name, lib_substr);
  else if (!p) VLOG_DEBUG("%s is not defined by the loaded %s", name, lib_substr);
  return p;
}

}  // namespace vgpu
