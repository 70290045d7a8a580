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

void* resolve_real(const char* lib_substr, const char* name, const char* ver) {
  Dl_info self;
  void* self_base = nullptr;
  if (dladdr(reinterpret_cast<void*>(&resolve_real), &self)) self_base = self.dli_fbase;
  Find f{lib_substr, self_base, nullptr};
  dl_iterate_phdr(find_cb, &f);
  void* p = nullptr;
  if (f.path) {
    void* h = dlopen(f.path, RTLD_NOLOAD | RTLD_LAZY);
    if (h) {
      p = ver ? dlvsym(h, name, ver) : nullptr;
      if (!p) p = real_dlsym(h, name);
      // dlopen(RTLD_NOLOAD) took a reference; the object stays loaded regardless.
      dlclose(h);
    }
  }
  if (!p) p = ver ? dlvsym(RTLD_NEXT, name, ver) : nullptr;
  if (!p) p = real_dlsym(RTLD_NEXT, name);
  if (!p) VLOG_ERROR("cannot resolve real %s in %s", name, lib_substr);
  return p;
}

}  // namespace vgpu
