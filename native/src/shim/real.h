// Resolution of the real (next) definitions of interposed entry points.
//
// PyTorch loads the ROCm libraries it bundles (libamdhip64, libhsa-runtime64) from
// a Python extension opened with RTLD_LOCAL, so they are not in the global search
// scope and dlsym(RTLD_NEXT, ...) from a preloaded library cannot see them
// (measured on box: the RTLD_NEXT-only probe crashed). The resolver finds the loaded
// object by soname with dl_iterate_phdr and looks the symbol up in that object's
// own scope, which never contains the preloaded shim.
#pragma once

namespace vgpu {

// glibc's dlsym (bypassing the shim's interposer, dlsym_hook.cpp) and dlvsym.
void* real_dlsym(void* handle, const char* name);
void* real_dlvsym(void* handle, const char* name, const char* version);

// Routing of runtime lookups (gates.cpp): the shim's hook for the HIP entry point at
// `real`, or for `name` (with `version`, may be null) when the lookup found `real` - the
// entry point that hook forwards to. Null when the entry point is not hooked.
void* hip_hook_for_real(const void* real);
void* hip_hook_for_name(const char* name, const char* version, const void* real);
// The shim's own definition of ROCr entry point `name` (exported as name@ROCR_1), or null
// when the shim does not hook it (hsa_hooks.cpp).
void* hsa_hook_for_name(const char* name);

// Looks `name` (version `ver`, may be null) up in the first loaded object whose path
// contains `lib_substr`; falls back to RTLD_NEXT. Returns null when absent (logged as an
// error unless `quiet`: a runtime may lack an entry point the shim knows).
void* resolve_real(const char* lib_substr, const char* name, const char* ver, bool quiet = false);

}  // namespace vgpu

#define VGPU_REAL_AS(fn, type, lib, ver)                                                    \
  static void* real_ptr_##fn = nullptr;                                                     \
  void* real_p_##fn = __atomic_load_n(&real_ptr_##fn, __ATOMIC_ACQUIRE);                    \
  if (__builtin_expect(!real_p_##fn, 0)) {                                                  \
    real_p_##fn = ::vgpu::resolve_real(lib, #fn, ver);                                      \
    __atomic_store_n(&real_ptr_##fn, real_p_##fn, __ATOMIC_RELEASE);                        \
  }                                                                                         \
  auto real_##fn = reinterpret_cast<type>(real_p_##fn);

#define VGPU_REAL_IMPL(fn, lib, ver) VGPU_REAL_AS(fn, decltype(&fn), lib, ver)
#define VGPU_REAL_HSA(fn) VGPU_REAL_IMPL(fn, "libhsa-runtime64", "ROCR_1")
#define VGPU_REAL_HIP(fn) VGPU_REAL_IMPL(fn, "libamdhip64", nullptr)
// For HIP entry points that C++ overloads with templates (decltype is ambiguous).
#define VGPU_REAL_HIP_T(fn, type) VGPU_REAL_AS(fn, type, "libamdhip64", nullptr)
