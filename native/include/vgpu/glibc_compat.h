// Oldest-version bindings for the C library symbols the shim uses.
//
// libvgpu_hip.so is preloaded into every tenant process, so it must load with the C
// library of the tenant's image, not the one it was built against. Built against glibc
// >= 2.34, references to the pthread and dl functions bind to their GLIBC_2.34 versions
// (the release that merged libpthread and libdl into libc), which images with an older
// glibc (Ubuntu 20.04: 2.31, RHEL 8: 2.28) do not have. Every glibc since then still
// exports the original versions, so the references are pinned to them here, and the shim
// links libdl / libpthread explicitly for the older images that keep the functions there.
// stat/fstat (GLIBC_2.33) are not used at all (access / lseek / a raw newfstatat instead).
// dlsym / dlvsym / dlopen / dlmopen are not listed: the shim defines (interposes) them, in
// every version, and reaches glibc's through the C library's symbol table
// (src/shim/dlsym_hook.cpp). The reference's
// libvgpu.so was built on Ubuntu 20.04 for the same reason.
//
// Force-included (-include) into every object of the non-sanitizer build; the sanitizer
// runtimes interpose these functions themselves and are left alone. Checked by
// tests/test_native_core.py::test_shim_needs_only_old_glibc.
#pragma once
#if defined(__x86_64__) && !defined(VGPU_NO_GLIBC_COMPAT)
__asm__(".symver dlclose,dlclose@GLIBC_2.2.5");
__asm__(".symver dladdr,dladdr@GLIBC_2.2.5");
__asm__(".symver dlerror,dlerror@GLIBC_2.2.5");
__asm__(".symver dl_iterate_phdr,dl_iterate_phdr@GLIBC_2.2.5");
__asm__(".symver pthread_create,pthread_create@GLIBC_2.2.5");
__asm__(".symver pthread_once,pthread_once@GLIBC_2.2.5");
__asm__(".symver pthread_mutex_timedlock,pthread_mutex_timedlock@GLIBC_2.2.5");
__asm__(".symver pthread_mutexattr_init,pthread_mutexattr_init@GLIBC_2.2.5");
__asm__(".symver pthread_mutexattr_destroy,pthread_mutexattr_destroy@GLIBC_2.2.5");
__asm__(".symver pthread_mutexattr_setpshared,pthread_mutexattr_setpshared@GLIBC_2.2.5");
__asm__(".symver pthread_mutexattr_setrobust,pthread_mutexattr_setrobust@GLIBC_2.12");
__asm__(".symver pthread_mutex_consistent,pthread_mutex_consistent@GLIBC_2.12");
__asm__(".symver pthread_attr_init,pthread_attr_init@GLIBC_2.2.5");
__asm__(".symver pthread_attr_destroy,pthread_attr_destroy@GLIBC_2.2.5");
__asm__(".symver pthread_attr_setdetachstate,pthread_attr_setdetachstate@GLIBC_2.2.5");
__asm__(".symver pthread_atfork,pthread_atfork@GLIBC_2.2.5");
__asm__(".symver pthread_key_create,pthread_key_create@GLIBC_2.2.5");
__asm__(".symver pthread_setspecific,pthread_setspecific@GLIBC_2.2.5");
__asm__(".symver pthread_getspecific,pthread_getspecific@GLIBC_2.2.5");
__asm__(".symver pthread_detach,pthread_detach@GLIBC_2.2.5");
__asm__(".symver pthread_join,pthread_join@GLIBC_2.2.5");
#endif
