// Local definitions for the three C library symbols that the statically linked libstdc++
// references at versions newer than the oldest glibc the shim supports (glibc_compat.h):
//   __libc_single_threaded  GLIBC_2.32  libstdc++'s "is this process single-threaded"
//                                       shortcut; 0 = always use atomics (the shim lives
//                                       in multi-threaded processes anyway)
//   pthread_once            GLIBC_2.34  std::call_once
//   __pthread_key_create    GLIBC_2.34  libstdc++'s "are threads in use" probe
// They are hidden, so only the shim's own copy of libstdc++ binds to them (at static
// link time); each forwards to the C library's original version. This file is built
// without the force-included glibc_compat.h (it defines, not references, pthread_once).
#include <pthread.h>

extern "C" {

int vgpu_real_pthread_once(pthread_once_t* once, void (*fn)(void));
int vgpu_real_pthread_key_create(pthread_key_t* key, void (*dtor)(void*));
__asm__(".symver vgpu_real_pthread_once,pthread_once@GLIBC_2.2.5");
__asm__(".symver vgpu_real_pthread_key_create,pthread_key_create@GLIBC_2.2.5");

__attribute__((visibility("hidden"))) char __libc_single_threaded = 0;

__attribute__((visibility("hidden"))) int pthread_once(pthread_once_t* once, void (*fn)(void)) {
  return vgpu_real_pthread_once(once, fn);
}

__attribute__((visibility("hidden"))) int __pthread_key_create(pthread_key_t* key, void (*dtor)(void*)) {
  return vgpu_real_pthread_key_create(key, dtor);
}

}  // extern "C"
