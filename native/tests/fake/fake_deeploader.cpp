// A library that dlopens by bare file name, relying on its own RUNPATH ($ORIGIN) - the
// situation in which the shim's DEEPBIND handling must keep the caller's search path
// (tests/test_loader_bypass.py).
#include <dlfcn.h>
#include <stdio.h>

extern "C" void* deep_open(const char* name, int mode) {
  void* h = dlopen(name, mode);
  if (!h) fprintf(stderr, "deep_open(%s): %s\n", name, dlerror());
  return h;
}
