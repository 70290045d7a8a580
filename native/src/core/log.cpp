#include "vgpu/log.h"

#include <sys/syscall.h>
#include <unistd.h>

#include <cstdarg>
#include <cstdlib>
#include <cstring>

namespace vgpu {

int g_log_level = kWarn;

void log_init_from_env() {
  const char* s = getenv("VGPU_LOG_LEVEL");
  if (!s || !*s) s = getenv("LIBCUDA_LOG_LEVEL");  // reference name (README.md:224-234)
  if (s && *s) g_log_level = atoi(s);
}

void log_write(int level, const char* file, int line, const char* fmt, ...) {
  static const char* const kNames[] = {"ERROR", "WARN", "INFO", "DEBUG"};
  const char* name = kNames[level < 0 ? 0 : (level > 3 ? 3 : level)];
  const char* base = strrchr(file, '/');
  base = base ? base + 1 : file;
  char buf[1024];
  int n = snprintf(buf, sizeof(buf), "[vGPU %s(%d:%ld:%s:%d)]: ", name, (int)getpid(),
                   (long)syscall(SYS_gettid), base, line);
  if (n < 0) return;
  va_list ap;
  va_start(ap, fmt);
  int m = vsnprintf(buf + n, sizeof(buf) - (size_t)n - 1, fmt, ap);
  va_end(ap);
  if (m < 0) return;
  size_t len = strlen(buf);
  if (len == 0 || buf[len - 1] != '\n') {
    buf[len] = '\n';
    buf[len + 1] = 0;
    len++;
  }
  ssize_t w = write(2, buf, len);
  (void)w;
}

}  // namespace vgpu
