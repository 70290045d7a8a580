// Structured, level-gated logging for the vGPU shim.
//
// The reference shim calls getenv("LIBCUDA_LOG_LEVEL") at every log site, including
// on the kernel-launch hot path ("Per-call costs"). Here the level is
// parsed once (VGPU_LOG_LEVEL) and cached in a plain int, so a disabled log site
// costs one predictable branch.
//
// Levels: 0 = errors only, 1 = +warnings (default), 2 = +info, 3 = +debug.
#pragma once

#include <cstdio>

namespace vgpu {

enum LogLevel : int { kError = 0, kWarn = 1, kInfo = 2, kDebug = 3 };

extern int g_log_level;
void log_init_from_env();
void log_write(int level, const char* file, int line, const char* fmt, ...)
    __attribute__((format(printf, 4, 5)));

}  // namespace vgpu

#define VGPU_LOG(level, ...)                                              \
  do {                                                                    \
    if (__builtin_expect((level) <= ::vgpu::g_log_level, 0))              \
      ::vgpu::log_write((level), __FILE__, __LINE__, __VA_ARGS__);        \
  } while (0)

#define VLOG_ERROR(...) ::vgpu::log_write(::vgpu::kError, __FILE__, __LINE__, __VA_ARGS__)
#define VLOG_WARN(...) VGPU_LOG(::vgpu::kWarn, __VA_ARGS__)
#define VLOG_INFO(...) VGPU_LOG(::vgpu::kInfo, __VA_ARGS__)
#define VLOG_DEBUG(...) VGPU_LOG(::vgpu::kDebug, __VA_ARGS__)
