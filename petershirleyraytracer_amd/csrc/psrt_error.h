// psrt_error.h — the C ABI's thread-local error message (rt_last_error).
#pragma once

namespace psrt {
// Records a printf-style message for rt_last_error() and returns `code`.
int set_error(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
}  // namespace psrt
