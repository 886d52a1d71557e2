// psrt_error.h — the C ABI's thread-local error message (rt_last_error).
#pragma once

namespace psrt {
// Records a printf-style message for rt_last_error() and returns `code`.
int set_error(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
// The render entries' parameter check (psrt_capi.hip): image size, spp,
// depth, shard, flags. RT_OK or RT_E_INVALID with the message set.
int check_render_params(const void* rt_params_ptr);
}  // namespace psrt
