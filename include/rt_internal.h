/*
 * rt_internal.h -- shared between the library's own translation units
 * (rt_device.hip, rt_scene_device.hip).  Not installed, not part of the ABI.
 */
#ifndef RT_INTERNAL_H
#define RT_INTERNAL_H

#include <hip/hip_runtime.h>

#include "rt_hip.h"

namespace rt_internal {
int ctx_device(const rt_ctx* ctx);
// the context's own stream, created on first use (nullptr if that fails):
// a context used only with caller streams never takes a hardware queue
hipStream_t ctx_stream(rt_ctx* ctx);
// load rt_scene_device.hip's kernels onto the current device (rt_init)
int preload_scene_kernels();
}  // namespace rt_internal

#endif /* RT_INTERNAL_H */
