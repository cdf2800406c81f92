/*
 * rt_hip_diag.h -- exported only by the diagnostics build of librt_hip.so
 * (`make -C opencl-ray-tracer_amd/csrc RT_DIAG=1`).  The default library
 * instantiates none of the ablation kernels and exports none of these.
 * No reference counterpart; a MainState integration never calls them.
 */
#ifndef RT_HIP_DIAG_H
#define RT_HIP_DIAG_H

#include <stdint.h>

#include "rt_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Trace-kernel ablation for measurements: 0 = the real kernel, 1 = stores
 * only, 2 = no per-pixel tests, 3 = no stores, 4 = no colour gather (a
 * constant colour).  Modes 1-4 produce wrong frames by design. */
int rt_debug_set_trace_mode(rt_ctx* ctx, int mode);

/* RT_DIAG=1 RT_TIMELINE=1 builds: per-wave phase timestamps (8 x uint32 per
 * wave) into `device_buf` (scripts/timeline.py). */
int rt_debug_set_timeline(rt_ctx* ctx, void* device_buf);

#ifdef __cplusplus
}
#endif
#endif /* RT_HIP_DIAG_H */
