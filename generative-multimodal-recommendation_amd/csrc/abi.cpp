// C-ABI plumbing of libgmr_hip.so: error reporting and version.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include "../../include/gmr.h"

namespace gmr {
static thread_local char g_err[512] = "";

void set_error(const char* fn, const char* msg) { snprintf(g_err, sizeof(g_err), "%s: %s", fn, msg); }

int hip_status(const char* fn, hipError_t e) {
  snprintf(g_err, sizeof(g_err), "%s: HIP error %d (%s)", fn, (int)e, hipGetErrorString(e));
  return -(int)e;
}
}  // namespace gmr

extern "C" const char* gmr_last_error_string(void) { return gmr::g_err; }

extern "C" int gmr_version(void) { return GMR_ABI_VERSION; }

extern "C" int gmr_device_name(char* buf, int32_t len) {
  hipDeviceProp_t p;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipGetDeviceProperties(&p, dev);
  if (e != hipSuccess) return gmr::hip_status(__func__, e);
  snprintf(buf, (size_t)len, "%s", p.gcnArchName);
  return GMR_OK;
}

// Stream fork/join for the host layer: record `ev` on `from`, make `to` wait for it.  The
// DiffMM rec step forks and joins side streams ~17 times per step; doing it here costs one
// ctypes call instead of torch Stream/Event objects, and the step is host-issue-bound.
extern "C" int gmr_event_create(void** ev) {
  if (!ev) {
    gmr::set_error(__func__, "null pointer");
    return GMR_ERR_ARG;
  }
  hipEvent_t e = nullptr;
  const hipError_t rc = hipEventCreateWithFlags(&e, hipEventDisableTiming);
  if (rc != hipSuccess) return gmr::hip_status(__func__, rc);
  *ev = (void*)e;
  return GMR_OK;
}

extern "C" int gmr_event_destroy(void* ev) {
  if (!ev) return GMR_OK;
  const hipError_t rc = hipEventDestroy((hipEvent_t)ev);
  if (rc != hipSuccess) return gmr::hip_status(__func__, rc);
  return GMR_OK;
}

extern "C" int gmr_stream_fork(void* from, void* to, void* ev) {
  if (!ev) {
    gmr::set_error(__func__, "null event");
    return GMR_ERR_ARG;
  }
  hipError_t rc = hipEventRecord((hipEvent_t)ev, (hipStream_t)from);
  if (rc == hipSuccess) rc = hipStreamWaitEvent((hipStream_t)to, (hipEvent_t)ev, 0);
  if (rc != hipSuccess) return gmr::hip_status(__func__, rc);
  return GMR_OK;
}
