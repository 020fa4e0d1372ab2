// C-ABI plumbing: version, thread-local error string.
#include <stdarg.h>
#include "ncf_common.h"

static thread_local char g_err[512] = "";

void ncf_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

extern "C" const char* ncf_last_error(void) { return g_err; }

extern "C" int ncf_version(void) { return 10000; }  // 1.0.0

// Build identity (build_ext.sh passes both hashes for this file: _abi.py)
#ifndef NCF_ABI_HASH
#define NCF_ABI_HASH "unset"
#endif
#ifndef NCF_SRC_HASH
#define NCF_SRC_HASH "unset"
#endif
extern "C" const char* ncf_build_info(void) { return "abi=" NCF_ABI_HASH " src=" NCF_SRC_HASH; }

// Sanity probe used by the loader: returns the HIP device count seen by the runtime the
// library is bound to (torch's libamdhip64 when torch is imported first).
extern "C" int ncf_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// Cross-stream ordering through the C-ABI (the fork / join points of a step: the id sort beside
// the forward, the overlapped sweep): the same hipEventRecord / hipStreamWaitEvent torch's Event
// would issue, as entry points, so a recorded launch sequence (the fast-call binding's launch
// tape) replays them in order with the kernels.
extern "C" int ncf_event_create(void** event) {
  if (!event) { ncf_set_error("ncf_event_create: NULL out pointer"); return NCF_ERR_ARG; }
  hipEvent_t e = nullptr;
  hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableTiming);
  if (r != hipSuccess) { ncf_set_error("hipEventCreateWithFlags: %s", hipGetErrorString(r)); return NCF_ERR_LAUNCH; }
  *event = (void*)e;
  return NCF_OK;
}

extern "C" int ncf_event_create_scoped(void** event, int32_t scope) {
  if (!event) { ncf_set_error("ncf_event_create_scoped: NULL out pointer"); return NCF_ERR_ARG; }
  if (scope < 0 || scope > 2) { ncf_set_error("ncf_event_create_scoped: scope must be 0, 1 or 2"); return NCF_ERR_ARG; }
  const unsigned flags = hipEventDisableTiming | (scope == 1   ? hipEventReleaseToDevice
                                                  : scope == 2 ? hipEventDisableSystemFence
                                                               : 0u);
  hipEvent_t e = nullptr;
  hipError_t r = hipEventCreateWithFlags(&e, flags);
  if (r != hipSuccess) { ncf_set_error("hipEventCreateWithFlags: %s", hipGetErrorString(r)); return NCF_ERR_LAUNCH; }
  *event = (void*)e;
  return NCF_OK;
}

extern "C" int ncf_event_destroy(void* event) {
  if (!event) return NCF_OK;
  hipError_t r = hipEventDestroy((hipEvent_t)event);
  if (r != hipSuccess) { ncf_set_error("hipEventDestroy: %s", hipGetErrorString(r)); return NCF_ERR_LAUNCH; }
  return NCF_OK;
}

extern "C" int ncf_event_record(void* event, void* stream) {
  if (!event) { ncf_set_error("ncf_event_record: NULL event"); return NCF_ERR_ARG; }
  hipError_t r = hipEventRecord((hipEvent_t)event, (hipStream_t)stream);
  if (r != hipSuccess) { ncf_set_error("hipEventRecord: %s", hipGetErrorString(r)); return NCF_ERR_LAUNCH; }
  return NCF_OK;
}

extern "C" int ncf_stream_wait_event(void* stream, void* event) {
  if (!event) { ncf_set_error("ncf_stream_wait_event: NULL event"); return NCF_ERR_ARG; }
  hipError_t r = hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)event, 0);
  if (r != hipSuccess) { ncf_set_error("hipStreamWaitEvent: %s", hipGetErrorString(r)); return NCF_ERR_LAUNCH; }
  return NCF_OK;
}

// Host wait for an event (the row-sharded step's split sizes: RCCL takes them on the host).
extern "C" int ncf_event_synchronize(void* event) {
  if (!event) { ncf_set_error("ncf_event_synchronize: NULL event"); return NCF_ERR_ARG; }
  hipError_t r = hipEventSynchronize((hipEvent_t)event);
  if (r != hipSuccess) { ncf_set_error("hipEventSynchronize: %s", hipGetErrorString(r)); return NCF_ERR_LAUNCH; }
  return NCF_OK;
}

// Stream-ordered copy of `bytes` (device <-> device or device -> pinned host), so it can sit in a
// recorded launch sequence.
extern "C" int ncf_memcpy_async(void* dst, const void* src, int64_t bytes, void* stream) {
  if (bytes < 0 || (bytes > 0 && (!dst || !src))) { ncf_set_error("ncf_memcpy_async: bad arguments"); return NCF_ERR_ARG; }
  if (bytes == 0) return NCF_OK;
  hipError_t r = hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDefault, (hipStream_t)stream);
  if (r != hipSuccess) { ncf_set_error("hipMemcpyAsync: %s", hipGetErrorString(r)); return NCF_ERR_LAUNCH; }
  return NCF_OK;
}

// A one-wavefront kernel that waits `microseconds` of wall-clock time on `stream` (the
// side-stream overlap probe: two of them on two streams finish in about one span when the
// streams reach the GPU through different hardware queues, in two when they share one).
// Every wave leaves once the span has passed (bounded by the argument check: at most 1 s).
__global__ void k_stream_spin(int64_t ticks) {
  const int64_t t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

extern "C" int ncf_stream_spin(int64_t microseconds, void* stream) {
  NCF_CHECK_ARG(microseconds >= 0 && microseconds <= 1000000,
                "ncf_stream_spin: microseconds in [0, 1e6]");
  static int rate_khz = 0;
  if (rate_khz <= 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess ||
        rate_khz <= 0)
      rate_khz = 100000;   // (the 100 MHz constant clock of CDNA3/4)
  }
  const int64_t ticks = microseconds * (int64_t)rate_khz / 1000;
  hipLaunchKernelGGL(k_stream_spin, dim3(1), dim3(64), 0, (hipStream_t)stream, ticks);
  NCF_CHECK_LAUNCH("ncf_stream_spin");
  return NCF_OK;
}

// A stream whose kernels run only on `keep_per8` of every 8 compute units (the CUs whose index
// mod 8 is below it; hipExtStreamCreateWithCUMask): side work such as the rolling table sweep
// then leaves the other CUs to the step's kernels (A/B knob, deferred.SIDE_CU_KEEP).  A
// CU-masked stream gets a hardware queue of its own.  Destroy with ncf_stream_destroy.
extern "C" int ncf_stream_create_cu_mask(int32_t keep_per8, void** out) {
  NCF_CHECK_ARG(out && keep_per8 >= 1 && keep_per8 <= 8, "ncf_stream_create_cu_mask: bad args");
  int dev = 0;
  (void)hipGetDevice(&dev);
  int n = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) {
    ncf_set_error("ncf_stream_create_cu_mask: no CU count");
    return NCF_ERR_LAUNCH;
  }
  uint32_t mask[32] = {0};
  const int words = (n + 31) / 32;
  NCF_CHECK_ARG(words <= 32, "ncf_stream_create_cu_mask: more than 1024 CUs");
  for (int i = 0; i < n; ++i)
    if (i % 8 < keep_per8) mask[i / 32] |= 1u << (i % 32);
  hipStream_t s = nullptr;
  const hipError_t r = hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask);
  if (r != hipSuccess) {
    ncf_set_error("hipExtStreamCreateWithCUMask: %s", hipGetErrorString(r));
    return NCF_ERR_LAUNCH;
  }
  *out = (void*)s;
  return NCF_OK;
}

extern "C" int ncf_stream_destroy(void* stream) {
  if (!stream) return NCF_OK;
  const hipError_t r = hipStreamDestroy((hipStream_t)stream);
  if (r != hipSuccess) {
    ncf_set_error("hipStreamDestroy: %s", hipGetErrorString(r));
    return NCF_ERR_LAUNCH;
  }
  return NCF_OK;
}
