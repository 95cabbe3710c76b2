// capi.cpp -- device plumbing and error reporting of the ti_hip.h C-ABI.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>

#include "ti_hip.h"

namespace {
thread_local std::string g_last_error;
}

int ti_set_error(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

int ti_check_hip(hipError_t e, const char* what) {
  if (e == hipSuccess) return TI_OK;
  return ti_set_error(e == hipErrorOutOfMemory ? TI_ERR_NOMEM : TI_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
}

#define CHECK(expr, what)                               \
  do {                                                  \
    hipError_t _e = (expr);                             \
    if (_e != hipSuccess) return ti_check_hip(_e, what); \
  } while (0)

extern "C" {

const char* ti_last_error(void) { return g_last_error.c_str(); }

int ti_device_count(int* count) {
  if (!count) return ti_set_error(TI_ERR_ARG, "ti_device_count: null");
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *count = n;
  return TI_OK;
}

int ti_init(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return ti_set_error(TI_ERR_NODEV, "ti_init: no HIP device visible");
  if (device < 0 || device >= n) return ti_set_error(TI_ERR_ARG, "ti_init: device %d of %d", device, n);
  CHECK(hipSetDevice(device), "hipSetDevice");
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, device), "hipGetDeviceProperties");
  if (std::strncmp(p.gcnArchName, "gfx950", 6) != 0)
    return ti_set_error(TI_ERR_NODEV, "ti_init: device %d is %s, kernels are built for gfx950", device, p.gcnArchName);
  return TI_OK;
}

int ti_device_name(int device, char* buf, int len) {
  if (!buf || len <= 0) return ti_set_error(TI_ERR_ARG, "ti_device_name: buffer");
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, device), "hipGetDeviceProperties");
  std::snprintf(buf, (size_t)len, "%s (%s, %d CUs)", p.name, p.gcnArchName, p.multiProcessorCount);
  return TI_OK;
}

int ti_malloc(void** ptr, size_t bytes) {
  if (!ptr) return ti_set_error(TI_ERR_ARG, "ti_malloc: null");
  *ptr = nullptr;
  if (bytes == 0) bytes = 16;
  CHECK(hipMalloc(ptr, bytes), "hipMalloc");
  return TI_OK;
}

int ti_free(void* ptr) {
  if (ptr) CHECK(hipFree(ptr), "hipFree");
  return TI_OK;
}

int ti_memcpy_h2d(void* dst, const void* src, size_t bytes, ti_stream_t s) {
  if (bytes == 0) return TI_OK;
  CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)s), "hipMemcpyAsync(H2D)");
  CHECK(hipStreamSynchronize((hipStream_t)s), "hipStreamSynchronize");
  return TI_OK;
}

int ti_memcpy_d2h(void* dst, const void* src, size_t bytes, ti_stream_t s) {
  if (bytes == 0) return TI_OK;
  CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)s), "hipMemcpyAsync(D2H)");
  CHECK(hipStreamSynchronize((hipStream_t)s), "hipStreamSynchronize");
  return TI_OK;
}

int ti_memcpy_d2d(void* dst, const void* src, size_t bytes, ti_stream_t s) {
  if (bytes == 0) return TI_OK;
  CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)s), "hipMemcpyAsync(D2D)");
  return TI_OK;
}

int ti_memset(void* ptr, int value, size_t bytes, ti_stream_t s) {
  if (bytes == 0) return TI_OK;
  CHECK(hipMemsetAsync(ptr, value, bytes, (hipStream_t)s), "hipMemsetAsync");
  return TI_OK;
}

int ti_stream_create(ti_stream_t* s) {
  if (!s) return ti_set_error(TI_ERR_ARG, "ti_stream_create: null");
  hipStream_t h;
  CHECK(hipStreamCreateWithFlags(&h, hipStreamNonBlocking), "hipStreamCreate");
  *s = (ti_stream_t)h;
  return TI_OK;
}

int ti_stream_destroy(ti_stream_t s) {
  if (s) CHECK(hipStreamDestroy((hipStream_t)s), "hipStreamDestroy");
  return TI_OK;
}

int ti_stream_sync(ti_stream_t s) {
  CHECK(hipStreamSynchronize((hipStream_t)s), "hipStreamSynchronize");
  return TI_OK;
}

int ti_device_sync(void) {
  CHECK(hipDeviceSynchronize(), "hipDeviceSynchronize");
  return TI_OK;
}

int ti_event_create(void** ev) {
  if (!ev) return ti_set_error(TI_ERR_ARG, "ti_event_create: null");
  hipEvent_t e;
  CHECK(hipEventCreate(&e), "hipEventCreate");
  *ev = (void*)e;
  return TI_OK;
}

int ti_event_destroy(void* ev) {
  if (ev) CHECK(hipEventDestroy((hipEvent_t)ev), "hipEventDestroy");
  return TI_OK;
}

int ti_event_record(void* ev, ti_stream_t s) {
  CHECK(hipEventRecord((hipEvent_t)ev, (hipStream_t)s), "hipEventRecord");
  return TI_OK;
}

int ti_event_elapsed_ms(void* start, void* stop, float* ms) {
  if (!ms) return ti_set_error(TI_ERR_ARG, "ti_event_elapsed_ms: null");
  CHECK(hipEventSynchronize((hipEvent_t)stop), "hipEventSynchronize");
  CHECK(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop), "hipEventElapsedTime");
  return TI_OK;
}

}  // extern "C"
