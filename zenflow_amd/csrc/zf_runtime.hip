// Runtime plumbing behind the C ABI: errors, devices, memory, streams, events.
#include <cstring>
#include <mutex>

#include "zf_internal.h"

namespace zf {
static thread_local std::string g_err;

// Device -> host copies up to kStageMax go through one pinned staging
// buffer: into pageable memory HIP stages internally at a higher fixed cost
// per call (cfg1's 16 KB log_prob download: 12 us more).  A download waits
// for its DMA either way.  (Uploads stay on HIP's pageable path: staging
// them measured slower, each one waiting for the previous one's DMA.)
struct Stage {
  std::mutex mu;
  void* buf = nullptr;
  size_t cap = 0;
};
static Stage g_stage;
constexpr size_t kStageMax = size_t(4) << 20;

// Under g_stage.mu: a buffer of at least `bytes`.
static int stage_reserve(size_t bytes) {
  if (bytes > g_stage.cap) {
    if (g_stage.buf) ZF_TRY_HIP(hipHostFree(g_stage.buf));
    g_stage.buf = nullptr;
    g_stage.cap = 0;
    size_t cap = size_t(64) << 10;
    while (cap < bytes) cap *= 2;
    ZF_TRY_HIP(hipHostMalloc(&g_stage.buf, cap, hipHostMallocDefault));
    g_stage.cap = cap;
  }
  return ZF_OK;
}

void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
}
}  // namespace zf

extern "C" {

const char* zf_last_error(void) { return zf::g_err.c_str(); }

int zf_version(void) { return 1; }

int zf_device_count(int* count) {
  if (!count) return zf::einval("count is NULL");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    *count = 0;
    return zf::hip_status(e, "hipGetDeviceCount");
  }
  *count = n;
  return ZF_OK;
}

int zf_set_device(int device) { ZF_TRY_HIP(hipSetDevice(device)); return ZF_OK; }

int zf_get_device(int* device) {
  if (!device) return zf::einval("device is NULL");
  ZF_TRY_HIP(hipGetDevice(device));
  return ZF_OK;
}

int zf_device_name(int device, char* buf, int buflen) {
  if (!buf || buflen <= 0) return zf::einval("bad buffer");
  hipDeviceProp_t p;
  ZF_TRY_HIP(hipGetDeviceProperties(&p, device));
  // p.name is the marketing name from libdrm's amdgpu.ids; boxes without that
  // file report "": a generic name (the arch string follows)
  char name[64];
  if (p.name[0]) snprintf(name, sizeof(name), "%s", p.name);
  else snprintf(name, sizeof(name), "AMD GPU");
  snprintf(buf, buflen, "%s (%s, %d CUs)", name, p.gcnArchName, p.multiProcessorCount);
  return ZF_OK;
}

int zf_device_synchronize(void) { ZF_TRY_HIP(hipDeviceSynchronize()); return ZF_OK; }

int zf_malloc(void** ptr, size_t bytes) {
  if (!ptr) return zf::einval("ptr is NULL");
  *ptr = nullptr;
  if (bytes == 0) bytes = 16;  // keep a valid, freeable pointer for empty arrays
  ZF_TRY_HIP(hipMalloc(ptr, bytes));
  return ZF_OK;
}

int zf_free(void* ptr) {
  if (!ptr) return ZF_OK;
  ZF_TRY_HIP(hipFree(ptr));
  return ZF_OK;
}

int zf_memset_async(void* ptr, int value, size_t bytes, void* stream) {
  if (bytes == 0) return ZF_OK;
  ZF_TRY_HIP(hipMemsetAsync(ptr, value, bytes, (hipStream_t)stream));
  return ZF_OK;
}

int zf_memcpy_htod(void* dst, const void* src, size_t bytes, void* stream) {
  if (bytes == 0) return ZF_OK;
  ZF_TRY_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
  return ZF_OK;
}

int zf_memcpy_dtoh(void* dst, const void* src, size_t bytes, void* stream) {
  if (bytes == 0) return ZF_OK;
  if (bytes <= zf::kStageMax) {
    std::lock_guard<std::mutex> lk(zf::g_stage.mu);
    const int rc = zf::stage_reserve(bytes);
    if (rc) return rc;
    ZF_TRY_HIP(hipMemcpyAsync(zf::g_stage.buf, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream));
    ZF_TRY_HIP(hipStreamSynchronize((hipStream_t)stream));
    std::memcpy(dst, zf::g_stage.buf, bytes);
    return ZF_OK;
  }
  ZF_TRY_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream));
  return ZF_OK;
}

int zf_memcpy_dtod(void* dst, const void* src, size_t bytes, void* stream) {
  if (bytes == 0) return ZF_OK;
  ZF_TRY_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return ZF_OK;
}

int zf_stream_create(void** stream) {
  if (!stream) return zf::einval("stream is NULL");
  hipStream_t s;
  ZF_TRY_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  *stream = (void*)s;
  return ZF_OK;
}

int zf_stream_destroy(void* stream) {
  if (!stream) return ZF_OK;
  ZF_TRY_HIP(hipStreamDestroy((hipStream_t)stream));
  return ZF_OK;
}

int zf_stream_synchronize(void* stream) {
  ZF_TRY_HIP(hipStreamSynchronize((hipStream_t)stream));
  return ZF_OK;
}

int zf_event_create(void** event) {
  if (!event) return zf::einval("event is NULL");
  hipEvent_t e;
  ZF_TRY_HIP(hipEventCreate(&e));
  *event = (void*)e;
  return ZF_OK;
}

int zf_event_destroy(void* event) {
  if (!event) return ZF_OK;
  ZF_TRY_HIP(hipEventDestroy((hipEvent_t)event));
  return ZF_OK;
}

int zf_stream_wait_event(void* stream, void* event) {
  if (!event) return zf::einval("event is NULL");
  ZF_TRY_HIP(hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)event, 0));
  return ZF_OK;
}

int zf_event_record(void* event, void* stream) {
  ZF_TRY_HIP(hipEventRecord((hipEvent_t)event, (hipStream_t)stream));
  return ZF_OK;
}

int zf_event_elapsed_ms(void* start, void* stop, float* ms) {
  if (!ms) return zf::einval("ms is NULL");
  ZF_TRY_HIP(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop));
  return ZF_OK;
}

int zf_event_synchronize(void* event) {
  ZF_TRY_HIP(hipEventSynchronize((hipEvent_t)event));
  return ZF_OK;
}

}  // extern "C"
