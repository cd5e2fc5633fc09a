// host_stage_hip.h -- the pageable bounce ring (host_stage.h) bound to HIP: one page-locked
// arena from hipHostMalloc, DMAs with hipMemcpyAsync on the pipeline's streams, one
// timing-free event per part in flight.
#pragma once
#include <hip/hip_runtime.h>

#include "host_stage.h"

namespace mipgpu {

struct HipStageDev {
  using Err = hipError_t;
  using Stream = hipStream_t;
  using Event = hipEvent_t;
  static constexpr Err kOk = hipSuccess;
  static constexpr Err kNotReady = hipErrorNotInitialized;
  Err host_alloc(char **p, size_t n, bool numa_user) {
    return hipHostMalloc((void **)p, n, numa_user ? hipHostMallocNumaUser : hipHostMallocDefault);
  }
  void host_free(char *p) { (void)hipHostFree(p); }
  Err event_create(Event *e) { return hipEventCreateWithFlags(e, hipEventDisableTiming); }
  void event_destroy(Event e) { (void)hipEventDestroy(e); }
  Err copy_h2d(void *dev, const void *host, size_t n, Stream s) {
    return hipMemcpyAsync(dev, host, n, hipMemcpyHostToDevice, s);
  }
  Err copy_d2h(void *host, const void *dev, size_t n, Stream s) {
    return hipMemcpyAsync(host, dev, n, hipMemcpyDeviceToHost, s);
  }
  Err record(Event e, Stream s) { return hipEventRecord(e, s); }
  Err sync(Event e) { return hipEventSynchronize(e); }
  void bind_thread(int device) { (void)hipSetDevice(device); }
};

using HostStage = BounceRing<HipStageDev>;

// Page-locked host memory (mip_host_alloc / hipHostRegister) or device memory: transfers
// run at DMA rate without staging.
inline bool host_pinned(const void *p) {
  hipPointerAttribute_t at{};
  const hipError_t e = hipPointerGetAttributes(&at, p);
  if (e != hipSuccess) {
    (void)hipGetLastError();  // unregistered host memory reports an error: clear it
    return false;
  }
  return at.type == hipMemoryTypeHost || at.type == hipMemoryTypeDevice || at.type == hipMemoryTypeManaged;
}

}  // namespace mipgpu
