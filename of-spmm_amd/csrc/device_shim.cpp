// device_shim.cpp — the ep device layer reduced to a thin C-ABI over the HIP runtime.
//
// Replaces, for this op only: ep::Device (oneflow/core/ep/include/device.h:33-62; 512-B
// alignment requirement device.h:29), ep::Stream / CudaStream (stream.h:30-49,
// oneflow/core/ep/cuda/cuda_stream.cpp:90-142), ep::Event (event.h:26-34),
// primitive::Memcpy (memcpy.h:33-39) and primitive::Memset (memset.h:26-32).
// There is no device-manager registry: one process drives one GPU.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstring>
#include <mutex>

#include "ofx_internal.h"

// ---- device-side error words ------------------------------------------------------------------
// Kernels report a loud failure (a work-list plan that gave up, a planned launch over a workspace
// holding no valid plan; spmm_plan.h) by storing 1 into one of these host-mapped words; the
// next launching entry, stream / event / device sync and graph launch report it as OFX_EPLAN and
// clear it.  Allocated once per process (portable: any device may write it), on first use, with
// the capture mode relaxed so that a first call inside a stream capture can still allocate.
namespace {
constexpr int kErrWords = 16;  // 64 B: [0] plan gave up, [1] launch found no valid plan
std::atomic<unsigned*> g_err_words{nullptr};  // host address (set last)
unsigned* g_err_dev = nullptr;                 // device address of the same words
std::once_flag g_err_once;
}  // namespace

namespace ofx {
unsigned* device_error_words() {
  std::call_once(g_err_once, [] {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
      (void)hipGetLastError();
      return;
    }
    hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
    (void)hipThreadExchangeStreamCaptureMode(&mode);
    void* p = nullptr;
    const hipError_t e =
        hipHostMalloc(&p, kErrWords * sizeof(unsigned), hipHostMallocMapped | hipHostMallocPortable);
    if (e != hipSuccess) {
      (void)hipThreadExchangeStreamCaptureMode(&mode);
      (void)hipGetLastError();
      return;
    }
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess || d == nullptr) {
      (void)hipGetLastError();
      d = p;  // one address space for host-mapped memory on this platform
    }
    (void)hipThreadExchangeStreamCaptureMode(&mode);
    std::memset(p, 0, kErrWords * sizeof(unsigned));
    g_err_dev = static_cast<unsigned*>(d);
    g_err_words.store(static_cast<unsigned*>(p), std::memory_order_release);
  });
  return g_err_words.load(std::memory_order_acquire) ? g_err_dev : nullptr;
}

int take_device_error(const char* where) {
  unsigned* w = g_err_words.load(std::memory_order_acquire);
  if (w == nullptr) return OFX_OK;  // nothing was ever launched that could raise one
  volatile unsigned* vw = w;
  const unsigned failed = vw[0], invalid = vw[1];
  if (!failed && !invalid) return OFX_OK;
  vw[0] = 0;
  vw[1] = 0;
  return fail(OFX_EPLAN,
              "%s: an earlier launch failed: %s (reported at the next call, process-wide; its "
              "output was filled with quiet NaN)",
              where,
              failed ? "its device-side work-list plan gave up waiting for a predecessor block "
                       "(look-back spin limit)"
                     : "it found no valid work-list plan in its workspace (a failed plan, or "
                       "options.planned over a workspace ofx_spmm_csr_plan did not fill)");
}
}  // namespace ofx

extern "C" int ofx_device_error_check(void) {
  return ofx::guarded(__func__, [&]() -> int { return ofx::take_device_error("device_error_check"); });
}

extern "C" int ofx_device_count(int* count) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(count, OFX_EINVAL, "device_count: NULL");
    OFX_HIP_CHECK(hipGetDeviceCount(count));
    return OFX_OK;
  });
}
extern "C" int ofx_set_device(int device) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_HIP_CHECK(hipSetDevice(device));
    return OFX_OK;
  });
}
extern "C" int ofx_get_device(int* device) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(device, OFX_EINVAL, "get_device: NULL");
    OFX_HIP_CHECK(hipGetDevice(device));
    return OFX_OK;
  });
}
extern "C" int ofx_device_synchronize(void) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_HIP_CHECK(hipDeviceSynchronize());
    OFX_TAKE_DEVICE_ERROR("device_synchronize");
    return OFX_OK;
  });
}
extern "C" int ofx_malloc(void** ptr, size_t bytes) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(ptr, OFX_EINVAL, "malloc: NULL");
    *ptr = nullptr;
    if (bytes == 0) return OFX_OK;
    hipError_t e = hipMalloc(ptr, (bytes + 511) / 512 * 512);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      return ofx::fail(OFX_ENOMEM, "hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
    }
    return OFX_OK;
  });
}
extern "C" int ofx_free(void* ptr) {
  return ::ofx::guarded(__func__, [&]() -> int {
    if (ptr) OFX_HIP_CHECK(hipFree(ptr));
    return OFX_OK;
  });
}
extern "C" int ofx_host_malloc(void** ptr, size_t bytes) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(ptr, OFX_EINVAL, "host_malloc: NULL");
    OFX_HIP_CHECK(hipHostMalloc(ptr, bytes ? bytes : 1, hipHostMallocDefault));
    return OFX_OK;
  });
}
extern "C" int ofx_host_free(void* ptr) {
  return ::ofx::guarded(__func__, [&]() -> int {
    if (ptr) OFX_HIP_CHECK(hipHostFree(ptr));
    return OFX_OK;
  });
}
extern "C" int ofx_stream_create(void** stream) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(stream, OFX_EINVAL, "stream_create: NULL");
    hipStream_t s;
    OFX_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    *stream = s;
    return OFX_OK;
  });
}
extern "C" int ofx_stream_destroy(void* stream) {
  return ::ofx::guarded(__func__, [&]() -> int {
    if (stream) OFX_HIP_CHECK(hipStreamDestroy(static_cast<hipStream_t>(stream)));
    return OFX_OK;
  });
}
extern "C" int ofx_stream_sync(void* stream) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_HIP_CHECK(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
    OFX_TAKE_DEVICE_ERROR("stream_sync");
    return OFX_OK;
  });
}
extern "C" int ofx_memcpy_async(void* stream, void* dst, const void* src, size_t bytes, int kind) {
  return ::ofx::guarded(__func__, [&]() -> int {
    if (bytes == 0) return OFX_OK;
    hipMemcpyKind k;
    switch (kind) {
      case OFX_MEMCPY_H2D: k = hipMemcpyHostToDevice; break;
      case OFX_MEMCPY_D2H: k = hipMemcpyDeviceToHost; break;
      case OFX_MEMCPY_D2D: k = hipMemcpyDeviceToDevice; break;
      case OFX_MEMCPY_DEFAULT: k = hipMemcpyDefault; break;
      default: return ofx::fail(OFX_EINVAL, "memcpy_async: bad kind %d", kind);
    }
    OFX_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, k, static_cast<hipStream_t>(stream)));
    return OFX_OK;
  });
}
extern "C" int ofx_memset_async(void* stream, void* dst, int value, size_t bytes) {
  return ::ofx::guarded(__func__, [&]() -> int {
    if (bytes == 0) return OFX_OK;
    OFX_HIP_CHECK(hipMemsetAsync(dst, value, bytes, static_cast<hipStream_t>(stream)));
    return OFX_OK;
  });
}
extern "C" int ofx_event_create(void** event, int timing) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(event, OFX_EINVAL, "event_create: NULL");
    hipEvent_t e;
    OFX_HIP_CHECK(hipEventCreateWithFlags(&e, timing ? hipEventDefault : hipEventDisableTiming));
    *event = e;
    return OFX_OK;
  });
}
extern "C" int ofx_event_destroy(void* event) {
  return ::ofx::guarded(__func__, [&]() -> int {
    if (event) OFX_HIP_CHECK(hipEventDestroy(static_cast<hipEvent_t>(event)));
    return OFX_OK;
  });
}
extern "C" int ofx_event_record(void* event, void* stream) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_HIP_CHECK(hipEventRecord(static_cast<hipEvent_t>(event), static_cast<hipStream_t>(stream)));
    return OFX_OK;
  });
}
extern "C" int ofx_event_sync(void* event) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_HIP_CHECK(hipEventSynchronize(static_cast<hipEvent_t>(event)));
    OFX_TAKE_DEVICE_ERROR("event_sync");
    return OFX_OK;
  });
}
extern "C" int ofx_event_elapsed_ms(void* start, void* end, float* ms) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(ms, OFX_EINVAL, "event_elapsed_ms: NULL");
    OFX_HIP_CHECK(hipEventElapsedTime(ms, static_cast<hipEvent_t>(start),
                                      static_cast<hipEvent_t>(end)));
    return OFX_OK;
  });
}
extern "C" int ofx_stream_wait_event(void* stream, void* event) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_HIP_CHECK(hipStreamWaitEvent(static_cast<hipStream_t>(stream),
                                     static_cast<hipEvent_t>(event), 0));
    return OFX_OK;
  });
}

// ---- hipGraph executable + stream capture ----------------------------------------------------
// ep::CudaGraphExecutable (oneflow/core/ep/cuda/cuda_stream.h:41-56, cuda_stream.cpp:49-80):
// Update() first tries hipGraphExecUpdate on the live executable (same topology, new kernel
// arguments) and re-instantiates only when the update is refused.  CudaStream's
// BeginGraphCapture / EndGraphCapture / LaunchGraph (cuda_stream.cpp:178-196) capture in
// thread-local mode, so other host threads keep launching eagerly meanwhile.
namespace {
struct GraphExec {
  hipGraphExec_t exec = nullptr;
  int device = -1;
  int64_t instantiations = 0;  // full hipGraphInstantiate calls
  int64_t updates = 0;         // in-place hipGraphExecUpdate successes
  int64_t launches = 0;
};
}  // namespace

extern "C" int ofx_graph_exec_create(void** exec) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(exec, OFX_EINVAL, "graph_exec_create: NULL");
    *exec = new GraphExec();
    return OFX_OK;
  });
}
extern "C" int ofx_graph_exec_destroy(void* exec) {
  return ::ofx::guarded(__func__, [&]() -> int {
    GraphExec* g = static_cast<GraphExec*>(exec);
    if (!g) return OFX_OK;
    if (g->exec) {
      int cur = -1;
      OFX_HIP_CHECK(hipGetDevice(&cur));
      if (g->device >= 0 && g->device != cur) OFX_HIP_CHECK(hipSetDevice(g->device));
      const hipError_t e = hipGraphExecDestroy(g->exec);
      if (g->device >= 0 && g->device != cur) (void)hipSetDevice(cur);
      if (e != hipSuccess) {
        (void)hipGetLastError();
        delete g;
        return ofx::fail(OFX_EDEVICE, "hipGraphExecDestroy: %s", hipGetErrorString(e));
      }
    }
    delete g;
    return OFX_OK;
  });
}
extern "C" int ofx_graph_exec_stats(void* exec, int* instantiated, int64_t* instantiations,
                                    int64_t* updates, int64_t* launches) {
  return ::ofx::guarded(__func__, [&]() -> int {
    const GraphExec* g = static_cast<const GraphExec*>(exec);
    OFX_REQUIRE(g, OFX_EINVAL, "graph_exec_stats: NULL executable");
    if (instantiated) *instantiated = g->exec != nullptr;
    if (instantiations) *instantiations = g->instantiations;
    if (updates) *updates = g->updates;
    if (launches) *launches = g->launches;
    return OFX_OK;
  });
}
extern "C" int ofx_stream_begin_capture(void* stream) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(stream, OFX_EINVAL, "stream_begin_capture: the null stream cannot be captured");
    OFX_HIP_CHECK(hipStreamBeginCapture(static_cast<hipStream_t>(stream),
                                        hipStreamCaptureModeThreadLocal));
    return OFX_OK;
  });
}
extern "C" int ofx_stream_is_capturing(void* stream, int* capturing) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(capturing, OFX_EINVAL, "stream_is_capturing: NULL");
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    OFX_HIP_CHECK(hipStreamIsCapturing(static_cast<hipStream_t>(stream), &st));
    *capturing = st != hipStreamCaptureStatusNone;
    return OFX_OK;
  });
}
extern "C" int ofx_stream_end_capture(void* stream, void* exec) {
  return ::ofx::guarded(__func__, [&]() -> int {
    GraphExec* g = static_cast<GraphExec*>(exec);
    hipGraph_t graph = nullptr;
    const hipError_t ec = hipStreamEndCapture(static_cast<hipStream_t>(stream), &graph);
    if (ec != hipSuccess || graph == nullptr) {  // capture invalidated by an unsupported call
      (void)hipGetLastError();
      if (graph) (void)hipGraphDestroy(graph);
      return ofx::fail(OFX_EDEVICE, "hipStreamEndCapture: %s", hipGetErrorString(ec));
    }
    if (!g) {  // capture discarded on request (an error path of the caller)
      OFX_HIP_CHECK(hipGraphDestroy(graph));
      return OFX_OK;
    }
    int rc = OFX_OK;
    bool done = false;
    if (g->exec) {
      hipGraphExecUpdateResult res = hipGraphExecUpdateError;
      hipGraphNode_t err_node = nullptr;
      const hipError_t eu = hipGraphExecUpdate(g->exec, graph, &err_node, &res);
      if (eu == hipSuccess && res == hipGraphExecUpdateSuccess) {
        ++g->updates;
        done = true;
      } else {
        (void)hipGetLastError();
        (void)hipGraphExecDestroy(g->exec);
        g->exec = nullptr;
      }
    }
    if (!done) {
      const hipError_t ei = hipGraphInstantiate(&g->exec, graph, nullptr, nullptr, 0);
      if (ei != hipSuccess) {
        (void)hipGetLastError();
        g->exec = nullptr;
        rc = ofx::fail(OFX_EDEVICE, "hipGraphInstantiate: %s", hipGetErrorString(ei));
      } else {
        ++g->instantiations;
        (void)hipGetDevice(&g->device);
      }
    }
    const hipError_t ed = hipGraphDestroy(graph);
    if (rc == OFX_OK && ed != hipSuccess)
      return ofx::fail(OFX_EDEVICE, "hipGraphDestroy: %s", hipGetErrorString(ed));
    return rc;
  });
}
extern "C" int ofx_graph_launch(void* exec, void* stream) {
  return ::ofx::guarded(__func__, [&]() -> int {
    GraphExec* g = static_cast<GraphExec*>(exec);
    OFX_REQUIRE(g && g->exec, OFX_EINVAL, "graph_launch: executable not instantiated");
    OFX_TAKE_DEVICE_ERROR("graph_launch");  // a replay after a failed one is not silent
    OFX_HIP_CHECK(hipGraphLaunch(g->exec, static_cast<hipStream_t>(stream)));
    ++g->launches;
    return OFX_OK;
  });
}
