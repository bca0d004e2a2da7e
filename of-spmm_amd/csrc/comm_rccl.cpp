// comm_rccl.cpp — RCCL all-gather of the dense matrix for the row-split operator.
//
// Replaces ccl::AllGather (oneflow/user/kernels/collective_communication/include/all_gather.h:24-38)
// and its CUDA implementation CudaAllGather::Launch -> ncclAllGather
// (oneflow/user/kernels/collective_communication/cuda/cuda_all_gather.cpp:25-47), plus the comm
// bootstrap of EagerNcclCommMgr::CreateNcclComm (oneflow/core/job/eager_nccl_comm_manager.cpp:57-80):
// rank 0 creates the unique id; the caller moves its 128 bytes to the other ranks (the reference
// uses its gRPC ctrl KV; we use the torch.distributed store) and every rank calls init.
// dtype map as oneflow/core/device/nccl_util.h:37-60.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <memory>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>

#include "ofx_internal.h"
#include "spmm_common.h"

// A call on a communicator.  Communicators made by ofx_comm_init_rank_deadline are non-blocking
// (ncclConfig_t.blocking = 0): any call on them may return ncclInProgress, and the operation is
// then complete once ncclCommGetAsyncError stops reporting ncclInProgress (comm_wait, bounded by
// the communicator's deadline).  Blocking communicators return ncclSuccess or an error.
#define OFX_NCCL_CHECK(expr)                                                                   \
  do {                                                                                         \
    ncclResult_t ofx_r_ = (expr);                                                              \
    if (ofx_r_ != ncclSuccess)                                                                 \
      return ::ofx::fail(OFX_ECOMM, "%s failed: %s (%s:%d)", #expr, ncclGetErrorString(ofx_r_), \
                         __FILE__, __LINE__);                                                  \
  } while (0)
#define OFX_NCCL_CALL(comm, expr)                                                              \
  do {                                                                                         \
    const int ofx_rc_ = comm_wait((comm), (expr), #expr);                                      \
    if (ofx_rc_ != OFX_OK) return ofx_rc_;                                                     \
  } while (0)
// The communicator behind a handle, or OFX_ECOMM if it was aborted (its NCCL object is gone).
// The entry holds an EnqueueGuard for its whole body: an abort from another thread
// (a watchdog) meanwhile only marks the communicator, and ncclCommAbort runs when the last entry
// using it returns, so no enqueue ever reaches a freed communicator.
#define OFX_LIVE_COMM(h, fn)                                                                   \
  OfxComm* ofx_cm_ = static_cast<OfxComm*>(h);                                                 \
  OFX_REQUIRE(ofx_cm_ != nullptr, OFX_EINVAL, "%s: NULL communicator", fn);                     \
  EnqueueGuard ofx_eg_(ofx_cm_);                                                               \
  OFX_REQUIRE(!ofx_cm_->aborted.load(), OFX_ECOMM, "%s: the communicator was aborted (%s)", fn, \
              ofx_cm_->why.c_str());                                                           \
  ncclComm_t c = ofx_cm_->nccl
// Between ncclGroupStart and ncclGroupEnd a call only records its operation: ncclInProgress
// there is not waited for (the group's ncclGroupEnd is, through OFX_NCCL_CALL).
#define OFX_NCCL_GROUPED(expr)                                                                 \
  do {                                                                                         \
    ncclResult_t ofx_r_ = (expr);                                                              \
    if (ofx_r_ != ncclSuccess && ofx_r_ != ncclInProgress)                                     \
      return ::ofx::fail(OFX_ECOMM, "%s failed: %s (%s:%d)", #expr, ncclGetErrorString(ofx_r_), \
                         __FILE__, __LINE__);                                                  \
  } while (0)

static_assert(sizeof(ncclUniqueId) <= OFX_UNIQUE_ID_BYTES, "unique id does not fit");

namespace {
bool nccl_dtype(int dt, ncclDataType_t* out) {
  switch (dt) {
    case OFX_DT_FLOAT: *out = ncclFloat32; return true;
    case OFX_DT_DOUBLE: *out = ncclFloat64; return true;
    case OFX_DT_INT32: *out = ncclInt32; return true;
    case OFX_DT_INT64: *out = ncclInt64; return true;
    case OFX_DT_FLOAT16: *out = ncclFloat16; return true;
    case OFX_DT_BFLOAT16: *out = ncclBfloat16; return true;
    default: return false;
  }
}

double seconds_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

// The handle behind `void* comm`: the NCCL communicator with its own deadlines and an
// aborted flag.  An abort (a deadline expiring, or ofx_comm_abort from a watchdog) frees the NCCL
// object at once and leaves the handle alive: every later call returns OFX_ECOMM naming why, and
// ofx_comm_destroy only frees the handle, so nothing touches the freed communicator.  `mu`
// serialises an abort against a poll of the same communicator from another thread; `entries`
// counts the C-ABI calls using the NCCL object (EnqueueGuard), and an abort while any is inside
// only sets `aborted` (those calls see it and return OFX_ECOMM): ncclCommAbort then runs when the
// last of them leaves.
struct OfxComm {
  ncclComm_t nccl = nullptr;
  double call_timeout_s = 300.0;  // a call left ncclInProgress (non-blocking communicators)
  double device_timeout_s = 0.0;  // the exchange's completion on the device; 0 = not waited for
  std::mutex mu;
  std::atomic<bool> aborted{false};
  std::string why;
  int entries = 0;             // calls inside (under mu)
  bool abort_pending = false;  // aborted while entries > 0: ncclCommAbort at the last exit
  int* barrier_word = nullptr;  // device int of the stream-ordered barrier (ofx_allgather_pull)

  ~OfxComm() {
    if (barrier_word != nullptr) (void)hipFree(barrier_word);
  }

  // ncclCommAbort once (deferred while a call is inside); the caller holds no lock
  void abort(const std::string& reason) {
    std::lock_guard<std::mutex> lock(mu);
    if (aborted.load()) return;
    why = reason;
    aborted.store(true);
    if (entries > 0) {
      abort_pending = true;
      return;
    }
    (void)ncclCommAbort(nccl);
    nccl = nullptr;
  }
  void enter() {
    std::lock_guard<std::mutex> lock(mu);
    ++entries;
  }
  void leave() {
    std::lock_guard<std::mutex> lock(mu);
    if (--entries == 0 && abort_pending) {
      abort_pending = false;
      (void)ncclCommAbort(nccl);
      nccl = nullptr;
    }
  }
};

// A C-ABI call using a communicator's NCCL object (OFX_LIVE_COMM).
struct EnqueueGuard {
  OfxComm* cm;
  explicit EnqueueGuard(OfxComm* c) : cm(c) { cm->enter(); }
  ~EnqueueGuard() { cm->leave(); }
  EnqueueGuard(const EnqueueGuard&) = delete;
  EnqueueGuard& operator=(const EnqueueGuard&) = delete;
};

// Completes a call that returned ncclInProgress (non-blocking communicator): polls the
// communicator's state until it leaves ncclInProgress, or aborts it after the communicator's call
// timeout so that peers blocked on this rank fail as well instead of hanging.
int comm_wait(OfxComm* cm, ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return OFX_OK;
  if (r != ncclInProgress)
    return ofx::fail(OFX_ECOMM, "%s failed: %s", what, ncclGetErrorString(r));
  const auto t0 = std::chrono::steady_clock::now();
  ncclResult_t st = ncclInProgress;
  while (true) {
    {
      std::lock_guard<std::mutex> lock(cm->mu);
      if (cm->aborted.load())
        return ofx::fail(OFX_ECOMM, "%s: the communicator was aborted meanwhile (%s)", what,
                         cm->why.c_str());
      const ncclResult_t q = ncclCommGetAsyncError(cm->nccl, &st);
      if (q != ncclSuccess)
        return ofx::fail(OFX_ECOMM, "%s: ncclCommGetAsyncError failed: %s", what,
                         ncclGetErrorString(q));
    }
    if (st != ncclInProgress) break;
    if (seconds_since(t0) > cm->call_timeout_s) {
      char why[256];
      snprintf(why, sizeof(why), "%s still in progress after %.0f s", what, cm->call_timeout_s);
      cm->abort(why);
      return ofx::fail(OFX_ECOMM, "%s; communicator aborted", why);
    }
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
  if (st != ncclSuccess) return ofx::fail(OFX_ECOMM, "%s failed: %s", what, ncclGetErrorString(st));
  return OFX_OK;
}

// The optional device-side deadline of an exchange: the host call enqueues the
// collective and returns at once, so a peer that never joins leaves the stream stuck with no host
// call to time out.  With device_timeout_s > 0 the exchange's completion is awaited here (an event
// on the stream, queried until done); past the deadline the communicator is aborted (its kernels
// are dropped, the peers' calls fail) and OFX_ECOMM names the exchange.  Skipped while the stream
// is being captured (a graph replay is waited for by its launcher).  The test knob
// OFX_DEBUG_EXCHANGE_STALL treats the exchange as never completing.
int device_deadline(OfxComm* cm, hipStream_t s, const char* what) {
  if (cm->device_timeout_s <= 0) return OFX_OK;
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  OFX_HIP_CHECK(hipStreamIsCapturing(s, &cap));
  if (cap != hipStreamCaptureStatusNone) return OFX_OK;
  hipEvent_t ev;
  OFX_HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  hipError_t e = hipEventRecord(ev, s);
  const bool stall = ofx::debug_knob(OFX_DEBUG_EXCHANGE_STALL, 0) != 0;
  const auto t0 = std::chrono::steady_clock::now();
  while (e == hipSuccess) {
    e = hipEventQuery(ev);
    if (e == hipSuccess && !stall) break;
    if (e == hipErrorNotReady || (e == hipSuccess && stall)) {
      e = hipSuccess;
      if (cm->aborted.load()) {  // a watchdog aborted the communicator meanwhile
        (void)hipEventDestroy(ev);
        return ofx::fail(OFX_ECOMM, "%s: the communicator was aborted meanwhile (%s)", what,
                         cm->why.c_str());
      }
      if (seconds_since(t0) > cm->device_timeout_s) {
        (void)hipEventDestroy(ev);
        char why[256];
        snprintf(why, sizeof(why), "%s did not complete on the device within %.1f s", what,
                 cm->device_timeout_s);
        cm->abort(why);
        return ofx::fail(OFX_ECOMM, "%s; communicator aborted", why);
      }
      std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
  }
  (void)hipEventDestroy(ev);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return ofx::fail(OFX_EDEVICE, "%s: waiting for the exchange: %s", what, hipGetErrorString(e));
  }
  return OFX_OK;
}
}  // namespace

extern "C" int ofx_comm_get_unique_id(void* uid_out) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(uid_out, OFX_EINVAL, "comm_get_unique_id: NULL");
    ncclUniqueId id;
    OFX_NCCL_CHECK(ncclGetUniqueId(&id));
    std::memset(uid_out, 0, OFX_UNIQUE_ID_BYTES);
    std::memcpy(uid_out, &id, sizeof(id));
    return OFX_OK;
  });
}

extern "C" int ofx_comm_init_rank(void** comm, int nranks, const void* uid, int rank) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(comm && uid && nranks > 0 && rank >= 0 && rank < nranks, OFX_EINVAL,
                "comm_init_rank: bad arguments (nranks=%d rank=%d)", nranks, rank);
    ncclUniqueId id;
    std::memcpy(&id, uid, sizeof(id));
    ncclComm_t c;
    OFX_NCCL_CHECK(ncclCommInitRank(&c, nranks, id, rank));
    OfxComm* cm = new OfxComm();
    cm->nccl = c;
    *comm = cm;
    return OFX_OK;
  });
}

// ofx_comm_init_rank with a deadline: a non-blocking communicator
// (ncclCommInitRankConfig, config.blocking = 0) whose set-up is polled with
// ncclCommGetAsyncError; a rank whose peers have not all joined within `timeout_s` seconds aborts
// the communicator (ncclCommAbort) and returns OFX_ECOMM naming the wait, instead of blocking
// forever inside ncclCommInitRank.  Every later call on the communicator is bounded the same way
// (OFX_NCCL_CALL, this communicator's own timeout: ofx_comm_set_timeouts).  The reference's
// EagerNcclCommMgr::CreateNcclComm (oneflow/core/job/eager_nccl_comm_manager.cpp:57-80) blocks
// without a bound.
extern "C" int ofx_comm_init_rank_deadline(void** comm, int nranks, const void* uid, int rank,
                                           double timeout_s) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(comm && uid && nranks > 0 && rank >= 0 && rank < nranks && timeout_s > 0, OFX_EINVAL,
                "comm_init_rank_deadline: bad arguments (nranks=%d rank=%d timeout=%g)", nranks, rank,
                timeout_s);
    ncclUniqueId id;
    std::memcpy(&id, uid, sizeof(id));
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclComm_t c = nullptr;
    const ncclResult_t r = ncclCommInitRankConfig(&c, nranks, id, rank, &cfg);
    if (r != ncclSuccess && r != ncclInProgress) {
      if (c != nullptr) ncclCommAbort(c);
      return ofx::fail(OFX_ECOMM, "comm_init_rank_deadline: ncclCommInitRankConfig failed: %s",
                       ncclGetErrorString(r));
    }
    const auto t0 = std::chrono::steady_clock::now();
    ncclResult_t st = r;
    while (st == ncclInProgress) {
      const ncclResult_t q = ncclCommGetAsyncError(c, &st);
      if (q != ncclSuccess) st = q;
      if (st != ncclInProgress) break;
      if (seconds_since(t0) > timeout_s) {
        ncclCommAbort(c);
        return ofx::fail(OFX_ECOMM,
                         "comm_init_rank_deadline: rank %d of %d: communicator not set up after %.0f s "
                         "(a peer did not join); aborted", rank, nranks, timeout_s);
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    if (st != ncclSuccess) {
      ncclCommAbort(c);
      return ofx::fail(OFX_ECOMM, "comm_init_rank_deadline: rank %d of %d: %s", rank, nranks,
                       ncclGetErrorString(st));
    }
    OfxComm* cm = new OfxComm();
    cm->nccl = c;
    cm->call_timeout_s = timeout_s;
    *comm = cm;
    return OFX_OK;
  });
}

// This communicator's deadlines (per communicator, not one process-wide value):
// call_timeout_s bounds a call left in progress (non-blocking communicators; <= 0 keeps the
// current one), device_timeout_s > 0 awaits every exchange's completion on the device for at most
// that long (0 = off: the exchanges stay asynchronous, as a timed step needs).
extern "C" int ofx_comm_set_timeouts(void* comm, double call_timeout_s, double device_timeout_s) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_LIVE_COMM(comm, "comm_set_timeouts");
    (void)c;
    OFX_REQUIRE(device_timeout_s >= 0, OFX_EINVAL, "comm_set_timeouts: negative device timeout");
    if (call_timeout_s > 0) ofx_cm_->call_timeout_s = call_timeout_s;
    ofx_cm_->device_timeout_s = device_timeout_s;
    return OFX_OK;
  });
}

// Aborts a communicator (ncclCommAbort): its pending operations are dropped and peers blocked on
// it fail.  Called by a rank's phase watchdog before it exits (bench.py).  The handle stays valid
// (every call on it returns OFX_ECOMM); ofx_comm_destroy frees it.
extern "C" int ofx_comm_abort(void* comm) {
  return ::ofx::guarded(__func__, [&]() -> int {
    if (comm) static_cast<OfxComm*>(comm)->abort("ofx_comm_abort");
    return OFX_OK;
  });
}

// Frees a handle.  A live communicator is finalized first (flushes its operations; a non-blocking
// one may report ncclInProgress, waited for with its call timeout), then destroyed; if finalizing
// fails it is aborted instead, so it is never leaked.  An aborted one only has its handle freed.
extern "C" int ofx_comm_destroy(void* comm) {
  return ::ofx::guarded(__func__, [&]() -> int {
    if (comm == nullptr) return OFX_OK;
    std::unique_ptr<OfxComm> cm(static_cast<OfxComm*>(comm));
    if (cm->aborted.load()) return OFX_OK;
    const int rc = comm_wait(cm.get(), ncclCommFinalize(cm->nccl), "ncclCommFinalize");
    if (cm->aborted.load()) return rc;  // the finalize timed out: comm_wait aborted it
    if (rc != OFX_OK) {
      cm->abort("finalize failed");
      return rc;
    }
    OFX_NCCL_CHECK(ncclCommDestroy(cm->nccl));
    return OFX_OK;
  });
}

// Ranks and this rank's index in a communicator (what bench.py reports as the RCCL comm size).
extern "C" int ofx_comm_count(void* comm, int* nranks, int* rank) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(nranks && rank, OFX_EINVAL, "comm_count: NULL argument");
    OFX_LIVE_COMM(comm, "comm_count");
    OFX_NCCL_CHECK(ncclCommCount(c, nranks));
    OFX_NCCL_CHECK(ncclCommUserRank(c, rank));
    return OFX_OK;
  });
}

extern "C" int ofx_allgather(void* stream, const void* in, void* out, size_t count, int dtype,
                             void* comm) {
  return ::ofx::guarded(__func__, [&]() -> int {
    ncclDataType_t t;
    OFX_REQUIRE(nccl_dtype(dtype, &t), OFX_EUNSUPPORTED, "allgather: unsupported dtype %d", dtype);
    OFX_REQUIRE(count == 0 || (in && out), OFX_EINVAL, "allgather: NULL argument");
    OFX_LIVE_COMM(comm, "allgather");
    hipStream_t s = static_cast<hipStream_t>(stream);
    OFX_NCCL_CALL(ofx_cm_, ncclAllGather(in, out, count, t, c, s));
    return device_deadline(ofx_cm_, s, "allgather");
  });
}

// All-gather as grouped point-to-point transfers: every rank sends its slot to every peer and
// receives every peer's slot directly (one xGMI link per peer on a fully connected MI355X node),
// instead of RCCL's ring/tree schedule.  `buf` holds nranks slots of `count` elements; this
// rank's slot (rank * count) is the send buffer (in place).  Same bytes as ofx_allgather.
extern "C" int ofx_allgather_p2p(void* stream, void* buf, size_t count, int dtype, void* comm) {
  return ::ofx::guarded(__func__, [&]() -> int {
    ncclDataType_t t;
    OFX_REQUIRE(nccl_dtype(dtype, &t), OFX_EUNSUPPORTED, "allgather_p2p: unsupported dtype %d", dtype);
    OFX_REQUIRE(count == 0 || buf, OFX_EINVAL, "allgather_p2p: NULL argument");
    OFX_LIVE_COMM(comm, "allgather_p2p");
    int nranks = 0, rank = 0;
    OFX_NCCL_CHECK(ncclCommCount(c, &nranks));
    OFX_NCCL_CHECK(ncclCommUserRank(c, &rank));
    const size_t esz = (size_t)ofx::dtype_size(dtype);
    char* base = static_cast<char*>(buf);
    hipStream_t s = static_cast<hipStream_t>(stream);
    OFX_NCCL_CHECK(ncclGroupStart());
    for (int d = 1; d < nranks; ++d) {  // peers in a rotated order so links are loaded evenly
      const int to = (rank + d) % nranks, from = (rank - d + nranks) % nranks;
      OFX_NCCL_GROUPED(ncclSend(base + (size_t)rank * count * esz, count, t, to, c, s));
      OFX_NCCL_GROUPED(ncclRecv(base + (size_t)from * count * esz, count, t, from, c, s));
    }
    OFX_NCCL_CALL(ofx_cm_, ncclGroupEnd());
    return device_deadline(ofx_cm_, s, "allgather_p2p");
  });
}

// A stream-ordered barrier: a 1-element max all-reduce.  When it completes on this rank's stream,
// every rank's stream has reached it, i.e. finished everything enqueued before it.
static int stream_barrier(OfxComm* cm, hipStream_t s, const char* what) {
  if (cm->barrier_word == nullptr) {
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    OFX_HIP_CHECK(hipStreamIsCapturing(s, &cap));
    OFX_REQUIRE(cap == hipStreamCaptureStatusNone, OFX_EINVAL,
                "%s: run the exchange once before capturing it (its barrier word is allocated on "
                "first use)", what);
    OFX_HIP_CHECK(hipMalloc(&cm->barrier_word, 256));
    OFX_HIP_CHECK(hipMemsetAsync(cm->barrier_word, 0, 256, s));
  }
  OFX_NCCL_CALL(cm, ncclAllReduce(cm->barrier_word, cm->barrier_word, 1, ncclInt32, ncclMax,
                                  cm->nccl, s));
  return OFX_OK;
}

// The pull all-gather (include/ofx_spmm.h): publish this rank's slot, barrier (every slot ready),
// read every peer's slot out of its buffer, barrier (no rank rewrites its slot -- the next step's
// shard -- while a peer still reads it).  Same bytes as ofx_allgather.
extern "C" int ofx_allgather_pull(void* stream, void* comm, const void* const* peer_bufs, void* buf,
                                  size_t count, int dtype) {
  return ::ofx::guarded(__func__, [&]() -> int {
    ncclDataType_t t;
    OFX_REQUIRE(nccl_dtype(dtype, &t), OFX_EUNSUPPORTED, "allgather_pull: unsupported dtype %d", dtype);
    OFX_LIVE_COMM(comm, "allgather_pull");
    int nranks = 0, rank = 0;
    OFX_NCCL_CHECK(ncclCommCount(c, &nranks));
    OFX_NCCL_CHECK(ncclCommUserRank(c, &rank));
    if (nranks == 1 || count == 0) return OFX_OK;
    OFX_REQUIRE(peer_bufs && buf, OFX_EINVAL, "allgather_pull: NULL argument");
    hipStream_t s = static_cast<hipStream_t>(stream);
    const uint64_t slot = (uint64_t)count * (uint64_t)ofx::dtype_size(dtype);
    int rc = ofx_peer_publish(s);
    if (rc == OFX_OK) rc = stream_barrier(ofx_cm_, s, "allgather_pull (slots ready)");
    if (rc == OFX_OK) rc = ofx_peer_pull(s, nranks, rank, peer_bufs, buf, slot);
    if (rc == OFX_OK) rc = stream_barrier(ofx_cm_, s, "allgather_pull (pulls done)");
    if (rc != OFX_OK) return rc;
    return device_deadline(ofx_cm_, s, "allgather_pull");
  });
}

// Halo exchange of B rows: grouped point-to-point send/recv with
// per-peer row counts, the pattern of ShuffleData in
// oneflow/user/kernels/data_shuffle_kernel.cu:119-135 (ncclGroupStart; ncclSend/ncclRecv per
// peer; ncclGroupEnd).  Counts and offsets are in rows of `n` elements, host arrays of nranks;
// this rank's own entry and zero counts are skipped (both sides agree by construction).
extern "C" int ofx_exchange_rows(void* stream, void* comm, int dtype, int64_t n,
                                 const void* send_buf, const int64_t* send_counts,
                                 const int64_t* send_offsets, void* recv_buf,
                                 const int64_t* recv_counts, const int64_t* recv_offsets) {
  return ::ofx::guarded(__func__, [&]() -> int {
    ncclDataType_t t;
    OFX_REQUIRE(nccl_dtype(dtype, &t), OFX_EUNSUPPORTED, "exchange_rows: unsupported dtype %d", dtype);
    OFX_REQUIRE(send_counts && send_offsets && recv_counts && recv_offsets && n >= 0,
                OFX_EINVAL, "exchange_rows: NULL argument");
    OFX_LIVE_COMM(comm, "exchange_rows");
    int nranks = 0, rank = 0;
    OFX_NCCL_CHECK(ncclCommCount(c, &nranks));
    OFX_NCCL_CHECK(ncclCommUserRank(c, &rank));
    const size_t row_bytes = (size_t)n * (size_t)ofx::dtype_size(dtype);
    const char* sb = static_cast<const char*>(send_buf);
    char* rb = static_cast<char*>(recv_buf);
    hipStream_t s = static_cast<hipStream_t>(stream);
    OFX_NCCL_CHECK(ncclGroupStart());
    for (int d = 1; d < nranks; ++d) {
      const int to = (rank + d) % nranks, from = (rank - d + nranks) % nranks;
      if (send_counts[to] > 0)
        OFX_NCCL_GROUPED(ncclSend(sb + (size_t)send_offsets[to] * row_bytes,
                                  (size_t)(send_counts[to] * n), t, to, c, s));
      if (recv_counts[from] > 0)
        OFX_NCCL_GROUPED(ncclRecv(rb + (size_t)recv_offsets[from] * row_bytes,
                                  (size_t)(recv_counts[from] * n), t, from, c, s));
    }
    OFX_NCCL_CALL(ofx_cm_, ncclGroupEnd());
    return device_deadline(ofx_cm_, s, "exchange_rows");
  });
}

// One step of the row-split operator on this rank (SURVEY.md §8b "ofx_spmm_rowsplit"): the
// S(0) -> B boxing of b as an in-place all-gather of the padded shards (each rank has written
// its rows at [rank * P, rank * P + K_r) of b_gathered), then the local SpMM of this rank's rows
// (CSR slice with row_ptr rebased to 0 and columns remapped by ofx_padded_owner_remap).  The
// same two launches RowSplitSpmm issues; stream-ordered, no host synchronisation.
extern "C" int ofx_spmm_rowsplit(void* stream, void* comm, int idx_dtype, int val_dtype,
                                 int64_t m_local, int64_t k_padded, int64_t n, int64_t nnz_local,
                                 const void* row_ptr, const void* col_idx, const void* values,
                                 void* b_gathered, void* c, int64_t ldc, void* workspace,
                                 size_t workspace_bytes, const ofx_spmm_options* opts) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(k_padded >= 0 && n >= 0, OFX_EINVAL, "spmm_rowsplit: bad arguments");
    int nranks = 0, rank = 0;
    const int rc0 = ofx_comm_count(comm, &nranks, &rank);  // a live communicator, or its error
    if (rc0 != OFX_OK) return rc0;
    OFX_REQUIRE(k_padded % nranks == 0, OFX_EINVAL,
                "spmm_rowsplit: k_padded=%lld is not a multiple of %d ranks", (long long)k_padded,
                nranks);
    const int64_t pad = k_padded / nranks;
    const size_t esz = (size_t)ofx::dtype_size(val_dtype);
    if (pad * n > 0) {
      char* slot = static_cast<char*>(b_gathered) + (size_t)(rank * pad * n) * esz;
      const int rc = ofx_allgather(stream, slot, b_gathered, (size_t)(pad * n), val_dtype, comm);
      if (rc) return rc;
    }
    return ofx_spmm_csr(stream, idx_dtype, val_dtype, m_local, k_padded, n, nnz_local, row_ptr,
                        col_idx, values, b_gathered, n, c, ldc, 0, m_local, workspace,
                        workspace_bytes, opts);
  });
}
