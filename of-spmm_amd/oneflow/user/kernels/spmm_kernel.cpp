/*
 * spmm_kernel.cpp — kernels of op "spmm_csr" for DeviceType::kCPU and DeviceType::kHIP.
 *
 * Pattern of a OneFlow user kernel with a row-range cache, following
 * oneflow/user/kernels/unsorted_segment_sum_kernel.cpp:46-78 (OpKernelCache holding
 * [lower, upper) from the out SBP, BalancedSplitter via GetTensorSliceView4ParallelId,
 * oneflow/core/job/nd_sbp_util.cpp:98-104) and :146-205 (tmp buffer via SetInferTmpSizeFn).
 * The device work is the C-ABI: ofx_spmm_csr (HIP, async on the op's stream) and
 * ofx_spmm_csr_cpu (host).  Kernel errors are fatal CHECKs as in
 * oneflow/user/kernels/matrix_vector_product_kernel.cpp:98-109.
 */
#include <list>
#include <mutex>

#include "oneflow/core/framework/framework.h"
#include "oneflow/core/functional/spmm_functor.h"
#include "ofx_spmm.h"

namespace oneflow {

// ---- static CSR: the work-list plan kept across calls (attr static_csr) -----
// The kernel state of OpKernel::CreateOpKernelState (oneflow/core/framework/op_kernel.h:292),
// which OneFlow keeps per StatefulOpKernel (eager: per op expression and device) or per
// UserKernel (lazy).  For a caller that promises an unchanged CSR (static_csr != 0) it holds the
// planner's work list in a device workspace of its own, so the launch skips the planner kernel
// (options.planned = 1, ofx_spmm_csr_plan).  A plan is a pure function of row_ptr, the row range,
// the shapes and the schedule; the key holds those plus the static_csr value (the caller's name
// for this CSR: a new CSR at reused addresses gets a new one) and the stream (the in-kernel hub
// reduce's arrival counters live in the workspace, so two streams never share one).
class SpmmCsrPlanState final : public user_op::OpKernelState {
 public:
  struct Key {
    int64_t static_csr;
    const void* row_ptr;
    const void* stream;
    int device, idx_dt, val_dt;
    int64_t m, k, n, nnz, row_begin, row_end, split, chunk, heavy, range_nnz;
    bool operator==(const Key& o) const {
      return static_csr == o.static_csr && row_ptr == o.row_ptr && stream == o.stream &&
             device == o.device && idx_dt == o.idx_dt && val_dt == o.val_dt && m == o.m &&
             k == o.k && n == o.n && nnz == o.nnz && row_begin == o.row_begin &&
             row_end == o.row_end && split == o.split && chunk == o.chunk && heavy == o.heavy &&
             range_nnz == o.range_nnz;
    }
  };
  static constexpr size_t kMaxPlans = 8;

  // key_on_stream: an eager op's state may see calls on any stream, so the stream is part of the
  // key; a lazy op's (a compiled job's) launches are ordered on its one named stream, and its
  // graph is captured on another stream than it replays on, so the key leaves the stream out.
  explicit SpmmCsrPlanState(bool key_on_stream) : key_on_stream_(key_on_stream) {}
  ~SpmmCsrPlanState() override { Release(); }
  bool key_on_stream() const { return key_on_stream_; }
  // Held by a static call from Acquire through its launch's enqueue, so no other thread evicts
  // (and frees) the workspace in between.
  std::recursive_mutex& launch_mutex() { return mu_; }

  // The workspace for `key`: *planned = true when it already holds key's plan (a hit).  On a miss
  // a workspace of `bytes` is allocated on the key's device (past kMaxPlans the least recently
  // used entry no capture has used is evicted) and the caller plans into it; a miss while the
  // stream is capturing a graph takes no workspace (*ws = NULL: the ordinary path), as
  // allocation and eviction are not capturable.  A hit while capturing pins the entry: the graph
  // holds its pointer and may replay at any later time, so the workspace is never evicted or
  // freed before Release (the state's end, or ofx_spmm_static_plans(release = 1)).
  int Acquire(const Key& key, size_t bytes, bool capturing, void** ws, bool* planned) {
    std::lock_guard<std::recursive_mutex> lock(mu_);
    *ws = nullptr;
    *planned = false;
    for (auto it = entries_.begin(); it != entries_.end(); ++it) {
      if (it->key == key && it->bytes >= bytes) {
        entries_.splice(entries_.begin(), entries_, it);  // most recently used first
        if (capturing) it->pinned = true;
        *ws = it->ws;
        *planned = true;
        ++hits_;
        return OFX_OK;
      }
    }
    if (capturing) return OFX_OK;
    int rc = OFX_OK;
    if (entries_.size() >= kMaxPlans) {
      // the least recently used unpinned entry (none: the state grows past the cap); an
      // in-flight launch may still read its plan, so the device drains first
      auto victim = entries_.end();
      for (auto it = entries_.begin(); it != entries_.end(); ++it)
        if (!it->pinned) victim = it;
      if (victim != entries_.end()) {
        rc = WithDevice(victim->key.device, [&]() {
          const int r = ofx_device_synchronize();
          return r != OFX_OK ? r : ofx_free(victim->ws);
        });
        entries_.erase(victim);
        if (rc != OFX_OK) return rc;
      }
    }
    void* p = nullptr;
    rc = WithDevice(key.device, [&]() { return ofx_malloc(&p, bytes); });
    if (rc != OFX_OK) return rc;
    entries_.push_front(Entry{key, p, bytes, false});
    *ws = p;
    ++plans_;
    return OFX_OK;
  }

  // Forget key's plan (its launch failed): the next call plans again.  A pinned entry's
  // workspace (a captured graph holds it) is retired, not freed, until Release; so is one dropped
  // while the stream captures (the device cannot be drained inside a capture).
  void Drop(const Key& key, bool capturing) {
    std::lock_guard<std::recursive_mutex> lock(mu_);
    for (auto it = entries_.begin(); it != entries_.end(); ++it) {
      if (it->key == key) {
        if (capturing || it->pinned) {
          retired_.push_back(*it);
        } else {
          WithDevice(it->key.device, [&]() {
            ofx_device_synchronize();
            return ofx_free(it->ws);
          });
        }
        entries_.erase(it);
        return;
      }
    }
  }

  void Stats(int64_t* entries, int64_t* plans, int64_t* hits) {
    std::lock_guard<std::recursive_mutex> lock(mu_);
    *entries += (int64_t)entries_.size();
    *plans += plans_;
    *hits += hits_;
  }

  // Frees every workspace, pinned ones included: the graphs that captured static calls of this
  // state must be gone (the state's end, or the caller's explicit release).
  void Release() {
    std::lock_guard<std::recursive_mutex> lock(mu_);
    for (auto* list : {&retired_, &entries_}) {
      for (Entry& e : *list) {
        WithDevice(e.key.device, [&]() {
          ofx_device_synchronize();
          return ofx_free(e.ws);
        });
      }
      list->clear();
    }
  }

 private:
  struct Entry {
    Key key;
    void* ws;
    size_t bytes;
    bool pinned;  // used by a graph capture: never evicted
  };
  template <typename F>
  static int WithDevice(int device, F&& f) {
    int prev = -1;
    if (ofx_get_device(&prev) != OFX_OK) prev = -1;
    if (prev != device && ofx_set_device(device) != OFX_OK) return OFX_EDEVICE;
    const int rc = f();
    if (prev >= 0 && prev != device) ofx_set_device(prev);
    return rc;
  }

  const bool key_on_stream_;
  std::recursive_mutex mu_;  // held by Acquire / Drop / Release, and by Compute across a launch
  std::list<Entry> entries_;
  std::list<Entry> retired_;  // dropped but possibly held by a captured graph: freed at Release
  int64_t plans_ = 0, hits_ = 0;
};

bool SpmmCsrPlanStateStats(user_op::OpKernelState* state, int64_t* entries, int64_t* plans,
                           int64_t* hits, bool release) {
  auto* s = dynamic_cast<SpmmCsrPlanState*>(state);
  if (s == nullptr) return false;
  if (release) s->Release();
  s->Stats(entries, plans, hits);
  return true;
}

namespace {

// Row range [lower, upper) of this rank's physical out and the logical width N.  The range
// follows unsorted_segment_sum_kernel.cpp:59-78: GetTensorSliceView4ParallelId over out's nd_sbp
// and the placement hierarchy (1-D: BalancedSplitter; 2-D: e.g. (S(0), S(1)) rows x columns).
// The logical N fixes the hub-row schedule: split = default_split(N) whatever slice of the
// columns this rank computes, so a column-split rank's bits equal the single-device op's.
class SpmmCsrOpKernelCache final : public user_op::OpKernelCache {
 public:
  SpmmCsrOpKernelCache(int64_t lower, int64_t upper, int64_t logical_n)
      : lower_(lower), upper_(upper), logical_n_(logical_n) {}
  ~SpmmCsrOpKernelCache() override = default;
  int64_t lower() const { return lower_; }
  int64_t upper() const { return upper_; }
  int64_t logical_n() const { return logical_n_; }

 private:
  const int64_t lower_;
  const int64_t upper_;
  const int64_t logical_n_;
};

std::shared_ptr<user_op::OpKernelCache> CreateSpmmCsrOpKernelCache(user_op::KernelCacheContext* ctx) {
  const user_op::TensorDesc* out_logical = ctx->LogicalTensorDesc4ArgNameAndIndex("out", 0);
  const Shape& shape = out_logical->shape();
  int64_t lower = 0, upper = shape.At(0);
  if (ctx->parallel_ctx().parallel_num() > 1) {
    const TensorSliceView view =
        GetTensorSliceView4ParallelId(*ctx->parallel_desc().hierarchy(),
                                      ctx->NdSbp4ArgNameAndIndex("out", 0), shape,
                                      ctx->parallel_ctx().parallel_id());
    lower = view.At(0).begin();
    upper = view.At(0).end();
  }
  return std::make_shared<SpmmCsrOpKernelCache>(lower, upper, shape.At(1));
}

// Options of a launch: the contract's schedule for the logical width (no cache: local op, the
// physical width is the logical one).
ofx_spmm_options OptionsOf(const SpmmCsrOpKernelCache* cache) {
  ofx_spmm_options o = OFX_SPMM_OPTIONS_INIT;
  if (cache != nullptr) o.split_threshold = ofx_spmm_default_split(cache->logical_n());
  return o;
}

int DtCode(DataType dt) { return static_cast<int>(dt); }

// A static call on the HIP kernel (attr static_csr != 0): the workspace of `plans` that holds
// this launch's plan -- built here on a miss -- replaces the tmp buffer, and opts->planned is
// set.  sp->hold keeps the state's lock until the launch is enqueued (the caller's scope);
// sp->keyed says a plan is in use (the caller drops it if the launch fails).  A miss while the
// stream captures keeps the ordinary path (the tmp buffer, planned = 0).
struct StaticPlan {
  SpmmCsrPlanState::Key key{};
  bool keyed = false;
  std::unique_lock<std::recursive_mutex> hold;
};

void UseStaticPlan(SpmmCsrPlanState* plans, int64_t static_csr, ep::HipStream* hs,
                   const void* row_ptr, int idx_dt, int val_dt, int64_t m, int64_t k, int64_t n,
                   int64_t nnz, int64_t row_begin, int64_t row_end, const char* op_name,
                   ofx_spmm_options* opts, void** ws, size_t* ws_bytes, StaticPlan* sp) {
  if (row_end <= row_begin || n <= 0) return;
  sp->hold = std::unique_lock<std::recursive_mutex>(plans->launch_mutex());
  size_t need = 0;
  int rc = ofx_spmm_csr_workspace_size(idx_dt, val_dt, m, k, n, nnz, opts, &need);
  OFX_KERNEL_CHECK(rc == OFX_OK, op_name << " workspace query failed: " << ofx_last_error());
  if (need == 0) return;  // no work list to keep (the small form, or the identity order)
  void* stream = hs->hip_stream();
  sp->key = SpmmCsrPlanState::Key{static_csr, row_ptr, plans->key_on_stream() ? stream : nullptr,
                                  hs->device_index(), idx_dt, val_dt, m, k, n, nnz, row_begin,
                                  row_end, opts->split_threshold, opts->chunk,
                                  opts->heavy_threshold, opts->range_nnz};
  void* sws = nullptr;
  bool planned = false;
  rc = plans->Acquire(sp->key, need, hs->IsGraphCapturing(), &sws, &planned);
  OFX_KERNEL_CHECK(rc == OFX_OK, op_name << " static_csr plan workspace: " << ofx_last_error());
  if (sws == nullptr) return;
  sp->keyed = true;
  if (!planned) {
    rc = ofx_spmm_csr_plan(stream, idx_dt, val_dt, m, k, n, nnz, row_ptr, row_begin, row_end, sws,
                           need, opts);
    if (rc != OFX_OK) plans->Drop(sp->key, hs->IsGraphCapturing());
    OFX_KERNEL_CHECK(rc == OFX_OK, op_name << " kernel failed (" << rc << "): " << ofx_last_error());
  }
  opts->planned = 1;
  *ws = sws;
  *ws_bytes = need;
}

// Shared body of "spmm_csr" and "fused_spmm_csr": bias (optional T[N]) and relu are the fused
// epilogue; the plain op passes none (ofx_spmm_csr_fused with NULL/none == ofx_spmm_csr).
template <DeviceType device_type>
void ComputeSpmmCsr(user_op::KernelComputeContext* ctx, const user_op::OpKernelCache* cache,
                    const user_op::Tensor* bias, bool relu, const char* op_name,
                    SpmmCsrPlanState* plans = nullptr, int64_t static_csr = 0) {
  TestHookCompute(op_name);
  const user_op::Tensor* row_ptr = ctx->Tensor4ArgNameAndIndex("a_csr_row_ptr", 0);
  const user_op::Tensor* col_idx = ctx->Tensor4ArgNameAndIndex("a_csr_col_idx", 0);
  const user_op::Tensor* values = ctx->Tensor4ArgNameAndIndex("a_csr_values", 0);
  const user_op::Tensor* b = ctx->Tensor4ArgNameAndIndex("b", 0);
  user_op::Tensor* out = ctx->Tensor4ArgNameAndIndex("out", 0);
  const int64_t m = ctx->Attr<int64_t>("a_num_rows");
  const int64_t k = ctx->Attr<int64_t>("a_num_cols");
  OFX_KERNEL_CHECK(b->shape_view().NumAxes() == 2, "b Numdims should be equal to 2. ");
  OFX_KERNEL_CHECK(out->shape_view().NumAxes() == 2, "out Numdims should be equal to 2. ");
  OFX_KERNEL_CHECK(out->data_type() == b->data_type(), "out datatype should be equal to b. ");
  const int64_t n = out->shape_view().At(1);
  const int64_t nnz = col_idx->shape_view().elem_cnt();
  int64_t row_begin = 0;
  int64_t row_end = m;
  const auto* range = dynamic_cast<const SpmmCsrOpKernelCache*>(cache);
  OFX_KERNEL_CHECK(cache == nullptr || range != nullptr, "unexpected kernel cache type");
  if (range != nullptr) {
    row_begin = range->lower();
    row_end = range->upper();
  }
  ofx_spmm_options opts = OptionsOf(range);
  OFX_KERNEL_CHECK(out->shape_view().At(0) == row_end - row_begin,
                   "out rows " << out->shape_view().At(0) << " != row range "
                               << row_end - row_begin);
  if (bias != nullptr)
    OFX_KERNEL_CHECK(bias->shape_view().elem_cnt() == n && bias->data_type() == b->data_type(),
                     "bias must be [" << n << "] of b's dtype");
  const int idx_dt = DtCode(row_ptr->data_type());
  const int val_dt = DtCode(values->data_type());
  const void* bias_ptr = bias ? bias->dptr() : nullptr;
  const int act = relu ? OFX_ACT_RELU : OFX_ACT_NONE;
  int rc;
  if (device_type == DeviceType::kHIP) {
    user_op::Tensor* tmp = ctx->Tensor4ArgNameAndIndex("tmp_buffer", 0);
    void* ws = tmp ? tmp->mut_dptr() : nullptr;
    size_t ws_bytes = tmp ? (size_t)tmp->shape_view().elem_cnt() : 0;
    ep::HipStream* hs = ctx->stream()->As<ep::HipStream>();
    void* stream = hs->hip_stream();
    StaticPlan sp;
    if (plans != nullptr && static_csr != 0)
      UseStaticPlan(plans, static_csr, hs, row_ptr->dptr(), idx_dt, val_dt, m, k, n, nnz,
                    row_begin, row_end, op_name, &opts, &ws, &ws_bytes, &sp);
    rc = ofx_spmm_csr_fused(stream, idx_dt, val_dt, m, k, n, nnz, row_ptr->dptr(),
                            col_idx->dptr(), values->dptr(), b->dptr(), b->row_stride(),
                            out->mut_dptr(), out->row_stride(), row_begin, row_end, bias_ptr, act,
                            ws, ws_bytes, &opts);
    // an earlier launch's loud failure (OFX_EPLAN) may have been this key's plan: plan again
    if (rc != OFX_OK && sp.keyed) plans->Drop(sp.key, hs->IsGraphCapturing());
  } else {
    const int threads = ctx->stream()->As<ep::CpuStream>()->num_threads();
    rc = ofx_spmm_csr_fused_cpu(threads, idx_dt, val_dt, m, k, n, nnz, row_ptr->dptr(),
                                col_idx->dptr(), values->dptr(), b->dptr(), b->row_stride(),
                                out->mut_dptr(), out->row_stride(), row_begin, row_end, bias_ptr,
                                act, &opts);
  }
  OFX_KERNEL_CHECK(rc == OFX_OK, op_name << " kernel failed (" << rc << "): " << ofx_last_error());
}

template <DeviceType device_type>
class SpmmCsrKernel final : public user_op::OpKernel, public user_op::CudaGraphSupport {
 public:
  SpmmCsrKernel() = default;
  ~SpmmCsrKernel() override = default;

  std::shared_ptr<user_op::OpKernelCache> InitOpKernelCache(
      user_op::KernelCacheContext* ctx) const override {
    return CreateSpmmCsrOpKernelCache(ctx);
  }

  // The plans of static CSRs (HIP only: the kCPU kernel has no work list).
  std::shared_ptr<user_op::OpKernelState> CreateOpKernelState(
      user_op::KernelInitContext* ctx) const override {
    if (device_type != DeviceType::kHIP) return nullptr;
    return std::make_shared<SpmmCsrPlanState>(!ctx->has_stream_name_hint());
  }

  bool AlwaysComputeWhenAllOutputsEmpty() const override { return false; }

 private:
  using user_op::OpKernel::Compute;
  void Compute(user_op::KernelComputeContext* ctx, user_op::OpKernelState* state,
               const user_op::OpKernelCache* cache) const override {
    const int64_t static_csr = ctx->Attr<int64_t>("static_csr");
    ComputeSpmmCsr<device_type>(ctx, cache, nullptr, false, "spmm_csr",
                                dynamic_cast<SpmmCsrPlanState*>(state), static_csr);
  }
};

template <DeviceType device_type>
class FusedSpmmCsrKernel final : public user_op::OpKernel, public user_op::CudaGraphSupport {
 public:
  FusedSpmmCsrKernel() = default;
  ~FusedSpmmCsrKernel() override = default;

  std::shared_ptr<user_op::OpKernelCache> InitOpKernelCache(
      user_op::KernelCacheContext* ctx) const override {
    return CreateSpmmCsrOpKernelCache(ctx);
  }

  // The plans of static CSRs, as spmm_csr's (the fused epilogue does not change the work list).
  std::shared_ptr<user_op::OpKernelState> CreateOpKernelState(
      user_op::KernelInitContext* ctx) const override {
    if (device_type != DeviceType::kHIP) return nullptr;
    return std::make_shared<SpmmCsrPlanState>(!ctx->has_stream_name_hint());
  }

  bool AlwaysComputeWhenAllOutputsEmpty() const override { return false; }

 private:
  using user_op::OpKernel::Compute;
  void Compute(user_op::KernelComputeContext* ctx, user_op::OpKernelState* state,
               const user_op::OpKernelCache* cache) const override {
    ComputeSpmmCsr<device_type>(ctx, cache, ctx->Tensor4ArgNameAndIndex("bias", 0),
                                ctx->Attr<bool>("relu"), "fused_spmm_csr",
                                dynamic_cast<SpmmCsrPlanState*>(state),
                                ctx->Attr<int64_t>("static_csr"));
  }
};

// "spmm_csr_gathered": out = A @ b with nonzero j's value a_csr_values[values_perm[j]] (the
// d(b) gradient with learnable values).  HIP reads the values through the permutation inside
// the SpMM (ofx_spmm_csr_gathered); the CPU kernel gathers them into its tmp buffer first and
// runs the kCPU SpMM on the copy (same bits).
template <DeviceType device_type>
class SpmmCsrGatheredKernel final : public user_op::OpKernel, public user_op::CudaGraphSupport {
 public:
  SpmmCsrGatheredKernel() = default;
  ~SpmmCsrGatheredKernel() override = default;

  std::shared_ptr<user_op::OpKernelCache> InitOpKernelCache(
      user_op::KernelCacheContext* ctx) const override {
    return CreateSpmmCsrOpKernelCache(ctx);
  }

  // The plans of static CSRs (the autograd's cached A^T: static while its cache entry lives).
  std::shared_ptr<user_op::OpKernelState> CreateOpKernelState(
      user_op::KernelInitContext* ctx) const override {
    if (device_type != DeviceType::kHIP) return nullptr;
    return std::make_shared<SpmmCsrPlanState>(!ctx->has_stream_name_hint());
  }

  bool AlwaysComputeWhenAllOutputsEmpty() const override { return false; }

 private:
  using user_op::OpKernel::Compute;
  void Compute(user_op::KernelComputeContext* ctx, user_op::OpKernelState* state,
               const user_op::OpKernelCache* cache) const override {
    const user_op::Tensor* row_ptr = ctx->Tensor4ArgNameAndIndex("a_csr_row_ptr", 0);
    const user_op::Tensor* col_idx = ctx->Tensor4ArgNameAndIndex("a_csr_col_idx", 0);
    const user_op::Tensor* values = ctx->Tensor4ArgNameAndIndex("a_csr_values", 0);
    const user_op::Tensor* perm = ctx->Tensor4ArgNameAndIndex("values_perm", 0);
    const user_op::Tensor* b = ctx->Tensor4ArgNameAndIndex("b", 0);
    user_op::Tensor* out = ctx->Tensor4ArgNameAndIndex("out", 0);
    user_op::Tensor* tmp = ctx->Tensor4ArgNameAndIndex("tmp_buffer", 0);
    const int64_t m = ctx->Attr<int64_t>("a_num_rows");
    const int64_t k = ctx->Attr<int64_t>("a_num_cols");
    const int64_t n = out->shape_view().At(1);
    const int64_t nnz = col_idx->shape_view().elem_cnt();
    int64_t row_begin = 0, row_end = m;
    const auto* range = dynamic_cast<const SpmmCsrOpKernelCache*>(cache);
    OFX_KERNEL_CHECK(cache == nullptr || range != nullptr, "unexpected kernel cache type");
    if (range != nullptr) {
      row_begin = range->lower();
      row_end = range->upper();
    }
    ofx_spmm_options opts = OptionsOf(range);
    OFX_KERNEL_CHECK(out->shape_view().At(0) == row_end - row_begin,
                     "out rows " << out->shape_view().At(0) << " != row range "
                                 << row_end - row_begin);
    const int idx_dt = DtCode(row_ptr->data_type());
    const int val_dt = DtCode(values->data_type());
    void* ws = tmp ? tmp->mut_dptr() : nullptr;
    size_t ws_bytes = tmp ? (size_t)tmp->shape_view().elem_cnt() : 0;
    int rc;
    if (device_type == DeviceType::kHIP) {
      ep::HipStream* hs = ctx->stream()->As<ep::HipStream>();
      auto* plans = dynamic_cast<SpmmCsrPlanState*>(state);
      const int64_t static_csr = ctx->Attr<int64_t>("static_csr");
      StaticPlan sp;
      if (plans != nullptr && static_csr != 0)
        UseStaticPlan(plans, static_csr, hs, row_ptr->dptr(), idx_dt, val_dt, m, k, n, nnz,
                      row_begin, row_end, "spmm_csr_gathered", &opts, &ws, &ws_bytes, &sp);
      rc = ofx_spmm_csr_gathered(hs->hip_stream(), idx_dt, val_dt, m, k, n, nnz, row_ptr->dptr(),
                                 col_idx->dptr(), values->dptr(), perm->dptr(), b->dptr(),
                                 b->row_stride(), out->mut_dptr(), out->row_stride(), row_begin,
                                 row_end, ws, ws_bytes, &opts);
      if (rc != OFX_OK && sp.keyed) plans->Drop(sp.key, hs->IsGraphCapturing());
    } else {
      const size_t vbytes = (size_t)nnz * (size_t)GetSizeOfDataType(values->data_type());
      OFX_KERNEL_CHECK(nnz == 0 || ws_bytes >= vbytes, "tmp buffer smaller than the values");
      rc = ofx_gather_values_host(idx_dt, val_dt, nnz, perm->dptr(), values->dptr(), ws);
      if (rc == OFX_OK)
        rc = ofx_spmm_csr_cpu(ctx->stream()->As<ep::CpuStream>()->num_threads(), idx_dt, val_dt,
                              m, k, n, nnz, row_ptr->dptr(), col_idx->dptr(), ws, b->dptr(),
                              b->row_stride(), out->mut_dptr(), out->row_stride(), row_begin,
                              row_end, &opts);
    }
    OFX_KERNEL_CHECK(rc == OFX_OK,
                     "spmm_csr_gathered kernel failed (" << rc << "): " << ofx_last_error());
  }
};

size_t InferSpmmCsrGatheredCpuTmpSize(user_op::InferSizeContext* ctx) {
  const user_op::TensorDesc& values = ctx->InputTensorDesc("a_csr_values", 0);
  return (size_t)values.shape().elem_cnt() * (size_t)GetSizeOfDataType(values.data_type());
}

// Workspace for the physical width with the logical width's schedule (as Compute launches it).
size_t InferSpmmCsrTmpSize(user_op::InferSizeContext* ctx) {
  const user_op::TensorDesc& row_ptr = ctx->InputTensorDesc("a_csr_row_ptr", 0);
  const user_op::TensorDesc& col_idx = ctx->InputTensorDesc("a_csr_col_idx", 0);
  const user_op::TensorDesc& b = ctx->InputTensorDesc("b", 0);
  const user_op::TensorDesc* out_logical = ctx->LogicalTensorDesc4ArgNameAndIndex("out", 0);
  ofx_spmm_options o = OFX_SPMM_OPTIONS_INIT;
  if (out_logical != nullptr) o.split_threshold = ofx_spmm_default_split(out_logical->shape().At(1));
  size_t bytes = 0;
  const int rc = ofx_spmm_csr_workspace_size(
      DtCode(row_ptr.data_type()), DtCode(b.data_type()), ctx->Attr<int64_t>("a_num_rows"),
      ctx->Attr<int64_t>("a_num_cols"), b.shape().At(1), col_idx.shape().At(0), &o, &bytes);
  return rc == OFX_OK ? bytes : 0;
}

}  // namespace

#define REGISTER_SPMM_CSR_KERNEL_OF(op, kernel, device, dtype, itype)                          \
  REGISTER_USER_KERNEL(op)                                                                    \
      .SetCreateFn<kernel<device>>()                                                          \
      .SetIsMatchedHob((user_op::HobDeviceType() == device)                                   \
                       && (user_op::HobDataType("out", 0) == dtype)                           \
                       && (user_op::HobDataType("a_csr_row_ptr", 0) == itype))                \
      .SetInferTmpSizeFn(device == DeviceType::kHIP                                           \
                             ? std::function<size_t(user_op::InferSizeContext*)>(             \
                                   InferSpmmCsrTmpSize)                                       \
                             : std::function<size_t(user_op::InferSizeContext*)>(             \
                                   [](user_op::InferSizeContext*) -> size_t { return 0; }));

#define REGISTER_SPMM_CSR_KERNEL(device, dtype, itype)                                     \
  REGISTER_SPMM_CSR_KERNEL_OF("spmm_csr", SpmmCsrKernel, device, dtype, itype)            \
  REGISTER_SPMM_CSR_KERNEL_OF("fused_spmm_csr", FusedSpmmCsrKernel, device, dtype, itype)

#define REGISTER_SPMM_CSR_KERNEL_ALL_INDEX(device, dtype) \
  REGISTER_SPMM_CSR_KERNEL(device, dtype, kInt32)         \
  REGISTER_SPMM_CSR_KERNEL(device, dtype, kInt64)

#define REGISTER_SPMM_CSR_KERNEL_ALL(device)              \
  REGISTER_SPMM_CSR_KERNEL_ALL_INDEX(device, kFloat)      \
  REGISTER_SPMM_CSR_KERNEL_ALL_INDEX(device, kDouble)     \
  REGISTER_SPMM_CSR_KERNEL_ALL_INDEX(device, kFloat16)    \
  REGISTER_SPMM_CSR_KERNEL_ALL_INDEX(device, kBFloat16)

REGISTER_SPMM_CSR_KERNEL_ALL(DeviceType::kCPU)
REGISTER_SPMM_CSR_KERNEL_ALL(DeviceType::kHIP)

#define REGISTER_SPMM_CSR_GATHERED_KERNEL(device, dtype, itype)                                \
  REGISTER_USER_KERNEL("spmm_csr_gathered")                                                   \
      .SetCreateFn<SpmmCsrGatheredKernel<device>>()                                           \
      .SetIsMatchedHob((user_op::HobDeviceType() == device)                                   \
                       && (user_op::HobDataType("out", 0) == dtype)                           \
                       && (user_op::HobDataType("a_csr_row_ptr", 0) == itype))                \
      .SetInferTmpSizeFn(device == DeviceType::kHIP ? InferSpmmCsrTmpSize                     \
                                                    : InferSpmmCsrGatheredCpuTmpSize);

#define REGISTER_SPMM_CSR_GATHERED_KERNEL_ALL(device)                 \
  REGISTER_SPMM_CSR_GATHERED_KERNEL(device, kFloat, kInt32)           \
  REGISTER_SPMM_CSR_GATHERED_KERNEL(device, kFloat, kInt64)           \
  REGISTER_SPMM_CSR_GATHERED_KERNEL(device, kDouble, kInt32)          \
  REGISTER_SPMM_CSR_GATHERED_KERNEL(device, kDouble, kInt64)          \
  REGISTER_SPMM_CSR_GATHERED_KERNEL(device, kFloat16, kInt32)         \
  REGISTER_SPMM_CSR_GATHERED_KERNEL(device, kFloat16, kInt64)         \
  REGISTER_SPMM_CSR_GATHERED_KERNEL(device, kBFloat16, kInt32)        \
  REGISTER_SPMM_CSR_GATHERED_KERNEL(device, kBFloat16, kInt64)

REGISTER_SPMM_CSR_GATHERED_KERNEL_ALL(DeviceType::kCPU)
REGISTER_SPMM_CSR_GATHERED_KERNEL_ALL(DeviceType::kHIP)

}  // namespace oneflow
