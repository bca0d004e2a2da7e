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
#include "oneflow/core/framework/framework.h"
#include "oneflow/core/functional/spmm_functor.h"
#include "oneflow/user/kernels/spmm_plan_state.h"
#include "ofx_spmm.h"

namespace oneflow {

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

// The static plan of an spmm_csr-family launch: key and workspace size from the launch's
// shapes, row range and schedule; the plan built by ofx_spmm_csr_plan.
void UseStaticSpmmPlan(SpmmCsrPlanState* plans, int64_t static_csr, ep::HipStream* hs,
                       const void* row_ptr, int idx_dt, int val_dt, int64_t m, int64_t k,
                       int64_t n, int64_t nnz, int64_t row_begin, int64_t row_end,
                       const char* op_name, ofx_spmm_options* opts, void** ws, size_t* ws_bytes,
                       StaticPlan* sp) {
  if (row_end <= row_begin || n <= 0) return;
  size_t need = 0;
  const int rc = ofx_spmm_csr_workspace_size(idx_dt, val_dt, m, k, n, nnz, opts, &need);
  OFX_KERNEL_CHECK(rc == OFX_OK, op_name << " workspace query failed: " << ofx_last_error());
  void* stream = hs->hip_stream();
  const SpmmCsrPlanState::Key key{static_csr, row_ptr, plans->key_on_stream() ? stream : nullptr,
                                  hs->device_index(), idx_dt, val_dt, m, k, n, nnz, row_begin,
                                  row_end, opts->split_threshold, opts->chunk,
                                  opts->heavy_threshold, opts->range_nnz};
  auto plan = [&](void* sws, size_t bytes) {
    return ofx_spmm_csr_plan(stream, idx_dt, val_dt, m, k, n, nnz, row_ptr, row_begin, row_end,
                             sws, bytes, opts);
  };
  if (UseStaticPlan(plans, key, need, hs->IsGraphCapturing(), op_name, plan, ws, ws_bytes, sp))
    opts->planned = 1;
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
      UseStaticSpmmPlan(plans, static_csr, hs, row_ptr->dptr(), idx_dt, val_dt, m, k, n, nnz,
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
        UseStaticSpmmPlan(plans, static_csr, hs, row_ptr->dptr(), idx_dt, val_dt, m, k, n, nnz,
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
