/*
 * sddmm_kernel.cpp — kernels of the gradient ops "sddmm_csr" and "csr_transpose" for
 * DeviceType::kCPU and DeviceType::kHIP (same registration pattern as spmm_kernel.cpp; device
 * work through the C-ABI of include/ofx_spmm.h).
 */
#include "oneflow/core/framework/framework.h"
#include "oneflow/user/kernels/spmm_plan_state.h"
#include "ofx_spmm.h"

namespace oneflow {

namespace {

int DtCode(DataType dt) { return static_cast<int>(dt); }

template <DeviceType device_type>
class SddmmCsrKernel final : public user_op::OpKernel, public user_op::CudaGraphSupport {
 public:
  // The SDDMM's plans of static CSRs (attr static_csr, as spmm_csr's: spmm_plan_state.h).
  std::shared_ptr<user_op::OpKernelState> CreateOpKernelState(
      user_op::KernelInitContext* ctx) const override {
    if (device_type != DeviceType::kHIP) return nullptr;
    return std::make_shared<SpmmCsrPlanState>(!ctx->has_stream_name_hint());
  }

  bool AlwaysComputeWhenAllOutputsEmpty() const override { return false; }

 private:
  using user_op::OpKernel::Compute;
  void Compute(user_op::KernelComputeContext* ctx, user_op::OpKernelState* state,
               const user_op::OpKernelCache*) const override {
    const user_op::Tensor* row_ptr = ctx->Tensor4ArgNameAndIndex("a_csr_row_ptr", 0);
    const user_op::Tensor* col_idx = ctx->Tensor4ArgNameAndIndex("a_csr_col_idx", 0);
    const user_op::Tensor* a = ctx->Tensor4ArgNameAndIndex("a", 0);
    const user_op::Tensor* b = ctx->Tensor4ArgNameAndIndex("b", 0);
    user_op::Tensor* out = ctx->Tensor4ArgNameAndIndex("out", 0);
    const int64_t m = ctx->Attr<int64_t>("a_num_rows");
    const int64_t k = ctx->Attr<int64_t>("a_num_cols");
    const int64_t n = b->shape_view().At(1);
    const int64_t nnz = col_idx->shape_view().elem_cnt();
    const int idx_dt = DtCode(row_ptr->data_type()), val_dt = DtCode(b->data_type());
    int rc;
    if (device_type == DeviceType::kHIP) {
      user_op::Tensor* tmp = ctx->Tensor4ArgNameAndIndex("tmp_buffer", 0);
      void* ws = tmp ? tmp->mut_dptr() : nullptr;
      size_t ws_bytes = tmp ? (size_t)tmp->shape_view().elem_cnt() : 0;
      ep::HipStream* hs = ctx->stream()->As<ep::HipStream>();
      void* stream = hs->hip_stream();
      ofx_spmm_options opts = OFX_SPMM_OPTIONS_INIT;
      auto* plans = dynamic_cast<SpmmCsrPlanState*>(state);
      const int64_t static_csr = ctx->Attr<int64_t>("static_csr");
      StaticPlan sp;
      if (plans != nullptr && static_csr != 0 && m > 0 && n > 0 && nnz > 0) {
        size_t need = 0;
        rc = ofx_sddmm_csr_workspace_size(idx_dt, val_dt, m, n, nnz, &need);
        OFX_KERNEL_CHECK(rc == OFX_OK, "sddmm_csr workspace query failed: " << ofx_last_error());
        // the SDDMM's schedule is a function of n alone: no options in the key
        const SpmmCsrPlanState::Key key{static_csr, row_ptr->dptr(),
                                        plans->key_on_stream() ? stream : nullptr,
                                        hs->device_index(), idx_dt, val_dt, m, k, n, nnz, 0, m,
                                        0, 0, 0, 0};
        auto plan = [&](void* sws, size_t bytes) {
          return ofx_sddmm_csr_plan(stream, idx_dt, val_dt, m, n, nnz, row_ptr->dptr(), 0, m, sws,
                                    bytes);
        };
        if (UseStaticPlan(plans, key, need, hs->IsGraphCapturing(), "sddmm_csr", plan, &ws,
                          &ws_bytes, &sp))
          opts.planned = 1;
      }
      rc = ofx_sddmm_csr_ex(stream, idx_dt, val_dt, m, k, n, nnz, row_ptr->dptr(),
                            col_idx->dptr(), a->dptr(), a->row_stride(), b->dptr(),
                            b->row_stride(), out->mut_dptr(), 0, m, ws, ws_bytes, &opts);
      if (rc != OFX_OK && sp.keyed) plans->Drop(sp.key, hs->IsGraphCapturing());
    } else {
      rc = ofx_sddmm_csr_cpu(ctx->stream()->As<ep::CpuStream>()->num_threads(), idx_dt, val_dt, m,
                             k, n, nnz, row_ptr->dptr(), col_idx->dptr(), a->dptr(),
                             a->row_stride(), b->dptr(), b->row_stride(), out->mut_dptr(), 0, m);
    }
    OFX_KERNEL_CHECK(rc == OFX_OK, "sddmm_csr kernel failed (" << rc << "): " << ofx_last_error());
  }
};

template <DeviceType device_type>
class CsrTransposeKernel final : public user_op::OpKernel {
 public:
  bool AlwaysComputeWhenAllOutputsEmpty() const override { return true; }

 private:
  using user_op::OpKernel::Compute;
  void Compute(user_op::KernelComputeContext* ctx, user_op::OpKernelState*,
               const user_op::OpKernelCache*) const override {
    const user_op::Tensor* row_ptr = ctx->Tensor4ArgNameAndIndex("a_csr_row_ptr", 0);
    const user_op::Tensor* col_idx = ctx->Tensor4ArgNameAndIndex("a_csr_col_idx", 0);
    user_op::Tensor* out_rp = ctx->Tensor4ArgNameAndIndex("out_row_ptr", 0);
    user_op::Tensor* out_ci = ctx->Tensor4ArgNameAndIndex("out_col_idx", 0);
    user_op::Tensor* out_perm = ctx->Tensor4ArgNameAndIndex("out_perm", 0);
    const int64_t m = ctx->Attr<int64_t>("a_num_rows");
    const int64_t k = ctx->Attr<int64_t>("a_num_cols");
    const int64_t nnz = col_idx->shape_view().elem_cnt();
    const int idx_dt = DtCode(row_ptr->data_type());
    int rc;
    if (device_type == DeviceType::kHIP) {
      user_op::Tensor* tmp = ctx->Tensor4ArgNameAndIndex("tmp_buffer", 0);
      rc = ofx_csr_transpose(ctx->stream()->As<ep::HipStream>()->hip_stream(), idx_dt, m, k, nnz,
                             row_ptr->dptr(), col_idx->dptr(), out_rp->mut_dptr(),
                             out_ci->mut_dptr(), out_perm->mut_dptr(),
                             tmp ? tmp->mut_dptr() : nullptr,
                             tmp ? (size_t)tmp->shape_view().elem_cnt() : 0);
    } else {
      rc = ofx_csr_transpose_cpu(idx_dt, m, k, nnz, row_ptr->dptr(), col_idx->dptr(),
                                 out_rp->mut_dptr(), out_ci->mut_dptr(), out_perm->mut_dptr());
    }
    OFX_KERNEL_CHECK(rc == OFX_OK, "csr_transpose kernel failed (" << rc << "): " << ofx_last_error());
  }
};

size_t InferSddmmTmpSize(user_op::InferSizeContext* ctx) {
  const user_op::TensorDesc& row_ptr = ctx->InputTensorDesc("a_csr_row_ptr", 0);
  const user_op::TensorDesc& col_idx = ctx->InputTensorDesc("a_csr_col_idx", 0);
  const user_op::TensorDesc& b = ctx->InputTensorDesc("b", 0);
  size_t bytes = 0;
  const int rc = ofx_sddmm_csr_workspace_size(DtCode(row_ptr.data_type()), DtCode(b.data_type()),
                                              ctx->Attr<int64_t>("a_num_rows"), b.shape().At(1),
                                              col_idx.shape().At(0), &bytes);
  return rc == OFX_OK ? bytes : 0;
}

size_t InferTransposeTmpSize(user_op::InferSizeContext* ctx) {
  const user_op::TensorDesc& row_ptr = ctx->InputTensorDesc("a_csr_row_ptr", 0);
  const user_op::TensorDesc& col_idx = ctx->InputTensorDesc("a_csr_col_idx", 0);
  size_t bytes = 0;
  const int rc = ofx_csr_transpose_workspace_size(
      DtCode(row_ptr.data_type()), ctx->Attr<int64_t>("a_num_rows"),
      ctx->Attr<int64_t>("a_num_cols"), col_idx.shape().At(0), &bytes);
  return rc == OFX_OK ? bytes : 0;
}

size_t NoTmp(user_op::InferSizeContext*) { return 0; }

}  // namespace

#define REGISTER_SDDMM_CSR_KERNEL(device, dtype, itype)                                       \
  REGISTER_USER_KERNEL("sddmm_csr")                                                         \
      .SetCreateFn<SddmmCsrKernel<device>>()                                                \
      .SetIsMatchedHob((user_op::HobDeviceType() == device)                                 \
                       && (user_op::HobDataType("out", 0) == dtype)                         \
                       && (user_op::HobDataType("a_csr_row_ptr", 0) == itype))              \
      .SetInferTmpSizeFn(device == DeviceType::kHIP ? InferSddmmTmpSize : NoTmp);

#define REGISTER_SDDMM_CSR_KERNEL_ALL(device)                                                 \
  REGISTER_SDDMM_CSR_KERNEL(device, kFloat, kInt32)                                          \
  REGISTER_SDDMM_CSR_KERNEL(device, kFloat, kInt64)                                          \
  REGISTER_SDDMM_CSR_KERNEL(device, kDouble, kInt32)                                         \
  REGISTER_SDDMM_CSR_KERNEL(device, kDouble, kInt64)                                         \
  REGISTER_SDDMM_CSR_KERNEL(device, kFloat16, kInt32)                                        \
  REGISTER_SDDMM_CSR_KERNEL(device, kFloat16, kInt64)                                        \
  REGISTER_SDDMM_CSR_KERNEL(device, kBFloat16, kInt32)                                       \
  REGISTER_SDDMM_CSR_KERNEL(device, kBFloat16, kInt64)

REGISTER_SDDMM_CSR_KERNEL_ALL(DeviceType::kCPU)
REGISTER_SDDMM_CSR_KERNEL_ALL(DeviceType::kHIP)

#define REGISTER_CSR_TRANSPOSE_KERNEL(device, itype)                                          \
  REGISTER_USER_KERNEL("csr_transpose")                                                     \
      .SetCreateFn<CsrTransposeKernel<device>>()                                            \
      .SetIsMatchedHob((user_op::HobDeviceType() == device)                                 \
                       && (user_op::HobDataType("a_csr_row_ptr", 0) == itype))              \
      .SetInferTmpSizeFn(device == DeviceType::kHIP ? InferTransposeTmpSize : NoTmp);

REGISTER_CSR_TRANSPOSE_KERNEL(DeviceType::kCPU, kInt32)
REGISTER_CSR_TRANSPOSE_KERNEL(DeviceType::kCPU, kInt64)
REGISTER_CSR_TRANSPOSE_KERNEL(DeviceType::kHIP, kInt32)
REGISTER_CSR_TRANSPOSE_KERNEL(DeviceType::kHIP, kInt64)

}  // namespace oneflow
