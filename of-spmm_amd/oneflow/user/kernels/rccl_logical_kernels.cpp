/*
 * rccl_logical_kernels.cpp — kernel of the lazy graph's "_nccl_logical_all_gather" for
 * DeviceType::kHIP: the op the compiler inserts for an S(0) -> B edge
 * (insert_nccl_logical_op_pass.cpp:189-198), i.e. the B operand of a row-split spmm_csr in an
 * nn.Graph.  The reference registers it for kCUDA only (oneflow/user/kernels/
 * nccl_logical_kernels.cpp:175-205 Compute, :512-514 registration); this is the kHIP kernel:
 * a kernel state holding the placement's RCCL communicator for the op's stream name
 * (NcclLogicalKernelCommState, :27-57), Compute = ncclAllGather on the kernel's HIP stream.
 */
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include "oneflow/core/framework/framework.h"
#include "oneflow/core/job/eager_rccl_comm_manager.h"

namespace oneflow {

namespace {

ncclDataType_t RcclDataType(DataType dt) {
  switch (dt) {
    case kInt32: return ncclInt32;
    case kInt64: return ncclInt64;
    case kFloat: return ncclFloat32;
    case kDouble: return ncclFloat64;
    case kFloat16: return ncclFloat16;
    case kBFloat16: return ncclBfloat16;
    case kChar: case kInt8: return ncclInt8;
    case kUInt8: case kBool: return ncclUint8;
    default: OFX_KERNEL_CHECK(false, "no RCCL type for " << DataType_Name(dt));
  }
  return ncclInt8;
}

class RcclLogicalKernelCommState : public user_op::OpKernelState {
 public:
  explicit RcclLogicalKernelCommState(user_op::KernelInitContext* ctx)
      : stream_name_(EagerRcclCommMgr::kDefaultStreamName), parallel_desc_(ctx->parallel_desc()) {
    if (ctx->has_stream_name_hint()) stream_name_ = ctx->stream_name_hint();
  }
  void* comm() {
    if (!is_init_) {
      DeviceSet device_set;
      for (int64_t p = 0; p < parallel_desc_.parallel_num(); ++p)
        device_set.emplace(parallel_desc_.MachineId4ParallelId(p),
                           parallel_desc_.DeviceId4ParallelId(p));
      comm_ = EagerRcclCommMgr::Get()->GetCommForDeviceAndStreamName(device_set, stream_name_);
      is_init_ = true;
    }
    return comm_;
  }
  const std::string& stream_name() const { return stream_name_; }

 private:
  bool is_init_ = false;
  std::string stream_name_;
  ParallelDesc parallel_desc_;
  void* comm_ = nullptr;
};

class RcclLogicalAllGatherKernel final : public user_op::OpKernel {
 public:
  std::shared_ptr<user_op::OpKernelState> CreateOpKernelState(
      user_op::KernelInitContext* ctx) const override {
    return std::make_shared<RcclLogicalKernelCommState>(ctx);
  }

 private:
  using user_op::OpKernel::Compute;
  void Compute(user_op::KernelComputeContext* ctx, user_op::OpKernelState* state,
               const user_op::OpKernelCache*) const override {
    auto* comm_state = dynamic_cast<RcclLogicalKernelCommState*>(state);
    OFX_KERNEL_CHECK(comm_state != nullptr, "_nccl_logical_all_gather: no kernel state");
    const user_op::Tensor* in = ctx->Tensor4ArgNameAndIndex("in", 0);
    user_op::Tensor* out = ctx->Tensor4ArgNameAndIndex("out", 0);
    OFX_KERNEL_CHECK(in->data_type() == out->data_type(), "in/out dtypes differ");
    const int64_t num_ranks = ctx->parallel_ctx().parallel_num();
    OFX_KERNEL_CHECK(in->shape_view().elem_cnt() * num_ranks == out->shape_view().elem_cnt(),
                     "in " << in->shape_view().ToString() << " x " << num_ranks << " ranks != out "
                           << out->shape_view().ToString());
    const ncclResult_t r = ncclAllGather(
        in->dptr(), out->mut_dptr(), (size_t)in->shape_view().elem_cnt(),
        RcclDataType(in->data_type()), static_cast<ncclComm_t>(comm_state->comm()),
        static_cast<hipStream_t>(ctx->stream()->As<ep::HipStream>()->hip_stream()));
    OFX_KERNEL_CHECK(r == ncclSuccess, "ncclAllGather: " << ncclGetErrorString(r));
  }
  bool AlwaysComputeWhenAllOutputsEmpty() const override { return false; }
};

}  // namespace

REGISTER_USER_KERNEL("_nccl_logical_all_gather")
    .SetCreateFn<RcclLogicalAllGatherKernel>()
    .SetIsMatchedHob(user_op::HobDeviceType() == DeviceType::kHIP);

}  // namespace oneflow
