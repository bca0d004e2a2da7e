/*
 * eager_ccl_kernel.cpp — kernel of op "eager_ccl_all_gather" for every device type that has a
 * registered ccl::AllGather and communication context (kHIP: RCCL, kCPU: host ring).  The
 * pattern of oneflow/user/kernels/eager_ccl_kernel.cpp:20-75,177-207: a custom HOB on the
 * collective registry, a kernel cache holding the placement's communication context, and
 * Compute = AllGather::Launch(stream, in, out, in elem_cnt, ctx).  The shim hands the cache
 * context the placement itself instead of its "parallel_conf" text attribute.
 */
#include "oneflow/core/framework/framework.h"
#include "oneflow/user/kernels/collective_communication/include/all_gather.h"

namespace oneflow {

namespace {

auto AllGatherCollectiveCommunicationExists() {
  return hob::make_custom("AllGatherCollectiveCommunicationExists",
                          [](const user_op::KernelRegContext& ctx) {
                            const DeviceType device_type = ctx.device_type();
                            return ccl::IsCommunicationContextRegistered(device_type) &&
                                   ccl::IsAllGatherRegistered(device_type);
                          });
}

class EagerCclOpKernelCache final : public user_op::OpKernelCache {
 public:
  explicit EagerCclOpKernelCache(user_op::KernelCacheContext* ctx) {
    communication_ctx_ = ccl::NewCommunicationContext(ctx->device_type(), ctx->parallel_desc());
  }
  const std::shared_ptr<ccl::CommunicationContext>& communication_ctx() const {
    return communication_ctx_;
  }

 private:
  std::shared_ptr<ccl::CommunicationContext> communication_ctx_;
};

}  // namespace

class EagerCclAllGatherKernel final : public user_op::OpKernel {
 public:
  std::shared_ptr<user_op::OpKernelCache> InitOpKernelCache(
      user_op::KernelCacheContext* ctx) const override {
    return std::make_shared<EagerCclOpKernelCache>(ctx);
  }

 private:
  using user_op::OpKernel::Compute;
  void Compute(user_op::KernelComputeContext* ctx, user_op::OpKernelState*,
               const user_op::OpKernelCache* cache) const override {
    auto* kernel_cache = dynamic_cast<const EagerCclOpKernelCache*>(cache);
    OFX_KERNEL_CHECK(kernel_cache != nullptr, "eager_ccl_all_gather: no kernel cache");
    const user_op::Tensor* in = ctx->Tensor4ArgNameAndIndex("in", 0);
    user_op::Tensor* out = ctx->Tensor4ArgNameAndIndex("out", 0);
    OFX_KERNEL_CHECK(in->data_type() == out->data_type(), "in/out dtypes differ");
    std::unique_ptr<ccl::AllGather> all_gather =
        ccl::NewCollectiveCommunication<ccl::AllGather>(ctx->device_type(), in->data_type());
    OFX_KERNEL_CHECK(all_gather != nullptr, "no AllGather for " << DeviceTypeName(ctx->device_type()));
    all_gather->Launch(ctx->stream(), in->dptr(), out->mut_dptr(), in->shape_view().elem_cnt(),
                       kernel_cache->communication_ctx());
  }
  bool AlwaysComputeWhenAllOutputsEmpty() const override { return false; }
};

REGISTER_USER_KERNEL("eager_ccl_all_gather")
    .SetCreateFn<EagerCclAllGatherKernel>()
    .SetIsMatchedHob(AllGatherCollectiveCommunicationExists());

}  // namespace oneflow
