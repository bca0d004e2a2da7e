// hip_all_gather.cpp — ccl::AllGather for DeviceType::kHIP: ncclAllGather on the kernel's HIP
// stream over the placement's RCCL communicator.  Registered the way CudaAllGather is
// (oneflow/user/kernels/collective_communication/cuda/cuda_all_gather.cpp:25-47); dtypes as
// oneflow/core/device/nccl_util.h:37-60.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include "oneflow/user/kernels/collective_communication/hip/hip_communication_context.h"
#include "oneflow/user/kernels/collective_communication/include/all_gather.h"

namespace oneflow {
namespace ccl {

namespace {
ncclDataType_t GetRcclDataType(DataType dt) {
  switch (dt) {
    case kChar: case kInt8: return ncclInt8;
    case kUInt8: case kBool: return ncclUint8;
    case kInt32: return ncclInt32;
    case kInt64: return ncclInt64;
    case kFloat: return ncclFloat32;
    case kDouble: return ncclFloat64;
    case kFloat16: return ncclFloat16;
    case kBFloat16: return ncclBfloat16;
    default: OFX_KERNEL_CHECK(false, "no RCCL type for " << DataType_Name(dt));
  }
  return ncclInt8;
}
}  // namespace

class HipAllGather final : public AllGather {
 public:
  HipAllGather() = default;
  ~HipAllGather() override = default;

  void Init(DataType datatype) override { rccl_datatype_ = GetRcclDataType(datatype); }

  void Launch(ep::Stream* stream, const void* in, void* out, size_t elem_cnt,
              const std::shared_ptr<CommunicationContext>& communication_ctx) const override {
    const auto hip_ctx = std::dynamic_pointer_cast<HipCommunicationContext>(communication_ctx);
    OFX_KERNEL_CHECK(hip_ctx != nullptr, "HipAllGather needs a HipCommunicationContext");
    OFX_KERNEL_CHECK(stream->device_type() == DeviceType::kHIP, "HipAllGather on a non-HIP stream");
    const ncclResult_t r =
        ncclAllGather(in, out, elem_cnt, rccl_datatype_, static_cast<ncclComm_t>(hip_ctx->rccl_comm()),
                      static_cast<hipStream_t>(stream->As<ep::HipStream>()->hip_stream()));
    OFX_KERNEL_CHECK(r == ncclSuccess, "ncclAllGather: " << ncclGetErrorString(r));
  }

 private:
  ncclDataType_t rccl_datatype_ = ncclFloat32;
};

REGISTER_COLLECTIVE_COMMUNICATION(DeviceType::kHIP, AllGather, HipAllGather);

}  // namespace ccl
}  // namespace oneflow
