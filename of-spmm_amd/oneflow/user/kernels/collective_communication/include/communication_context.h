// communication_context.h — per-placement communicator of a device type
// (oneflow/user/kernels/collective_communication/include/communication_context.h): created once
// per placement by the eager ccl kernels' cache and held by them.
#ifndef OFX_ONEFLOW_CCL_COMMUNICATION_CONTEXT_H_
#define OFX_ONEFLOW_CCL_COMMUNICATION_CONTEXT_H_

#include <memory>

#include "oneflow/core/common/auto_registration_factory.h"

namespace oneflow {
namespace ccl {

class CommunicationContext {
 public:
  CommunicationContext() = default;
  virtual ~CommunicationContext() = default;
  virtual void Init(const ParallelDesc& parallel_desc) = 0;
};

inline bool IsCommunicationContextRegistered(DeviceType device_type) {
  return IsClassRegistered<DeviceType, CommunicationContext>(device_type);
}

// Throws KernelCheckError when the placement's device type differs or has no communicator.
inline std::shared_ptr<CommunicationContext> NewCommunicationContext(
    DeviceType device_type, const ParallelDesc& parallel_desc) {
  OFX_KERNEL_CHECK(device_type == parallel_desc.device_type(),
                   "device_type does not match the placement (" << DeviceTypeName(device_type)
                       << " vs. " << DeviceTypeName(parallel_desc.device_type()) << ")");
  std::shared_ptr<CommunicationContext> ctx(NewObj<DeviceType, CommunicationContext>(device_type));
  OFX_KERNEL_CHECK(ctx != nullptr, "no communication context for " << DeviceTypeName(device_type));
  ctx->Init(parallel_desc);
  return ctx;
}

#define REGISTER_COLLECTIVE_COMMUNICATION_COMMUNICATOR(device, Derived) \
  REGISTER_CLASS(::oneflow::DeviceType, device, ::oneflow::ccl::CommunicationContext, Derived)

}  // namespace ccl
}  // namespace oneflow

#endif  // OFX_ONEFLOW_CCL_COMMUNICATION_CONTEXT_H_
