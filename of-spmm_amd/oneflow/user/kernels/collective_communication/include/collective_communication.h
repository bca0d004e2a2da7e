// collective_communication.h — the device-neutral collective interface of OneFlow's user kernels
// (oneflow/user/kernels/collective_communication/include/collective_communication.h), written for
// the shim: one implementation per DeviceType, created through the keyed registry.  kHIP is
// served by RCCL (hip/), kCPU by a ring over the host transport (cpu/).
#ifndef OFX_ONEFLOW_CCL_COLLECTIVE_COMMUNICATION_H_
#define OFX_ONEFLOW_CCL_COLLECTIVE_COMMUNICATION_H_

#include <memory>
#include <utility>

#include "oneflow/core/common/auto_registration_factory.h"
#include "oneflow/user/kernels/collective_communication/include/communication_context.h"

namespace oneflow {
namespace ccl {

class CollectiveCommunication {
 public:
  CollectiveCommunication() = default;
  CollectiveCommunication(const CollectiveCommunication&) = delete;
  CollectiveCommunication& operator=(const CollectiveCommunication&) = delete;
  virtual ~CollectiveCommunication() = default;
};

// The registered implementation of `CollectiveCommunicationType` for `device_type`, initialised
// with `args` (e.g. the DataType); nullptr if the device type has none.
template <typename CollectiveCommunicationType, typename... Args>
std::unique_ptr<CollectiveCommunicationType> NewCollectiveCommunication(DeviceType device_type,
                                                                       Args&&... args) {
  std::unique_ptr<CollectiveCommunicationType> entry =
      NewObjUniquePtr<DeviceType, CollectiveCommunicationType>(device_type);
  if (!entry) return nullptr;
  entry->Init(std::forward<Args>(args)...);
  return entry;
}

#define REGISTER_COLLECTIVE_COMMUNICATION(device, Base, Derived) \
  REGISTER_CLASS(::oneflow::DeviceType, device, Base, Derived)

}  // namespace ccl
}  // namespace oneflow

#endif  // OFX_ONEFLOW_CCL_COLLECTIVE_COMMUNICATION_H_
