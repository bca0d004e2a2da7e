// all_gather.h — ccl::AllGather (oneflow/user/kernels/collective_communication/include/
// all_gather.h:24-38): out = the concatenation of every rank's `elem_cnt` elements of `in`, in
// parallel-id order; `in` may be this rank's slot of `out` (in place).
#ifndef OFX_ONEFLOW_CCL_ALL_GATHER_H_
#define OFX_ONEFLOW_CCL_ALL_GATHER_H_

#include "oneflow/user/kernels/collective_communication/include/collective_communication.h"

namespace oneflow {
namespace ccl {

class AllGather : public CollectiveCommunication {
 public:
  AllGather() = default;
  ~AllGather() override = default;
  virtual void Init(DataType dtype) = 0;
  virtual void Launch(ep::Stream* stream, const void* in, void* out, size_t elem_cnt,
                      const std::shared_ptr<CommunicationContext>& communicator) const = 0;
};

inline bool IsAllGatherRegistered(DeviceType device_type) {
  return IsClassRegistered<DeviceType, AllGather>(device_type);
}

}  // namespace ccl
}  // namespace oneflow

#endif  // OFX_ONEFLOW_CCL_ALL_GATHER_H_
