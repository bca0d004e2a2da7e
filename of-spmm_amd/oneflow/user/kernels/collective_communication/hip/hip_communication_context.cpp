// hip_communication_context.cpp — see the header.
#include "oneflow/user/kernels/collective_communication/hip/hip_communication_context.h"

#include "oneflow/core/job/eager_rccl_comm_manager.h"

namespace oneflow {
namespace ccl {

void HipCommunicationContext::Init(const ParallelDesc& parallel_desc) {
  DeviceSet device_set;
  for (int64_t parallel_id = 0; parallel_id < parallel_desc.parallel_num(); ++parallel_id) {
    const int64_t machine_id = parallel_desc.MachineId4ParallelId(parallel_id);
    const int64_t device_id = parallel_desc.DeviceId4ParallelId(parallel_id);
    device_set.emplace(machine_id, device_id);
    rank2rccl_index_.emplace(machine_id, parallel_id);
  }
  comm_ = EagerRcclCommMgr::Get()->GetCommForDevice(device_set);
}

REGISTER_COLLECTIVE_COMMUNICATION_COMMUNICATOR(DeviceType::kHIP, HipCommunicationContext);

}  // namespace ccl
}  // namespace oneflow
