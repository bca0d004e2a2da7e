// hip_communication_context.h — the kHIP communicator of a placement: an RCCL comm from
// EagerRcclCommMgr for the placement's device set (role of CudaCommunicationContext,
// oneflow/user/kernels/collective_communication/cuda/cuda_communication_context.cpp:24-35).
#ifndef OFX_ONEFLOW_CCL_HIP_COMMUNICATION_CONTEXT_H_
#define OFX_ONEFLOW_CCL_HIP_COMMUNICATION_CONTEXT_H_

#include <map>

#include "oneflow/user/kernels/collective_communication/include/communication_context.h"

namespace oneflow {
namespace ccl {

class HipCommunicationContext : public CommunicationContext {
 public:
  HipCommunicationContext() = default;
  ~HipCommunicationContext() override = default;
  void Init(const ParallelDesc& parallel_desc) override;
  void* rccl_comm() const { return comm_; }  // ncclComm_t
  int64_t rccl_index4rank(int64_t rank) const { return rank2rccl_index_.at(rank); }

 private:
  void* comm_ = nullptr;
  std::map<int64_t, int64_t> rank2rccl_index_;
};

}  // namespace ccl
}  // namespace oneflow

#endif  // OFX_ONEFLOW_CCL_HIP_COMMUNICATION_CONTEXT_H_
