// cpu_communication_context.h — the kCPU communicator: the placement itself; bytes move over the
// host transport (collective_communication/cpu/cpu_communication_context.h).
#ifndef OFX_ONEFLOW_CCL_CPU_COMMUNICATION_CONTEXT_H_
#define OFX_ONEFLOW_CCL_CPU_COMMUNICATION_CONTEXT_H_

#include "oneflow/user/kernels/collective_communication/include/communication_context.h"

namespace oneflow {
namespace ccl {

class CpuCommunicationContext : public CommunicationContext {
 public:
  void Init(const ParallelDesc& parallel_desc) override { parallel_desc_ = parallel_desc; }
  const ParallelDesc& parallel_desc() const { return parallel_desc_; }

 private:
  ParallelDesc parallel_desc_;
};

}  // namespace ccl
}  // namespace oneflow

#endif  // OFX_ONEFLOW_CCL_CPU_COMMUNICATION_CONTEXT_H_
