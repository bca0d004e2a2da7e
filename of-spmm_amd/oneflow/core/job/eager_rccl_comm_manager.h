// eager_rccl_comm_manager.h — RCCL communicators per device set, the role of OneFlow's
// EagerNcclCommMgr (oneflow/core/job/eager_nccl_comm_manager.cpp:57-131) for DeviceType::kHIP.
// A device set is {(machine = process rank, local device)}; its sorted order gives the RCCL rank;
// rank 0 makes the unique id and publishes it under a key naming the set, the others pull it
// from the host control plane (CtrlClient), then every member calls ncclCommInitRank.
#ifndef OFX_ONEFLOW_EAGER_RCCL_COMM_MANAGER_H_
#define OFX_ONEFLOW_EAGER_RCCL_COMM_MANAGER_H_

#include <map>
#include <mutex>
#include <set>
#include <string>
#include <utility>
#include <vector>

namespace oneflow {

using DeviceSet = std::set<std::pair<int64_t, int64_t>>;

class EagerRcclCommMgr {
 public:
  static const std::string kDefaultStreamName;
  static EagerRcclCommMgr* Get();
  ~EagerRcclCommMgr();

  // ncclComm_t (as void*) of this process's current device within `device_set`.
  void* GetCommForDevice(const DeviceSet& device_set);
  // A separate communicator per stream name (the logical collectives of a lazy job).
  void* GetCommForDeviceAndStreamName(const DeviceSet& device_set, const std::string& stream_name);

  // The key rank 0 publishes the unique id under, and this process's rank in the set (tests).
  static std::string UniqueIdKey(const std::vector<std::pair<int64_t, int64_t>>& sorted_devices,
                                 const std::string& stream_name);
  static int RankInSet(const std::vector<std::pair<int64_t, int64_t>>& sorted_devices,
                       int64_t machine, int64_t device);

 private:
  std::mutex mutex_;
  std::map<std::pair<DeviceSet, std::string>, std::map<int, void*>> comms_;
};

}  // namespace oneflow

#endif  // OFX_ONEFLOW_EAGER_RCCL_COMM_MANAGER_H_
