// eager_rccl_comm_manager.cpp — see the header.  Written from the behaviour of
// EagerNcclCommMgr::GetCommForDevice / CreateNcclComm (oneflow/core/job/eager_nccl_comm_manager.cpp:
// 57-131): sorted device vector, rank by position, unique id through the control plane's KV store.
#include "oneflow/core/job/eager_rccl_comm_manager.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <sstream>

#include "oneflow/core/control/ctrl_client.h"

namespace oneflow {

const std::string EagerRcclCommMgr::kDefaultStreamName = "DEFAULT";

EagerRcclCommMgr* EagerRcclCommMgr::Get() {
  static EagerRcclCommMgr mgr;
  return &mgr;
}

EagerRcclCommMgr::~EagerRcclCommMgr() {
  // Communicators live for the process, as in the reference's singleton; the runtime may already
  // be torn down at static destruction, so they are not destroyed here.
}

std::string EagerRcclCommMgr::UniqueIdKey(
    const std::vector<std::pair<int64_t, int64_t>>& sorted_devices, const std::string& stream_name) {
  std::ostringstream oss;
  oss << "eager_rccl_unique_id_rpc_key";
  if (stream_name != kDefaultStreamName) oss << "/" << stream_name;
  for (const auto& p : sorted_devices) oss << "," << p.first << ":" << p.second;
  return oss.str();
}

int EagerRcclCommMgr::RankInSet(const std::vector<std::pair<int64_t, int64_t>>& sorted_devices,
                                int64_t machine, int64_t device) {
  auto it = std::find(sorted_devices.begin(), sorted_devices.end(), std::make_pair(machine, device));
  return it == sorted_devices.end() ? -1 : (int)std::distance(sorted_devices.begin(), it);
}

namespace {

void* CreateRcclComm(int dev, const std::string& key,
                     const std::vector<std::pair<int64_t, int64_t>>& device_vec) {
  const int64_t machine = GlobalProcessCtx::Rank();
  const int rank = EagerRcclCommMgr::RankInSet(device_vec, machine, dev);
  OFX_KERNEL_CHECK(rank >= 0, "this process (rank " << machine << ", device " << dev
                                                      << ") is not in the placement");
  ncclUniqueId id;
  std::memset(&id, 0, sizeof(id));
  if (rank == 0) {
    OFX_KERNEL_CHECK(ncclGetUniqueId(&id) == ncclSuccess, "ncclGetUniqueId failed");
    if (device_vec.size() > 1) {
      CtrlClient* ctrl = CtrlClient::Get();
      OFX_KERNEL_CHECK(ctrl != nullptr, "a multi-rank RCCL communicator needs the host control "
                                        "plane (ofx_process_ctx_init)");
      ctrl->PushKV(key, std::string(id.internal, sizeof(id.internal)));
    }
  } else {
    CtrlClient* ctrl = CtrlClient::Get();
    OFX_KERNEL_CHECK(ctrl != nullptr, "no host control plane to pull the RCCL unique id from");
    ctrl->PullKV(key, [&id](const std::string& v) {
      OFX_KERNEL_CHECK(v.size() == sizeof(id.internal), "bad unique id of " << v.size() << " bytes");
      std::memcpy(id.internal, v.data(), sizeof(id.internal));
    });
  }
  ncclComm_t comm;
  const ncclResult_t r = ncclCommInitRank(&comm, (int)device_vec.size(), id, rank);
  OFX_KERNEL_CHECK(r == ncclSuccess, "ncclCommInitRank (" << device_vec.size() << " ranks, rank "
                                                          << rank << "): " << ncclGetErrorString(r));
  return comm;
}

}  // namespace

void* EagerRcclCommMgr::GetCommForDeviceAndStreamName(const DeviceSet& device_set,
                                                      const std::string& stream_name) {
  int dev = 0;
  OFX_KERNEL_CHECK(hipGetDevice(&dev) == hipSuccess, "hipGetDevice failed");
  const auto key = std::make_pair(device_set, stream_name);
  {
    std::lock_guard<std::mutex> lock(mutex_);
    auto it = comms_.find(key);
    if (it != comms_.end() && it->second.count(dev)) return it->second.at(dev);
  }
  // std::set of pairs is already in (machine, device) order (CompareDeviceSetPair)
  std::vector<std::pair<int64_t, int64_t>> device_vec(device_set.begin(), device_set.end());
  void* comm = CreateRcclComm(dev, UniqueIdKey(device_vec, stream_name), device_vec);
  std::lock_guard<std::mutex> lock(mutex_);
  comms_[key][dev] = comm;
  return comm;
}

void* EagerRcclCommMgr::GetCommForDevice(const DeviceSet& device_set) {
  return GetCommForDeviceAndStreamName(device_set, kDefaultStreamName);
}

}  // namespace oneflow
