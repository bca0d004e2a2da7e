// peer_pull.hip — the pull form of the row-split all-gather.
//
// The reference boxes B from S(0) to B with ccl::AllGather -> ncclAllGather
// (oneflow/user/kernels/collective_communication/cuda/cuda_all_gather.cpp:25-47): RCCL's ring or
// tree moves every shard through its own FIFOs.  On a fully connected MI355X node every peer's
// HBM is one xGMI hop away, so a rank can instead READ each peer's shard straight out of the
// peer's gathered buffer into its own (the buffers have one layout on every rank): one copy
// kernel that keeps all 7 links busy at once, no intermediate FIFO, no per-step protocol.  This
// file holds the device side:
//
//   ofx_peer_export / ofx_peer_open / ofx_peer_close  IPC handles of a gathered buffer (dmabuf,
//                                                     hipIpcGetMemHandle on the allocation that
//                                                     holds the pointer, plus the offset into it)
//   ofx_peer_publish                                  makes this rank's stores visible to peer
//                                                     readers (system-scope release on every XCD)
//   ofx_peer_pull / ofx_peer_pull_host                the copy, on the device / the same tile plan
//                                                     on host memory (the gloo layout test)
//
// The stream-ordered barriers around the pull (shards ready; every peer done reading) are RCCL
// calls: ofx_allgather_pull in comm_rccl.cpp composes publish -> barrier -> pull -> barrier.
#include <hip/hip_runtime.h>

#include <cstring>
#include <map>
#include <mutex>
#include <string>

#include "ofx_internal.h"
#include "spmm_common.h"

namespace ofx {
namespace {

constexpr int kPullBlock = 256;
constexpr int kPullUnroll = 4;       // 16-B loads in flight per lane
constexpr int kMaxPullBlocks = 2048;  // 8 per CU; blocks stride over the tiles
constexpr int kPublishBlocks = 1024;  // one wave each, over all 256 CUs: every XCD's L2 (below)

struct PeerSrc {
  const char* base[OFX_PEER_MAX_RANKS];  // peer p's buffer (the same layout as ours)
};

// The tile plan, shared by the kernel and the host executor: tile t of the pull reads peer
// rank p = the q-th peer (q = t mod (nranks - 1), skipping this rank), bytes
// [off, off + len) of the buffer, off = p * slot_bytes + (t / (nranks - 1)) * tile.  Consecutive
// tiles -- consecutive blocks, dealt over the XCDs round-robin -- belong to different peers, so
// every link carries traffic from the first wave on.
struct Tile {
  int peer;
  uint64_t off;
  uint64_t len;
};

__host__ __device__ inline Tile pull_tile(int64_t t, int nranks, int rank, uint64_t slot_bytes,
                                          uint64_t tile) {
  const int npeers = nranks - 1;
  const int q = (int)(t % npeers);
  Tile r;
  r.peer = q < rank ? q : q + 1;
  const uint64_t in_slot = (uint64_t)(t / npeers) * tile;
  r.off = (uint64_t)r.peer * slot_bytes + in_slot;
  const uint64_t left = slot_bytes - in_slot;
  r.len = left < tile ? left : tile;
  return r;
}

inline int64_t tiles_of(int nranks, uint64_t slot_bytes, uint64_t tile) {
  return (int64_t)((slot_bytes + tile - 1) / tile) * (nranks - 1);
}

template <int UNIT>
struct Word;
template <>
struct Word<16> {
  typedef uint32_t T __attribute__((ext_vector_type(4)));
  static __device__ T load(__amdgpu_buffer_rsrc_t r, uint32_t o) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, o, 0, 17);  // sc0 sc1: system-coherent
  }
};
template <>
struct Word<4> {
  typedef uint32_t T;
  static __device__ T load(__amdgpu_buffer_rsrc_t r, uint32_t o) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, o, 0, 17);
  }
};
template <>
struct Word<2> {
  typedef unsigned short T;
  static __device__ T load(__amdgpu_buffer_rsrc_t r, uint32_t o) {
    return __builtin_amdgcn_raw_buffer_load_b16(r, o, 0, 17);
  }
};

// One block per tile (blocks stride over the tiles): kPullUnroll loads of UNIT bytes per lane, all
// issued before the first store.  The buffer resource spans exactly the tile, so the hardware
// range check zeroes anything past a slot's end and the stores are masked by the same bound.
// Loads are sc0 sc1 (system scope): a line of the peer's memory cached by an earlier step is not
// served stale.  Stores go to this rank's own HBM (plain: the SpMM that follows on the stream reads
// them after the kernel boundary).
template <int UNIT>
__global__ void __launch_bounds__(kPullBlock)
    peer_pull_kernel(PeerSrc src, char* __restrict__ dst, int nranks, int rank,
                     uint64_t slot_bytes, int64_t tiles) {
  using W = Word<UNIT>;
  constexpr uint64_t kTile = (uint64_t)kPullBlock * kPullUnroll * UNIT;
  for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
    const Tile tl = pull_tile(t, nranks, rank, slot_bytes, kTile);
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>(src.base[tl.peer] + tl.off), 0, (int)tl.len, 0x00020000);
    typename W::T v[kPullUnroll];
#pragma unroll
    for (int u = 0; u < kPullUnroll; ++u)
      v[u] = W::load(r, (uint32_t)((u * kPullBlock + threadIdx.x) * UNIT));
    char* d = dst + tl.off;
#pragma unroll
    for (int u = 0; u < kPullUnroll; ++u) {
      const uint32_t o = (uint32_t)((u * kPullBlock + threadIdx.x) * UNIT);
      if (o + UNIT <= tl.len) *reinterpret_cast<typename W::T*>(d + o) = v[u];
    }
  }
}

// A system-scope release on every XCD: each block's first lane writes its XCD's L2 dirty lines
// back to HBM, where a peer's xGMI reads find them (the L2s are not probed by remote readers).
// Blocks are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md, "workgroup dispatch"), so
// 8 would do; kPublishBlocks = 1024 one-wave blocks (4 per CU) keep every XCD covered whatever
// the dispatch order (the publish must not rest on that order), for a few µs.
__global__ void peer_publish_kernel() {
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// IPC handle bytes: the allocation's hipIpcMemHandle_t, then the pointer's offset into it.
struct PeerHandle {
  hipIpcMemHandle_t ipc;
  uint64_t offset;
};
static_assert(sizeof(PeerHandle) <= OFX_PEER_HANDLE_BYTES, "peer handle does not fit");

// Opened allocations, by handle bytes (a handle opened twice in one process maps once), and the
// pointers handed out, each with its own count (a pointer closed more often than opened is refused
// rather than taken off another pointer's count).
struct Opened {
  void* base;
  int refs;
};
struct Handed {
  std::string key;
  int refs = 0;
};
std::mutex g_open_mu;
std::map<std::string, Opened> g_opened;
std::map<void*, Handed> g_opened_by_ptr;

int choose_unit(const void* const* bufs, int nranks, const void* dst, uint64_t slot_bytes) {
  auto ok = [&](uint64_t a) {
    if (slot_bytes % a || (uintptr_t)dst % a) return false;
    for (int p = 0; p < nranks; ++p)
      if (bufs[p] != nullptr && (uintptr_t)bufs[p] % a) return false;
    return true;
  };
  return ok(16) ? 16 : ok(4) ? 4 : ok(2) ? 2 : 0;
}

}  // namespace
}  // namespace ofx

using namespace ofx;

extern "C" int ofx_peer_export(const void* ptr, void* handle_out) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(ptr && handle_out, OFX_EINVAL, "peer_export: NULL argument");
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    OFX_HIP_CHECK(hipMemGetAddressRange(&base, &size, const_cast<void*>(ptr)));
    PeerHandle h;
    std::memset(&h, 0, sizeof(h));
    OFX_HIP_CHECK(hipIpcGetMemHandle(&h.ipc, base));
    h.offset = (uint64_t)((const char*)ptr - (const char*)base);
    std::memset(handle_out, 0, OFX_PEER_HANDLE_BYTES);
    std::memcpy(handle_out, &h, sizeof(h));
    return OFX_OK;
  });
}

extern "C" int ofx_peer_open(const void* handle, void** ptr_out) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(handle && ptr_out, OFX_EINVAL, "peer_open: NULL argument");
    PeerHandle h;
    std::memcpy(&h, handle, sizeof(h));
    const std::string key(reinterpret_cast<const char*>(&h.ipc), sizeof(h.ipc));
    std::lock_guard<std::mutex> lock(g_open_mu);
    auto it = g_opened.find(key);
    if (it == g_opened.end()) {
      void* base = nullptr;
      OFX_HIP_CHECK(hipIpcOpenMemHandle(&base, h.ipc, hipIpcMemLazyEnablePeerAccess));
      it = g_opened.emplace(key, Opened{base, 0}).first;
    }
    it->second.refs += 1;
    void* p = static_cast<char*>(it->second.base) + h.offset;
    *ptr_out = p;
    Handed& hd = g_opened_by_ptr[p];
    hd.key = key;
    hd.refs += 1;
    return OFX_OK;
  });
}

extern "C" int ofx_peer_close(void* ptr) {
  return ::ofx::guarded(__func__, [&]() -> int {
    if (ptr == nullptr) return OFX_OK;
    std::lock_guard<std::mutex> lock(g_open_mu);
    auto pk = g_opened_by_ptr.find(ptr);
    OFX_REQUIRE(pk != g_opened_by_ptr.end(), OFX_EINVAL, "peer_close: %p was not opened here", ptr);
    const std::string key = pk->second.key;
    if (--pk->second.refs == 0) g_opened_by_ptr.erase(pk);
    auto it = g_opened.find(key);
    if (--it->second.refs == 0) {
      void* base = it->second.base;
      g_opened.erase(it);
      OFX_HIP_CHECK(hipIpcCloseMemHandle(base));
    }
    return OFX_OK;
  });
}

extern "C" int ofx_peer_publish(void* stream) {
  return ::ofx::guarded(__func__, [&]() -> int {
    hipLaunchKernelGGL(peer_publish_kernel, dim3(kPublishBlocks), dim3(64), 0,
                       static_cast<hipStream_t>(stream));
    OFX_HIP_CHECK(hipGetLastError());
    return OFX_OK;
  });
}

extern "C" int ofx_peer_pull(void* stream, int nranks, int rank, const void* const* peer_bufs,
                             void* buf, uint64_t slot_bytes) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(nranks >= 1 && nranks <= OFX_PEER_MAX_RANKS && rank >= 0 && rank < nranks,
                OFX_EINVAL, "peer_pull: %d ranks (rank %d); at most %d", nranks, rank,
                OFX_PEER_MAX_RANKS);
    if (nranks == 1 || slot_bytes == 0) return OFX_OK;
    OFX_REQUIRE(peer_bufs && buf, OFX_EINVAL, "peer_pull: NULL argument");
    PeerSrc src{};
    for (int p = 0; p < nranks; ++p) {
      OFX_REQUIRE(p == rank || peer_bufs[p] != nullptr, OFX_EINVAL, "peer_pull: peer %d NULL", p);
      src.base[p] = p == rank ? nullptr : static_cast<const char*>(peer_bufs[p]);
    }
    const int unit = choose_unit(peer_bufs, nranks, buf, slot_bytes);
    OFX_REQUIRE(unit > 0, OFX_EINVAL, "peer_pull: slot of %llu bytes or a buffer not 2-B aligned",
                (unsigned long long)slot_bytes);
    hipStream_t s = static_cast<hipStream_t>(stream);
    const uint64_t tile = (uint64_t)kPullBlock * kPullUnroll * unit;
    const int64_t tiles = tiles_of(nranks, slot_bytes, tile);
    const unsigned grid = (unsigned)std::min<int64_t>(tiles, kMaxPullBlocks);
    char* dst = static_cast<char*>(buf);
    switch (unit) {
      case 16:
        hipLaunchKernelGGL(peer_pull_kernel<16>, dim3(grid), dim3(kPullBlock), 0, s, src, dst,
                           nranks, rank, slot_bytes, tiles);
        break;
      case 4:
        hipLaunchKernelGGL(peer_pull_kernel<4>, dim3(grid), dim3(kPullBlock), 0, s, src, dst,
                           nranks, rank, slot_bytes, tiles);
        break;
      default:
        hipLaunchKernelGGL(peer_pull_kernel<2>, dim3(grid), dim3(kPullBlock), 0, s, src, dst,
                           nranks, rank, slot_bytes, tiles);
        break;
    }
    OFX_HIP_CHECK(hipGetLastError());
    return OFX_OK;
  });
}

// The same tiles over host memory, in tile order (the gloo test maps each rank's buffer from
// shared memory and checks the result against torch.distributed.all_gather).
extern "C" int ofx_peer_pull_host(int nranks, int rank, const void* const* peer_bufs, void* buf,
                                  uint64_t slot_bytes) {
  return ::ofx::guarded(__func__, [&]() -> int {
    OFX_REQUIRE(nranks >= 1 && nranks <= OFX_PEER_MAX_RANKS && rank >= 0 && rank < nranks,
                OFX_EINVAL, "peer_pull_host: %d ranks (rank %d)", nranks, rank);
    if (nranks == 1 || slot_bytes == 0) return OFX_OK;
    OFX_REQUIRE(peer_bufs && buf, OFX_EINVAL, "peer_pull_host: NULL argument");
    const int unit = choose_unit(peer_bufs, nranks, buf, slot_bytes);
    OFX_REQUIRE(unit > 0, OFX_EINVAL, "peer_pull_host: slot of %llu bytes or a buffer not 2-B aligned",
                (unsigned long long)slot_bytes);
    const uint64_t tile = (uint64_t)kPullBlock * kPullUnroll * unit;
    const int64_t tiles = tiles_of(nranks, slot_bytes, tile);
    for (int64_t t = 0; t < tiles; ++t) {
      const Tile tl = pull_tile(t, nranks, rank, slot_bytes, tile);
      OFX_REQUIRE(peer_bufs[tl.peer] != nullptr, OFX_EINVAL, "peer_pull_host: peer %d NULL", tl.peer);
      std::memcpy(static_cast<char*>(buf) + tl.off,
                  static_cast<const char*>(peer_bufs[tl.peer]) + tl.off, tl.len);
    }
    return OFX_OK;
  });
}
