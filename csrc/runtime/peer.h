// Cross-device guard for the paths that move frames between GPUs over xGMI:
//   * the split topology (SplitInstance: detector on GPU i, classifier on GPU j; Executor::submit_peer pulls the
//     detector's slot with hipMemcpyPeerAsync),
//   * the arm-B device transport opened on another GPU (ipc_open of a ring exported on GPU i into a process on
//     GPU j; Executor::submit_device copies the frames peer to peer).
//
// On the 8-GPU MI355X node every pair is linked point to point, so peer access is expected; on a box or a
// container that exposes GPUs without it, HIP would either stage the copy through the host silently or fault in
// the kernel that dereferences a mapped pointer.  Both paths instead fail at setup with an error that names
// the two devices (reference triton instance_group, infrastructure/minio/triton_config.py:114-117).
//
// `can_access` is injectable so the policy is testable without a GPU (csrc/tests/peer_check.cpp).
#pragma once
#include <functional>
#include <stdexcept>
#include <string>

namespace arena {

using PeerQuery = std::function<int(int dst, int src)>;  // 1 if `dst` can access `src`'s memory

// Throws std::runtime_error unless `dst` may read `src`'s memory directly (same device: always).
inline void require_peer_access(int dst, int src, const char* what, const PeerQuery& can_access) {
  if (dst < 0 || src < 0 || dst == src) return;
  if (!can_access(dst, src))
    throw std::runtime_error(std::string(what) + ": GPU " + std::to_string(dst) + " cannot access GPU " +
                             std::to_string(src) + "'s memory (hipDeviceCanAccessPeer = 0; no xGMI peer path)" +
                             ": place both stages on one GPU or on a linked pair");
}

// hipDeviceCanAccessPeer (csrc/runtime/ipc_buffer.cpp)
int hip_can_access_peer(int dst, int src);

}  // namespace arena
