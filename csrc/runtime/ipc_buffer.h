// Device memory shared between processes (arm B device crop hand-off, ARENA_CROP_TRANSPORT=device).
//
// The reference ships every crop from the detection to the classification service as a JPEG inside a gRPC
// message (architectures/microservices/detection/app/grpc_client.py:99-168).  Here the detection process
// keeps a ring of decoded images in device memory exported with hipIpcGetMemHandle (dmabuf IPC:
// HSA_ENABLE_IPC_MODE_LEGACY=0); the RPC carries the 64-byte handle, an offset and the boxes, and the
// classification process maps the ring once (ipc_open) and copies the images device to device into its own
// staging (Executor::submit_device).  No pixel crosses the host or the socket.
#pragma once
#include <cstddef>
#include <cstdint>
#include <mutex>
#include <string>

namespace arena {

class IpcBuffer {
 public:
  IpcBuffer(size_t bytes, int device);
  ~IpcBuffer();
  IpcBuffer(const IpcBuffer&) = delete;
  IpcBuffer& operator=(const IpcBuffer&) = delete;

  std::string handle() const { return handle_; }  // hipIpcMemHandle_t bytes (64)
  uintptr_t ptr() const { return (uintptr_t)ptr_; }
  size_t size() const { return bytes_; }
  int device() const { return device_; }
  // host -> device copy of n bytes at byte offset off (synchronous: the bytes are in place on return, so the
  // RPC that names them can be sent right after)
  void write(size_t off, const void* src, size_t n);
  // device -> host copy (tests)
  void read(size_t off, void* dst, size_t n) const;

 private:
  void* ptr_ = nullptr;
  size_t bytes_ = 0;
  int device_ = 0;
  std::string handle_;
  void* stream_ = nullptr;  // hipStream_t of write(), created on first use
  std::mutex mu_;
};

// Map another process's IpcBuffer (its handle()) into this process on `device`; returns the device pointer.
// The mapping is process-wide and reference-counted by the driver; ipc_close() releases it.  `src_device`
// (>= 0: the GPU that exported the buffer) is checked for peer access first (runtime/peer.h): a ring on
// another GPU without an xGMI peer path is refused with a clear error instead of faulting in a kernel.
uintptr_t ipc_open(const std::string& handle, int device, int src_device = -1);
// Size of the allocation an (IPC-)mapped device pointer belongs to, from its base (hipMemGetAddressRange):
// the classification side bounds every frame reference against it.
size_t ipc_mapped_bytes(uintptr_t ptr);
void ipc_close(uintptr_t ptr);

}  // namespace arena
