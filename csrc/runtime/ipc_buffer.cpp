// See ipc_buffer.h.
#include "runtime/ipc_buffer.h"
#include "runtime/peer.h"

#include <hip/hip_runtime.h>

#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>

namespace arena {

namespace {
void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e) + " (" + what + ")");
}
}  // namespace

IpcBuffer::IpcBuffer(size_t bytes, int device) : bytes_(bytes), device_(device) {
  if (bytes == 0) throw std::runtime_error("IpcBuffer: zero size");
  check(hipSetDevice(device), "hipSetDevice");
  check(hipMalloc(&ptr_, bytes), "hipMalloc");
  hipIpcMemHandle_t h;
  const hipError_t e = hipIpcGetMemHandle(&h, ptr_);
  if (e != hipSuccess) {
    (void)hipFree(ptr_);
    ptr_ = nullptr;
    check(e, "hipIpcGetMemHandle (dmabuf IPC needs HSA_ENABLE_IPC_MODE_LEGACY=0)");
  }
  handle_.assign((const char*)&h, sizeof h);
}

IpcBuffer::~IpcBuffer() {
  if (stream_ != nullptr) {
    (void)hipSetDevice(device_);
    (void)hipStreamDestroy((hipStream_t)stream_);
  }
  if (ptr_ != nullptr) {
    (void)hipSetDevice(device_);
    (void)hipFree(ptr_);
  }
}

void IpcBuffer::write(size_t off, const void* src, size_t n) {
  if (off > bytes_ || n > bytes_ - off) throw std::runtime_error("IpcBuffer::write out of range");
  check(hipSetDevice(device_), "hipSetDevice");
  // another process reads these bytes on its own stream right after the RPC naming them: the copy must have
  // landed in device memory, not just left the pageable source (a plain hipMemcpy only promises the latter).
  // A copy on the buffer's own stream + a sync of that stream waits for exactly this copy; a device-wide sync
  // would also drain every in-flight detector batch of the process from the request thread.
  std::lock_guard<std::mutex> lk(mu_);
  if (stream_ == nullptr) check(hipStreamCreateWithFlags((hipStream_t*)&stream_, hipStreamNonBlocking), "hipStreamCreate");
  check(hipMemcpyAsync((uint8_t*)ptr_ + off, src, n, hipMemcpyHostToDevice, (hipStream_t)stream_), "hipMemcpyAsync H2D");
  check(hipStreamSynchronize((hipStream_t)stream_), "hipStreamSynchronize after IPC write");
}

void IpcBuffer::read(size_t off, void* dst, size_t n) const {
  if (off > bytes_ || n > bytes_ - off) throw std::runtime_error("IpcBuffer::read out of range");
  check(hipSetDevice(device_), "hipSetDevice");
  check(hipMemcpy(dst, (const uint8_t*)ptr_ + off, n, hipMemcpyDeviceToHost), "hipMemcpy D2H");
}

int hip_can_access_peer(int dst, int src) {
  int can = 0;
  check(hipDeviceCanAccessPeer(&can, dst, src), "hipDeviceCanAccessPeer");
  return can;
}

uintptr_t ipc_open(const std::string& handle, int device, int src_device) {
  require_peer_access(device, src_device, "ipc_open", hip_can_access_peer);
  hipIpcMemHandle_t h;
  if (handle.size() != sizeof h) throw std::runtime_error("ipc_open: handle must be " + std::to_string(sizeof h) + " bytes");
  std::memcpy(&h, handle.data(), sizeof h);
  check(hipSetDevice(device), "hipSetDevice");
  void* p = nullptr;
  check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
  return (uintptr_t)p;
}

size_t ipc_mapped_bytes(uintptr_t ptr) {
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  check(hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)ptr), "hipMemGetAddressRange");
  const size_t skip = (size_t)(ptr - (uintptr_t)base);
  return size > skip ? size - skip : 0;
}

void ipc_close(uintptr_t ptr) { check(hipIpcCloseMemHandle((void*)ptr), "hipIpcCloseMemHandle"); }

}  // namespace arena
