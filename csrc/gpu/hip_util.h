// Thin RAII helpers over the HIP runtime (device memory, pinned host memory,
// streams, events).  No CUDA compatibility layer: HIP/ROCm only.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <utility>

namespace sca::gpu {

#define SCA_HIP_CHECK(expr)                                                                                  \
  do {                                                                                                       \
    hipError_t _e = (expr);                                                                                  \
    if (_e != hipSuccess)                                                                                    \
      throw std::runtime_error(std::string("HIP error: ") + #expr + " -> " + hipGetErrorString(_e) + " @ " + \
                               __FILE__ + ":" + std::to_string(__LINE__));                                   \
  } while (0)

int device_count();  // 0 when no GPU / no driver
bool available();

class DeviceGuard {
 public:
  explicit DeviceGuard(int dev) {
    (void)hipGetDevice(&prev_);
    if (dev != prev_) SCA_HIP_CHECK(hipSetDevice(dev));
  }
  ~DeviceGuard() { (void)hipSetDevice(prev_); }

 private:
  int prev_ = 0;
};

// Device (HBM) allocation.
class DeviceBuffer {
 public:
  DeviceBuffer() = default;
  DeviceBuffer(size_t bytes, int device) { alloc(bytes, device); }
  ~DeviceBuffer() { reset(); }
  DeviceBuffer(const DeviceBuffer&) = delete;
  DeviceBuffer& operator=(const DeviceBuffer&) = delete;
  DeviceBuffer(DeviceBuffer&& o) noexcept { swap(o); }
  DeviceBuffer& operator=(DeviceBuffer&& o) noexcept { reset(); swap(o); return *this; }
  // fine: fine-grained (coherent) device memory -- for buffers another GPU
  // writes into over xGMI while this GPU's kernels read them
  void alloc(size_t bytes, int device, bool fine = false) {
    reset();
    device_ = device;
    bytes_ = bytes;
    if (!bytes) return;
    DeviceGuard g(device);
    if (fine) SCA_HIP_CHECK(hipExtMallocWithFlags(&ptr_, bytes, hipDeviceMallocFinegrained));
    else SCA_HIP_CHECK(hipMalloc(&ptr_, bytes));
    // Zero it (workspaces may hold counters that must start at 0) and WAIT:
    // hipMemset is queued on the null stream, which our non-blocking streams
    // do not order against, so a buffer grown mid-stream could be zeroed
    // after the copy that fills it -- tests/test_fabric_loopback.py caught a
    // worker slot's fresh input buffer read back as zeros.
    SCA_HIP_CHECK(hipMemsetAsync(ptr_, 0, bytes, nullptr));
    SCA_HIP_CHECK(hipStreamSynchronize(nullptr));
  }
  void reset() {
    if (ptr_) {
      DeviceGuard g(device_);
      (void)hipFree(ptr_);
    }
    ptr_ = nullptr;
    bytes_ = 0;
  }
  void upload(const void* src, size_t bytes) {
    if (bytes > bytes_) throw std::runtime_error("DeviceBuffer::upload overflow");
    DeviceGuard g(device_);
    SCA_HIP_CHECK(hipMemcpy(ptr_, src, bytes, hipMemcpyHostToDevice));
  }
  template <class T> T* as() const { return static_cast<T*>(ptr_); }
  void* get() const { return ptr_; }
  size_t bytes() const { return bytes_; }
  int device() const { return device_; }

 private:
  void swap(DeviceBuffer& o) {
    std::swap(ptr_, o.ptr_);
    std::swap(bytes_, o.bytes_);
    std::swap(device_, o.device_);
  }
  void* ptr_ = nullptr;
  size_t bytes_ = 0;
  int device_ = 0;
};

// Pinned, device-mapped, fine-grained host allocation: the kernel can read its
// input / write its output straight over PCIe (zero-copy), or it can be the
// endpoint of an async DMA.
class PinnedBuffer {
 public:
  PinnedBuffer() = default;
  explicit PinnedBuffer(size_t bytes) { alloc(bytes); }
  ~PinnedBuffer() { reset(); }
  PinnedBuffer(const PinnedBuffer&) = delete;
  PinnedBuffer& operator=(const PinnedBuffer&) = delete;
  void alloc(size_t bytes) {
    reset();
    bytes_ = bytes;
    if (!bytes) return;
    SCA_HIP_CHECK(hipHostMalloc(&host_, bytes, hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent));
    SCA_HIP_CHECK(hipHostGetDevicePointer(&dev_, host_, 0));
  }
  void reset() {
    if (host_) (void)hipHostFree(host_);
    host_ = dev_ = nullptr;
    bytes_ = 0;
  }
  template <class T> T* host() const { return static_cast<T*>(host_); }
  template <class T> T* dev() const { return static_cast<T*>(dev_); }
  size_t bytes() const { return bytes_; }

 private:
  void* host_ = nullptr;
  void* dev_ = nullptr;
  size_t bytes_ = 0;
};

// Fine-grained device memory that the CPU writes through the PCIe BAR (the
// MI355X exposes all of HBM to the host: large BAR).  A small batch's rows go
// straight into HBM with write-combined stores, so the kernel's first loads
// hit local memory instead of crossing PCIe (tools/micro/vram_probe.hip).
// The CPU never reads it back (uncached reads over PCIe are slow).
class BarBuffer {
 public:
  BarBuffer() = default;
  ~BarBuffer() { reset(); }
  BarBuffer(const BarBuffer&) = delete;
  BarBuffer& operator=(const BarBuffer&) = delete;
  void alloc(size_t bytes, int device) {
    reset();
    device_ = device;
    bytes_ = bytes;
    if (!bytes) return;
    DeviceGuard g(device);
    SCA_HIP_CHECK(hipExtMallocWithFlags(&ptr_, bytes, hipDeviceMallocFinegrained));
  }
  void reset() {
    if (ptr_) {
      DeviceGuard g(device_);
      (void)hipFree(ptr_);
    }
    ptr_ = nullptr;
    bytes_ = 0;
  }
  template <class T> T* as() const { return static_cast<T*>(ptr_); }
  size_t bytes() const { return bytes_; }

 private:
  void* ptr_ = nullptr;
  size_t bytes_ = 0;
  int device_ = 0;
};

// True when the device's whole memory is CPU-visible (BarBuffer usable).
bool large_bar(int device);

class Stream {
 public:
  Stream() = default;
  explicit Stream(int device) { create(device); }
  ~Stream() { reset(); }
  Stream(const Stream&) = delete;
  Stream& operator=(const Stream&) = delete;
  void create(int device) {
    reset();
    device_ = device;
    DeviceGuard g(device);
    SCA_HIP_CHECK(hipStreamCreateWithFlags(&s_, hipStreamNonBlocking));
  }
  void reset() {
    if (s_) {
      DeviceGuard g(device_);
      (void)hipStreamDestroy(s_);
    }
    s_ = nullptr;
  }
  hipStream_t get() const { return s_; }

 private:
  hipStream_t s_ = nullptr;
  int device_ = 0;
};

class Event {
 public:
  Event() = default;
  ~Event() { reset(); }
  Event(const Event&) = delete;
  Event& operator=(const Event&) = delete;
  void create(int device) {
    reset();
    device_ = device;
    DeviceGuard g(device);
    SCA_HIP_CHECK(hipEventCreateWithFlags(&e_, hipEventDisableTiming));
  }
  void reset() {
    if (e_) {
      DeviceGuard g(device_);
      (void)hipEventDestroy(e_);
    }
    e_ = nullptr;
  }
  hipEvent_t get() const { return e_; }

 private:
  hipEvent_t e_ = nullptr;
  int device_ = 0;
};

}  // namespace sca::gpu
