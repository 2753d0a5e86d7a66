// Dynamic-LDS opt-in above 64 KB (hipFuncAttributeMaxDynamicSharedMemorySize)
// applies to the CURRENT device: record the largest size raised per (kernel,
// device), thread-safe; a later launch needing more raises it again.
#pragma once
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>
#include <utility>

namespace orbgpu {

inline hipError_t lds_optin(const void* fn, int bytes) {
  static std::mutex mu;
  static std::map<std::pair<const void*, int>, int> raised;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return hipErrorInvalidDevice;
  std::lock_guard<std::mutex> lock(mu);
  auto it = raised.find({fn, dev});
  if (it != raised.end() && it->second >= bytes) return hipSuccess;
  const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess) raised[{fn, dev}] = bytes;
  return e;
}

}  // namespace orbgpu
