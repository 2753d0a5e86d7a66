// Dynamic-LDS opt-in above 64 KB (hipFuncAttributeMaxDynamicSharedMemorySize)
// applies to the CURRENT device: record it per (kernel, device), thread-safe.
#pragma once
#include <hip/hip_runtime.h>

#include <mutex>
#include <set>
#include <utility>

namespace orbgpu {

inline hipError_t lds_optin(const void* fn, int bytes) {
  static std::mutex mu;
  static std::set<std::pair<const void*, int>> done;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return hipErrorInvalidDevice;
  std::lock_guard<std::mutex> lock(mu);
  if (done.count({fn, dev})) return hipSuccess;
  const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess) done.insert({fn, dev});
  return e;
}

}  // namespace orbgpu
