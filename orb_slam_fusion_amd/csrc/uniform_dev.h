// Wave-uniform branch conditions.  Several device helpers are written for
// callers whose every active lane holds the same argument (one problem or one
// IMU link per wave: PoseOptimization's exp, the inertial edges' ExpSO3 /
// LogSO3 / right Jacobians / delta rotation); they branch on
// readfirstlane(cond) so the branch is scalar, not exec-masked.  That is only
// correct while the caller keeps its promise -- round 3 shipped a per-lane
// use of such a helper that took lane 0's branch for every lane.
//
// Builds with ORBGPU_CHECK_UNIFORM=1 (`make checkuniform`) verify the promise
// at every such branch: any active lane whose condition differs from lane 0's
// counts one violation in a device counter, read and cleared by
// orbgpu_debug_uniform_violations() (tests/conftest.py fails the test that
// raised it).  The default build compiles to the plain readfirstlane.
#pragma once
#include <hip/hip_runtime.h>

#ifndef ORBGPU_CHECK_UNIFORM
#define ORBGPU_CHECK_UNIFORM 0
#endif

namespace orbgpu {

#if ORBGPU_CHECK_UNIFORM
// one counter per translation unit (no relocatable device code): each kernel
// TU exports its reader through ORBGPU_UNIFORM_READER
static __device__ unsigned int g_uniform_violations;
#endif

// v as the wave's uniform value (lane 0's among the active lanes).
__device__ __forceinline__ int uniform_branch(int v) {
  const int r = __builtin_amdgcn_readfirstlane(v);
#if ORBGPU_CHECK_UNIFORM
  const unsigned long long bad = __ballot(v != r);
  if (bad && (threadIdx.x & 63) == (unsigned)(__builtin_ctzll(bad)))
    atomicAdd(&g_uniform_violations, 1u);
#endif
  return r;
}

}  // namespace orbgpu

#if ORBGPU_CHECK_UNIFORM
// extern "C" unsigned orbgpu_uniform_violations_<tu>(void): this TU's count, cleared
#define ORBGPU_UNIFORM_READER(tu)                                                                     \
  extern "C" unsigned orbgpu_uniform_violations_##tu(void) {                                          \
    unsigned v = 0;                                                                                   \
    const unsigned z = 0;                                                                             \
    if (hipDeviceSynchronize() != hipSuccess ||                                                       \
        hipMemcpyFromSymbol(&v, HIP_SYMBOL(orbgpu::g_uniform_violations), sizeof(v)) != hipSuccess || \
        hipMemcpyToSymbol(HIP_SYMBOL(orbgpu::g_uniform_violations), &z, sizeof(z)) != hipSuccess)    \
      return ~0u;                                                                                     \
    return v;                                                                                         \
  }
#else
#define ORBGPU_UNIFORM_READER(tu)
#endif
