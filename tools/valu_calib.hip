// VALU-issue calibration for the SQ counters (tools/profile_round.sh).
//
// k_valu_sat keeps every SIMD's vector issue busy: 2048 workgroups x 256
// threads = 8 waves per SIMD on 256 CUs, each lane running 8 independent
// v_fma_f32 chains (no memory traffic inside the loop).  Its SQ_INSTS_VALU per
// nanosecond is the device's saturated wave64-VALU issue rate as the counters
// report it; a kernel's VALU-busy fraction is its own SQ_INSTS_VALU per
// nanosecond over this rate (same counter, same clock domain, no assumption
// about the counters' units).  k_valu_int is the same with 32-bit integer
// ops (v_xad_u32: xor + add fused), the kind the extractor kernels issue.
//
//   build/valu_calib [reps]  -> prints one JSON line (HIP-event durations)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr int kIters = 2048;

__global__ __launch_bounds__(256) void k_valu_sat(float* out, float s) {
  float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
        a6 = a0 + 6, a7 = a0 + 7;
  for (int i = 0; i < kIters; ++i) {
    a0 = __builtin_fmaf(a0, s, 1.0f);
    a1 = __builtin_fmaf(a1, s, 1.0f);
    a2 = __builtin_fmaf(a2, s, 1.0f);
    a3 = __builtin_fmaf(a3, s, 1.0f);
    a4 = __builtin_fmaf(a4, s, 1.0f);
    a5 = __builtin_fmaf(a5, s, 1.0f);
    a6 = __builtin_fmaf(a6, s, 1.0f);
    a7 = __builtin_fmaf(a7, s, 1.0f);
  }
  const float r = ((a0 + a1) + (a2 + a3)) + ((a4 + a5) + (a6 + a7));
  if (r == 12345.0f) out[blockIdx.x * 256 + threadIdx.x] = r;  // never true: keeps the chains live
}

__global__ __launch_bounds__(256) void k_valu_int(unsigned* out, unsigned s) {
  unsigned a0 = threadIdx.x, a1 = a0 ^ 1, a2 = a0 ^ 2, a3 = a0 ^ 3, a4 = a0 ^ 4, a5 = a0 ^ 5,
           a6 = a0 ^ 6, a7 = a0 ^ 7;
  for (int i = 0; i < kIters; ++i) {
    a0 = (a0 ^ s) + a1;
    a1 = (a1 ^ s) + a2;
    a2 = (a2 ^ s) + a3;
    a3 = (a3 ^ s) + a4;
    a4 = (a4 ^ s) + a5;
    a5 = (a5 ^ s) + a6;
    a6 = (a6 ^ s) + a7;
    a7 = (a7 ^ s) + a0;
  }
  const unsigned r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (r == 0x9E3779B9u) out[blockIdx.x * 256 + threadIdx.x] = r;
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess) return 1;
  const int blocks = cus * 8;  // 8 x 256 threads = 32 waves per CU = 8 per SIMD
  void* out = nullptr;
  if (hipMalloc(&out, sizeof(float) * 256 * (size_t)blocks) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float ms[2] = {0, 0};
  for (int k = 0; k < 2; ++k) {
    for (int w = 0; w < 3; ++w) {
      if (k == 0)
        hipLaunchKernelGGL(k_valu_sat, dim3(blocks), dim3(256), 0, 0, (float*)out, 0.999f);
      else
        hipLaunchKernelGGL(k_valu_int, dim3(blocks), dim3(256), 0, 0, (unsigned*)out, 0x5bd1e995u);
    }
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < reps; ++r) {
      if (k == 0)
        hipLaunchKernelGGL(k_valu_sat, dim3(blocks), dim3(256), 0, 0, (float*)out, 0.999f);
      else
        hipLaunchKernelGGL(k_valu_int, dim3(blocks), dim3(256), 0, 0, (unsigned*)out, 0x5bd1e995u);
    }
    (void)hipEventRecord(e1, 0);
    if (hipEventSynchronize(e1) != hipSuccess) return 1;
    (void)hipEventElapsedTime(&ms[k], e0, e1);
    ms[k] /= reps;
  }
  // VALU instructions per wave in the loop: 8 v_fma_f32 / 8 v_xad_u32 per iteration
  const double waves = blocks * 4.0;
  printf("{\"cus\": %d, \"blocks\": %d, \"waves\": %.0f, \"k_valu_sat_us\": %.3f, "
         "\"k_valu_int_us\": %.3f, \"loop_valu_per_wave_sat\": %d, \"loop_valu_per_wave_int\": %d}\n",
         cus, blocks, waves, ms[0] * 1e3, ms[1] * 1e3, 8 * kIters, 8 * kIters);
  (void)hipFree(out);
  return 0;
}
