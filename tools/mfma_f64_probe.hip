// Cycle probe of the fp64 building blocks of k_lba_solve on one wave (gfx950):
//   v_mfma_f64_16x16x4_f64: one dependent accumulation chain, 2 and 4
//   interleaved chains; v_fma_f64 dependent chain and 8 independent chains;
//   a dependent ds_read_b64 chain (LDS latency).
// Cycles per operation from s_memtime around 256 repetitions, lane 0 of
// wave 0, one workgroup (the solve's situation: one CU).
//   hipcc --offload-arch=gfx950 -O3 -o build/mfma_f64_probe tools/mfma_f64_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int kReps = 256;

__global__ void k_probe(double* out, double seed) {
  __shared__ double lds[1024];
  const int lane = threadIdx.x & 63;
  for (int i = lane; i < 1024; i += 64) lds[i] = (double)((i * 7 + 3) & 1023);
  __syncthreads();
  const double a = seed + lane * 1e-3, b = seed - lane * 1e-3;
  d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  unsigned long long t0, t1;
  double sink = 0;
  if (threadIdx.x < 64) {  // wave 0 alone: the solve's serial sections
  // 1 dependent chain
  t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < kReps; ++r) c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
  sink += c0[0];
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[0] = (double)(t1 - t0) / kReps;

  // 2 chains
  t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < kReps / 2; ++r) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, c1, 0, 0, 0);
  }
  sink += c0[1] + c1[0];
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[1] = (double)(t1 - t0) / kReps;

  // 4 chains
  t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < kReps / 4; ++r) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, b, c3, 0, 0, 0);
  }
  sink += c0[2] + c1[1] + c2[0] + c3[3];
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[2] = (double)(t1 - t0) / kReps;

  // MFMA result -> VALU use -> next MFMA (a tile's store/reuse path)
  t0 = __builtin_amdgcn_s_memtime();
  double x = a;
  for (int r = 0; r < kReps / 4; ++r) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, b, c0, 0, 0, 0);
    x = c0[0] * 0.5;
  }
  sink += x;
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[3] = (double)(t1 - t0) / (kReps / 4);

  // v_fma_f64 dependent chain
  double f = a;
  t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < kReps; ++r) f = fma(f, b, a);
  sink += f;
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[4] = (double)(t1 - t0) / kReps;

  // 8 independent v_fma_f64 chains
  double g[8];
  for (int k = 0; k < 8; ++k) g[k] = a + k;
  t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < kReps / 8; ++r)
#pragma unroll
    for (int k = 0; k < 8; ++k) g[k] = fma(g[k], b, a);
  for (int k = 0; k < 8; ++k) sink += g[k];
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[5] = (double)(t1 - t0) / kReps;

  // dependent LDS read chain
  int idx = lane;
  t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < kReps / 4; ++r) idx = (int)lds[idx & 1023];
  t1 = __builtin_amdgcn_s_memtime();
  sink += idx;
  if (lane == 0) out[6] = (double)(t1 - t0) / (kReps / 4);

  // v_readlane_b32 x2 + v_fma_f64 (the old pivot broadcast) dependent chain
  double h = a;
  t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < kReps / 4; ++r) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(h), 3);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(h), 3);
    h = fma(__hiloint2double(hi, lo), b, h);
  }
  t1 = __builtin_amdgcn_s_memtime();
  sink += h;
  if (lane == 0) out[7] = (double)(t1 - t0) / (kReps / 4);
  }
  __syncthreads();

  // s_barrier round trip with 8 waves (all waves of the block)
  t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < kReps / 4; ++r) __syncthreads();
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[8] = (double)(t1 - t0) / (kReps / 4);
  if (sink == 12345.678) out[15] = sink;
}

int main() {
  double* d;
  (void)hipMalloc(&d, 16 * sizeof(double));
  (void)hipMemset(d, 0, 16 * sizeof(double));
  for (int it = 0; it < 3; ++it) hipLaunchKernelGGL(k_probe, dim3(1), dim3(512), 0, 0, d, 1.0);
  double h[16];
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* names[9] = {"mfma_f64_1chain", "mfma_f64_2chains", "mfma_f64_4chains",
                          "mfma_to_valu_to_mfma", "fma_f64_dep", "fma_f64_8indep",
                          "ds_read_b64_dep", "readlane2_fma_dep", "syncthreads_8waves"};
  std::printf("{");
  for (int k = 0; k < 9; ++k) std::printf("%s\"%s\": %.1f", k ? ", " : "", names[k], h[k]);
  std::printf("}  (s_memtime cycles per op, wave 0 of a 512-thread block)\n");
  return 0;
}
