// Cycle probe of the DPP64 elimination building blocks on one wave (gfx950):
// v_fmac_f64_dpp row_newbcast (8 independent accumulators, and a dependent
// chain), plain v_fmac_f64 (8 independent), v_rcp_f64 + Newton dependent
// chain, ds_write_b64 -> ds_read_b64 round trip.  Cycles per operation from
// s_memtime around the loop, lane 0 of wave 0 of a 512-thread block.
//   hipcc --offload-arch=gfx950 -O3 -o build/dpp_f64_probe tools/dpp_f64_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kReps = 64;

#define FMAC_DPP(d, s, m) "v_fmac_f64_dpp " d ", " s ", " m " row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
#define FMAC(d, s, m) "v_fmac_f64 " d ", " s ", " m "\n\t"

__global__ void k_probe(double* out, double seed) {
  __shared__ double lds[256];
  const int lane = threadIdx.x & 63;
  if (threadIdx.x < 64) {
    double a0 = seed + lane, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
           a6 = a0 + 6, a7 = a0 + 7;
    const double m = 1e-9 * seed;
    unsigned long long t0, t1;
    // 8 independent DPP fmacs per iteration
    t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < kReps; ++r)
      asm volatile("s_nop 1\n\t" FMAC_DPP("%0", "%1", "%8") FMAC_DPP("%1", "%2", "%8")
                       FMAC_DPP("%2", "%3", "%8") FMAC_DPP("%3", "%4", "%8") FMAC_DPP("%4", "%5", "%8")
                           FMAC_DPP("%5", "%6", "%8") FMAC_DPP("%6", "%7", "%8") FMAC_DPP("%7", "%0", "%8")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                   : "v"(m));
    t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[0] = (double)(t1 - t0) / (kReps * 8);
    // 8 independent plain fmacs
    t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < kReps; ++r)
      asm volatile(FMAC("%0", "%1", "%8") FMAC("%1", "%2", "%8") FMAC("%2", "%3", "%8")
                       FMAC("%3", "%4", "%8") FMAC("%4", "%5", "%8") FMAC("%5", "%6", "%8")
                           FMAC("%6", "%7", "%8") FMAC("%7", "%0", "%8")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                   : "v"(m));
    t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[1] = (double)(t1 - t0) / (kReps * 8);
    // dependent DPP fmac chain (each reads the previous result through DPP)
    t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < kReps; ++r)
      asm volatile("s_nop 1\n\t" FMAC_DPP("%1", "%0", "%2") "s_nop 1\n\t" FMAC_DPP("%0", "%1", "%2")
                   : "+v"(a0), "+v"(a1)
                   : "v"(m));
    t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[2] = (double)(t1 - t0) / (kReps * 2);
    // rcp + Newton + mul dependent chain (a pivot's reciprocal)
    double d = a2 + 3.0;
    t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < kReps; ++r) {
      double q = __builtin_amdgcn_rcp(d);
      q = fma(q, fma(-d, q, 1.0), q);
      d = q * 1.5 + 0.25;
      asm volatile("" : "+v"(d));
    }
    t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[3] = (double)(t1 - t0) / kReps;
    // ds_write_b64 -> ds_read_b64 of another lane's value (exchange round trip)
    double x = a3;
    t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < kReps; ++r) {
      lds[lane] = x;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      x = lds[(lane + 16) & 63] + 1.0;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[4] = (double)(t1 - t0) / kReps;
    // v_mov_b64_dpp row_newbcast dependent chain
    double y = a4;
    t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < kReps; ++r) {
      asm volatile("s_nop 1\n\tv_mov_b64_dpp %0, %1 row_newbcast:5 row_mask:0xf bank_mask:0xf"
                   : "=v"(y) : "v"(y));
    }
    t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[5] = (double)(t1 - t0) / kReps;
    if (lane == 0) out[15] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + d + x + y;
  }
}

int main() {
  double* d;
  (void)hipMalloc(&d, 16 * sizeof(double));
  (void)hipMemset(d, 0, 16 * sizeof(double));
  for (int it = 0; it < 3; ++it) hipLaunchKernelGGL(k_probe, dim3(1), dim3(512), 0, 0, d, 1.0);
  double h[16];
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* names[6] = {"fmac_f64_dpp_8indep", "fmac_f64_8indep", "fmac_f64_dpp_dep",
                          "rcp_newton_mul_dep", "ds_write_read_roundtrip", "mov_b64_dpp_dep"};
  std::printf("{");
  for (int k = 0; k < 6; ++k) std::printf("%s\"%s\": %.1f", k ? ", " : "", names[k], h[k]);
  std::printf("}  (s_memtime cycles per op, wave 0 of a 512-thread block)\n");
  return 0;
}
