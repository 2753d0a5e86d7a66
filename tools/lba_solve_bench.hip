// Standalone timing of the LBA reduced-camera-system solve (k_lba_solve, the
// 16 x 16 MFMA-tiled LDLT) on a random SPD system, with per-phase s_memtime
// clocks (LBA_SOLVE_STAMPS) and a check of x against a host LDLT.
//   hipcc --offload-arch=gfx950 -O3 -DLBA_SOLVE_STAMPS -o build/lba_solve_bench tools/lba_solve_bench.hip
//   ./build/lba_solve_bench [n_free=18] [reps=200]
#include "../orb_slam_fusion_amd/csrc/lba_kernels.hip"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace orbgpu;

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                        \
    }                                                                  \
  } while (0)

int main(int argc, char** argv) {
  const int nf = argc > 1 ? std::atoi(argv[1]) : 18, reps = argc > 2 ? std::atoi(argv[2]) : 200;
  const int n = 6 * nf, npad = (n + 15) / 16 * 16;
  std::vector<double> sys((size_t)n * n + 2 * n);
  unsigned long long s = 12345;
  auto rnd = [&]() {
    s ^= s >> 12;
    s ^= s << 25;
    s ^= s >> 27;
    return ((s * 2685821657736338717ull) >> 11) * (1.0 / 9007199254740992.0) - 0.5;
  };
  std::vector<double> R((size_t)n * n);
  for (auto& v : R) v = rnd();
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double acc = i == j ? n : 0.0;
      for (int k = 0; k < n; ++k) acc += R[(size_t)i * n + k] * R[(size_t)j * n + k];
      sys[(size_t)i * n + j] = acc;
    }
  for (int i = 0; i < 2 * n; ++i) sys[(size_t)n * n + i] = rnd();
  const double lambda = 1e-3;
  // host LDLT of S + lambda I
  std::vector<double> A(sys.begin(), sys.begin() + (size_t)n * n), d(n), x(n);
  for (int i = 0; i < n; ++i) A[(size_t)i * n + i] += lambda;
  for (int k = 0; k < n; ++k) {
    double dk = A[(size_t)k * n + k];
    for (int j = 0; j < k; ++j) dk -= A[(size_t)k * n + j] * A[(size_t)k * n + j] * d[j];
    d[k] = dk;
    for (int i = k + 1; i < n; ++i) {
      double v = A[(size_t)i * n + k];
      for (int j = 0; j < k; ++j) v -= A[(size_t)i * n + j] * A[(size_t)k * n + j] * d[j];
      A[(size_t)i * n + k] = v / dk;
    }
  }
  for (int i = 0; i < n; ++i) {
    double v = sys[(size_t)n * n + i];
    for (int j = 0; j < i; ++j) v -= A[(size_t)i * n + j] * x[j];
    x[i] = v;
  }
  for (int i = 0; i < n; ++i) x[i] /= d[i];
  for (int i = n - 1; i >= 0; --i)
    for (int j = i + 1; j < n; ++j) x[i] -= A[(size_t)j * n + i] * x[j];

  double *d_sys, *d_xp, *d_scal, *d_work;
  LbaCtrl* d_ctrl;
  CK(hipMalloc(&d_sys, sizeof(double) * sys.size()));
  CK(hipMalloc(&d_xp, sizeof(double) * (n + 2)));
  CK(hipMalloc(&d_scal, sizeof(double) * 4));
  CK(hipMalloc(&d_work, sizeof(double) * ((size_t)npad * (npad + 1) + (npad / 16) * 272 + 2)));
  CK(hipMalloc(&d_ctrl, sizeof(LbaCtrl)));
  CK(hipMemcpy(d_sys, sys.data(), sizeof(double) * sys.size(), hipMemcpyHostToDevice));
  LbaCtrl c0{};
  c0.lambda = lambda;
  CK(hipMemcpy(d_ctrl, &c0, sizeof(c0), hipMemcpyHostToDevice));
  LbaArgs a{};
  a.n_sys = n;
  a.n_pad = npad;
  a.sys = d_sys;
  a.xp = d_xp;
  a.scal = d_scal;
  a.work = d_work;
  a.ctrl = d_ctrl;
  const size_t lds = lba_solve_lds_bytes(npad);
  const bool in_lds = lds <= 160 * 1024;
  if (in_lds) CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_lba_solve<true>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  auto launch = [&]() {
    if (in_lds)
      hipLaunchKernelGGL(k_lba_solve<true>, dim3(1), dim3(kSolveThreads), lds, 0, a);
    else
      hipLaunchKernelGGL(k_lba_solve<false>, dim3(1), dim3(kSolveThreads), 16 * (size_t)npad, 0, a);
  };
  launch();
  CK(hipDeviceSynchronize());
  unsigned long long zero[16] = {0};
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_lba_stamps), zero, sizeof(zero)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, 0));
  for (int r = 0; r < reps; ++r) launch();
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long st[16];
  CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_lba_stamps), sizeof(st)));
  std::vector<double> xg(n);
  CK(hipMemcpy(xg.data(), d_xp, sizeof(double) * n, hipMemcpyDeviceToHost));
  double err = 0, nrm = 0;
  for (int i = 0; i < n; ++i) {
    err = std::fmax(err, std::fabs(xg[i] - x[i]));
    nrm = std::fmax(nrm, std::fabs(x[i]));
  }
  const char* names[11] = {"load", "diag0", "w0_row+diag", "step_sync", "trailing(hbm path)", "dinv", "backward", "scale", "w0_row_L", "w0_row_R", "w0_row_tiles"};
  std::printf("{\"n\": %d, \"lds\": %d, \"us_per_solve\": %.2f, \"max_rel_err\": %.3e, \"clocks_per_solve\": {",
              n, in_lds ? 1 : 0, ms * 1e3 / reps, err / nrm);
  for (int k = 0; k < 11; ++k)
    std::printf("%s\"%s\": %.0f", k ? ", " : "", names[k], (double)st[k] / reps);
  std::printf("}}\n");
  return err / nrm < 1e-9 ? 0 : 2;
}
