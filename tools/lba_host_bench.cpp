// Host-side cost of one orbgpu_lba_optimize call (layout, staging, result
// unpacking) without a GPU: lba_api.cpp built against no-op HIP and launcher
// stubs, the C4 window from liborbsynth (iterations = 0: no LM steps).
//   hipcc -O2 -std=c++17 -o build/lba_host_bench tools/lba_host_bench.cpp -ldl
//   ./build/lba_host_bench [reps]
#define LBA_HOST_PHASES 1
#include "../orb_slam_fusion_amd/csrc/lba_api.cpp"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>

namespace orbgpu {
hipError_t lba_begin(const LbaArgs&, hipStream_t) { return hipSuccess; }
hipError_t lba_step(const LbaArgs&, hipStream_t, bool) { return hipSuccess; }
hipError_t lba_build(const LbaArgs&, hipStream_t, bool) { return hipSuccess; }
hipError_t lba_schur(const LbaArgs&, hipStream_t) { return hipSuccess; }
hipError_t lba_solve_trial(const LbaArgs&, hipStream_t) { return hipSuccess; }
hipError_t lba_ctl(const LbaArgs&, int, hipStream_t) { return hipSuccess; }
hipError_t lba_classify(const LbaArgs&, uint8_t*, double*, void*, hipStream_t) { return hipSuccess; }
hipError_t lba_classify_to_host(const LbaArgs& a, hipStream_t) {  // the results flag, as the device would
  a.host->results = (uint32_t)reinterpret_cast<const LbaCtrl*>(a.ctrl)->call;
  return hipSuccess;
}
size_t lba_solve_lds_bytes(int) { return 0; }
int lba_solve_mode(int) { return 0; }
bool lba_solve_mode_fits(int, int) { return true; }
size_t lba_solve_work_doubles(int, int) { return 1; }
}  // namespace orbgpu

extern "C" {
hipError_t hipSetDevice(int) { return hipSuccess; }
hipError_t hipFree(void* p) { std::free(p); return hipSuccess; }
hipError_t hipHostFree(void* p) { std::free(p); return hipSuccess; }
hipError_t hipMalloc(void** p, size_t n) { *p = std::malloc(n); return hipSuccess; }
hipError_t hipHostMalloc(void** p, size_t n, unsigned int) { *p = std::calloc(1, n); return hipSuccess; }
hipError_t hipHostGetDevicePointer(void** d, void* h, unsigned int) { *d = h; return hipSuccess; }
hipError_t hipMemcpyAsync(void* d, const void* s, size_t n, hipMemcpyKind, hipStream_t) {
  std::memcpy(d, s, n < 128 ? n : 128);  // the LbaCtrl at the image's head only (the call number)
  return hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
hipError_t hipStreamQuery(hipStream_t) { return hipSuccess; }
hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned int) { *s = nullptr; return hipSuccess; }
hipError_t hipStreamDestroy(hipStream_t) { return hipSuccess; }
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 200;
  // a C4-like window: 20 key frames (2 fixed), 3000 points, 6 observations each
  const int n_kf = 20, n_pts = 3000, obs = 6;
  std::mt19937 rng(7);
  std::vector<orbgpu_pose> poses(n_kf, orbgpu_pose{0, 0, 0, 1, 0, 0, 0});
  std::vector<uint8_t> fixed(n_kf, 0);
  fixed[0] = fixed[1] = 1;
  std::vector<float> pts(3 * n_pts, 1.0f);
  std::vector<orbgpu_lba_edge> edges;
  for (int p = 0; p < n_pts; ++p) {
    std::vector<int> kfs(n_kf);
    for (int k = 0; k < n_kf; ++k) kfs[k] = k;
    std::shuffle(kfs.begin(), kfs.end(), rng);
    for (int u = 0; u < obs; ++u) {
      orbgpu_lba_edge e{};
      e.point = p;
      e.kf = kfs[u];
      e.u = 100;
      e.v = 100;
      e.ur = (u & 1) ? 90.f : -1.f;
      e.inv_sigma2 = 1;
      edges.push_back(e);
    }
  }
  if (std::getenv("SHUFFLE")) std::shuffle(edges.begin(), edges.end(), rng);  // the reference inserts point-major (optimizer.cc:1187-1262)
  orbgpu_lba_ctx* h = nullptr;
  if (orbgpu_lba_ctx_create(0, &h) != ORBGPU_OK) return 1;
  orbgpu_camera cam{400, 400, 300, 200, 40};
  std::vector<orbgpu_pose> po(n_kf);
  std::vector<double> pd(7 * n_kf);
  std::vector<float> xo(3 * n_pts);
  std::vector<uint8_t> out(edges.size());
  double st[6];
  double best = 1e30, tot = 0;
  for (int r = 0; r < reps; ++r) {
    const auto t0 = std::chrono::steady_clock::now();
    orbgpu_lba_optimize(h, &cam, n_kf, poses.data(), fixed.data(), n_pts, pts.data(), (int)edges.size(),
                        edges.data(), 0, n_pts, 0, 0.0, nullptr, nullptr, nullptr, po.data(), pd.data(),
                        xo.data(), out.data(), st);
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    best = std::min(best, us);
    tot += us;
  }
  std::printf("{\"edges\": %zu, \"host_us_best\": %.1f, \"host_us_mean\": %.1f, \"phases_us\": [", edges.size(), best,
              tot / reps);
  for (int k = 1; k <= 10; ++k) std::printf("%s%.1f", k > 1 ? ", " : "", g_host_phase_us[k] / reps);
  std::printf("]}\n");
  if (std::getenv("LIA")) {
    // the LocalInertialBA layout on the same graph: 12 free key frames with
    // IMU, 8 fixed, a link between consecutive key frames (the last flagged
    // robust + downweighted), iterations = 0 (the explicit results launch)
    std::vector<orbgpu_imu_state> ks(n_kf);
    for (auto& k : ks) {
      std::memset(&k, 0, sizeof(k));
      k.Rwb[0] = k.Rwb[4] = k.Rwb[8] = 1.f;
      k.Rcw[0] = k.Rcw[4] = k.Rcw[8] = 1.f;
    }
    std::vector<uint8_t> lfixed(n_kf, 0), has_imu(n_kf, 1), close(n_pts, 0);
    for (int k = 12; k < n_kf; ++k) lfixed[k] = 1;
    std::vector<orbgpu_lia_imu_edge> links;
    for (int k = 1; k < 13; ++k) {
      orbgpu_lia_imu_edge l;
      std::memset(&l, 0, sizeof(l));
      l.kf1 = k;
      l.kf2 = k - 1;
      l.flags = k == 12 ? (ORBGPU_LIA_ROBUST | ORBGPU_LIA_DOWNWEIGHT) : 0;
      l.preint.dT = 0.2f;
      links.push_back(l);
    }
    orbgpu_imu_calib cal;
    std::memset(&cal, 0, sizeof(cal));
    std::vector<orbgpu_imu_state> ko(n_kf);
    std::vector<double> kd(21 * n_kf);
    double ls[7];
    const orbgpu_status r = orbgpu_lia_optimize(h, &cal, n_kf, ks.data(), lfixed.data(), has_imu.data(), n_pts,
                                                pts.data(), close.data(), (int)edges.size(), edges.data(),
                                                (int)links.size(), links.data(), 0, 1e-2, ko.data(), kd.data(),
                                                xo.data(), out.data(), ls);
    std::printf("{\"lia_status\": %d}\n", (int)r);
    if (r != ORBGPU_OK) return 2;
  }
  orbgpu_lba_ctx_destroy(h);
  return 0;
}
