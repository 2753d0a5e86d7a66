// Per-frame wall clock of the stereo-inertial tracking thread after IMU
// initialisation, called the way the C++ drop-ins call the C ABI (no Python
// between the calls): the inputs tools/bench_latency_inertial.py --dump wrote
// (the same frames, local maps and IMU states its Python leg times), one frame
// at a time --
//
//   Frame():        the left / right extraction of frame.cc:179-182 from this
//                   thread, both launches in flight (orbgpu_extract_stereo, the
//                   ORBGPU_STEREO Frame shim; "threads" as 2nd argument: a
//                   std::thread per frame as the reference starts them), then
//                   ComputeStereoMatches (:189) = orbgpu_stereo_match;
//   SearchLocalPoints: isInFrustum + SearchByProjection(F, vpMapPoints, th 6,
//                   nn 0.8) = orbgpu_search_local_points (tracking.cc:2626-2690);
//   PoseInertialOptimizationLastFrame over the matches it left: the
//                   observation rows gathered on the host from the Frame fields
//                   as the reference's graph build does (optimizer.cc:4806-4880),
//                   then orbgpu_pose_inertial.
//
// Prints one JSON object: medians (and p90s) per part and per frame, and
// whether every frame's observation count and n_good equal the Python leg's
// (same work).
//
//   build/latency_inertial DUMP [WARMUP] [stereo|threads] [REPS]  (REPS passes over the frames)
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "../include/orbgpu.h"

namespace {

struct Frame {
  std::vector<uint8_t> left, right;
  float R[9], t[3], Ow[3];
  std::vector<orbgpu_map_point> pts;
  orbgpu_imu_state cur, prev;
  orbgpu_imu_preint preint;
  orbgpu_imu_prior prior;
  int expect_nobs, expect_good;
};

struct Dump {
  int frames, W, H, n_levels, cap;
  orbgpu_orb_params params;
  float bf, mb, th, nn, view_cos;
  orbgpu_frame_geom geom;
  orbgpu_camera cam;
  orbgpu_imu_calib calib;
  std::vector<float> inv_sigma2;
  std::vector<Frame> f;
};

bool rd(FILE* fp, void* p, size_t n) { return fread(p, 1, n, fp) == n; }

bool load(const char* path, Dump& d) {
  FILE* fp = fopen(path, "rb");
  if (!fp) return false;
  char magic[8];
  int32_t hdr[5], sizes[8];
  bool ok = rd(fp, magic, 8) && memcmp(magic, "OSLATIN1", 8) == 0 && rd(fp, hdr, sizeof hdr) &&
            rd(fp, sizes, sizeof sizes);
  const int32_t want[8] = {(int32_t)sizeof(orbgpu_frame_geom),  (int32_t)sizeof(orbgpu_camera),
                           (int32_t)sizeof(orbgpu_map_point),   (int32_t)sizeof(orbgpu_imu_calib),
                           (int32_t)sizeof(orbgpu_imu_state),   (int32_t)sizeof(orbgpu_imu_preint),
                           (int32_t)sizeof(orbgpu_imu_prior),   (int32_t)sizeof(orbgpu_inertial_obs)};
  if (!ok || memcmp(sizes, want, sizeof want) != 0) {
    fprintf(stderr, "latency_inertial: bad dump header or struct sizes\n");
    fclose(fp);
    return false;
  }
  d.frames = hdr[0], d.W = hdr[1], d.H = hdr[2], d.n_levels = hdr[3], d.cap = hdr[4];
  float fl[5];
  ok = rd(fp, &d.params, sizeof d.params) && rd(fp, fl, sizeof fl) && rd(fp, &d.geom, sizeof d.geom) &&
       rd(fp, &d.cam, sizeof d.cam) && rd(fp, &d.calib, sizeof d.calib);
  d.bf = fl[0], d.mb = fl[1], d.th = fl[2], d.nn = fl[3], d.view_cos = fl[4];
  d.inv_sigma2.resize(d.n_levels);
  ok = ok && rd(fp, d.inv_sigma2.data(), 4 * d.n_levels);
  d.f.resize(d.frames);
  for (Frame& f : d.f) {
    const size_t px = (size_t)d.W * d.H;
    f.left.resize(px), f.right.resize(px);
    int32_t np = 0, ex[2];
    ok = ok && rd(fp, f.left.data(), px) && rd(fp, f.right.data(), px) && rd(fp, f.R, 36) &&
         rd(fp, f.t, 12) && rd(fp, f.Ow, 12) && rd(fp, &np, 4);
    if (!ok || np < 0) break;
    f.pts.resize(np);
    ok = ok && rd(fp, f.pts.data(), sizeof(orbgpu_map_point) * np) && rd(fp, &f.cur, sizeof f.cur) &&
         rd(fp, &f.prev, sizeof f.prev) && rd(fp, &f.preint, sizeof f.preint) &&
         rd(fp, &f.prior, sizeof f.prior) && rd(fp, ex, sizeof ex);
    f.expect_nobs = ex[0], f.expect_good = ex[1];
  }
  fclose(fp);
  if (!ok) fprintf(stderr, "latency_inertial: truncated dump\n");
  return ok;
}

#define CHECK(x)                                                          \
  do {                                                                    \
    const orbgpu_status s_ = (x);                                         \
    if (s_ != ORBGPU_OK) {                                                \
      fprintf(stderr, "latency_inertial: %s -> %d\n", #x, (int)s_);       \
      return 1;                                                           \
    }                                                                     \
  } while (0)

using Clock = std::chrono::steady_clock;
double ms(Clock::time_point a, Clock::time_point b) {
  return std::chrono::duration<double, std::milli>(b - a).count();
}
double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  const size_t n = v.size();
  return n == 0 ? 0.0 : (n % 2 ? v[n / 2] : 0.5 * (v[n / 2 - 1] + v[n / 2]));
}
double p90(std::vector<double> v) {  // nearest rank
  if (v.empty()) return 0.0;
  std::sort(v.begin(), v.end());
  return v[std::min(v.size() - 1, (size_t)(0.9 * (double)v.size()))];
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s DUMP [WARMUP]\n", argv[0]);
    return 2;
  }
  const int warmup = argc > 2 ? atoi(argv[2]) : 3;
  const bool two_threads = argc > 3 && strcmp(argv[3], "threads") == 0;
  const int reps = argc > 4 ? std::max(1, atoi(argv[4])) : 1;
  Dump d;
  if (!load(argv[1], d)) return 1;

  orbgpu_extractor *exl = nullptr, *exr = nullptr;
  CHECK(orbgpu_extractor_create(&d.params, 0, d.W, d.H, 1, &exl));
  CHECK(orbgpu_extractor_create(&d.params, 0, d.W, d.H, 1, &exr));
  size_t max_pts = 1;
  for (const Frame& f : d.f) max_pts = std::max(max_pts, f.pts.size());
  orbgpu_matcher* mt = nullptr;
  CHECK(orbgpu_matcher_create(0, d.cap, (int)max_pts, &mt));
  orbgpu_inertial_ctx* ic = nullptr;
  CHECK(orbgpu_inertial_ctx_create(0, 1, d.cap, &ic));

  // the Frame's fields (sized once, as the reference's vectors are reused)
  std::vector<orbgpu_keypoint> kl(d.cap), kr(d.cap);
  std::vector<uint8_t> dl((size_t)d.cap * 32), dr((size_t)d.cap * 32);
  std::vector<float> ur(d.cap), depth(d.cap);
  std::vector<orbgpu_track_view> views(max_pts);
  std::vector<int32_t> match(d.cap);
  std::vector<orbgpu_inertial_obs> obs(d.cap);
  std::vector<uint8_t> outlier(d.cap);
  orbgpu_inertial_result res;
  const int lap[2] = {0, 0};

  std::vector<double> t_ex, t_st, t_sl, t_pi, t_tot;
  bool same = true;
  for (int i = 0; i < warmup + d.frames * reps; ++i) {
    const Frame& f = d.f[i % d.frames];
    const auto t0 = Clock::now();
    int nl = 0, nr = 0, ml = 0, mr = 0;
    if (two_threads) {
      orbgpu_status sr = ORBGPU_OK;
      std::thread th([&] {
        sr = orbgpu_extract(exr, f.right.data(), d.W, d.H, d.W, lap, kr.data(), dr.data(), d.cap, &nr, &mr);
      });
      const orbgpu_status sl =
          orbgpu_extract(exl, f.left.data(), d.W, d.H, d.W, lap, kl.data(), dl.data(), d.cap, &nl, &ml);
      th.join();
      CHECK(sl);
      CHECK(sr);
    } else {
      CHECK(orbgpu_extract_stereo(exl, exr, f.left.data(), f.right.data(), d.W, d.H, d.W, lap, lap, kl.data(),
                                  dl.data(), d.cap, &nl, &ml, kr.data(), dr.data(), d.cap, &nr, &mr));
    }
    const auto t1 = Clock::now();
    CHECK(orbgpu_stereo_match(exl, exr, d.bf, d.mb, ur.data(), depth.data(), d.cap));
    const auto t2 = Clock::now();
    int nm = 0;
    CHECK(orbgpu_search_local_points(mt, &d.geom, &d.cam, f.R, f.t, f.Ow, kl.data(), dl.data(),
                                     ur.data(), nullptr, nl, f.pts.data(), (int)f.pts.size(),
                                     d.view_cos, d.th, d.nn, 0, 0.f, views.data(), match.data(), &nm));
    const auto t3 = Clock::now();
    int n = 0;
    for (int k = 0; k < nl; ++k) {
      const int j = match[k];
      if (j < 0) continue;
      orbgpu_inertial_obs& o = obs[n++];
      memcpy(o.Xw, f.pts[j].Xw, sizeof o.Xw);
      o.u = kl[k].x, o.v = kl[k].y, o.ur = ur[k];
      o.inv_sigma2 = d.inv_sigma2[kl[k].octave];
      o.close = views[j].in_view != 0 && views[j].depth < 10.0f;
    }
    CHECK(orbgpu_pose_inertial(ic, ORBGPU_INERTIAL_LAST_FRAME, &d.calib, &f.cur, &f.prev, &f.preint,
                               &f.prior, obs.data(), n, 0, &res, outlier.data()));
    const auto t4 = Clock::now();
    if (i >= warmup) {
      t_ex.push_back(ms(t0, t1)), t_st.push_back(ms(t1, t2)), t_sl.push_back(ms(t2, t3));
      t_pi.push_back(ms(t3, t4)), t_tot.push_back(ms(t0, t4));
      if (n != f.expect_nobs || res.n_good != f.expect_good) {
        fprintf(stderr, "frame %d: %d observations, n_good %d (Python leg: %d, %d)\n", i % d.frames, n,
                res.n_good, f.expect_nobs, f.expect_good);
        same = false;
      }
    }
  }
  printf("{\"host\": \"C++ through the C ABI (tools/latency_inertial.cc)\", \"extraction\": \"%s\", "
         "\"frames\": %d, \"gpu_ms_per_frame\": %.3f, \"gpu_ms_per_frame_p90\": %.3f, "
         "\"gpu_extract_ms\": %.3f, \"gpu_extract_ms_p90\": %.3f, \"gpu_stereo_ms\": %.3f, "
         "\"gpu_search_local_ms\": %.3f, \"gpu_pose_inertial_ms\": %.3f, \"gpu_pose_inertial_ms_p90\": %.3f, "
         "\"same_work_as_python_leg\": %s}\n",
         two_threads ? "two std::threads (frame.cc:179-182)" : "orbgpu_extract_stereo from one thread", d.frames,
         median(t_tot), p90(t_tot), median(t_ex), p90(t_ex), median(t_st), median(t_sl), median(t_pi), p90(t_pi),
         same ? "true" : "false");
  orbgpu_inertial_ctx_destroy(ic);
  orbgpu_matcher_destroy(mt);
  orbgpu_extractor_destroy(exl);
  orbgpu_extractor_destroy(exr);
  return same ? 0 : 3;
}
