// Per-frame wall clock of north_star's target sequence -- one stereo frame's
// ORB extraction + Optimizer::PoseOptimization -- called the way the C++
// drop-ins call the C ABI (no Python between the calls):
//
//   Frame():          the left / right OrbExtractor::operator() on two threads,
//                     a std::thread per frame as frame.cc:179-182 starts them;
//   ComputeStereoMatches (frame.cc:189) = orbgpu_stereo_match (its own column,
//                     not part of the extract+pose figure);
//   PoseOptimization: orbgpu_pose_opt on a 600-observation problem
//                     (optimizer.cc:762-1051).
//
// Inputs are generated in-process by liborbsynth with the seeds the Python
// leg (tools/bench_latency.py) uses, so both time the same frames.  Prints one
// JSON object: per part the median and the 90th percentile over the timed
// frames, and per frame the keypoint counts and inliers (the Python leg checks
// them against its own).
//
//   build/latency [FRAMES] [WARMUP] [stereo | pair | mono | mono_thread]
// (mono: the left image only, on the calling thread -- the extraction's own
// latency without the second thread)
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "../include/orbgpu.h"

extern "C" {
void synth_stereo_frame(uint64_t seed, int w, int h, int disparity, uint8_t* left, uint8_t* right);
void synth_pose_problem(uint64_t seed, int n, int outlier_pct, float* obs, float* cam,
                        float* pose_true, float* pose_init);
}

namespace {

constexpr uint64_t kFrameSeedBase = 0x5EED0000ull;  // synth.FRAME_SEED_BASE
constexpr uint64_t kPoseSeed = 7;                   // synth.POSE_SEED
constexpr int kW = 752, kH = 480, kObs = 600;

using Clock = std::chrono::steady_clock;
double ms(Clock::time_point a, Clock::time_point b) {
  return std::chrono::duration<double, std::milli>(b - a).count();
}
double quantile(std::vector<double> v, double q) {  // nearest rank above
  if (v.empty()) return 0.0;
  std::sort(v.begin(), v.end());
  if (q == 0.5 && v.size() % 2 == 0) return 0.5 * (v[v.size() / 2 - 1] + v[v.size() / 2]);
  size_t k = (size_t)(q * (double)v.size());
  if (k >= v.size()) k = v.size() - 1;
  return v[k];
}

#define CHECK(x)                                                   \
  do {                                                             \
    const orbgpu_status s_ = (x);                                  \
    if (s_ != ORBGPU_OK) {                                         \
      fprintf(stderr, "latency: %s -> %d\n", #x, (int)s_);         \
      return 1;                                                    \
    }                                                              \
  } while (0)

}  // namespace

int main(int argc, char** argv) {
  const int frames = argc > 1 ? atoi(argv[1]) : 40;
  const int warmup = argc > 2 ? atoi(argv[2]) : 5;
  const std::string mode = argc > 3 ? argv[3] : "stereo";
  // mono: the left image on the calling thread; mono_thread: on a std::thread
  // started per frame (the thread's own cost, as frame.cc:179-182 pays it)
  const bool mono = mode == "mono" || mode == "mono_thread", mono_thread = mode == "mono_thread";
  // pair: both images by orbgpu_extract_stereo from this thread (the Frame
  // drop-in, shim/frame_stereo_gpu.cc); stereo: a std::thread for the right
  // image per frame, as the reference's Frame constructor starts them
  const bool pair = mode == "pair";
  if (frames <= 0 || warmup < 0) return 2;

  struct In {
    std::vector<uint8_t> left, right;
    std::vector<orbgpu_pose_obs> obs;
    orbgpu_camera cam;
    orbgpu_pose pin;
  };
  std::vector<In> in(frames);
  for (int i = 0; i < frames; ++i) {
    In& f = in[i];
    f.left.resize((size_t)kW * kH), f.right.resize((size_t)kW * kH);
    synth_stereo_frame(kFrameSeedBase + i, kW, kH, 24, f.left.data(), f.right.data());
    f.obs.resize(kObs);
    float cam[5], pt[7], pi[7];
    synth_pose_problem(kPoseSeed + i, kObs, 10, reinterpret_cast<float*>(f.obs.data()), cam, pt, pi);
    f.cam = {cam[0], cam[1], cam[2], cam[3], cam[4]};
    f.pin = {pi[0], pi[1], pi[2], pi[3], pi[4], pi[5], pi[6]};
  }

  const orbgpu_orb_params params{1000, 1.2f, 8, 20, 7};
  orbgpu_extractor *exl = nullptr, *exr = nullptr;
  CHECK(orbgpu_extractor_create(&params, 0, kW, kH, 1, &exl));
  CHECK(orbgpu_extractor_create(&params, 0, kW, kH, 1, &exr));
  orbgpu_pose_ctx* pc = nullptr;
  CHECK(orbgpu_pose_ctx_create(0, 1, kObs, &pc));
  const int cap = orbgpu_extractor_max_keypoints(exl, kW, kH);
  std::vector<orbgpu_keypoint> kl(cap), kr(cap);
  std::vector<uint8_t> dl((size_t)cap * 32), dr((size_t)cap * 32), outlier(kObs);
  std::vector<float> ur(cap), depth(cap);
  const float bf = (float)(435.2 * 0.11), mb = bf / 435.2f;  // tools/bench_latency.py FX, BASE
  const int lap[2] = {0, 0};

  std::vector<double> t_ex, t_po, t_st, t_tot;
  std::vector<int> n_left(frames), n_right(frames), inliers(frames);
  for (int i = 0; i < warmup + frames; ++i) {
    const In& f = in[i % frames];
    int nl = 0, nr = 0, ml = 0, mr = 0, ninl = 0;
    const auto t0 = Clock::now();
    orbgpu_status sr = ORBGPU_OK, sl = ORBGPU_OK;
    if (mono_thread) {
      std::thread th([&] {
        sl = orbgpu_extract(exl, f.left.data(), kW, kH, kW, lap, kl.data(), dl.data(), cap, &nl, &ml);
      });
      th.join();
    } else if (mono) {
      sl = orbgpu_extract(exl, f.left.data(), kW, kH, kW, lap, kl.data(), dl.data(), cap, &nl, &ml);
    } else if (pair) {
      sl = orbgpu_extract_stereo(exl, exr, f.left.data(), f.right.data(), kW, kH, kW, lap, lap, kl.data(), dl.data(),
                                 cap, &nl, &ml, kr.data(), dr.data(), cap, &nr, &mr);
    } else {
      std::thread th([&] {
        sr = orbgpu_extract(exr, f.right.data(), kW, kH, kW, lap, kr.data(), dr.data(), cap, &nr, &mr);
      });
      sl = orbgpu_extract(exl, f.left.data(), kW, kH, kW, lap, kl.data(), dl.data(), cap, &nl, &ml);
      th.join();
    }
    const auto t1 = Clock::now();
    CHECK(sl);
    CHECK(sr);
    if (mono) {
      if (i >= warmup) t_ex.push_back(ms(t0, t1)), n_left[i % frames] = nl;
      continue;
    }
    // ComputeStereoMatches on the two handles' resident outputs (frame.cc:189):
    // its own column, not part of the extract + pose figure
    CHECK(orbgpu_stereo_match(exl, exr, bf, mb, ur.data(), depth.data(), cap));
    const auto t2 = Clock::now();
    orbgpu_pose pout;
    CHECK(orbgpu_pose_opt(pc, &f.cam, &f.pin, f.obs.data(), kObs, &pout, outlier.data(), &ninl));
    const auto t3 = Clock::now();
    if (i >= warmup) {
      t_ex.push_back(ms(t0, t1)), t_st.push_back(ms(t1, t2)), t_po.push_back(ms(t2, t3));
      t_tot.push_back(ms(t0, t1) + ms(t2, t3));
      n_left[i % frames] = nl, n_right[i % frames] = nr, inliers[i % frames] = ninl;
    }
  }
  auto list = [](const std::vector<int>& v) {
    std::string s = "[";
    for (size_t k = 0; k < v.size(); ++k) s += (k ? "," : "") + std::to_string(v[k]);
    return s + "]";
  };
  if (mono) {
    printf("{\"mode\": \"%s\", \"frames\": %d, \"gpu_extract_ms\": %.3f, \"gpu_extract_ms_p90\": %.3f}\n",
           mode.c_str(), frames, quantile(t_ex, 0.5), quantile(t_ex, 0.9));
    return 0;
  }
  printf("{\"host\": \"C++ through the C ABI (tools/latency.cc)\", \"mode\": \"%s\", \"frames\": %d, "
         "\"gpu_ms_per_frame\": %.3f, \"gpu_ms_per_frame_p90\": %.3f, "
         "\"gpu_extract_ms\": %.3f, \"gpu_extract_ms_p90\": %.3f, "
         "\"gpu_pose_ms\": %.3f, \"gpu_pose_ms_p90\": %.3f, "
         "\"gpu_stereo_ms\": %.3f, \"n_left\": %s, \"n_right\": %s, \"inliers\": %s}\n",
         mode.c_str(), frames, quantile(t_tot, 0.5), quantile(t_tot, 0.9), quantile(t_ex, 0.5), quantile(t_ex, 0.9),
         quantile(t_po, 0.5), quantile(t_po, 0.9), quantile(t_st, 0.5), list(n_left).c_str(),
         list(n_right).c_str(), list(inliers).c_str());
  orbgpu_pose_ctx_destroy(pc);
  orbgpu_extractor_destroy(exl);
  orbgpu_extractor_destroy(exr);
  return 0;
}
