// Deterministic synthetic workloads: stereo frames for the
// extractor and seeded pose-only problems.  Host-only helper library
// (liborbsynth.so) shared by tests/ and bench.py so both sides of every parity
// and timing run see byte-identical inputs.  Not part of the hot path.
#include <array>
#include <cmath>
#include <cstdio>
#include <string>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

struct XorShift64Star {
  uint64_t s;
  explicit XorShift64Star(uint64_t seed) : s(seed ? seed : 0x9E3779B97F4A7C15ull) {}
  uint64_t next() {
    s ^= s >> 12;
    s ^= s << 25;
    s ^= s >> 27;
    return s * 0x2545F4914F6CDD1Dull;
  }
  int uniform(int lo, int hi) {  // inclusive
    return lo + (int)((next() >> 33) % (uint64_t)(hi - lo + 1));
  }
  double unit() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
  double gauss() {  // Box-Muller
    double u1 = unit(), u2 = unit();
    if (u1 < 1e-300) u1 = 1e-300;
    return std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
  }
};

}  // namespace

namespace {

// Canvas = vertical gradient 40..200, 300 axis-aligned rectangles (sides
// U[4,60], grey U[0,255]), 150 discs (radius U[3,25]), then per-pixel U[-6,6]
// noise, clamped.
std::vector<int> make_canvas(uint64_t seed, int cw, int h, int n_rect = 300, int n_disc = 150) {
  std::vector<int> c((size_t)cw * h);
  XorShift64Star rng(seed);
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < cw; ++x) c[(size_t)y * cw + x] = 40 + (160 * y) / (h > 1 ? h - 1 : 1);
  for (int r = 0; r < n_rect; ++r) {
    const int x0 = rng.uniform(0, cw - 1), y0 = rng.uniform(0, h - 1);
    const int rw = rng.uniform(4, 60), rh = rng.uniform(4, 60), g = rng.uniform(0, 255);
    for (int y = y0; y < y0 + rh && y < h; ++y)
      for (int x = x0; x < x0 + rw && x < cw; ++x) c[(size_t)y * cw + x] = g;
  }
  for (int d = 0; d < n_disc; ++d) {
    const int x0 = rng.uniform(0, cw - 1), y0 = rng.uniform(0, h - 1);
    const int rad = rng.uniform(3, 25), g = rng.uniform(0, 255);
    for (int y = y0 - rad; y <= y0 + rad; ++y)
      for (int x = x0 - rad; x <= x0 + rad; ++x)
        if (y >= 0 && y < h && x >= 0 && x < cw &&
            (x - x0) * (x - x0) + (y - y0) * (y - y0) <= rad * rad)
          c[(size_t)y * cw + x] = g;
  }
  for (size_t i = 0; i < c.size(); ++i) {
    int v = c[i] + rng.uniform(-6, 6);
    c[i] = v < 0 ? 0 : v > 255 ? 255 : v;
  }
  return c;
}

void crop(const std::vector<int>& c, int cw, int w, int h, int x0, uint8_t* out) {
  if (!out) return;
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) out[(size_t)y * w + x] = (uint8_t)c[(size_t)y * cw + x + x0];
}

}  // namespace

extern "C" {

// Stereo pair from one canvas of width w + disparity: left(x) = canvas(x),
// right(x) = canvas(x + disparity).  seed = 0x5EED0000 + frame.
void synth_stereo_frame(uint64_t seed, int w, int h, int disparity, uint8_t* left,
                        uint8_t* right) {
  const int cw = w + disparity;
  const std::vector<int> c = make_canvas(seed, cw, h);
  crop(c, cw, w, h, 0, left);
  crop(c, cw, w, h, disparity, right);
}

// Two consecutive stereo frames of a camera translating along x over the
// fronto-parallel canvas plane (depth bf / disparity): last(x) = canvas(x +
// shift), current(x) = canvas(x), so every feature moves +shift px from the
// last frame to the current one.  Canvas width w + disparity + shift.
void synth_track_pair(uint64_t seed, int w, int h, int disparity, int shift, uint8_t* last_l,
                      uint8_t* last_r, uint8_t* cur_l, uint8_t* cur_r) {
  const int cw = w + disparity + shift;
  const std::vector<int> c = make_canvas(seed, cw, h);
  crop(c, cw, w, h, shift, last_l);
  crop(c, cw, w, h, shift + disparity, last_r);
  crop(c, cw, w, h, 0, cur_l);
  crop(c, cw, w, h, disparity, cur_r);
}

// A stereo sequence of n_frames frames of a camera translating along x over
// the canvas plane (configs C3 / C5 on synthetic data): frame k crops the
// canvas at (n_frames - 1 - k) * shift, so every feature moves +shift px
// per frame; the object counts scale with the canvas width (the density of
// one 752-px frame).  left_all / right_all: n_frames * w * h bytes.
void synth_sequence(uint64_t seed, int n_frames, int w, int h, int disparity, int shift,
                    uint8_t* left_all, uint8_t* right_all) {
  const int cw = w + disparity + shift * (n_frames - 1);
  const double k = (double)cw / (double)(w + disparity);
  const std::vector<int> c = make_canvas(seed, cw, h, (int)(300 * k), (int)(150 * k));
  for (int f = 0; f < n_frames; ++f) {
    const int x0 = (n_frames - 1 - f) * shift;
    crop(c, cw, w, h, x0, left_all + (size_t)f * w * h);
    crop(c, cw, w, h, x0 + disparity, right_all + (size_t)f * w * h);
  }
}

// Plain noise image (stress case: dense FAST responses, large octree input).
void synth_noise_image(uint64_t seed, int w, int h, uint8_t* out) {
  XorShift64Star rng(seed);
  for (size_t i = 0; i < (size_t)w * h; ++i) out[i] = (uint8_t)rng.uniform(0, 255);
}

}  // extern "C"

namespace {
void quat_from_axis_angle(double ax, double ay, double az, double ang, double q[4]) {
  const double n = std::sqrt(ax * ax + ay * ay + az * az);
  const double s = std::sin(ang / 2) / n;
  q[0] = ax * s;
  q[1] = ay * s;
  q[2] = az * s;
  q[3] = std::cos(ang / 2);
}
void quat_mul(const double a[4], const double b[4], double r[4]) {  // (x, y, z, w)
  r[3] = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
  r[0] = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
  r[1] = a[3] * b[1] + a[1] * b[3] + a[2] * b[0] - a[0] * b[2];
  r[2] = a[3] * b[2] + a[2] * b[3] + a[0] * b[1] - a[1] * b[0];
}
void quat_rotate(const double q[4], const double v[3], double o[3]) {
  const double p[4] = {v[0], v[1], v[2], 0};
  const double qc[4] = {-q[0], -q[1], -q[2], q[3]};
  double t[4], r[4];
  quat_mul(q, p, t);
  quat_mul(t, qc, r);
  o[0] = r[0];
  o[1] = r[1];
  o[2] = r[2];
}
}  // namespace

extern "C" {

// Seeded pose-only problem: n matches, ~70 % stereo, points
// uniform in the 752x480 EuRoC frustum at depth U[1,8] m, octave U{0..7},
// Gaussian pixel noise sigma = 1.2^octave, `outlier_pct` % gross outliers
// (+-U[20,60] px), initial pose = truth perturbed by 2 cm / 0.5 deg.
// obs: n x 7 floats {Xw[3], u, v, ur (<0 mono), inv_sigma2};
// cam: {fx, fy, cx, cy, bf}; poses (qx, qy, qz, qw, tx, ty, tz).
void synth_pose_problem(uint64_t seed, int n, int outlier_pct, float* obs, float* cam,
                        float* pose_true, float* pose_init) {
  XorShift64Star rng(seed * 0x9E3779B97F4A7C15ull + 7);
  const double fx = 458.654, fy = 457.296, cx = 367.215, cy = 248.375, bf = 0.11 * fx;
  cam[0] = (float)fx;
  cam[1] = (float)fy;
  cam[2] = (float)cx;
  cam[3] = (float)cy;
  cam[4] = (float)bf;
  double q[4], t[3];
  quat_from_axis_angle(rng.unit() - 0.5, rng.unit() - 0.5, rng.unit() - 0.5, 0.6 * rng.unit(), q);
  for (int k = 0; k < 3; ++k) t[k] = 2.0 * (rng.unit() - 0.5);
  const double qc[4] = {-q[0], -q[1], -q[2], q[3]};
  for (int i = 0; i < n; ++i) {
    const double u = 60 + rng.unit() * (752 - 61), v = rng.unit() * 479;
    const double z = 1 + 7 * rng.unit();
    const double Xc[3] = {(u - cx) / fx * z, (v - cy) / fy * z, z};
    const double d[3] = {Xc[0] - t[0], Xc[1] - t[1], Xc[2] - t[2]};
    double Xw[3];
    quat_rotate(qc, d, Xw);
    const int oct = rng.uniform(0, 7);
    float s2 = 1.0f;
    for (int l = 0; l < oct; ++l) s2 = (float)(s2 * 1.2) * 1.0f;
    const float scale = s2;
    const float inv_sigma2 = 1.0f / (scale * scale);
    const double sig = scale;
    const double u_true = fx * Xc[0] / z + cx, v_true = fy * Xc[1] / z + cy;
    double uo = u_true + sig * rng.gauss();
    double vo = v_true + sig * rng.gauss();
    const bool stereo = (i % 10) < 7;
    double ur = stereo ? u_true - bf / z + sig * rng.gauss() : -1.0;
    if (rng.uniform(0, 99) < outlier_pct) {
      const double du = (rng.uniform(0, 1) ? 1 : -1) * (20 + 40 * rng.unit());
      const double dv = (rng.uniform(0, 1) ? 1 : -1) * (20 + 40 * rng.unit());
      uo += du;
      vo += dv;
      if (stereo) ur += du;
    }
    if (stereo && ur < 0) ur = 0;
    float* o = obs + 7 * i;
    o[0] = (float)Xw[0];
    o[1] = (float)Xw[1];
    o[2] = (float)Xw[2];
    o[3] = (float)uo;
    o[4] = (float)vo;
    o[5] = (float)ur;
    o[6] = inv_sigma2;
  }
  for (int k = 0; k < 4; ++k) pose_true[k] = (float)q[k];
  for (int k = 0; k < 3; ++k) pose_true[4 + k] = (float)t[k];
  double dq[4], qi[4];
  quat_from_axis_angle(rng.unit() - 0.5, rng.unit() - 0.5, rng.unit() - 0.5,
                       0.5 * 3.14159265358979 / 180, dq);
  quat_mul(dq, q, qi);
  double dir[3] = {rng.unit() - 0.5, rng.unit() - 0.5, rng.unit() - 0.5};
  const double dn = std::sqrt(dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2]);
  for (int k = 0; k < 4; ++k) pose_init[k] = (float)qi[k];
  for (int k = 0; k < 3; ++k) pose_init[4 + k] = (float)(t[k] + 0.02 * dir[k] / dn);
  // unit quaternion in float, w >= 0
  float nq = 0;
  for (int k = 0; k < 4; ++k) nq += pose_init[k] * pose_init[k];
  nq = std::sqrt(nq);
  const float sgn = pose_init[3] < 0 ? -1.f : 1.f;
  for (int k = 0; k < 4; ++k) pose_init[k] = sgn * pose_init[k] / nq;
}

}  // extern "C"

namespace {
// Rotation matrix (row-major) -> unit quaternion (x, y, z, w), w >= 0.
void quat_from_matrix(const double R[3][3], double q[4]) {
  const double tr = R[0][0] + R[1][1] + R[2][2];
  if (tr > 0) {
    const double s = std::sqrt(tr + 1.0) * 2;
    q[3] = 0.25 * s;
    q[0] = (R[2][1] - R[1][2]) / s;
    q[1] = (R[0][2] - R[2][0]) / s;
    q[2] = (R[1][0] - R[0][1]) / s;
  } else if (R[0][0] > R[1][1] && R[0][0] > R[2][2]) {
    const double s = std::sqrt(1.0 + R[0][0] - R[1][1] - R[2][2]) * 2;
    q[3] = (R[2][1] - R[1][2]) / s;
    q[0] = 0.25 * s;
    q[1] = (R[0][1] + R[1][0]) / s;
    q[2] = (R[0][2] + R[2][0]) / s;
  } else if (R[1][1] > R[2][2]) {
    const double s = std::sqrt(1.0 + R[1][1] - R[0][0] - R[2][2]) * 2;
    q[3] = (R[0][2] - R[2][0]) / s;
    q[0] = (R[0][1] + R[1][0]) / s;
    q[1] = 0.25 * s;
    q[2] = (R[1][2] + R[2][1]) / s;
  } else {
    const double s = std::sqrt(1.0 + R[2][2] - R[0][0] - R[1][1]) * 2;
    q[3] = (R[1][0] - R[0][1]) / s;
    q[0] = (R[0][2] + R[2][0]) / s;
    q[1] = (R[1][2] + R[2][1]) / s;
    q[2] = 0.25 * s;
  }
  if (q[3] < 0)
    for (int k = 0; k < 4; ++k) q[k] = -q[k];
}
void store_pose(const double q[4], const double t[3], float* o) {
  double n = 0;
  for (int k = 0; k < 4; ++k) n += q[k] * q[k];
  n = std::sqrt(n);
  for (int k = 0; k < 4; ++k) o[k] = (float)(q[k] / n);
  for (int k = 0; k < 3; ++k) o[4 + k] = (float)t[k];
}
}  // namespace

extern "C" {

// Seeded LocalBundleAdjustment window: n_kf
// keyframes on a 4 m arc (radius 6 m) all facing a 4 x 3 x 2 m box of n_pts
// points centred on the world origin; point j is observed by the obs_per_pt
// consecutive keyframes (j + i) mod n_kf, i < obs_per_pt, in ascending
// keyframe order; half the observations stereo; octave U{0..7}, pixel noise
// sigma = 1.2^octave; `outlier_pct` % gross outliers (+-U[20,60] px).  The
// first n_fixed keyframes are fixed.  Initial guesses: poses perturbed by
// 5 cm / 1 deg, points by 5 cm.  Poses are Tcw (qx, qy, qz, qw, tx, ty, tz);
// edges are {point, kf, u, v, ur (< 0: mono), inv_sigma2} (int, int, 4 floats).
// Returns the number of edges (n_pts * obs_per_pt).
int synth_lba_problem(uint64_t seed, int n_kf, int n_pts, int obs_per_pt, int n_fixed,
                      int outlier_pct, float* cam, float* poses_true, float* poses_init,
                      uint8_t* fixed, float* pts_true, float* pts_init, void* edges) {
  XorShift64Star rng(seed * 0x9E3779B97F4A7C15ull + 11);
  const double fx = 458.654, fy = 457.296, cx = 367.215, cy = 248.375, bf = 0.11 * fx;
  cam[0] = (float)fx;
  cam[1] = (float)fy;
  cam[2] = (float)cx;
  cam[3] = (float)cy;
  cam[4] = (float)bf;
  const double radius = 6.0, arc = 4.0;
  std::vector<double> Rcw((size_t)n_kf * 9), tcw((size_t)n_kf * 3);
  for (int k = 0; k < n_kf; ++k) {
    const double th = -0.5 * arc / radius + (n_kf > 1 ? k * (arc / radius) / (n_kf - 1) : 0.0);
    const double C[3] = {radius * std::sin(th), 0.0, -radius * std::cos(th)};
    double z[3] = {-C[0], -C[1], -C[2]};
    const double zn = std::sqrt(z[0] * z[0] + z[1] * z[1] + z[2] * z[2]);
    for (double& v : z) v /= zn;
    const double up[3] = {0, -1, 0};  // image rows grow downwards
    double x[3] = {up[1] * z[2] - up[2] * z[1], up[2] * z[0] - up[0] * z[2], up[0] * z[1] - up[1] * z[0]};
    const double xn = std::sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
    for (double& v : x) v /= xn;
    const double y[3] = {z[1] * x[2] - z[2] * x[1], z[2] * x[0] - z[0] * x[2], z[0] * x[1] - z[1] * x[0]};
    double R[3][3];  // rows = camera axes in world coordinates (R_cw)
    for (int c = 0; c < 3; ++c) {
      R[0][c] = x[c];
      R[1][c] = y[c];
      R[2][c] = z[c];
    }
    double t[3];
    for (int r = 0; r < 3; ++r) t[r] = -(R[r][0] * C[0] + R[r][1] * C[1] + R[r][2] * C[2]);
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) Rcw[(size_t)k * 9 + 3 * r + c] = R[r][c];
    for (int r = 0; r < 3; ++r) tcw[(size_t)k * 3 + r] = t[r];
    double q[4];
    quat_from_matrix(R, q);
    store_pose(q, t, poses_true + 7 * k);
    // perturbed initial pose: 1 deg about a random axis, 5 cm along a random direction
    double dq[4], qi[4];
    quat_from_axis_angle(rng.unit() - 0.5, rng.unit() - 0.5, rng.unit() - 0.5,
                         3.14159265358979 / 180, dq);
    quat_mul(dq, q, qi);
    double dir[3] = {rng.unit() - 0.5, rng.unit() - 0.5, rng.unit() - 0.5};
    const double dn = std::sqrt(dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2]);
    double ti[3];
    for (int r = 0; r < 3; ++r) ti[r] = t[r] + 0.05 * dir[r] / dn;
    if (k < n_fixed) {
      store_pose(q, t, poses_init + 7 * k);
    } else {
      if (qi[3] < 0)
        for (double& v : qi) v = -v;
      store_pose(qi, ti, poses_init + 7 * k);
    }
    fixed[k] = k < n_fixed ? 1 : 0;
  }
  struct Edge {
    int32_t point, kf;
    float u, v, ur, inv_sigma2;
  };
  Edge* E = static_cast<Edge*>(edges);
  int ne = 0;
  for (int j = 0; j < n_pts; ++j) {
    const double X[3] = {4.0 * (rng.unit() - 0.5), 3.0 * (rng.unit() - 0.5), 2.0 * (rng.unit() - 0.5)};
    for (int c = 0; c < 3; ++c) pts_true[3 * j + c] = (float)X[c];
    double dir[3] = {rng.unit() - 0.5, rng.unit() - 0.5, rng.unit() - 0.5};
    const double dn = std::sqrt(dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2]);
    for (int c = 0; c < 3; ++c) pts_init[3 * j + c] = (float)(X[c] + 0.05 * dir[c] / dn);
    // observing keyframes in ascending index order
    std::vector<int> kfs;
    for (int i = 0; i < obs_per_pt && i < n_kf; ++i) kfs.push_back((j + i) % n_kf);
    for (size_t a = 1; a < kfs.size(); ++a)
      for (size_t b = a; b > 0 && kfs[b - 1] > kfs[b]; --b) std::swap(kfs[b - 1], kfs[b]);
    for (int k : kfs) {
      const double* R = &Rcw[(size_t)k * 9];
      const double* t = &tcw[(size_t)k * 3];
      double Xc[3];
      for (int r = 0; r < 3; ++r) Xc[r] = R[3 * r] * X[0] + R[3 * r + 1] * X[1] + R[3 * r + 2] * X[2] + t[r];
      const int oct = rng.uniform(0, 7);
      float s2 = 1.0f;
      for (int l = 0; l < oct; ++l) s2 = (float)(s2 * 1.2) * 1.0f;
      const float inv_sigma2 = 1.0f / (s2 * s2);
      const double sig = s2;
      const double u_true = fx * Xc[0] / Xc[2] + cx, v_true = fy * Xc[1] / Xc[2] + cy;
      double uo = u_true + sig * rng.gauss(), vo = v_true + sig * rng.gauss();
      const bool stereo = rng.unit() < 0.5;
      double ur = stereo ? u_true - bf / Xc[2] + sig * rng.gauss() : -1.0;
      if (rng.uniform(0, 99) < outlier_pct) {
        const double du = (rng.uniform(0, 1) ? 1 : -1) * (20 + 40 * rng.unit());
        const double dv = (rng.uniform(0, 1) ? 1 : -1) * (20 + 40 * rng.unit());
        uo += du;
        vo += dv;
        if (stereo) ur += du;
      }
      if (stereo && ur < 0) ur = 0;
      E[ne++] = Edge{j, k, (float)uo, (float)vo, (float)ur, inv_sigma2};
    }
  }
  return ne;
}

// DBoW2 text vocabulary (TemplatedVocabulary::saveToTextFile layout,
// TemplatedVocabulary.h:1333-1353): a full k-ary tree of depth L, nodes in
// breadth-first order; a child's descriptor is its parent's with each bit
// flipped with probability 1/4 (so a descent stays coherent), one sibling in
// 16 duplicates its left neighbour (ties); leaf weights U[0.2, 8] (idf-like),
// stop_pct percent of them 0 (stopped words); inner nodes weight 0.
// trailing_newline reproduces the reference writer's final endl.  Returns the
// number of nodes written (root excluded) or -1.
int synth_vocab_text(uint64_t seed, int k, int L, int scoring, int weighting, int stop_pct,
                     int trailing_newline, const char* path) {
  FILE* f = std::fopen(path, "w");
  if (!f) return -1;
  XorShift64Star rng(seed);
  std::fprintf(f, "%d %d  %d %d\n", k, L, scoring, weighting);
  std::vector<std::array<uint8_t, 32>> prev(1), cur;
  for (int i = 0; i < 32; ++i) prev[0][i] = (uint8_t)rng.uniform(0, 255);
  int written = 0, prev_start = 0;  // id of the first node of the previous level (root: 0)
  std::string buf;
  for (int lev = 1; lev <= L; ++lev) {
    cur.clear();
    const bool leaf = lev == L;
    for (size_t p = 0; p < prev.size(); ++p) {
      for (int c = 0; c < k; ++c) {
        std::array<uint8_t, 32> d;
        if (c > 0 && rng.uniform(0, 15) == 0) {
          d = cur.back();
        } else {
          for (int i = 0; i < 32; ++i) {
            uint8_t flip = 0;
            for (int b = 0; b < 8; ++b) flip |= (uint8_t)((rng.uniform(0, 3) == 0) << b);
            d[i] = prev[p][i] ^ flip;
          }
        }
        cur.push_back(d);
        const int parent = prev_start + (int)p;
        double w = 0.0;
        if (leaf) w = rng.uniform(0, 99) < stop_pct ? 0.0 : 0.2 + 7.8 * rng.unit();
        char line[512];
        int o = std::snprintf(line, sizeof line, "%d %d ", parent, leaf ? 1 : 0);
        for (int i = 0; i < 32; ++i) o += std::snprintf(line + o, sizeof line - o, "%d ", d[i]);
        std::snprintf(line + o, sizeof line - o, " %g", w);
        if (written > 0) std::fputc('\n', f);
        std::fputs(line, f);
        ++written;
      }
    }
    prev_start = written - (int)cur.size() + 1;  // ids are 1 + line index
    prev.swap(cur);
  }
  if (trailing_newline) std::fputc('\n', f);
  std::fclose(f);
  return written;
}

}  // extern "C"
