// Deterministic synthetic workloads: stereo frames for the
// extractor and seeded pose-only problems.  Host-only helper library
// (liborbsynth.so) shared by tests/ and bench.py so both sides of every parity
// and timing run see byte-identical inputs.  Not part of the hot path.
#include <cmath>
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

extern "C" {

// Stereo pair from one canvas of width w + disparity: left(x) = canvas(x),
// right(x) = canvas(x + disparity).  Canvas = vertical gradient 40..200, 300
// axis-aligned rectangles (sides U[4,60], grey U[0,255]), 150 discs (radius
// U[3,25]), then per-pixel U[-6,6] noise, clamped.  seed = 0x5EED0000 + frame.
void synth_stereo_frame(uint64_t seed, int w, int h, int disparity, uint8_t* left,
                        uint8_t* right) {
  const int cw = w + disparity;
  std::vector<int> c((size_t)cw * h);
  XorShift64Star rng(seed);
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < cw; ++x) c[(size_t)y * cw + x] = 40 + (160 * y) / (h > 1 ? h - 1 : 1);
  for (int r = 0; r < 300; ++r) {
    const int x0 = rng.uniform(0, cw - 1), y0 = rng.uniform(0, h - 1);
    const int rw = rng.uniform(4, 60), rh = rng.uniform(4, 60), g = rng.uniform(0, 255);
    for (int y = y0; y < y0 + rh && y < h; ++y)
      for (int x = x0; x < x0 + rw && x < cw; ++x) c[(size_t)y * cw + x] = g;
  }
  for (int d = 0; d < 150; ++d) {
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
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      if (left) left[(size_t)y * w + x] = (uint8_t)c[(size_t)y * cw + x];
      if (right) right[(size_t)y * w + x] = (uint8_t)c[(size_t)y * cw + x + disparity];
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
