// ORACLE (test infrastructure only).  See cv_semantics.h for scope and pinning.
#include "cv_semantics.h"

#include <algorithm>
#include <cassert>
#include <cfloat>
#include <cstring>

namespace oracle {

namespace {
constexpr int kCoefBits = 11;                // INTER_RESIZE_COEF_BITS
constexpr int kCoefScale = 1 << kCoefBits;   // INTER_RESIZE_COEF_SCALE = 2048

inline short sat_short(float v) {
  int r = cv_round(v);
  return (short)std::min(std::max(r, -32768), 32767);
}
inline uint8_t sat_u8(int v) { return (uint8_t)std::min(std::max(v, 0), 255); }
inline int16_t sat_s16(int v) { return (int16_t)std::min(std::max(v, -32768), 32767); }
}  // namespace

int g_resize_rounding = kResizeSse;

void resize_linear_u8(const uint8_t* src, int sw, int sh, int sstride, uint8_t* dst,
                      int dw, int dh, int dstride) {
  // Scale factors exactly as cv::resize derives them from the sizes.
  const double inv_sx = (double)dw / sw, inv_sy = (double)dh / sh;
  const double scale_x = 1. / inv_sx, scale_y = 1. / inv_sy;

  std::vector<int> xofs(dw);
  std::vector<short> ialpha(2 * dw);
  int xmax = dw;
  for (int dx = 0; dx < dw; ++dx) {
    float fx = (float)((dx + 0.5) * scale_x - 0.5);
    int sx = cv_floor(fx);
    fx -= sx;
    if (sx < 0) fx = 0.f, sx = 0;
    if (sx + 1 >= sw) {
      xmax = std::min(xmax, dx);
      if (sx >= sw - 1) fx = 0.f, sx = sw - 1;
    }
    xofs[dx] = sx;
    ialpha[2 * dx] = sat_short((1.f - fx) * kCoefScale);
    ialpha[2 * dx + 1] = sat_short(fx * kCoefScale);
  }

  std::vector<int> row0(dw), row1(dw);
  auto hresize = [&](const uint8_t* S, int* D) {
    for (int dx = 0; dx < xmax; ++dx) {
      int sx = xofs[dx];
      D[dx] = S[sx] * ialpha[2 * dx] + S[sx + 1] * ialpha[2 * dx + 1];
    }
    for (int dx = xmax; dx < dw; ++dx) D[dx] = S[xofs[dx]] * kCoefScale;
  };

  for (int dy = 0; dy < dh; ++dy) {
    float fy = (float)((dy + 0.5) * scale_y - 0.5);
    int sy = cv_floor(fy);
    fy -= sy;
    const short b0 = sat_short((1.f - fy) * kCoefScale);
    const short b1 = sat_short(fy * kCoefScale);
    const int r0 = std::min(std::max(sy, 0), sh - 1);
    const int r1 = std::min(std::max(sy + 1, 0), sh - 1);
    hresize(src + (size_t)r0 * sstride, row0.data());
    hresize(src + (size_t)r1 * sstride, row1.data());

    uint8_t* D = dst + (size_t)dy * dstride;
    // VResizeLinearVec_32s8u: 16-lane blocks while x <= w-16, then 8-lane
    // blocks while x < w-8; both use the >>4 / mulhi / (+2)>>2 rounding.
    auto vec_px = [&](int x) {
      int16_t h0 = sat_s16(row0[x] >> 4), h1 = sat_s16(row1[x] >> 4);
      int16_t m0 = (int16_t)((h0 * b0) >> 16), m1 = (int16_t)((h1 * b1) >> 16);
      int16_t s = sat_s16(m0 + m1);
      return sat_u8((s + 2) >> 2);
    };
    int x = 0;
    if (g_resize_rounding == kResizeSse) {
      for (; x <= dw - 16; x += 16)
        for (int k = 0; k < 16; ++k) D[x + k] = vec_px(x + k);
      for (; x < dw - 8; x += 8)
        for (int k = 0; k < 8; ++k) D[x + k] = vec_px(x + k);
    }
    // Scalar tail: FixedPtCast<int, uchar, 22>.
    for (; x < dw; ++x) D[x] = sat_u8((row0[x] * b0 + row1[x] * b1 + (1 << 21)) >> 22);
  }
}

namespace {
// Bresenham circle of radius 3, (dx, dy) per index; indices 16..24 repeat 0..8.
const int kCircle16[16][2] = {{0, 3},  {1, 3},   {2, 2},   {3, 1},  {3, 0},  {3, -1},
                              {2, -2}, {1, -3},  {0, -3},  {-1, -3}, {-2, -2}, {-3, -1},
                              {-3, 0}, {-3, 1},  {-2, 2},  {-1, 3}};
}

int fast_corner_score(const uint8_t* p, const int pixel[25], int threshold) {
  const int v = p[0];
  int d[25];
  for (int k = 0; k < 25; ++k) d[k] = v - p[pixel[k]];
  int a0 = threshold;
  for (int k = 0; k < 16; k += 2) {
    int a = std::min(std::min(d[k + 1], d[k + 2]), d[k + 3]);
    if (a <= a0) continue;
    for (int m = 4; m <= 8; ++m) a = std::min(a, d[k + m]);
    a0 = std::max(a0, std::min(a, d[k]));
    a0 = std::max(a0, std::min(a, d[k + 9]));
  }
  int b0 = -a0;
  for (int k = 0; k < 16; k += 2) {
    int b = d[k + 1];
    for (int m = 2; m <= 5; ++m) b = std::max(b, d[k + m]);
    if (b >= b0) continue;
    for (int m = 6; m <= 8; ++m) b = std::max(b, d[k + m]);
    b0 = std::min(b0, std::max(b, d[k]));
    b0 = std::min(b0, std::max(b, d[k + 9]));
  }
  return -b0 - 1;
}

void fast9_16(const uint8_t* img, int stride, int cols, int rows, int threshold,
              std::vector<FastCorner>& out) {
  out.clear();
  const int K = 8, N = 25;
  int pixel[25];
  for (int k = 0; k < 16; ++k) pixel[k] = kCircle16[k][0] + kCircle16[k][1] * stride;
  for (int k = 16; k < 25; ++k) pixel[k] = pixel[k - 16];
  threshold = std::min(std::max(threshold, 0), 255);

  uint8_t tab[512];
  for (int i = -255; i <= 255; ++i)
    tab[i + 255] = (uint8_t)(i < -threshold ? 1 : i > threshold ? 2 : 0);

  if (cols <= 0 || rows <= 0) return;
  // Three score rows and three corner-position lists, used as a ring.
  std::vector<uint8_t> sbuf(3 * (size_t)cols, 0);
  std::vector<int> pbuf(3 * ((size_t)cols + 1), 0);
  auto score_row = [&](int r) { return sbuf.data() + (size_t)(((r % 3) + 3) % 3) * cols; };
  auto pos_row = [&](int r) { return pbuf.data() + (size_t)(((r % 3) + 3) % 3) * (cols + 1); };

  for (int i = 3; i < rows - 2; ++i) {
    uint8_t* curr = score_row(i - 3);
    int* cpos = pos_row(i - 3) + 1;
    std::memset(curr, 0, cols);
    int nc = 0;
    if (i < rows - 3) {
      const uint8_t* ptr = img + (size_t)i * stride;
      for (int j = 3; j < cols - 3; ++j) {
        const uint8_t* p = ptr + j;
        const int v = p[0];
        const uint8_t* t = tab - v + 255;
        int d = t[p[pixel[0]]] | t[p[pixel[8]]];
        if (d == 0) continue;
        d &= t[p[pixel[2]]] | t[p[pixel[10]]];
        d &= t[p[pixel[4]]] | t[p[pixel[12]]];
        d &= t[p[pixel[6]]] | t[p[pixel[14]]];
        if (d == 0) continue;
        d &= t[p[pixel[1]]] | t[p[pixel[9]]];
        d &= t[p[pixel[3]]] | t[p[pixel[11]]];
        d &= t[p[pixel[5]]] | t[p[pixel[13]]];
        d &= t[p[pixel[7]]] | t[p[pixel[15]]];
        for (int polarity = 1; polarity <= 2; ++polarity) {
          if (!(d & polarity)) continue;
          const int vt = polarity == 1 ? v - threshold : v + threshold;
          int run = 0;
          for (int k = 0; k < N; ++k) {
            const int x = p[pixel[k]];
            const bool hit = polarity == 1 ? x < vt : x > vt;
            if (!hit) {
              run = 0;
              continue;
            }
            if (++run > K) {
              cpos[nc++] = j;
              curr[j] = (uint8_t)fast_corner_score(p, pixel, threshold);
              break;
            }
          }
        }
      }
    }
    cpos[-1] = nc;
    if (i == 3) continue;

    const uint8_t* prev = score_row(i - 4);
    const uint8_t* pprev = score_row(i - 5);
    const int* ppos = pos_row(i - 4) + 1;
    const int np = ppos[-1];
    for (int k = 0; k < np; ++k) {
      const int j = ppos[k];
      const int s = prev[j];
      if (s > prev[j + 1] && s > prev[j - 1] && s > pprev[j - 1] && s > pprev[j] &&
          s > pprev[j + 1] && s > curr[j - 1] && s > curr[j] && s > curr[j + 1])
        out.push_back({j, i - 1, s});
    }
  }
}

void gaussian7_sigma2_kernel_q8(int k[7]) {
  // getGaussianKernelBitExact(n=7, sigma=2): exp(-x^2 / (2 sigma^2)), center 1,
  // normalised by the sum; then getGaussianKernelFixedPoint_ED(.., 8 bits):
  // error-diffused rounding of the outer taps, center = 256 - 2 * sum(outer).
  const double sigma = 2.0, mul = 2.0 * sigma * sigma;
  double v[7], sum = 0;
  for (int i = 0; i < 3; ++i) {
    double x = i - 3;
    v[i] = v[6 - i] = std::exp(-(x * x) / mul);
    sum += v[i];
  }
  sum = 2 * sum + 1.0;
  v[3] = 1.0;
  double err = 0;
  int outer = 0;
  for (int i = 0; i < 3; ++i) {
    double adj = v[i] / sum * 256.0 + err;
    int q = cv_round(adj);
    err = adj - q;
    k[i] = k[6 - i] = q;
    outer += q;
  }
  k[3] = 256 - 2 * outer;
}

void gaussian7_sigma2_u8(const uint8_t* src, int w, int h, int stride, uint8_t* dst,
                         int dstride) {
  int k[7];
  gaussian7_sigma2_kernel_q8(k);
  auto reflect101 = [](int i, int n) {
    if (n == 1) return 0;
    while (i < 0 || i >= n) i = i < 0 ? -i : 2 * n - 2 - i;
    return i;
  };
  // Horizontal pass in Q8 (exact: <= 255*256), vertical in Q16, round once.
  std::vector<uint32_t> hrow((size_t)w * h);
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      uint32_t s = 0;
      for (int j = 0; j < 7; ++j) s += k[j] * src[(size_t)y * stride + reflect101(x + j - 3, w)];
      hrow[(size_t)y * w + x] = s;
    }
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      uint32_t s = 0;
      for (int i = 0; i < 7; ++i) s += k[i] * hrow[(size_t)reflect101(y + i - 3, h) * w + x];
      dst[(size_t)y * dstride + x] = (uint8_t)std::min<uint32_t>((s + (1u << 15)) >> 16, 255u);
    }
}

float fast_atan2(float y, float x) {
  static const float k180_pi = (float)(180 / 3.14159265358979323846);
  static const float p1 = 0.9997878412794807f * k180_pi;
  static const float p3 = -0.3258083974640975f * k180_pi;
  static const float p5 = 0.1555786518463281f * k180_pi;
  static const float p7 = -0.04432655554792128f * k180_pi;
  const float eps = (float)DBL_EPSILON;
  float ax = std::fabs(x), ay = std::fabs(y), a, c, c2;
  if (ax >= ay) {
    c = ay / (ax + eps);
    c2 = c * c;
    a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  } else {
    c = ax / (ay + eps);
    c2 = c * c;
    a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  }
  if (x < 0) a = 180.f - a;
  if (y < 0) a = 360.f - a;
  return a;
}

}  // namespace oracle
