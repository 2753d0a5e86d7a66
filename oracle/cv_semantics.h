// ORACLE (test infrastructure only; never linked into the product).
//
// Restatement of the OpenCV primitives the reference extractor calls, pinned to
// OpenCV 4.5.4 as built by Ubuntu 22.04 (no IPP, x86-64 SSE baseline).  OpenCV is
// NOT present in this container, so these rules cannot be checked against the
// real library here: at the OpenCV boundary parity is UNPINNED (SURVEY.md §8c,
// Appendix A; DESIGN.md "Oracle").  Every rule carries an
// `OPENCV-4.5.4 SEMANTICS` tag so it can be revisited against a real OpenCV.
//
// Call sites in the reference (/root/reference):
//   cv::resize INTER_LINEAR          orb_extractor.cc:1106
//   cv::FAST(img, kps, th, true)     orb_extractor.cc:783-784, 800-801
//   cv::GaussianBlur 7x7 sigma 2     orb_extractor.cc:1054-1055
//   cv::fastAtan2                    orb_extractor.cc:99
//   cvRound / cvFloor / cvCeil       orb_extractor.cc:79,108,440,457,1096
#pragma once
#include <cmath>
#include <cstdint>
#include <vector>

namespace oracle {

// cvRound(float) -> cvtss2si, round-half-to-even in the default MXCSR mode.
static inline int cv_round(float v) { return (int)std::lrintf(v); }
static inline int cv_round(double v) { return (int)std::lrint(v); }
static inline int cv_floor(float v) { return (int)std::floor(v); }
static inline int cv_floor(double v) { return (int)std::floor(v); }
static inline int cv_ceil(double v) { return (int)std::ceil(v); }

struct FastCorner {
  int x, y;   // ROI-relative (col, row)
  int score;  // cornerScore<16>, stored as uchar by OpenCV
};

// OPENCV-4.5.4 SEMANTICS: resize(src, dst, dsize, 0, 0, INTER_LINEAR), 8UC1,
// non-integer downscale (hal::resize -> resizeGeneric_ with HResizeLinear and
// VResizeLinear + VResizeLinearVec_32s8u at 128-bit universal intrinsics).
// The vertical pass's rounding is the least certain rule: which
// columns take the SIMD body's rounding depends on how OpenCV was built.
// g_resize_rounding selects it: kResizeSse (default: 16-lane blocks while
// x <= w-16, 8-lane blocks while x < w-8, the scalar FixedPtCast tail after)
// or kResizeScalar (a build without the vectorised VResizeLinear: every
// column FixedPtCast<int, uchar, 22>).  Test infrastructure: set it only
// between extractions.
enum { kResizeSse = 0, kResizeScalar = 1 };
extern int g_resize_rounding;
void resize_linear_u8(const uint8_t* src, int sw, int sh, int sstride, uint8_t* dst,
                      int dw, int dh, int dstride);

// OPENCV-4.5.4 SEMANTICS: FAST_t<16>(roi, kps, threshold, nonmax=true) on a
// ROI of `cols` x `rows` pixels; corners appended in raster order.
void fast9_16(const uint8_t* roi, int stride, int cols, int rows, int threshold,
              std::vector<FastCorner>& out);

// OPENCV-4.5.4 SEMANTICS: cornerScore<16>.
int fast_corner_score(const uint8_t* p, const int pixel[25], int threshold);

// OPENCV-4.5.4 SEMANTICS: GaussianBlur(src, dst, Size(7,7), 2, 2,
// BORDER_REFLECT_101) on a non-submatrix 8U image: bit-exact fixed-point path,
// Q8 kernel from getGaussianKernelBitExact + error-diffusion quantisation.
void gaussian7_sigma2_u8(const uint8_t* src, int w, int h, int stride, uint8_t* dst,
                         int dstride);
// The Q8 kernel the path above uses (exposed for tests): sums to 256.
void gaussian7_sigma2_kernel_q8(int k[7]);

// OPENCV-4.5.4 SEMANTICS: fastAtan2 (degrees, [0, 360)), scalar, no FMA.
float fast_atan2(float y, float x);

}  // namespace oracle
