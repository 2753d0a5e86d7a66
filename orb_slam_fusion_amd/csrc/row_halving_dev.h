// Per-16-lane-row totals of up to 64 fp64 accumulators a lane, by recursive
// halving: four exchange steps -- partner lane ^ 8 (DPP row_ror:8), 7 - i
// within each 8 (row_half_mirror), ^ 2 and ^ 1 (quad_perm) -- in each of
// which a lane keeps the half of its values its bit selects and adds the
// partner's copy of that half.  Lane i of a row then holds the row's totals
// of accumulators R i .. R i + R - 1 (R = 2 for up to 32, 4 for up to 64)
// and stores those: 16 + 8 + 4 + 2 exchanges for 32 (x 2 for 64) and R
// stores a lane, against 4 x NV row_shr steps and NV stores by one lane of
// the chain it replaces (the order of the additions differs: the
// callers' sums are fp64 with parity by tolerance).
#pragma once
#include <hip/hip_runtime.h>

namespace orbgpu {

template <int CTRL>
__device__ __forceinline__ double dpp_xchg_f64(double v) {
  // every lane's source lies in its own row (a permutation): no bound_ctrl
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}

template <int M, int CTRL>
__device__ __forceinline__ void halve_step(double (&out)[M], const double (&in)[2 * M], bool up) {
#pragma unroll
  for (int j = 0; j < M; ++j) {
    const double lo = in[j], hi = in[j + M];
    out[j] = (up ? hi : lo) + dpp_xchg_f64<CTRL>(up ? lo : hi);
  }
}

// row_dst: this lane's row's NV totals (row = lane >> 4 of the wave).  NV is
// padded to 32 (each lane stores 2 totals) or 64 (4 totals).
template <int NV>
__device__ __forceinline__ void row_totals_halving(const double (&v)[NV], int lane, double* row_dst) {
  static_assert(NV <= 64, "at most 64 accumulators");
  constexpr int P = NV <= 32 ? 32 : 64, R = P / 16;
  const int li = lane & 15;
  double a[P], h1[P / 2], h2[P / 4], h3[P / 8], h4[R];
#pragma unroll
  for (int k = 0; k < P; ++k) a[k] = k < NV ? v[k] : 0.0;
  halve_step<P / 2, 0x128>(h1, a, (li >> 3) & 1);   // row_ror:8
  halve_step<P / 4, 0x141>(h2, h1, (li >> 2) & 1);  // row_half_mirror
  halve_step<P / 8, 0x4E>(h3, h2, (li >> 1) & 1);   // quad_perm [2,3,0,1]
  halve_step<R, 0xB1>(h4, h3, li & 1);              // quad_perm [1,0,3,2]
#pragma unroll
  for (int r = 0; r < R; ++r)
    if (R * li + r < NV) row_dst[R * li + r] = h4[r];
}

}  // namespace orbgpu
