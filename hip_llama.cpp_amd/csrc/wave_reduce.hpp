// wave_reduce.hpp — many independent sums over the 64 lanes of a wave at once (gfx950).
#pragma once
#include "common.hpp"

namespace tl {

// Transposed wave reduction: v[0..NV) per lane (NV = 8, 16, 32) summed over the 64 lanes.  Each
// step pairs every lane with one partner, keeps half of the values and adds the partner's copy of
// them (v_permlane32/16_swap for the lane^32 / lane^16 pairs, DPP row_mirror / row_half_mirror /
// quad_perm for lane^15 / ^7 / ^3), so 32 sums cost ~70 VALU ops instead of 32 x 11.  Lane l ends
// with the total of value (l >> 1) & (NV - 1) (lanes l and l ^ 1 hold the same; for NV < 32 only
// lanes < 2 NV hold the totals of their index).  A fixed sequence of additions: deterministic.
template <int H, int N>
TL_DEVICE void swap_fold32(float (&v)[N]) {
#pragma unroll
  for (int j = 0; j < H; ++j) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[j]), __float_as_uint(v[j + H]), false, false);
    v[j] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
}
template <int H, int N>
TL_DEVICE void swap_fold16(float (&v)[N]) {
#pragma unroll
  for (int j = 0; j < H; ++j) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[j]), __float_as_uint(v[j + H]), false, false);
    v[j] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
}
template <int CTRL, int H, int N>
TL_DEVICE void dpp_fold(float (&v)[N], bool hi) {
#pragma unroll
  for (int j = 0; j < H; ++j) {
    const float keep = hi ? v[j + H] : v[j];
    const float send = hi ? v[j] : v[j + H];
    v[j] = keep + dpp_f<CTRL>(send);
  }
}
template <int NV>
TL_DEVICE float wave_reduce_t(float (&v)[NV], int lane) {
  static_assert(NV == 8 || NV == 16 || NV == 32, "8, 16 or 32 values");
  if constexpr (NV == 32) swap_fold32<16>(v);            // index bit 4 <- lane bit 5
  if constexpr (NV >= 16) swap_fold16<8>(v);             // bit 3 <- lane bit 4
  dpp_fold<0x140, 4>(v, (lane & 8) != 0);                // row_mirror (lane ^ 15): bit 2 <- lane bit 3
  dpp_fold<0x141, 2>(v, (lane & 4) != 0);                // row_half_mirror (lane ^ 7): bit 1 <- lane bit 2
  dpp_fold<0x1B, 1>(v, (lane & 2) != 0);                 // quad_perm [3,2,1,0] (lane ^ 3): bit 0 <- lane bit 1
  float t = v[0] + dpp_f<0xB1>(v[0]);                    // quad_perm [1,0,3,2] (lane ^ 1)
  if constexpr (NV <= 16) {                              // the lane bits no value index took
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(t), __float_as_uint(t), false, false);
    t = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  if constexpr (NV == 8) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(t), __float_as_uint(t), false, false);
    t = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  return t;
}

}  // namespace tl
