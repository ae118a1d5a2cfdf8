// seqsum.hpp — the reference's left-to-right fp32 sums, reproduced bit for bit by one wave.
//
// The reference sums with a single sequential chain s = fl(s + a[k]), k = 0..n-1: the RMSNorm sum
// of squares (src/seq.cpp:5-8, runq.c:284-287) and the softmax denominator (src/seq.cpp:27-31,
// runq.c:306-310).  The int8 path re-quantises the activations after every norm, so the chain's
// exact rounding matters (tools/probes/q8drift.c: a tree-ordered norm sum alone makes runq's
// greedy decode diverge).  A literal chain is n dependent adds (4096 x 4 cycles ~ 8 us per norm);
// this is the same chain in ~n/64 dependent steps per round:
//
//  * lane L owns the consecutive elements [L ch, (L+1) ch) (a lane-chunked LDS layout, below);
//  * guesses: lane L chains its chunk from 0; a double prefix over the lanes of those chunk sums
//    gives a start G_L close to the true running value S_L; chaining from G_L gives the
//    increment D_L = f_L(G_L) - G_L;
//  * round: starts S_L = S_lo + sum_{lo <= j < L} D_j (exact in double), every lane re-chains its
//    chunk from S_L and checks that it lands on S_{L+1}.  Lanes below lo are proven; if all
//    check, S_64 is the chain's value (by induction: lane 0 starts at the exact 0).  Otherwise
//    the first failing lane c is proven to end at its re-chained value (its start was proven),
//    which becomes S_{c+1}; every lane refreshes D_L from its re-chain; repeat from lo = c + 1.
//  * a chunk's increment is start-independent while its partial sums stay in one binade and no
//    element rounds to a tie, so the rounds are few (mean 5.3 on 4096 Gaussian squares, one per
//    binade crossing; tools/probes/seqsum.c emulates the algorithm: 0 mismatches on 12000 typical
//    and adversarial arrays); every round advances lo, so at most 64 rounds, for any data.
#pragma once
#include "common.hpp"

namespace tl {

// DPP move of a double (both 32-bit halves); rows outside ROWS and out-of-row sources give 0.
template <int CTRL, int ROWS>
TL_DEVICE double dpp_d(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, ROWS, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, ROWS, 0xF, true);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// Inclusive prefix sum over the 64 lanes (row_shr 1/2/4/8, then row_bcast15 / row_bcast31).
// All 64 lanes active.
TL_DEVICE double wave_incl_scan_d(double x) {
  x += dpp_d<0x111, 0xF>(x);
  x += dpp_d<0x112, 0xF>(x);
  x += dpp_d<0x114, 0xF>(x);
  x += dpp_d<0x118, 0xF>(x);
  x += dpp_d<0x142, 0xA>(x);
  x += dpp_d<0x143, 0xC>(x);
  return x;
}

TL_DEVICE double lane_d(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// s = fl(s + x) over the ch4 float4s of one chunk, in order.
TL_DEVICE float chunk_chain(const float* my, int ch4, float s) {
  const f4* p = reinterpret_cast<const f4*>(my);
  for (int k = 0; k < ch4; ++k) {
    const f4 v = p[k];
    s = __fadd_rn(s, v.x);
    s = __fadd_rn(s, v.y);
    s = __fadd_rn(s, v.z);
    s = __fadd_rn(s, v.w);
  }
  return s;
}

// Layout of n values for wave_seqsum: chunk length ch = 4 * ceil(n / 256) (a multiple of 4),
// element e at e / ch * stride + e % ch with stride = ch + 4 (16-B aligned rows; b128 reads by
// 64 lanes spread over the banks), zeros from n up to 64 ch.
TL_DEVICE int seqsum_ch(int n) { return 4 * ((n + 255) >> 8); }
TL_DEVICE int seqsum_index(int e, int ch) { return e / ch * (ch + 4) + e % ch; }
TL_DEVICE int seqsum_floats(int n) { return 64 * (seqsum_ch(n) + 4); }

// The left-to-right fp32 sum of the n values laid out by seqsum_index in `a` (LDS).  One full
// wave; every lane returns the sum.  The caller orders the layout's writes before the call.
TL_DEVICE float wave_seqsum(const float* a, int n, int lane) {
  const int ch = seqsum_ch(n), ch4 = ch >> 2;
  const float* my = a + lane * (ch + 4);
  // guesses from a double prefix of the chunk sums
  float e = chunk_chain(my, ch4, 0.f);
  double inc = (double)e;
  float start = lane == 0 ? 0.f : (float)(wave_incl_scan_d(inc) - inc);
  e = chunk_chain(my, ch4, start);
  inc = (double)e - (double)start;
  int lo = 0;
  for (int round = 0; round < 64; ++round) {
    const double base = (double)lane_f(start, lo);
    const double incm = lane >= lo ? inc : 0.0;
    const double incl = wave_incl_scan_d(incm);
    if (lane > lo) start = (float)(base + (incl - incm));
    const float total = (float)(base + lane_d(incl, 63));
    e = chunk_chain(my, ch4, start);
    float next = __shfl_down(start, 1, 64);
    if (lane == 63) next = total;
    const unsigned long long bad = __ballot(lane >= lo && __float_as_uint(e) != __float_as_uint(next) &&
                                            !(e != e && next != next));
    if (!bad) return total;
    const int c = (int)__builtin_ctzll(bad);
    const float ec = lane_f(e, c);
    if (c == 63) return ec;
    inc = (double)e - (double)start;
    if (lane == c + 1) start = ec;
    lo = c + 1;
  }
  return lane_f(e, 63);  // not reached: every round proves at least one more lane
}

}  // namespace tl
