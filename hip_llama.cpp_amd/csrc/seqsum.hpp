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

// Lane l + 1's value (lane 63: 0), by DPP wave_shl:1 (no LDS round trip, unlike __shfl_down).
TL_DEVICE float wave_next_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x130, 0xF, 0xF, false));
}

TL_DEVICE double lane_d(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// s = fl(s + x) over the n4 float4s at p (LDS), in order, reading NB float4 per batch (the
// compiler waits for all of a batch's LDS reads at the first use: one LDS latency per 4 NB
// elements).
template <int NB = 8>
TL_DEVICE float chain_f4(const f4* p, int n4, float s) {
  for (int j0 = 0; j0 < n4; j0 += NB) {
    f4 v[NB];
#pragma unroll
    for (int k = 0; k < NB; ++k) v[k] = j0 + k < n4 ? p[j0 + k] : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < NB; ++k)
      if (j0 + k < n4) {
        s = __fadd_rn(s, v[k].x);
        s = __fadd_rn(s, v[k].y);
        s = __fadd_rn(s, v[k].z);
        s = __fadd_rn(s, v[k].w);
      }
  }
  return s;
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
// The same with the division by ch as a multiply-high (m = seqsum_magic(ch); exact for e < 2^20).
TL_DEVICE unsigned seqsum_magic(int ch) { return 0xFFFFFFFFu / (unsigned)ch + 1u; }
TL_DEVICE int seqsum_index_m(int e, int ch, unsigned m) {
  const int q = (int)__umulhi((unsigned)e, m);
  return e + 4 * q;  // q (ch + 4) + (e - q ch)
}
TL_DEVICE int seqsum_floats(int n) { return 64 * (seqsum_ch(n) + 4); }

// The left-to-right fp32 sum of the n values laid out by seqsum_index in `a` (LDS).  One full
// wave; every lane returns the sum.  The caller orders the layout's writes before the call.
TL_DEVICE float wave_seqsum(const float* a, int n, int lane) {
  const int ch = seqsum_ch(n), ch4 = ch >> 2;
  const float* my = a + lane * (ch + 4);
  // guesses from a double prefix of the chunk sums
  float e = chunk_chain(my, ch4, 0.f);
  double inc = (double)e;
  // the scan runs with every lane active (inside the select's lane-0 branch it read lane 0 as
  // zero: every guess missed chunk 0, and a round was spent per lane the scan fed from lane 0)
  const double guess = wave_incl_scan_d(inc) - inc;
  float start = lane == 0 ? 0.f : (float)guess;
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
    float next = wave_next_f(start);
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

// The same sum with each lane's chunk held in registers (ch <= 64, i.e. n <= 4096): the rounds'
// re-chains are register-only (an LDS read per element put ~100 cycles of latency on every
// step of every round).  Identical result.
TL_DEVICE float reg_chain(const f4 (&r)[16], int ch4, float s) {
#pragma unroll
  for (int k = 0; k < 16; ++k)
    if (k < ch4) {
      s = __fadd_rn(s, r[k].x);
      s = __fadd_rn(s, r[k].y);
      s = __fadd_rn(s, r[k].z);
      s = __fadd_rn(s, r[k].w);
    }
  return s;
}

// nrounds: the repair rounds taken (a register); fails (FAILS, diagnostics): the failing lane per round
template <bool FAILS>
TL_DEVICE float seqsum_reg_core(const float* a, int n, int lane, int& nrounds, int* fails) {
  const int ch = seqsum_ch(n), ch4 = ch >> 2;
  const f4* my = reinterpret_cast<const f4*>(a + lane * (ch + 4));
  f4 r[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) r[k] = k < ch4 ? my[k] : f4{0.f, 0.f, 0.f, 0.f};
  float e = reg_chain(r, ch4, 0.f);
  double inc = (double)e;
  // the scan runs with every lane active (inside the select's lane-0 branch it read lane 0 as
  // zero: every guess missed chunk 0, and a round was spent per lane the scan fed from lane 0)
  const double guess = wave_incl_scan_d(inc) - inc;
  float start = lane == 0 ? 0.f : (float)guess;
  e = reg_chain(r, ch4, start);
  inc = (double)e - (double)start;
  // one prefix of the guessed increments serves every round: a round re-bases the lanes above
  // the last proven one on its value (P[L] - P[lo] = the increments in between); a lane whose
  // increment depends on its start (a binade crossing, a tie) fails in its round and is fixed
  const double incl = wave_incl_scan_d(inc);
  const double pre = incl - inc;  // exclusive
  const float total0 = (float)lane_d(incl, 63);
  int lo = 0;
  float slo = 0.f;     // proven start of lane lo
  double plo = 0.0;    // pre[lo]
  for (int round = 0; round < 64; ++round) {
    if (lane > lo) start = (float)((double)slo + (pre - plo));
    const float total = round == 0 ? total0 : (float)((double)slo + (lane_d(incl, 63) - plo));
    e = reg_chain(r, ch4, start);
    float next = wave_next_f(start);
    if (lane == 63) next = total;
    const unsigned long long bad = __ballot(lane >= lo && __float_as_uint(e) != __float_as_uint(next) &&
                                            !(e != e && next != next));
    if (!bad) {
      nrounds = round + 1;
      return total;
    }
    const int c = (int)__builtin_ctzll(bad);
    const float ec = lane_f(e, c);
    if (FAILS && round < 15) fails[round] = c;  // (diagnostics: the failing lane per round)
    if (c == 63) {
      nrounds = round + 1;
      return ec;
    }
    lo = c + 1;
    slo = ec;
    plo = lane_d(pre, lo);
    if (lane == lo) start = ec;
  }
  nrounds = 64;
  return lane_f(e, 63);
}

// rounds_out (optional): [0] the repair rounds, [1..15] the failing lane per round (diagnostics).
// Callers that only want the count use seqsum_reg_core<false> (no array in the caller's frame).
TL_DEVICE float wave_seqsum_reg(const float* a, int n, int lane, int* rounds_out = nullptr) {
  int nr = 0;
  if (!rounds_out) return seqsum_reg_core<false>(a, n, lane, nr, nullptr);
  const float v = seqsum_reg_core<true>(a, n, lane, nr, rounds_out + 1);
  rounds_out[0] = nr;
  return v;
}

// Short sums (n <= 512): the chain itself, run by every lane over the values read back from the
// seqsum layout (broadcast LDS reads, a float4 at a time).  The layout's padding must be zero
// (s + 0 = s for the chain's s >= +0, so whole float4s are added).  Reads in batches of 12
// float4 (the compiler waits for all of a batch's LDS reads at the first use).
TL_DEVICE float wave_seqsum_short(const float* a, int n) {
  const int ch4 = seqsum_ch(n) >> 2, n4 = (n + 3) >> 2;  // ch4 = 1 or 2
  const f4* a4 = reinterpret_cast<const f4*>(a);
  float s = 0.f;
  for (int j0 = 0; j0 < n4; j0 += 12) {
    f4 v[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) {  // float4 j of the sequence: rows of ch4 + 1 float4s
      const int j = j0 + k;
      v[k] = j < n4 ? a4[ch4 == 1 ? 2 * j : j + (j >> 1)] : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int k = 0; k < 12; ++k) {
      s = __fadd_rn(s, v[k].x);
      s = __fadd_rn(s, v[k].y);
      s = __fadd_rn(s, v[k].z);
      s = __fadd_rn(s, v[k].w);
    }
  }
  return s;
}

}  // namespace tl
