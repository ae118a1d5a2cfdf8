// persist_b.hip — the whole decode step of 2..8 sequences as ONE persistent launch (fp32).
//
// Semantics: the reference forward (src/seq.cpp:53-168; its GPU twin thaDNN_s_forward_batch,
// src/thaDNN.cpp:13-81, for B sequences at their own positions) followed, in greedy mode, by
// sample_argmax per sequence (src/llama.cpp:275-286).
//
// Why: the multi-launch batched step (gemv_mfma.hpp / gemv_rr.hpp, 5 launches per layer) pays
// ~5-7 us of ramp and tail per launch — about 1 ms of the 5.6 ms llama2-7B step at 8 sequences
// (DESIGN.md section 3).  The batch-1 persistent step (persist.hip) removed that cost by keeping
// one block per CU alive for the whole step and handing phase outputs over as tagged granules;
// this is the same engine for B sequences.
//
// What changes with B sequences:
//  * The activations of every sequence are needed for each weight byte.  The LDS holds a strip of
//    KP floats of every sequence (KP = 4096 at B = 8: 128 KiB; 8192 at 4; 12288 at 2), so a
//    phase whose rows are longer (W2's K = 11008 at B = 4 or 8) runs in K-passes: pass q stages
//    x[b][q*KP .. q*KP + KP) of every sequence, then the streaming waves sweep those chunks of
//    every row the block owns.  A slot is one 8-KiB row chunk (KC = 2048 floats), as in the
//    batch-1 step, and its consume does B dot products with the strip (B ds_read_b128 per weight
//    float4).
//  * RMSNorm needs the whole row's sum of squares before any element is scaled, which a K-pass
//    does not have; the norm is applied as (W (w * x)) * ss_b: the staging multiplies by the norm
//    weight w[k], accumulates sum x^2 per sequence over the passes (fixed order), and the
//    epilogue multiplies each row result by ss_b (src/seq.cpp:3-16 up to rounding: fp32 parity).
//  * Every hand-off buffer, the residual slice each block keeps in LDS, the per-block argmax
//    and the attention units carry a sequence index; attention runs B * H * NS units.
//
// Unchanged from persist.hip: grid = one 576-thread block per CU, all co-resident (cooperative
// launch); wave 0 = control (epilogues, attention units, norm-weight preloads), waves 1-8
// stream with two 8-KiB slots in flight each and issue the next pass's / phase's first slots
// before the hand-off; granules {value, tag} with tags (launch sequence << 12) + phase + 1; every
// wait bounded with a sticky error word; one grid barrier (the final argmax).
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <mutex>
#include "attention.hpp"
#include "gemv.hpp"
#include "persist.hpp"

namespace tl {
namespace pb {

constexpr int PW = 9;           // waves per block: 1 control + 8 streaming
constexpr int PT = PW * 64;
constexpr int NSW = PW - 1;
constexpr int NBUF = 2;         // register slots in flight per streaming wave
constexpr int PL = 8;           // wave-loads per slot (8 KiB)
constexpr int KC = PL * 256;    // floats per row chunk = one K-pass
constexpr int KC4 = KC / 4;     // float4 per chunk
constexpr int SBU = 4;          // staging: (sequence, float4) units in flight per thread
constexpr int kResid = 256;     // residual-stream slice per block and sequence (LDS)
constexpr unsigned kSpinLimit = 1u << 18;
constexpr unsigned kXcdSkew = 4;  // percent; odd blockIdx (XCDs 1,3,5,7) stream slower (persist.hip)

enum PKind : int { PK_QKV = 0, PK_ATTN = 1, PK_WO = 2, PK_UP = 3, PK_DOWN = 4, PK_CLS = 5 };

struct PDesc {
  int kind;
  int K;                          // row length = input length (floats)
  int n_items;                    // rows, or row pairs (QKV, SwiGLU)
  int rpi;                        // rows per item
  int out_stride;                 // granules per sequence in gout
  const float *W0, *W1, *W2;
  const unsigned long long* gin;  // input granules [B][K] (null: the tokens' embedding rows)
  unsigned tag_in;
  const float* rms;               // fused RMSNorm weight or null
  unsigned long long* gout;       // output granules (null for the classifier)
  unsigned tag_out;
};

TL_DEVICE PDesc make_desc(const PStep& p, int kind, int l, unsigned tb) {
  PDesc d = {};
  d.kind = kind;
  const long long ll = l, dim = p.dim, hid = p.hid, kvd = p.kvd;
  const unsigned t0 = tb + 5u * l;  // tag of the phase before QKV(l), i.e. W2(l-1)
  switch (kind) {
    case PK_QKV:
      d.K = p.dim; d.n_items = (p.dim + 2 * p.kvd) / 2; d.rpi = 2; d.out_stride = p.dim + 2 * p.kvd;
      d.W0 = p.wq + ll * dim * dim; d.W1 = p.wk + ll * dim * kvd; d.W2 = p.wv + ll * dim * kvd;
      d.gin = l == 0 ? nullptr : p.gx; d.tag_in = t0;
      d.rms = p.rms_att + ll * dim; d.gout = p.gqkv; d.tag_out = t0 + 1;
      break;
    case PK_WO:
      d.K = p.dim; d.n_items = p.dim; d.rpi = 1; d.out_stride = p.dim;
      d.W0 = p.wo + ll * dim * dim; d.gin = p.gxb; d.tag_in = t0 + 2; d.gout = p.gx; d.tag_out = t0 + 3;
      break;
    case PK_UP:
      d.K = p.dim; d.n_items = p.hid; d.rpi = 2; d.out_stride = p.hid;
      d.W0 = p.w1 + ll * dim * hid; d.W1 = p.w3 + ll * dim * hid;
      d.gin = p.gx; d.tag_in = t0 + 3; d.rms = p.rms_ffn + ll * dim; d.gout = p.ghb; d.tag_out = t0 + 4;
      break;
    case PK_DOWN:
      d.K = p.hid; d.n_items = p.dim; d.rpi = 1; d.out_stride = p.dim;
      d.W0 = p.w2 + ll * dim * hid; d.gin = p.ghb; d.tag_in = t0 + 4; d.gout = p.gx; d.tag_out = t0 + 5;
      break;
    default:  // PK_CLS (l = L)
      d.K = p.dim; d.n_items = p.V; d.rpi = 1; d.out_stride = 0;
      d.W0 = p.wcls; d.gin = p.gx; d.tag_in = tb + 5u * p.L; d.rms = p.rms_final;
      break;
  }
  return d;
}

TL_DEVICE PDesc next_desc(const PStep& p, int kind, int l, unsigned tb) {
  if (kind == PK_QKV) return make_desc(p, PK_WO, l, tb);
  if (kind == PK_WO) return make_desc(p, PK_UP, l, tb);
  if (kind == PK_UP) return make_desc(p, PK_DOWN, l, tb);
  return l + 1 < p.L ? make_desc(p, PK_QKV, l + 1, tb) : make_desc(p, PK_CLS, p.L, tb);
}

// This block's share of a phase (wave-uniform): items [i0, i0 + ni), their rows, the passes.
struct PGeo {
  int i0, ni;
  int nrow;  // ni * rpi
  int nch;   // row chunks (KC floats each)
};

// Pass q of a phase whose rows have nch chunks, cpp chunks per pass: chunks [c0, c0 + npc).
struct PPass {
  int c0, npc;
  int nslot;  // nrow * npc: slot s = chunk c0 + s % npc of row s / npc
};
TL_DEVICE PPass pass_of(const PGeo& g, int cpp, int q) {
  PPass r;
  r.c0 = q * cpp;
  r.npc = g.nch - r.c0 < cpp ? g.nch - r.c0 : cpp;
  r.nslot = g.nrow * r.npc;
  return r;
}

__host__ __device__ inline unsigned part_weight(unsigned b) { return (b >> 1) * 200u + (b & 1u) * (100u + kXcdSkew); }

TL_DEVICE PGeo geo(const PDesc& d) {
  PGeo g;
  const unsigned G = gridDim.x, bi = blockIdx.x, n = (unsigned)d.n_items;
  const unsigned wt = part_weight(G);
  g.i0 = (int)(n * part_weight(bi) / wt);
  g.ni = (int)(n * part_weight(bi + 1) / wt) - g.i0;
  g.nrow = g.ni * d.rpi;
  g.nch = (d.K + KC - 1) / KC;
  return g;
}

TL_DEVICE const float* row_ptr(const PDesc& d, const PStep& p, int R) {
  const long long K = d.K;
  if (d.kind == PK_UP) return ((R & 1) ? d.W1 : d.W0) + (long long)(R >> 1) * K;
  if (d.kind == PK_QKV) {
    if (R < p.dim) return d.W0 + (long long)R * K;
    R -= p.dim;
    if (R < p.kvd) return d.W1 + (long long)R * K;
    return d.W2 + (long long)(R - p.kvd) * K;
  }
  return d.W0 + (long long)R * K;
}

// Chunk c of the block's row rl: 8 wave-loads of 1 KiB (raw buffer loads sized to what is left
// of the row: loads past its end return 0 without touching memory), non-temporal.
TL_DEVICE void load_slot(const PDesc& d, const PGeo& g, const PStep& p, int rl, int c, int lane, f4 (&buf)[PL]) {
  const float* row = row_ptr(d, p, g.i0 * d.rpi + rl);
#pragma unroll
  for (int q = 0; q < PL / 4; ++q) {
    const int off = c * (KC * 4) + q * 4096;  // bytes into the row
    const int left = d.K * 4 - off;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(row) + off / 4, (short)0,
                                                      left > 0 ? left : 0, 0x00020000);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      buf[q * 4 + u] =
          __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16 + u * 1024, 0, 2 /*nt*/));
  }
}

// NB dot products of one row chunk with the staged strip (chunk cc of the pass: xs [NB][KP4] at
// cc * KC4): row partial res[(rl * nch + c) * NB + b].  NB is the exact batch (no run-time guards:
// a branch around each read made the compiler wait for it singly).
template <int NB>
TL_DEVICE void consume_slot(int rl, int c, int cc, int nch, int KP4, int lane, const f4 (&buf)[PL], const f4* xs,
                            float* res) {
  float a[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) a[b] = 0.f;
  // the strip offset is laundered so the compiler cannot prove the reads loop-invariant across
  // the slots of a pass (a pass of one chunk reads the same strip for every slot)
  int xo = cc * KC4 + lane;
  asm volatile("" : "+v"(xo));
  const f4* xc = xs + xo;
  // one sequence at a time: its 8 strip reads in flight, then its 32 FMAs
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    f4 xv[PL];
#pragma unroll
    for (int u = 0; u < PL; ++u) xv[u] = xc[b * KP4 + u * 64];
#pragma unroll
    for (int u = 0; u < PL; ++u) a[b] = dot4(buf[u], xv[u], a[b]);
    __builtin_amdgcn_sched_barrier(0);
  }
  // lane b keeps sequence b's sum and ONE store writes them all (a store per sequence under
  // lane == 0 let the compiler sink each sequence's FMAs into its branch, after every read, and
  // hold 8 float4 per sequence live: spills from 6 sequences on)
  float mine = 0.f;
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const float sm = wave_sum_u(a[b]);
    mine = lane == b ? sm : mine;
  }
  if (lane < NB) res[(rl * nch + c) * NB + lane] = mine;
}

// A wave's slots in pass c: its two prefetched rows (sw, sw + NSW), then rows dealt from the
// block's LDS counter; loads past the block's rows are skipped.
TL_DEVICE int take_slot(unsigned* ctr, int lane) {
  unsigned v = 0;
  if (lane == 0) v = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  return NBUF * NSW + (int)__builtin_amdgcn_readlane(v, 0);
}

template <int NB>
TL_DEVICE void run_pass(const PDesc& d, const PGeo& g, const PPass& q, const PStep& p, int sw, int lane,
                        const f4* xs, float* res, f4 (&buf)[NBUF][PL], unsigned* ctr, unsigned long long* ts) {
  const int KP4 = p.pad_floats >> 2;
  int sl[NBUF];
#pragma unroll
  for (int i = 0; i < NBUF; ++i) sl[i] = sw + i * NSW;
  bool first = true;
  while (sl[0] < q.nslot) {
#pragma unroll
    for (int i = 0; i < NBUF; ++i) {
      if (sl[i] < q.nslot) {
        const int rl = sl[i] / q.npc, cc = sl[i] - rl * q.npc;
        consume_slot<NB>(rl, q.c0 + cc, cc, g.nch, KP4, lane, buf[i], xs, res);
      }
      if (i == 0 && ts && first && lane == 0) *ts = __builtin_amdgcn_s_memrealtime();  // first slot landed
      first = false;
      __builtin_amdgcn_sched_barrier(0);
      sl[i] = take_slot(ctr, lane);
      if (sl[i] < q.nslot) load_slot(d, g, p, sl[i] / q.npc, q.c0 + sl[i] % q.npc, lane, buf[i]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// A pass's first NBUF slots of this wave (its prefetch).
TL_DEVICE void prefetch_pass(const PDesc& d, const PGeo& g, const PPass& q, const PStep& p, int sw, int lane,
                             f4 (&buf)[NBUF][PL]) {
#pragma unroll
  for (int i = 0; i < NBUF; ++i) {
    const int s = sw + i * NSW;
    if (s < q.nslot) load_slot(d, g, p, s / q.npc, q.c0 + s % q.npc, lane, buf[i]);
  }
}

// Stage pass q (floats [q*KP, q*KP + KP) of the row) of every sequence into xs [NB][KP4],
// multiplied by the norm weight when the phase has one (read from global memory: constants, in
// L2); the squares go, per wave and sequence, to red[wave * NB + b].  Input: the previous
// phase's granules (SBU (sequence, float4) units in flight per thread, re-polled until their
// tags match), or — QKV at layer 0 — the tokens' embedding rows.  Unit u = t + k * PT covers
// float4 u % KP4 of sequence u / KP4, so a wave reads 2 KiB of consecutive granules.
template <int NB>
TL_DEVICE void stage_pass(const PDesc& d, const PStep& p, int q, f4* xs, float* red, int wave, int lane,
                          unsigned long long* ts) {
  const int t = threadIdx.x;
  const int KP4 = p.pad_floats >> 2;
  const int n4 = d.K >> 2;
  const int U = NB * KP4;
  float sq[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) sq[b] = 0.f;
  const auto r = rsrc_of(d.gin ? (const void*)d.gin : (const void*)p.emb);
  for (int u0 = t; u0 < U; u0 += SBU * PT) {
    v4u ga[SBU], gb[SBU];
#pragma unroll
    for (int k = 0; k < SBU; ++k) {
      const int u = u0 + k * PT, b = u / KP4, k4 = q * KP4 + (u - b * KP4);
      if (d.gin && u < U && k4 < n4) {
        const unsigned off = (unsigned)(b * n4 + k4) * 32u;
        ga[k] = ld16_sc1(r, off);
        gb[k] = ld16_sc1(r, off + 16u);
      }
    }
#pragma unroll
    for (int k = 0; k < SBU; ++k) {
      const int u = u0 + k * PT, b = u / KP4, j = u - b * KP4, k4 = q * KP4 + j;
      if (u >= U) continue;
      f4 v = f4{0.f, 0.f, 0.f, 0.f};
      if (k4 < n4) {
        if (d.gin)
          v = gran4_ok(ga[k], gb[k], d.tag_in) ? gran4_val(ga[k], gb[k])
                                               : gran_wait4(r, (unsigned)(b * n4 + k4) * 32u, d.tag_in, p.err, p.poll_long != 0);
        else
          v = reinterpret_cast<const f4*>(p.emb + (long long)p.tok[b] * p.dim)[k4];
        if (d.rms) {
          float s2 = 0.f;
          s2 = fmaf(v.x, v.x, s2); s2 = fmaf(v.y, v.y, s2); s2 = fmaf(v.z, v.z, s2); s2 = fmaf(v.w, v.w, s2);
#pragma unroll
          for (int bb = 0; bb < NB; ++bb) sq[bb] += bb == b ? s2 : 0.f;
          const f4 w = reinterpret_cast<const f4*>(d.rms)[k4];
          v = f4{__fmul_rn(w.x, v.x), __fmul_rn(w.y, v.y), __fmul_rn(w.z, v.z), __fmul_rn(w.w, v.w)};
        }
      }
      xs[b * KP4 + j] = v;
    }
    if (ts && lane == 0 && u0 == t) ts[0] = __builtin_amdgcn_s_memrealtime();  // first batch in
  }
  if (ts && lane == 0) ts[1] = __builtin_amdgcn_s_memrealtime();  // swept
  if (d.rms) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const float s2 = wave_sum_u(sq[b]);
      if (lane == 0) red[wave * NB + b] = s2;
    }
  }
}

// Control wave, while the QKV rows stream: the RoPE (cos, sin) of every (item, sequence) pair of
// this block into LDS (a table read inside the epilogue put an L2 round trip per 64 pairs on
// the hand-off's critical path).
template <int NB>
TL_DEVICE void rope_preload(const PGeo& g, const PStep& p, float2* rcs, int lane) {
  for (int j = lane; j < g.ni * NB; j += 64) {
    const int it = j / NB, b = j - it * NB;
    const int row = 2 * (g.i0 + it);
    float2 cs = make_float2(1.f, 0.f);
    if (row < p.dim + p.kvd) {
      const int i = row < p.dim ? row : row - p.dim;
      cs = p.rope[(long long)p.pos[b] * (p.hs >> 1) + ((i % p.hs) >> 1)];
    }
    rcs[j] = cs;
  }
}

// Control wave: row values from the pass partials (chunks in order), the norm scale, the fused
// epilogue, granule stores.  xres: this block's slice of every sequence's residual stream.
template <int NB>
TL_DEVICE void epilogue(const PDesc& d, const PGeo& g, const PStep& p, const float* res, float* xres,
                        const float* ss, int wave, int lane, int l, const uint64_t* etab, const float2* rcs,
                        unsigned long long* cbest) {
  unsigned long long best[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) best[b] = 0;
  // (item, sequence) pairs over the lanes: a block owns 16-130 items, so items alone would
  // leave most lanes idle on this hand-off's critical path
  const int npair = g.ni * NB;
  for (int j = wave * 64 + lane; j < npair; j += PW * 64) {
    const int it = j / NB, b = j - it * NB;
    const int item = g.i0 + it;
    float v[2] = {0.f, 0.f};
    for (int r = 0; r < d.rpi; ++r) {
      const float* rr = res + ((it * d.rpi + r) * g.nch) * NB + b;
      float s = rr[0];
      for (int c = 1; c < g.nch; ++c) s = __fadd_rn(s, rr[c * NB]);
      v[r] = d.rms ? __fmul_rn(s, ss[b]) : s;
    }
    if (d.kind == PK_CLS) {
      p.logits[(long long)b * p.V + item] = v[0];  // read by the host after the launch only
      const unsigned long long k = argmax_pack(v[0], item);
#pragma unroll
      for (int bb = 0; bb < NB; ++bb)
        if (bb == b) best[bb] = k > best[bb] ? k : best[bb];
    } else if (d.kind == PK_WO || d.kind == PK_DOWN) {
      const float xr = __fadd_rn(xres[b * kResid + it], v[0]);  // residual (src/seq.cpp:139-141, 163-166)
      xres[b * kResid + it] = xr;
      st8_sc1(d.gout + (long long)b * d.out_stride + item, gran(d.tag_out, xr));
      if (d.kind == PK_DOWN && l == p.L - 1) p.x[(long long)b * p.dim + item] = xr;  // final residual (state)
    } else if (d.kind == PK_UP) {
      st8_sc1(d.gout + (long long)b * d.out_stride + item, gran(d.tag_out, silu_mul_tab(v[0], v[1], etab)));
    } else {  // PK_QKV: RoPE (src/seq.cpp:86-101), q / k_new / v_new granules, KV-cache row
      const int row = 2 * item;
      const int pb = p.pos[b];
      float a0 = v[0], a1 = v[1];
      if (row < p.dim + p.kvd) {
        const float2 cs = rcs[j];  // (loaded during the sweep: rope_preload)
        const float r0 = __fsub_rn(__fmul_rn(a0, cs.x), __fmul_rn(a1, cs.y));
        const float r1 = __fadd_rn(__fmul_rn(a0, cs.y), __fmul_rn(a1, cs.x));
        a0 = r0; a1 = r1;
      }
      st_gran2(rsrc_of(d.gout + (long long)b * d.out_stride), (unsigned)row * 8u, d.tag_out, a0, a1);
      if (row >= p.dim) {  // the cache row for later steps (this launch reads the granules)
        int rk = row - p.dim;
        float* base = p.kc;
        if (rk >= p.kvd) { rk -= p.kvd; base = p.vc; }
        *reinterpret_cast<float2*>(base + (long long)b * p.L * p.S * p.kvd + ((long long)l * p.S + pb) * p.kvd + rk) =
            make_float2(a0, a1);
      }
    }
  }
  if (d.kind == PK_CLS) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      unsigned long long bv = best[b];
      for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long other = __shfl_xor(bv, o, 64);
        bv = other > bv ? other : bv;
      }
      if (lane == 0) cbest[wave * NB + b] = bv;  // (reduced over the waves before the final barrier)
    }
  }
}

// Sharded-counter grid barrier (the final one only), as persist.hip.
TL_DEVICE void grid_barrier(const PStep& p) {
  __syncthreads();
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const int G = gridDim.x;
    if (lane == 0)
      __hip_atomic_fetch_add(as_g32(p.sync + (blockIdx.x & 7) * 32), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int sh = lane & 7;
    const unsigned need = (unsigned)((G - sh + 7) >> 3);
    const unsigned* word = lane < 8 ? p.sync + sh * 32 : p.err;
    for (unsigned spins = 0;; ++spins) {
      const unsigned v = __hip_atomic_load(as_g32(word), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__all(lane >= 8 || v >= need)) break;
      if (__any(lane == 8 && v != 0)) break;  // a wait already gave up: do not wait again
      if (spins > kSpinLimit) {
        if (lane == 0) __hip_atomic_store(as_g32(p.err), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
}

// Optional timeline (PStep::trace, [grid][phase][kTraceSlots], 100-MHz clock), control wave:
// 0 phase start, 1 first pass staged, 2 last pass swept, 3 epilogue (or attention units) done,
// 8 + q pass q swept (q < 6), 5 / 6 pass 0's first staging batch in / its sweep done; streaming
// wave 1: 4 its first slot of pass 0 consumed, 14 / 15 its first staging batch in / sweep done.
#define TRACE_B(k)                                                                              \
  do {                                                                                          \
    if (p.trace && lane == 0)                                                                   \
      p.trace[((long long)blockIdx.x * nph + ph) * kTraceSlots + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)

// The phase sequence as one wave sees it.  ROLE0 = the control wave.  Both run the same
// workgroup barriers: per GEMV phase and pass, one after the staging and one after the sweep.
template <int HS, int NB, bool ROLE0>
TL_DEVICE void phases(const PStep& p, int wave, int lane, float* res, float* xres, float* red, f4* xs,
                      const uint64_t* etab, float2* rcs, unsigned long long* cbest, unsigned tb) {
  const int G = gridDim.x;
  const int nph = 5 * p.L + 1;
  const int cpp = p.pad_floats / KC;  // row chunks per K-pass
  float* ssum = red + PW * NB;                                   // [NB] this phase's sum of squares
  float* sscale = ssum + NB;                                     // [NB] its norm scales (epilogue)
  unsigned* ctr = reinterpret_cast<unsigned*>(sscale + NB);      // dynamic slot counter
  f4 buf[NBUF][PL];
  const int sw = wave - 1;
  if constexpr (ROLE0) {
    // this block's slice of every sequence's residual stream starts as its embedding row
    const PGeo gx = geo(make_desc(p, PK_WO, 0, tb));
    for (int b = 0; b < NB; ++b) {
      const float* er = p.emb + (long long)p.tok[b] * p.dim + gx.i0;
      for (int it = lane; it < gx.ni; it += 64) xres[b * kResid + it] = er[it];
    }
    if (lane < NB) ssum[lane] = 0.f;
    if (lane == 0) *ctr = 0u;
  } else {
    const PDesc d0 = make_desc(p, PK_QKV, 0, tb);
    const PGeo g0 = geo(d0);
    prefetch_pass(d0, g0, pass_of(g0, cpp, 0), p, sw, lane, buf);
  }
  __syncthreads();  // counters set

  for (int ph = 0; ph < nph; ++ph) {
    const int l = ph / 5;
    const int kind = ph == nph - 1 ? PK_CLS : ph % 5;
    if constexpr (ROLE0) TRACE_B(0);
    if (kind == PK_ATTN) {
      if constexpr (!ROLE0) {  // the slot buffers are empty here: say so, so they are not kept live
#pragma unroll
        for (int i = 0; i < NBUF; ++i)
#pragma unroll
          for (int u = 0; u < PL; ++u) buf[i][u] = f4{0.f, 0.f, 0.f, 0.f};
      }
      {
        // one wave per (sequence, head, key-split) unit, B * H * NS of them over EVERY wave of the
        // grid (the streaming waves issue Wo's first slots after theirs: attention's registers and
        // two slot buffers do not fit a wave together): unit u runs on block u % G, wave (u / G) % PW
        AttnWaveParams aw = {};
        aw.a.q = p.xb; aw.a.kc = p.kc; aw.a.vc = p.vc;  // (q comes from the granules)
        aw.a.kv_b_stride = (long long)p.L * p.S * p.kvd;
        aw.a.kv_l_off = (long long)l * p.S * p.kvd;
        aw.a.pos = p.pos; aw.a.out = p.xb; aw.a.part = p.part;
        aw.a.dim = p.dim; aw.a.kv_dim = p.kvd; aw.a.head_size = HS; aw.a.n_heads = p.H;
        aw.a.kv_mul = p.kv_mul; aw.a.seq_len = p.S; aw.a.nsplit = p.NS; aw.a.min_chunk = 16;
        aw.cnt = p.tickets + (long long)l * NB * p.H; aw.B = NB; aw.NS = p.NS;
        aw.gqkv = p.gqkv; aw.gout = p.gxb;
        aw.etab = etab;
        aw.tag_in = tb + 5u * l + 1; aw.tag_out = tb + 5u * l + 2; aw.err = p.err;
        aw.poll_long = p.poll_long;
        const int units = NB * p.H * p.NS;
        for (int u = blockIdx.x + G * wave; u < units; u += G * PW) attn_unit<HS, 16, true>(aw, u, lane);
        if constexpr (ROLE0) TRACE_B(3);
      }
      if constexpr (!ROLE0) {  // Wo's first slots stream in while its input is gathered
        const PDesc nd = make_desc(p, PK_WO, l, tb);
        const PGeo ng = geo(nd);
        prefetch_pass(nd, ng, pass_of(ng, cpp, 0), p, sw, lane, buf);
      }
      continue;
    }
    const PDesc d = make_desc(p, kind, kind == PK_CLS ? p.L : l, tb);
    const PGeo g = geo(d);
    const int npass = (g.nch + cpp - 1) / cpp;
    for (int q = 0; q < npass; ++q) {
      stage_pass<NB>(d, p, q, xs, red, wave, lane,
                     p.trace && q == 0 && (wave == 0 || wave == 1)
                         ? p.trace + ((long long)blockIdx.x * nph + ph) * kTraceSlots + (wave == 0 ? 5 : 14)
                         : nullptr);
      __syncthreads();  // strip staged (and this pass's squares per wave in red)
      if constexpr (ROLE0) {
        if (q == 0) TRACE_B(1);
        if (d.rms && lane < NB) {
          float s = ssum[lane];
          for (int w = 0; w < PW; ++w) s = __fadd_rn(s, red[w * NB + lane]);
          ssum[lane] = s;
        }
        if (kind == PK_QKV && q == 0) rope_preload<NB>(g, p, rcs, lane);
        if (q == npass - 1 && lane < NB) {
          // reference rmsnorm scale (src/seq.cpp:3-16): 1 / sqrtf(sum / size + 1e-5f), for every
          // wave's epilogue share (after the pass-end barrier)
          sscale[lane] = d.rms ? __fdiv_rn(1.0f, sqrtf(__fadd_rn(__fdiv_rn(ssum[lane], (float)d.K), 1e-5f))) : 1.f;
          ssum[lane] = 0.f;
        }
      } else {
        run_pass<NB>(d, g, pass_of(g, cpp, q), p, sw, lane, xs, res, buf, ctr,
                     p.trace && sw == 0 && q == 0 ? p.trace + ((long long)blockIdx.x * nph + ph) * kTraceSlots + 4
                                                  : nullptr);
      }
      __syncthreads();  // every slot of the pass reduced into res; the strip may be restaged
      if constexpr (ROLE0) {
        if (q < 6) TRACE_B(8 + q);
        if (q == npass - 1) TRACE_B(2);
        if (lane == 0) *ctr = 0u;  // the next pass's slot counter (used after its staging barrier)
      } else {
        // the next pass's (or the next GEMV phase's) first slots: their data streams in while the
        // strip is restaged, the hand-off is waited for and the epilogue runs
        if (q + 1 < npass) {
          prefetch_pass(d, g, pass_of(g, cpp, q + 1), p, sw, lane, buf);
        } else if (kind != PK_CLS && kind != PK_QKV) {  // (after QKV: once the attention units ran)
          const PDesc nd = next_desc(p, kind, l, tb);
          const PGeo ng = geo(nd);
          prefetch_pass(nd, ng, pass_of(ng, cpp, 0), p, sw, lane, buf);
        }
      }
    }
    // every wave takes a share of the (item, sequence) pairs (the control wave alone spent ~0.5 us
    // per 64 pairs on this hand-off's critical path); the streaming waves' next slots are in flight
    epilogue<NB>(d, g, p, res, xres, sscale, wave, lane, l, etab, rcs, cbest);
    if constexpr (ROLE0) TRACE_B(3);
  }
  __syncthreads();  // every wave's classifier winners in cbest
  if constexpr (ROLE0) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      unsigned long long bv = lane < PW ? cbest[lane * NB + b] : 0ull;
      for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long other = __shfl_xor(bv, o, 64);
        bv = other > bv ? other : bv;
      }
      if (lane == 0) st8_sc1(p.bmax + (long long)blockIdx.x * NB + b, bv);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drained before the final arrival
  }
  grid_barrier(p);
  if constexpr (ROLE0) {
    if (blockIdx.x != 0) return;
    if (p.argmax) {
      // per sequence: argmax over the per-block winners + advance (src/llama.cpp:275-286)
      for (int b = 0; b < NB; ++b) {
        unsigned long long best = 0;
        for (int i = lane; i < G; i += 64) {
          const unsigned long long k = ld8_sc1(p.bmax + (long long)i * NB + b);
          best = k > best ? k : best;
        }
        for (int o = 32; o > 0; o >>= 1) {
          const unsigned long long other = __shfl_xor(best, o, 64);
          best = other > best ? other : best;
        }
        if (lane == 0) {
          const int next = best ? (int)(0xFFFFFFFFu - (uint32_t)(best & 0xFFFFFFFFull)) : 0;
          const int pp = p.pos[b];
          if (p.out && pp < p.S) p.out[(long long)b * p.S + pp] = next;
          p.tok[b] = next;
          p.pos[b] = pp + 1;
        }
      }
    }
    if (lane == 0) p.seq[0] = (tb >> 12) + 1;  // every block read the sequence before the final barrier
  }
}

template <int HS, int NB>
__global__ void __launch_bounds__(PT) persistent_step_b_kernel(PStep p) {
  if (p.fault && blockIdx.x == 0) return;  // test hook: a missing block (every wait is bounded)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  f4* xs = reinterpret_cast<f4*>(smem);                          // NB * KP floats: the staged strip
  float* xres = reinterpret_cast<float*>(xs + NB * (p.pad_floats >> 2));  // NB * kResid: residual slices
  float* red = xres + NB * kResid;                              // PW * NB + 2 * NB + 4
  float* res = red + PW * NB + 2 * NB + 4;                  // n_res: row-chunk partials
  uint64_t* etab = reinterpret_cast<uint64_t*>(res + p.n_scr);  // the expf table (32 doubles' bits)
  unsigned long long* cbest = reinterpret_cast<unsigned long long*>(etab + 32);  // [PW][NB] per-wave winners
  float2* rcs = reinterpret_cast<float2*>(cbest + PW * NB);    // [QKV items][NB] RoPE (cos, sin)
  {
    constexpr uint64_t tab[32] = TL_EXPF_TABLE;
    if (threadIdx.x < 32) etab[threadIdx.x] = tab[threadIdx.x];  // (read after the first barrier)
  }
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const unsigned tb = p.seq[0] << 12;  // tag base of this launch
  if (wave == 0) {
    // the control wave's epilogues are every other block's hand-off: first call on the issue slots
    __builtin_amdgcn_s_setprio(2);
    phases<HS, NB, true>(p, wave, lane, res, xres, red, xs, etab, rcs, cbest, tb);
  } else {
    phases<HS, NB, false>(p, wave, lane, res, xres, red, xs, etab, rcs, cbest, tb);
  }
}

static int nb_of(int B) { return B; }  // one instantiation per batch size: no run-time sequence guards

static size_t lds_bytes(const PStep& p) {
  const int NB = nb_of(p.B);
  return (size_t)NB * p.pad_floats * 4 + (size_t)NB * kResid * 4 + (size_t)(PW * NB + 2 * NB + 4) * 4 +
         (size_t)p.n_scr * 4 + 32 * 8 + (size_t)PW * NB * 8 + (size_t)p.n_sqa * 8;
}

template <int HS, int NB>
static const void* kfn() { return (const void*)persistent_step_b_kernel<HS, NB>; }
template <int HS>
static const void* kfn_b(int B) {
  switch (B) {
    case 2: return kfn<HS, 2>();
    case 3: return kfn<HS, 3>();
    case 4: return kfn<HS, 4>();
    case 5: return kfn<HS, 5>();
    case 6: return kfn<HS, 6>();
    case 7: return kfn<HS, 7>();
    default: return kfn<HS, 8>();
  }
}
static const void* kernel_of(const PStep& p) { return p.hs == 128 ? kfn_b<128>(p.B) : kfn_b<64>(p.B); }

}  // namespace pb

bool persistent_prepare_b(PStep& p, int ncu, const char** why) {
  using namespace pb;
  auto fail = [&](const char* m) { if (why) *why = m; return false; };
  if (p.B < 2 || p.B > 8) return fail("batched persistent step: 2..8 sequences");
  if (p.q8) return fail("batched persistent step: fp32 weights only");
  if (p.hs != 64 && p.hs != 128) return fail("head size must be 64 or 128");
  if (p.dim % 256 || p.hid % 256) return fail("dim and hidden_dim must be multiples of 256");
  if (p.L < 1) return fail("no layers");
  if (p.NS < 1 || p.NS > kMaxNS) return fail("attention splits out of range");
  if (ncu < 8) return fail("too few compute units");
  if ((long long)part_weight(ncu) * (p.V > p.hid ? p.V : p.hid) >= (1ll << 32)) return fail("grid x rows exceeds 32 bits");
  if (5 * p.L + 1 >= 4096) return fail("too many layers for the phase tags");
  p.poll_long = p.dim >= 2048;  // (common.hpp gran_backoff, as persistent_prepare)
  if ((long long)p.B * (p.hid > p.dim + 2 * p.kvd ? p.hid : p.dim + 2 * p.kvd) * 32 >= (1ll << 31))
    return fail("granule offsets exceed 31 bits");
  auto owns = [&](long long n) {  // every block's share non-empty (write-after-read safety, persist.hip)
    for (int b = 0; b < ncu; ++b)
      if (n * part_weight(b + 1) / part_weight(ncu) == n * part_weight(b) / part_weight(ncu)) return false;
    return true;
  };
  if (!owns(p.dim) || !owns((p.dim + 2 * p.kvd) / 2) || !owns(p.hid)) return fail("model too small for the grid");
  const int NB = nb_of(p.B);
  auto nres = [&](int K, long long n_items, int rpi) {
    return (int)((n_items * (100 + kXcdSkew) / part_weight(ncu) + 2) * rpi * ((K + KC - 1) / KC) * NB);
  };
  int nr = 0;
  for (int v : {nres(p.dim, (p.dim + 2 * p.kvd) / 2, 2), nres(p.dim, p.dim, 1), nres(p.dim, p.hid, 2),
                nres(p.hid, p.dim, 1), nres(p.dim, p.V, 1)})
    nr = v > nr ? v : nr;
  p.n_scr = (nr + 3) & ~3;
  p.n_sqa = (int)(((long long)(p.dim + 2 * p.kvd) / 2 * (100 + kXcdSkew) / part_weight(ncu) + 2) * NB);  // RoPE pairs
  if ((long long)p.dim * (100 + kXcdSkew) / part_weight(ncu) + 2 > kResid) return fail("residual slice per block too large");
  // the K-pass strip: as many whole chunks of every sequence as the LDS leaves room for, at most
  // the longest row (one pass per phase where it fits)
  {
    const int kmax = ((p.dim > p.hid ? p.dim : p.hid) + KC - 1) / KC * KC;
    p.pad_floats = 0;
    const size_t rest = lds_bytes(p);
    const long long room = (160 * 1024 - (long long)rest) / (NB * 4) / KC * KC;
    if (room < KC) return fail("activations do not fit the LDS");
    p.pad_floats = (int)(room < kmax ? room : kmax);
  }
  if (lds_bytes(p) > 160 * 1024) return fail("activations do not fit the LDS");
  {  // more than 64 KiB of dynamic LDS (gfx950: 160 KiB per CU), once per device
    static std::mutex mu;
    static unsigned long long done = 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return fail("no current device");
    std::lock_guard<std::mutex> lock(mu);
    const unsigned long long bit = dev < 64 ? 1ull << dev : 0ull;
    if (!bit || !(done & bit)) {
      for (int b = 2; b <= 8; ++b)
        for (const void* f : {kfn_b<64>(b), kfn_b<128>(b)})
          if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
            return fail("cannot raise the dynamic LDS limit");
      done |= bit;
    }
  }
  int nb = 0;
  const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel_of(p), PT, lds_bytes(p));
  if (e != hipSuccess || nb < 1) return fail("batched persistent kernel does not fit one block per CU");
  return true;
}

// The caller zeroes p.sync and the tickets on the same stream right before (persist.hpp).
hipError_t launch_persistent_step_b(const PStep& p, hipStream_t s, int ncu) {
  using namespace pb;
  if (persistent_cooperative()) {
    PStep arg = p;
    void* args[] = {&arg};
    return hipLaunchCooperativeKernel(kernel_of(p), dim3(ncu), dim3(PT), args, (unsigned)lds_bytes(p), s);
  }
  PStep arg = p;
  void* args[] = {&arg};
  return hipLaunchKernel(kernel_of(p), dim3(ncu), dim3(PT), args, lds_bytes(p), s);
}

}  // namespace tl
