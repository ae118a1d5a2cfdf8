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
//  * The activations of every sequence are needed for each weight byte, but B x K floats do not
//    fit the LDS for B = 8 (128 KiB at K = 4096, 344 KiB for W2's K = 11008).  So a GEMV phase
//    runs in K-passes of one row chunk (KC = 2048 floats, 8 KiB of a row): pass c stages
//    x[b][c*KC .. c*KC + KC) of every sequence (64 KiB at B = 8), then the streaming waves sweep
//    chunk c of every row the block owns.  A slot is one 8-KiB row chunk, as in the batch-1 step,
//    and its consume does B dot products with the staged strip (B ds_read_b128 per weight
//    float4: ~40% of the LDS rate at the HBM stream rate, 8 sequences).
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
  int nrow;  // ni * rpi: the slots of every pass
  int nch;   // K-passes (row chunks)
};

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

// B dot products of one row chunk with the staged strip xs [NB][KC4] (sequences >= B skipped):
// row partial res[(rl * nch + c) * NB + b].  One weight float4 at a time against every
// sequence (B LDS reads in flight: the slot buffers stay the only large register set).
template <int NB>
TL_DEVICE void consume_slot(int rl, int c, int nch, int B, int lane, const f4 (&buf)[PL], const f4* xs, float* res) {
  float a[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) a[b] = 0.f;
#pragma unroll
  for (int u = 0; u < PL; ++u) {
#pragma unroll
    for (int b = 0; b < NB; ++b)
      if (b < B) a[b] = dot4(buf[u], xs[b * KC4 + u * 64 + lane], a[b]);
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    if (b < B) {
      const float s = wave_sum_u(a[b]);
      if (lane == 0) res[(rl * nch + c) * NB + b] = s;
    }
  }
}

// A wave's slots in pass c: its two prefetched rows (sw, sw + NSW), then rows dealt from the
// block's LDS counter; loads past the block's rows are skipped.
TL_DEVICE int take_slot(unsigned* ctr, int lane) {
  unsigned v = 0;
  if (lane == 0) v = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  return NBUF * NSW + (int)__builtin_amdgcn_readlane(v, 0);
}

template <int NB>
TL_DEVICE void run_pass(const PDesc& d, const PGeo& g, const PStep& p, int c, int sw, int lane, const f4* xs,
                        float* res, f4 (&buf)[NBUF][PL], unsigned* ctr) {
  int sl[NBUF];
#pragma unroll
  for (int i = 0; i < NBUF; ++i) sl[i] = sw + i * NSW;
  while (sl[0] < g.nrow) {
#pragma unroll
    for (int i = 0; i < NBUF; ++i) {
      if (sl[i] < g.nrow) consume_slot<NB>(sl[i], c, g.nch, p.B, lane, buf[i], xs, res);
      __builtin_amdgcn_sched_barrier(0);
      sl[i] = take_slot(ctr, lane);
      if (sl[i] < g.nrow) load_slot(d, g, p, sl[i], c, lane, buf[i]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// Stage pass c of the phase input for every sequence into xs [NB][KC4], multiplied by the norm
// weight when the phase has one; its squares go, per wave and sequence, to red[wave * NB + b]
// (summed there, not carried: the staging runs while the slot buffers are live).  Input: the
// previous phase's granules (a group of sequences in flight at once, re-polled until their tags
// match), or — QKV at layer 0 — the tokens' embedding rows.  Thread t < 512 owns float4 column t.
template <int NB>
TL_DEVICE void stage_pass(const PDesc& d, const PStep& p, int c, f4* xs, const float* rmsw, float* red, int wave,
                          int lane) {
  const int t = threadIdx.x;
  const bool act = t < KC4;
  const int n4 = d.K >> 2;
  const int k4 = c * KC4 + t;  // float4 index in the row
  const bool live = act && k4 < n4;
  f4 w = f4{1.f, 1.f, 1.f, 1.f};
  if (d.rms && live) w = reinterpret_cast<const f4*>(rmsw)[k4];
  constexpr int GS = NB < 2 ? NB : 2;  // sequences whose granules are in flight together
#pragma unroll
  for (int b0 = 0; b0 < NB; b0 += GS) {
    f4 v[GS];
    if (d.gin) {
      const auto r = rsrc_of(d.gin);
      v4u a[GS], bb[GS];
#pragma unroll
      for (int j = 0; j < GS; ++j) {
        const int b = b0 + j;
        if (live && b < p.B) {
          const unsigned off = (unsigned)(b * n4 + k4) * 32u;
          a[j] = ld16_sc1(r, off);
          bb[j] = ld16_sc1(r, off + 16u);
        }
      }
#pragma unroll
      for (int j = 0; j < GS; ++j) {
        const int b = b0 + j;
        v[j] = f4{0.f, 0.f, 0.f, 0.f};
        if (live && b < p.B)
          v[j] = gran4_ok(a[j], bb[j], d.tag_in) ? gran4_val(a[j], bb[j])
                                                : gran_wait4(r, (unsigned)(b * n4 + k4) * 32u, d.tag_in, p.err);
      }
    } else {
#pragma unroll
      for (int j = 0; j < GS; ++j) {
        const int b = b0 + j;
        v[j] = live && b < p.B ? reinterpret_cast<const f4*>(p.emb + (long long)p.tok[b] * p.dim)[k4]
                               : f4{0.f, 0.f, 0.f, 0.f};
      }
    }
#pragma unroll
    for (int j = 0; j < GS; ++j) {
      const int b = b0 + j;
      if (d.rms) {
        float q = 0.f;
        q = fmaf(v[j].x, v[j].x, q); q = fmaf(v[j].y, v[j].y, q);
        q = fmaf(v[j].z, v[j].z, q); q = fmaf(v[j].w, v[j].w, q);
        q = wave_sum_u(q);
        if (lane == 0) red[wave * NB + b] = q;
        v[j] = f4{__fmul_rn(w.x, v[j].x), __fmul_rn(w.y, v[j].y), __fmul_rn(w.z, v[j].z), __fmul_rn(w.w, v[j].w)};
      }
      if (act) xs[b * KC4 + t] = v[j];
    }
  }
}

TL_DEVICE void preload_rms(const float* w, int dim, float* rmsw, int lane) {
  const f4* s4 = reinterpret_cast<const f4*>(w);
  f4* d4 = reinterpret_cast<f4*>(rmsw);
  for (int j = lane; j < (dim >> 2); j += 64) d4[j] = s4[j];
}

// Control wave: row values from the pass partials (chunks in order), the norm scale, the fused
// epilogue, granule stores.  xres: this block's slice of every sequence's residual stream.
template <int NB>
TL_DEVICE void epilogue(const PDesc& d, const PGeo& g, const PStep& p, const float* res, float* xres,
                        const float* ss, int lane, int l, const uint64_t* etab) {
  unsigned long long best[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) best[b] = 0;
  // (item, sequence) pairs over the lanes: a block owns 16-130 items, so items alone would
  // leave most lanes idle on this hand-off's critical path
  const int npair = g.ni * p.B;
  for (int j = lane; j < npair; j += 64) {
    const int it = j / p.B, b = j - it * p.B;
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
        const int i = row < p.dim ? row : row - p.dim;
        const float2 cs = p.rope[(long long)pb * (p.hs >> 1) + ((i % p.hs) >> 1)];
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
      if (lane == 0 && b < p.B) st8_sc1(p.bmax + (long long)blockIdx.x * NB + b, bv);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drained before the final arrival
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

// The phase sequence as one wave sees it.  ROLE0 = the control wave.  Both run the same
// workgroup barriers: per GEMV phase and pass, one after the staging and one after the sweep.
template <int HS, int NB, bool ROLE0>
TL_DEVICE void phases(const PStep& p, int wave, int lane, float* res, float* xres, float* red, float* rmsw,
                      f4* xs, const uint64_t* etab, unsigned tb) {
  const int G = gridDim.x;
  const int nph = 5 * p.L + 1;
  float* ssum = red + PW * NB;                                   // [NB] this phase's sum of squares
  float* sscale = ssum + NB;                                     // [NB] its norm scales (epilogue)
  unsigned* ctr = reinterpret_cast<unsigned*>(sscale + NB);      // dynamic slot counter
  f4 buf[NBUF][PL];
  const int sw = wave - 1;
  if constexpr (ROLE0) {
    // this block's slice of every sequence's residual stream starts as its embedding row
    const PGeo gx = geo(make_desc(p, PK_WO, 0, tb));
    for (int b = 0; b < p.B; ++b) {
      const float* er = p.emb + (long long)p.tok[b] * p.dim + gx.i0;
      for (int it = lane; it < gx.ni; it += 64) xres[b * kResid + it] = er[it];
    }
    preload_rms(p.rms_att, p.dim, rmsw, lane);
    if (lane < NB) ssum[lane] = 0.f;
    if (lane == 0) *ctr = 0u;
  } else {
    const PDesc d0 = make_desc(p, PK_QKV, 0, tb);
    const PGeo g0 = geo(d0);
#pragma unroll
    for (int i = 0; i < NBUF; ++i)
      if (sw + i * NSW < g0.nrow) load_slot(d0, g0, p, sw + i * NSW, 0, lane, buf[i]);
  }
  __syncthreads();  // first norm weights preloaded, counters set

  for (int ph = 0; ph < nph; ++ph) {
    const int l = ph / 5;
    const int kind = ph == nph - 1 ? PK_CLS : ph % 5;
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
        aw.cnt = p.tickets + (long long)l * p.B * p.H; aw.B = p.B; aw.NS = p.NS;
        aw.gqkv = p.gqkv; aw.gout = p.gxb;
        aw.etab = etab;
        aw.tag_in = tb + 5u * l + 1; aw.tag_out = tb + 5u * l + 2; aw.err = p.err;
        const int units = p.B * p.H * p.NS;
        for (int u = blockIdx.x + G * wave; u < units; u += G * PW) attn_unit<HS, 16, true>(aw, u, lane);
      }
      if constexpr (!ROLE0) {  // Wo's first slots stream in while its input is gathered
        const PDesc nd = make_desc(p, PK_WO, l, tb);
        const PGeo ng = geo(nd);
#pragma unroll
        for (int i = 0; i < NBUF; ++i)
          if (sw + i * NSW < ng.nrow) load_slot(nd, ng, p, sw + i * NSW, 0, lane, buf[i]);
      }
      continue;
    }
    const PDesc d = make_desc(p, kind, kind == PK_CLS ? p.L : l, tb);
    const PGeo g = geo(d);
    for (int c = 0; c < g.nch; ++c) {
      stage_pass<NB>(d, p, c, xs, rmsw, red, wave, lane);
      __syncthreads();  // strip staged (and this pass's squares per wave in red)
      if constexpr (ROLE0) {
        if (d.rms && lane < NB) {
          float s = ssum[lane];
          for (int w = 0; w < PW; ++w) s = __fadd_rn(s, red[w * NB + lane]);
          ssum[lane] = s;
        }
        if (c == g.nch - 1) {  // the staging is done with this phase's norm weights: the next
          if (kind == PK_QKV) preload_rms(p.rms_ffn + (long long)l * p.dim, p.dim, rmsw, lane);
          if (kind == PK_UP)
            preload_rms(l + 1 < p.L ? p.rms_att + (long long)(l + 1) * p.dim : p.rms_final, p.dim, rmsw, lane);
        }
      } else {
        run_pass<NB>(d, g, p, c, sw, lane, xs, res, buf, ctr);
      }
      __syncthreads();  // every slot of the pass reduced into res; the strip may be restaged
      if constexpr (ROLE0) {
        if (lane == 0) *ctr = 0u;  // the next pass's slot counter (used after its staging barrier)
      } else {
        // the next pass's (or the next GEMV phase's) first slots: their data streams in while the
        // strip is restaged, the hand-off is waited for and the epilogue runs
        if (c + 1 < g.nch) {
#pragma unroll
          for (int i = 0; i < NBUF; ++i)
            if (sw + i * NSW < g.nrow) load_slot(d, g, p, sw + i * NSW, c + 1, lane, buf[i]);
        } else if (kind != PK_CLS && kind != PK_QKV) {  // (after QKV: once the attention units ran)
          const PDesc nd = next_desc(p, kind, l, tb);
          const PGeo ng = geo(nd);
#pragma unroll
          for (int i = 0; i < NBUF; ++i)
            if (sw + i * NSW < ng.nrow) load_slot(nd, ng, p, sw + i * NSW, 0, lane, buf[i]);
        }
      }
    }
    if constexpr (ROLE0) {
      if (lane < NB) {
        // reference rmsnorm scale (src/seq.cpp:3-16): 1 / sqrtf(sum / size + 1e-5f); kept in LDS
        // because the epilogue indexes it by a run-time sequence (a register array would go to scratch)
        sscale[lane] = d.rms ? __fdiv_rn(1.0f, sqrtf(__fadd_rn(__fdiv_rn(ssum[lane], (float)d.K), 1e-5f))) : 1.f;
        ssum[lane] = 0.f;
      }
      epilogue<NB>(d, g, p, res, xres, sscale, lane, l, etab);
    }
  }
  grid_barrier(p);
  if constexpr (ROLE0) {
    if (blockIdx.x != 0) return;
    if (p.argmax) {
      // per sequence: argmax over the per-block winners + advance (src/llama.cpp:275-286)
      for (int b = 0; b < p.B; ++b) {
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
  f4* xs = reinterpret_cast<f4*>(smem);                      // NB * KC floats: the staged strip
  float* xres = reinterpret_cast<float*>(xs + NB * KC4);    // NB * kResid: residual slices
  float* rmsw = xres + NB * kResid;                         // dim: the norm weights
  float* red = rmsw + p.dim;                                // PW * NB + 2 * NB + 4
  float* res = red + PW * NB + 2 * NB + 4;                  // n_res: row-chunk partials
  uint64_t* etab = reinterpret_cast<uint64_t*>(res + p.n_scr);  // the expf table (32 doubles' bits)
  {
    constexpr uint64_t tab[32] = TL_EXPF_TABLE;
    if (threadIdx.x < 32) etab[threadIdx.x] = tab[threadIdx.x];  // (read after the first barrier)
  }
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const unsigned tb = p.seq[0] << 12;  // tag base of this launch
  if (wave == 0) phases<HS, NB, true>(p, wave, lane, res, xres, red, rmsw, xs, etab, tb);
  else phases<HS, NB, false>(p, wave, lane, res, xres, red, rmsw, xs, etab, tb);
}

static int nb_of(int B) { return B <= 2 ? 2 : B <= 4 ? 4 : 8; }

static size_t lds_bytes(const PStep& p) {
  const int NB = nb_of(p.B);
  return (size_t)NB * KC * 4 + (size_t)NB * kResid * 4 + (size_t)p.dim * 4 + (size_t)(PW * NB + 2 * NB + 4) * 4 +
         (size_t)p.n_scr * 4 + 32 * 8;
}

template <int HS, int NB>
static const void* kfn() { return (const void*)persistent_step_b_kernel<HS, NB>; }
static const void* kernel_of(const PStep& p) {
  const int NB = nb_of(p.B);
  if (p.hs == 128) return NB == 2 ? kfn<128, 2>() : NB == 4 ? kfn<128, 4>() : kfn<128, 8>();
  return NB == 2 ? kfn<64, 2>() : NB == 4 ? kfn<64, 4>() : kfn<64, 8>();
}

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
  if ((long long)p.dim * (100 + kXcdSkew) / part_weight(ncu) + 2 > kResid) return fail("residual slice per block too large");
  if (lds_bytes(p) > 160 * 1024) return fail("activations do not fit the LDS");
  {  // more than 64 KiB of dynamic LDS (gfx950: 160 KiB per CU), once per device
    static std::mutex mu;
    static unsigned long long done = 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return fail("no current device");
    std::lock_guard<std::mutex> lock(mu);
    const unsigned long long bit = dev < 64 ? 1ull << dev : 0ull;
    if (!bit || !(done & bit)) {
      for (const void* f : {kfn<64, 2>(), kfn<64, 4>(), kfn<64, 8>(), kfn<128, 2>(), kfn<128, 4>(), kfn<128, 8>()})
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
