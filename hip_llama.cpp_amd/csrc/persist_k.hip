// persist_k.hip — the whole decode step of 8 sequences as ONE persistent launch, with K-split
// ownership of every GEMV phase (fp32 weights).
//
// Semantics: the reference forward (src/seq.cpp:53-168; its GPU twin thaDNN_s_forward_batch,
// src/thaDNN.cpp:13-81, for 8 sequences at their own positions) followed, in greedy mode, by
// sample_argmax per sequence (src/llama.cpp:275-286).
//
// Why a third persistent engine: the batched one (persist_b.hip) has each CU own whole rows, so
// every CU gathers every phase's whole input for all 8 sequences — 1.5 MB of hand-off granules
// per CU per layer at 7B, ~12 us of staging per phase (profiles/r03/persist_trace_b8_pos8_v2.txt),
// and it loses to the multi-launch step at 8 sequences.  Here a CU owns a (row group, K slice)
// tile instead, so it gathers only its K slice:
//   * grid = G blocks (one per CU), G % 64 == 0; block bi sits on XCD bi % 8 (round-robin
//     dispatch).  K group kg = (bi / 8) % 8 and row group rg = (bi % 8) * (G / 64) + bi / 64, so
//     the 8 blocks of a row group (its 8 K slices) share one XCD and one L2;
//   * phase input (B x K floats) -> the block stages x[b][K slice kg] (K / 8 per sequence: 16 KiB
//     of granules at K = 4096) into LDS, times the RMSNorm weight where the phase has one;
//   * the streaming waves sweep the row group's rows over that slice; each slot's row partials of
//     the 8 sequences go to LDS, and the control wave publishes finished slots as granules
//     P[kg][row][b] while the sweep runs (a global store in the streaming waves sat in their vmcnt
//     queue ahead of the next slot's loads);
//   * reduce-scatter inside the row group: block (rg, kg) owns sub-slice kg of the row group's
//     items, sums their 8 partials in K-group order (fixed: deterministic), applies the norm scale
//     and the fused epilogue (RoPE + K/V row, residual, SwiGLU, logits + argmax) and publishes the
//     phase output as granules — which the next phase's blocks gather by K slice;
//   * RMSNorm is (W (w * x)) * ss_b as in persist_b.hip (a K slice cannot see the whole row's
//     sum of squares): the residual phases' reducers publish per-sub-slice sums of squares and
//     the normed phases' control waves add them up (fixed order) while the rows stream.
// Two hand-offs per phase (partials, then outputs) of ~1-2 KiB per block each, instead of one
// all-gather of B x K granules; each streaming wave has one slot of the next phase in flight across
// them, issued after the reduce (more weight traffic there slows the hand-offs: kPrefetchSlots).
//
// Hand-off buffers (granules, PStep::gk) are per kind and layer PARITY: a block writes the buffers
// of phase (l + 2) only after its staging of that phase, which transitively waited for every
// block to finish reading those of phase l (the staging of a K slice waits for the 4 row groups
// that produce it, whose reducers each waited for their 8 K groups, whose staging waited for all
// 32 row groups of the phase before: every block is then past the reduce of phase l).
//
// Shared with persist_b.hip: one block per CU (here 512 threads), all co-resident (cooperative
// launch); wave 0 = control, the others stream with two register slots in flight each; granules {value, tag}
// with tags (launch sequence << 12) + phase + 1; every wait bounded with the sticky error word;
// attention as wave units over every wave of the grid (attention.hpp attn_unit); one grid barrier
// (the final argmax).
#include <hip/hip_runtime.h>
#include <mutex>
#include "attention.hpp"
#include "gemv.hpp"
#include "persist.hpp"
#include "wave_reduce.hpp"

namespace tl {
namespace pk {

constexpr int NB = 8;           // sequences (the only instantiated batch)
constexpr int NKG = 8;          // K groups per row group
constexpr int PW = 8;           // waves per block: 1 control + 7 streaming (two waves per SIMD: 256
                                // VGPRs each; at 9 waves the 168-VGPR budget spilled ~1000 VGPRs)
constexpr int PT = PW * 64;
constexpr int NSW = PW - 1;
constexpr int NBUF = 2;         // register slots in flight per streaming wave
// (a third register slot spilled; a third slot in LDS by LDS-DMA, during the sweep or only across
// the boundary, lost 2-3%: DESIGN.md section 7)
// The next phase's slots a streaming wave issues before that phase's input is staged, and when:
// ONE slot, after this phase's reduce.  Weight loads in flight slow the latency-bound hand-off loads
// they share the memory path with (7B B=8, same box: two slots after the sweep 1226 tok/s, one
// slot after the sweep 1399, two after the reduce 1256, one after the reduce 1425, none 1349 on
// another box where two after the sweep gave 1363 and one 1379; profiles/r06/ksplit_ab.txt).
#ifndef PK_PREFETCH_SLOTS
#define PK_PREFETCH_SLOTS 1
#endif
constexpr int kPrefetchSlots = PK_PREFETCH_SLOTS;
#ifndef PK_PREFETCH_AFTER_REDUCE
#define PK_PREFETCH_AFTER_REDUCE 1
#endif
constexpr bool kPrefetchAfterReduce = PK_PREFETCH_AFTER_REDUCE;
#ifndef PK_PREFETCH_WAVES
#define PK_PREFETCH_WAVES NSW
#endif
constexpr int kPrefetchWaves = PK_PREFETCH_WAVES;  // streaming waves that prefetch (the first ones)

constexpr int PLM = 8;          // wave-loads (1 KiB) per slot at most
constexpr int SBU = 4;          // staging: (sequence, float4) units in flight per thread
constexpr int kRes = 64;        // residual rows per block and sequence (a sub-slice of dim)
constexpr int kRcs = 64;        // QKV items per reduce sub-slice (RoPE table in LDS)
constexpr int kMaxSlots = 1280; // slots per phase and block at most (rows of a row group)
constexpr unsigned kSpinLimit = 1u << 18;
// Re-poll pause of the hand-off waits on the critical path (staging, reduce, attention inputs):
// common.hpp gran_backoff's long form (up to 2048 cycles after 6 misses).
#ifndef PK_POLL_LONG
#define PK_POLL_LONG 1
#endif
constexpr bool kPollLong = PK_POLL_LONG;  // (short pauses: 1308 vs 1394-1418 tok/s, the extra polls slow the sweeps)

enum PKind : int { PK_QKV = 0, PK_ATTN = 1, PK_WO = 2, PK_UP = 3, PK_DOWN = 4, PK_CLS = 5 };

// Rows per slot for RW wave-loads per row slice (a slot is <= 8 wave-loads).
__host__ __device__ constexpr int sr_of(int RW) { return RW <= 2 ? 4 : RW <= 4 ? 2 : 1; }

// Granule offsets of the hand-off area (PStep::gk): per layer parity the activations (x after W2,
// q|k|v, the attention output, x after Wo, the SwiGLU output), the K-group partials of the four
// layer GEMVs and the residual phases' sums of squares; the classifier's partials once.
struct KLayout {
  long long xdown, qkv, xb, xmid, hb, act;       // offsets inside a parity's activation block, its size
  long long pqkv, pwo, pup, pdown, part;         // offsets inside a parity's partial block, its size
  long long sswo, ssdown, ss;                    // sums of squares [G][NB]
  long long act0, part0, ss0, cls, total;        // block bases
};
__host__ __device__ inline long long al64(long long n) { return (n + 63) & ~63ll; }
__host__ __device__ inline KLayout klayout(int dim, int hid, int kvd, int V, int G) {
  KLayout k;
  const long long B = NB, qr = dim + 2ll * kvd;
  k.xdown = 0; k.qkv = al64(B * dim); k.xb = k.qkv + al64(B * qr); k.xmid = k.xb + al64(B * dim);
  k.hb = k.xmid + al64(B * dim); k.act = k.hb + al64(B * hid);
  k.pqkv = 0; k.pwo = al64(NKG * qr * B); k.pup = k.pwo + al64(NKG * (long long)dim * B);
  k.pdown = k.pup + al64(NKG * 2ll * hid * B); k.part = k.pdown + al64(NKG * (long long)dim * B);
  k.sswo = 0; k.ssdown = al64((long long)G * B); k.ss = 2 * k.ssdown;
  k.act0 = 0; k.part0 = 2 * k.act; k.ss0 = k.part0 + 2 * k.part; k.cls = k.ss0 + 2 * k.ss;
  k.total = k.cls + al64(NKG * (long long)V * B);
  return k;
}

struct KDesc {
  int kind;
  int K;                               // row length = input length (floats)
  int n_items;                         // rows, or row pairs (QKV, SwiGLU)
  int rpi;                             // rows per item
  const float *W0, *W1, *W2;
  const unsigned long long* gin;       // input granules [NB][K] (null: the tokens' embedding rows)
  unsigned tag_in;
  const float* rms;                    // fused RMSNorm weight or null
  const unsigned long long* gss_in;    // its sums of squares [G][NB] (null at layer 0: the embedding)
  unsigned long long* gout;            // output granules [NB][...] (null for the classifier)
  unsigned tag_out;                    // (also the tag of the partials and the sums of squares)
  unsigned long long* gpart;           // K-group partials [NKG][rows][NB]
  unsigned long long* gss_out;         // residual phases: this phase's sums of squares [G][NB]
};

// The attention fused into the QKV phase: row group h = head h's q, k and v rows (virtual row
// order: head-major, q | k | v inside a head), block (h, b) reduces sequence b's rows and runs the
// attention of (b, h) with its waves — one hand-off and the attention units' ticket combine fewer
// per layer.  Needs one row group per head (H = G / 8), one K/V head per head and head size 128.
// Off by default: same box, 7B B=8, 1431 vs 1416 tok/s unfused (multi-launch 1419) over positions
// 0..255 but 770 vs 1009 at 1792..2047 — its per-wave key loop (8-B loads, one 16-key chunk in
// flight, a wave reduction per key) is latency-bound where the attention units are not
// (profiles/r06/ksplit_ab.txt).  Parity-tested like the rest (PK_FUSE_ATTN=1: 16 passed).
#ifndef PK_FUSE_ATTN
#define PK_FUSE_ATTN 0
#endif
TL_DEVICE bool attn_fusable(const PStep& p) {
  return PK_FUSE_ATTN && p.H == (int)(gridDim.x >> 3) && p.kv_mul == 1 && p.hs == 128;
}

TL_DEVICE KDesc make_desc(const PStep& p, int kind, int l, unsigned tb) {
  const KLayout k = klayout(p.dim, p.hid, p.kvd, p.V, gridDim.x);
  unsigned long long* g = p.gk;
  auto act = [&](int l_, long long off) { return g + k.act0 + (l_ & 1) * k.act + off; };
  auto part = [&](int l_, long long off) { return g + k.part0 + (l_ & 1) * k.part + off; };
  auto ss = [&](int l_, long long off) { return g + k.ss0 + (l_ & 1) * k.ss + off; };
  KDesc d = {};
  d.kind = kind;
  const long long ll = l, dim = p.dim, hid = p.hid, kvd = p.kvd;
  const unsigned t0 = tb + 5u * l;  // tag of the phase before QKV(l), i.e. W2(l-1)
  switch (kind) {
    case PK_QKV:
      d.K = p.dim; d.n_items = (p.dim + 2 * p.kvd) / 2; d.rpi = 2;
      d.W0 = p.wq + ll * dim * dim; d.W1 = p.wk + ll * dim * kvd; d.W2 = p.wv + ll * dim * kvd;
      d.gin = l == 0 ? nullptr : act(l - 1, k.xdown); d.tag_in = t0;
      d.rms = p.rms_att + ll * dim; d.gss_in = l == 0 ? nullptr : ss(l - 1, k.ssdown);
      d.gout = act(l, k.qkv); d.tag_out = t0 + 1; d.gpart = part(l, k.pqkv);
      if (attn_fusable(p)) d.gout = act(l, k.xb);  // (its output: the attention output xb, tag t0 + 2)
      break;
    case PK_WO:
      d.K = p.dim; d.n_items = p.dim; d.rpi = 1;
      d.W0 = p.wo + ll * dim * dim; d.gin = act(l, k.xb); d.tag_in = t0 + 2;
      d.gout = act(l, k.xmid); d.tag_out = t0 + 3; d.gpart = part(l, k.pwo); d.gss_out = ss(l, k.sswo);
      break;
    case PK_UP:
      d.K = p.dim; d.n_items = p.hid; d.rpi = 2;
      d.W0 = p.w1 + ll * dim * hid; d.W1 = p.w3 + ll * dim * hid;
      d.gin = act(l, k.xmid); d.tag_in = t0 + 3; d.rms = p.rms_ffn + ll * dim; d.gss_in = ss(l, k.sswo);
      d.gout = act(l, k.hb); d.tag_out = t0 + 4; d.gpart = part(l, k.pup);
      break;
    case PK_DOWN:
      d.K = p.hid; d.n_items = p.dim; d.rpi = 1;
      d.W0 = p.w2 + ll * dim * hid; d.gin = act(l, k.hb); d.tag_in = t0 + 4;
      d.gout = act(l, k.xdown); d.tag_out = t0 + 5; d.gpart = part(l, k.pdown); d.gss_out = ss(l, k.ssdown);
      break;
    default:  // PK_CLS (l = L)
      d.K = p.dim; d.n_items = p.V; d.rpi = 1;
      d.W0 = p.wcls; d.gin = act(p.L - 1, k.xdown); d.tag_in = tb + 5u * p.L;
      d.rms = p.rms_final; d.gss_in = ss(p.L - 1, k.ssdown);
      d.tag_out = tb + 5u * p.L + 1; d.gpart = g + k.cls;
      break;
  }
  return d;
}

// This block's tile of a phase (wave-uniform).
struct KGeo {
  int rg, kg;
  int i0, ni, nrow;  // the row group's items, its rows (ni * rpi)
  int s0, ns;        // this block's reduce sub-slice of those items
  int k4lo, n4;      // the K slice (float4 units)
  int ssi;           // the sub-slice's index among all G (sums of squares, in row order)
};
// Row groups may get items in proportion to their XCD's streaming rate: the row groups of the even
// XCDs (rg / (G / 64) even) kXcdSkew percent more than the odd ones, which stream that much slower
// (ffn_up 49.6-50.9 vs 53.5-55.3 us per block, ffn_down likewise: tools/persist_trace.py --batch 8).
// Off (0): at 7 the per-XCD sweeps evened out but the step did not move (the XCDs share one
// bandwidth).  rg_weight(r) = the weight of row groups 0..r-1.
#ifndef PK_XCD_SKEW
#define PK_XCD_SKEW 0
#endif
constexpr unsigned kXcdSkew = PK_XCD_SKEW;
static_assert(!PK_FUSE_ATTN || PK_XCD_SKEW == 0, "the fused attention's row group h is head h: uniform row groups");
__host__ __device__ inline long long rg_weight(int r, int G) {
  const int per = G >> 6;  // row groups per XCD
  const int x = r / per, rem = r - x * per;
  // whole XCDs before r: pairs (even, odd) weigh 200 + skew per row group
  const long long full = (long long)(x >> 1) * per * (200 + kXcdSkew) + (x & 1) * (long long)per * (100 + kXcdSkew);
  return full + (long long)rem * ((x & 1) ? 100 : 100 + kXcdSkew);
}

TL_DEVICE KGeo geo(const KDesc& d) {
  KGeo g;
  const int G = gridDim.x, bi = blockIdx.x;
  const int j = bi >> 3;
  g.kg = j & 7;
  g.rg = (bi & 7) * (G >> 6) + (j >> 3);
  const long long n = d.n_items;
  g.i0 = (int)(n * rg_weight(g.rg, G) / rg_weight(G >> 3, G));
  g.ni = (int)(n * rg_weight(g.rg + 1, G) / rg_weight(G >> 3, G)) - g.i0;
  g.nrow = g.ni * d.rpi;
  g.s0 = g.i0 + g.ni * g.kg / NKG;
  g.ns = g.i0 + g.ni * (g.kg + 1) / NKG - g.s0;
  const int K4 = d.K >> 2;
  g.k4lo = K4 * g.kg / NKG;
  g.n4 = K4 * (g.kg + 1) / NKG - g.k4lo;
  g.ssi = g.rg * NKG + g.kg;
  return g;
}

// (The descriptor's matrix pointers are copied out through an empty asm first: a select between
// struct fields became an indexed access to the struct, which then lived in scratch memory — and a
// scratch load waits in the wave's vmcnt queue behind its weight loads.)
TL_DEVICE const float* pick3(const KDesc& d, int i) {
  const float *w0 = d.W0, *w1 = d.W1, *w2 = d.W2;
  asm volatile("" : "+s"(w0), "+s"(w1), "+s"(w2));
  return i == 0 ? w0 : i == 1 ? w1 : w2;
}
TL_DEVICE const float* row_ptr(const KDesc& d, const PStep& p, int R) {
  const long long K = d.K;
  if (d.kind == PK_UP) return pick3(d, R & 1) + (long long)(R >> 1) * K;
  if (d.kind == PK_QKV && attn_fusable(p)) {  // virtual row R = head h's row r of q | k | v
    const int h = R / (3 * 128), r = R - h * (3 * 128);
    return pick3(d, r >> 7) + (long long)(h * 128 + (r & 127)) * K;
  }
  if (d.kind == PK_QKV) {
    const int seg = R < p.dim ? 0 : R < p.dim + p.kvd ? 1 : 2;
    return pick3(d, seg) + (long long)(R - (seg == 0 ? 0 : seg == 1 ? p.dim : p.dim + p.kvd)) * K;
  }
  return d.W0 + (long long)R * K;
}

// Slot s: rows s*SR .. s*SR+SR-1 of the row group, each its K slice as RW wave-loads of 1 KiB
// (lane l: float4 64 u + l of the slice), non-temporal raw buffer loads clamped to the slice
// (loads past it, or for rows past the group — slots past the phase included — return 0 without
// touching memory: the loads are unconditional, so the slot registers are never merged with older
// contents).
template <int RW>
TL_DEVICE void load_slot(const KDesc& d, const KGeo& g, const PStep& p, int s, int lane, f4 (&buf)[PLM]) {
  constexpr int SR = sr_of(RW);
#pragma unroll
  for (int r = 0; r < SR; ++r) {
    const int rl = s * SR + r;
    const bool live = rl < g.nrow;
    const float* row = row_ptr(d, p, g.i0 * d.rpi + (live ? rl : 0)) + 4 * g.k4lo;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(row), (short)0, live ? g.n4 * 16 : 0, 0x00020000);
#pragma unroll
    for (int u = 0; u < RW; ++u)
      buf[r * RW + u] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16 + u * 1024, 0, 2 /*nt*/));
  }
}

// Consume slot s: SR rows x RW wave-loads against the staged slice (the same columns for every
// row, so each slice read serves SR rows), then the SR x NB partials of the slot, reduced over the
// wave, into the block's LDS partials pres[row][b] (publish_partials sends them on).  The slice is staged as 8
// planes (column c of a float4, sequences 4h..4h+3): xs[(c * 2 + h) * XS4 + j] = x[4h..4h+3][4j + c],
// so a lane's 8 reads are contiguous across the wave (no bank conflicts) and every weight float
// multiplies sequence PAIRS with one packed FMA (v_pk_fma_f32, the weight broadcast): 128 instead of
// 256 FMA instructions per slot, half of the consume's VALU time at 8 sequences.
typedef float f2 __attribute__((ext_vector_type(2)));
template <int RW>
TL_DEVICE void consume_slot(const KDesc& d, const KGeo& g, int s, int lane, const f4 (&buf)[PLM], const f4* xs,
                            float* pres) {
  constexpr int SR = sr_of(RW);
  constexpr int NV = SR * NB;
  constexpr int XS4 = RW * 64;
  f2 acc[SR][NB / 2];
#pragma unroll
  for (int r = 0; r < SR; ++r)
#pragma unroll
    for (int q = 0; q < NB / 2; ++q) acc[r][q] = f2{0.f, 0.f};
  // the slice offset is laundered so the compiler cannot prove the reads loop-invariant across
  // slots (it would keep RW x 8 float4 live over the whole sweep)
  int xo = lane;
  asm volatile("" : "+v"(xo));
  const f4* xc = xs + xo;
#pragma unroll
  for (int u = 0; u < RW; ++u) {
    f4 xq[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) xq[k] = xc[k * XS4 + u * 64];
#pragma unroll
    for (int r = 0; r < SR; ++r) {
      const f4 w = buf[r * RW + u];
      const float wc[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const f2 ww = f2{wc[c], wc[c]};
        acc[r][0] = __builtin_elementwise_fma(ww, f2{xq[2 * c].x, xq[2 * c].y}, acc[r][0]);
        acc[r][1] = __builtin_elementwise_fma(ww, f2{xq[2 * c].z, xq[2 * c].w}, acc[r][1]);
        acc[r][2] = __builtin_elementwise_fma(ww, f2{xq[2 * c + 1].x, xq[2 * c + 1].y}, acc[r][2]);
        acc[r][3] = __builtin_elementwise_fma(ww, f2{xq[2 * c + 1].z, xq[2 * c + 1].w}, acc[r][3]);
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // one wave-load's slice reads live at a time
  }
  float v[NV];
#pragma unroll
  for (int r = 0; r < SR; ++r)
#pragma unroll
    for (int q = 0; q < NB / 2; ++q) {
      v[r * NB + 2 * q] = acc[r][q].x;
      v[r * NB + 2 * q + 1] = acc[r][q].y;
    }
  const float t = wave_reduce_t<NV>(v, lane);
  const int i = (lane >> 1) & (NV - 1), rl = s * SR + i / NB;
  // into the block's LDS partials (published after the sweep: a global store here would sit in the
  // wave's vmcnt queue ahead of the next slot's loads)
  if ((lane & 1) == 0 && lane < 2 * NV && rl < g.nrow) pres[rl * NB + (i % NB)] = t;
}

// Control wave, during the sweep: publish the block's partials P[kg][rows of the group][b] as
// granules slot by slot, in slot order, as the streaming waves mark them done (sdone[s] == mark), so
// only the last slot's are left when the sweep ends.  Every slot is consumed by some streaming
// wave, so the loop ends.
template <int RW>
TL_DEVICE void publish_partials(const KDesc& d, const KGeo& g, const float* pres, const unsigned* sdone,
                                unsigned mark, int lane) {
  constexpr int SR = sr_of(RW);
  const long long rows = (long long)d.n_items * d.rpi;
  unsigned long long* dst = d.gpart + ((long long)g.kg * rows + (long long)g.i0 * d.rpi) * NB;
  const int nslot = (g.nrow + SR - 1) / SR;
  for (int s = 0; s < nslot;) {
    // the run of consecutive done slots from s (one flag per lane), published in one pass
    const bool done = s + lane < nslot &&
                      __hip_atomic_load(sdone + s + lane, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == mark;
    const unsigned long long nd = ~__ballot(done);
    const int run = nd ? __builtin_ctzll(nd) : 64;
    if (run == 0) {
      __builtin_amdgcn_s_sleep(4);
      continue;
    }
    const int e1 = (s + run) * SR * NB < g.nrow * NB ? (s + run) * SR * NB : g.nrow * NB;
    for (int e = s * SR * NB + lane; e < e1; e += 64) st8_sc1(dst + e, gran(d.tag_out, pres[e]));
    s += run;
  }
}

TL_DEVICE int take_slot(unsigned* ctr, int lane) {
  unsigned v = 0;
  if (lane == 0) v = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  return NBUF * NSW + (int)__builtin_amdgcn_readlane(v, 0);
}

// A wave's first slots of a phase (its prefetch: issued before the hand-offs they overlap; see
// kPrefetchSlots for how many and when).
template <int RW>
TL_DEVICE void prefetch(const KDesc& d, const KGeo& g, const PStep& p, int sw, int lane, f4 (&buf)[NBUF][PLM]) {
#pragma unroll
  for (int i = 0; i < NBUF; ++i)
    if (i < kPrefetchSlots && sw < kPrefetchWaves) load_slot<RW>(d, g, p, sw + i * NSW, lane, buf[i]);
}

// The sweep: the first slots (sw, sw + NSW; those prefetch() did not issue are issued here), then
// slots dealt from the block's counter, each refilling the buffer it was consumed from (slots are
// taken in increasing order per wave).
template <int RW>
TL_DEVICE void run_slots(const KDesc& d, const KGeo& g, const PStep& p, int sw, int lane, const f4* xs,
                         f4 (&buf)[NBUF][PLM], float* pres, unsigned* sdone, unsigned mark, unsigned* ctr,
                         unsigned long long* ts) {
  const int nslot = (g.nrow + sr_of(RW) - 1) / sr_of(RW);
  int sl[NBUF];
#pragma unroll
  for (int i = 0; i < NBUF; ++i) {
    sl[i] = sw + i * NSW;
    if (!(i < kPrefetchSlots && sw < kPrefetchWaves)) load_slot<RW>(d, g, p, sl[i], lane, buf[i]);
  }
  while (sl[0] < nslot) {  // (sl[0] < sl[1] always: a later take draws a larger slot)
#pragma unroll
    for (int i = 0; i < NBUF; ++i) {
      if (sl[i] < nslot) {
        consume_slot<RW>(d, g, sl[i], lane, buf[i], xs, pres);
        // the slot's partials are in pres: the control wave may publish them (release: after them)
        if (lane == 0) __hip_atomic_store(sdone + sl[i], mark, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      if (i == 0 && ts && lane == 0 && sl[0] == sw) ts[6] = __builtin_amdgcn_s_memrealtime();  // first slot in
      __builtin_amdgcn_sched_barrier(0);
      sl[i] = take_slot(ctr, lane);
      load_slot<RW>(d, g, p, sl[i], lane, buf[i]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// Stage the K slice of every sequence's phase input into xs (consume_slot's 8 planes of RW * 64
// float4, zeros past the slice),
// times the norm weight where the phase has one (constants, from L2).  Input: the previous
// phase's granules (SBU units in flight per thread, late ones re-polled until their tags match),
// or — QKV at layer 0 — the tokens' embedding rows.
template <int RW>
TL_DEVICE void stage(const KDesc& d, const KGeo& g, const PStep& p, f4* xs) {
  constexpr int XS4 = RW * 64;
  constexpr int U = NB * XS4;
  const int t = threadIdx.x;
  const int K4 = d.K >> 2;
  const auto r = rsrc_of(d.gin ? (const void*)d.gin : (const void*)p.emb);
  for (int u0 = t; u0 < U; u0 += SBU * PT) {
    v4u ga[SBU], gb[SBU];
#pragma unroll
    for (int k = 0; k < SBU; ++k) {
      const int u = u0 + k * PT, b = u / XS4, j = u - b * XS4;
      if (d.gin && u < U && j < g.n4) {
        const unsigned off = (unsigned)(b * K4 + g.k4lo + j) * 32u;
        ga[k] = ld16_sc1(r, off);
        gb[k] = ld16_sc1(r, off + 16u);
      }
    }
#pragma unroll
    for (int k = 0; k < SBU; ++k) {
      const int u = u0 + k * PT, b = u / XS4, j = u - b * XS4;
      if (u >= U) continue;
      f4 v = f4{0.f, 0.f, 0.f, 0.f};
      if (j < g.n4) {
        const int k4 = g.k4lo + j;
        if (d.gin)
          v = gran4_ok(ga[k], gb[k], d.tag_in) ? gran4_val(ga[k], gb[k])
                                               : gran_wait4(r, (unsigned)(b * K4 + k4) * 32u, d.tag_in, p.err, kPollLong);
        else
          v = reinterpret_cast<const f4*>(p.emb + (long long)p.tok[b] * p.dim)[k4];
        if (d.rms) {
          const f4 w = reinterpret_cast<const f4*>(d.rms)[k4];
          v = f4{__fmul_rn(w.x, v.x), __fmul_rn(w.y, v.y), __fmul_rn(w.z, v.z), __fmul_rn(w.w, v.w)};
        }
      }
      float* xp = reinterpret_cast<float*>(xs) + ((b >> 2) * XS4 + j) * 4 + (b & 3);  // plane (c, b / 4), entry j
      xp[0] = v.x;
      xp[2 * XS4 * 4] = v.y;
      xp[4 * XS4 * 4] = v.z;
      xp[6 * XS4 * 4] = v.w;
    }
  }
}

// Control wave while the rows stream: the norm scale of every sequence (sum of squares of the
// phase input from the residual reducers' G sub-slice partials, in sub-slice order — or, at layer
// 0, from the embedding rows — then src/seq.cpp:3-16's 1 / sqrtf(ss / n + 1e-5f)), and for QKV
// the RoPE (cos, sin) of every (item, sequence) of this block's reduce sub-slice.
TL_DEVICE void prep(const KDesc& d, const KGeo& g, const PStep& p, float* sscale, float2* rcs, int lane) {
  if (d.rms) {
    float s[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) s[b] = 0.f;
    if (d.gss_in) {
      // (the sums carry the residual phase's output tag, which is this phase's input tag)
      const int per = gridDim.x >> 6;  // sub-slices per lane, consecutive
      const auto r = rsrc_of(d.gss_in);
      for (int q = 0; q < per; ++q) {
        const int si = lane * per + q;
        v4u a[NB / 2];
#pragma unroll
        for (int k = 0; k < NB / 2; ++k) a[k] = ld16_sc1(r, (unsigned)(si * NB) * 8u + 16u * k);
#pragma unroll
        for (int k = 0; k < NB / 2; ++k) {
          const unsigned long long* gs = d.gss_in + (long long)si * NB + 2 * k;
          const float x0 = a[k].y == d.tag_in ? __uint_as_float(a[k].x) : gran_wait(gs, d.tag_in, p.err, true);
          const float x1 = a[k].w == d.tag_in ? __uint_as_float(a[k].z) : gran_wait(gs + 1, d.tag_in, p.err, true);
          s[2 * k] = __fadd_rn(s[2 * k], x0);
          s[2 * k + 1] = __fadd_rn(s[2 * k + 1], x1);
        }
      }
    } else {  // layer 0: the embedding rows, dim / 64 consecutive elements per lane
      const int per = p.dim >> 6;
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const float* e = p.emb + (long long)p.tok[b] * p.dim + lane * per;
        float a = 0.f;
        for (int i = 0; i < per; ++i) a = __fadd_rn(a, __fmul_rn(e[i], e[i]));
        s[b] = a;
      }
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const float tot = wave_sum_u(s[b]);
      if (lane == b) sscale[b] = __fdiv_rn(1.0f, sqrtf(__fadd_rn(__fdiv_rn(tot, (float)d.K), 1e-5f)));
    }
  }
  if (d.kind == PK_QKV && attn_fusable(p)) {  // the head's 64 q and 64 k pairs of sequence kg
    for (int j = lane; j < 128; j += 64)
      rcs[j] = p.rope[(long long)p.pos[g.kg] * (p.hs >> 1) + (j & 63)];
  } else if (d.kind == PK_QKV) {
    for (int j = lane; j < g.ns * NB; j += 64) {
      const int it = g.s0 + j / NB, b = j % NB;
      const int row = 2 * it;
      float2 cs = make_float2(1.f, 0.f);
      if (row < p.dim + p.kvd) {
        const int i = row < p.dim ? row : row - p.dim;
        cs = p.rope[(long long)p.pos[b] * (p.hs >> 1) + ((i % p.hs) >> 1)];
      }
      rcs[j] = cs;
    }
  }
}

// Every wave: this block's reduce sub-slice — (item, sequence) pairs over the block's threads —
// sums the 8 K-group partials of its rows in K-group order, scales by the norm, runs the fused
// epilogue and publishes the phase output.  The residual phases also publish the sub-slice's sum
// of squares per sequence (rows in order: one block barrier).
TL_DEVICE void reduce(const KDesc& d, const KGeo& g, const PStep& p, int l, float* xres, float* ssred,
                      const float* sscale, const float2* rcs, const uint64_t* etab, unsigned long long* cbest,
                      int wave, int lane) {
  const int t = threadIdx.x;
  const int b = t % NB;  // (PT is a multiple of NB: every pair of this thread has sequence b)
  const long long rows = (long long)d.n_items * d.rpi;
  unsigned long long best = 0;
  for (int j = t; j < g.ns * NB; j += PT) {
    const int il = j / NB, it = g.s0 + il;
    // the item's row(s): 8 partials each, all requested at once, summed in K-group order
    const unsigned long long* src = d.gpart + (long long)it * d.rpi * NB + b;
    const bool two = d.rpi == 2;
    unsigned long long x[2][NKG];
#pragma unroll
    for (int kg = 0; kg < NKG; ++kg) {
      x[0][kg] = ld8_sc1(src + kg * rows * NB);
      x[1][kg] = two ? ld8_sc1(src + kg * rows * NB + NB) : 0ull;
    }
    float v[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      float s = 0.f;
#pragma unroll
      for (int kg = 0; kg < NKG; ++kg) {
        const float e = (unsigned)(x[r][kg] >> 32) == d.tag_out || (r == 1 && !two)
                            ? __uint_as_float((unsigned)x[r][kg])
                            : gran_wait(src + kg * rows * NB + r * NB, d.tag_out, p.err, kPollLong);
        s = kg == 0 ? e : __fadd_rn(s, e);
      }
      v[r] = d.rms ? __fmul_rn(s, sscale[b]) : s;
    }
    if (d.kind == PK_CLS) {
      p.logits[(long long)b * p.V + it] = v[0];  // read by the host after the launch only
      const unsigned long long k = argmax_pack(v[0], it);
      best = k > best ? k : best;
    } else if (d.kind == PK_WO || d.kind == PK_DOWN) {
      const float xr = __fadd_rn(xres[b * kRes + il], v[0]);  // residual (src/seq.cpp:139-141, 163-166)
      xres[b * kRes + il] = xr;
      ssred[il * NB + b] = __fmul_rn(xr, xr);
      st8_sc1(d.gout + (long long)b * p.dim + it, gran(d.tag_out, xr));
      if (d.kind == PK_DOWN && l == p.L - 1) p.x[(long long)b * p.dim + it] = xr;  // final residual (state)
    } else if (d.kind == PK_UP) {
      st8_sc1(d.gout + (long long)b * p.hid + it, gran(d.tag_out, silu_mul_tab(v[0], v[1], etab)));
    } else {  // PK_QKV: RoPE (src/seq.cpp:86-101), q / k_new / v_new granules, the K/V cache row
      const int row = 2 * it;
      float a0 = v[0], a1 = v[1];
      if (row < p.dim + p.kvd) {
        const float2 cs = rcs[j];
        const float r0 = __fsub_rn(__fmul_rn(a0, cs.x), __fmul_rn(a1, cs.y));
        const float r1 = __fadd_rn(__fmul_rn(a0, cs.y), __fmul_rn(a1, cs.x));
        a0 = r0; a1 = r1;
      }
      st_gran2(rsrc_of(d.gout + (long long)b * (p.dim + 2 * p.kvd)), (unsigned)row * 8u, d.tag_out, a0, a1);
      if (row >= p.dim) {  // the cache row for later steps (this launch's attention reads the granules)
        int rk = row - p.dim;
        float* base = p.kc;
        if (rk >= p.kvd) { rk -= p.kvd; base = p.vc; }
        *reinterpret_cast<float2*>(base + (long long)b * p.L * p.S * p.kvd + ((long long)l * p.S + p.pos[b]) * p.kvd + rk) =
            make_float2(a0, a1);
      }
    }
  }
  if (d.kind == PK_CLS) {  // per wave and sequence: lanes b, b + 8, ... hold sequence b
#pragma unroll
    for (int o = 8; o < 64; o <<= 1) {
      const unsigned long long other = __shfl_xor(best, o, 64);
      best = other > best ? other : best;
    }
    if (lane < NB) cbest[wave * NB + lane] = best;  // (reduced over the waves before the final barrier)
  }
  if (d.gss_out) {
    __syncthreads();  // every pair's square in ssred
    if (t < NB) {
      float s = 0.f;
      for (int il = 0; il < g.ns; ++il) s = __fadd_rn(s, ssred[il * NB + t]);
      st8_sc1(d.gss_out + (long long)g.ssi * NB + t, gran(d.tag_out, s));
    }
  }
}

// Fused QKV reduce + attention (attn_fusable), every wave of block (h, b = kg):
//  1. sequence b's 384 rows of head h: the 8 K-group partials of each row in K-group order, the
//     norm scale, RoPE on q and k (src/seq.cpp:86-101) -> q | k | v of (b, h) in LDS; k and v also
//     to the K/V cache row at pos (for later steps);
//  2. the attention of (b, h) over keys 0..T-1 (src/seq.cpp:103-136): the keys split over the
//     block's waves, each an online softmax over 16-key chunks (cached rows from global memory,
//     row T-1 from LDS); the waves' (max, sum, output) combined in LDS in wave order;
//  3. the head's output published as granules (the Wo phase gathers them by K slice).
// Differs from the reference's order only in rounding (fp32 parity, 1e-4).
TL_DEVICE void reduce_qkv_attn(const KDesc& d, const KGeo& g, const PStep& p, int l, const float* sscale,
                               const float2* rcs, float* lds, int wave, int lane) {
  constexpr int HS = 128;
  const int t = threadIdx.x, h = g.rg, b = g.kg;
  const long long rows = (long long)d.n_items * d.rpi;
  float* qkv = lds;  // [3 HS]
  const int pb = p.pos[b];
  if (t < 3 * HS / 2) {
    const unsigned long long* src = d.gpart + ((long long)(g.i0 + t) * 2) * NB + b;
    unsigned long long x[2][NKG];
#pragma unroll
    for (int kg = 0; kg < NKG; ++kg) {
      x[0][kg] = ld8_sc1(src + kg * rows * NB);
      x[1][kg] = ld8_sc1(src + kg * rows * NB + NB);
    }
    float v[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      float sum = 0.f;
#pragma unroll
      for (int kg = 0; kg < NKG; ++kg) {
        const float e = (unsigned)(x[r][kg] >> 32) == d.tag_out
                            ? __uint_as_float((unsigned)x[r][kg])
                            : gran_wait(src + kg * rows * NB + r * NB, d.tag_out, p.err, kPollLong);
        sum = kg == 0 ? e : __fadd_rn(sum, e);
      }
      v[r] = __fmul_rn(sum, sscale[b]);
    }
    const int seg = t / (HS / 2), c = 2 * (t % (HS / 2));  // q | k | v, column pair within the head
    float a0 = v[0], a1 = v[1];
    if (seg < 2) {
      const float2 cs = rcs[t & 63];
      const float r0 = __fsub_rn(__fmul_rn(a0, cs.x), __fmul_rn(a1, cs.y));
      const float r1 = __fadd_rn(__fmul_rn(a0, cs.y), __fmul_rn(a1, cs.x));
      a0 = r0; a1 = r1;
    }
    qkv[seg * HS + c] = a0;
    qkv[seg * HS + c + 1] = a1;
    if (seg > 0)  // the cache row for later steps
      *reinterpret_cast<float2*>((seg == 1 ? p.kc : p.vc) + (long long)b * p.L * p.S * p.kvd +
                                 ((long long)l * p.S + pb) * p.kvd + h * HS + c) = make_float2(a0, a1);
  }
  __syncthreads();  // q | k | v of (b, h) in LDS
  const int T = pb + 1;
  const int w0 = (int)((long long)T * wave / PW), w1 = (int)((long long)T * (wave + 1) / PW);
  const float rs = sqrtf((float)HS);
  const float2 qv = make_float2(qkv[2 * lane], qkv[2 * lane + 1]);  // lane: columns 2 lane, 2 lane + 1
  const float* kb = p.kc + (long long)b * p.L * p.S * p.kvd + (long long)l * p.S * p.kvd + h * HS + 2 * lane;
  const float* vb = p.vc + (long long)b * p.L * p.S * p.kvd + (long long)l * p.S * p.kvd + h * HS + 2 * lane;
  const float2 kn = make_float2(qkv[HS + 2 * lane], qkv[HS + 2 * lane + 1]);
  const float2 vn = make_float2(qkv[2 * HS + 2 * lane], qkv[2 * HS + 2 * lane + 1]);
  float m = -3.402823466e+38f, lsum = 0.f;
  float2 o = make_float2(0.f, 0.f);
  constexpr int CH = 16;
  for (int t0 = w0; t0 < w1; t0 += CH) {
    const int n = w1 - t0 < CH ? w1 - t0 : CH;
    float2 kk[CH], vv[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) {  // rows past the chunk: its last row again, weighted 0
      const int tt = t0 + (i < n ? i : n - 1);
      const int tc = tt < T - 1 ? tt : 0;  // (row T-1 is this step's: LDS)
      kk[i] = *reinterpret_cast<const float2*>(kb + (long long)tc * p.kvd);
      vv[i] = *reinterpret_cast<const float2*>(vb + (long long)tc * p.kvd);
      if (tt == T - 1) { kk[i] = kn; vv[i] = vn; }
    }
    float sc[CH];
    float mc = -3.402823466e+38f;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      sc[i] = __fdiv_rn(wave_sum_u(fmaf(qv.y, kk[i].y, __fmul_rn(qv.x, kk[i].x))), rs);
      if (i < n) mc = fmaxf(mc, sc[i]);
    }
    const float mn = fmaxf(m, mc);
    const float scale = expf_libm(__fsub_rn(m, mn));  // rescale what earlier chunks summed
    lsum = __fmul_rn(lsum, scale);
    o.x = __fmul_rn(o.x, scale);
    o.y = __fmul_rn(o.y, scale);
#pragma unroll
    for (int i = 0; i < CH; ++i)
      if (i < n) {
        const float e = expf_libm(__fsub_rn(sc[i], mn));
        lsum = __fadd_rn(lsum, e);
        o.x = fmaf(e, vv[i].x, o.x);
        o.y = fmaf(e, vv[i].y, o.y);
      }
    m = mn;
  }
  // the waves' partial softmax states, combined in wave order
  float* cmb = qkv + 3 * HS;  // [PW][HS + 2]
  cmb[wave * (HS + 2) + 2 * lane] = o.x;
  cmb[wave * (HS + 2) + 2 * lane + 1] = o.y;
  if (lane == 0) {
    cmb[wave * (HS + 2) + HS] = m;
    cmb[wave * (HS + 2) + HS + 1] = lsum;
  }
  __syncthreads();
  if (wave == 0) {
    float M = -3.402823466e+38f;
    for (int w = 0; w < PW; ++w) M = fmaxf(M, cmb[w * (HS + 2) + HS]);
    float L = 0.f, ox = 0.f, oy = 0.f;
    for (int w = 0; w < PW; ++w) {
      const float lw = cmb[w * (HS + 2) + HS + 1];
      if (lw == 0.f) continue;  // (a wave without keys)
      const float f = expf_libm(__fsub_rn(cmb[w * (HS + 2) + HS], M));
      L = fmaf(lw, f, L);
      ox = fmaf(cmb[w * (HS + 2) + 2 * lane], f, ox);
      oy = fmaf(cmb[w * (HS + 2) + 2 * lane + 1], f, oy);
    }
    st_gran2(rsrc_of(d.gout + (long long)b * p.dim), (unsigned)(h * HS + 2 * lane) * 8u, d.tag_out + 1,
             __fdiv_rn(ox, L), __fdiv_rn(oy, L));
  }
}

// Sharded-counter grid barrier (the final one only), as persist_b.hip.
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

// The next GEMV phase's first slots after phase `kind` of layer l (none after QKV: the attention
// units run first, and the streaming waves issue Wo's after theirs; none after the classifier).
template <int RWD, int RWH>
TL_DEVICE void prefetch_next(const PStep& p, int kind, int l, unsigned tb, int sw, int lane, f4 (&buf)[NBUF][PLM]) {
  if (kind == PK_WO || kind == PK_UP) {
    const KDesc nd = make_desc(p, kind + 1, l, tb);
    if (kind + 1 == PK_DOWN) prefetch<RWH>(nd, geo(nd), p, sw, lane, buf);
    else prefetch<RWD>(nd, geo(nd), p, sw, lane, buf);
  } else if (kind == PK_DOWN) {
    const KDesc nd = l + 1 < p.L ? make_desc(p, PK_QKV, l + 1, tb) : make_desc(p, PK_CLS, p.L, tb);
    prefetch<RWD>(nd, geo(nd), p, sw, lane, buf);
  }
}

// Optional timeline (PStep::trace, [grid][5L+1][kTraceSlots], 100-MHz clock; tools/persist_trace.py
// --batch 8): control wave — 0 phase start, 1 slice staged, 2 norm scales / RoPE ready, 4 sweep
// barrier passed, 5 reduce done (attention: 3 units done); streaming wave 1 — 6 first slot
// consumed, 3 its last slot consumed.
#define TRACE_K(k)                                                                              \
  do {                                                                                          \
    if (p.trace && lane == 0)                                                                   \
      p.trace[((long long)blockIdx.x * nph + ph) * kTraceSlots + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)

// The phase sequence as one wave sees it (ROLE0 = the control wave).  Per GEMV phase two block
// barriers: after the staging, and after the sweep (every partial of the block published, the
// norm scales and RoPE table in LDS).
template <int HS, int RWD, int RWH, bool ROLE0>
TL_DEVICE void phases(const PStep& p, int wave, int lane, f4* xs, float* pres, unsigned* sdone, float* xres, float* ssred, float* sscale,
                      unsigned* ctr, const uint64_t* etab, float2* rcs, unsigned long long* cbest, unsigned tb) {
  const int G = gridDim.x;
  const int nph = 5 * p.L + 1;
  f4 buf[NBUF][PLM];
  const int sw = wave - 1;
  if constexpr (ROLE0) {
    // this block's residual rows (its reduce sub-slice of the Wo / W2 outputs) start as the
    // embedding rows
    const KGeo gx = geo(make_desc(p, PK_WO, 0, tb));
    for (int j = lane; j < gx.ns * NB; j += 64) {
      const int il = j / NB, b = j % NB;
      xres[b * kRes + il] = p.emb[(long long)p.tok[b] * p.dim + gx.s0 + il];
    }
    if (lane == 0) *ctr = 0u;
  } else {
    const KDesc d0 = make_desc(p, PK_QKV, 0, tb);
    prefetch<RWD>(d0, geo(d0), p, sw, lane, buf);
  }
  __syncthreads();

  for (int ph = 0; ph < nph; ++ph) {
    const int l = ph / 5;
    const int kind = ph == nph - 1 ? PK_CLS : ph % 5;
    if constexpr (ROLE0) TRACE_K(0);
    if (kind == PK_ATTN && attn_fusable(p)) continue;  // (ran inside the QKV phase's reduce)
    if (kind == PK_ATTN) {
      if constexpr (!ROLE0) {  // the slot buffers are empty here: say so, so they are not kept live
#pragma unroll
        for (int i = 0; i < NBUF; ++i)
#pragma unroll
          for (int u = 0; u < PLM; ++u) buf[i][u] = f4{0.f, 0.f, 0.f, 0.f};
      }
      {
        // one wave per (sequence, head, key-split) unit over EVERY wave of the grid: unit u runs
        // on block u % G, wave (u / G) % PW
        const KLayout k = klayout(p.dim, p.hid, p.kvd, p.V, G);
        AttnWaveParams aw = {};
        aw.a.q = p.xb; aw.a.kc = p.kc; aw.a.vc = p.vc;  // (q comes from the granules)
        aw.a.kv_b_stride = (long long)p.L * p.S * p.kvd;
        aw.a.kv_l_off = (long long)l * p.S * p.kvd;
        aw.a.pos = p.pos; aw.a.out = p.xb; aw.a.part = p.part;
        aw.a.dim = p.dim; aw.a.kv_dim = p.kvd; aw.a.head_size = HS; aw.a.n_heads = p.H;
        aw.a.kv_mul = p.kv_mul; aw.a.seq_len = p.S; aw.a.nsplit = p.NS; aw.a.min_chunk = 16;
        aw.cnt = p.tickets + (long long)l * NB * p.H; aw.B = NB; aw.NS = p.NS;
        aw.gqkv = p.gk + k.act0 + (l & 1) * k.act + k.qkv;
        aw.gout = p.gk + k.act0 + (l & 1) * k.act + k.xb;
        aw.etab = etab;
        aw.tag_in = tb + 5u * l + 1; aw.tag_out = tb + 5u * l + 2; aw.err = p.err;
        aw.poll_long = kPollLong;
        const int units = NB * p.H * p.NS;
        for (int u = blockIdx.x + G * wave; u < units; u += G * PW) attn_unit<HS, 16, true>(aw, u, lane);
        if constexpr (ROLE0) TRACE_K(3);
      }
      if constexpr (!ROLE0) {  // Wo's first slots stream in while its input is gathered
        const KDesc nd = make_desc(p, PK_WO, l, tb);
        prefetch<RWD>(nd, geo(nd), p, sw, lane, buf);
      }
      continue;
    }
    const KDesc d = make_desc(p, kind, kind == PK_CLS ? p.L : l, tb);
    const KGeo g = geo(d);
    if (kind == PK_DOWN) stage<RWH>(d, g, p, xs);
    else stage<RWD>(d, g, p, xs);
    __syncthreads();  // slice staged
    if constexpr (ROLE0) {
      TRACE_K(1);
      prep(d, g, p, sscale, rcs, lane);
      TRACE_K(2);
      if (kind == PK_DOWN) publish_partials<RWH>(d, g, pres, sdone, (unsigned)ph + 1u, lane);
      else publish_partials<RWD>(d, g, pres, sdone, (unsigned)ph + 1u, lane);
    } else {
      unsigned long long* ts = p.trace && sw == 0 ? p.trace + ((long long)blockIdx.x * nph + ph) * kTraceSlots : nullptr;
      if (kind == PK_DOWN) run_slots<RWH>(d, g, p, sw, lane, xs, buf, pres, sdone, (unsigned)ph + 1u, ctr, ts);
      else run_slots<RWD>(d, g, p, sw, lane, xs, buf, pres, sdone, (unsigned)ph + 1u, ctr, ts);
      if (ts && lane == 0) ts[3] = __builtin_amdgcn_s_memrealtime();
      // the next GEMV phase's first slots: in flight through both hand-offs and its staging
      // (after QKV: once the attention units ran)
      if (!kPrefetchAfterReduce) prefetch_next<RWD, RWH>(p, kind, l, tb, sw, lane, buf);
    }
    __syncthreads();  // the block's partials published; norm scales / RoPE table in LDS
    if constexpr (ROLE0) {
      TRACE_K(4);
      if (lane == 0) *ctr = 0u;  // the next phase's slot counter (used after its staging barrier)
    }
    if (kind == PK_QKV && attn_fusable(p)) {
      // (LDS scratch: the row partials, free from the sweep barrier until the next phase's sweep —
      // the staged slice is not: the Wo staging of the faster waves would overwrite the combine)
      reduce_qkv_attn(d, g, p, l, sscale, rcs, pres, wave, lane);
      if constexpr (!ROLE0) {  // Wo's first slots
        const KDesc nd = make_desc(p, PK_WO, l, tb);
        prefetch<RWD>(nd, geo(nd), p, sw, lane, buf);
      }
    } else {
      reduce(d, g, p, l, xres, ssred, sscale, rcs, etab, cbest, wave, lane);
      if constexpr (!ROLE0) {
        if (kPrefetchAfterReduce) prefetch_next<RWD, RWH>(p, kind, l, tb, sw, lane, buf);
      }
    }
    if constexpr (ROLE0) TRACE_K(5);
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

template <int HS, int RWD, int RWH>
__global__ void __launch_bounds__(PT) persistent_step_k_kernel(PStep p) {
  if (p.fault && blockIdx.x == 0) return;  // test hook: a missing block (every wait is bounded)
  constexpr int XSM = (RWD > RWH ? RWD : RWH) * 64;
  // dynamic LDS (kdyn_bytes): the staged K slice of every sequence (8 planes of XSM float4), then the
  // row partials
  extern __shared__ __attribute__((aligned(16))) unsigned char kdyn[];
  f4* xs = reinterpret_cast<f4*>(kdyn);
  float* pres = reinterpret_cast<float*>(xs + 8 * XSM);  // the block's row partials [rows][NB]
  __shared__ float xres[NB * kRes];                         // this block's residual rows
  __shared__ float ssred[kRes * NB];                        // their squares (sums of squares)
  __shared__ float sscale[NB];                              // the phase's norm scales
  __shared__ unsigned ctr;                                  // the dynamic slot counter
  __shared__ uint64_t etab[32];                             // the expf table
  __shared__ unsigned long long cbest[PW * NB];             // per-wave classifier winners
  __shared__ float2 rcs[kRcs * NB];                         // RoPE (cos, sin) of the QKV sub-slice
  __shared__ unsigned sdone[kMaxSlots];                     // slot s of phase ph consumed: ph + 1
  for (int i = threadIdx.x; i < kMaxSlots; i += PT) sdone[i] = 0u;  // (read after the first barrier)
  {
    constexpr uint64_t tab[32] = TL_EXPF_TABLE;
    if (threadIdx.x < 32) etab[threadIdx.x] = tab[threadIdx.x];  // (read after the first barrier)
  }
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const unsigned tb = p.seq[0] << 12;  // tag base of this launch
  if (wave == 0) {
    __builtin_amdgcn_s_setprio(2);  // the control wave's work is every other block's hand-off
    phases<HS, RWD, RWH, true>(p, wave, lane, xs, pres, sdone, xres, ssred, sscale, &ctr, etab, rcs, cbest, tb);
  } else {
    phases<HS, RWD, RWH, false>(p, wave, lane, xs, pres, sdone, xres, ssred, sscale, &ctr, etab, rcs, cbest, tb);
  }
}

// Instantiated shapes: K slices of dim = RWD wave-loads, of hidden_dim = RWH — llama2-7B (dim 4096,
// hidden 11008: 2, 6) and a 4x smaller test class (dim 2048, hidden 5632: 1, 3).
static int rw_of(int K) { return ((K / 4 + NKG - 1) / NKG + 63) / 64; }  // wave-loads per K slice

template <int HS>
static const void* kernel_hs(int rwd, int rwh) {
  if (rwd == 2 && rwh == 6) return (const void*)persistent_step_k_kernel<HS, 2, 6>;
  if (rwd == 1 && rwh == 3) return (const void*)persistent_step_k_kernel<HS, 1, 3>;
  return nullptr;
}
static const void* kernel_of(const PStep& p) {
  const int rwd = rw_of(p.dim), rwh = rw_of(p.hid);
  return p.hs == 128 ? kernel_hs<128>(rwd, rwh) : p.hs == 64 ? kernel_hs<64>(rwd, rwh) : nullptr;
}

// Rows of a row group at most, over the phases (the LDS partials).
static long long max_group_rows(const PStep& p, int ncu) {
  const long long nrg = ncu / NKG;
  long long m = 0;
  for (long long n : {2ll * ((p.dim + 2ll * p.kvd) / 2), (long long)p.dim, 2ll * p.hid, (long long)p.V}) {
    const long long r = (n * (100 + kXcdSkew) * nrg / rg_weight((int)nrg, ncu) + nrg - 1) / nrg + 2;
    m = r > m ? r : m;
  }
  return m;
}
// Dynamic LDS of an instantiation: 8 planes of XSM float4, the partials.
static size_t kdyn_bytes(const PStep& p, int ncu) {
  const int rwd = rw_of(p.dim), rwh = rw_of(p.hid);
  const size_t xsm = (size_t)(rwd > rwh ? rwd : rwh) * 64;
  return 8 * xsm * 16 + (size_t)max_group_rows(p, ncu) * NB * 4;
}

}  // namespace pk

long long persistent_k_granules(const PStep& p, int ncu) {
  return pk::klayout(p.dim, p.hid, p.kvd, p.V, ncu).total;
}

bool persistent_prepare_k(PStep& p, int ncu, const char** why) {
  using namespace pk;
  auto fail = [&](const char* m) { if (why) *why = m; return false; };
  if (p.B != NB) return fail("K-split persistent step: 8 sequences");
  if (p.q8) return fail("K-split persistent step: fp32 weights only");
  if (p.hs != 64 && p.hs != 128) return fail("head size must be 64 or 128");
  if (ncu < 64 || ncu % 64) return fail("K-split persistent step: a multiple of 64 compute units");
  if (p.dim % (4 * NKG) || p.hid % (4 * NKG)) return fail("dim and hidden_dim must be multiples of 32");
  if (!kernel_of(p)) return fail("K-split persistent step: shape not instantiated");
  if (p.L < 1) return fail("no layers");
  if (p.NS < 1 || p.NS > kMaxNS) return fail("attention splits out of range");
  if (5 * p.L + 2 >= 4096) return fail("too many layers for the phase tags");
  const int nrg = ncu / NKG;
  auto sub = [&](long long n) {  // items per reduce sub-slice, at most (the even XCDs' row groups)
    return n * (100 + kXcdSkew) / rg_weight(nrg, ncu) / NKG + 2;
  };
  if (sub(p.dim) > kRes) return fail("residual rows per block exceed the LDS slice");
  if (sub((p.dim + 2 * p.kvd) / 2) > kRcs) return fail("QKV items per block exceed the RoPE table");
  if ((long long)NB * (p.dim + 2 * p.kvd) * 8 >= (1ll << 31)) return fail("granule offsets exceed 31 bits");
  if (kdyn_bytes(p, ncu) + 16 * 1024 > 160 * 1024) return fail("K-split persistent step: LDS");
  if (max_group_rows(p, ncu) > kMaxSlots) return fail("K-split persistent step: rows per group exceed the slot flags");
  {  // more than 64 KiB of dynamic LDS (gfx950: 160 KiB per CU), once per device
    static std::mutex mu;
    static unsigned long long done = 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return fail("no current device");
    std::lock_guard<std::mutex> lock(mu);
    const unsigned long long bit = dev < 64 ? 1ull << dev : 0ull;
    if (!bit || !(done & bit)) {
      for (const void* f : {kernel_hs<64>(1, 3), kernel_hs<64>(2, 6), kernel_hs<128>(1, 3), kernel_hs<128>(2, 6)})
        if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 144 * 1024) != hipSuccess)
          return fail("cannot raise the dynamic LDS limit");
      done |= bit;
    }
  }
  int nb = 0;
  const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel_of(p), PT, kdyn_bytes(p, ncu));
  if (e != hipSuccess || nb < 1) return fail("K-split persistent kernel does not fit one block per CU");
  return true;
}

// The caller zeroes p.sync and the tickets on the same stream right before (persist.hpp).
hipError_t launch_persistent_step_k(const PStep& p, hipStream_t s, int ncu) {
  using namespace pk;
  PStep arg = p;
  void* args[] = {&arg};
  const unsigned lds = (unsigned)kdyn_bytes(p, ncu);
  if (persistent_cooperative()) return hipLaunchCooperativeKernel(kernel_of(p), dim3(ncu), dim3(PT), args, lds, s);
  return hipLaunchKernel(kernel_of(p), dim3(ncu), dim3(PT), args, lds, s);
}

}  // namespace tl
