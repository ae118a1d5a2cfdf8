// persist.hip — the whole batch-1 decode step as ONE persistent launch (fp32 or Q8_0 weights).
//
// Semantics: the reference forward (src/seq.cpp:53-168; GPU twin src/thaDNN.cpp:13-260)
// followed, in greedy mode, by sample_argmax (src/llama.cpp:275-286).
//
// Why one launch: every launch of the streaming GEMV pays a fixed ~4 us (first-byte HBM
// latency, tail, boundary; fitted over profiles/r01_gemv_sweep.json: t = bytes / ~7 TB/s +
// ~4.2 us), and the multi-launch step (forward.hip) has 5 launches per layer.
//
// Structure: grid = one 576-thread block (9 waves) per CU, all co-resident.  Phases per layer:
// QKV (+RMSNorm, RoPE, KV write) | attention | Wo + residual | W1/W3 + RMSNorm + SwiGLU |
// W2 + residual; then the classifier (+RMSNorm) and the argmax.  Per phase a block owns a
// contiguous range of items (rows, or row pairs for QKV / SwiGLU); their 8-KiB row chunks
// ("slots") are dealt round-robin to the 8 streaming waves, which keep two slots in flight
// and, as soon as they finish a phase, issue their first two slots of the NEXT phase.
// Wave 0 is the control wave: epilogues, attention units, norm-weight preloads.
//
// Hand-offs between phases carry their own readiness (MI355X_MICROARCH.md § visibility, R2
// granules): every float another block needs (x, q / k_new / v_new, the attention output,
// hb) is published as an 8-byte {value, tag} granule with one sc1 store, and the consumer
// (the next phase's staging, or an attention unit) re-reads until the tag matches.  No grid
// barrier, fence, drain or flag between phases: a phase starts as soon as ITS inputs exist.
// Tags are (launch sequence << 12) + phase + 1 — unique between consecutive launches, with
// the sequence word kept in device memory (advanced by block 0 after the final barrier), so
// granule buffers never need clearing and graph replays stay correct.  The only grid barrier
// is the final one (per-block argmax winners -> block 0).  Every wait is bounded and sets a
// sticky error word the host checks (a grid that is not co-resident cannot hang the GPU).
//
// Why hand-offs are safe to overwrite (write-after-read): a buffer is rewritten only by a
// phase whose inputs transitively required EVERY block to finish the phase that read it
// (e.g. x is rewritten by W2(l) only after every block published hb(l), i.e. finished
// staging x for W1/W3(l)); see DESIGN.md.
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <mutex>
#include "attention.hpp"
#include "gemv.hpp"
#include "gemv_q8.hpp"
#include "persist.hpp"

namespace tl {

// Register slots in flight per streaming wave: 2, with 9 waves (3 on one SIMD, <= 168 VGPRs).  4
// register slots with 8 waves (28 instead of 16 slots in flight per CU) spilled and lost 1-8%
// (DESIGN.md §3); the knob that built it is gone.
constexpr int NBUF = 2;
// Buffers refilled with the next phase's slots before its staging (the rest right after it).
// A wave's loads return in order, so its granule sweep waits behind what it prefetched: with
// int8 weights (short phases, the hand-off dominates) one buffer is best (+2.2% over two),
// with fp32 both (+1.5% over one); deeper buffering (3-4 per wave, 8 waves) lost 1-8%.
template <bool Q8>
constexpr int pfn() { return Q8 ? 1 : NBUF; }
constexpr int PW = NBUF == 2 ? 9 : 8;  // waves per block: 1 control + PW-1 streaming
constexpr int PT = PW * 64;  // threads per block
constexpr int PL = 8;        // wave-loads per slot (8 KiB per wave)
constexpr int NSW = PW - 1;  // streaming waves per block
constexpr int SB = 2;        // staged float4 per thread and batch (granule loads in flight; profiles/r04/persist_knobs_ab.txt)
constexpr int kPResidFloats = 256;  // residual-stream slice per block (LDS)
constexpr unsigned kSpinLimit = 1u << 18;
// fp32 attention units keep their keys in LDS windows (attn_unit_win).
// From kAttnHelpMinKeys keys on (fp32, batch 1; persist.hpp), the attention phase runs twice as
// many units (key splits) per head: one on each block's control wave and one on streaming wave 1,
// whose window is the staging strip (free between the QKV and Wo stagings).  One wave keeps at
// most ~63 KiB of K/V in flight (vmcnt), so at long contexts the phase is latency-bound per unit.
// The helper lives in its own kernel instantiation (HELP), launched only at such positions: its
// registers (the streaming wave's slots stay live across the unit) spill 20 B in the shared
// code, which cost the short-context step 1.2% (profiles/r04/attn_help_ab.txt).
constexpr unsigned kXcdSkew = 4;  // percent (geo); 2 / 6 / 8 measured no better (profiles/r04/xcd_skew_sweep.txt)
#define TL_HOST_DEVICE_INLINE __host__ __device__ inline

enum PKind : int { PK_QKV = 0, PK_ATTN = 1, PK_WO = 2, PK_UP = 3, PK_DOWN = 4, PK_CLS = 5 };

// One GEMV phase, described at run time (a single copy of the streaming loop serves every
// phase, so the compiler has nothing per phase to hoist and keep live across the step).
struct PDesc {
  int kind;                      // PKind (never PK_ATTN)
  int K;                         // row length (floats)
  int n_items;                   // rows, or row pairs (QKV, SwiGLU)
  int rpi;                       // rows per item
  const float* W0;               // QKV: Wq | W1 (SwiGLU) | W
  const float* W1;               // QKV: Wk | W3
  const float* W2;               // QKV: Wv
  const float *S0, *S1, *S2;     // Q8: the matching scale blocks (W* then point at int8 rows)
  const unsigned long long* gin; // input granules (null: the token's embedding row)
  unsigned tag_in;
  const float* rms;              // fused RMSNorm weight or null
  unsigned long long* gout;      // output granules (null for the classifier)
  unsigned tag_out;
};

template <bool Q8>
TL_DEVICE PDesc make_desc(const PStep& p, int kind, int l, unsigned tb) {
  PDesc d = {};
  d.kind = kind;
  const long long ll = l, dim = p.dim, hid = p.hid, kvd = p.kvd;
  const unsigned t0 = tb + 5u * l;  // tag of the phase before QKV(l), i.e. W2(l-1)
  switch (kind) {
    case PK_QKV:
      d.K = p.dim; d.n_items = (p.dim + 2 * p.kvd) / 2; d.rpi = 2;
      d.W0 = p.wq + ll * dim * dim; d.W1 = p.wk + ll * dim * kvd; d.W2 = p.wv + ll * dim * kvd;
      d.gin = l == 0 ? nullptr : p.gx; d.tag_in = t0;
      d.rms = p.rms_att + ll * dim; d.gout = p.gqkv; d.tag_out = t0 + 1;
      break;
    case PK_WO:
      d.K = p.dim; d.n_items = p.dim; d.rpi = 1;
      d.W0 = p.wo + ll * dim * dim; d.gin = p.gxb; d.tag_in = t0 + 2; d.gout = p.gx; d.tag_out = t0 + 3;
      break;
    case PK_UP:
      d.K = p.dim; d.n_items = p.hid; d.rpi = 2;
      d.W0 = p.w1 + ll * dim * hid; d.W1 = p.w3 + ll * dim * hid;
      d.gin = p.gx; d.tag_in = t0 + 3; d.rms = p.rms_ffn + ll * dim; d.gout = p.ghb; d.tag_out = t0 + 4;
      break;
    case PK_DOWN:
      d.K = p.hid; d.n_items = p.dim; d.rpi = 1;
      d.W0 = p.w2 + ll * dim * hid; d.gin = p.ghb; d.tag_in = t0 + 4; d.gout = p.gx; d.tag_out = t0 + 5;
      break;
    default:  // PK_CLS (l = L)
      d.K = p.dim; d.n_items = p.V; d.rpi = 1;
      d.W0 = p.wcls; d.gin = p.L == 0 ? nullptr : p.gx; d.tag_in = tb + 5u * p.L; d.rms = p.rms_final;
      break;
  }
  if constexpr (Q8) {
    // tensor t of layer l: int8 block at q8w[t] + l * q8ls[t], its rows x K scales after it.
    // Tensor ids and shapes are picked as scalars and every field is assigned once: per-arm
    // field stores were merged into stores through a phi of stack slots (scratch traffic).
    // QKV: wq wk wv | WO: wo | UP: w1, w3 | DOWN: w2 | CLS: the classifier pair
    const int t0 = kind == PK_QKV ? 0 : kind == PK_WO ? 3 : kind == PK_UP ? 4 : 5;
    const int t1 = kind == PK_UP ? 6 : 1;
    const long long rows0 = kind == PK_QKV || kind == PK_WO || kind == PK_DOWN ? dim : hid;
    const long long rows1 = kind == PK_UP ? hid : kvd;
    const long long K0 = kind == PK_DOWN ? hid : dim;
    const signed char* b0 = p.q8w[t0] + ll * p.q8ls[t0];
    const signed char* b1 = p.q8w[t1] + ll * p.q8ls[t1];
    const signed char* b2 = p.q8w[2] + ll * p.q8ls[2];
    const bool cls = kind == PK_CLS;
    d.W0 = reinterpret_cast<const float*>(cls ? p.qcls : b0);
    d.S0 = cls ? p.scls : reinterpret_cast<const float*>(b0 + rows0 * K0);
    d.W1 = reinterpret_cast<const float*>(b1);
    d.S1 = reinterpret_cast<const float*>(b1 + rows1 * dim);
    d.W2 = reinterpret_cast<const float*>(b2);
    d.S2 = reinterpret_cast<const float*>(b2 + kvd * dim);
  }
  return d;
}

// The GEMV phase that follows `kind` at layer l (attention has no weights).
template <bool Q8>
TL_DEVICE PDesc next_desc(const PStep& p, int kind, int l, unsigned tb) {
  if (kind == PK_QKV) return make_desc<Q8>(p, PK_WO, l, tb);
  if (kind == PK_WO) return make_desc<Q8>(p, PK_UP, l, tb);
  if (kind == PK_UP) return make_desc<Q8>(p, PK_DOWN, l, tb);
  return l + 1 < p.L ? make_desc<Q8>(p, PK_QKV, l + 1, tb) : make_desc<Q8>(p, PK_CLS, p.L, tb);
}

// Geometry of a phase for this block (all wave-uniform).  fp32: a slot is one 8-KiB chunk
// of one row (row rl of the block, floats [c*2048, c*2048 + 2048)) and has one result.
// Q8: a chunk is 4 KiB of one int8 row (one result each) and a slot is two consecutive
// chunks, which may belong to two rows (a 4096-wide int8 row is one chunk).
struct PGeo {
  int rowb;  // row length in bytes
  int nch;   // chunks (results) per row
  int i0;    // first item of this block
  int ni;    // items of this block
  int nres;  // results of this block (ni * rpi * nch)
  int nslot; // slots of this block
};

// Cumulative partition weight of blocks [0, b) (see geo).
TL_HOST_DEVICE_INLINE unsigned part_weight(unsigned b) { return (b >> 1) * 200u + (b & 1u) * (100u + kXcdSkew); }

template <bool Q8>
TL_DEVICE PGeo geo(const PDesc& d) {
  PGeo g;
  g.rowb = Q8 ? d.K : d.K * 4;
  g.nch = Q8 ? (d.K + 4095) / 4096 : (d.K + PL * 256 - 1) / (PL * 256);
  // Blocks with odd blockIdx (XCDs 1, 3, 5, 7 under round-robin dispatch) stream measurably
  // slower, so the items are dealt in proportion to 100 + kXcdSkew (even) and
  // 100 - kXcdSkew (odd); speed only, any placement is correct.  32-bit: n_items * 200 *
  // gridDim / 2 < 2^32 for every supported shape (persistent_prepare).
  const unsigned G = gridDim.x, bi = blockIdx.x, n = (unsigned)d.n_items;
  const unsigned wt = part_weight(G);
  g.i0 = (int)(n * part_weight(bi) / wt);
  g.ni = (int)(n * part_weight(bi + 1) / wt) - g.i0;
  g.nres = g.ni * d.rpi * g.nch;
  g.nslot = Q8 ? (g.nres + 1) / 2 : g.nres;
  return g;
}

// Weight row R (global row index within the phase's matrix set).
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

// Issue the 8 wave-loads of `slot` into buf: raw buffer loads over one row (the resource's
// size is what is left of the row, so loads past its end return 0 without touching memory;
// a slot past the block's end gives a zero-size resource, but callers skip those).
TL_DEVICE void load_slot(const PDesc& d, const PGeo& g, const PStep& p, int slot, int lane, f4 (&buf)[PL]) {
  const bool sv = slot < g.nslot;
  const int rl = slot / g.nch, c = slot - rl * g.nch;
  const float* row = sv ? row_ptr(d, p, g.i0 * d.rpi + rl) : d.W0;
  // one resource per 4 KiB quarter, so the per-load offsets fit the 12-bit immediate
#pragma unroll
  for (int q = 0; q < PL / 4; ++q) {
    const int off = c * (PL * 1024) + q * 4096;  // bytes into the row
    const int left = sv ? g.rowb - off : 0;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(row) + off / 4, (short)0,
                                                      left > 0 ? left : 0, 0x00020000);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      buf[q * 4 + u] =
          __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16 + u * 1024, 0, 2 /*nt*/));
  }
}

TL_DEVICE void consume_slot(const PGeo& g, int slot, int lane, const f4 (&buf)[PL], const f4* xs, float* res) {
  const int c = slot % g.nch;
  const f4* xc = xs + c * (PL * 64) + lane;
  float a = 0.f;
  // four LDS reads in flight at a time: the activations must not need a third register set
#pragma unroll
  for (int q = 0; q < PL / 4; ++q) {
#pragma unroll
    for (int u = q * 4; u < q * 4 + 4; ++u) a = dot4(buf[u], xc[u * 64], a);
    __builtin_amdgcn_sched_barrier(0);
  }
  a = wave_sum_u(a);
  if (lane == 0) res[slot] = a;
}

// Q8 row R: int8 row and its scale row (runq.c QuantizedTensor, GS = 64).  Returned by value
// and chosen by integer arithmetic: reference out-parameters behind a condition became a phi
// of stack slots (scratch traffic in the streaming loop).
struct Q8Row {
  const signed char* q;
  const float* s;
};

TL_DEVICE Q8Row q8_row_ptr(const PDesc& d, const PStep& p, int R) {
  const long long K = d.K;
  int m = 0;
  long long r = R;
  if (d.kind == PK_UP) {
    m = R & 1;
    r = R >> 1;
  } else if (d.kind == PK_QKV) {
    if (R >= p.dim + p.kvd) { m = 2; r = R - p.dim - p.kvd; }
    else if (R >= p.dim) { m = 1; r = R - p.dim; }
  }
  const unsigned long long w0 = (unsigned long long)d.W0, s0 = (unsigned long long)d.S0;
  const unsigned long long W = w0 + (m == 1 ? (unsigned long long)d.W1 - w0 : 0ull) +
                               (m == 2 ? (unsigned long long)d.W2 - w0 : 0ull);
  const unsigned long long S = s0 + (m == 1 ? (unsigned long long)d.S1 - s0 : 0ull) +
                               (m == 2 ? (unsigned long long)d.S2 - s0 : 0ull);
  return Q8Row{reinterpret_cast<const signed char*>(W) + r * K, reinterpret_cast<const float*>(S) + r * (K >> 6)};
}

// Q8 slot = chunks 2 slot and 2 slot + 1: four 1-KiB wave-loads of int8 each, plus the
// weight scale of every lane's 16 bytes (one group of 64 spans 4 lanes).  Chunks past the
// block's end, and bytes past a row's end, are zero-size resources (zeros, no traffic).
TL_DEVICE void load_slot_q8(const PDesc& d, const PGeo& g, const PStep& p, int slot, int lane, f4 (&buf)[PL],
                            float (&sc)[PL]) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int Q = 2 * slot + h;
    const bool qv = Q < g.nres;
    const int rl = Q / g.nch, c = Q - rl * g.nch;
    const Q8Row qr = q8_row_ptr(d, p, qv ? g.i0 * d.rpi + rl : 0);
    const signed char* row = qr.q;
    const float* srow = qr.s;
    const int off = c * 4096;
    const int left = qv ? g.rowb - off : 0;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<signed char*>(row) + off, (short)0,
                                                      left > 0 ? left : 0, 0x00020000);
    const int sleft = qv ? ((g.rowb - off) >> 6) * 4 : 0;
    const auto ss = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(srow) + (off >> 6), (short)0,
                                                      sleft > 0 ? sleft : 0, 0x00020000);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      buf[h * 4 + u] =
          __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16 + u * 1024, 0, 2 /*nt*/));
    // one scale per lane: lane 4q + j holds group j*16 + q of the chunk, the group whose int32
    // sum the quad reduce-scatter in consume_slot_q8 leaves in that lane
    sc[h] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ss, ((lane & 3) * 16 + (lane >> 2)) * 4, 0, 0));
  }
}

// runq.c:317-342 per chunk: per group the int32 dot (v_dot4_i32_i8 + quad reduce-scatter), then
// the group's ((float)ival * w.s) * x.s (runq.c:336), and the row value as runq's left-to-right
// chain val = fl(val + product) over the row's groups (runq.c:330-338; a tree over the groups
// moves last bits, and the int8 path re-quantises every activation — tools/probes/q8drift.c).
// A row of one chunk (K <= 4096) is chained here: the products go through the wave's LDS
// scratch `cw` and lanes 0 / 1 chain the slot's two rows into res.  Longer rows (W2) leave their
// products in pbuf (row stride pgp) and the epilogue chains them.
TL_DEVICE void consume_slot_q8(const PGeo& g, int K, int slot, int lane, const f4 (&buf)[PL], const float (&sc)[PL],
                               const signed char* xq, const float* xsc, float* res, float* pbuf, int pgp, float* cw) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int Q = 2 * slot + h;
    const int c = Q % g.nch;
    int dd[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int kb = c * 4096 + u * 1024 + lane * 16;
      const q8i4 xv = *reinterpret_cast<const q8i4*>(xq + kb);
      const q8i4 wv = __builtin_bit_cast(q8i4, buf[h * 4 + u]);
      int t = __builtin_amdgcn_sdot4(wv.x, xv.x, 0, false);
      t = __builtin_amdgcn_sdot4(wv.y, xv.y, t, false);
      t = __builtin_amdgcn_sdot4(wv.z, xv.z, t, false);
      dd[u] = __builtin_amdgcn_sdot4(wv.w, xv.w, t, false);
    }
    // quad reduce-scatter (exact int32): lane 4q + j ends with the quad's sum for u = j, i.e.
    // group j*16 + q of the chunk (3 DPP moves instead of a full quad sum per u)
    const bool b0 = lane & 1, b1 = lane & 2;
    int s0 = b0 ? dd[1] : dd[0], s1 = b0 ? dd[3] : dd[2];
    s0 += __builtin_amdgcn_mov_dpp(b0 ? dd[0] : dd[1], 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    s1 += __builtin_amdgcn_mov_dpp(b0 ? dd[2] : dd[3], 0xB1, 0xF, 0xF, false);
    int gs = b1 ? s1 : s0;
    gs += __builtin_amdgcn_mov_dpp(b1 ? s0 : s1, 0x4E, 0xF, 0xF, false);       // quad_perm [2,3,0,1]
    const int gi = (lane & 3) * 16 + (lane >> 2);  // group within the chunk
    const float a = __fmul_rn(__fmul_rn((float)gs, sc[h]), xsc[c * 64 + gi]);  // runq.c:336
    if (Q < g.nres) {
      if (g.nch == 1) cw[h * 68 + gi] = a;
      else pbuf[(Q / g.nch) * pgp + c * 64 + gi] = a;
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  if (g.nch == 1) {
    wave_lds_fence();
    if (lane < 2 && 2 * slot + lane < g.nres) {
      res[2 * slot + lane] = chain_f4(reinterpret_cast<const f4*>(cw + lane * 68), K >> 8, 0.f);
    }
    wave_lds_fence();  // the scratch is rewritten by the next slot
  }
}

// Stream this wave's slots (sw, sw + NSW, ...), sw = streaming-wave index; the NBUF buffers
// already hold the first NBUF.  Every path loads the buffers in the same places, so the
// register allocator keeps one set of NBUF register buffers for the whole step.
template <bool Q8>
TL_DEVICE void load_any(const PDesc& d, const PGeo& g, const PStep& p, int slot, int lane, f4 (&buf)[PL],
                        float (&sc)[PL]) {
  if constexpr (Q8) load_slot_q8(d, g, p, slot, lane, buf, sc);
  else load_slot(d, g, p, slot, lane, buf);
}

// int8 chain buffers of one wave: the products of rows longer than one chunk (pbuf, row stride
// pgp) and the wave's own 2 x 68-float scratch (cw)
struct PChain {
  float* pbuf;
  int pgp;
  float* cw;
};

template <bool Q8>
TL_DEVICE void consume_any(const PGeo& g, int K, int slot, int lane, const f4 (&buf)[PL], const float (&sc)[PL],
                           const f4* xs, const signed char* xq, const float* xsc, float* res, const PChain& pc) {
  if constexpr (Q8) consume_slot_q8(g, K, slot, lane, buf, sc, xq, xsc, res, pc.pbuf, pc.pgp, pc.cw);
  else consume_slot(g, slot, lane, buf, xs, res);
}

// Slot indices past the first two per wave are dealt dynamically from a block-wide LDS
// counter (reset by the control wave between phases): the waves of a block stream at
// different rates (measured: the slowest wave of a block finished its static round-robin
// share up to ~25% after the fastest), and a phase ends with its slowest wave.  Slots a wave
// holds only ever increase (A's next slot is taken after B's), so the first invalid slot
// in A ends the wave's phase.  Refills past the phase's end are skipped rather than issued
// as zero-size loads: at the phase end those issues sat on the path to the epilogue (+6-8%
// int8), and the compiler's vmcnt bookkeeping stays tight enough over the two branches.
TL_DEVICE int take_slot(unsigned* ctr, int lane) {
  unsigned v = 0;
  if (lane == 0) v = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  return NBUF * NSW + (int)__builtin_amdgcn_readlane(v, 0);
}

template <bool Q8>
TL_DEVICE void run_gemv(const PDesc& d, const PGeo& g, const PStep& p, int sw, int lane, const f4* xs,
                        const signed char* xq, const float* xsc, float* res, f4 (&buf)[NBUF][PL],
                        float (&sc)[NBUF][PL], unsigned* ctr, unsigned long long* ts, const PChain& pc) {
  int sl[NBUF];  // the slots the buffers hold (the phase's prefetch: sw, sw + NSW, ...)
#pragma unroll
  for (int i = 0; i < NBUF; ++i) sl[i] = sw + i * NSW;
  bool first = true;
  // sched_barrier: keep each refill behind the slot's last use (no extra register set)
  while (sl[0] < g.nslot) {
#pragma unroll
    for (int i = 0; i < NBUF; ++i) {
      if (sl[i] < g.nslot) consume_any<Q8>(g, d.K, sl[i], lane, buf[i], sc[i], xs, xq, xsc, res, pc);
      if (i == 0 && ts && first && lane == 0) *ts = __builtin_amdgcn_s_memrealtime();  // first slot landed
      first = false;
      __builtin_amdgcn_sched_barrier(0);
      sl[i] = take_slot(ctr, lane);
      if (sl[i] < g.nslot) load_any<Q8>(d, g, p, sl[i], lane, buf[i], sc[i]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// The reference's products x[j] * x[j] (runq.c:286) of float4 j into the seqsum layout.
TL_DEVICE void put_squares(float* sqa, int ch, int j, f4 v) {
  const int e = 4 * j;  // ch % 4 == 0: the four land in one chunk
  float* d = sqa + seqsum_index(e, ch);
  d[0] = __fmul_rn(v.x, v.x); d[1] = __fmul_rn(v.y, v.y); d[2] = __fmul_rn(v.z, v.z); d[3] = __fmul_rn(v.w, v.w);
}

// Granule sweep of the phase input into the LDS strip by threads t, t + T, ...: batches of NB
// float4 (2*NB loads in flight per thread), then re-poll what was late.  sq: sum of squares.
// UNC: unconditional (clamped) loads, so loads issued by `mid` after them keep the compiler's
// vmcnt waits exact (int8, where mid issues slots); otherwise only threads with input load.
template <int NB, bool UNC, class F>
TL_DEVICE void gather(__amdgpu_buffer_rsrc_t r, unsigned tag, int n4, int pad4, int t, int T, f4* xs, float& sq,
                      unsigned* err, bool lng, float* sqa, int sqch, F&& mid) {
  for (int k0 = 0; k0 * T < pad4; k0 += NB) {
    v4u a[NB], b[NB];
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const int j = t + (k0 + k) * T, jc = j < n4 ? j : n4 - 1;
      if (UNC || j < n4) {
        a[k] = ld16_sc1(r, (unsigned)jc * 32u);
        b[k] = ld16_sc1(r, (unsigned)jc * 32u + 16u);
      }
    }
    if ((k0 + NB) * T >= pad4) mid();  // after the sweep's last loads
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const int j = t + (k0 + k) * T;
      if (j < pad4) {
        f4 v = f4{0.f, 0.f, 0.f, 0.f};
        if (j < n4)
          v = gran4_ok(a[k], b[k], tag) ? gran4_val(a[k], b[k]) : gran_wait4(r, (unsigned)j * 32u, tag, err, lng);
        sq = fmaf(v.x, v.x, sq); sq = fmaf(v.y, v.y, sq); sq = fmaf(v.z, v.z, sq); sq = fmaf(v.w, v.w, sq);
        xs[j] = v;
        if (sqa && j < n4) put_squares(sqa, sqch, j, v);
      }
    }
  }
}

// int8 phase without a norm (W2: the SwiGLU output): the sweep quantises as it goes.  With
// j = t + k PT (PT a multiple of 64) the 16 lanes of a row hold the 16 float4s of one group of
// 64, so the group max is a DPP row max; each lane writes its 4 codes and the row's first
// lane the scale (runq.c:145-171, the arithmetic of q8_pack).  n4 % 16 == 0; groups past K
// up to nch whole chunks get scale 0 (the products there are 0 * 0).
template <int NB, class F>
TL_DEVICE void gather_q8(__amdgpu_buffer_rsrc_t r, unsigned tag, int n4, int nch, signed char* xq, float* xsc,
                         unsigned* err, bool lng, F&& mid) {
  const int t = threadIdx.x, lane = t & 63;
  for (int k0 = 0; k0 * PT < n4; k0 += NB) {
    v4u a[NB], b[NB];
#pragma unroll
    for (int k = 0; k < NB; ++k) {  // unconditional (clamped) loads: exact vmcnt bookkeeping
      const int j = t + (k0 + k) * PT, jc = j < n4 ? j : n4 - 1;
      a[k] = ld16_sc1(r, (unsigned)jc * 32u);
      b[k] = ld16_sc1(r, (unsigned)jc * 32u + 16u);
    }
    if ((k0 + NB) * PT >= n4) mid();  // after the sweep's last loads
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const int j = t + (k0 + k) * PT;
      if (j - lane >= n4) continue;  // wave-uniform: the whole wave is past the input
      f4 v = f4{0.f, 0.f, 0.f, 0.f};
      if (j < n4) v = gran4_ok(a[k], b[k], tag) ? gran4_val(a[k], b[k]) : gran_wait4(r, (unsigned)j * 32u, tag, err, lng);
      const float m = row16_max(fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
      const float scale = __fdiv_rn(m, 127.0f);
      int c0, c1, c2, c3;
      if (q8_fast_scale(scale)) {
        const float rc = __fdiv_rn(1.0f, scale);
        c0 = q8_code_fast(v.x, scale, rc); c1 = q8_code_fast(v.y, scale, rc);
        c2 = q8_code_fast(v.z, scale, rc); c3 = q8_code_fast(v.w, scale, rc);
      } else {
        c0 = q8_round(__fdiv_rn(v.x, scale)); c1 = q8_round(__fdiv_rn(v.y, scale));
        c2 = q8_round(__fdiv_rn(v.z, scale)); c3 = q8_round(__fdiv_rn(v.w, scale));
      }
      if (j < n4) {
        *reinterpret_cast<int*>(xq + 4 * j) = (c0 & 0xFF) | ((c1 & 0xFF) << 8) | ((c2 & 0xFF) << 16) | ((c3 & 0xFF) << 24);
        if ((lane & 15) == 0) xsc[j >> 4] = scale;
      }
    }
  }
  for (int gi = n4 / 16 + t; gi < nch * 64; gi += PT) xsc[gi] = 0.f;
}

// Every wave stages the phase input into LDS (zero-padded to whole chunks), RMSNorm'd when
// the phase has a norm (its weights were preloaded into LDS `rmsw` by the control wave).
// The input is the previous phase's granules (all issued at once, then re-polled until
// their tags match), or — QKV at layer 0, or the classifier of a model without layers —
// the token's embedding row (weights: plain loads).  Ends with a workgroup barrier.
template <bool Q8, bool ROLE0, class F>
TL_DEVICE void stage(const PDesc& d, const PGeo& g, const PStep& p, f4* xs, signed char* xq, float* xsc,
                     const float* rmsw, float* red, float* sqa, int wave, int lane, unsigned long long* ts, F&& mid) {
  const int n4 = d.K >> 2, pad4 = Q8 ? n4 : g.nch * PL * 64;
#ifdef PERSIST_DIAG_NO_GATHER
  // traffic-attribution build only (tools/build_variant.sh; profiles/r06/handoff_traffic_bisect.txt):
  // the Wo and W2 phases do not gather their input (xb, hb) — wrong results; what the rest of the
  // step reads is the point.  The normed phases (QKV, W1/W3) still gather x from every block, so
  // every hand-off buffer is still rewritten only after all its readers are done.
  if (d.gin && !d.rms) {
    mid();
    __syncthreads();
    return;
  }
#endif
  if (Q8 && !d.rms && d.gin) {  // Wo, W2: quantised while it is gathered
    gather_q8<SB>(rsrc_of(d.gin), d.tag_in, n4, g.nch, xq, xsc, p.err, p.poll_long != 0, mid);
    if (ts && lane == 0) ts[wave == 0 ? 8 : 10] = __builtin_amdgcn_s_memrealtime();  // input gathered
    if (ts && lane == 0 && wave == 0) ts[9] = __builtin_amdgcn_s_memrealtime();
    __syncthreads();
    return;
  }
  float sq = 0.f;
  // int8: the norm's sum of squares is runq's left-to-right chain (seqsum.hpp), so the squares
  // go to the seqsum layout as they arrive
  float* sqd = Q8 && d.rms ? sqa : nullptr;
  const int sqch = d.K >> 6;  // seqsum_ch(K) for K % 256 == 0
  if (!d.gin) {
    mid();
    const f4* emb = reinterpret_cast<const f4*>(p.emb + (long long)p.tok[0] * p.dim);
    for (int j = threadIdx.x; j < pad4; j += PT) {
      const f4 v = j < n4 ? emb[j] : f4{0.f, 0.f, 0.f, 0.f};
      sq = fmaf(v.x, v.x, sq); sq = fmaf(v.y, v.y, sq); sq = fmaf(v.z, v.z, sq); sq = fmaf(v.w, v.w, sq);
      xs[j] = v;
      if (sqd && j < n4) put_squares(sqd, sqch, j, v);
    }
  } else {
    // every wave sweeps (the control wave alone, 16-24 loads in flight, was 1.4x slower per
    // step: the sweep is bound by loads in flight, not by the streaming waves' queued slots)
    gather<SB, Q8>(rsrc_of(d.gin), d.tag_in, n4, pad4, threadIdx.x, PT, xs, sq, p.err, p.poll_long != 0, sqd, sqch, mid);
  }
  if (ts && lane == 0) ts[wave == 0 ? 8 : 10] = __builtin_amdgcn_s_memrealtime();  // input gathered
  float ss = 1.f;
  if (d.rms) {
    // reference rmsnorm (src/seq.cpp:3-16, runq.c:282-295): ss = 1/sqrtf(sum/size + 1e-5f).
    // fp32: the block sum in a fixed order (waves 0..PW-1), so every block gets the same ss;
    // int8: the sum is runq's own chain, taken by wave 0 (seqsum.hpp), bit for bit
    float t;
    if constexpr (Q8) {
      __syncthreads();  // the squares are in sqa
      if constexpr (ROLE0) {
        int rounds = 0;  // (a register: an array here lived in scratch, zeroed on every norm)
        const float v = d.K <= 4096 ? seqsum_reg_core<false>(sqa, d.K, lane, rounds, nullptr) : wave_seqsum(sqa, d.K, lane);
        if (ts && lane == 0 && d.K <= 4096) ts[13] = (unsigned long long)rounds;  // (diagnostics: repair rounds)
        if (lane == 0) red[0] = v;
      }
      __syncthreads();
      t = red[0];
    } else {
      sq = wave_sum_u(sq);
      if (lane == 0) red[wave] = sq;
      __syncthreads();
      t = red[0];
#pragma unroll
      for (int w = 1; w < PW; ++w) t += red[w];
    }
    ss = __fdiv_rn(1.0f, sqrtf(__fadd_rn(__fdiv_rn(t, (float)d.K), 1e-5f)));
    if constexpr (!Q8) {
      const f4* w4 = reinterpret_cast<const f4*>(rmsw);
      for (int j = threadIdx.x; j < n4; j += PT) xs[j] = rms_apply(xs[j], w4[j], ss);
    }
  }
  if (ts && lane == 0 && wave == 0) {
    ts[9] = __builtin_amdgcn_s_memrealtime();  // normalised
    ts[11] = ((unsigned long long)__float_as_uint(ss) << 32) | (d.rms ? __float_as_uint(red[0]) : 0u);  // diagnostics
  }
  if constexpr (Q8) {
    // runq.c:145-171 quantize over the padded strip (the RMSNorm applied on the fly, same
    // arithmetic as the fp32 strip): 8 consecutive threads per group of 64, 8 values each;
    // scale = max|x| / 127, q = round(x / scale)
    if (!d.rms) __syncthreads();  // (with a norm, the sum's barrier already ordered the sweep)
    const f4* w4 = reinterpret_cast<const f4*>(rmsw);
    const int nsl = g.nch * 512;
    for (int sl = threadIdx.x; sl < nsl; sl += PT) {
      f4 v[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int j = sl * 2 + u;
        v[u] = j < n4 ? (d.rms ? rms_apply(xs[j], w4[j], ss) : xs[j]) : f4{0.f, 0.f, 0.f, 0.f};
      }
      float m = fmaxf(fmaxf(fmaxf(fabsf(v[0].x), fabsf(v[0].y)), fmaxf(fabsf(v[0].z), fabsf(v[0].w))),
                      fmaxf(fmaxf(fabsf(v[1].x), fabsf(v[1].y)), fmaxf(fabsf(v[1].z), fabsf(v[1].w))));
      m = fmaxf(m, dpp_f<0xB1>(m));
      m = fmaxf(m, dpp_f<0x4E>(m));
      m = fmaxf(m, dpp_f<0x141>(m));  // row_half_mirror: the two quads of the group
      const float scale = __fdiv_rn(m, 127.0f);
      *reinterpret_cast<q8i2*>(xq + sl * 8) = q8_pack8(v, scale);
      if ((sl & 7) == 0) xsc[sl >> 3] = scale;
    }
  }
  __syncthreads();
}

// Control wave, while the others stream: the next norm's weights into LDS (constants; only
// the staging reads rmsw, and it has finished).
TL_DEVICE void preload_rms(const float* w, int dim, float* rmsw, int lane) {
#ifdef PERSIST_DIAG_NO_RMSW  // traffic-attribution build only (as PERSIST_DIAG_NO_GATHER): no preload
  return;
#endif
  const f4* s4 = reinterpret_cast<const f4*>(w);
  f4* d4 = reinterpret_cast<f4*>(rmsw);
  for (int j = lane; j < (dim >> 2); j += 64) d4[j] = s4[j];
}

// (cos, sin) of the RoPE pair at QKV row `row` (< dim + kv_dim) for this step's position.
TL_DEVICE float2 rope_cs(const PStep& p, int pb, int row) {
  const int i = row < p.dim ? row : row - p.dim;
  return p.rope[(long long)pb * (p.hs >> 1) + ((i % p.hs) >> 1)];
}

// Control wave: row values from the LDS row-chunk sums, fused epilogue, granule stores.
// cs0: the RoPE (cos, sin) of this lane's first QKV item, loaded while the slots streamed
// (a table read at the epilogue put one L2 round trip on every layer's critical path).
// xres: this block's slice of the residual stream x (rows i0.. of the dim-row phases, the
// same slice for Wo and W2), kept in LDS so the residual add never re-reads x.
// int8: the body with the phase kind read at run time (the per-kind instantiations below cost the
// int8 step 0.6-0.8%: profiles/r04/epilogue_kind_ab.txt).
TL_DEVICE void epilogue_rt(const PDesc& d, const PGeo& g, const PStep& p, const float* res, float* xres, int lane,
                        int l, int pb, float2 cs0, const float* pbuf, const uint64_t* etab) {
  unsigned long long best = 0;
  for (int it = lane; it < g.ni; it += 64) {
    float v[2] = {0.f, 0.f};
    for (int r = 0; r < d.rpi; ++r) {
      float s;
      if (p.q8 && g.nch > 1) {
        // int8 rows longer than a chunk: runq's chain over the row's group products (runq.c:330-338)
        s = chain_f4<24>(reinterpret_cast<const f4*>(pbuf + (it * d.rpi + r) * p.pgp), d.K >> 8, 0.f);
      } else {
        const float* rr = res + (it * d.rpi + r) * g.nch;
        s = rr[0];
        for (int c = 1; c < g.nch; ++c) s = __fadd_rn(s, rr[c]);
      }
      v[r] = s;
    }
    if (p.trace && it == 0)  // (diagnostics: the first item's row values are computed)
      p.trace[((long long)blockIdx.x * (5 * p.L + 1) + (d.kind == PK_CLS ? 5 * p.L : 5 * l + d.kind)) * kTraceSlots + 12] =
          __builtin_amdgcn_s_memrealtime();
    const int item = g.i0 + it;
    if (d.kind == PK_CLS) {
      p.logits[item] = v[0];  // read by the host after the launch only
      const unsigned long long k = argmax_pack(v[0], item);
      best = k > best ? k : best;
    } else if (d.kind == PK_WO || d.kind == PK_DOWN) {
      xres[it] = __fadd_rn(xres[it], v[0]);  // residual (src/seq.cpp:139-141, 163-166)
      st8_sc1(d.gout + item, gran(d.tag_out, xres[it]));
      if (d.kind == PK_DOWN && l == p.L - 1) p.x[item] = xres[it];  // final residual stream (state)
    } else if (d.kind == PK_UP) {
      st8_sc1(d.gout + item, gran(d.tag_out, silu_mul_tab(v[0], v[1], etab)));
    } else {  // PK_QKV: RoPE (src/seq.cpp:86-101), q / k_new / v_new granules, KV-cache row
      const int row = 2 * item;
      float a0 = v[0], a1 = v[1];
      if (row < p.dim + p.kvd) {
        const float2 cs = it == lane ? cs0 : rope_cs(p, pb, row);
        const float r0 = __fsub_rn(__fmul_rn(a0, cs.x), __fmul_rn(a1, cs.y));
        const float r1 = __fadd_rn(__fmul_rn(a0, cs.y), __fmul_rn(a1, cs.x));
        a0 = r0; a1 = r1;
      }
      st_gran2(rsrc_of(d.gout), (unsigned)row * 8u, d.tag_out, a0, a1);
      if (row >= p.dim) {  // the cache row for later steps (this launch reads the granules)
        int rk = row - p.dim;
        float* base = p.kc;
        if (rk >= p.kvd) { rk -= p.kvd; base = p.vc; }
        *reinterpret_cast<float2*>(base + ((long long)l * p.S + pb) * p.kvd + rk) = make_float2(a0, a1);
      }
    }
  }
  if (d.kind == PK_CLS) {
    for (int o = 32; o > 0; o >>= 1) {
      const unsigned long long other = __shfl_xor(best, o, 64);
      best = other > best ? other : best;
    }
    if (lane == 0) st8_sc1(p.bmax + blockIdx.x, best);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drained before the final arrival
  }
}

// fp32: one instantiation per phase kind (KIND): the body with the kind read at run time was
// ~200 scalar-heavy instructions (branches, spilled SGPRs) before the first row value, on every
// hand-off's critical path (epilogues 2.9 / 1.4 / 1.4 / 1.3 -> 2.1 / 0.4 / 0.7 / 0.6 us for QKV /
// Wo / W1-W3 / W2; 7B +1.0-1.4%, 110M +1.9%, profiles/r04/epilogue_kind_ab.txt).
template <int KIND>
TL_DEVICE void epilogue_k(const PDesc& d, const PGeo& g, const PStep& p, const float* res, float* xres, int lane,
                          int l, int pb, float2 cs0, const uint64_t* etab) {
  constexpr int kind = KIND, rpi = KIND == PK_QKV || KIND == PK_UP ? 2 : 1;
  unsigned long long best = 0;
  for (int it = lane; it < g.ni; it += 64) {
    float v[2] = {0.f, 0.f};
#pragma unroll
    for (int r = 0; r < rpi; ++r) {
      float s;
      {
        const float* rr = res + (it * rpi + r) * g.nch;
        s = rr[0];
        for (int c = 1; c < g.nch; ++c) s = __fadd_rn(s, rr[c]);
      }
      v[r] = s;
    }
    if (p.trace && it == 0)  // (diagnostics: the first item's row values are computed)
      p.trace[((long long)blockIdx.x * (5 * p.L + 1) + (kind == PK_CLS ? 5 * p.L : 5 * l + kind)) * kTraceSlots + 12] =
          __builtin_amdgcn_s_memrealtime();
    const int item = g.i0 + it;
    if (kind == PK_CLS) {
      p.logits[item] = v[0];  // read by the host after the launch only
      const unsigned long long k = argmax_pack(v[0], item);
      best = k > best ? k : best;
    } else if (kind == PK_WO || kind == PK_DOWN) {
      xres[it] = __fadd_rn(xres[it], v[0]);  // residual (src/seq.cpp:139-141, 163-166)
      st8_sc1(d.gout + item, gran(d.tag_out, xres[it]));
      if (kind == PK_DOWN && l == p.L - 1) p.x[item] = xres[it];  // final residual stream (state)
    } else if (kind == PK_UP) {
      st8_sc1(d.gout + item, gran(d.tag_out, silu_mul_tab(v[0], v[1], etab)));
    } else {  // PK_QKV: RoPE (src/seq.cpp:86-101), q / k_new / v_new granules, KV-cache row
      const int row = 2 * item;
      float a0 = v[0], a1 = v[1];
      if (row < p.dim + p.kvd) {
        const float2 cs = it == lane ? cs0 : rope_cs(p, pb, row);
        const float r0 = __fsub_rn(__fmul_rn(a0, cs.x), __fmul_rn(a1, cs.y));
        const float r1 = __fadd_rn(__fmul_rn(a0, cs.y), __fmul_rn(a1, cs.x));
        a0 = r0; a1 = r1;
      }
      st_gran2(rsrc_of(d.gout), (unsigned)row * 8u, d.tag_out, a0, a1);
      if (row >= p.dim) {  // the cache row for later steps (this launch reads the granules)
        int rk = row - p.dim;
        float* base = p.kc;
        if (rk >= p.kvd) { rk -= p.kvd; base = p.vc; }
        *reinterpret_cast<float2*>(base + ((long long)l * p.S + pb) * p.kvd + rk) = make_float2(a0, a1);
      }
    }
  }
  if (kind == PK_CLS) {
    for (int o = 32; o > 0; o >>= 1) {
      const unsigned long long other = __shfl_xor(best, o, 64);
      best = other > best ? other : best;
    }
    if (lane == 0) st8_sc1(p.bmax + blockIdx.x, best);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drained before the final arrival
  }
}

template <bool Q8>
TL_DEVICE void epilogue(const PDesc& d, const PGeo& g, const PStep& p, const float* res, float* xres, int lane,
                        int l, int pb, float2 cs0, const float* pbuf, const uint64_t* etab) {
  if constexpr (Q8) {
    epilogue_rt(d, g, p, res, xres, lane, l, pb, cs0, pbuf, etab);
    return;
  }
  switch (d.kind) {
    case PK_QKV: epilogue_k<PK_QKV>(d, g, p, res, xres, lane, l, pb, cs0, etab); break;
    case PK_WO: epilogue_k<PK_WO>(d, g, p, res, xres, lane, l, pb, cs0, etab); break;
    case PK_UP: epilogue_k<PK_UP>(d, g, p, res, xres, lane, l, pb, cs0, etab); break;
    case PK_DOWN: epilogue_k<PK_DOWN>(d, g, p, res, xres, lane, l, pb, cs0, etab); break;
    default: epilogue_k<PK_CLS>(d, g, p, res, xres, lane, l, pb, cs0, etab); break;
  }
}

// Sharded-counter grid barrier (the final one only).  Callers have drained every storing
// wave.  One lane per block adds to its shard; lanes 0..7 of wave 0 poll the eight shards.
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

// Optional timeline (PStep::trace, [grid][phase][kTraceSlots]): the control wave of every block
// stamps the 100-MHz real-time clock at phase start, input staged, all slots reduced, epilogue
// issued (0-3), input gathered and normalised (8-9); streaming wave 0 at input staged, first
// slot consumed, last slot consumed, next phase's slots issued (4-7), input gathered (10).
#define TRACE(k)                                                                                \
  do {                                                                                          \
    if (p.trace && lane == 0)                                                                   \
      p.trace[((long long)blockIdx.x * nph + ph) * kTraceSlots + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)

// The phase sequence as seen by one wave.  ROLE0 = the control wave (epilogues, attention,
// norm preloads); the other waves stream.  Both execute the same workgroup barriers.
template <int HS, bool ROLE0, bool Q8, bool HELP>
TL_DEVICE void phases(const PStep& p, int wave, int lane, float* res, float* xres, float* red,
                      float* rmsw, f4* xs, signed char* xq, float* xsc, float* sqa, float* scr, float* cwb,
                      const uint64_t* etab, unsigned tb, float* awin) {
  const int G = gridDim.x;
  const int nph = 5 * p.L + 1;
  unsigned* ctr = reinterpret_cast<unsigned*>(red + 15);  // dynamic slot counter (red[0..PW) is the norm sum)
  if constexpr (ROLE0) {
    // this block's slice of the residual stream starts as the token's embedding row
    const PGeo gx = geo<Q8>(make_desc<Q8>(p, PK_WO, 0, tb));
    const float* er = p.emb + (long long)p.tok[0] * p.dim + gx.i0;
    for (int it = lane; it < gx.ni; it += 64) xres[it] = er[it];
    preload_rms(p.L > 0 ? p.rms_att : p.rms_final, p.dim, rmsw, lane);
    if (lane == 0) *ctr = 0u;
    // the step's position, read once: the QKV epilogues' cache-row address and RoPE rows (a
    // global read there put a scalar-cache miss behind every layer's granule publish)
    const int pos_b = p.pos[0];
    __syncthreads();  // first norm weights preloaded
    // the attention units of layer l (fp32 at long contexts: twice the key splits, the helper)
    const bool help = !Q8 && HELP && p.attn_help && p.pos[0] + 1 >= kAttnHelpMinKeys;
    auto attn_params = [&](int l) {
      AttnWaveParams aw = {};
      aw.a.q = p.xb; aw.a.kc = p.kc; aw.a.vc = p.vc;  // (q comes from the granules)
      aw.a.kv_b_stride = (long long)p.L * p.S * p.kvd;
      aw.a.kv_l_off = (long long)l * p.S * p.kvd;
      aw.a.pos = p.pos; aw.a.out = p.xb; aw.a.part = p.part;
      aw.a.dim = p.dim; aw.a.kv_dim = p.kvd; aw.a.head_size = HS; aw.a.n_heads = p.H;
      aw.a.kv_mul = p.kv_mul; aw.a.seq_len = p.S; aw.a.nsplit = p.NS; aw.a.min_chunk = 16;
      aw.cnt = p.tickets + (long long)l * p.H; aw.B = 1; aw.NS = p.NS;
      if (help) aw.NS = aw.a.nsplit = 2 * p.NS < kMaxNS ? 2 * p.NS : kMaxNS;
      aw.gqkv = p.gqkv; aw.gout = p.gxb;
      aw.gsc = p.gsc; aw.etab = etab;
      aw.tag_in = tb + 5u * l + 1; aw.tag_out = tb + 5u * l + 2; aw.err = p.err;
      aw.poll_long = p.poll_long;
      return aw;
    };
    bool pre = false;  // this block's attention unit of the coming phase has its K/V rows requested
    for (int ph = 0; ph < nph; ++ph) {
      const int l = ph / 5;
      const int kind = ph == nph - 1 ? PK_CLS : ph % 5;
      TRACE(0);
      if (kind == PK_ATTN) {
        // one wave per (head, key-split) unit: unit u on block u % G
        AttnWaveParams aw = attn_params(l);
        aw.ts = p.trace ? p.trace + ((long long)blockIdx.x * nph + ph) * kTraceSlots + 8 : nullptr;
        if constexpr (Q8) {
          // int8: runq's attention bit for bit, each head split over p.ang units (attention.hpp
          // attn_unit_split).  K / V go through the fp32 staging strip xs: nothing reads it before
          // the next normed staging (FFN-up), which this block starts after this unit.
          for (int u = blockIdx.x; u < p.H * p.ang; u += G)
            attn_unit_split<HS>(aw, u / p.ang, u % p.ang, p.ang, scr, reinterpret_cast<float*>(xs), p.pad_floats, lane);
        } else {
          // long contexts: twice the splits, the second unit of each block on streaming wave 1
          const int units = p.H * aw.NS;
          for (int u = blockIdx.x; u < units; u += (help ? 2 : 1) * G) attn_unit_win<HS>(aw, u, awin, lane, pre);
          pre = false;
          if (help) __syncthreads();  // the helper's window (the strip) is free for the Wo staging
        }
        TRACE(3);
        continue;
      }
      const PDesc d = make_desc<Q8>(p, kind, l, tb);
      const PGeo g = geo<Q8>(d);
      stage<Q8, true>(d, g, p, xs, xq, xsc, rmsw, red, sqa, wave, lane,
                      p.trace ? p.trace + ((long long)blockIdx.x * nph + ph) * kTraceSlots : nullptr, [] {});
      TRACE(1);
      if constexpr (!Q8) {
        // the coming attention unit's cached K/V rows, ahead of this block's next-phase prefetch
        if (kind == PK_QKV && !help && p.H * p.NS <= G) pre = attn_win_preissue<HS>(attn_params(l), blockIdx.x, awin, lane);
      }
      float2 cs0 = make_float2(1.f, 0.f);
      if (kind == PK_QKV) {
        preload_rms(p.rms_ffn + (long long)l * p.dim, p.dim, rmsw, lane);
        if (lane < g.ni && 2 * (g.i0 + lane) < p.dim + p.kvd) cs0 = rope_cs(p, pos_b, 2 * (g.i0 + lane));
      }
      if (kind == PK_UP) preload_rms(l + 1 < p.L ? p.rms_att + (long long)(l + 1) * p.dim : p.rms_final, p.dim, rmsw, lane);
      __syncthreads();  // every slot reduced into res
      if (lane == 0) *ctr = 0u;  // next GEMV phase's slot counter (used after its staging barrier)
      TRACE(2);
      epilogue<Q8>(d, g, p, res, xres, lane, l, pos_b, cs0, scr, etab);
      TRACE(3);
    }
  } else {
    const int sw = wave - 1;
    f4 buf[NBUF][PL];
    float sc[NBUF][PL];  // Q8 weight scales (unused for fp32)
    __syncthreads();  // first norm weights preloaded
    {
      const PDesc d0 = make_desc<Q8>(p, p.L > 0 ? PK_QKV : PK_CLS, p.L > 0 ? 0 : p.L, tb);
      const PGeo g0 = geo<Q8>(d0);
#pragma unroll
      for (int i = 0; i < NBUF; ++i)
        if (sw + i * NSW < g0.nslot) load_any<Q8>(d0, g0, p, sw + i * NSW, lane, buf[i], sc[i]);
    }
    for (int ph = 0; ph < nph; ++ph) {
      const int l = ph / 5;
      const int kind = ph == nph - 1 ? PK_CLS : ph % 5;
      if (kind == PK_ATTN) {
        if constexpr (!Q8) {
          if (HELP && p.attn_help && p.pos[0] + 1 >= kAttnHelpMinKeys) {
            if (sw == 0) {  // the block's second attention unit (control wave: the first)
              AttnWaveParams aw = {};
              aw.a.q = p.xb; aw.a.kc = p.kc; aw.a.vc = p.vc;
              aw.a.kv_b_stride = (long long)p.L * p.S * p.kvd;
              aw.a.kv_l_off = (long long)l * p.S * p.kvd;
              aw.a.pos = p.pos; aw.a.out = p.xb; aw.a.part = p.part;
              aw.a.dim = p.dim; aw.a.kv_dim = p.kvd; aw.a.head_size = HS; aw.a.n_heads = p.H;
              aw.a.kv_mul = p.kv_mul; aw.a.seq_len = p.S; aw.a.min_chunk = 16;
              aw.NS = aw.a.nsplit = 2 * p.NS < kMaxNS ? 2 * p.NS : kMaxNS;
              aw.cnt = p.tickets + (long long)l * p.H; aw.B = 1;
              aw.gqkv = p.gqkv; aw.gout = p.gxb; aw.etab = etab;
              aw.tag_in = tb + 5u * l + 1; aw.tag_out = tb + 5u * l + 2; aw.err = p.err;
              aw.poll_long = p.poll_long;
              for (int u = blockIdx.x + G; u < p.H * aw.NS; u += 2 * G)
                attn_unit_win<HS>(aw, u, reinterpret_cast<float*>(xs), lane);
            }
            __syncthreads();  // (the control wave's matching barrier ends its attention phase)
          }
        }
        continue;
      }
      const PDesc d = make_desc<Q8>(p, kind, kind == PK_CLS ? p.L : l, tb);
      const PGeo g = geo<Q8>(d);
      const bool tr = p.trace && sw == 0;
      // The buffers not prefetched across the boundary (pfn) are issued inside the staging,
      // right after this wave's last granule loads: their data returns behind the granules
      // (a wave's loads return in order) and the issue overlaps the sweep (issued after the
      // staging they delayed the first slot ~2 us, after the first slot's consume -2.5%).
      // Every load around them is unconditional, so the compiler's vmcnt waits for the
      // granules do not cover them (with a conditional issue they did: -18%); whole slots,
      // zero-size past the phase's end (at phase 0 this re-issues the initial prefetch).
      auto mid = [&] {
#pragma unroll
        for (int i = pfn<Q8>(); i < NBUF; ++i) load_any<Q8>(d, g, p, sw + i * NSW, lane, buf[i], sc[i]);
      };
      stage<Q8, false>(d, g, p, xs, xq, xsc, rmsw, red, sqa, wave, lane,
                       tr ? p.trace + ((long long)blockIdx.x * nph + ph) * kTraceSlots : nullptr, mid);
      if (tr) TRACE(4);
      run_gemv<Q8>(d, g, p, sw, lane, xs, xq, xsc, res, buf, sc, ctr,
                   tr ? p.trace + ((long long)blockIdx.x * nph + ph) * kTraceSlots + 5 : nullptr,
                   PChain{scr, p.pgp, cwb + sw * 136});
      if (tr) TRACE(6);
      // every slot reduced into res: the control wave's epilogue (the hand-off every other
      // block waits for) starts now, not after this wave's next-phase issue (measured +5%)
      __syncthreads();
      if (kind != PK_CLS) {
        const PDesc nd = next_desc<Q8>(p, kind, l, tb);
        const PGeo ng = geo<Q8>(nd);
#pragma unroll
        for (int i = 0; i < pfn<Q8>(); ++i)
          if (sw + i * NSW < ng.nslot) load_any<Q8>(nd, ng, p, sw + i * NSW, lane, buf[i], sc[i]);
      }
      if (tr) TRACE(7);
    }
  }
  grid_barrier(p);
  if constexpr (ROLE0) {
    if (blockIdx.x != 0) return;
    unsigned long long best = 0;
    if (p.argmax) {
      // argmax over the per-block winners + advance (src/llama.cpp:275-286)
      for (int i = lane; i < G; i += 64) {
        const unsigned long long k = ld8_sc1(p.bmax + i);
        best = k > best ? k : best;
      }
      for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long other = __shfl_xor(best, o, 64);
        best = other > best ? other : best;
      }
    }
    if (lane == 0) {
      p.seq[0] = (tb >> 12) + 1;  // every block read the sequence before the final barrier
      if (p.argmax) {
        const int next = best ? (int)(0xFFFFFFFFu - (uint32_t)(best & 0xFFFFFFFFull)) : 0;
        const int pp = p.pos[0];
        if (p.out && pp < p.S) p.out[pp] = next;
        p.tok[0] = next;
        p.pos[0] = pp + 1;
      }
    }
  }
}

template <int HS, bool Q8, bool HELP>
__global__ void __launch_bounds__(PT) persistent_step_kernel(PStep p) {
  if (p.fault && blockIdx.x == 0) return;  // test hook: a missing block (every wait is bounded)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* xres = reinterpret_cast<float*>(smem);     // kPResidFloats: residual slice
  float* res = xres + kPResidFloats;                // kPResFloats: row-chunk sums
  float* red = res + kPResFloats;                   // 16: block reductions
  float* rmsw = red + 16;                           // dim: the next norm's weights
  f4* xs = reinterpret_cast<f4*>(rmsw + p.dim);     // pad_floats: the staged input
  signed char* xq = reinterpret_cast<signed char*>(rmsw + p.dim + p.pad_floats);  // Q8: q8_pad int8
  float* xsc = reinterpret_cast<float*>(xq + p.q8_pad);                           //     q8_pad/64 scales
  // int8 only (exact arithmetic): the norm's squares (seqsum layout) | the long rows' group
  // products, aliased with the attention unit's strip | the streaming waves' chain scratch
  float* sqa = xsc + p.q8_pad / 64;
  float* scr = sqa + p.n_sqa;
  float* cwb = scr + p.n_scr;
  uint64_t* etab = reinterpret_cast<uint64_t*>(cwb + p.n_cw);  // the expf table (32 doubles' bits)
  float* awin = reinterpret_cast<float*>(etab + 32);             // fp32: the attention window
  {
    constexpr uint64_t tab[32] = TL_EXPF_TABLE;
    if (threadIdx.x < 32) etab[threadIdx.x] = tab[threadIdx.x];  // (read after the first barrier)
  }
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const unsigned tb = p.seq[0] << 12;  // tag base of this launch
  if (wave == 0) phases<HS, true, Q8, HELP>(p, wave, lane, res, xres, red, rmsw, xs, xq, xsc, sqa, scr, cwb, etab, tb, awin);
  else phases<HS, false, Q8, HELP>(p, wave, lane, res, xres, red, rmsw, xs, xq, xsc, sqa, scr, cwb, etab, tb, awin);
}

constexpr size_t kDynLdsCap = 160 * 1024;  // dynamic LDS per block (gfx950: 160 KiB per CU)

static size_t lds_bytes(const PStep& p) {
  return (size_t)(kPResidFloats + kPResFloats + 16 + p.dim + p.pad_floats) * 4 + (size_t)p.q8_pad +
         (size_t)p.q8_pad / 16 + (size_t)(p.n_sqa + p.n_scr + p.n_cw) * 4 + 32 * 8 +
         (p.q8 ? 0 : (size_t)attn_win_floats(p.hs) * 4);
}

template <int HS, bool Q8, bool HELP = false>
static const void* kfn() { return (const void*)persistent_step_kernel<HS, Q8, HELP>; }
static const void* kernel_of(const PStep& p) {
  if (p.q8) return p.hs == 128 ? kfn<128, true>() : kfn<64, true>();
  if (p.attn_help && p.long_ctx) return p.hs == 128 ? kfn<128, false, true>() : kfn<64, false, true>();
  return p.hs == 128 ? kfn<128, false>() : kfn<64, false>();
}

bool persistent_prepare(PStep& p, int ncu, const char** why) {
  auto fail = [&](const char* m) { if (why) *why = m; return false; };
  if (p.hs != 64 && p.hs != 128) return fail("head size must be 64 or 128");
  if (p.dim % 256 || p.hid % 256) return fail("dim and hidden_dim must be multiples of 256");
  if (p.NS < 1 || p.NS > kMaxNS) return fail("attention splits out of range");
  if (ncu < 8) return fail("too few compute units");
  if ((long long)part_weight(ncu) * (p.V > p.hid ? p.V : p.hid) >= (1ll << 32)) return fail("grid x rows exceeds 32 bits");
  if (p.q8 && p.q8 != 64) return fail("int8 group size must be 64");
  if (p.dim / 64 > PT) return fail("dim too large for the int8 Wo staging");
  if (5 * p.L + 1 >= 4096) return fail("too many layers for the phase tags");
  // every block must own work in every phase: a hand-off buffer may be rewritten as soon as
  // the next phase's outputs are complete, which then implies every block has staged it
  auto owns = [&](long long n) {  // the partition of geo(): every block's share non-empty
    for (int b = 0; b < ncu; ++b)
      if (n * part_weight(b + 1) / part_weight(ncu) == n * part_weight(b) / part_weight(ncu)) return false;
    return true;
  };
  if (!owns(p.dim) || !owns((p.dim + 2 * p.kvd) / 2) || !owns(p.hid)) return fail("model too small for the grid");
  auto nchunks = [&](int K) { return p.q8 ? (K + 4095) / 4096 : (K + PL * 256 - 1) / (PL * 256); };
  auto padf = [&](int K) { return p.q8 ? K : nchunks(K) * PL * 256; };
  auto nrc = [&](int K, int n_items, int rpi) {
    return (int)((long long)n_items * (100 + kXcdSkew) / part_weight(ncu) + 2) * rpi * nchunks(K);
  };
  p.pad_floats = padf(p.dim) > padf(p.hid) ? padf(p.dim) : padf(p.hid);
  // int8: the exact attention splits each head over ang units (<= 8, at most one per block, >= 8
  // columns each; attention.hpp attn_unit_split)
  p.ang = 1;
  if (p.q8)
    while (p.ang < 8 && (long long)p.H * p.ang * 2 <= ncu && p.hs / (p.ang * 2) >= 8) p.ang *= 2;
  p.q8_pad = p.q8 ? 4096 * (nchunks(p.dim) > nchunks(p.hid) ? nchunks(p.dim) : nchunks(p.hid)) : 0;
  p.n_sqa = p.n_scr = p.n_cw = p.pgp = 0;
  if (p.q8) {
    // the norm's squares: seqsum layout of dim values (ch = dim / 64, rows of ch + 4)
    p.n_sqa = 64 * (p.dim / 64 + 4);
    // group products of the rows longer than a chunk (row stride pgp), per phase
    int rows_max = 0, gp = 0;
    auto longrows = [&](int K, int n_items, int rpi) {
      if (nchunks(K) < 2) return;
      const int stride = nchunks(K) * 64 + 4;
      const int rows = (int)((long long)n_items * (100 + kXcdSkew) / part_weight(ncu) + 2) * rpi;
      gp = stride > gp ? stride : gp;
      rows_max = rows > rows_max ? rows : rows_max;
    };
    longrows(p.dim, (p.dim + 2 * p.kvd) / 2, 2);
    longrows(p.dim, p.dim, 1);
    longrows(p.dim, p.hid, 2);
    longrows(p.hid, p.dim, 1);
    longrows(p.dim, p.V, 1);
    p.pgp = gp;  // one stride for every long-row phase
    const int pb = rows_max * gp;
    const int attn = 3 * p.hs + 64 * (4 * ((p.S + 255) / 256) + 4) + ((p.S + 3) & ~3) + 64;  // attn_exact_floats
    p.n_scr = ((pb > attn ? pb : attn) + 3) & ~3;
    p.n_cw = NSW * 136;
  }
  if (nrc(p.dim, (p.dim + 2 * p.kvd) / 2, 2) > kPResFloats || nrc(p.dim, p.hid, 2) > kPResFloats ||
      nrc(p.hid, p.dim, 1) > kPResFloats || nrc(p.dim, p.V, 1) > kPResFloats)
    return fail("too many rows per block");
  if ((long long)p.dim * (100 + kXcdSkew) / part_weight(ncu) + 2 > kPResidFloats)
    return fail("residual slice per block too large");
  if (p.q8) {
    // the strip xs doubles as the attention unit's LDS window: a round of 64 keys and then V rows
    // of hs / ang floats, 512 rows a round (64 when the LDS is short)
    const int base = p.pad_floats;
    for (int rows : {512, 64}) {
      const int need = 64 * p.hs + rows * (p.hs / p.ang);
      p.pad_floats = base > need ? base : need;
      if (lds_bytes(p) <= kDynLdsCap) break;
    }
  }
  if (lds_bytes(p) > kDynLdsCap) return fail("activations do not fit the LDS");
  p.attn_help = 0;
  p.poll_long = p.dim >= 2048;
  if (!p.q8 && p.NS * 2 <= kMaxNS) {  // room for a second attention window in the strip?
    const int base = p.pad_floats, need = attn_win_floats(p.hs);
    if (base < need) p.pad_floats = need;
    if (lds_bytes(p) <= kDynLdsCap) p.attn_help = 1;
    else p.pad_floats = base;
  }
  {  // allow more than 64 KiB of dynamic LDS (gfx950: 160 KiB per CU): a per-device attribute,
     // raised once for each device a decoder is prepared on (decoders of several devices may be
     // created from several threads, app/run.cpp)
    static std::mutex mu;
    static unsigned long long done = 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return fail("no current device");
    std::lock_guard<std::mutex> lock(mu);
    const unsigned long long bit = dev < 64 ? 1ull << dev : 0ull;
    if (!bit || !(done & bit)) {
      for (const void* f : {kfn<128, false>(), kfn<64, false>(), kfn<128, true>(), kfn<64, true>(),
                            kfn<128, false, true>(), kfn<64, false, true>()})
        if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kDynLdsCap) != hipSuccess) {
          (void)hipGetLastError();  // (not sticky for the caller's next launch check)
          return fail("cannot raise the dynamic LDS limit");
        }
      done |= bit;
    }
  }
  int nb = 0;
  const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel_of(p), PT, lds_bytes(p));
  if (e != hipSuccess || nb < 1) return fail("persistent kernel does not fit one block per CU");
  return true;
}

// Co-residency of the grid (one block per CU, spin-waiting on each other's hand-offs): a direct
// launch is cooperative — the runtime dispatches it on a cooperative queue, which starts the grid
// only when every block can be resident at once, and refuses (hipErrorCooperativeLaunchTooLarge)
// a grid that could never be.  The greedy loop captures the step into a hipGraph; a captured
// cooperative launch replays cooperatively on ROCm 7.2 (MI355X_MICROARCH.md, residency: +17-20 us
// per replay, although hipKernelNodeAttributeCooperative reads 0) — an observation, not an API
// guarantee, so what holds in every case is the rest: the grid is sized by the occupancy query
// (one block per CU), every wait is bounded, and a launch whose waits gave up is reported and
// re-run on the multi-launch step (tests/test_persist_gpu.py, test_persist_b_gpu.py
// test_give_up_falls_back: a launch missing a block, eager and from a graph).
// THALLAMA_PERSIST_COOP=0 selects a plain launch (measurement only).
static bool use_cooperative() {
  static const bool on = [] {
    const char* e = getenv("THALLAMA_PERSIST_COOP");
    int dev = 0, coop = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev) != hipSuccess)
      coop = 0;
    return coop != 0 && !(e && e[0] == '0');
  }();
  return on;
}

bool persistent_cooperative() { return use_cooperative(); }

// The caller zeroes p.sync (kPSyncWords) and the tickets on the same stream right before.
hipError_t launch_persistent_step(const PStep& p, hipStream_t s, int ncu) {
  if (use_cooperative()) {
    PStep arg = p;
    void* args[] = {&arg};
    return hipLaunchCooperativeKernel(kernel_of(p), dim3(ncu), dim3(PT), args, (unsigned)lds_bytes(p), s);
  }
  PStep arg = p;
  void* args[] = {&arg};
  return hipLaunchKernel(kernel_of(p), dim3(ncu), dim3(PT), args, lds_bytes(p), s);
}

}  // namespace tl
