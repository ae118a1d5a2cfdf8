// attention.hpp — fused single-token decode attention for one layer.
//
// Semantics: reference src/seq.cpp:103-136 (scores q.k/sqrtf(hs) for t <= pos,
// softmax, weighted sum of V), which the reference GPU path splits into three
// launches (src/thaDNN/thaDNN_mha.cpp:246-426).  Here it is ONE launch over a
// (head, sequence, key-split) grid plus, when the keys are split, a tiny
// combine launch (flash-decoding).  K/V stay in the reference layout
// [b][layer][seq_len][kv_dim]; each key row of a head is 4*hs contiguous bytes,
// read by hs/4 lanes with one float4 each.
#pragma once
#include "common.hpp"
#include "libm_exact.hpp"
#include "seqsum.hpp"

namespace tl {

struct AttnParams {
  const float* q;       // [B][dim]  (RoPE already applied)
  const float* kc;      // key_cache base   [B][L][S][kv_dim]
  const float* vc;      // value_cache base
  long long kv_b_stride, kv_l_off;
  const int* pos;       // [B]
  float* out;           // [B][dim]
  float* part;          // [B][H][nsplit][hs + 4]  (o, m, l, pad) when nsplit > 1
  int dim, kv_dim, head_size, n_heads, kv_mul, seq_len, nsplit, min_chunk;
};

TL_DEVICE void split_range(int T, int nsplit, int min_chunk, int s, int& t0, int& t1) {
  int chunk = (T + nsplit - 1) / nsplit;
  chunk = max(chunk, min_chunk);
  t0 = s * chunk;
  t1 = min(T, t0 + chunk);
}

// LPK = lanes per key row = hs/4.
template <int LPK>
__global__ void __launch_bounds__(256) attn_decode_kernel(AttnParams p) {
  keep_implicit_args();  // common.hpp: rocprofv3 --pmc needs the hidden kernargs
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* red = reinterpret_cast<float*>(smem);  // 16
  float* sc = red + 16;                         // scores for this split (<= seq_len)
  constexpr int HS = LPK * 4;
  const int h = blockIdx.x, b = blockIdx.y, s = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int T = p.pos[b] + 1;
  int t0, t1;
  split_range(T, p.nsplit, p.min_chunk, s, t0, t1);
  if (t0 >= t1) return;  // nothing for this split (combine ignores it)
  const int n = t1 - t0;

  const int kvh = h / p.kv_mul;
  const float* kbase = p.kc + (long long)b * p.kv_b_stride + p.kv_l_off + (long long)kvh * HS;
  const float* vbase = p.vc + (long long)b * p.kv_b_stride + p.kv_l_off + (long long)kvh * HS;
  const f4 qv = reinterpret_cast<const f4*>(p.q + (long long)b * p.dim + h * HS)[lane % LPK];
  const float rs = sqrtf((float)HS);

  // ---- scores: each wave handles KPW = 64/LPK keys per step
  constexpr int KPW = 64 / LPK;
  const int sub = lane / LPK;
  for (int t = t0 + wave * KPW + sub; t - sub < t1; t += 4 * KPW) {
    float d = 0.f;
    if (t < t1) {
      const f4 kv = reinterpret_cast<const f4*>(kbase + (long long)t * p.kv_dim)[lane % LPK];
      d = dot4(qv, kv, 0.f);
    }
    d = group_sum<LPK>(d);
    if (t < t1 && (lane % LPK) == 0) sc[t - t0] = __fdiv_rn(d, rs);
  }
  __syncthreads();

  // ---- softmax over this split (reference src/seq.cpp:18-36)
  float m = -3.402823466e+38f;
  for (int i = tid; i < n; i += 256) m = fmaxf(m, sc[i]);
  m = block_max(m, red);
  float l = 0.f;
  for (int i = tid; i < n; i += 256) {
    float e = expf_libm(__fsub_rn(sc[i], m));
    sc[i] = e;
    l += e;
  }
  l = block_sum(l, red);
  const bool whole = p.nsplit == 1 || (t0 == 0 && t1 == T);
  if (whole) {
    for (int i = tid; i < n; i += 256) sc[i] = __fdiv_rn(sc[i], l);
    __syncthreads();
  }

  // ---- weighted V sum: LPK float4 columns x G groups over t
  constexpr int G = 256 / LPK;
  const int col = tid % LPK, g = tid / LPK;
  f4 o = {0.f, 0.f, 0.f, 0.f};
  for (int t = t0 + g; t < t1; t += G) {
    const float a = sc[t - t0];
    const f4 vv = reinterpret_cast<const f4*>(vbase + (long long)t * p.kv_dim)[col];
    o.x = fmaf(a, vv.x, o.x); o.y = fmaf(a, vv.y, o.y);
    o.z = fmaf(a, vv.z, o.z); o.w = fmaf(a, vv.w, o.w);
  }
  // reduce the G groups through LDS (reuse the score area after a barrier)
  __syncthreads();
  f4* ob = reinterpret_cast<f4*>(sc);
  ob[g * LPK + col] = o;
  __syncthreads();
  if (tid < LPK) {
    f4 r = ob[tid];
    for (int gg = 1; gg < G; ++gg) {
      f4 x = ob[gg * LPK + tid];
      r.x += x.x; r.y += x.y; r.z += x.z; r.w += x.w;
    }
    if (whole) {
      reinterpret_cast<f4*>(p.out + (long long)b * p.dim + h * HS)[tid] = r;
    } else {
      float* pp = p.part + (((long long)b * p.n_heads + h) * p.nsplit + s) * (HS + 4);
      reinterpret_cast<f4*>(pp)[tid] = r;  // records are HS+4 floats: 16-B aligned
      if (tid == 0) { pp[HS] = m; pp[HS + 1] = l; }
    }
  }
}

// ---------------------------------------------------------------------------
// Wave-level decode attention: one 64-lane wave (= one 64-thread block) per
// (sequence b, head h, unit s), NS units per (b, h).  Unit s walks key chunks
// c = s, s+NS, s+2NS, ... of CH keys; for every chunk the K rows AND the V rows
// are requested together (one memory latency per chunk, not three), key t's
// score lands in lane t (DPP row sums + readlane + lane select, no LDS strip), and
// chunks are merged with an online softmax.  No block barriers: max/sum are
// DPP wave reductions (the ds_bpermute forms put an LDS round trip per step on
// the decode critical path).
//  * if the context fits one chunk (T <= CH) unit 0 alone computes the reference
//    order exactly (normalise the probabilities, then sum) and writes the output;
//  * otherwise each live unit publishes (o, m, l) with write-through (sc1)
//    stores, drains them (s_waitcnt vmcnt(0)) and takes a ticket from an
//    agent-scope atomic counter; the unit that draws the last ticket reads every
//    partial with sc1 loads, combines them and re-arms the counter
//    (MI355X_MICROARCH.md §visibility, "Valid forms", row 1: no fences needed).
// Units are numbered s-major (blockIdx = s*B*H + b*H + h) so the live ones at short
// contexts are the lowest block ids and spread over every CU.
constexpr int kMaxNS = 16;  // units per (b, h) at most

struct AttnWaveParams {
  AttnParams a;
  unsigned* cnt;  // [B*H] tickets, zero between launches
  int B, NS;      // NS <= kMaxNS
  // granule mode (persistent step, B = 1): q and the new K/V row of this step arrive as
  // tagged granules (common.hpp) from the QKV phase of the same launch; the output leaves
  // as granules for the Wo phase
  const unsigned long long* gqkv;  // [dim + 2*kv_dim]: q | k_new | v_new
  unsigned long long* gout;        // [dim]
  unsigned tag_in, tag_out;
  unsigned* err;
  unsigned long long* ts;          // optional timeline (persistent step trace): q ready, k/v ready, done
  // int8 weights (persistent step, attn_unit_split): the score granules [H][seq_len]
  unsigned long long* gsc;
  const uint64_t* etab;  // the expf table (libm_exact.hpp), an LDS copy
  // int8 weights, multi-launch batched step: the output row is also stored quantised (codes
  // [b][dim], group scales [b][dim/64]) so the Wo launch that follows needs no quantise pass
  signed char* xq8;
  float* xq8s;
  int poll_long;  // persistent step of a large model: granule waits back off (common.hpp gran_backoff)
};

TL_DEVICE void st_sc1(float* p, float v) { st1_sc1(p, v); }
TL_DEVICE float ld_sc1(const float* p) { return ld1_sc1(p); }

// Orders one wave's LDS strip writes before its reads (and vice versa): LDS ops of a
// wave retire in order, this only stops the compiler from moving them.
TL_DEVICE void wave_lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// runq's activation quantisation of one head's output row (lane holds columns lane*VPL + c)
// over its 64-value groups: returns this lane's VPL codes packed low byte first; lane g < VPL
// gets group g's scale in `lsc`.  All 64 lanes active.
template <int HS>
TL_DEVICE unsigned head_q8(const float* v, int lane, float& lsc) {
  constexpr int VPL = HS / 64;
  // group g of the head: lanes [g*64/VPL, (g+1)*64/VPL), i.e. 16-lane rows [g*RPG, (g+1)*RPG)
  constexpr int RPG = 4 / VPL;
  float m = 0.f;
#pragma unroll
  for (int c = 0; c < VPL; ++c) m = fmaxf(m, fabsf(v[c]));
  m = row16_max(m);
  float sc[VPL];
#pragma unroll
  for (int g = 0; g < VPL; ++g) {
    float gm = lane_f(m, 16 * g * RPG);
#pragma unroll
    for (int r = 1; r < RPG; ++r) gm = fmaxf(gm, lane_f(m, 16 * (g * RPG + r)));
    sc[g] = __fdiv_rn(gm, 127.0f);
  }
  const int mg = (lane >> 4) / RPG;  // this lane's group
  float scale = sc[0];
  lsc = sc[0];
#pragma unroll
  for (int g = 1; g < VPL; ++g) {
    scale = mg == g ? sc[g] : scale;
    lsc = lane == g ? sc[g] : lsc;
  }
  unsigned packed = 0;
#pragma unroll
  for (int c = 0; c < VPL; ++c) packed |= (unsigned)(q8_code(v[c], scale) & 0xFF) << (8 * c);
  return packed;
}

// Multi-launch step: store head h of sequence b (fp32 row, and the int8 codes + group scales
// when w.xq8 is set).
template <int HS>
TL_DEVICE void store_head(const AttnWaveParams& w, int b, int h, const float* v, int lane) {
  constexpr int VPL = HS / 64;
  const AttnParams& p = w.a;
  float* out = p.out + (long long)b * p.dim + h * HS + lane * VPL;
#pragma unroll
  for (int c = 0; c < VPL; ++c) out[c] = v[c];
  if (!w.xq8) return;
  float lsc;
  const unsigned packed = head_q8<HS>(v, lane, lsc);
  signed char* q = w.xq8 + (long long)b * p.dim + h * HS + lane * VPL;
  if constexpr (VPL == 1) *q = (signed char)packed;
  else if constexpr (VPL == 2) *reinterpret_cast<unsigned short*>(q) = (unsigned short)packed;
  else *reinterpret_cast<unsigned*>(q) = packed;
  if (lane < VPL) w.xq8s[(long long)b * (p.dim / 64) + h * VPL + lane] = lsc;
}

// Persistent step (fp32 weights): publish head h's output row (lane holds columns lane*VPL + c)
// as {value, tag} granules.
template <int HS>
TL_DEVICE void publish_head(const AttnWaveParams& w, int b, int h, const float* v, int lane) {
  constexpr int VPL = HS / 64;
  unsigned long long* go = w.gout + (long long)b * w.a.dim;  // sequence b's row (batched step)
#pragma unroll
  for (int c = 0; c < VPL; ++c) st8_sc1(go + h * HS + lane * VPL + c, gran(w.tag_out, v[c]));
}

// The body of one attention unit, run by one full wave; `unit` must be wave-uniform.  Also used
// inside the persistent step
// kernel (persist.hip) with GR = true: q and the K/V rows at position pos come from the
// granules the QKV phase of the same launch published (rows < pos were written by earlier
// launches and are read from the cache), and the output is published as granules.
template <int HS, int CH, bool GR = false>
TL_DEVICE void attn_unit(const AttnWaveParams& w, int unit, int lane) {
  constexpr int LPK = HS / 4;    // lanes per key row (one float4 each)
  constexpr int KPI = 64 / LPK;  // keys per wave-instruction
  constexpr int NI = CH / KPI;   // K wave-loads per chunk
  constexpr int VPL = HS / 64;   // output columns per lane
  static_assert(CH <= 64 && HS % 64 == 0, "chunk <= 64 keys, head size multiple of 64");
  const AttnParams& p = w.a;
  const int BH = w.B * p.n_heads;
  const int s = unit / BH, bh = unit % BH;
  const int b = bh / p.n_heads, h = bh % p.n_heads;
  const int T = p.pos[b] + 1;
  const int nchunks = (T + CH - 1) / CH;
  const int nact = nchunks < w.NS ? nchunks : w.NS;  // live units for this (b, h)
  if (s >= nact) return;

  const int kvh = h / p.kv_mul;
  const float* kbase = p.kc + (long long)b * p.kv_b_stride + p.kv_l_off + (long long)kvh * HS;
  const float* vbase = p.vc + (long long)b * p.kv_b_stride + p.kv_l_off + (long long)kvh * HS;
  const float* qrow = p.q + (long long)b * p.dim + h * HS;
  f4 qv;
  // granule mode: q and the new key / value row (position T-1) are waited for only after the
  // first chunk's cached rows are in flight
  __amdgpu_buffer_rsrc_t rg;
  bool qready = false;
  // sequence b's q | k_new | v_new granules (the batched persistent step keeps B rows)
  const unsigned long long* gq = w.gqkv + (long long)b * (p.dim + 2 * p.kv_dim);
  if constexpr (GR) rg = rsrc_of(gq);
  else qv = reinterpret_cast<const f4*>(qrow)[lane % LPK];
  const float rs = sqrtf((float)HS);
  const bool whole = nchunks == 1;

  float m = -3.402823466e+38f, l = 0.f;
  float o[VPL];
#pragma unroll
  for (int c = 0; c < VPL; ++c) o[c] = 0.f;

  for (int ch = s; ch < nchunks; ch += w.NS) {
    const int t0 = ch * CH, t1 = min(T, t0 + CH), n = t1 - t0;
    // K and V rows of the chunk, all in flight at once (rows past the chunk are
    // clamped to its last row: loaded, weighted by 0)
    f4 kv[NI];
    float vv[CH][VPL];
    if constexpr (GR) {
      // rows already in the cache (t < T-1) first; the row this step writes (t = T-1) is
      // patched in from the granules once they are published
      const int tc = T >= 2 ? T - 2 : 0;
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int t = min(min(t0 + i * KPI + lane / LPK, t1 - 1), tc);
        kv[i] = reinterpret_cast<const f4*>(kbase + (long long)t * p.kv_dim)[lane % LPK];
      }
#pragma unroll
      for (int u = 0; u < CH; ++u) {
        const float* vr = vbase + (long long)min(min(t0 + u, t1 - 1), tc) * p.kv_dim + lane * VPL;
#pragma unroll
        for (int c = 0; c < VPL; ++c) vv[u][c] = vr[c];
      }
      const unsigned qo = (unsigned)(h * HS + (lane % LPK) * 4) * 8u;
      const unsigned ko = (unsigned)(p.dim + kvh * HS + (lane % LPK) * 4) * 8u;
      const unsigned vo = (unsigned)(p.dim + p.kv_dim + kvh * HS + lane * VPL) * 8u;
      // the new key / value row: granules of this chunk when it holds position T-1
      f4 kn = f4{0.f, 0.f, 0.f, 0.f};
      float vn[VPL];
#pragma unroll
      for (int c = 0; c < VPL; ++c) vn[c] = 0.f;
      bool kvready = false;
      if (!qready) {
        // q, and the new k / v row if this chunk holds it, requested together: one round
        // trip once the QKV epilogues have published (late granules are re-polled singly)
        const v4u qa = ld16_sc1(rg, qo), qb = ld16_sc1(rg, qo + 16);
        v4u ka = v4u{0u, 0u, 0u, 0u}, kb = ka;
        unsigned long long vr[VPL];
        if (t1 == T) {
          ka = ld16_sc1(rg, ko);
          kb = ld16_sc1(rg, ko + 16);
#pragma unroll
          for (int c = 0; c < VPL; ++c) vr[c] = ld8_sc1(gq + vo / 8 + c);
        }
        qv = gran4_ok(qa, qb, w.tag_in) ? gran4_val(qa, qb) : gran_wait4(rg, qo, w.tag_in, w.err, w.poll_long != 0);
        qready = true;
        if (w.ts && lane == 0) w.ts[0] = __builtin_amdgcn_s_memrealtime();
        if (t1 == T) {
          kn = gran4_ok(ka, kb, w.tag_in) ? gran4_val(ka, kb) : gran_wait4(rg, ko, w.tag_in, w.err, w.poll_long != 0);
#pragma unroll
          for (int c = 0; c < VPL; ++c)
            vn[c] = (unsigned)(vr[c] >> 32) == w.tag_in ? __uint_as_float((unsigned)vr[c])
                                                       : gran_wait(gq + vo / 8 + c, w.tag_in, w.err, w.poll_long != 0);
          kvready = true;
        }
      }
      if (t1 == T) {  // this chunk holds the new row
        if (!kvready) {
          kn = gran_wait4(rg, ko, w.tag_in, w.err, w.poll_long != 0);
#pragma unroll
          for (int c = 0; c < VPL; ++c) vn[c] = gran_wait(gq + vo / 8 + c, w.tag_in, w.err, w.poll_long != 0);
        }
        if (w.ts && lane == 0) w.ts[1] = __builtin_amdgcn_s_memrealtime();
#pragma unroll
        for (int i = 0; i < NI; ++i)
          if (min(t0 + i * KPI + lane / LPK, t1 - 1) == T - 1) kv[i] = kn;
#pragma unroll
        for (int u = 0; u < CH; ++u)
          if (min(t0 + u, t1 - 1) == T - 1) {
#pragma unroll
            for (int c = 0; c < VPL; ++c) vv[u][c] = vn[c];
          }
      }
    } else {
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int t = min(t0 + i * KPI + lane / LPK, t1 - 1);
        kv[i] = reinterpret_cast<const f4*>(kbase + (long long)t * p.kv_dim)[lane % LPK];
      }
#pragma unroll
      for (int u = 0; u < CH; ++u) {
        const float* vr = vbase + (long long)min(t0 + u, t1 - 1) * p.kv_dim + lane * VPL;
#pragma unroll
        for (int c = 0; c < VPL; ++c) vv[u][c] = vr[c];
      }
    }
    // scores (reference src/seq.cpp:107-117): row sums by DPP, a key's rows added through
    // SGPRs, key t's score written into lane t (no LDS strip, no ds_bpermute round trips)
    constexpr int R = LPK / 16;  // 16-lane rows per key row
    float raw = 0.f;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const float d = row16_sum(dot4(qv, kv[i], 0.f));
#pragma unroll
      for (int j = 0; j < KPI; ++j) {
        float sj = lane_f(d, 16 * j * R);
#pragma unroll
        for (int r = 1; r < R; ++r) sj += lane_f(d, 16 * (j * R + r));
        raw = lane == i * KPI + j ? sj : raw;
      }
    }
    const float my = lane < n ? __fdiv_rn(raw, rs) : -3.402823466e+38f;
    const float mc = wave_max_u(my);
    float pr;
    if (whole) {
      // reference softmax (src/seq.cpp:18-36): exp, sum, divide, then the weighted sum
      const float e = lane < n ? expf_libm(__fsub_rn(my, mc)) : 0.f;
      pr = __fdiv_rn(e, wave_sum_u(e));
      m = mc;
    } else {
      const float mn = fmaxf(m, mc);
      const float e = lane < n ? expf_libm(__fsub_rn(my, mn)) : 0.f;
      const float scale = expf_libm(__fsub_rn(m, mn));  // rescale what earlier chunks summed
      l = fmaf(l, scale, wave_sum_u(e));
#pragma unroll
      for (int c = 0; c < VPL; ++c) o[c] *= scale;
      m = mn;
      pr = e;
    }
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const float a = lane_f(pr, u);
#pragma unroll
      for (int c = 0; c < VPL; ++c) o[c] = fmaf(a, vv[u][c], o[c]);
    }
  }

  if (whole) {
    if constexpr (GR) {
      if (w.ts && lane == 0) w.ts[2] = __builtin_amdgcn_s_memrealtime();
      publish_head<HS>(w, b, h, o, lane);
    } else {
      store_head<HS>(w, b, h, o, lane);
    }
    return;
  }
  // publish this unit's partial (write-through), drain, take a ticket
  float* rec = p.part + ((long long)bh * w.NS + s) * (HS + 4);
#pragma unroll
  for (int c = 0; c < VPL; ++c) st_sc1(rec + lane * VPL + c, o[c]);
  if (lane == 0) {
    st_sc1(rec + HS, m);
    st_sc1(rec + HS + 1, l);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  unsigned ticket = 0;
  if (lane == 0) ticket = __hip_atomic_fetch_add(w.cnt + bh, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  ticket = (unsigned)__builtin_amdgcn_readfirstlane((int)ticket);
  if (ticket != (unsigned)(nact - 1)) return;
  // last unit: combine every partial (sc1 loads only).  Lane k reads unit k's (m, l);
  // every lane then reads its columns of all kMaxNS records at once (records past nact
  // are clamped to the last live one and weighted 0), so the combine costs one memory
  // latency instead of one per partial.
  const float* recs = p.part + (long long)bh * w.NS * (HS + 4);
  const int kl = lane < nact ? lane : nact - 1;
  const float mk = ld_sc1(recs + kl * (HS + 4) + HS);
  const float lk = ld_sc1(recs + kl * (HS + 4) + HS + 1);
  float ov[kMaxNS][VPL];
#pragma unroll
  for (int k = 0; k < kMaxNS; ++k) {
    const int kk = k < nact ? k : nact - 1;
#pragma unroll
    for (int c = 0; c < VPL; ++c) ov[k][c] = ld_sc1(recs + kk * (HS + 4) + lane * VPL + c);
  }
  const float M = wave_max_u(lane < nact ? mk : -3.402823466e+38f);
  const float sk = lane < nact ? expf_libm(__fsub_rn(mk, M)) : 0.f;
  const float L = wave_sum_u(lk * sk);
  float acc[VPL];
#pragma unroll
  for (int c = 0; c < VPL; ++c) acc[c] = 0.f;
#pragma unroll
  for (int k = 0; k < kMaxNS; ++k) {
    const float a = lane_f(sk, k);
#pragma unroll
    for (int c = 0; c < VPL; ++c) acc[c] = fmaf(ov[k][c], a, acc[c]);
  }
#pragma unroll
  for (int c = 0; c < VPL; ++c) acc[c] = __fdiv_rn(acc[c], L);
  if constexpr (GR) {
    publish_head<HS>(w, b, h, acc, lane);
  } else {
    store_head<HS>(w, b, h, acc, lane);
  }
  if (lane == 0) __hip_atomic_store(w.cnt + bh, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Stand-alone launch: one 64-thread block per unit.
template <int HS, int CH>
__global__ void __launch_bounds__(64) attn_wave_kernel(AttnWaveParams w) {
  keep_implicit_args();  // common.hpp: rocprofv3 --pmc needs the hidden kernargs
  attn_unit<HS, CH>(w, blockIdx.x, threadIdx.x);
}

// ---------------------------------------------------------------------------
// runq's attention, bit for bit (runq.c:396-434; the same order as src/seq.cpp:103-136), for the
// int8 persistent step: the Wo input is re-quantised, so the head output must be the reference's
// floats.
//   score_t = (((0 + q0 k0) + q1 k1) + ...) / sqrtf(hs)      one lane per key, sequential dot
//   e_t = expf(score_t - max);  sum = e_0 + e_1 + ...         libm_exact.hpp; seqsum.hpp
//   a_t = e_t / sum;  xb_i = ((0 + a_0 v0_i) + a_1 v1_i) + ...  one lane per output column
// Every score and every column is independent; only the sum and the column chains are ordered.
// So a head is split over NG units (blocks) c = 0..NG-1: unit c scores keys [T c/NG, T (c+1)/NG)
// and publishes them as {score, tag} granules (gsc, [H][S]); every unit of the head gathers all T
// scores, repeats the softmax (max, expf, the exact sum: identical in every unit) and chains its
// HS/NG columns over all T rows; the columns leave as fp32 {value, tag} granules (gout) and the
// Wo phase quantises them while it gathers (runq.c:145-171, persist.hip gather_q8).
// Memory: a unit's K slice (<= 64 keys a round) and V column slice (rows of HS/NG floats) reach
// LDS by LDS-DMA (global_load_lds: no registers), all requested at the unit's start — before q
// has arrived — so the whole head costs about one memory latency instead of one per 64 keys.
// q and this step's k/v rows come from the QKV phase's granules.  Products and sums are single
// roundings (the library is built with -ffp-contract=off).
// LDS: `strip` holds attn_split_floats(hs, T) floats; `win` (nwin floats) holds a K round
// (64 keys transposed: piece i of key l at win[i*256 + 4l], so lane l reads its key
// conflict-free) followed by the V rows [rows][HS/NG].
TL_DEVICE int attn_split_floats(int hs, int T) { return 3 * hs + seqsum_floats(T) + ((T + 3) & ~3) + 64; }

TL_DEVICE void dma16(const float* src, float* dst_lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)dst_lds, 16, 0, 0);
}
TL_DEVICE void dma_wait_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

template <int HS>
TL_DEVICE void attn_unit_split(const AttnWaveParams& w, int h, int c, int NG, float* strip, float* win, int nwin,
                               int lane) {
  constexpr int VPL = HS / 64;
  constexpr int PC = HS / 4;  // 16-byte pieces per key row
  const AttnParams& p = w.a;
  const int T = p.pos[0] + 1;
  const int tc = T - 1;  // rows read from the cache (row T-1 is this step's, from the granules)
  const int kvh = h / p.kv_mul;
  const float* kbase = p.kc + p.kv_l_off + (long long)kvh * HS;
  const float* vbase = p.vc + p.kv_l_off + (long long)kvh * HS;
  const int CW = HS / NG;           // this unit's columns
  const int col0 = c * CW;
  const int PPR = CW / 4;           // 16-byte pieces per V row slice
  const int RPI = 64 / PPR;         // V rows per DMA instruction (1 KiB)
  const int k0 = (int)((long long)T * c / NG), k1 = (int)((long long)T * (c + 1) / NG);
  const int kc1 = min(k1, tc);      // cached keys of this unit: [k0, kc1)
  float* qs = strip;                // q [HS]
  float* kn = qs + HS;              // k row of position T-1 [HS]
  float* vn = kn + HS;              // v row of position T-1 [HS]
  float* sa = vn + HS;              // exp values, seqsum layout
  float* at = sa + seqsum_floats(T);  // scores, then probabilities [T]
  const int ch = seqsum_ch(T);
  float* vw = win + 64 * HS;        // V rows [rv][CW]
  const int rq = RPI > 4 ? RPI : 4;
  const int rv = (nwin - 64 * HS) / CW / rq * rq;  // V rows per round (host: >= 64; a multiple of 4)
  unsigned long long* gs = w.gsc + (long long)h * p.seq_len;
  // q / k_new / v_new granules first (their wait then does not cover the DMA behind them)
  const unsigned long long* src[3] = {w.gqkv + h * HS, w.gqkv + p.dim + kvh * HS,
                                      w.gqkv + p.dim + p.kv_dim + kvh * HS};
  float* dst[3] = {qs, kn, vn};
  unsigned long long g[3][VPL];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int cc = 0; cc < VPL; ++cc) g[r][cc] = ld8_sc1(src[r] + lane * VPL + cc);
  auto issue_keys = [&](int t0) {  // keys t0 + lane (< kc1), transposed into win
    if (t0 + lane < kc1) {
      const float* row = kbase + (long long)(t0 + lane) * p.kv_dim;
#pragma unroll
      for (int i = 0; i < PC; ++i) dma16(row + 4 * i, win + i * 256);
    }
  };
  auto issue_rows = [&](int r0, int n) {  // V rows [r0, r0 + n) of this unit's columns into vw
    for (int k = 0; k * RPI < n; ++k) {
      const int rr = k * RPI + lane / PPR;
      if (rr < n) dma16(vbase + (long long)(r0 + rr) * p.kv_dim + col0 + (lane % PPR) * 4, vw + k * 256);
    }
  };
  if (k0 < kc1) issue_keys(k0);
  if (tc > 0) issue_rows(0, min(rv, tc));
  for (int i = lane; i < seqsum_floats(T); i += 64) sa[i] = 0.f;
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int cc = 0; cc < VPL; ++cc)
      dst[r][lane * VPL + cc] = (unsigned)(g[r][cc] >> 32) == w.tag_in
                                    ? __uint_as_float((unsigned)g[r][cc])
                                    : gran_wait(src[r] + lane * VPL + cc, w.tag_in, w.err, w.poll_long != 0);
  if (w.ts && lane == 0) w.ts[0] = __builtin_amdgcn_s_memrealtime();
  wave_lds_fence();
  const f4* q4 = reinterpret_cast<const f4*>(qs);
  // sequential dot of q with the HS floats at base + i*stride4*4 (piece i); the pieces are read
  // RA at a time ahead of the chain (an LDS read's latency per step otherwise)
  constexpr int RA = 8;
  auto dot_lds = [&](const float* base, int stride4) {
    float sc = 0.f;
    for (int i0 = 0; i0 < PC; i0 += RA) {
      f4 k4[RA], qv[RA];
#pragma unroll
      for (int i = 0; i < RA; ++i) {
        k4[i] = reinterpret_cast<const f4*>(base)[(i0 + i) * stride4];
        qv[i] = q4[i0 + i];
      }
#pragma unroll
      for (int i = 0; i < RA; ++i) {
        sc = __fadd_rn(sc, __fmul_rn(qv[i].x, k4[i].x));
        sc = __fadd_rn(sc, __fmul_rn(qv[i].y, k4[i].y));
        sc = __fadd_rn(sc, __fmul_rn(qv[i].z, k4[i].z));
        sc = __fadd_rn(sc, __fmul_rn(qv[i].w, k4[i].w));
      }
    }
    return sc;
  };
  // this unit's scores, published as granules
  const float rs = sqrtf((float)HS);
  for (int t0 = k0; t0 < kc1; t0 += 64) {
    if (t0 > k0) issue_keys(t0);  // rounds past the first (contexts over 64 NG keys)
    dma_wait_all();
    const float sc = __fdiv_rn(dot_lds(win + 4 * lane, 64), rs);
    if (t0 + lane < kc1) st8_sc1(gs + t0 + lane, gran(w.tag_out, sc));
    wave_lds_fence();  // the window's reads are done before the next round lands in it
  }
  if (k1 == T && lane == 0) st8_sc1(gs + T - 1, gran(w.tag_out, __fdiv_rn(dot_lds(kn, 1), rs)));
  // every score of the head (the other units' granules)
  float mx = -__builtin_inff();
  for (int t = lane; t < T; t += 64) {
    const unsigned long long x = ld8_sc1(gs + t);
    const float sc = (unsigned)(x >> 32) == w.tag_out ? __uint_as_float((unsigned)x) : gran_wait(gs + t, w.tag_out, w.err, w.poll_long != 0);
    at[t] = sc;
    mx = fmaxf(mx, sc);
  }
  if (w.ts && lane == 0) w.ts[1] = __builtin_amdgcn_s_memrealtime();
  mx = wave_max_u(mx);  // exact (a maximum)
  wave_lds_fence();
  const unsigned chm = seqsum_magic(ch);
  for (int t = lane; t < T; t += 64) sa[seqsum_index_m(t, ch, chm)] = expf_libm_tab(__fsub_rn(at[t], mx), w.etab);
  wave_lds_fence();
  const float sum = T <= 512 ? wave_seqsum_short(sa, T) : T <= 4096 ? wave_seqsum_reg(sa, T, lane) : wave_seqsum(sa, T, lane);
  if (w.ts && lane == 0) w.ts[3] = __builtin_amdgcn_s_memrealtime();
  for (int t = lane; t < T; t += 64) at[t] = __fdiv_rn(sa[seqsum_index_m(t, ch, chm)], sum);
  wave_lds_fence();
  // this unit's columns: lane < CW owns column col0 + lane, a chain over t
  float o = 0.f;
  const int cl = lane < CW ? lane : 0;
  for (int r0 = 0; r0 < tc; r0 += rv) {
    const int n = min(rv, tc - r0);
    if (r0 > 0) {
      wave_lds_fence();  // the previous round's reads are done
      issue_rows(r0, n);
    }
    dma_wait_all();
    // batches of 16 rows: all their LDS reads issued, then chained (the compiler waits for every
    // LDS read before the first use, so a read-ahead across batches would not overlap)
    const int n4 = n & ~15;
    for (int u = 0; u < n4; u += 16) {
      f4 a4[4];
      float v16[16];
#pragma unroll
      for (int k = 0; k < 4; ++k) a4[k] = *reinterpret_cast<const f4*>(at + r0 + u + 4 * k);
#pragma unroll
      for (int k = 0; k < 16; ++k) v16[k] = vw[(u + k) * CW + cl];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        o = __fadd_rn(o, __fmul_rn(a4[k].x, v16[4 * k]));
        o = __fadd_rn(o, __fmul_rn(a4[k].y, v16[4 * k + 1]));
        o = __fadd_rn(o, __fmul_rn(a4[k].z, v16[4 * k + 2]));
        o = __fadd_rn(o, __fmul_rn(a4[k].w, v16[4 * k + 3]));
      }
    }
    for (int u = n4; u < n; ++u) o = __fadd_rn(o, __fmul_rn(at[r0 + u], vw[u * CW + cl]));
  }
  o = __fadd_rn(o, __fmul_rn(at[T - 1], vn[col0 + cl]));
  if (w.ts && lane == 0) w.ts[2] = __builtin_amdgcn_s_memrealtime();
  if (lane < CW) st8_sc1(w.gout + h * HS + col0 + lane, gran(w.tag_out, o));
  wave_lds_fence();  // the strip and window are rewritten by the next unit
}

// fp32 persistent step (batch 1): attn_unit with the keys in LDS windows.  attn_unit holds one
// 16-key chunk in registers per memory latency, so at long contexts a unit's key range (T / NS
// keys) is a chain of latencies (7B at position 2000: ~15 chunks, ~30 us per layer).  Here the
// unit's keys come in rounds of up to 64: K rows row-major (key l at kw[l * HS], read by its lane
// from piece l on: conflict-free) and V rows (vw[u * HS + c]) by LDS-DMA, all of a round requested
// at once — one latency per 64 keys; one lane per key for the scores, online softmax across rounds, a lane's VPL columns for
// the output.  Unit s of (b, h) takes the contiguous keys [T s / nact, T (s+1) / nact); the last
// row (T-1, written by this launch's QKV phase) comes from the granules.  Partials combine as in
// attn_unit (same records and tickets).  win: attn_win_floats(HS) floats of LDS.
__host__ __device__ constexpr int attn_win_floats(int hs) { return 2 * 64 * hs + 2 * hs; }

#ifndef ATTN_MERGE_LAST  // (0: key T-1 folded after the round; same-box A/B only)
#define ATTN_MERGE_LAST 1
#endif

// The key range of attn_unit_win's unit (b, h, split s): [k0, k1) of T keys, the cached ones
// [k0, ke); live = the unit has keys.
struct WinUnit {
  int b, h, s, T, nact, k0, k1, ke;
  bool live;
};
TL_DEVICE WinUnit win_unit(const AttnWaveParams& w, int unit) {
  const AttnParams& p = w.a;
  const int BH = w.B * p.n_heads;
  WinUnit u;
  u.s = unit / BH;
  const int bh = unit % BH;
  u.b = bh / p.n_heads;
  u.h = bh % p.n_heads;
  u.T = p.pos[u.b] + 1;
  u.nact = min(w.NS, (u.T + 15) / 16);  // live units for this (b, h): >= 16 keys each
  u.live = u.s < u.nact;
  u.k0 = (int)((long long)u.T * u.s / u.nact);
  u.k1 = (int)((long long)u.T * (u.s + 1) / u.nact);
  u.ke = min(u.k1, u.T - 1);  // row T-1 comes from the granules
  return u;
}

// The DMAs of one round of attn_unit_win: n K rows (or, with v, V rows) from t0 into the window.
// Units of more than one 64-key round issue exactly PC + 64 / RPI (= 2 PC) wave-instructions per
// round whatever n (lanes past n re-read row t0 into slots nothing reads), so the unit's waits can
// count them; a single-round unit issues only its n rows.
template <int HS>
TL_DEVICE void win_issue(const float* base, int kv_dim, int t0, int n, bool multi, float* dst, int lane) {
  constexpr int PC = HS / 4;     // 16-B pieces per row
  constexpr int RPI = 256 / HS;  // rows per 1-KiB DMA instruction
  const int kq = lane / PC, pc = lane % PC;
  const int ni = multi ? 64 / RPI : (n + RPI - 1) / RPI;
#pragma unroll 4
  for (int j = 0; j < ni; ++j) {
    const int kl = j * RPI + kq;  // this lane's row in the round
    if (multi || kl < n) dma16(base + (long long)(t0 + (kl < n ? kl : 0)) * kv_dim + 4 * pc, dst + j * 256);
  }
}

// A single-round unit's cached K/V rows (written by earlier launches) requested into its window
// ahead of the attention phase, while the QKV phase streams: issued at the phase start they
// queued behind the CU's own next-phase weight prefetch (~2 us at short contexts).  Returns
// whether it issued them (then attn_unit_win(..., pre = true) does not).
template <int HS>
TL_DEVICE bool attn_win_preissue(const AttnWaveParams& w, int unit, float* win, int lane) {
  const WinUnit u = win_unit(w, unit);
  if (!u.live || u.k0 >= u.ke || u.ke - u.k0 > 64) return false;
  const AttnParams& p = w.a;
  const int kvh = u.h / p.kv_mul;
  const float* kbase = p.kc + (long long)u.b * p.kv_b_stride + p.kv_l_off + (long long)kvh * HS;
  const float* vbase = p.vc + (long long)u.b * p.kv_b_stride + p.kv_l_off + (long long)kvh * HS;
  win_issue<HS>(kbase, p.kv_dim, u.k0, u.ke - u.k0, false, win, lane);
  win_issue<HS>(vbase, p.kv_dim, u.k0, u.ke - u.k0, false, win + 64 * HS, lane);
  return true;
}

template <int HS>
TL_DEVICE void attn_unit_win(const AttnWaveParams& w, int unit, float* win, int lane, bool pre = false) {
  constexpr int VPL = HS / 64;
  constexpr int PC = HS / 4;     // 16-B pieces per row
  constexpr int RPI = 256 / HS;  // V rows per 1-KiB DMA instruction
  const AttnParams& p = w.a;
  const WinUnit u = win_unit(w, unit);
  if (!u.live) return;
  const int s = u.s, b = u.b, h = u.h, T = u.T, nact = u.nact, k0 = u.k0, k1 = u.k1, ke = u.ke;
  const int bh = b * p.n_heads + h;
  const int kvh = h / p.kv_mul;
  const float* kbase = p.kc + (long long)b * p.kv_b_stride + p.kv_l_off + (long long)kvh * HS;
  const float* vbase = p.vc + (long long)b * p.kv_b_stride + p.kv_l_off + (long long)kvh * HS;
  float* kw = win;              // [64][HS]: the round's K rows, row-major
  float* vw = kw + 64 * HS;     // [64][HS]
  float* qs = vw + 64 * HS;     // q [HS]
  float* kn = qs + HS;          // k row T-1 [HS]
  // Units of more than one 64-key round (long contexts) issue a round's K and V rows as exactly
  // PC + 64 / RPI (= 2 PC) wave-instructions whatever its key count n (lanes past n re-read row
  // t0 into slots nothing reads), so the waits below can count them: the next round's K rows land
  // while this round's V rows are folded, its V rows while its scores are taken (K and V share no
  // LDS, one window of each).  A single-round unit (short contexts) issues only its n rows.
  // K rows whole, RPI per wave-instruction (coalesced 1-KiB pieces; a transposed image, one 16-B
  // piece of 64 rows per instruction, measured the same on one box: profiles/r04/attn_k_layout_
  // ab.json); the lane-per-key dot below walks its row from piece `lane` on, so the 16 lanes of a
  // read hit 16 different bank groups
  const bool multi = ke - k0 > 64;
  auto issue_k = [&](int t0, int n) { win_issue<HS>(kbase, p.kv_dim, t0, n, multi, kw, lane); };
  auto issue_v = [&](int t0, int n) { win_issue<HS>(vbase, p.kv_dim, t0, n, multi, vw, lane); };
  static_assert(64 / RPI == PC, "K and V rounds are the same instruction count");
  auto wait_all_but_round_half = [] {  // every DMA but the last PC instructions landed
    if constexpr (PC == 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  };
  if (k0 < ke && !pre) {  // the first round is in flight before q has arrived
    issue_k(k0, min(64, ke - k0));
    issue_v(k0, min(64, ke - k0));
  }
  // q, and the new k / v row if this unit holds it, from the QKV phase's granules
  const unsigned long long* gq = w.gqkv + (long long)b * (p.dim + 2 * p.kv_dim);
  const unsigned long long* srcq = gq + h * HS;
  const unsigned long long* srck = gq + p.dim + kvh * HS;
  const unsigned long long* srcv = gq + p.dim + p.kv_dim + kvh * HS;
  const bool last = k1 == T;
  // A single-round unit holding key T-1 takes its k / v rows as window row ke - k0 and folds all
  // its keys in one round (one max, one rescale); a separate fold of that key after the round was
  // one more dependent chain of LDS reads and wave reductions on the attention phase's critical path.
  const bool merge = ATTN_MERGE_LAST && last && !multi && ke - k0 < 64;
  float* kdst = merge ? kw + (ke - k0) * HS : kn;
  float vn[VPL];
  {
    unsigned long long g[3][VPL];
#pragma unroll
    for (int c = 0; c < VPL; ++c) {
      g[0][c] = ld8_sc1(srcq + lane * VPL + c);
      if (last) {
        g[1][c] = ld8_sc1(srck + lane * VPL + c);
        g[2][c] = ld8_sc1(srcv + lane * VPL + c);
      }
    }
#pragma unroll
    for (int c = 0; c < VPL; ++c) {
      qs[lane * VPL + c] = (unsigned)(g[0][c] >> 32) == w.tag_in ? __uint_as_float((unsigned)g[0][c])
                                                                  : gran_wait(srcq + lane * VPL + c, w.tag_in, w.err, w.poll_long != 0);
      if (last) {
        kdst[lane * VPL + c] = (unsigned)(g[1][c] >> 32) == w.tag_in ? __uint_as_float((unsigned)g[1][c])
                                                                      : gran_wait(srck + lane * VPL + c, w.tag_in, w.err, w.poll_long != 0);
        vn[c] = (unsigned)(g[2][c] >> 32) == w.tag_in ? __uint_as_float((unsigned)g[2][c])
                                                       : gran_wait(srcv + lane * VPL + c, w.tag_in, w.err, w.poll_long != 0);
      }
    }
    if (merge)  // (rows 0 .. ke - k0 - 1 are the DMAs' own)
#pragma unroll
      for (int c = 0; c < VPL; ++c) vw[(ke - k0) * HS + lane * VPL + c] = vn[c];
  }
  wave_lds_fence();
  if (w.ts && lane == 0) w.ts[0] = __builtin_amdgcn_s_memrealtime();  // (diagnostics: q / k / v granules in)
  const float rs = sqrtf((float)HS);
  const f4* q4 = reinterpret_cast<const f4*>(qs);
  float m = -3.402823466e+38f, l = 0.f;
  float o[VPL];
#pragma unroll
  for (int c = 0; c < VPL; ++c) o[c] = 0.f;
  // one lane's dot of q with the HS floats at base + i * stride4 * 4 (piece i); 4 partial sums
  auto dot = [&](const float* base, int stride4) {
    float a[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
    for (int i = 0; i < PC; ++i) a[i & 3] = dot4(q4[i], reinterpret_cast<const f4*>(base)[i * stride4], a[i & 3]);
    return (a[0] + a[1]) + (a[2] + a[3]);
  };
  // fold n scores (lane t: key t; lanes >= n: none) and their V rows (vrow(t)) into (m, l, o)
  auto fold = [&](float sc, int n, const float* vrows, int vstride) {
    const float my = lane < n ? __fdiv_rn(sc, rs) : -3.402823466e+38f;
    const float mn = fmaxf(m, wave_max_u(my));
    const float e = lane < n ? expf_libm_tab(__fsub_rn(my, mn), w.etab) : 0.f;
    const float scale = expf_libm_tab(__fsub_rn(m, mn), w.etab);
    l = fmaf(l, scale, wave_sum_u(e));
#pragma unroll
    for (int c = 0; c < VPL; ++c) o[c] *= scale;
    // keys in order; the V reads of 8 keys are issued together (one LDS latency per 8 keys, not
    // per key)
    int u = 0;
    for (; u + 8 <= n; u += 8) {
      float vv[8][VPL];
#pragma unroll
      for (int k = 0; k < 8; ++k)
#pragma unroll
        for (int c = 0; c < VPL; ++c) vv[k][c] = vrows[(u + k) * vstride + lane * VPL + c];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float a = lane_f(e, u + k);
#pragma unroll
        for (int c = 0; c < VPL; ++c) o[c] = fmaf(a, vv[k][c], o[c]);
      }
    }
    for (; u < n; ++u) {
      const float a = lane_f(e, u);
#pragma unroll
      for (int c = 0; c < VPL; ++c) o[c] = fmaf(a, vrows[u * vstride + lane * VPL + c], o[c]);
    }
    m = mn;
  };
  const int kend = merge ? ke + 1 : ke;  // the window's last key (merge: row ke - k0 is key T-1)
  for (int t0 = k0; t0 < kend; t0 += 64) {
    const int n = min(64, kend - t0);
    const bool more = t0 + 64 < ke;
    if (multi) wait_all_but_round_half();  // this round's K rows (its V rows may still be in flight)
    else dma_wait_all();
    if (w.ts && lane == 0 && t0 == k0) w.ts[4] = __builtin_amdgcn_s_memrealtime();  // (diagnostics: first K rows in)
    float sc;
    {  // key `lane`, pieces in the order lane, lane + 1, ... (mod PC)
      float a[4] = {0.f, 0.f, 0.f, 0.f};
      const f4* kr = reinterpret_cast<const f4*>(kw + HS * lane);
#pragma unroll 8
      for (int i = 0; i < PC; ++i) {
        const int pc = (i + lane) & (PC - 1);
        a[i & 3] = dot4(q4[pc], kr[pc], a[i & 3]);
      }
      sc = (a[0] + a[1]) + (a[2] + a[3]);
    }
    wave_lds_fence();  // the K window's reads are done before the next round lands in it
    if (w.ts && lane == 0 && t0 == k0) w.ts[5] = __builtin_amdgcn_s_memrealtime();  // (diagnostics: first scores)
    if (more) {
      issue_k(t0 + 64, min(64, ke - t0 - 64));
      wait_all_but_round_half();  // this round's V rows
    } else {
      dma_wait_all();
    }
    fold(sc, n, vw, HS);
    wave_lds_fence();  // the V window's reads are done
    if (more) issue_v(t0 + 64, min(64, ke - t0 - 64));
  }
  if (w.ts && lane == 0) w.ts[1] = __builtin_amdgcn_s_memrealtime();  // (diagnostics: cached keys folded)
  if (last && !merge) {  // key T-1: every lane computes its score (one key), lane 0's counts
    const float sc = dot(kn, 1);
    // fold one key whose V row is vn (in registers): the same arithmetic inline
    const float my = lane < 1 ? __fdiv_rn(sc, rs) : -3.402823466e+38f;
    const float mn = fmaxf(m, wave_max_u(my));
    const float e0 = expf_libm_tab(__fsub_rn(lane_f(my, 0), mn), w.etab);
    const float scale = expf_libm_tab(__fsub_rn(m, mn), w.etab);
    l = fmaf(l, scale, e0);
#pragma unroll
    for (int c = 0; c < VPL; ++c) o[c] = fmaf(e0, vn[c], o[c] * scale);
    m = mn;
  }
  wave_lds_fence();  // the window is rewritten by the block's next unit
  if (w.ts && lane == 0) w.ts[3] = __builtin_amdgcn_s_memrealtime();  // (diagnostics: unit computed)
  if (nact == 1) {
#pragma unroll
    for (int c = 0; c < VPL; ++c) o[c] = __fdiv_rn(o[c], l);
    publish_head<HS>(w, b, h, o, lane);
    if (w.ts && lane == 0) w.ts[2] = __builtin_amdgcn_s_memrealtime();  // (diagnostics: head published)
    return;
  }
  // publish this unit's partial (write-through), drain, take a ticket; the last unit combines
  float* rec = p.part + ((long long)bh * w.NS + s) * (HS + 4);
#pragma unroll
  for (int c = 0; c < VPL; ++c) st_sc1(rec + lane * VPL + c, o[c]);
  if (lane == 0) {
    st_sc1(rec + HS, m);
    st_sc1(rec + HS + 1, l);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  unsigned ticket = 0;
  if (lane == 0) ticket = __hip_atomic_fetch_add(w.cnt + bh, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  ticket = (unsigned)__builtin_amdgcn_readfirstlane((int)ticket);
  if (ticket != (unsigned)(nact - 1)) return;
  const float* recs = p.part + (long long)bh * w.NS * (HS + 4);
  const int kl = lane < nact ? lane : nact - 1;
  const float mk = ld_sc1(recs + kl * (HS + 4) + HS);
  const float lk = ld_sc1(recs + kl * (HS + 4) + HS + 1);
  float ov[kMaxNS][VPL];
#pragma unroll
  for (int k = 0; k < kMaxNS; ++k) {
    const int kk = k < nact ? k : nact - 1;
#pragma unroll
    for (int c = 0; c < VPL; ++c) ov[k][c] = ld_sc1(recs + kk * (HS + 4) + lane * VPL + c);
  }
  const float M = wave_max_u(lane < nact ? mk : -3.402823466e+38f);
  const float sk = lane < nact ? expf_libm_tab(__fsub_rn(mk, M), w.etab) : 0.f;
  const float L = wave_sum_u(lk * sk);
  float acc[VPL];
#pragma unroll
  for (int c = 0; c < VPL; ++c) acc[c] = 0.f;
#pragma unroll
  for (int k = 0; k < kMaxNS; ++k) {
    const float a = lane_f(sk, k);
#pragma unroll
    for (int c = 0; c < VPL; ++c) acc[c] = fmaf(ov[k][c], a, acc[c]);
  }
#pragma unroll
  for (int c = 0; c < VPL; ++c) acc[c] = __fdiv_rn(acc[c], L);
  publish_head<HS>(w, b, h, acc, lane);
  if (w.ts && lane == 0) w.ts[2] = __builtin_amdgcn_s_memrealtime();  // (diagnostics: head combined, published)
  if (lane == 0) __hip_atomic_store(w.cnt + bh, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// out[b][h*hs + i] = sum_s o_s[i] e^{m_s-M} / sum_s l_s e^{m_s-M}
template <int kUnused = 0>
__global__ void __launch_bounds__(256) attn_combine_kernel(AttnParams p) {
  keep_implicit_args();  // common.hpp: rocprofv3 --pmc needs the hidden kernargs
  const int h = blockIdx.x, b = blockIdx.y;
  const int hs = p.head_size;
  const int T = p.pos[b] + 1;
  int t0, t1;
  split_range(T, p.nsplit, p.min_chunk, 0, t0, t1);
  if (t1 == T) return;  // single split covered everything and wrote `out` directly
  const float* base = p.part + ((long long)b * p.n_heads + h) * p.nsplit * (hs + 4);
  float M = -3.402823466e+38f;
  int ns = 0;
  for (int s = 0; s < p.nsplit; ++s) {
    int a0, a1;
    split_range(T, p.nsplit, p.min_chunk, s, a0, a1);
    if (a0 >= a1) break;
    M = fmaxf(M, base[s * (hs + 4) + hs]);
    ns = s + 1;
  }
  float L = 0.f;
  for (int s = 0; s < ns; ++s) L += base[s * (hs + 4) + hs + 1] * expf_libm(base[s * (hs + 4) + hs] - M);
  for (int i = threadIdx.x; i < hs; i += blockDim.x) {
    float acc = 0.f;
    for (int s = 0; s < ns; ++s) acc = fmaf(base[s * (hs + 4) + i], expf_libm(base[s * (hs + 4) + hs] - M), acc);
    p.out[(long long)b * p.dim + h * hs + i] = acc / L;
  }
}

}  // namespace tl
