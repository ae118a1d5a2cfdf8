// forward.hip — the fused decode step (thaDNN_s_forward_batch) and the native decoder.
//
// Reference: src/thaDNN.cpp:13-81 issues, per layer, 9 + 4*B launches (RMSNorm,
// 7 GEMVs that each re-read the weights once per sequence, per-sequence RoPE /
// residual / SwiGLU launches, 3 attention kernels) plus a hipMalloc/hipFree and
// B blocking D2D copies per step.  Here one step is, per layer:
//
//   1. QKV    : RMSNorm(att) prologue + [Wq;Wk;Wv] GEMV + RoPE + KV-cache write
//               (layer 0 also folds the embedding lookup)
//   2. ATTN   : scores + softmax + V-sum, one launch (+ combine when keys split)
//   3. WO     : Wo GEMV + residual add
//   4. FFN_UP : RMSNorm(ffn) prologue + [W1;W3] GEMV + SwiGLU
//   5. FFN_DN : W2 GEMV + residual add
//
// then RMSNorm(final) + classifier, and (greedy loop only) an argmax that feeds
// the next token and position back on the device.  Every launch reads every
// weight byte once for all B sequences.  Nothing allocates or synchronises
// inside a step, so a step can be captured into a hipGraph.
#include <math.h>
#include <string.h>
#include <algorithm>
#include <atomic>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <tuple>
#include <vector>
#include <string>
#include "../../include/thaDNN.hpp"
#include "../../include/thallama.h"
#include "../../include/hip_helper.hpp"
#include "../../include/thaQ8.hpp"
#include "attention.hpp"
#include "gemv_dispatch.hpp"
#include "q8_dispatch.hpp"
#include "persist.hpp"
#include "prefill.hpp"
#include "api_lock.hpp"

using tl::f4;

static thread_local std::string g_last_error;
extern "C" const char* thallama_last_error(void) { return g_last_error.c_str(); }

#define TL_TRY(cmd)                                                                   \
  do {                                                                                \
    hipError_t e_ = (cmd);                                                            \
    if (e_ != hipSuccess) {                                                           \
      g_last_error = std::string(#cmd) + ": " + hipGetErrorString(e_) + " @" +        \
                     std::to_string(__LINE__);                                        \
      return (int)e_;                                                                 \
    }                                                                                 \
  } while (0)

// ------------------------------------------------------------------ concurrent callers
// Every per-call operation of a decoder is ordered on its own non-blocking stream (async copies
// and memsets + hipStreamSynchronize; workspaces allocated at creation).  What must stay
// device-wide — allocation, frees and zeroing at create/destroy, the diagnostics' one-time buffers,
// kernel attributes — and every capture (begin .. instantiate) run under tl::api_mu()
// (api_lock.hpp), so no such call can fall inside another thread's capture.
using tl::ApiLock;
using tl::api_mu;

// ------------------------------------------------------------------ argmax + advance
// next = argmax(logits[b]) with lowest-index ties (sample_argmax, reference
// src/llama.cpp:275-286); then tok[b] = next, out[b*cap + pos[b]] = next, pos[b]++.
// One 1024-thread block per sequence; float4 loads, 8 in flight per thread, then a
// (value, index) reduction that keeps the lower index on ties.
__global__ void __launch_bounds__(1024) k_argmax_advance(const float* logits, int V, int* tok, int* pos,
                                                         int* out, int cap) {
  tl::keep_implicit_args();  // common.hpp: rocprofv3 --pmc needs the hidden kernargs
  __shared__ unsigned long long red[16];
  const int b = blockIdx.x;
  const float* l = logits + (long long)b * V;
  float bv = -INFINITY;
  int bi = 0x7FFFFFFF;
  const bool vec = ((V & 3) == 0) && (((uintptr_t)l & 15) == 0);
  if (vec) {
    const f4* l4 = reinterpret_cast<const f4*>(l);
    const int n4 = V >> 2;
    for (int i0 = threadIdx.x; i0 < n4; i0 += 1024 * 8) {
      f4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + u * 1024;
        v[u] = i < n4 ? l4[i] : f4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = 4 * (i0 + u * 1024);
        if (v[u].x > bv) { bv = v[u].x; bi = i; }
        if (v[u].y > bv) { bv = v[u].y; bi = i + 1; }
        if (v[u].z > bv) { bv = v[u].z; bi = i + 2; }
        if (v[u].w > bv) { bv = v[u].w; bi = i + 3; }
      }
    }
  } else {
    for (int i = threadIdx.x; i < V; i += 1024)
      if (l[i] > bv) { bv = l[i]; bi = i; }
  }
  // a thread's indices increase along its stream, so strict '>' kept its lowest; across
  // threads the packed key orders by value, then by lower index
  unsigned long long best = bi == 0x7FFFFFFF ? 0ull : tl::argmax_pack(bv, bi);
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long other = __shfl_xor(best, o, 64);
    best = other > best ? other : best;
  }
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 16; ++w) best = red[w] > best ? red[w] : best;
    // all-NaN logits: sample_argmax keeps index 0
    const int next = best ? (int)(0xFFFFFFFFu - (uint32_t)(best & 0xFFFFFFFFull)) : 0;
    const int p = pos[b];
    if (out && p < cap) out[(long long)b * cap + p] = next;
    tok[b] = next;
    pos[b] = p + 1;
  }
}

// ------------------------------------------------------------------ decoder
static constexpr int kAttnChunk = 32;  // keys per attention wave unit
// batched prefill (thallama_decoder_prefill): tokens per chunk and attention splits per token
static constexpr int kPrefillChunk = 128;
static constexpr int kPrefillMaxSplits = 16;
static constexpr int kPrefillQ8Chunk = 8;  // int8: the exact batched kernels take up to 8 sequences

struct thallama_decoder {
  Config cfg;
  TransformerWeights w;
  RunState s;
  int B = 1;
  int dev = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  int dim, hidden, L, H, kv_dim, kv_mul, hs, V, S;
  // workspace
  int* tok_d = nullptr;
  int* pos_d = nullptr;
  int* out_d = nullptr;  // [B][S] greedy tokens by position
  int* tok_h = nullptr;  // pinned staging
  int* pos_h = nullptr;
  int* nxt_h = nullptr;  // pinned: argmax ids of a greedy step
  unsigned* perr_h = nullptr;  // pinned: the persistent step's error word, read back on d->stream
  float* lg_pin = nullptr;     // pinned staging of a step's logits for pageable caller buffers (logits_dst)
  const float* lg_last = nullptr;
  bool lg_last_pinned = false;
  unsigned lg_checks = 0;      // steps since the last pointer query (re-queried every 256)
  hipEvent_t ev_stage = nullptr;  // pipeline stage done (thallama_decoder_stage)
  // layer streaming (thaDNN_s_forward_70B): the H2D copy stream and, per staging slot, layer
  // copied / layer consumed events
  hipStream_t copy_stream = nullptr;
  hipEvent_t ev_copied[2] = {nullptr, nullptr}, ev_used[2] = {nullptr, nullptr};
  bool err_pending = false;    // perr_h holds the word of launches not yet checked
  float2* rope_d = nullptr;
  float* xn_d = nullptr;        // [<=16][dim] normed rows for the matrix-core GEMV (batch >= 2)
  float* ssq_d = nullptr;       // [B][dim/16] per-tile sums of squares carried from Wo / W2 to the next norm
  bool ssq_carry = false;       // this step carries them (ssq_carry_ok)
  signed char* xq_d = nullptr;  // int8 batched: activations quantised once per launch [8][max(dim, hidden)]
  float* xqs_d = nullptr;       //   and their group scales
  float* mpart_d = nullptr;     // matrix-core GEMV split-K partial tiles
  unsigned* mcnt_d = nullptr;   //   and their tickets
  float* part_d = nullptr;      // attention partials [B][H][<=16 units][hs+4]
  unsigned* cnt_d = nullptr;    // attention combine tickets [B][H]
  bool q8 = false;              // int8 (runq Q8_0) weights in w8; w then holds only norms + embedding
  bool q8x = false;             // int8 multi-launch steps in runq's arithmetic order (q8_exact.hip)
  float* q8att_d = nullptr;     //   their attention scores [B][H][S]
  Q8TransformerWeights w8 = {};
  int nsplit = 1;
  bool nt = true;
  bool use_graph = false;
  bool profile = false;
  bool persist = true;          // requested (THALLAMA_OPT_PERSISTENT)
  bool pfault = false;          // test hook: the next persistent launch loses block 0
  bool pasync = false;          // an asynchronous greedy call ran persistent launches not yet checked
  // [lc]: lc = 1 is the persistent step's long-context instantiation (persistent_long_ctx)
  hipGraphExec_t exec[2] = {};      // one greedy step (step + argmax), replayed per token
  hipGraphExec_t exec_fwd[2] = {};  // one forward step (no argmax), replayed by decoder_forward
  // persistent one-launch step (persist.hip)
  int ncu = 0;
  unsigned* psync = nullptr;    // [kPSyncWords shards][L*H tickets] (zeroed per launch), err, seq
  size_t psync_zero = 0;        // words zeroed before every launch
  unsigned long long* pbmax = nullptr;
  unsigned long long* pgran = nullptr;  // hand-off granules: x | xb | hb | qkv
  const signed char* pq8w[7] = {};       // int8: layer-0 int8 block of wq wk wv wo w1 w2 w3
  long long pq8ls[7] = {};                // and the byte stride between layers
  bool pok = false;             // shape supported
  bool pk = false;              // 8 sequences: the K-split persistent step is supported (persist_k.hip)
  bool ksplit = true;           //   and taken when the step is persistent (THALLAMA_OPT_KSPLIT)
  unsigned long long* pkgran = nullptr;  // its hand-off area
  unsigned long long* ptrace = nullptr;  // optional timeline of the persistent step
  size_t ptrace_n = 0;
  // batched prompt processing (prefill.hip) for kPrefillChunk tokens, allocated at creation
  float *pf_x = nullptr, *pf_xn = nullptr, *pf_q = nullptr, *pf_xb = nullptr, *pf_hb = nullptr;
  float* pf_part = nullptr;
  unsigned* pf_cnt = nullptr;
  int *pf_tok = nullptr, *pf_pos = nullptr;
  int* pf_tok_h = nullptr;      // pinned staging of a chunk's prompt tokens
  float* pf_att = nullptr;      // int8 prefill: exact attention scores [8][H][S]
  std::string pwhy;             // why not
  // profiling
  std::vector<hipEvent_t> ev_pool;
  std::vector<std::pair<int, int>> ev_marks;  // (class, event index of start)
  size_t ev_next = 0;
  double prof_ms[THALLAMA_K_COUNT] = {0};
  long long prof_n[THALLAMA_K_COUNT] = {0};
};

// Options, buffers and the persistent path's state are baked into the captured graphs: drop them
// (recaptured on next use).
static void drop_graphs(thallama_decoder* d) {
  for (int i = 0; i < 2; ++i) {
    if (d->exec[i]) (void)hipGraphExecDestroy(d->exec[i]);
    if (d->exec_fwd[i]) (void)hipGraphExecDestroy(d->exec_fwd[i]);
    d->exec[i] = d->exec_fwd[i] = nullptr;
  }
}

static int prof_begin(thallama_decoder* d) {
  if (!d->profile) return -1;
  if (d->ev_next + 2 > d->ev_pool.size()) {
    for (int i = 0; i < 512; ++i) {
      hipEvent_t e;
      if (hipEventCreate(&e) != hipSuccess) return -1;
      d->ev_pool.push_back(e);
    }
  }
  int i = (int)d->ev_next;
  d->ev_next += 2;
  (void)hipEventRecord(d->ev_pool[i], d->stream);
  return i;
}

static void prof_end(thallama_decoder* d, int kclass, int i) {
  if (i < 0) return;
  (void)hipEventRecord(d->ev_pool[i + 1], d->stream);
  d->ev_marks.push_back({kclass, i});
}

static void prof_collect(thallama_decoder* d) {
  if (d->ev_marks.empty()) return;
  (void)hipStreamSynchronize(d->stream);
  for (auto& m : d->ev_marks) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, d->ev_pool[m.second], d->ev_pool[m.second + 1]) == hipSuccess) {
      d->prof_ms[m.first] += ms;
      d->prof_n[m.first] += 1;
    }
  }
  d->ev_marks.clear();
  d->ev_next = 0;
}

static int auto_splits(const thallama_decoder* d) {
  // Enough (head, seq, split) blocks to cover the 256 CUs, at most 16 splits
  // (THALLAMA_OPT_ATTN_SPLITS overrides per decoder, for measurements).
  // batches aim for 8 waves per CU: a unit walks its keys one 32-key chunk (one memory latency)
  // after another, so at B = 8 x 32 heads one unit per (b, h) left 256-step decodes latency-bound
  // (fp32 7B B=8: splits 1 / 2 / 4 / 8 / 16 -> 1366 / 1405 / 1414 / 1417 / 1417 tok/s)
  const int target = d->B == 1 ? 256 : 2048;
  int blocks = d->H * d->B;
  int ns = (target + blocks - 1) / blocks;
  if (ns < 1) ns = 1;
  if (ns > 16) ns = 16;
  return ns;
}

// Hand-off granules of the persistent step: x | xb | hb | q k v | int8 attention scores [H][S]
// (batch 1); B rows of each of the first four for the batched step (persist_b.hip).
static size_t granule_count(const thallama_decoder* d) {
  if (d->B > 1) return (size_t)d->B * (3 * d->dim + d->hidden + 2 * d->kv_dim) + 2;
  return (size_t)3 * d->dim + d->hidden + 2 * d->kv_dim + (size_t)d->H * d->S + 2;
}

// The batched persistent step (persist_b.hip) is prepared for 2..8 sequences and taken BY DEFAULT
// for up to kBatchPersistDefaultMax of them (THALLAMA_OPT_PERSISTENT selects it, or the
// multi-launch step, per decoder).  7B fp32 ms/step, persistent vs multi-launch
// (profiles/r03/batch_persist_ab.json): B=2 4.69 vs 5.30, B=3 4.94 vs 7.04, B=4 5.21 vs 5.35, B=6
// 5.90 vs 5.59, B=8 6.57 vs 5.63 — past 4 sequences the all-gather hand-off of every phase's input
// to every CU (B x K x 8 B of granules per CU per phase, 1.5 MB per layer at B=8) costs more than
// the launches it saves; the matrix-core multi-launch kernels read K-split slices.
constexpr int kBatchPersistDefaultMax = 4;

// Shapes the batched prefill handles (head size 64/128/256, rows in multiples of 32).
static bool prefill_shape_ok(const thallama_decoder* d) {
  return (d->hs == 64 || d->hs == 128 || d->hs == 256) && d->dim % 32 == 0 && d->hidden % 32 == 0;
}

extern "C" int thallama_decoder_create(thallama_decoder** out, const Config* cfg, const TransformerWeights* w,
                                       const RunState* s, int batch, hipStream_t stream) {
  if (!out || !cfg || !w || !s || batch <= 0) {
    g_last_error = "thallama_decoder_create: invalid argument";
    return (int)hipErrorInvalidValue;
  }
  const Config& c = *cfg;
  const int hs_ = c.n_heads > 0 ? c.dim / c.n_heads : 0;
  if (c.dim <= 0 || c.n_heads <= 0 || c.n_kv_heads <= 0 || c.dim % c.n_heads || c.n_heads % c.n_kv_heads ||
      hs_ < 8 || hs_ > 256 || (hs_ & (hs_ - 1)) || c.seq_len <= 0) {
    g_last_error = "thallama_decoder_create: unsupported config (head_size must be a power of two in [8, 256])";
    return (int)hipErrorInvalidValue;
  }
  thallama_decoder* d = new thallama_decoder();
  d->cfg = c;
  d->cfg.vocab_size = c.vocab_size < 0 ? -c.vocab_size : c.vocab_size;
  d->w = *w;
  d->s = *s;
  d->B = batch;
  d->dim = c.dim;
  d->hidden = c.hidden_dim;
  d->L = c.n_layers;
  d->H = c.n_heads;
  d->hs = c.dim / c.n_heads;
  d->kv_dim = c.dim * c.n_kv_heads / c.n_heads;
  d->kv_mul = c.n_heads / c.n_kv_heads;
  d->V = d->cfg.vocab_size;
  d->S = c.seq_len;
  ApiLock lock(api_mu());
  TL_TRY(hipGetDevice(&d->dev));
  if (stream) {
    d->stream = stream;
  } else {
    TL_TRY(hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking));
    d->own_stream = true;
  }
  TL_TRY(hipMalloc(&d->tok_d, sizeof(int) * batch));
  TL_TRY(hipMalloc(&d->pos_d, sizeof(int) * batch));
  TL_TRY(hipMalloc(&d->out_d, sizeof(int) * (size_t)batch * d->S));
  TL_TRY(hipHostMalloc(&d->tok_h, sizeof(int) * batch, hipHostMallocDefault));
  TL_TRY(hipHostMalloc(&d->pos_h, sizeof(int) * batch, hipHostMallocDefault));
  TL_TRY(hipHostMalloc(&d->nxt_h, sizeof(int) * batch, hipHostMallocDefault));
  // RoPE table with the reference's exact host formula (src/seq.cpp:88-92), so the
  // device rotation uses bit-identical cos/sin.
  std::vector<float2> rope((size_t)d->S * (d->hs / 2));
  for (int p = 0; p < d->S; ++p)
    for (int hd = 0; hd < d->hs; hd += 2) {
      float freq = 1.0f / powf(10000.0f, hd / (float)d->hs);
      float val = p * freq;
      rope[(size_t)p * (d->hs / 2) + hd / 2] = make_float2(cosf(val), sinf(val));
    }
  TL_TRY(hipMalloc(&d->rope_d, rope.size() * sizeof(float2)));
  TL_TRY(hipMemcpy(d->rope_d, rope.data(), rope.size() * sizeof(float2), hipMemcpyHostToDevice));
  d->nsplit = auto_splits(d);
  if (batch >= 2) {
    const size_t nblk = (size_t)tl::mfma_target_blocks();
    TL_TRY(hipMalloc(&d->xn_d, sizeof(float) * (size_t)(batch < 16 ? batch : 16) * d->dim));
    TL_TRY(hipMalloc(&d->ssq_d, sizeof(float) * (size_t)batch * ((d->dim + 15) / 16)));
    TL_TRY(hipMemset(d->ssq_d, 0, sizeof(float) * (size_t)batch * ((d->dim + 15) / 16)));
    TL_TRY(hipMalloc(&d->mpart_d, sizeof(float) * nblk * 2 * 256));
    TL_TRY(hipMalloc(&d->mcnt_d, sizeof(unsigned) * nblk));
    TL_TRY(hipMemset(d->mcnt_d, 0, sizeof(unsigned) * nblk));
  }
  {
    const size_t nsmax = (size_t)((d->S + kAttnChunk - 1) / kAttnChunk);
    const size_t recs = (size_t)batch * d->H * (nsmax > 16 ? nsmax : 16);
    TL_TRY(hipMalloc(&d->part_d, sizeof(float) * recs * (d->hs + 4)));
    TL_TRY(hipMalloc(&d->cnt_d, sizeof(unsigned) * (size_t)batch * d->H));
    TL_TRY(hipMemset(d->cnt_d, 0, sizeof(unsigned) * (size_t)batch * d->H));
  }
  // weights far beyond the 256 MiB Infinity Cache stream once per step: nt loads
  const double wbytes = 4.0 * ((double)d->L * (2.0 * d->dim * d->dim + 2.0 * d->dim * d->kv_dim +
                                               3.0 * d->dim * d->hidden) + (double)d->V * d->dim);
  d->nt = wbytes > 1024.0 * 1024.0 * 1024.0;
  // persistent step: batch 1, fp32 (decided again for int8 in _create_q8)
  TL_TRY(hipDeviceGetAttribute(&d->ncu, hipDeviceAttributeMultiprocessorCount, d->dev));
  if (batch == 1) {  // measurement only: a smaller batch-1 persistent grid (a multiple of 8 blocks)
    const char* e = getenv("THALLAMA_PERSIST_GRID");
    const int g = e ? atoi(e) : 0;
    if (g >= 8 && g % 8 == 0 && g < d->ncu) d->ncu = g;
  }
  {
    tl::PStep ps = {};
    ps.dim = d->dim; ps.hid = d->hidden; ps.kvd = d->kv_dim; ps.hs = d->hs; ps.NS = d->nsplit;
    ps.L = d->L; ps.H = d->H; ps.S = d->S; ps.V = d->V; ps.B = batch;
    const char* why = nullptr;
    if (batch == 1) {
      d->pok = tl::persistent_prepare(ps, d->ncu, &why);
    } else if (batch <= 8) {
      d->pok = tl::persistent_prepare_b(ps, d->ncu, &why);
      d->persist = batch <= kBatchPersistDefaultMax;
      if (batch == 8) {
        // the K-split step (persist_k.hip) is the persistent step at 8 sequences where its shape is
        // instantiated, but not the default: 7B fp32 1374-1376 vs 1438 tok/s multi-launch (positions
        // 0..255), 974-976 vs 1007 at 1792..2047, same box; THALLAMA_KSPLIT=1
        // in the environment selects it at creation (THALLAMA_OPT_PERSISTENT per decoder)
        tl::PStep pk = ps;
        const char* kwhy = nullptr;
        d->pk = tl::persistent_prepare_k(pk, d->ncu, &kwhy);
        if (d->pk) {
          d->pok = true;
          const char* ev = getenv("THALLAMA_KSPLIT");
          d->persist = ev && ev[0] == '1';
        }
      }
    } else {
      why = "batch > 8";
    }
    if (!d->pok && why) d->pwhy = why;
  }
  if (!d->mpart_d) {  // split-K scratch of the matrix-core GEMV (batch 1: prefill's short chunks)
    const size_t nblk = (size_t)tl::mfma_target_blocks();
    TL_TRY(hipMalloc(&d->mpart_d, sizeof(float) * nblk * 2 * 256));
    TL_TRY(hipMalloc(&d->mcnt_d, sizeof(unsigned) * nblk));
    TL_TRY(hipMemset(d->mcnt_d, 0, sizeof(unsigned) * nblk));
  }
  TL_TRY(hipHostMalloc(&d->perr_h, sizeof(unsigned), hipHostMallocDefault));
  TL_TRY(hipEventCreateWithFlags(&d->ev_stage, hipEventDisableTiming));
  *d->perr_h = 0;
  if (prefill_shape_ok(d)) {  // batched prompt processing (thallama_decoder_prefill)
    const size_t CH = kPrefillChunk, dim = d->dim, hid = d->hidden;
    TL_TRY(hipMalloc(&d->pf_x, sizeof(float) * CH * dim));
    TL_TRY(hipMalloc(&d->pf_xn, sizeof(float) * CH * (dim > hid ? dim : hid)));
    TL_TRY(hipMalloc(&d->pf_q, sizeof(float) * CH * dim));
    TL_TRY(hipMalloc(&d->pf_xb, sizeof(float) * CH * dim));
    TL_TRY(hipMalloc(&d->pf_hb, sizeof(float) * CH * hid));
    TL_TRY(hipMalloc(&d->pf_part, sizeof(float) * CH * d->H * kPrefillMaxSplits * (d->hs + 4)));
    TL_TRY(hipMalloc(&d->pf_cnt, sizeof(unsigned) * CH * d->H));
    TL_TRY(hipMemset(d->pf_cnt, 0, sizeof(unsigned) * CH * d->H));
    TL_TRY(hipMalloc(&d->pf_tok, sizeof(int) * (size_t)d->S));
    TL_TRY(hipMalloc(&d->pf_pos, sizeof(int) * CH));
    TL_TRY(hipHostMalloc(&d->pf_tok_h, sizeof(int) * (size_t)d->S, hipHostMallocDefault));
  }
  if (d->pok) {
    d->psync_zero = tl::kPSyncWords + (((size_t)d->L * d->H * batch + 3) & ~(size_t)3);
    TL_TRY(hipMalloc(&d->psync, sizeof(unsigned) * (d->psync_zero + 32)));
    TL_TRY(hipMemset(d->psync, 0, sizeof(unsigned) * (d->psync_zero + 32)));
    TL_TRY(hipMalloc(&d->pbmax, sizeof(unsigned long long) * d->ncu * (batch > 1 ? 8 : 1)));
    const size_t ng = granule_count(d);
    TL_TRY(hipMalloc(&d->pgran, sizeof(unsigned long long) * ng));
    TL_TRY(hipMemset(d->pgran, 0, sizeof(unsigned long long) * ng));
  }
  if (d->pk) {
    tl::PStep ps = {};
    ps.dim = d->dim; ps.hid = d->hidden; ps.kvd = d->kv_dim; ps.V = d->V;
    const size_t nk = (size_t)tl::persistent_k_granules(ps, d->ncu);
    TL_TRY(hipMalloc(&d->pkgran, sizeof(unsigned long long) * nk));
    TL_TRY(hipMemset(d->pkgran, 0, sizeof(unsigned long long) * nk));
  }
  *out = d;
  return 0;
}

extern "C" void thallama_decoder_destroy(thallama_decoder* d) {
  if (!d) return;
  (void)hipStreamSynchronize(d->stream);
  ApiLock lock(api_mu());
  drop_graphs(d);
  for (auto e : d->ev_pool) (void)hipEventDestroy(e);
  if (d->ev_stage) (void)hipEventDestroy(d->ev_stage);
  for (int i = 0; i < 2; ++i) {
    if (d->ev_copied[i]) (void)hipEventDestroy(d->ev_copied[i]);
    if (d->ev_used[i]) (void)hipEventDestroy(d->ev_used[i]);
  }
  if (d->copy_stream) (void)hipStreamDestroy(d->copy_stream);
  (void)hipFree(d->tok_d);
  (void)hipFree(d->pos_d);
  (void)hipFree(d->out_d);
  (void)hipHostFree(d->tok_h);
  (void)hipHostFree(d->pos_h);
  (void)hipHostFree(d->nxt_h);
  (void)hipHostFree(d->perr_h);
  if (d->lg_pin) (void)hipHostFree(d->lg_pin);
  (void)hipHostFree(d->pf_tok_h);
  (void)hipFree(d->rope_d);
  (void)hipFree(d->xn_d);
  (void)hipFree(d->ssq_d);
  (void)hipFree(d->mpart_d);
  (void)hipFree(d->xq_d);
  (void)hipFree(d->q8att_d);
  (void)hipFree(d->xqs_d);
  (void)hipFree(d->mcnt_d);
  (void)hipFree(d->part_d);
  (void)hipFree(d->cnt_d);
  (void)hipFree(d->psync);
  (void)hipFree(d->pbmax);
  (void)hipFree(d->pgran);
  (void)hipFree(d->pkgran);
  (void)hipFree(d->ptrace);
  for (void* b : {(void*)d->pf_att, (void*)d->pf_x, (void*)d->pf_xn, (void*)d->pf_q, (void*)d->pf_xb, (void*)d->pf_hb,
                  (void*)d->pf_part, (void*)d->pf_cnt, (void*)d->pf_tok, (void*)d->pf_pos})
    (void)hipFree(b);
  if (d->own_stream) (void)hipStreamDestroy(d->stream);
  delete d;
}

extern "C" int thallama_decoder_set(thallama_decoder* d, int key, int value) {
  if (!d) return (int)hipErrorInvalidValue;
  switch (key) {
    case THALLAMA_OPT_NT_WEIGHTS: d->nt = value != 0; break;
    case THALLAMA_OPT_ATTN_SPLITS: d->nsplit = value <= 0 ? auto_splits(d) : (value > 16 ? 16 : value); break;
    case THALLAMA_OPT_USE_GRAPH: d->use_graph = value != 0; break;
    case THALLAMA_OPT_PROFILE: d->profile = value != 0; break;
    case THALLAMA_OPT_PERSISTENT: d->persist = value != 0; break;
    case THALLAMA_OPT_KSPLIT: d->ksplit = value != 0; break;
    case THALLAMA_OPT_PERSIST_FAULT:
      d->pfault = value != 0;
      drop_graphs(d);
      break;
    default: return (int)hipErrorInvalidValue;
  }
  drop_graphs(d);  // options are baked into a captured graph: recapture on next use
  return 0;
}

extern "C" hipStream_t thallama_decoder_stream(thallama_decoder* d) { return d ? d->stream : nullptr; }

// One GEMV launch: fp32 weights from p.W*, or — for an int8 decoder — the Q8_0 tensors
// t0..t2 (runq layout) through the int8 kernel (gemv_q8.hpp).
static hipError_t gemv(thallama_decoder* d, int mode, tl::GemvParams& p, const QuantizedTensor* t0,
                       const QuantizedTensor* t1, const QuantizedTensor* t2) {
  if (!d->q8) {
    p.mpart = d->mpart_d;
    p.mcnt = d->mcnt_d;
    return tl::launch_gemv(mode, p, d->stream, d->nt);
  }
  p.Q0 = t0 ? t0->q : nullptr;
  p.S0 = t0 ? t0->s : nullptr;
  p.Q1 = t1 ? t1->q : nullptr;
  p.S1 = t1 ? t1->s : nullptr;
  p.Q2 = t2 ? t2->q : nullptr;
  p.S2 = t2 ? t2->s : nullptr;
  p.gs = d->w8.group_size;
  if (!p.xq) {
    p.xq = d->xq_d;
    p.xqs = d->xqs_d;
  }
  if (d->q8x) return tl::launch_gemv_q8_exact(mode, p, d->stream, d->nt);
  return tl::launch_gemv_q8(mode, p, d->stream, d->nt);
}
#define Q8L(name) (d->q8 ? &d->w8.name[l] : nullptr)

// int8 decoder, 2..8 sequences, wave-level attention, runq groups of 64: attention stores its
// output row quantised as well (attention.hpp: store_head), the codes Wo's quantise pass would
// have produced from the same floats, so that pass is skipped
static int q8_attn_quant(const thallama_decoder* d) {
  return d->q8 && !d->q8x && d->xq_d && d->B >= 2 && d->B <= 8 && d->w8.group_size == 64 &&
         (d->hs == 64 || d->hs == 128 || d->hs == 256) && (d->dim % 64) == 0;
}

// Enqueue one decode step reading tok_d / pos_d; logits land in s.logits.
// fp32 batched steps on the matrix cores: the residual launches (Wo, W2) leave per-tile sums of
// squares of the residual stream and the next normed launch reduces them instead of running a
// norm prologue launch (gemv_mfma.hpp).  Both ends use the matrix-core kernel or neither (same nb).
// The sums are carried only when EVERY residual launch of the step takes one of the two kernels
// that write them (gemv_matrix_path, the launcher's own predicate): W2 has K = hidden, which can
// fail the matrix-path shape while K = dim passes (e.g. dim 512, hidden 1376), and a consumer
// would then read sums the previous step or another layer left.  Consumers that do not take the
// matrix path ignore ssq_in (the streaming kernels normalise from x).
static bool ssq_carry_ok(const thallama_decoder* d) {
  if (d->q8 || !d->ssq_d || (d->dim + 15) / 16 > 256) return false;  // (the kernel sums <= 256 tiles)
  for (int l = 0; l < d->L; ++l) {
    tl::GemvParams wo = {}, w2 = {};
    wo.W0 = d->w.wo + (long long)l * d->dim * d->dim;
    wo.K = d->dim; wo.n_items = d->dim; wo.nb = d->B; wo.x = d->s.xb; wo.x_stride = d->dim;
    w2.W0 = d->w.w2 + (long long)l * d->dim * d->hidden;
    w2.K = d->hidden; w2.n_items = d->dim; w2.nb = d->B; w2.x = d->s.hb; w2.x_stride = d->hidden;
    if (!tl::gemv_matrix_path(wo) || !tl::gemv_matrix_path(w2)) return false;
  }
  return true;
}
static void ssq_to_next_norm(const thallama_decoder* d, tl::GemvParams& p) {
  if (!d->ssq_carry) return;
  p.ssq_out = d->ssq_d;
  p.ssq_nt = (d->dim + 15) / 16;
}
static void norm_from_ssq(const thallama_decoder* d, tl::GemvParams& p) {
  if (!d->ssq_carry) return;
  p.ssq_in = d->ssq_d;
  p.ssq_nt = (d->dim + 15) / 16;
}

// Where a multi-launch step reads and writes: the decoder's RunState for its B sequences, or
// (prefill) a chunk of one sequence's prompt tokens as nb "sequences" at their own positions over
// that sequence's cache (kv_b_stride 0), with no classifier.
// One layer's fp32 weights.
struct LayerW {
  const float *rms_att, *wq, *wk, *wv, *wo, *rms_ffn, *w1, *w2, *w3;
};

struct StepIO {
  float *x, *xb, *q, *hb, *logits;  // logits == nullptr: layers only
  float *kc, *vc;
  long long kv_b_stride;
  int *tok, *pos;
  int nb;
  float* att;  // int8 exact attention scores [nb][H][S]
  bool embed = true;  // layer 0 reads the tokens' embedding rows (false: x already holds the input)
  // layer-streamed weights (thaDNN_s_forward_70B): layer l's pointers and the stream work around
  // it; null: the decoder's own TransformerWeights
  std::function<LayerW(int)> layer_w;
  std::function<int(int)> before_layer, after_layer;
};

static StepIO step_io(thallama_decoder* d) {
  const RunState& s = d->s;
  return StepIO{s.x, s.xb, s.q, s.hb, s.logits, s.key_cache, s.value_cache, (long long)d->L * d->S * d->kv_dim,
                d->tok_d, d->pos_d, d->B, d->q8att_d};
}

static LayerW layer_of(const TransformerWeights& w, int l, long long dim, long long kvd, long long hid) {
  const long long ll = l;
  return LayerW{w.rms_att_weight + ll * dim, w.wq + ll * dim * dim, w.wk + ll * dim * kvd, w.wv + ll * dim * kvd,
                w.wo + ll * dim * dim, w.rms_ffn_weight + ll * dim, w.w1 + ll * dim * hid, w.w2 + ll * dim * hid,
                w.w3 + ll * dim * hid};
}

static bool use_persist(const thallama_decoder* d) { return d->persist && d->pok; }
// The persistent step at 8 sequences is the K-split one (persist_k.hip) unless THALLAMA_OPT_KSPLIT
// is 0 (then persist_b.hip, if that shape check passed).
static bool use_ksplit(const thallama_decoder* d) { return use_persist(d) && d->pk && d->ksplit; }

static int enqueue_step_io(thallama_decoder* d, const StepIO& io) {
  const int dim = d->dim, hid = d->hidden, kvd = d->kv_dim, S = d->S;
  const long long kv_b_stride = io.kv_b_stride;
  const TransformerWeights& w = d->w;
  d->ssq_carry = ssq_carry_ok(d) && io.nb == d->B && !io.layer_w && io.embed;
  for (int l = 0; l < d->L; ++l) {
    const long long ll = l;
    if (io.before_layer) {
      const int r = io.before_layer(l);
      if (r) return r;
    }
    const LayerW lw = io.layer_w ? io.layer_w(l) : layer_of(w, l, dim, kvd, hid);
    // 1. QKV (+ embedding at layer 0)
    {
      tl::GemvParams p = {};
      p.W0 = lw.wq;
      p.W1 = lw.wk;
      p.W2 = lw.wv;
      p.K = dim;
      p.n_items = (dim + 2 * kvd) / 2;
      p.nb = io.nb;
      p.x = io.x;
      p.x_stride = dim;
      p.rms_w = lw.rms_att;
      p.xn = d->xn_d;
      if (l > 0) norm_from_ssq(d, p);
      if (l == 0 && io.embed) {
        p.tok = io.tok;
        p.emb = w.token_embedding_table;
        p.x_out = io.x;
      }
      p.y = io.q;
      p.y_stride = dim;
      p.pos = io.pos;
      p.kc = io.kc;
      p.vc = io.vc;
      p.kv_b_stride = kv_b_stride;
      p.kv_l_off = ll * S * kvd;
      p.dim = dim;
      p.kv_dim = kvd;
      p.head_size = d->hs;
      p.rope = d->rope_d;
      int ev = prof_begin(d);
      TL_TRY(gemv(d, tl::GM_QKV, p, Q8L(wq), Q8L(wk), Q8L(wv)));
      prof_end(d, THALLAMA_K_QKV, ev);
    }
    // 2. attention
    {
      tl::AttnParams a = {};
      a.q = io.q;
      a.kc = io.kc;
      a.vc = io.vc;
      a.kv_b_stride = kv_b_stride;
      a.kv_l_off = ll * S * kvd;
      a.pos = io.pos;
      a.out = io.xb;
      a.part = d->part_d;
      a.dim = dim;
      a.kv_dim = kvd;
      a.head_size = d->hs;
      a.n_heads = d->H;
      a.kv_mul = d->kv_mul;
      a.seq_len = S;
      a.nsplit = d->nsplit;
      a.min_chunk = 32;
      const int lpk = d->hs / 4;
      const size_t lds = 64 + (size_t)(S > 1024 ? S : 1024) * 4;
      int ev = prof_begin(d);
      if (d->q8x) {
        // int8 in runq's order: scores, softmax and the column chains of q8_exact.hip
        TL_TRY(tl::launch_attn_q8_exact(a, io.nb, io.att, d->stream));
      } else if (d->hs == 64 || d->hs == 128 || d->hs == 256) {
        // wave-level units, in-kernel combine (attention.hpp: attn_wave_kernel)
        tl::AttnWaveParams wp = {};
        wp.a = a;
        wp.cnt = d->cnt_d;
        wp.B = io.nb;
        const int max_chunks = (S + kAttnChunk - 1) / kAttnChunk;
        wp.NS = d->nsplit < max_chunks ? d->nsplit : max_chunks;
        const int units = io.nb * d->H * wp.NS;
        if (q8_attn_quant(d)) {
          wp.xq8 = d->xq_d;
          wp.xq8s = d->xqs_d;
        }
        if (d->hs == 64)
          hipLaunchKernelGGL((tl::attn_wave_kernel<64, kAttnChunk>), dim3(units), dim3(64), 0, d->stream, wp);
        else if (d->hs == 128)
          hipLaunchKernelGGL((tl::attn_wave_kernel<128, kAttnChunk>), dim3(units), dim3(64), 0, d->stream, wp);
        else  // half-size chunks keep head-256 K/V rows in registers without spills
          hipLaunchKernelGGL((tl::attn_wave_kernel<256, kAttnChunk / 2>), dim3(units), dim3(64), 0, d->stream, wp);
        TL_TRY(hipGetLastError());
      } else {
        // generic head sizes: block kernel + separate combine launch
        dim3 grid(d->H, io.nb, d->nsplit);
      switch (lpk) {
        case 2: hipLaunchKernelGGL(tl::attn_decode_kernel<2>, grid, dim3(256), lds, d->stream, a); break;
        case 4: hipLaunchKernelGGL(tl::attn_decode_kernel<4>, grid, dim3(256), lds, d->stream, a); break;
        case 8: hipLaunchKernelGGL(tl::attn_decode_kernel<8>, grid, dim3(256), lds, d->stream, a); break;
        case 16: hipLaunchKernelGGL(tl::attn_decode_kernel<16>, grid, dim3(256), lds, d->stream, a); break;
        case 32: hipLaunchKernelGGL(tl::attn_decode_kernel<32>, grid, dim3(256), lds, d->stream, a); break;
        case 64: hipLaunchKernelGGL(tl::attn_decode_kernel<64>, grid, dim3(256), lds, d->stream, a); break;
        default:
          g_last_error = "unsupported head_size for fused attention";
          return (int)hipErrorInvalidValue;
      }
      TL_TRY(hipGetLastError());
      if (d->nsplit > 1) {
        hipLaunchKernelGGL(tl::attn_combine_kernel<0>, dim3(d->H, io.nb), dim3(128), 0, d->stream, a);
        TL_TRY(hipGetLastError());
      }
      }
      prof_end(d, THALLAMA_K_ATTN, ev);
    }
    // 3. Wo + residual
    {
      tl::GemvParams p = {};
      p.W0 = lw.wo;
      p.K = dim;
      p.n_items = dim;
      p.nb = io.nb;
      p.x = io.xb;
      p.x_stride = dim;
      p.y = io.x;
      p.y_stride = dim;
      p.xq_ready = q8_attn_quant(d);
      ssq_to_next_norm(d, p);
      int ev = prof_begin(d);
      TL_TRY(gemv(d, tl::GM_RESID, p, Q8L(wo), nullptr, nullptr));
      prof_end(d, THALLAMA_K_WO, ev);
    }
    // 4. RMSNorm(ffn) + W1/W3 + SwiGLU
    {
      tl::GemvParams p = {};
      p.W0 = lw.w1;
      p.W1 = lw.w3;
      p.K = dim;
      p.n_items = hid;
      p.nb = io.nb;
      p.x = io.x;
      p.x_stride = dim;
      p.rms_w = lw.rms_ffn;
      p.xn = d->xn_d;
      norm_from_ssq(d, p);
      p.y = io.hb;
      p.y_stride = hid;
      int ev = prof_begin(d);
      TL_TRY(gemv(d, tl::GM_SWIGLU, p, Q8L(w1), Q8L(w3), nullptr));
      prof_end(d, THALLAMA_K_FFN_UP, ev);
    }
    // 5. W2 + residual
    {
      tl::GemvParams p = {};
      p.W0 = lw.w2;
      p.K = hid;
      p.n_items = dim;
      p.nb = io.nb;
      p.x = io.hb;
      p.x_stride = hid;
      p.y = io.x;
      p.y_stride = dim;
      ssq_to_next_norm(d, p);
      int ev = prof_begin(d);
      TL_TRY(gemv(d, tl::GM_RESID, p, Q8L(w2), nullptr, nullptr));
      prof_end(d, THALLAMA_K_FFN_DOWN, ev);
    }
    if (io.after_layer) {
      const int r = io.after_layer(l);
      if (r) return r;
    }
  }
  // final RMSNorm + classifier
  if (io.logits) {
    tl::GemvParams p = {};
    p.W0 = w.wcls;
    p.K = dim;
    p.n_items = d->V;
    p.nb = io.nb;
    p.x = io.x;
    p.x_stride = dim;
    p.rms_w = w.rms_final_weight;
    p.xn = d->xn_d;
    if (d->L > 0) norm_from_ssq(d, p);
    if (d->L == 0 && io.embed) {
      p.tok = io.tok;
      p.emb = w.token_embedding_table;
      p.x_out = io.x;
    }
    p.y = io.logits;
    p.y_stride = d->V;
    int ev = prof_begin(d);
    TL_TRY(gemv(d, tl::GM_STORE, p, d->q8 ? d->w8.wcls : nullptr, nullptr, nullptr));
    prof_end(d, THALLAMA_K_CLS, ev);
  }
  return 0;
}

static int enqueue_step(thallama_decoder* d) { return enqueue_step_io(d, step_io(d)); }

// The whole step (and, for greedy decoding, the argmax + advance) as one persistent launch.
// Which persistent instantiation a step at position pos0 (slot 0, batch 1) runs: 1 = the one with
// the long-context attention helper (fp32 only; persist.hip).
static int long_ctx(thallama_decoder* d, int pos0) {
  return d->B == 1 && !d->q8 && use_persist(d) && tl::persistent_long_ctx(pos0) ? 1 : 0;
}

static int enqueue_persistent(thallama_decoder* d, bool argmax, int lc) {
  const TransformerWeights& w = d->w;
  const RunState& s = d->s;
  tl::PStep p = {};
  p.emb = w.token_embedding_table; p.rms_att = w.rms_att_weight; p.rms_ffn = w.rms_ffn_weight;
  p.wq = w.wq; p.wk = w.wk; p.wv = w.wv; p.wo = w.wo; p.w1 = w.w1; p.w2 = w.w2; p.w3 = w.w3;
  p.rms_final = w.rms_final_weight; p.wcls = w.wcls;
  p.dim = d->dim; p.hid = d->hidden; p.kvd = d->kv_dim; p.L = d->L; p.S = d->S; p.V = d->V; p.H = d->H;
  p.kv_mul = d->kv_mul; p.hs = d->hs; p.NS = d->nsplit;
  p.x = s.x; p.xb = s.xb; p.logits = s.logits; p.kc = s.key_cache; p.vc = s.value_cache;
  p.part = d->part_d; p.rope = d->rope_d;
  p.tok = d->tok_d; p.pos = d->pos_d; p.out = d->out_d;
  p.B = d->B;
  {
    const size_t B = d->B;  // B rows of each hand-off buffer (batch 1: one)
    p.gx = d->pgran; p.gxb = p.gx + B * d->dim; p.ghb = p.gxb + B * d->dim; p.gqkv = p.ghb + B * d->hidden;
    p.gsc = p.gqkv + B * (d->dim + 2 * d->kv_dim);
  }
  p.sync = d->psync; p.tickets = d->psync + tl::kPSyncWords;
  p.err = d->psync + d->psync_zero; p.seq = p.err + 1; p.bmax = d->pbmax;
  p.argmax = argmax ? 1 : 0;
  p.long_ctx = lc;
  p.trace = d->ptrace;
  p.fault = d->pfault ? 1 : 0;
  d->pfault = false;  // one-shot (a captured graph keeps it; the give-up drops the graph)
  if (d->q8) {
    p.q8 = d->w8.group_size;
    for (int t = 0; t < 7; ++t) {
      p.q8w[t] = d->pq8w[t];
      p.q8ls[t] = d->pq8ls[t];
    }
    p.qcls = d->w8.wcls->q;
    p.scls = d->w8.wcls->s;
  }
  const char* why = nullptr;
  const bool ks = use_ksplit(d);
  p.gk = ks ? d->pkgran : nullptr;
  if (!(ks ? tl::persistent_prepare_k(p, d->ncu, &why)
           : d->B > 1 ? tl::persistent_prepare_b(p, d->ncu, &why) : tl::persistent_prepare(p, d->ncu, &why))) {
    g_last_error = std::string("persistent step: ") + (why ? why : "unsupported");
    return (int)hipErrorInvalidValue;
  }
  TL_TRY(hipMemsetAsync(p.sync, 0, sizeof(unsigned) * d->psync_zero, d->stream));
  const int ev = prof_begin(d);
  TL_TRY(ks ? tl::launch_persistent_step_k(p, d->stream, d->ncu)
            : d->B > 1 ? tl::launch_persistent_step_b(p, d->stream, d->ncu) : tl::launch_persistent_step(p, d->stream, d->ncu));
  prof_end(d, THALLAMA_K_STEP, ev);
  return 0;
}

// After a synchronisation: did a persistent grid barrier give up?  (Only possible if the
// grid was not co-resident; the step's results are then wrong and the path is disabled.)
// check_persist's status when a persistent launch gave up (its outputs are garbage) and the
// path is now disabled: the public entry points then re-run the call on the multi-launch path
// (every K/V row the failed call wrote is rewritten, in order, before it is read again).
constexpr int kPersistFellBack = (int)hipErrorLaunchFailure;

// Enqueued on d->stream after a call's persistent launches, before its synchronisation: the
// error word lands in pinned host memory with the rest of the call (no legacy-stream copy).
static int enqueue_err_read(thallama_decoder* d) {
  if (d->psync && use_persist(d)) {
    TL_TRY(hipMemcpyAsync(d->perr_h, d->psync + d->psync_zero, sizeof(unsigned), hipMemcpyDeviceToHost, d->stream));
    d->err_pending = true;
  }
  return 0;
}

// After the synchronisation that covered enqueue_err_read.
static int check_persist(thallama_decoder* d) {
  if (!d->err_pending) return 0;
  d->err_pending = false;
  if (!*d->perr_h) return 0;
  *d->perr_h = 0;
  TL_TRY(hipMemsetAsync(d->psync, 0, sizeof(unsigned) * (d->psync_zero + 32), d->stream));
  TL_TRY(hipMemsetAsync(d->cnt_d, 0, sizeof(unsigned) * (size_t)d->B * d->H, d->stream));
  TL_TRY(hipStreamSynchronize(d->stream));
  d->pok = false;
  d->pwhy = "a grid barrier timed out";
  {
    ApiLock lock(api_mu());
    drop_graphs(d);  // the captured graphs hold the persistent launch
  }
  g_last_error = "persistent step: a grid barrier timed out (grid not co-resident); path disabled";
  return kPersistFellBack;
}

extern "C" int thallama_decoder_persistent(thallama_decoder* d) { return d && use_persist(d) ? 1 : 0; }
extern "C" int thallama_decoder_ksplit(thallama_decoder* d) { return d && use_ksplit(d) ? 1 : 0; }
extern "C" int thallama_persistent_cooperative(void) { return tl::persistent_cooperative() ? 1 : 0; }

// Diagnostics: copy the persistent step's hand-off granules {value, tag} (x | xb | hb | q k v |
// int8 attention scores, the last layer's values after a launch) to host (n granules at most).
extern "C" int thallama_decoder_granules(thallama_decoder* d, unsigned long long* host, size_t n) {
  if (!d || !d->pgran) return (int)hipErrorInvalidValue;
  const size_t ng = granule_count(d);
  if (!host) return (int)ng;
  TL_TRY(hipMemcpyAsync(host, d->pgran, (n < ng ? n : ng) * 8, hipMemcpyDeviceToHost, d->stream));
  TL_TRY(hipStreamSynchronize(d->stream));
  return (int)ng;
}

// Timeline of the persistent step (tools/persist_trace.py): enable allocates the buffer;
// every later launch overwrites it; copy returns [grid][5L+1][kTraceSlots] 100-MHz stamps.
extern "C" int thallama_decoder_ptrace(thallama_decoder* d, int enable, unsigned long long* host, size_t n) {
  if (!d) return (int)hipErrorInvalidValue;
  const size_t need = (size_t)d->ncu * (5 * d->L + 1) * tl::kTraceSlots;
  if (enable && !d->ptrace) {
    ApiLock lock(api_mu());
    TL_TRY(hipMalloc(&d->ptrace, need * sizeof(unsigned long long)));
    TL_TRY(hipMemsetAsync(d->ptrace, 0, need * sizeof(unsigned long long), d->stream));
    d->ptrace_n = need;
    drop_graphs(d);
  }
  if (host && d->ptrace) {
    TL_TRY(hipMemcpyAsync(host, d->ptrace, (n < d->ptrace_n ? n : d->ptrace_n) * sizeof(unsigned long long),
                          hipMemcpyDeviceToHost, d->stream));
    TL_TRY(hipStreamSynchronize(d->stream));
  }
  return (int)need;
}

static int enqueue_argmax(thallama_decoder* d) {
  int ev = prof_begin(d);
  hipLaunchKernelGGL(k_argmax_advance, dim3(d->B), dim3(1024), 0, d->stream, d->s.logits, d->V, d->tok_d,
                     d->pos_d, d->out_d, d->S);
  TL_TRY(hipGetLastError());
  prof_end(d, THALLAMA_K_ARGMAX, ev);
  return 0;
}

// An asynchronous greedy call (sync = 0, no tokens requested) returns before its launches run,
// so a persistent give-up inside it is found only at the next synchronisation: that call's
// tokens and K/V rows are then invalid, and the error is reported for IT (kPersistAsyncLost),
// never silently repaired by re-running a later call.
constexpr int kPersistAsyncLost = (int)hipErrorIllegalState;

static int check_async(thallama_decoder* d) {
  if (!d->pasync) return 0;
  d->pasync = false;
  if (check_persist(d) == 0) return 0;
  g_last_error = "persistent step: an earlier asynchronous greedy call gave up (grid not co-resident); its tokens "
                 "and K/V rows are invalid; path disabled";
  return kPersistAsyncLost;
}

static int upload_tok_pos(thallama_decoder* d, const int* token_h, const int* pos_h) {
  int r = 0;
  for (int b = 0; b < d->B; ++b) {
    if (pos_h[b] < 0 || pos_h[b] >= d->S || token_h[b] < 0 || token_h[b] >= d->V) {
      g_last_error = "token/pos out of range";
      return (int)hipErrorInvalidValue;
    }
  }
  // the staging buffers may still feed an in-flight copy of the previous call
  TL_TRY(hipStreamSynchronize(d->stream));
  r = check_async(d);
  if (r) return r;
  memcpy(d->tok_h, token_h, sizeof(int) * d->B);
  memcpy(d->pos_h, pos_h, sizeof(int) * d->B);
  TL_TRY(hipMemcpyAsync(d->tok_d, d->tok_h, sizeof(int) * d->B, hipMemcpyHostToDevice, d->stream));
  TL_TRY(hipMemcpyAsync(d->pos_d, d->pos_h, sizeof(int) * d->B, hipMemcpyHostToDevice, d->stream));
  return 0;
}

static int decoder_forward_once(thallama_decoder* d, const int* token_h, const int* pos_h, float* logits_h);

// Ends the capture begun on d->stream (also after an enqueue error `e`, so the stream leaves capture
// mode) and instantiates it into *exec; the captured graph is destroyed on every path.
static int finish_capture(thallama_decoder* d, int e, hipGraphExec_t* exec) {
  hipGraph_t g = nullptr;
  hipError_t ce = hipStreamEndCapture(d->stream, &g);
  hipError_t ie = hipSuccess;
  if (!e && ce == hipSuccess) ie = hipGraphInstantiate(exec, g, nullptr, nullptr, 0);
  if (g) (void)hipGraphDestroy(g);
  if (e) return e;
  TL_TRY(ce);
  TL_TRY(ie);
  return 0;
}

// Where a step's B x V logits are copied to: the caller's buffer when it is pinned (the reference
// passes hipHostMalloc memory, src/llama.cpp:935), else the decoder's pinned staging, copied on
// after the synchronisation — a D2H copy into pageable memory is staged by the runtime at a fraction
// of the link rate (1 MB per step at batch 8).  The answer is remembered per address and re-queried
// every 256 steps, so a buffer freed and re-allocated at the same address as another kind of memory
// only costs the fast path (or an extra staging copy) until then — the result is right either way.
static float* logits_dst(thallama_decoder* d, float* logits_h) {
  if (logits_h != d->lg_last || (++d->lg_checks & 255u) == 0) {
    hipPointerAttribute_t a = {};
    d->lg_last = logits_h;
    const hipError_t e = hipPointerGetAttributes(&a, logits_h);
    d->lg_last_pinned = e == hipSuccess && a.type == hipMemoryTypeHost;
    if (e != hipSuccess) (void)hipGetLastError();  // (a pageable pointer reports an error: not sticky)
  }
  if (d->lg_last_pinned) return logits_h;
  if (!d->lg_pin) {
    ApiLock lock(api_mu());
    if (hipHostMalloc(&d->lg_pin, sizeof(float) * (size_t)d->B * d->V, hipHostMallocDefault) != hipSuccess) {
      d->lg_pin = nullptr;
      return logits_h;
    }
  }
  return d->lg_pin;
}

extern "C" int thallama_decoder_forward(thallama_decoder* d, const int* token_h, const int* pos_h, float* logits_h) {
  const bool persistent = d && use_persist(d);
  int r = decoder_forward_once(d, token_h, pos_h, logits_h);
  if (r == kPersistFellBack && persistent && !use_persist(d)) r = decoder_forward_once(d, token_h, pos_h, logits_h);
  return r;
}

static int decoder_forward_once(thallama_decoder* d, const int* token_h, const int* pos_h, float* logits_h) {
  if (!d || !token_h || !pos_h) return (int)hipErrorInvalidValue;
  int r = upload_tok_pos(d, token_h, pos_h);
  if (r) return r;
  if (d->use_graph && !d->profile) {  // the step (~160 launches at batch > 1) replayed as one graph
    const int lc = long_ctx(d, pos_h[0]);
    if (!d->exec_fwd[lc]) {
      ApiLock lock(api_mu());
      TL_TRY(hipStreamBeginCapture(d->stream, hipStreamCaptureModeThreadLocal));
      const int e = use_persist(d) ? enqueue_persistent(d, false, lc) : enqueue_step(d);
      if ((r = finish_capture(d, e, &d->exec_fwd[lc])) != 0) return r;
    }
    TL_TRY(hipGraphLaunch(d->exec_fwd[lc], d->stream));
  } else {
    r = use_persist(d) ? enqueue_persistent(d, false, long_ctx(d, pos_h[0])) : enqueue_step(d);
    if (r) return r;
  }
  float* staged = nullptr;
  if (logits_h) {
    staged = logits_dst(d, logits_h);
    TL_TRY(hipMemcpyAsync(staged, d->s.logits, sizeof(float) * (size_t)d->B * d->V, hipMemcpyDeviceToHost, d->stream));
  }
  if ((r = enqueue_err_read(d)) != 0) return r;
  TL_TRY(hipStreamSynchronize(d->stream));
  if (staged && staged != logits_h) memcpy(logits_h, staged, sizeof(float) * (size_t)d->B * d->V);
  prof_collect(d);
  return check_persist(d);
}

static int decoder_greedy_once(thallama_decoder* d, const int* token0_h, const int* pos0_h, int n_steps,
                               int* tokens_out_h, int sync);

// One greedy step (the step + the argmax that feeds tok/pos) captured as a graph, once.
static int ensure_greedy_graph(thallama_decoder* d, int lc) {
  if (d->exec[lc]) return 0;
  ApiLock lock(api_mu());
  TL_TRY(hipStreamBeginCapture(d->stream, hipStreamCaptureModeThreadLocal));
  int e = 0;
  if (use_persist(d)) {
    e = enqueue_persistent(d, true, lc);
  } else {
    e = enqueue_step(d);
    if (!e) e = enqueue_argmax(d);
  }
  return finish_capture(d, e, &d->exec[lc]);
}

// One greedy step with host token/pos: next_h[b] = the device argmax of slot b's logits (the
// scheduler's greedy step, thallama_argmax_step_fn).  B ids come back instead of B x V logits.
static int decoder_step_argmax_once(thallama_decoder* d, const int* token_h, const int* pos_h, int* next_h) {
  if (!d || !token_h || !pos_h || !next_h) return (int)hipErrorInvalidValue;
  int r = upload_tok_pos(d, token_h, pos_h);
  if (r) return r;
  if (d->use_graph && !d->profile) {
    const int lc = long_ctx(d, pos_h[0]);
    if ((r = ensure_greedy_graph(d, lc)) != 0) return r;
    TL_TRY(hipGraphLaunch(d->exec[lc], d->stream));
  } else {
    r = use_persist(d) ? enqueue_persistent(d, true, long_ctx(d, pos_h[0])) : enqueue_step(d);
    if (!r && !use_persist(d)) r = enqueue_argmax(d);
    if (r) return r;
  }
  TL_TRY(hipMemcpyAsync(d->nxt_h, d->tok_d, sizeof(int) * d->B, hipMemcpyDeviceToHost, d->stream));
  if ((r = enqueue_err_read(d)) != 0) return r;
  TL_TRY(hipStreamSynchronize(d->stream));
  memcpy(next_h, d->nxt_h, sizeof(int) * d->B);
  prof_collect(d);
  return check_persist(d);
}

extern "C" int thallama_decoder_step_argmax(thallama_decoder* d, const int* token_h, const int* pos_h, int* next_h) {
  const bool persistent = d && use_persist(d);
  int r = decoder_step_argmax_once(d, token_h, pos_h, next_h);
  if (r == kPersistFellBack && persistent && !use_persist(d)) r = decoder_step_argmax_once(d, token_h, pos_h, next_h);
  return r;
}

extern "C" int thallama_decoder_argmax_cb(void* ctx, int worker, int batch, const int* token, const int* pos,
                                          int* next) {
  (void)worker;
  thallama_decoder* d = (thallama_decoder*)ctx;
  if (!d || batch != d->B) return (int)hipErrorInvalidValue;
  return thallama_decoder_step_argmax(d, token, pos, next);
}

extern "C" int thallama_decoder_greedy(thallama_decoder* d, const int* token0_h, const int* pos0_h, int n_steps,
                                       int* tokens_out_h, int sync) {
  const bool persistent = d && use_persist(d);
  int r = decoder_greedy_once(d, token0_h, pos0_h, n_steps, tokens_out_h, sync);
  if (r == kPersistFellBack && persistent && !use_persist(d))
    r = decoder_greedy_once(d, token0_h, pos0_h, n_steps, tokens_out_h, sync);
  return r;
}

static int decoder_greedy_once(thallama_decoder* d, const int* token0_h, const int* pos0_h, int n_steps,
                               int* tokens_out_h, int sync) {
  if (!d || !token0_h || !pos0_h || n_steps < 0) return (int)hipErrorInvalidValue;
  for (int b = 0; b < d->B; ++b)
    if (pos0_h[b] + n_steps > d->S) {
      g_last_error = "greedy decode would run past seq_len";
      return (int)hipErrorInvalidValue;
    }
  int r = upload_tok_pos(d, token0_h, pos0_h);
  if (r) return r;
  const bool graph = d->use_graph && !d->profile;
  // step i runs at position pos0 + i: captured before the first replay, one graph per instantiation
  const int lc_first = n_steps > 0 ? long_ctx(d, pos0_h[0]) : 0;
  const int lc_last = n_steps > 0 ? long_ctx(d, pos0_h[0] + n_steps - 1) : 0;
  for (int lc = lc_first; graph && lc <= lc_last; ++lc)
    if ((r = ensure_greedy_graph(d, lc)) != 0) return r;
  for (int i = 0; i < n_steps; ++i) {
    const int lc = long_ctx(d, pos0_h[0] + i);
    if (graph) {
      TL_TRY(hipGraphLaunch(d->exec[lc], d->stream));
    } else if (use_persist(d)) {
      r = enqueue_persistent(d, true, lc);
      if (r) return r;
    } else {
      r = enqueue_step(d);
      if (r) return r;
      r = enqueue_argmax(d);
      if (r) return r;
    }
  }
  if (n_steps > 0 && (r = enqueue_err_read(d)) != 0) return r;
  if (tokens_out_h && n_steps > 0) {
    // tokens by position: sequence b generated out[b][pos0+1 .. pos0+n_steps] ... stored at pos index
    std::vector<int> tmp((size_t)d->B * d->S);
    TL_TRY(hipMemcpyAsync(tmp.data(), d->out_d, sizeof(int) * tmp.size(), hipMemcpyDeviceToHost, d->stream));
    TL_TRY(hipStreamSynchronize(d->stream));
    for (int i = 0; i < n_steps; ++i)
      for (int b = 0; b < d->B; ++b) tokens_out_h[(size_t)i * d->B + b] = tmp[(size_t)b * d->S + pos0_h[b] + i];
  } else if (sync) {
    TL_TRY(hipStreamSynchronize(d->stream));
  } else {
    d->pasync = d->pasync || (n_steps > 0 && use_persist(d));
    prof_collect(d);
    return 0;
  }
  prof_collect(d);
  return check_persist(d);
}

// thallama_step_fn / thallama_prefill_fn (include/thallama_host.h) over one decoder (ctx), so a
// host scheduler can drive it with no glue of its own (bench.py's request workload).
extern "C" int thallama_decoder_step_cb(void* ctx, int worker, int batch, const int* token, const int* pos,
                                        float* logits) {
  (void)worker;
  thallama_decoder* d = (thallama_decoder*)ctx;
  if (!d || batch != d->B) return (int)hipErrorInvalidValue;
  return thallama_decoder_forward(d, token, pos, logits);
}

extern "C" int thallama_decoder_prefill_cb(void* ctx, int worker, int slot, const int* tokens, int n, int pos0) {
  (void)worker;
  const int st = thallama_decoder_prefill((thallama_decoder*)ctx, slot, tokens, n, pos0);
  if (st == (int)hipErrorNotSupported) return 1;  // the scheduler then steps through the prompt
  return st ? -st : 0;
}

extern "C" int thallama_decoder_logits(thallama_decoder* d, float* logits_h) {
  if (!d || !logits_h) return (int)hipErrorInvalidValue;
  TL_TRY(hipMemcpyAsync(logits_h, d->s.logits, sizeof(float) * (size_t)d->B * d->V, hipMemcpyDeviceToHost,
                        d->stream));
  TL_TRY(hipStreamSynchronize(d->stream));
  return check_async(d);
}

// Synchronise the decoder's stream and report a give-up of an earlier asynchronous call.
extern "C" int thallama_decoder_sync(thallama_decoder* d) {
  if (!d) return (int)hipErrorInvalidValue;
  TL_TRY(hipStreamSynchronize(d->stream));
  prof_collect(d);
  return check_async(d);
}

extern "C" int thallama_decoder_prof(thallama_decoder* d, int kclass, double* total_ms, long long* count) {
  if (!d || kclass < 0 || kclass >= THALLAMA_K_COUNT) return (int)hipErrorInvalidValue;
  prof_collect(d);
  if (total_ms) *total_ms = d->prof_ms[kclass];
  if (count) *count = d->prof_n[kclass];
  return 0;
}

extern "C" void thallama_decoder_prof_reset(thallama_decoder* d) {
  if (!d) return;
  prof_collect(d);
  for (int i = 0; i < THALLAMA_K_COUNT; ++i) {
    d->prof_ms[i] = 0;
    d->prof_n[i] = 0;
  }
}

extern "C" double thallama_step_bytes(const Config* c, int B, int kclass, const int* pos_h) {
  const double dim = c->dim, hid = c->hidden_dim, V = c->vocab_size < 0 ? -c->vocab_size : c->vocab_size;
  const double kvd = (double)c->dim * c->n_kv_heads / c->n_heads;
  switch (kclass) {
    case THALLAMA_K_QKV: return 4.0 * ((dim * dim + 2 * dim * kvd) + dim + B * (dim + dim + 2 * kvd));
    case THALLAMA_K_ATTN: {
      double t = 0;
      for (int b = 0; b < B; ++b) t += (pos_h ? pos_h[b] + 1 : 1);
      return 4.0 * (2 * kvd * t + B * 2 * dim);
    }
    case THALLAMA_K_WO: return 4.0 * (dim * dim + B * 3 * dim);
    case THALLAMA_K_FFN_UP: return 4.0 * (2 * hid * dim + dim + B * (dim + hid));
    case THALLAMA_K_FFN_DOWN: return 4.0 * (hid * dim + B * (hid + 2 * dim));
    case THALLAMA_K_CLS: return 4.0 * (V * dim + dim + B * (dim + V));
    case THALLAMA_K_ARGMAX: return 4.0 * B * V;
    case THALLAMA_K_STEP: {
      double t = 0;
      for (int k = THALLAMA_K_QKV; k <= THALLAMA_K_FFN_DOWN; ++k) t += c->n_layers * thallama_step_bytes(c, B, k, pos_h);
      return t + thallama_step_bytes(c, B, THALLAMA_K_CLS, pos_h) + thallama_step_bytes(c, B, THALLAMA_K_ARGMAX, pos_h);
    }
  }
  return 0;
}

// ------------------------------------------------------------------ thaDNN_s_forward_batch
// The reference signature carries no workspace, so a decoder per (device, stream, batch, config,
// fp32|int8) is created on first use and reused.  A call with other weight / state buffers than
// the cached decoder's replaces it, and at most g_dec_cap decoders stay cached (least recently
// used evicted), so a host that reallocates its buffers does not grow without bound.  The cap
// starts at 8 and follows the caller's working set: a miss on a key evicted recently (a "ghost")
// means the cache was too small for the keys in use — e.g. the reference's pipeline test, 4 host
// threads x n_devices stage decoders (src/llama.cpp:1298) — and raises the cap by one, up to 256.
// The reference calls this entry from one host thread per GPU (src/llama.cpp:919, 1017), so
// entries are shared: a caller holds a reference (shared_ptr) for the whole forward, eviction only
// drops the cache's reference, and the decoder is destroyed when its last user returns; callers
// of one entry are serialised by its mutex.  thallama_forward_batch_cache_size() reports the count.
namespace {
typedef std::tuple<int, hipStream_t, int, int, int, int, int, int, int, int> DecKey;
struct CachedDecoder {
  thallama_decoder* d = nullptr;
  std::mutex use;           // one forward at a time per decoder
  TransformerWeights w{};   // fp32 buffers the decoder was made for
  Q8TransformerWeights w8{};  // (int8)
  RunState s{};
  ~CachedDecoder() {
    if (d) thallama_decoder_destroy(d);
  }
};
struct DecEntry {
  std::shared_ptr<CachedDecoder> c;
  unsigned long long used;
};
constexpr size_t kDecCacheMin = 8, kDecCacheCeil = 256;
size_t g_dec_cap = kDecCacheMin;
std::deque<DecKey> g_dec_ghosts;  // recently evicted keys, oldest first (at most kDecCacheCeil)
std::mutex g_dec_mu;
unsigned long long g_dec_clock = 0;
std::atomic<long long> g_dec_live{0};  // decoders alive (cached or still in use after eviction)
// Allocated once and never freed: decoders still cached at process exit are not destroyed during
// static destruction (after HIP's own teardown, with the lock object possibly gone).
std::map<DecKey, DecEntry>& dec_cache() {
  static auto* m = new std::map<DecKey, DecEntry>();
  return *m;
}

// The cached decoder for key, if it was made for exactly these buffers; else a new one (replacing
// a stale entry, evicting the least recently used beyond the cap).  Caller holds g_dec_mu.
std::shared_ptr<CachedDecoder> dec_lookup(const DecKey& key, const Config* p, const TransformerWeights* w,
                                          const Q8TransformerWeights* w8, const RunState* s, int B, hipStream_t st) {
  auto& m = dec_cache();
  auto it = m.find(key);
  if (it != m.end()) {
    CachedDecoder& e = *it->second.c;
    const bool same = memcmp(&e.s, s, sizeof(RunState)) == 0 &&
                      (w8 ? memcmp(&e.w8, w8, sizeof(*w8)) == 0 : memcmp(&e.w, w, sizeof(*w)) == 0);
    if (same) {
      it->second.used = ++g_dec_clock;
      return it->second.c;
    }
    m.erase(it);  // destroyed now, or when its last user returns
  } else {
    auto gh = std::find(g_dec_ghosts.begin(), g_dec_ghosts.end(), key);
    if (gh != g_dec_ghosts.end()) {  // thrashing: the working set is larger than the cap
      g_dec_ghosts.erase(gh);
      if (g_dec_cap < kDecCacheCeil) ++g_dec_cap;
    }
  }
  while (m.size() >= g_dec_cap) {
    auto lru = m.begin();
    for (auto i = m.begin(); i != m.end(); ++i)
      if (i->second.used < lru->second.used) lru = i;
    g_dec_ghosts.push_back(lru->first);
    if (g_dec_ghosts.size() > kDecCacheCeil) g_dec_ghosts.pop_front();
    m.erase(lru);
  }
  thallama_decoder* d = nullptr;
  const int r = w8 ? thallama_decoder_create_q8(&d, p, w8, s, B, st) : thallama_decoder_create(&d, p, w, s, B, st);
  if (r != 0) return nullptr;
  std::shared_ptr<CachedDecoder> c(new CachedDecoder(), [](CachedDecoder* x) {
    delete x;
    --g_dec_live;
  });
  ++g_dec_live;
  c->d = d;
  if (w8) c->w8 = *w8; else c->w = *w;
  c->s = *s;
  m[key] = DecEntry{c, ++g_dec_clock};
  return c;
}
}  // namespace

extern "C" int thallama_forward_batch_cache_size(void) {
  std::lock_guard<std::mutex> g(g_dec_mu);
  return (int)dec_cache().size();
}

extern "C" int thallama_forward_batch_cache_cap(void) {
  std::lock_guard<std::mutex> g(g_dec_mu);
  return (int)g_dec_cap;
}

// Decoders alive: the cached ones plus evicted ones a caller is still running.
extern "C" int thallama_forward_batch_live(void) { return (int)g_dec_live.load(); }

extern "C" void thallama_forward_batch_cache_clear(void) {
  std::map<DecKey, DecEntry> gone;
  {
    std::lock_guard<std::mutex> g(g_dec_mu);
    gone.swap(dec_cache());
    g_dec_ghosts.clear();  // the working set is forgotten too: the cap starts over
    g_dec_cap = kDecCacheMin;
  }
  // (destroyed here, outside the lock, unless a caller still holds one)
}

// Runs f(decoder) with the decoder for (key, buffers) pinned and its use lock held.
template <class F>
static int with_cached_decoder(const DecKey& key, const Config* p, const TransformerWeights* w,
                               const Q8TransformerWeights* w8, const RunState* s, int B, hipStream_t st,
                               const char* who, F f) {
  std::shared_ptr<CachedDecoder> c;
  {
    std::lock_guard<std::mutex> g(g_dec_mu);
    c = dec_lookup(key, p, w, w8, s, B, st);
  }
  if (!c) {
    fprintf(stderr, "%s: %s\n", who, thallama_last_error());
    return (int)hipErrorInvalidValue;
  }
  std::lock_guard<std::mutex> use(c->use);
  return f(c->d);
}

extern "C" thablasStatus_t thaDNN_s_forward_batch(thablasHandle_t handle1, thablasHandle_t handle2,
                                                  thablasHandle_t handle3, int n_batches, Config* p,
                                                  TransformerWeights* w, RunState* s_batch, int token[],
                                                  int pos[], float* logits_host) {
  (void)handle2;
  (void)handle3;
  if (!p || !w || !s_batch || !token || !pos || !logits_host || n_batches <= 0) return THABLAS_STATUS_INVALID_VALUE;
  int dev = 0;
  CHECK_HIP(hipGetDevice(&dev));
  DecKey key(dev, handle1.calc_stream, n_batches, p->dim, p->hidden_dim, p->n_layers, p->n_heads, p->n_kv_heads,
             p->seq_len, p->vocab_size);
  const int r = with_cached_decoder(
      key, p, w, nullptr, s_batch, n_batches, handle1.calc_stream, "thaDNN_s_forward_batch", [&](thallama_decoder* d) {
        // The reference's scheduler (src/llama.cpp:961-1017) runs every slot of the batch, and a
        // slot that never received a request carries uninitialised token/pos; its kernel would
        // read out of bounds.  Such slots run as token 0 at position 0 here: they write only their
        // own K/V row 0, which a request later admitted to the slot rewrites at its first step,
        // and their logits are never read.
        std::vector<int> tk(token, token + n_batches), ps(pos, pos + n_batches);
        for (int b = 0; b < n_batches; ++b)
          if (tk[b] < 0 || tk[b] >= d->V || ps[b] < 0 || ps[b] >= d->S) tk[b] = ps[b] = 0;
        const int e = thallama_decoder_forward(d, tk.data(), ps.data(), logits_host);
        if (e) fprintf(stderr, "thaDNN_s_forward_batch: %s\n", thallama_last_error());
        return e;
      });
  if (r) return r == (int)hipErrorInvalidValue ? THABLAS_STATUS_INVALID_VALUE : THABLAS_STATUS_EXECUTION_FAILED;
  return THABLAS_STATUS_SUCCESS;
}

// ------------------------------------------------------------------ pipeline stages (§8(f4))
// The reference's pipeline drivers (src/thaDNN.cpp:191-427) split the layers over devices:
// device g holds layers [g * pipe, (g + 1) * pipe) (copy_transformer_weight_pipeline_to_device_
// batch), runs them for the batch, and hands the residual stream x to device g + 1; the last
// device runs the final norm and the classifier.  Here a stage is a decoder over the stage's
// layer range (cfg.n_layers = pipe) on the multi-launch step: the first stage embeds the tokens,
// the others start from x, and the hand-off is an asynchronous peer copy over xGMI on the stage's
// stream followed by an event the next stage's stream waits on, so no host thread blocks between
// stages (the reference synchronises the device after every stage).
//
// One stage: tokens / positions in, the layers, then (last stage) logits into logits_h and a
// synchronisation, or (x_next) the residual stream copied into the next stage's x (device
// next_dev) and this stage's event recorded.  wait: the previous stage's decoder (its event).
extern "C" int thallama_decoder_stage(thallama_decoder* d, const int* token_h, const int* pos_h, int embed,
                                      float* logits_h, const thallama_decoder* wait, float* x_next, int next_dev) {
  if (!d || !token_h || !pos_h) return (int)hipErrorInvalidValue;
  int r = upload_tok_pos(d, token_h, pos_h);
  if (r) return r;
  if (wait) TL_TRY(hipStreamWaitEvent(d->stream, wait->ev_stage, 0));
  StepIO io = step_io(d);
  io.embed = embed != 0;
  io.logits = logits_h ? d->s.logits : nullptr;
  if ((r = enqueue_step_io(d, io)) != 0) return r;
  if (logits_h) {
    TL_TRY(hipMemcpyAsync(logits_h, d->s.logits, sizeof(float) * (size_t)d->B * d->V, hipMemcpyDeviceToHost,
                          d->stream));
    TL_TRY(hipStreamSynchronize(d->stream));
    return 0;
  }
  if (x_next) {
    const size_t bytes = sizeof(float) * (size_t)d->B * d->dim;
    if (next_dev == d->dev) TL_TRY(hipMemcpyAsync(x_next, d->s.x, bytes, hipMemcpyDeviceToDevice, d->stream));
    else TL_TRY(hipMemcpyPeerAsync(x_next, next_dev, d->s.x, d->dev, bytes, d->stream));
  }
  TL_TRY(hipEventRecord(d->ev_stage, d->stream));
  return 0;
}

// thaDNN_s_forward_70B's step on decoder d: d->w's per-layer tensors are staging slot 0 (slot 1
// follows it, alloc_weight_to_device_70B), h_w[l] the host copies of layer l.
static int forward_layer_streamed(thallama_decoder* d, TransformerWeights* h_w[], const int* token, const int* pos,
                                  float* logits_h) {
  const long long dim = d->dim, kvd = d->kv_dim, hid = d->hidden;
  const long long slot = 2 * dim + 2 * dim * dim + 2 * dim * kvd + 3 * dim * hid;  // floats per layer
  if (d->q8 || d->w.rms_ffn_weight != d->w.rms_att_weight + dim) {
    g_last_error = "thaDNN_s_forward_70B: device weights not from alloc_weight_to_device_70B";
    return (int)hipErrorInvalidValue;
  }
  if (!d->copy_stream) {
    ApiLock lock(api_mu());
    TL_TRY(hipStreamCreateWithFlags(&d->copy_stream, hipStreamNonBlocking));
    for (int i = 0; i < 2; ++i) {
      TL_TRY(hipEventCreateWithFlags(&d->ev_copied[i], hipEventDisableTiming));
      TL_TRY(hipEventCreateWithFlags(&d->ev_used[i], hipEventDisableTiming));
    }
  }
  int r = upload_tok_pos(d, token, pos);
  if (r) return r;
  auto slot_w = [&](int l) {
    const long long o = (l & 1) * slot;
    const TransformerWeights& w = d->w;
    return LayerW{w.rms_att_weight + o, w.wq + o, w.wk + o, w.wv + o, w.wo + o, w.rms_ffn_weight + o, w.w1 + o,
                  w.w2 + o, w.w3 + o};
  };
  // layer l's nine tensors into slot l & 1, once the layer that used the slot before is done
  auto copy_layer = [&](int l) -> int {
    const LayerW dst = slot_w(l);
    const TransformerWeights* h = h_w[l];
    if (!h) {
      g_last_error = "thaDNN_s_forward_70B: missing host layer";
      return (int)hipErrorInvalidValue;
    }
    if (l >= 2) TL_TRY(hipStreamWaitEvent(d->copy_stream, d->ev_used[l & 1], 0));
    const struct { const float* dst; const float* src; long long n; } t[9] = {
        {dst.rms_att, h->rms_att_weight, dim}, {dst.rms_ffn, h->rms_ffn_weight, dim}, {dst.wq, h->wq, dim * dim},
        {dst.wk, h->wk, dim * kvd}, {dst.wv, h->wv, dim * kvd}, {dst.wo, h->wo, dim * dim},
        {dst.w1, h->w1, dim * hid}, {dst.w2, h->w2, dim * hid}, {dst.w3, h->w3, dim * hid}};
    for (const auto& e : t)
      TL_TRY(hipMemcpyAsync(const_cast<float*>(e.dst), e.src, sizeof(float) * e.n, hipMemcpyHostToDevice, d->copy_stream));
    TL_TRY(hipEventRecord(d->ev_copied[l & 1], d->copy_stream));
    return 0;
  };
  if (d->L > 0 && (r = copy_layer(0)) != 0) return r;
  StepIO io = step_io(d);
  io.layer_w = slot_w;
  io.before_layer = [&](int l) -> int {
    if (l + 1 < d->L) {
      const int e = copy_layer(l + 1);  // overlaps layer l
      if (e) return e;
    }
    TL_TRY(hipStreamWaitEvent(d->stream, d->ev_copied[l & 1], 0));
    return 0;
  };
  io.after_layer = [&](int l) -> int {
    TL_TRY(hipEventRecord(d->ev_used[l & 1], d->stream));
    return 0;
  };
  if ((r = enqueue_step_io(d, io)) != 0) return r;
  TL_TRY(hipMemcpyAsync(logits_h, d->s.logits, sizeof(float) * (size_t)d->V, hipMemcpyDeviceToHost, d->stream));
  TL_TRY(hipStreamSynchronize(d->stream));
  return 0;
}

namespace {
// Peer access between the stages' devices, once per ordered pair (the x hand-off).
void enable_peer(int from, int to) {
  static std::mutex mu;
  static std::vector<std::pair<int, int>> done;
  std::lock_guard<std::mutex> g(mu);
  for (auto& e : done)
    if (e.first == from && e.second == to) return;
  int can = 0;
  if (hipDeviceCanAccessPeer(&can, from, to) == hipSuccess && can) {
    ApiLock lock(api_mu());
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(from);
    (void)hipDeviceEnablePeerAccess(to, 0);  // (already enabled: fine)
    (void)hipGetLastError();
    (void)hipSetDevice(cur);
  }
  done.emplace_back(from, to);
}

// The pipeline forward over n stages: stage g runs on the device of handle[g]'s stream with the
// stage's weights w[g] and this caller's state s[g].  Stage decoders are cached like
// thaDNN_s_forward_batch's (key: the stage's config and stream, a tag bit in the vocab field) and
// held for the whole call, in stage order.
int pipeline_forward(thablasHandle_t handle[], int n, int B, const Config* p, TransformerWeights* w[], RunState* s[],
                     const int* token, const int* pos, float* logits_host, const char* who) {
  if (!handle || !p || !w || !s || !token || !pos || !logits_host || n <= 0 || B <= 0 || p->n_layers % n)
    return (int)hipErrorInvalidValue;
  int dev0 = 0;
  TL_TRY(hipGetDevice(&dev0));
  Config c = *p;
  c.n_layers = p->n_layers / n;
  const int V = c.vocab_size < 0 ? -c.vocab_size : c.vocab_size;
  std::vector<int> tk(token, token + B), ps(pos, pos + B), dev((size_t)n);
  for (int b = 0; b < B; ++b)  // idle slots of the reference's scheduler: token 0 at position 0
    if (tk[b] < 0 || tk[b] >= V || ps[b] < 0 || ps[b] >= c.seq_len) tk[b] = ps[b] = 0;
  std::vector<std::shared_ptr<CachedDecoder>> st((size_t)n);
  std::vector<std::unique_lock<std::mutex>> held;
  int r = 0;
  for (int g = 0; g < n && !r; ++g) {
    if ((r = (int)hipStreamGetDevice(handle[g].calc_stream, &dev[g])) != 0) break;
    if ((r = (int)hipSetDevice(dev[g])) != 0) break;
    DecKey key(dev[g], handle[g].calc_stream, B, c.dim, c.hidden_dim, c.n_layers, c.n_heads, c.n_kv_heads, c.seq_len,
               V | (1 << 30) /* stage keyspace */);
    {
      std::lock_guard<std::mutex> lk(g_dec_mu);
      st[g] = dec_lookup(key, &c, w[g], nullptr, s[g], B, handle[g].calc_stream);
    }
    if (!st[g]) {
      fprintf(stderr, "%s: stage %d: %s\n", who, g, thallama_last_error());
      r = (int)hipErrorInvalidValue;
      break;
    }
    held.emplace_back(st[g]->use);
    if (g > 0 && dev[g] != dev[g - 1]) enable_peer(dev[g - 1], dev[g]);
  }
  for (int g = 0; g < n && !r; ++g) {
    if ((r = (int)hipSetDevice(dev[g])) != 0) break;
    const bool last = g == n - 1;
    r = thallama_decoder_stage(st[g]->d, tk.data(), ps.data(), g == 0, last ? logits_host : nullptr,
                               g > 0 ? st[g - 1]->d : nullptr, last ? nullptr : s[g + 1]->x, last ? 0 : dev[g + 1]);
    if (r) fprintf(stderr, "%s: stage %d: %s\n", who, g, thallama_last_error());
  }
  (void)hipSetDevice(dev0);
  return r;
}

thablasStatus_t status_of(int r) {
  return r == 0 ? THABLAS_STATUS_SUCCESS
                : r == (int)hipErrorInvalidValue ? THABLAS_STATUS_INVALID_VALUE : THABLAS_STATUS_EXECUTION_FAILED;
}
}  // namespace

// ------------------------------------------------------------------ layer streaming (§8(f4))
// reference src/thaDNN.cpp:83-189 (test_70B, src/llama.cpp:1085-1230): a model whose weights do not
// fit the device keeps each layer in pinned host memory (h_w[l], copy_transformer_to_host_70B) and
// streams it in per step.  The reference copies a layer, synchronises, computes it, and also moves
// that layer's K/V rows in and out of host memory every layer.  Here layer l + 1's nine tensors
// are copied on a second stream into the other of two device staging slots (alloc_weight_to_
// device_70B) while layer l computes (events: slot copied / slot consumed), and the K/V cache
// stays on the device (alloc_state_to_device_70B allocates every layer's: an MI355X's 288 GB hold
// a 70B model's cache with room to spare), so h_s is not used.  Batch 1, like the reference.
extern "C" thablasStatus_t thaDNN_s_forward_70B(thablasHandle_t handle, int batch_size, Config* p,
                                               TransformerWeights* h_w[], RunState* h_s, TransformerWeights* d_w,
                                               RunState* d_s, int token[], int pos[], float* logits_host) {
  (void)h_s;
  if (!p || !h_w || !d_w || !d_s || !token || !pos || !logits_host || batch_size != 1) return THABLAS_STATUS_INVALID_VALUE;
  int dev = 0;
  CHECK_HIP(hipGetDevice(&dev));
  const int V = p->vocab_size < 0 ? -p->vocab_size : p->vocab_size;
  if (token[0] < 0 || token[0] >= V || pos[0] < 0 || pos[0] >= p->seq_len) return THABLAS_STATUS_INVALID_VALUE;
  DecKey key(dev, handle.calc_stream, 1, p->dim, p->hidden_dim, p->n_layers, p->n_heads, p->n_kv_heads, p->seq_len,
             V | (1 << 29) /* layer-streaming keyspace */);
  const int r = with_cached_decoder(key, p, d_w, nullptr, d_s, 1, handle.calc_stream, "thaDNN_s_forward_70B",
                                    [&](thallama_decoder* d) { return forward_layer_streamed(d, h_w, token, pos, logits_host); });
  return status_of(r);
}

// reference src/thaDNN.cpp:191-289.  host_thread_status / device_host_thread / device_mtx are the
// reference scheduler's bookkeeping: its per-device locks serialise host threads on a device; the
// stages here run on each caller's own streams and states, so callers may share devices freely.
extern "C" thablasStatus_t thaDNN_s_forward_batch_multiple_pipe_line(thablasHandle_t handle[], int host_thread_id,
                                                                    int n_host_threads, int n_devices, int batch_size,
                                                                    Config* p, TransformerWeights* w[], RunState* s[],
                                                                    int token[], int pos[], float* logits_host,
                                                                    int* host_thread_status, int* device_host_thread,
                                                                    THALLAMA_OMP_LOCK* device_mtx) {
  (void)host_thread_id; (void)n_host_threads; (void)host_thread_status; (void)device_host_thread; (void)device_mtx;
  return status_of(pipeline_forward(handle, n_devices, batch_size, p, w, s, token, pos, logits_host,
                                    "thaDNN_s_forward_batch_multiple_pipe_line"));
}

// reference src/thaDNN.cpp:291-427: the same pipeline with the K/V rows past n_buffer_words kept in
// host memory and swapped per layer (its GPUs could not hold the whole cache).  An MI355X holds
// every position (alloc_swap_run_state_to_device_batch allocates the full cache), so nothing is
// swapped and s_host_batch is not used.
extern "C" thablasStatus_t thaDNN_s_forward_batch_multiple_pipe_line_layer_swap(
    thablasHandle_t handle[], int thread_id, int n_host_threads, int n_devices, int batch_size, int n_buffer_words,
    Config* p, TransformerWeights* w[], RunState* s[], RunState* s_host_batch[], int token[], int pos[],
    float* logits_host, THALLAMA_OMP_LOCK* device_locks) {
  (void)thread_id; (void)n_host_threads; (void)n_buffer_words; (void)s_host_batch; (void)device_locks;
  return status_of(pipeline_forward(handle, n_devices, batch_size, p, w, s, token, pos, logits_host,
                                    "thaDNN_s_forward_batch_multiple_pipe_line_layer_swap"));
}

// reference include/thaDNN.hpp:74 (declared there, never defined): the pipeline over one
// Transformer per device (weights and state from copy_transformer_pipeline_to_device_batch).
extern "C" thablasStatus_t thaDNN_s_forward_batch_pipe_line(thablasHandle_t handle[], int n_devices, int n_batches,
                                                           Transformer* transformer_d[], int token[], int pos[],
                                                           float* logits_host) {
  if (!transformer_d || n_devices <= 0) return THABLAS_STATUS_INVALID_VALUE;
  std::vector<TransformerWeights*> w((size_t)n_devices);
  std::vector<RunState*> s((size_t)n_devices);
  for (int g = 0; g < n_devices; ++g) {
    if (!transformer_d[g]) return THABLAS_STATUS_INVALID_VALUE;
    w[g] = &transformer_d[g]->weights;
    s[g] = &transformer_d[g]->state;
  }
  return status_of(pipeline_forward(handle, n_devices, n_batches, &transformer_d[0]->config, w.data(), s.data(), token,
                                    pos, logits_host, "thaDNN_s_forward_batch_pipe_line"));
}

// ------------------------------------------------------------------ int8 (runq Q8_0) decoder
extern "C" int thallama_decoder_create_q8(thallama_decoder** out, const Config* cfg, const Q8TransformerWeights* w8,
                                          const RunState* s, int batch, hipStream_t stream) {
  if (!w8 || !w8->wq || !w8->wcls || !w8->token_embedding_table || w8->group_size <= 0) {
    g_last_error = "thallama_decoder_create_q8: incomplete Q8 weights (map + dequantised embedding required)";
    return (int)hipErrorInvalidValue;
  }
  TransformerWeights w = {};
  w.token_embedding_table = w8->token_embedding_table;
  w.rms_att_weight = w8->rms_att_weight;
  w.rms_ffn_weight = w8->rms_ffn_weight;
  w.rms_final_weight = w8->rms_final_weight;
  ApiLock lock(api_mu());
  const int r = thallama_decoder_create(out, cfg, &w, s, batch, stream);
  if (r) return r;
  thallama_decoder* d = *out;
  d->q8 = true;
  d->w8 = *w8;
  {  // runq's arithmetic order on the multi-launch steps (env THALLAMA_Q8_EXACT=0: the faster
     // reordered kernels, logits within the Q8 tolerance instead)
    const char* e = getenv("THALLAMA_Q8_EXACT");
    d->q8x = !(e && e[0] == '0') && batch <= 8 && tl::q8_exact_ok(w8->group_size, d->dim, d->hidden, d->hs, d->S);
  }
  if (d->q8x) {
    TL_TRY(tl::q8_exact_prepare());  // the kernels' dynamic-LDS limit, once per device
    TL_TRY(hipMalloc(&d->q8att_d, sizeof(float) * (size_t)batch * d->H * d->S));
    if (d->pf_x) TL_TRY(hipMalloc(&d->pf_att, sizeof(float) * (size_t)kPrefillQ8Chunk * d->H * d->S));
    if (batch < 2) {  // (batch 1 multi-launch: the quantised activations' scratch too)
      const size_t kmax = (size_t)(d->dim > d->hidden ? d->dim : d->hidden);
      TL_TRY(hipMalloc(&d->xq_d, 8 * kmax));
      TL_TRY(hipMalloc(&d->xqs_d, sizeof(float) * 8 * (kmax / 16 + 1)));
    }
  }
  if (batch >= 2) {
    const size_t kmax = (size_t)(d->dim > d->hidden ? d->dim : d->hidden);
    TL_TRY(hipMalloc(&d->xq_d, 8 * kmax));
    TL_TRY(hipMalloc(&d->xqs_d, sizeof(float) * 8 * (kmax / 16 + 1)));
  }
  if (batch > 1 && d->pok) {  // the batched persistent steps are fp32 only: int8 batches run multi-launch
    d->pok = false;
    d->pk = false;
    (void)hipFree(d->pkgran);
    d->pkgran = nullptr;
    d->pwhy = "int8 weights with batch > 1";
  }
  // persistent step with int8 weights: re-check the shape (group size, LDS) and publish the
  // per-layer tensor addresses as a device table the kernel indexes by (tensor, layer)
  if (d->pok) {
    tl::PStep ps = {};
    ps.dim = d->dim; ps.hid = d->hidden; ps.kvd = d->kv_dim; ps.hs = d->hs; ps.NS = d->nsplit; ps.L = d->L;
    ps.H = d->H; ps.S = d->S; ps.V = d->V;
    ps.q8 = w8->group_size;
    const char* why = nullptr;
    d->pok = tl::persistent_prepare(ps, d->ncu, &why);
    if (!d->pok && why) d->pwhy = why;
  }
  if (d->pok) {
    // the kernel addresses layer l of tensor t as q(0) + l * stride with the scales right
    // after each int8 block (the v2 payload order, thallama_q8_map); anything else -> the
    // multi-launch int8 step
    const QuantizedTensor* ts[7] = {w8->wq, w8->wk, w8->wv, w8->wo, w8->w1, w8->w2, w8->w3};
    const long long dim = d->dim, kvd = d->kv_dim, hid = d->hidden;
    const long long nel[7] = {dim * dim, kvd * dim, kvd * dim, dim * dim, hid * dim, dim * hid, hid * dim};
    for (int t = 0; t < 7 && d->pok; ++t) {
      const signed char* b = (const signed char*)ts[t][0].q;
      const long long stride = d->L > 1 ? (const signed char*)ts[t][1].q - b : 0;
      for (int l = 0; l < d->L; ++l) {
        const signed char* q = (const signed char*)ts[t][l].q;
        if (q != b + l * stride || (const signed char*)ts[t][l].s != q + nel[t]) {
          d->pok = false;
          d->pwhy = "int8 tensors not in the v2 payload layout";
          break;
        }
      }
      d->pq8w[t] = b;
      d->pq8ls[t] = stride;
    }
    if ((const signed char*)w8->wcls->s != (const signed char*)w8->wcls->q + (long long)d->V * dim) {
      d->pok = false;
      d->pwhy = "int8 classifier not in the v2 payload layout";
    }
  }
  return 0;
}

extern "C" thablasStatus_t thaDNN_q8_forward_batch(thablasHandle_t handle, int n_batches, Config* p,
                                                   Q8TransformerWeights* w, RunState* s_batch, int token[], int pos[],
                                                   float* logits_host) {
  if (!p || !w || !s_batch || !token || !pos || !logits_host || n_batches <= 0) return THABLAS_STATUS_INVALID_VALUE;
  int dev = 0;
  CHECK_HIP(hipGetDevice(&dev));
  DecKey key(dev, handle.calc_stream, n_batches, p->dim, p->hidden_dim, p->n_layers, p->n_heads, p->n_kv_heads,
             p->seq_len, -(p->vocab_size < 0 ? -p->vocab_size : p->vocab_size) - 1 /* int8 keyspace */);
  const int r = with_cached_decoder(key, p, nullptr, w, s_batch, n_batches, handle.calc_stream,
                                    "thaDNN_q8_forward_batch", [&](thallama_decoder* d) {
                                      const int e = thallama_decoder_forward(d, token, pos, logits_host);
                                      if (e) fprintf(stderr, "thaDNN_q8_forward_batch: %s\n", thallama_last_error());
                                      return e;
                                    });
  if (r) return r == (int)hipErrorInvalidValue ? THABLAS_STATUS_INVALID_VALUE : THABLAS_STATUS_EXECUTION_FAILED;
  return THABLAS_STATUS_SUCCESS;
}

// ------------------------------------------------------------------ batched prefill
// Prompt tokens go through each layer together (prefill.hip): one fp32-MFMA GEMM per
// projection for up to kPrefillChunk tokens, the decode attention kernel over the chunk's
// positions, K/V rows written at pos0.. of sequence b.  No logits: the caller's next decode
// step starts from the token after the prefilled ones.  fp32 weights, head size 64/128/256.
// A prefill projection.  Up to kPrefillGemvMax tokens the decode GEMV (matrix cores from 4
// tokens on: gemv_mfma.hpp, ~4.5 TB/s) beats the GEMM, whose grid is only M/128 blocks at
// one 64-token tile (7B: 32-172 blocks, ~1 TB/s); the same epilogues either way.
static constexpr int kPrefillGemvMax = 16;
static constexpr int kPrefillGemmMin = 80;
static hipError_t prefill_proj(thallama_decoder* d, int mode, const tl::PGemmArgs& g, long long kv_l_off) {
  if (g.n > kPrefillGemvMax) return tl::prefill_gemm(mode, g, d->stream);
  tl::GemvParams p = {};
  p.W0 = g.W0; p.W1 = g.W1; p.W2 = g.W2;
  p.K = g.K;
  p.nb = g.n;
  p.x = g.X; p.x_stride = g.ldx;
  p.y = g.Y; p.y_stride = g.ldy;
  p.pos = d->pf_pos;
  if (mode == tl::GM_QKV) {
    p.n_items = g.M / 2;
    p.kc = g.kc - kv_l_off; p.vc = g.vc - kv_l_off;  // one sequence: no batch stride
    p.kv_b_stride = 0; p.kv_l_off = kv_l_off;
    p.dim = g.dim; p.kv_dim = g.kv_dim; p.head_size = g.head_size; p.rope = g.rope;
  } else {
    p.n_items = mode == tl::GM_SWIGLU ? g.M / 2 : g.M;
  }
  return gemv(d, mode, p, nullptr, nullptr, nullptr);
}

// int8 weights (runq group size 64, the exact multi-launch kernels of q8_exact.hip): chunks of up
// to 8 prompt tokens go through the batched exact step as 8 "sequences" at their own positions over
// slot b's cache — the QKV launch writes every chunk token's K/V row before the attention launch
// reads them, so token t sees rows 0..pos0+t as in a decode step, and every token's arithmetic is
// runq's (each sequence of the exact kernels is bit-identical to runq.c's forward): the K/V rows
// are bit-identical to stepping through the prompt, and the weights are read once per 8 tokens
// instead of once per token (src/llama.cpp:1029-1031 steps through the prompt).
static int prefill_q8(thallama_decoder* d, int b, const int* tokens_h, int n, int pos0) {
  if (!d->q8x || !d->pf_att || !d->pf_x) {
    g_last_error = "thallama_decoder_prefill: int8 prefill needs the exact int8 kernels (group size 64)";
    return (int)hipErrorNotSupported;
  }
  hipStream_t st = d->stream;
  const long long kv_b_stride = (long long)d->L * d->S * d->kv_dim;
  float* kc_b = d->s.key_cache + (long long)b * kv_b_stride;
  float* vc_b = d->s.value_cache + (long long)b * kv_b_stride;
  memcpy(d->pf_tok_h, tokens_h, sizeof(int) * n);
  TL_TRY(hipMemcpyAsync(d->pf_tok, d->pf_tok_h, sizeof(int) * n, hipMemcpyHostToDevice, st));
  for (int c = 0; c < n; c += kPrefillQ8Chunk) {
    const int m = n - c < kPrefillQ8Chunk ? n - c : kPrefillQ8Chunk;
    TL_TRY(tl::prefill_positions(d->pf_pos, pos0 + c, m, st));
    const StepIO io{d->pf_x, d->pf_xb, d->pf_q, d->pf_hb, nullptr, kc_b, vc_b, 0, d->pf_tok + c, d->pf_pos, m,
                    d->pf_att};
    const int r = enqueue_step_io(d, io);
    if (r) return r;
  }
  TL_TRY(hipStreamSynchronize(st));
  return 0;
}

extern "C" int thallama_decoder_prefill(thallama_decoder* d, int b, const int* tokens_h, int n, int pos0) {
  if (!d || !tokens_h || n < 0 || b < 0 || b >= d->B || pos0 < 0 || pos0 + n > d->S) {
    g_last_error = "thallama_decoder_prefill: invalid argument";
    return (int)hipErrorInvalidValue;
  }
  if (n == 0) return 0;
  if (!prefill_shape_ok(d)) {
    g_last_error = "thallama_decoder_prefill: unsupported (head size not 64/128/256)";
    return (int)hipErrorNotSupported;
  }
  for (int i = 0; i < n; ++i)
    if (tokens_h[i] < 0 || tokens_h[i] >= d->V) {
      g_last_error = "thallama_decoder_prefill: token out of range";
      return (int)hipErrorInvalidValue;
    }
  // the pinned staging may still feed a copy in flight (an earlier call that returned early, or an
  // asynchronous greedy call), and a persistent give-up of an asynchronous call is reported before
  // this call writes any K/V row (as upload_tok_pos does for the decode steps)
  TL_TRY(hipStreamSynchronize(d->stream));
  if (const int r = check_async(d)) return r;
  if (d->q8) return prefill_q8(d, b, tokens_h, n, pos0);
  const int CH = kPrefillChunk, dim = d->dim, hid = d->hidden, kvd = d->kv_dim, S = d->S;
  const int max_ns = kPrefillMaxSplits;
  if (!d->pf_x) {
    g_last_error = "thallama_decoder_prefill: no prefill workspace";
    return (int)hipErrorNotSupported;
  }
  const TransformerWeights& w = d->w;
  const long long kv_b_stride = (long long)d->L * S * kvd;
  float* kc_b = d->s.key_cache + (long long)b * kv_b_stride;
  float* vc_b = d->s.value_cache + (long long)b * kv_b_stride;
  hipStream_t st = d->stream;
  // the prompt's ids through pinned staging (idle: synchronised above)
  memcpy(d->pf_tok_h, tokens_h, sizeof(int) * n);
  TL_TRY(hipMemcpyAsync(d->pf_tok, d->pf_tok_h, sizeof(int) * n, hipMemcpyHostToDevice, st));
  for (int c = 0, m = 0; c < n; c += m) {
    // GEMM chunks of up to CH tokens; a rest of at most kPrefillGemmMin tokens goes through
    // the decode GEMV 16 tokens at a time (about 6 ms per 16 at 7B, against a GEMM floor of
    // about 31 ms for any chunk up to 64 tokens: tools/prefill_bench.py)
    const int rest = n - c;
    m = rest > kPrefillGemmMin ? (rest < CH ? rest : CH) : (rest < kPrefillGemvMax ? rest : kPrefillGemvMax);
    const int p0 = pos0 + c;
    TL_TRY(tl::prefill_positions(d->pf_pos, p0, m, st));
    TL_TRY(tl::prefill_embed(d->pf_x, w.token_embedding_table, d->pf_tok + c, m, dim, st));
    for (int l = 0; l < d->L; ++l) {
      const long long ll = l;
      tl::PGemmArgs g = {};
      g.n = m;
      g.dim = dim; g.kv_dim = kvd; g.head_size = d->hs; g.rope = d->rope_d; g.pos0 = p0;
      // RMSNorm + QKV + RoPE + K/V rows
      TL_TRY(tl::prefill_rmsnorm(d->pf_xn, d->pf_x, w.rms_att_weight + ll * dim, m, dim, st));
      g.X = d->pf_xn; g.ldx = dim; g.K = dim; g.M = dim + 2 * kvd;
      g.W0 = w.wq + ll * dim * dim; g.W1 = w.wk + ll * dim * kvd; g.W2 = w.wv + ll * dim * kvd;
      g.Y = d->pf_q; g.ldy = dim;
      g.kc = kc_b + ll * S * kvd; g.vc = vc_b + ll * S * kvd;
      TL_TRY(prefill_proj(d, tl::GM_QKV, g, ll * S * kvd));
      // causal attention: the chunk's m positions as "sequences" over this sequence's cache
      {
        tl::AttnWaveParams wp = {};
        tl::AttnParams& a = wp.a;
        a.q = d->pf_q; a.kc = kc_b; a.vc = vc_b; a.kv_b_stride = 0; a.kv_l_off = ll * S * kvd;
        a.pos = d->pf_pos; a.out = d->pf_xb; a.part = d->pf_part;
        a.dim = dim; a.kv_dim = kvd; a.head_size = d->hs; a.n_heads = d->H; a.kv_mul = d->kv_mul;
        a.seq_len = S; a.nsplit = 1; a.min_chunk = 32;
        wp.cnt = d->pf_cnt; wp.B = m;
        int ns = (256 + m * d->H - 1) / (m * d->H);
        ns = ns < 1 ? 1 : (ns > max_ns ? max_ns : ns);
        wp.NS = ns;
        const int units = m * d->H * ns;
        if (d->hs == 64)
          hipLaunchKernelGGL((tl::attn_wave_kernel<64, kAttnChunk>), dim3(units), dim3(64), 0, st, wp);
        else if (d->hs == 128)
          hipLaunchKernelGGL((tl::attn_wave_kernel<128, kAttnChunk>), dim3(units), dim3(64), 0, st, wp);
        else
          hipLaunchKernelGGL((tl::attn_wave_kernel<256, kAttnChunk / 2>), dim3(units), dim3(64), 0, st, wp);
        TL_TRY(hipGetLastError());
      }
      // Wo + residual
      g.X = d->pf_xb; g.ldx = dim; g.K = dim; g.M = dim; g.W0 = w.wo + ll * dim * dim; g.Y = d->pf_x; g.ldy = dim;
      TL_TRY(prefill_proj(d, tl::GM_RESID, g, 0));
      // RMSNorm + W1/W3 + SwiGLU
      TL_TRY(tl::prefill_rmsnorm(d->pf_xn, d->pf_x, w.rms_ffn_weight + ll * dim, m, dim, st));
      g.X = d->pf_xn; g.ldx = dim; g.K = dim; g.M = 2 * hid;
      g.W0 = w.w1 + ll * dim * hid; g.W1 = w.w3 + ll * dim * hid; g.Y = d->pf_hb; g.ldy = hid;
      TL_TRY(prefill_proj(d, tl::GM_SWIGLU, g, 0));
      // W2 + residual
      g.X = d->pf_hb; g.ldx = hid; g.K = hid; g.M = dim; g.W0 = w.w2 + ll * dim * hid; g.Y = d->pf_x; g.ldy = dim;
      TL_TRY(prefill_proj(d, tl::GM_RESID, g, 0));
    }
  }
  TL_TRY(hipStreamSynchronize(st));
  return 0;
}
