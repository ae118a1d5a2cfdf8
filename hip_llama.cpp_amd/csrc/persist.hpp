// persist.hpp — the one-launch decode step (persist.hip) for batch 1, fp32 or Q8_0 weights.
#pragma once
#include <hip/hip_runtime.h>

namespace tl {

struct PStep {
  // weights (reference TransformerWeights, include/models.hpp)
  const float *emb, *rms_att, *rms_ffn, *wq, *wk, *wv, *wo, *w1, *w2, *w3, *rms_final, *wcls;
  int dim, hid, kvd, L, S, V, H, kv_mul, hs, NS;
  // run state
  float *x, *xb, *logits, *kc, *vc, *part;
  unsigned* tickets;        // attention combine tickets [L][H], zeroed before every launch
  const float2* rope;       // [S][hs/2] (cos, sin)
  int* tok;                 // [1] read at layer 0; rewritten by the argmax tail
  int* pos;                 // [1] read everywhere; advanced by the argmax tail
  int* out;                 // [S] greedy tokens by position (argmax tail), may be null
  // hand-off granules {value, tag} (zero once at allocation; tags are never 0)
  unsigned long long *gx, *gxb, *ghb, *gqkv;  // [dim], [dim], [hidden], [dim + 2*kv_dim]
  unsigned long long* gsc;   // int8: attention score granules [H][S] (attention.hpp attn_unit_split)
  unsigned* sync;           // kPSyncWords barrier shards, zeroed before every launch
  unsigned* err;            // sticky: a wait gave up (1: barrier, 2: hand-off)
  unsigned* seq;            // launch sequence (tags), advanced by the kernel
  unsigned long long* bmax; // [grid] per-block classifier argmax
  int argmax;               // run the argmax + advance tail
  int pad_floats;           // LDS activation strip (floats), >= every phase's padded K
  unsigned long long* trace; // optional [grid][5L+1][kTraceSlots] timeline (100-MHz clock), or null
  // Q8_0 weights (runq.c layout, include/thaQ8.hpp) instead of the fp32 matrices: group size
  // (64; 0 = fp32); per tensor (wq, wk, wv, wo, w1, w2, w3) the layer-0 int8 block and the
  // byte stride between layers, each layer's fp32 scales directly after its int8 block (the
  // v2 payload order; the host checks it); the classifier's pair separately.  Norms and the
  // (dequantised) embedding stay fp32 in the fields above.  Plain arguments, so every
  // per-phase address is scalar arithmetic (a device table read put them in VGPRs / scratch).
  int q8;
  const signed char* q8w[7];
  long long q8ls[7];
  const signed char* qcls;
  const float* scls;
  int q8_pad;               // LDS bytes of the quantised activation strip (Q8 only)
  int n_sqa, n_scr, n_cw;   // Q8 (exact arithmetic) LDS floats: norm squares, long-row products /
                            // attention strip, streaming-wave chain scratch (persistent_prepare)
  int pgp;                  // Q8: row stride (floats) of the long-row products
  int ang;                  // Q8: attention units per head (persistent_prepare)
  int attn_help;            // fp32 batch 1: the staging strip also holds an attention window, so a
                            // streaming wave runs a second attention unit per block at long contexts
  int long_ctx;             // host: launch the instantiation with that helper (persistent_long_ctx)
  int poll_long;            // large model (dim >= 2048): input sweeps back off (common.hpp gran_backoff)
  int fault;                // test hook (THALLAMA_OPT_PERSIST_FAULT): block 0 exits at once, as
                            // if the grid were not co-resident; every other wait gives up
  int B;                    // batched step (persist_b.hip): 2..8 sequences; tok / pos / out and every
                            // hand-off buffer then hold B rows, bmax [grid][8], tickets [L][B*H];
                            // n_scr = the LDS row-chunk partials (persistent_prepare_b)
  unsigned long long* gk;   // K-split step (persist_k.hip): its hand-off area, persistent_k_granules
                            // granules, zeroed once at allocation
};

constexpr int kPSyncWords = 8 * 32;   // 8 shard counters, one 128-B line each
constexpr int kPResFloats = 1024;     // per-block row-chunk results (LDS)
constexpr int kTraceSlots = 16;       // timeline stamps per block and phase (PStep::trace)

// Host: can this step run as one launch on `ncu` co-resident blocks?  Sets pad_floats.
bool persistent_prepare(PStep& p, int ncu, const char** why);
// Launch only: the caller zeroes p.sync (kPSyncWords) on stream s right before (a memset
// node ahead of the kernel node when captured).
hipError_t launch_persistent_step(const PStep& p, hipStream_t s, int ncu);
// True if launch_persistent_step uses a cooperative launch (co-residency guaranteed).
bool persistent_cooperative();
// fp32 batch 1: from this many keys on the step runs the attention helper (persist.hip), so the
// caller sets PStep::long_ctx and keeps one captured graph per setting
constexpr int kAttnHelpMinKeys = 512;
inline bool persistent_long_ctx(int pos) { return pos + 1 >= kAttnHelpMinKeys; }
// The same for 2..8 sequences with fp32 weights (persist_b.hip; p.B set).
bool persistent_prepare_b(PStep& p, int ncu, const char** why);
hipError_t launch_persistent_step_b(const PStep& p, hipStream_t s, int ncu);
// 8 sequences with fp32 weights, every GEMV phase K-split over the CUs (persist_k.hip): the
// granules its hand-off area needs (PStep::gk), the shape check, the launch.
long long persistent_k_granules(const PStep& p, int ncu);
bool persistent_prepare_k(PStep& p, int ncu, const char** why);
hipError_t launch_persistent_step_k(const PStep& p, hipStream_t s, int ncu);

}  // namespace tl
