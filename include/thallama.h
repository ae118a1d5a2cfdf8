/* thallama.h — native runtime entry points of the MI355X build that sit beside the
 * reference-compatible thaBLAS/thaDNN surface.  Plain C ABI: opaque handles,
 * plain pointers and sizes; bound from C++ (apps/), ctypes (tests/, bench.py).
 *
 *  - decoder: the fused decode step of thaDNN_s_forward_batch
 *    (reference src/thaDNN.cpp:13-81) as a reusable object that owns its
 *    workspace (device token/pos, RoPE table, attention partials), can keep the
 *    whole greedy loop on the device (argmax feeding the next token; reference
 *    samples on the host every step, src/llama.cpp:1027-1050) and can replay
 *    one step as a hipGraph.
 *  - synthetic weights: deterministic counter-based N(0, sigma)-shaped init
 *    (train/model.py:232-247 distribution), bit-identical to the host oracle's
 *    generator (oracle/oracle.c).
 *  - small device-memory helpers so tests need nothing but ctypes.
 */
#ifndef THALLAMA_H
#define THALLAMA_H
#include <stddef.h>
#include <stdint.h>
#include "models.hpp"
#include "thaQ8.hpp"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct thallama_decoder thallama_decoder;

/* Option keys for thallama_decoder_set */
enum {
  THALLAMA_OPT_NT_WEIGHTS = 1,   /* 0/1: non-temporal weight loads (default: 1 if weights > 1 GiB) */
  THALLAMA_OPT_ATTN_SPLITS = 2,  /* key splits per (head, seq); 0 = auto */
  THALLAMA_OPT_USE_GRAPH = 3,    /* 0/1: replay greedy steps from a captured hipGraph */
  THALLAMA_OPT_PROFILE = 4,      /* 0/1: HIP events around every kernel class (eager only) */
  THALLAMA_OPT_PERSISTENT = 5,   /* 0/1: whole step as ONE persistent launch (fp32 batch 1..8,
                                    int8 batch 1; head size 64/128).  Default 1 where supported,
                                    except fp32 batch 5..8 (default 0: slower than multi-launch
                                    there; at batch 8 it is the K-split step).  Profiled as the single class THALLAMA_K_STEP. */
  THALLAMA_OPT_PERSIST_FAULT = 6,  /* test hook: the next persistent launch runs without its
                                    block 0 (as if the grid were not co-resident): its waits
                                    give up, the call disables the path and re-runs on the
                                    multi-launch step. */
  THALLAMA_OPT_KSPLIT = 7,       /* 0/1: at 8 sequences the persistent step gives each CU a
                                    (row group, K slice) tile (persist_k.hip) instead of whole
                                    rows (persist_b.hip).  Default 1 where the shape is supported
                                    (the persistent step itself stays off by default at 8
                                    sequences; THALLAMA_KSPLIT=1 in the environment at creation,
                                    or THALLAMA_OPT_PERSISTENT=1, turns it on). */
};

/* 1 if the decoder runs its steps as one persistent launch (THALLAMA_OPT_PERSISTENT
 * requested and the shape supported), else 0. */
int thallama_decoder_persistent(thallama_decoder* d);
/* 1 if that persistent step is the K-split one (8 sequences, THALLAMA_OPT_KSPLIT), else 0. */
int thallama_decoder_ksplit(thallama_decoder* d);
/* 1 if the persistent step is dispatched as a cooperative launch (the runtime checks the grid's
 * co-residency; replays of a captured step keep cooperative dispatch on ROCm 7.2 by observation,
 * and every wait is bounded either way), 0 for a plain launch (THALLAMA_PERSIST_COOP=0 or no
 * device support). */
int thallama_persistent_cooperative(void);
/* Diagnostics: the persistent step's hand-off granules ({value, tag}: x | xb | hb | q k v | int8
 * codes | scales; the last layer's after a launch) into host[n]; returns the count (host NULL:
 * count only). */
int thallama_decoder_granules(thallama_decoder* d, unsigned long long* host, size_t n);
/* Diagnostics: enable != 0 allocates a timeline buffer that every later persistent launch
 * fills with 100-MHz clock stamps, [grid][5*n_layers+1][4] (phase start, input staged,
 * slots reduced, epilogue drained); host != NULL copies up to n stamps out (synchronous).
 * Returns the number of stamps per launch, or a negative error. */
int thallama_decoder_ptrace(thallama_decoder* d, int enable, unsigned long long* host, size_t n);

/* Kernel classes for profiling */
enum {
  THALLAMA_K_QKV = 0, THALLAMA_K_ATTN = 1, THALLAMA_K_WO = 2, THALLAMA_K_FFN_UP = 3,
  THALLAMA_K_FFN_DOWN = 4, THALLAMA_K_CLS = 5, THALLAMA_K_ARGMAX = 6,
  THALLAMA_K_STEP = 7,  /* the whole step as one persistent launch (THALLAMA_OPT_PERSISTENT) */
  THALLAMA_K_COUNT = 8
};

/* w and s hold DEVICE pointers (as produced by copy_weight_to_device /
 * alloc_state_to_device_batch or any equivalent layout).  stream may be 0:
 * the decoder then creates its own non-blocking stream.  Returns 0 on success. */
int thallama_decoder_create(thallama_decoder** out, const Config* cfg, const TransformerWeights* w,
                            const RunState* s, int batch, hipStream_t stream);
/* Same, for int8 weights (include/thaQ8.hpp: a mapped v2 payload whose
 * token_embedding_table has been dequantised). */
int thallama_decoder_create_q8(thallama_decoder** out, const Config* cfg, const Q8TransformerWeights* w8,
                               const RunState* s, int batch, hipStream_t stream);
void thallama_decoder_destroy(thallama_decoder* d);
int thallama_decoder_set(thallama_decoder* d, int key, int value);
hipStream_t thallama_decoder_stream(thallama_decoder* d);

/* One synchronous step with host token/pos, logits copied to logits_h[batch*vocab]
 * (logits_h may be NULL).  Exactly thaDNN_s_forward_batch's contract. */
int thallama_decoder_forward(thallama_decoder* d, const int* token_h, const int* pos_h, float* logits_h);

/* Greedy decode n_steps on the device.  Sequence b starts from token0_h[b] at
 * pos0_h[b]; step i writes the argmax token of every sequence to
 * tokens_out_h[i*batch + b] (may be NULL).  Asynchronous unless sync != 0 (or tokens are
 * requested).  Returns 0 on success.  A persistent step that gave up inside an asynchronous
 * call is reported by the next call on the decoder (hipErrorIllegalState: that call's tokens
 * and K/V rows are invalid). */
int thallama_decoder_greedy(thallama_decoder* d, const int* token0_h, const int* pos0_h, int n_steps,
                            int* tokens_out_h, int sync);

/* Batched prompt processing for sequence slot b: the n tokens tokens_h[0..n) at positions
 * pos0..pos0+n-1 go through every layer together (fp32-MFMA GEMMs; K/V rows written), with
 * no logits — the next thallama_decoder_forward/greedy step continues from position pos0+n.
 * Equivalent to n forced decode steps of that slot (src/llama.cpp:1029-1031) within the fp32
 * tolerance.  Returns hipErrorNotSupported for int8 decoders or head sizes other than
 * 64/128/256 (callers then feed the prompt token by token).  Synchronous. */
int thallama_decoder_prefill(thallama_decoder* d, int b, const int* tokens_h, int n, int pos0);

/* The decoder as the host scheduler's callbacks (include/thallama_host.h thallama_step_fn /
 * thallama_prefill_fn, ctx = the decoder; worker ignored): step = thallama_decoder_forward,
 * prefill = thallama_decoder_prefill (1 = not supported, negative = error). */
int thallama_decoder_step_cb(void* ctx, int worker, int batch, const int* token, const int* pos, float* logits);
int thallama_decoder_prefill_cb(void* ctx, int worker, int slot, const int* tokens, int n, int pos0);
/* One greedy step with host token/pos whose argmax stays on the device: next_h[b] = the first
 * index of the maximum of slot b's logits (sample_argmax, src/llama.cpp:275-286); only the B ids
 * are copied back.  Synchronous.  And as thallama_argmax_step_fn (include/thallama_host.h). */
int thallama_decoder_step_argmax(thallama_decoder* d, const int* token_h, const int* pos_h, int* next_h);
int thallama_decoder_argmax_cb(void* ctx, int worker, int batch, const int* token, const int* pos, int* next);

/* Copy the device logits of the last step into logits_h[batch*vocab] (synchronous). */
int thallama_decoder_logits(thallama_decoder* d, float* logits_h);

/* Wait for the decoder's queued work; reports an earlier asynchronous call's give-up. */
int thallama_decoder_sync(thallama_decoder* d);

/* Profiling (THALLAMA_OPT_PROFILE=1): accumulated ms and launch count per kernel class
 * since the last reset. */
int thallama_decoder_prof(thallama_decoder* d, int kclass, double* total_ms, long long* count);
void thallama_decoder_prof_reset(thallama_decoder* d);

/* One pipeline stage (thaDNN_s_forward_batch_multiple_pipe_line's building block): decoder d is
 * built over the stage's layer range (cfg.n_layers = layers of the stage).  embed: layer 0 reads
 * the tokens' embedding rows (first stage), else d's RunState x holds the input.  logits_h
 * (last stage): final norm + classifier, logits copied out, synchronised.  Otherwise x_next
 * (device next_dev) receives the residual stream and the stage's event is recorded; a later
 * stage passes this decoder as `wait`.  Multi-launch step, fp32 weights. */
int thallama_decoder_stage(thallama_decoder* d, const int* token_h, const int* pos_h, int embed, float* logits_h,
                           const thallama_decoder* wait, float* x_next, int next_dev);

/* thaDNN_s_forward_batch / thaDNN_q8_forward_batch (and the pipeline drivers' stage decoders) keep
 * one decoder per (device, stream, batch, config, dtype), made for the caller's weight and state
 * buffers; a call with other buffers replaces it, and at most cap stay cached (least recently used
 * dropped; the cap starts at 8 and grows by one, up to 256, whenever a recently dropped key comes
 * back, so it follows the callers' working set; clearing the cache resets the cap).  Concurrent callers are safe: a dropped decoder is
 * freed when the last call using it returns.  The cached count, the cap, the live count (cached +
 * dropped but still running), and a way to drop them all (e.g. before the caller frees its
 * buffers). */
int thallama_forward_batch_cache_size(void);
int thallama_forward_batch_cache_cap(void);
int thallama_forward_batch_live(void);
void thallama_forward_batch_cache_clear(void);

/* Algorithmic HBM bytes of one step for kernel class kclass at the given positions
 * (weights once + KV rows read/written), used for roofline reporting. */
double thallama_step_bytes(const Config* cfg, int batch, int kclass, const int* pos_h);

/* Micro-benchmark of one streaming-GEMV launch shape (tools/gemv_sweep.py).  mode: 0 store,
 * 1 residual, 2 SwiGLU (two MxK matrices), 3 QKV (dim = kv_dim = K, M ignored).  Variant:
 * items per wave, waves per block, prefetch-before-staging, non-temporal loads.  Weights
 * rotate over >= 1.5 GiB so every launch streams from HBM.  *us_out = avg us per launch. */
int thallama_gemv_bench(int mode, int M, int K, int nb, int ipw, int waves, int pf, int nt, int iters,
                        double* us_out);

/* Test hook: the wave-parallel left-to-right fp32 sum (csrc/seqsum.hpp) of `count` arrays of n
 * floats (device in_d, n <= 8192) into out_d[count]; synchronous. */
int thallama_seqsum_check(const float* in_d, int n, int count, float* out_d);
/* Same with the register form (n <= 4096), plus the clock cycles of each call in cyc_d[count]. */
int thallama_seqsum_time(const float* in_d, int n, int count, float* out_d, long long* cyc_d);

/* ---- synthetic weights ------------------------------------------------- */
/* Fill a v0 arena (layout of thallama_map_weights) with the deterministic synthetic
 * model: N(0,0.02)-shaped linears/embedding, wo & w3 scaled by 1/sqrt(2L), norms 1,
 * the unused freq_cis block 0.  `arena` is a DEVICE pointer; enqueued on stream. */
int thallama_synth_arena(float* arena, const Config* cfg, int shared_weights, uint64_t seed,
                         hipStream_t stream);

/* ---- device memory helpers (ctypes convenience) ------------------------ */
int thallama_device_count(void);
int thallama_set_device(int dev);
void* thallama_malloc(size_t bytes);
int thallama_free(void* p);
int thallama_memcpy_h2d(void* dst, const void* src, size_t bytes);
int thallama_memcpy_d2h(void* dst, const void* src, size_t bytes);
int thallama_memcpy_d2d(void* dst, const void* src, size_t bytes);
int thallama_memset(void* dst, int value, size_t bytes);
int thallama_sync(void);
const char* thallama_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
