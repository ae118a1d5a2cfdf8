// q8.hip — int8 (Q8_0, runq layout) entry points: launcher of gemv_q8.hpp, activation /
// weight quantisation kernels, v2 payload mapping (include/thaQ8.hpp).
#include <fcntl.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <unistd.h>
#include "../../include/thaQ8.hpp"
#include "../../include/hip_helper.hpp"
#include "gemv_q8.hpp"
#include "gemv_q8_mfma.hpp"
#include "q8_dispatch.hpp"
#include "api_lock.hpp"

namespace tl {

static inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }


bool gemv_q8_fast_ok(const GemvParams& p) {
  if (p.K <= 0 || p.gs < 32 || p.gs > 128 || (p.gs & (p.gs - 1)) || p.K % p.gs || (p.K & 15)) return false;
  const void* ptrs[] = {p.Q0, p.Q1, p.Q2, p.x, p.emb, p.rms_w};
  for (const void* q : ptrs)
    if (q && !al16(q)) return false;
  if (p.x_stride & 3) return false;
  return true;
}

// Fallback: one wave per (row, sequence), scalar, any K / GS with K % GS == 0.
template <int MODE>
__global__ void __launch_bounds__(256) gemv_q8_generic_kernel(GemvParams p) {
  keep_implicit_args();  // (rocprofv3 --pmc: common.hpp)
  constexpr int RPI = RowsPerItem<MODE>::v;
  const int lane = threadIdx.x & 63;
  const int item = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int b = blockIdx.y;
  if (item >= p.n_items) return;
  const float* xin = p.tok ? p.emb + (long long)p.tok[b] * p.K : p.x + b * p.x_stride;
  float s = 1.f;
  if (p.rms_w) {
    float t = 0.f;
    for (int k = lane; k < p.K; k += 64) t = fmaf(xin[k], xin[k], t);
    t = wave_sum(t);
    s = __fdiv_rn(1.0f, sqrtf(__fadd_rn(__fdiv_rn(t, (float)p.K), 1e-5f)));
  }
  if (p.tok && item == 0 && (threadIdx.x >> 6) == 0)
    for (int k = lane; k < p.K; k += 64) p.x_out[b * p.x_stride + k] = xin[k];
  auto xv = [&](int k) { return p.rms_w ? __fmul_rn(p.rms_w[k], __fmul_rn(s, xin[k])) : xin[k]; };
  float v[2][1] = {{0.f}, {0.f}};
  const int ng = p.K / p.gs;
  for (int r = 0; r < RPI; ++r) {
    const int8_t* q;
    const float* sc;
    q8_item_row<MODE>(p, item, r, q, sc);
    float acc = 0.f;
    for (int g = lane; g < ng; g += 64) {  // lane owns whole groups
      float wmax = 0.f;
      for (int i = 0; i < p.gs; ++i) wmax = fmaxf(wmax, fabsf(xv(g * p.gs + i)));
      const float xs = __fdiv_rn(wmax, 127.0f);
      int isum = 0;
      for (int i = 0; i < p.gs; ++i) isum += q8_round(__fdiv_rn(xv(g * p.gs + i), xs)) * (int)q[g * p.gs + i];
      acc += __fmul_rn(__fmul_rn((float)isum, sc[g]), xs);
    }
    v[r][0] = wave_sum(acc);
  }
  GemvParams pp = p;
  pp.nb = 1;
  if constexpr (MODE == GM_STORE) {
    pp.y_off = p.y_off + (long long)b * p.y_stride + (p.has_pos ? (long long)p.has_pos * p.pos[b] : 0);
    pp.has_pos = 0;
  } else if constexpr (MODE == GM_QKV) {
    pp.y = p.y + (long long)b * p.y_stride;
    pp.kc = p.kc + (long long)b * p.kv_b_stride;
    pp.vc = p.vc + (long long)b * p.kv_b_stride;
    pp.pos = p.pos + b;
  } else {
    pp.y = p.y + (long long)b * p.y_stride;
  }
  epilogue<MODE, 1>(pp, item, v, lane);
}

template <int MODE, int NB, int LPG>
static void launch_q8_one(const GemvParams& p, hipStream_t s, bool nt) {
  // activation staging budget: int8 [NB][kc] + fp32 scales; chunks are whole wave-loads
  int kc = (40960 / NB) & ~1023;
  if (kc < 1024) kc = 1024;
  if (kc >= p.K) kc = p.K;
  kc -= kc % p.gs;
  const size_t lds = 64 + 256 + (size_t)NB * (kc / p.gs) * 4 + (size_t)NB * kc;
  // items per wave: 4 at one sequence (4-8 rows = 16-32 KiB in flight per wave), 2 above
  constexpr int IPW = NB == 1 ? 4 : 2;
  constexpr int WAVES = 4;
  const int blocks = (p.n_items + WAVES * IPW - 1) / (WAVES * IPW);
  if (nt)
    hipLaunchKernelGGL((gemv_q8_kernel<MODE, NB, LPG, true, WAVES, IPW>), dim3(blocks), dim3(WAVES * 64), lds, s, p, kc);
  else
    hipLaunchKernelGGL((gemv_q8_kernel<MODE, NB, LPG, false, WAVES, IPW>), dim3(blocks), dim3(WAVES * 64), lds, s, p,
                       kc);
}

template <int MODE, int NB>
static void launch_q8_nb(const GemvParams& p, hipStream_t s, bool nt) {
  switch (p.gs) {
    case 32: launch_q8_one<MODE, NB, 2>(p, s, nt); break;
    case 64: launch_q8_one<MODE, NB, 4>(p, s, nt); break;
    default: launch_q8_one<MODE, NB, 8>(p, s, nt); break;
  }
}

template <int MODE>
static hipError_t launch_q8_mode(const GemvParams& p0, hipStream_t s, bool nt) {
  if (p0.n_items <= 0 || p0.nb <= 0) return hipSuccess;
  if (!gemv_q8_fast_ok(p0)) {
    hipLaunchKernelGGL((gemv_q8_generic_kernel<MODE>), dim3((p0.n_items + 3) / 4, p0.nb), dim3(256), 0, s, p0);
    return hipGetLastError();
  }
  for (int b0 = 0; b0 < p0.nb; b0 += 8) {
    GemvParams p = p0;
    p.nb = p0.nb - b0 < 8 ? p0.nb - b0 : 8;
    if (b0) {
      if (p.x) p.x += b0 * p.x_stride;
      if (p.tok) p.tok += b0;
      if (p.x_out) p.x_out += b0 * p.x_stride;
      if (p.pos) p.pos += b0;
      if (MODE == GM_STORE) p.y_off += (long long)b0 * p.y_stride;
      else p.y += (long long)b0 * p.y_stride;
      if (p.kc) p.kc += (long long)b0 * p.kv_b_stride;
      if (p.vc) p.vc += (long long)b0 * p.kv_b_stride;
    }
    if (p.nb >= 2 && p.xq && p.xqs) {
      // quantise once per launch, then the GEMV copies the codes (no per-block prologue)
      const int lpg = p.gs / 16;
      if (p.xq_ready) {
        // the producer (attention, forward.hip) already stored codes + scales; nb <= 8 there
      } else if (p.K <= 3 * 256 * 16) {
        if (lpg == 2) hipLaunchKernelGGL(gemv_q8_prequant_reg_kernel<2>, dim3(p.nb), dim3(256), 0, s, p);
        else if (lpg == 4) hipLaunchKernelGGL(gemv_q8_prequant_reg_kernel<4>, dim3(p.nb), dim3(256), 0, s, p);
        else hipLaunchKernelGGL(gemv_q8_prequant_reg_kernel<8>, dim3(p.nb), dim3(256), 0, s, p);
      } else if (lpg == 2) hipLaunchKernelGGL(gemv_q8_prequant_kernel<2>, dim3(p.nb), dim3(256), 0, s, p);
      else if (lpg == 4) hipLaunchKernelGGL(gemv_q8_prequant_kernel<4>, dim3(p.nb), dim3(256), 0, s, p);
      else hipLaunchKernelGGL(gemv_q8_prequant_kernel<8>, dim3(p.nb), dim3(256), 0, s, p);
      p.rms_w = nullptr;
      p.tok = nullptr;
      p.x_out = nullptr;
    } else {
      p.xq = nullptr;
    }
    if (p.nb >= 4 && p.xq && p.gs == 64 && (p.K & 255) == 0) {
      // 4..8 sequences: the int8 matrix-core kernel (gemv_q8_mfma.hpp), K split across blocks
      // like the fp32 one (in 256-byte runs)
      const int rows = MODE == GM_QKV ? 2 * p.n_items : p.n_items;
      const int tiles = (rows + 15) / 16, nruns = p.K >> 8;
      int ms = p.mpart && p.mcnt ? mfma_target_blocks() / tiles : 1;
      const int cap = nruns / kMfmaWaves;
      if (ms > cap) ms = cap;
      if (ms < 1) ms = 1;
      p.msteps = (nruns + ms - 1) / ms;
      p.msplit = (nruns + p.msteps - 1) / p.msteps;
      if (nt) hipLaunchKernelGGL((gemv_q8_mfma_kernel<MODE, true>), dim3(tiles * p.msplit), dim3(kMfmaWaves * 64), 0, s, p);
      else hipLaunchKernelGGL((gemv_q8_mfma_kernel<MODE, false>), dim3(tiles * p.msplit), dim3(kMfmaWaves * 64), 0, s, p);
    } else if (p.nb == 1) launch_q8_nb<MODE, 1>(p, s, nt);
    else if (p.nb == 2) launch_q8_nb<MODE, 2>(p, s, nt);
    else if (p.nb <= 4) launch_q8_nb<MODE, 4>(p, s, nt);
    else launch_q8_nb<MODE, 8>(p, s, nt);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_gemv_q8(int mode, const GemvParams& p, hipStream_t s, bool nt) {
  switch (mode) {
    case GM_STORE: return launch_q8_mode<GM_STORE>(p, s, nt);
    case GM_RESID: return launch_q8_mode<GM_RESID>(p, s, nt);
    case GM_SWIGLU: return launch_q8_mode<GM_SWIGLU>(p, s, nt);
    case GM_QKV: return launch_q8_mode<GM_QKV>(p, s, nt);
  }
  return hipErrorInvalidValue;
}

}  // namespace tl

using tl::f4;

// ------------------------------------------------------------------ activation quantisation op
__global__ void __launch_bounds__(256) k_q8_quantize(int8_t* q, float* s, const float* x, int n, int gs,
                                                     long long x_stride) {
  const int b = blockIdx.y;
  const int ng = n / gs;
  for (int g = blockIdx.x * 256 + threadIdx.x; g < ng; g += gridDim.x * 256) {
    const float* xg = x + b * x_stride + (long long)g * gs;
    float wmax = 0.f;
    for (int i = 0; i < gs; ++i) wmax = fmaxf(wmax, fabsf(xg[i]));
    const float scale = __fdiv_rn(wmax, 127.0f);
    s[(long long)b * ng + g] = scale;
    int8_t* qg = q + (long long)b * n + (long long)g * gs;
    if (tl::q8_fast_scale(scale)) {  // the hot-path quotient (q8_pack16), exercised by the op tests
      const float r = __fdiv_rn(1.0f, scale);
      for (int i = 0; i < gs; ++i) qg[i] = (int8_t)tl::q8_code_fast(xg[i], scale, r);  // as q8_pack
    } else {
      for (int i = 0; i < gs; ++i) qg[i] = (int8_t)tl::q8_round(__fdiv_rn(xg[i], scale));
    }
  }
}

extern "C" thablasStatus_t thaBLAS_q8_quantize_batch(thablasHandle_t* handle, int n_batches, int8_t* q, float* s,
                                                     float* x, int n, int group_size, int x_stride) {
  if (!handle) return THABLAS_STATUS_HANDLE_IS_NULLPTR;
  if (n_batches < 0 || n < 0 || group_size <= 0 || n % group_size) return THABLAS_STATUS_INVALID_VALUE;
  if (!n_batches || !n) return THABLAS_STATUS_SUCCESS;
  if (!q || !s || !x) return THABLAS_STATUS_INVALID_VALUE;
  const int ng = n / group_size;
  dim3 grid((ng + 255) / 256, n_batches);
  hipLaunchKernelGGL(k_q8_quantize, grid, dim3(256), 0, handle->calc_stream, q, s, x, n, group_size,
                     (long long)x_stride);
  return hipGetLastError() == hipSuccess ? THABLAS_STATUS_SUCCESS : THABLAS_STATUS_EXECUTION_FAILED;
}

extern "C" thablasStatus_t thaBLAS_q8_matmul_batch(thablasHandle_t* handle, int n_batches, float* C, float* x,
                                                   int8_t* wq, float* ws, int K, int M, int group_size,
                                                   int C_batch_size, int x_batch_size) {
  if (!handle) return THABLAS_STATUS_HANDLE_IS_NULLPTR;
  if (n_batches < 0 || K <= 0 || M < 0 || group_size <= 0 || K % group_size) return THABLAS_STATUS_INVALID_VALUE;
  if (!n_batches || !M) return THABLAS_STATUS_SUCCESS;
  if (!C || !x || !wq || !ws) return THABLAS_STATUS_INVALID_VALUE;
  tl::GemvParams p = {};
  p.Q0 = wq;
  p.S0 = ws;
  p.gs = group_size;
  p.K = K;
  p.n_items = M;
  p.nb = n_batches;
  p.x = x;
  p.x_stride = x_batch_size;
  p.y = C;
  p.y_stride = C_batch_size;
  return tl::launch_gemv_q8(tl::GM_STORE, p, handle->calc_stream, false) == hipSuccess
             ? THABLAS_STATUS_SUCCESS : THABLAS_STATUS_EXECUTION_FAILED;
}

// ------------------------------------------------------------------ v2 payload
extern "C" size_t thallama_q8_payload_bytes(const Config* p, int shared, int gs) {
  const size_t L = p->n_layers, dim = p->dim, kvd = (size_t)p->dim * p->n_kv_heads / p->n_heads;
  const size_t hid = p->hidden_dim, V = p->vocab_size < 0 ? -p->vocab_size : p->vocab_size;
  auto qt = [&](size_t n) { return n + 4 * (n / gs); };
  size_t b = 4 * (2 * L * dim + dim);
  b += qt(V * dim);
  b += L * (2 * qt(dim * dim) + 2 * qt(dim * kvd) + 3 * qt(dim * hid));
  if (!shared) b += qt(V * dim);
  return b;
}

static QuantizedTensor* map_qt(unsigned char** ptr, int n, size_t each, int gs) {
  QuantizedTensor* r = (QuantizedTensor*)malloc(sizeof(QuantizedTensor) * (n > 0 ? n : 1));
  unsigned char* p = *ptr;
  for (int i = 0; i < n; ++i) {
    r[i].q = (int8_t*)p;
    p += each;
    r[i].s = (float*)p;
    p += 4 * (each / gs);
  }
  *ptr = p;
  return r;
}

extern "C" int thallama_q8_map(Q8TransformerWeights* w, const Config* p, void* payload, int shared, int gs,
                               float* emb_f32) {
  if (!w || !p || !payload || gs <= 0) return (int)hipErrorInvalidValue;
  const size_t L = p->n_layers, dim = p->dim, kvd = (size_t)p->dim * p->n_kv_heads / p->n_heads;
  const size_t hid = p->hidden_dim, V = p->vocab_size < 0 ? -p->vocab_size : p->vocab_size;
  memset(w, 0, sizeof(*w));
  w->group_size = gs;
  float* f = (float*)payload;
  w->rms_att_weight = f;
  f += L * dim;
  w->rms_ffn_weight = f;
  f += L * dim;
  w->rms_final_weight = f;
  f += dim;
  unsigned char* ptr = (unsigned char*)f;
  w->q_tokens = map_qt(&ptr, 1, V * dim, gs);
  w->token_embedding_table = emb_f32;
  w->wq = map_qt(&ptr, (int)L, dim * dim, gs);
  w->wk = map_qt(&ptr, (int)L, dim * kvd, gs);
  w->wv = map_qt(&ptr, (int)L, dim * kvd, gs);
  w->wo = map_qt(&ptr, (int)L, dim * dim, gs);
  w->w1 = map_qt(&ptr, (int)L, dim * hid, gs);
  w->w2 = map_qt(&ptr, (int)L, hid * dim, gs);
  w->w3 = map_qt(&ptr, (int)L, dim * hid, gs);
  w->wcls = shared ? w->q_tokens : map_qt(&ptr, 1, dim * V, gs);
  return 0;
}

extern "C" void thallama_q8_unmap(Q8TransformerWeights* w) {
  if (!w) return;
  if (w->wcls && w->wcls != w->q_tokens) free(w->wcls);
  free(w->q_tokens);
  free(w->wq); free(w->wk); free(w->wv); free(w->wo); free(w->w1); free(w->w2); free(w->w3);
  memset(w, 0, sizeof(*w));
}

__global__ void __launch_bounds__(256) k_dequant(float* out, const int8_t* q, const float* s, size_t n, int gs) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    out[i] = (float)q[i] * s[i / gs];  // runq.c:141: x[i] = q[i] * s[i / GS]
}

extern "C" int thallama_q8_dequant_embedding(const Q8TransformerWeights* w, const Config* p, hipStream_t stream) {
  if (!w || !p || !w->token_embedding_table) return (int)hipErrorInvalidValue;
  const size_t n = (size_t)(p->vocab_size < 0 ? -p->vocab_size : p->vocab_size) * p->dim;
  tl::ApiLock lock(tl::api_mu());  // (the legacy stream when stream is null: api_lock.hpp)
  hipLaunchKernelGGL(k_dequant, dim3(4096), dim3(256), 0, stream, w->token_embedding_table, w->q_tokens[0].q,
                     w->q_tokens[0].s, n, w->group_size);
  return (int)hipGetLastError();
}

// export.py:46-70 — one thread per group: scale = max|w|/127, q = rint(w/scale) (torch.round: half to even)
__global__ void __launch_bounds__(256) k_q8_weights(int8_t* q, float* s, const float* w, size_t ng, int gs) {
  for (size_t g = (size_t)blockIdx.x * 256 + threadIdx.x; g < ng; g += (size_t)gridDim.x * 256) {
    const float* wg = w + g * gs;
    float wmax = 0.f;
    for (int i = 0; i < gs; ++i) wmax = fmaxf(wmax, fabsf(wg[i]));
    const float scale = __fdiv_rn(wmax, 127.0f);
    s[g] = scale;
    for (int i = 0; i < gs; ++i) q[g * gs + i] = (int8_t)rintf(__fdiv_rn(wg[i], scale));
  }
}

extern "C" int thallama_q8_quantize_model(void* payload, const TransformerWeights* w, const Config* p, int shared,
                                          int gs, hipStream_t stream) {
  if (!payload || !w || !p || gs <= 0) return (int)hipErrorInvalidValue;
  const size_t L = p->n_layers, dim = p->dim, kvd = (size_t)p->dim * p->n_kv_heads / p->n_heads;
  const size_t hid = p->hidden_dim, V = p->vocab_size < 0 ? -p->vocab_size : p->vocab_size;
  unsigned char* ptr = (unsigned char*)payload;
  tl::ApiLock lock(tl::api_mu());  // (the legacy stream when stream is null: api_lock.hpp)
  hipError_t e;
  if ((e = hipMemcpyAsync(ptr, w->rms_att_weight, 4 * L * dim, hipMemcpyDeviceToDevice, stream))) return (int)e;
  ptr += 4 * L * dim;
  if ((e = hipMemcpyAsync(ptr, w->rms_ffn_weight, 4 * L * dim, hipMemcpyDeviceToDevice, stream))) return (int)e;
  ptr += 4 * L * dim;
  if ((e = hipMemcpyAsync(ptr, w->rms_final_weight, 4 * dim, hipMemcpyDeviceToDevice, stream))) return (int)e;
  ptr += 4 * dim;
  struct { const float* src; size_t each; size_t n; } list[9] = {
      {w->token_embedding_table, V * dim, 1}, {w->wq, dim * dim, L}, {w->wk, dim * kvd, L}, {w->wv, dim * kvd, L},
      {w->wo, dim * dim, L}, {w->w1, dim * hid, L}, {w->w2, dim * hid, L}, {w->w3, dim * hid, L},
      {w->wcls, V * dim, shared ? 0u : 1u}};
  for (auto& t : list)
    for (size_t i = 0; i < t.n; ++i) {
      const size_t ng = t.each / gs;
      hipLaunchKernelGGL(k_q8_weights, dim3(4096), dim3(256), 0, stream, (int8_t*)ptr, (float*)(ptr + t.each),
                         t.src + i * t.each, ng, gs);
      if ((e = hipGetLastError())) return (int)e;
      ptr += t.each + 4 * ng;
    }
  return 0;
}

// ---------------------------------------------------------------- v2 checkpoint (host)
// runq.c read_checkpoint (:219-251): magic 0x616b3432 "ak42", version 2, Config, one flag
// byte (shared classifier), int group size, payload at byte 256.  Errors are returned, not
// exit()ed, so a library caller can recover.
extern "C" int thallama_q8_read_checkpoint(const char* path, Q8Checkpoint* ck) {
  if (!path || !ck) return -1;
  memset(ck, 0, sizeof(*ck));
  ck->fd = -1;
  FILE* f = fopen(path, "rb");
  if (!f) return -1;
  uint32_t magic = 0;
  int version = 0;
  uint8_t shared = 0;
  int gs = 0;
  const bool ok = fread(&magic, 4, 1, f) == 1 && fread(&version, 4, 1, f) == 1 &&
                  fread(&ck->config, sizeof(Config), 1, f) == 1 && fread(&shared, 1, 1, f) == 1 &&
                  fread(&gs, 4, 1, f) == 1;
  fseek(f, 0, SEEK_END);
  const long size = ftell(f);
  fclose(f);
  if (!ok) return -1;
  if (magic != 0x616b3432u) return -2;
  if (version != 2) return -3;
  ck->shared_classifier = shared;
  ck->group_size = gs;
  if (size < 256 || gs <= 0 ||
      (size_t)(size - 256) < thallama_q8_payload_bytes(&ck->config, shared, gs))
    return -4;
  ck->fd = open(path, O_RDONLY);
  if (ck->fd < 0) return -1;
  void* m = mmap(nullptr, (size_t)size, PROT_READ, MAP_PRIVATE, ck->fd, 0);
  if (m == MAP_FAILED) {
    close(ck->fd);
    ck->fd = -1;
    return -1;
  }
  ck->data = m;
  ck->file_size = (size_t)size;
  ck->payload = (const char*)m + 256;
  ck->payload_bytes = (size_t)size - 256;
  return 0;
}

extern "C" void thallama_q8_close_checkpoint(Q8Checkpoint* ck) {
  if (!ck) return;
  if (ck->data) munmap(ck->data, ck->file_size);
  if (ck->fd >= 0) close(ck->fd);
  ck->data = nullptr;
  ck->fd = -1;
}
