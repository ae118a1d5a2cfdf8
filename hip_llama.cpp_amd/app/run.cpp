// run.cpp — the reference's `run` CLI (src/llama.cpp:1486-1639) on the MI355X library.
//
//   run <model.bin> [-t temp] [-p topp] [-s seed] [-n steps] [-i prompt] [-z tokenizer]
//                   [-m generate|chat|test] [-y system] [-f input] [-o output] [-b batch]
//
// Same flags, defaults, validation and output files.  What differs is underneath:
//  * the model — a v0 fp32 model.bin, or a runq v2 "ak42" int8 file (the int8 decoder) — is
//    read once (mmap, src/utils.cpp:150-170 / runq.c:219-251 semantics), uploaded to GPU 0 with
//    ONE copy and replicated to every other GPU with an RCCL broadcast over xGMI (the
//    reference uploads the full model from host memory once per GPU thread);
//  * every decode step is the fused decoder of libthallama.so (the persistent one-launch step
//    at batch 1), not 1300+ small launches;
//  * `generate` runs on the GPU (the reference's generate() uses the CPU forward);
//  * the host side — tokenizer, sampler, request files and the test-mode scheduler — is
//    libthallama_host.so (include/thallama_host.h), byte-for-byte the reference's.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <ctype.h>
#include <sched.h>

#include <string>
#include <vector>

#include "../../include/models.hpp"
#include "../../include/thallama.h"
#include "../../include/thallama_host.h"
#include "../../include/thaQ8.hpp"

#define HIP_OK(cmd)                                                                              \
  do {                                                                                           \
    hipError_t e_ = (cmd);                                                                       \
    if (e_ != hipSuccess) {                                                                      \
      fprintf(stderr, "HIP error %s at %s:%d: %s\n", hipGetErrorString(e_), __FILE__, __LINE__, #cmd); \
      exit(EXIT_FAILURE);                                                                        \
    }                                                                                            \
  } while (0)
static long time_in_ms() {
  struct timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return ts.tv_sec * 1000 + ts.tv_nsec / 1000000;
}

static void error_usage() {
  fprintf(stderr, "Usage:   run <checkpoint> [options]\n");
  fprintf(stderr, "Example: run model.bin -n 256 -i \"Once upon a time\"\n");
  fprintf(stderr, "Example: run model.bin -m test -f <input_filename> -o <output_filename>\n");
  fprintf(stderr, "Options:\n");
  fprintf(stderr, "  -t <float>  temperature in [0,inf], default 1.0 (ignore the arg for test mode)\n");
  fprintf(stderr, "  -p <float>  p value in top-p (nucleus) sampling in [0,1] default 0.9 (ignore the arg for test mode)\n");
  fprintf(stderr, "  -s <int>    random seed, default time(NULL) (ignore the arg for test mode)\n");
  fprintf(stderr, "  -n <int>    number of steps to run for, default 256. 0 = max_seq_len (for test mode steps = max_seq_len)\n");
  fprintf(stderr, "  -i <string> input prompt (ignore the arg for test mode)\n");
  fprintf(stderr, "  -z <string> optional path to custom tokenizer\n");
  fprintf(stderr, "  -m <string> mode: generate|chat|test, default: generate\n");
  fprintf(stderr, "  -y <string> (optional) system prompt in chat mode\n");
  fprintf(stderr, "  -f <string> (only for test mode) input filename\n");
  fprintf(stderr, "  -o <string> (only for test mode) output filename\n");
  fprintf(stderr, "  -b <string> batch size\n");
  fprintf(stderr, "  -g <int>    (test mode, not in the reference) 1 = greedy decoding instead of T=1.0/top-p 0.9\n");
  exit(EXIT_FAILURE);
}

// The model file: a llama2.c v0 fp32 checkpoint (src/utils.cpp:150-170) or a runq v2 "ak42"
// int8 checkpoint (runq.c:219-251), told apart by the v2 magic.  Not in the reference: a
// synthetic model, "synth:dim,hidden,layers,heads,kv_heads,vocab,seq_len:seed[:q8:gs]" (vocab < 0 =
// unshared classifier, as in the v0 header) — the deterministic generator of include/
// thallama_synth.h run on GPU 0 (int8: quantised there with export.py semantics) instead of a
// file read, so a 27 GB llama2-7B needs no model file (bench.py's CLI workload).
struct ModelFile {
  bool q8 = false;
  bool synth = false;
  unsigned long long seed = 0;
  int shared = 0, gs = 0;
  Transformer t{};     // v0: mmapped fp32 model (build_transformer)
  Q8Checkpoint ck{};   // v2: mmapped int8 payload
  Config cfg{};
  const void* payload = nullptr;  // host image of the device arena (nullptr: synthesised on GPU 0)
  size_t bytes = 0;
};

static void print_config(const Config& c) {
  printf("dim: %d\nhidden_dim: %d\nn_layers: %d\nn_heads: %d\nn_kv_heads: %d\nvocab_size: %d\nseq_len: %d\n", c.dim,
         c.hidden_dim, c.n_layers, c.n_heads, c.n_kv_heads, c.vocab_size, c.seq_len);
}

static bool open_synth(ModelFile& m, const char* spec) {
  int v[7];
  unsigned long long seed = 0;
  char q8tag[8] = {0};
  int gs = 64;
  const int n = sscanf(spec, "synth:%d,%d,%d,%d,%d,%d,%d:%llu:%2s:%d", &v[0], &v[1], &v[2], &v[3], &v[4], &v[5], &v[6],
                       &seed, q8tag, &gs);
  if (n < 8 || v[0] <= 0 || v[2] <= 0 || v[3] <= 0 || v[4] <= 0 || v[5] == 0 || v[6] <= 0) return false;
  m.synth = true;
  m.seed = seed;
  m.shared = v[5] > 0;
  m.cfg = Config{v[0], v[1], v[2], v[3], v[4], v[5] < 0 ? -v[5] : v[5], v[6]};
  m.t.config = m.cfg;
  if (n >= 9 && strcmp(q8tag, "q8") == 0) {
    m.q8 = true;
    m.gs = gs;
    m.bytes = thallama_q8_payload_bytes(&m.cfg, m.shared, gs);
  } else {
    m.bytes = thallama_v0_payload_floats(&m.cfg, m.shared) * sizeof(float);
  }
  printf("---------Model Information----------\n");
  printf("synthetic %s model, seed %llu%s\n", m.q8 ? "int8" : "fp32", seed, m.shared ? ", shared classifier" : "");
  print_config(m.cfg);
  printf("------------------------------------\n");
  return true;
}

static void open_model(ModelFile& m, char* path) {
  if (strncmp(path, "synth:", 6) == 0) {
    if (!open_synth(m, path)) {
      fprintf(stderr, "bad synthetic model spec %s\n", path);
      exit(EXIT_FAILURE);
    }
    return;
  }
  FILE* f = fopen(path, "rb");
  if (!f) {
    fprintf(stderr, "Couldn't open file %s\n", path);
    exit(EXIT_FAILURE);
  }
  uint32_t magic = 0;
  const bool got = fread(&magic, 4, 1, f) == 1;
  fclose(f);
  if (got && magic == 0x616b3432u) {
    const int r = thallama_q8_read_checkpoint(path, &m.ck);
    if (r != 0) {
      fprintf(stderr, "cannot read int8 checkpoint %s (%d)\n", path, r);
      exit(EXIT_FAILURE);
    }
    m.q8 = true;
    m.cfg = m.ck.config;
    m.shared = m.ck.shared_classifier;
    m.gs = m.ck.group_size;
    m.payload = m.ck.payload;
    m.bytes = thallama_q8_payload_bytes(&m.cfg, m.shared, m.gs);
    m.t.config = m.cfg;
    printf("---------Model Information----------\n");
    printf("int8 (runq v2) group_size: %d\n", m.gs);
    print_config(m.cfg);
    printf("------------------------------------\n");
  } else {
    build_transformer(&m.t, path);
    m.cfg = m.t.config;
    m.shared = m.t.weights.wcls == m.t.weights.token_embedding_table;
    m.payload = m.t.weights.token_embedding_table;
    m.bytes = thallama_v0_payload_floats(&m.cfg, m.shared) * sizeof(float);
  }
}

static void close_model(ModelFile& m) {
  if (m.synth) return;
  if (m.q8) thallama_q8_close_checkpoint(&m.ck);
  else free_transformer(&m.t);
}

// A synthetic model's weight image, made on the current device in `arena` (m.bytes).
static void synth_on_device(const ModelFile& m, void* arena) {
  Config hdr = m.cfg;  // (positive vocab; the classifier sharing is the flag, as in bench.py)
  if (!m.q8) {
    if (thallama_synth_arena((float*)arena, &hdr, m.shared, m.seed, nullptr) != 0) {
      fprintf(stderr, "synthetic weights: %s\n", thallama_last_error());
      exit(EXIT_FAILURE);
    }
  } else {
    const size_t nf = thallama_v0_payload_floats(&hdr, m.shared);
    float* fp = nullptr;
    HIP_OK(hipMalloc(&fp, nf * sizeof(float)));
    TransformerWeights w{};
    if (thallama_synth_arena(fp, &hdr, m.shared, m.seed, nullptr) != 0) {
      fprintf(stderr, "synthetic weights: %s\n", thallama_last_error());
      exit(EXIT_FAILURE);
    }
    thallama_map_weights(&w, &hdr, fp, m.shared);
    if (thallama_q8_quantize_model(arena, &w, &m.cfg, m.shared, m.gs, nullptr) != 0) {
      fprintf(stderr, "int8 quantisation: %s\n", thallama_last_error());
      exit(EXIT_FAILURE);
    }
    HIP_OK(hipDeviceSynchronize());
    HIP_OK(hipFree(fp));
  }
  HIP_OK(hipDeviceSynchronize());
}

// One GPU's replica: the weight arena, run state for `batch` sequences, the decoder, and the host
// core its worker thread is pinned to.
struct Replica {
  int dev = 0;
  int cpu = -1;
  void* arena = nullptr;
  TransformerWeights w{};
  Q8TransformerWeights w8{};
  float* emb = nullptr;  // int8: dequantised embedding
  RunState* s = nullptr;
  thallama_decoder* dec = nullptr;
  float* logits_h = nullptr;  // pinned [batch][V]: the sampling steps' logits (src/llama.cpp:935)
};

static double now_s() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

// How the weight image reached replicas 1..n-1 (printed, and parsed by bench.py).
enum class RepPath { none, rccl, peer, upload };
static const char* rep_name(RepPath p) {
  return p == RepPath::rccl ? "rccl" : p == RepPath::peer ? "peer" : p == RepPath::upload ? "upload" : "none";
}

// RCCL broadcast of replica 0's arena into replicas 1..k-1 (device of replica i = reps[i].dev), in
// 1 GiB pieces, one communicator per replica.  Every call is checked and the transfer is polled
// against a deadline, so a failed or stalled RCCL returns an error (communicators aborted) instead
// of ending the process: the caller then replicates another way.
static std::string rccl_broadcast(std::vector<Replica>& reps, int k, size_t bytes) {
  std::vector<ncclComm_t> comms((size_t)k, nullptr);
  std::vector<int> devs((size_t)k);
  for (int d = 0; d < k; ++d) devs[d] = reps[d].dev;
  ncclResult_t nr = ncclCommInitAll(comms.data(), k, devs.data());
  if (nr != ncclSuccess) return std::string("ncclCommInitAll: ") + ncclGetErrorString(nr);
  std::string err;
  std::vector<hipStream_t> st((size_t)k, nullptr);
  for (int d = 0; d < k && err.empty(); ++d) {
    if (hipSetDevice(reps[d].dev) != hipSuccess || hipStreamCreateWithFlags(&st[d], hipStreamNonBlocking) != hipSuccess)
      err = "stream creation on device " + std::to_string(reps[d].dev);
  }
  const size_t piece = (size_t)1 << 30;
  for (size_t off = 0; off < bytes && err.empty(); off += piece) {
    const size_t cnt = bytes - off < piece ? bytes - off : piece;
    nr = ncclGroupStart();
    for (int d = 0; d < k && nr == ncclSuccess; ++d)
      nr = ncclBroadcast((char*)reps[0].arena + off, (char*)reps[d].arena + off, cnt, ncclChar, 0, comms[d], st[d]);
    const ncclResult_t ne = ncclGroupEnd();
    if (nr != ncclSuccess || ne != ncclSuccess)
      err = std::string("ncclBroadcast: ") + ncclGetErrorString(nr != ncclSuccess ? nr : ne);
  }
  // poll to completion: ~0.1 s per GiB over xGMI; allow 60 s + 1 s per GiB before giving up
  const double deadline = now_s() + 60.0 + (double)bytes / (1 << 30);
  for (int d = 0; d < k && err.empty(); ++d) {
    (void)hipSetDevice(reps[d].dev);
    hipError_t q;
    while ((q = hipStreamQuery(st[d])) == hipErrorNotReady) {
      ncclResult_t async = ncclSuccess;
      ncclCommGetAsyncError(comms[d], &async);
      if (async != ncclSuccess) {
        err = std::string("RCCL async error: ") + ncclGetErrorString(async);
        break;
      }
      if (now_s() > deadline) {
        err = "RCCL broadcast did not complete before the deadline";
        break;
      }
      struct timespec ts = {0, 1000000};
      nanosleep(&ts, nullptr);
    }
    if (err.empty() && q != hipSuccess) err = std::string("broadcast stream: ") + hipGetErrorString(q);
  }
  for (int d = 0; d < k; ++d) {
    if (comms[d]) {
      if (err.empty()) ncclCommDestroy(comms[d]);
      else ncclCommAbort(comms[d]);
    }
  }
  for (int d = 0; d < k; ++d) {
    if (!st[d]) continue;
    (void)hipSetDevice(reps[d].dev);
    if (err.empty()) (void)hipStreamSynchronize(st[d]);
    (void)hipStreamDestroy(st[d]);
  }
  (void)hipSetDevice(0);
  return err;
}

// Device-to-device copies into replicas [from, n), in order.  Replica r lives on device r % n_dev, so
// replica r.dev is the first one on r's GPU: a replica past the first on its GPU copies locally from
// it (filled already: index r.dev < r), the first replica of every other GPU copies from replica 0
// over xGMI (hipMemcpyPeerAsync).
static std::string peer_copies(std::vector<Replica>& reps, int from, size_t bytes) {
  for (size_t d = (size_t)from; d < reps.size(); ++d) {
    Replica& r = reps[d];
    const Replica& src = (size_t)r.dev < d ? reps[(size_t)r.dev] : reps[0];
    hipStream_t st = nullptr;
    if (hipSetDevice(r.dev) != hipSuccess || hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess)
      return "stream creation on device " + std::to_string(r.dev);
    hipError_t e = hipMemcpyPeerAsync(r.arena, r.dev, src.arena, src.dev, bytes, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    (void)hipStreamDestroy(st);
    if (e != hipSuccess) return std::string("hipMemcpyPeer to device ") + std::to_string(r.dev) + ": " + hipGetErrorString(e);
  }
  (void)hipSetDevice(0);
  return "";
}

// The reference's way (src/models.cpp:86-125 once per GPU thread): each replica from the host image,
// or, for a synthetic model, the generator run again on the replica's device.
static void upload_each(ModelFile& m, std::vector<Replica>& reps, int from) {
  for (size_t d = (size_t)from; d < reps.size(); ++d) {
    HIP_OK(hipSetDevice(reps[d].dev));
    if (m.payload) HIP_OK(hipMemcpy(reps[d].arena, m.payload, m.bytes, hipMemcpyHostToDevice));
    else synth_on_device(m, reps[d].arena);
  }
  HIP_OK(hipSetDevice(0));
}

// The host cores next to a device: its PCI function's local_cpulist, intersected with this process's
// affinity mask (empty when sysfs does not say).
static std::vector<int> local_cpus(int dev, const cpu_set_t& allowed) {
  std::vector<int> out;
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof bus, dev) != hipSuccess) return out;
  for (char* c = bus; *c; ++c) *c = (char)tolower(*c);
  const std::string path = std::string("/sys/bus/pci/devices/") + bus + "/local_cpulist";
  FILE* f = fopen(path.c_str(), "r");
  if (!f) return out;
  char line[4096] = {0};
  const bool got = fgets(line, sizeof line, f) != nullptr;
  fclose(f);
  if (!got) return out;
  for (char* tok = strtok(line, ",\n"); tok; tok = strtok(nullptr, ",\n")) {
    int a = 0, b = 0;
    const int n = sscanf(tok, "%d-%d", &a, &b);
    if (n < 1) continue;
    if (n == 1) b = a;
    for (int c = a; c <= b && c < CPU_SETSIZE; ++c)
      if (CPU_ISSET(c, &allowed)) out.push_back(c);
  }
  return out;
}

// Worker w's core (the reference pins thread gid to core gid, src/llama.cpp:922-925): the next unused
// core local to its GPU, else the next unused core this process may run on.
static void assign_cpus(std::vector<Replica>& reps) {
  cpu_set_t allowed;
  CPU_ZERO(&allowed);
  if (sched_getaffinity(0, sizeof allowed, &allowed) != 0) return;
  std::vector<int> all;
  for (int c = 0; c < CPU_SETSIZE; ++c)
    if (CPU_ISSET(c, &allowed)) all.push_back(c);
  if (all.empty()) return;
  std::vector<char> used((size_t)CPU_SETSIZE, 0);
  for (auto& r : reps) {
    for (int c : local_cpus(r.dev, allowed))
      if (!used[c]) {
        r.cpu = c;
        break;
      }
    if (r.cpu < 0)
      for (int c : all)
        if (!used[c]) {
          r.cpu = c;
          break;
        }
    if (r.cpu < 0) r.cpu = all[(size_t)(&r - reps.data()) % all.size()];
    used[r.cpu] = 1;
  }
}

// Weights on every replica: one H2D copy (or on-device synthesis) into replica 0, then replicas
// 1..n-1 by, in order of preference:
//   rccl   — ncclBroadcast over xGMI from GPU 0 (one replica per GPU);
//   peer   — hipMemcpyPeer from GPU 0 (also how replicas that share a GPU are filled);
//   upload — every replica from the host image / the generator, as the reference does.
// A failing path falls through to the next, reported, instead of ending the run.
// THALLAMA_REPLICATE=rccl|peer|upload picks the first path tried (tests: forced RCCL over replicas
// that share one GPU fails in ncclCommInitAll and exercises the fall-through).  n_rep > n_dev
// (THALLAMA_REPLICAS, a rehearsal of the multi-GPU worker split on fewer GPUs): replica r lives on
// device r % n_dev.
static std::vector<Replica> replicate(ModelFile& m, int n_dev, int n_rep, int batch, RepPath* used, double* rep_s) {
  std::vector<Replica> reps((size_t)n_rep);
  for (int d = 0; d < n_rep; ++d) {
    reps[d].dev = d % n_dev;
    HIP_OK(hipSetDevice(reps[d].dev));
    HIP_OK(hipMalloc(&reps[d].arena, m.bytes));
  }
  HIP_OK(hipSetDevice(0));
  if (m.payload) HIP_OK(hipMemcpy(reps[0].arena, m.payload, m.bytes, hipMemcpyHostToDevice));
  else synth_on_device(m, reps[0].arena);
  const char* want = getenv("THALLAMA_REPLICATE");
  RepPath path = n_rep == 1 ? RepPath::none : n_dev > 1 ? RepPath::rccl : RepPath::peer;
  if (n_rep > 1 && want) {
    if (!strcmp(want, "rccl")) path = RepPath::rccl;
    else if (!strcmp(want, "peer")) path = RepPath::peer;
    else if (!strcmp(want, "upload")) path = RepPath::upload;
  }
  const double t0 = now_s();
  if (path == RepPath::rccl) {
    // one communicator per GPU: replicas 0..n_dev-1 (all replicas when the choice was forced)
    const int k = want && !strcmp(want, "rccl") ? n_rep : (n_dev < n_rep ? n_dev : n_rep);
    const std::string err = rccl_broadcast(reps, k, m.bytes);
    if (!err.empty()) {
      printf("replication: RCCL failed (%s); falling back to peer copies\n", err.c_str());
      path = RepPath::peer;
    } else if (k < n_rep) {
      const std::string e2 = peer_copies(reps, k, m.bytes);  // replicas sharing a GPU
      if (!e2.empty()) {
        printf("replication: %s; falling back to uploads\n", e2.c_str());
        upload_each(m, reps, k);
      }
    }
  }
  if (path == RepPath::peer) {
    const std::string err = peer_copies(reps, 1, m.bytes);
    if (!err.empty()) {
      printf("replication: %s; falling back to uploads\n", err.c_str());
      path = RepPath::upload;
    }
  }
  if (path == RepPath::upload) upload_each(m, reps, 1);
  *used = path;
  *rep_s = now_s() - t0;
  assign_cpus(reps);
  for (int d = 0; d < n_rep; ++d) {
    Replica& r = reps[d];
    HIP_OK(hipSetDevice(r.dev));
    alloc_state_to_device_batch(&m.t, r.s, batch);
    int rc;
    if (m.q8) {
      HIP_OK(hipMalloc(&r.emb, sizeof(float) * (size_t)m.cfg.vocab_size * m.cfg.dim));
      if (thallama_q8_map(&r.w8, &m.cfg, r.arena, m.shared, m.gs, r.emb) != 0 ||
          thallama_q8_dequant_embedding(&r.w8, &m.cfg, nullptr) != 0) {
        fprintf(stderr, "int8 weights on device %d: %s\n", d, thallama_last_error());
        exit(EXIT_FAILURE);
      }
      HIP_OK(hipDeviceSynchronize());
      rc = thallama_decoder_create_q8(&r.dec, &m.cfg, &r.w8, r.s, batch, nullptr);
    } else {
      thallama_map_weights(&r.w, &m.cfg, (float*)r.arena, m.shared);
      rc = thallama_decoder_create(&r.dec, &m.cfg, &r.w, r.s, batch, nullptr);
    }
    if (rc != 0) {
      fprintf(stderr, "decoder on device %d: %s\n", d, thallama_last_error());
      exit(EXIT_FAILURE);
    }
    thallama_decoder_set(r.dec, THALLAMA_OPT_USE_GRAPH, 1);  // each step replayed as one captured graph
    HIP_OK(hipHostMalloc(&r.logits_h, sizeof(float) * (size_t)batch * m.cfg.vocab_size, hipHostMallocDefault));
  }
  return reps;
}

static void release(std::vector<Replica>& reps) {
  for (auto& r : reps) {
    HIP_OK(hipSetDevice(r.dev));
    thallama_decoder_destroy(r.dec);
    free_state_device(r.s);
    if (r.logits_h) HIP_OK(hipHostFree(r.logits_h));
    if (r.emb) {
      thallama_q8_unmap(&r.w8);
      HIP_OK(hipFree(r.emb));
    }
    HIP_OK(hipFree(r.arena));
  }
}

// The scheduler's worker thread for replica r: pinned to r's core on its first callback.
static int enter(Replica& r) {
  thread_local int pinned = -1;
  if (pinned != r.cpu && r.cpu >= 0) {
    cpu_set_t one;
    CPU_ZERO(&one);
    CPU_SET(r.cpu, &one);
    sched_setaffinity(0, sizeof one, &one);  // 0 = the calling thread
    pinned = r.cpu;
  }
  return hipSetDevice(r.dev) == hipSuccess ? 0 : -3;
}

// test mode step callback: worker w drives replica w
static int replica_step(void* ctx, int worker, int batch, const int* token, const int* pos, float* logits) {
  Replica& r = (*(std::vector<Replica>*)ctx)[worker];
  if (enter(r)) return -3;
  (void)batch;
  const int st = thallama_decoder_forward(r.dec, token, pos, logits);
  if (st) fprintf(stderr, "device %d step: %s\n", r.dev, thallama_last_error());
  return st;
}

// greedy test mode (-g 1): the argmax stays on the device and only the batch's ids come back
static int replica_argmax(void* ctx, int worker, int batch, const int* token, const int* pos, int* next) {
  Replica& r = (*(std::vector<Replica>*)ctx)[worker];
  if (enter(r)) return -3;
  (void)batch;
  const int st = thallama_decoder_step_argmax(r.dec, token, pos, next);
  if (st) fprintf(stderr, "device %d step: %s\n", r.dev, thallama_last_error());
  return st;
}

// batched prompt processing (thallama_decoder_prefill); > 0 = not supported here (int8, or
// THALLAMA_NO_PREFILL=1), so the scheduler steps through the prompt like the reference
static int prefill_on(Replica& r, int slot, const int* tokens, int n, int pos0) {
  static const bool off = getenv("THALLAMA_NO_PREFILL") && atoi(getenv("THALLAMA_NO_PREFILL")) != 0;
  if (off) return 1;
  if (enter(r)) return -3;
  const int st = thallama_decoder_prefill(r.dec, slot, tokens, n, pos0);
  if (st == (int)hipErrorNotSupported) return 1;
  if (st) fprintf(stderr, "device %d prefill: %s\n", r.dev, thallama_last_error());
  return st ? -st : 0;
}

static int replica_prefill(void* ctx, int worker, int slot, const int* tokens, int n, int pos0) {
  return prefill_on((*(std::vector<Replica>*)ctx)[worker], slot, tokens, n, pos0);
}

// generate mode (src/llama.cpp:522-579), on GPU 0
static void generate(const Config& cfg, Replica& r, thallama_tokenizer* tok, thallama_sampler* smp, const char* prompt,
                     int steps) {
  if (!prompt) prompt = "";
  std::vector<int> ids(strlen(prompt) + 3);
  int n_ids = 0;
  thallama_tokenizer_encode(tok, prompt, 1, 0, ids.data(), &n_ids);
  if (n_ids < 1) {
    fprintf(stderr, "something is wrong, expected at least 1 prompt token\n");
    exit(EXIT_FAILURE);
  }
  std::vector<float> logits((size_t)cfg.vocab_size);
  long start = 0;
  int token = ids[0], pos = 0;
  // prompt tokens 0..m-1 in one prefill instead of m forced decode steps (same pieces)
  int m = n_ids - 1 < steps ? n_ids - 1 : steps;
  for (int i = 1; i <= m && i < n_ids; ++i)
    if (ids[i] == 1) m = 0;  // the prompt would end the loop: step through it instead
  if (m >= 1 && prefill_on(r, 0, ids.data(), m, 0) == 0) {
    for (int i = 0; i < m; ++i) {
      const char* piece = thallama_tokenizer_decode(tok, ids[i], ids[i + 1]);
      if (thallama_piece_is_safe(piece)) printf("%s", piece);
    }
    fflush(stdout);
    token = ids[m];
    pos = m;
    start = time_in_ms();
  }
  while (pos < steps) {
    if (thallama_decoder_forward(r.dec, &token, &pos, logits.data()) != 0) {
      fprintf(stderr, "forward: %s\n", thallama_last_error());
      exit(EXIT_FAILURE);
    }
    const int next = pos < n_ids - 1 ? ids[pos + 1] : thallama_sample(smp, logits.data());
    pos++;
    if (next == 1) break;  // BOS delimits sequences
    const char* piece = thallama_tokenizer_decode(tok, token, next);
    if (thallama_piece_is_safe(piece)) printf("%s", piece);
    fflush(stdout);
    token = next;
    if (start == 0) start = time_in_ms();
  }
  printf("\n");
  if (pos > 1) {
    const long end = time_in_ms();
    fprintf(stderr, "achieved tok/s: %f\n", (pos - 1) / (double)(end - start) * 1000);
  }
}

int main(int argc, char* argv[]) {
  const long total_start = time_in_ms();
  char* checkpoint_path = nullptr;
  const char* tokenizer_path = "./assets/tokenizer.bin";
  float temperature = 1.0f, topp = 0.9f;
  int steps = 256, batch = 1, greedy_test = 0;
  const char* prompt = nullptr;
  unsigned long long rng_seed = 0;
  const char* mode = "generate";
  const char* input_filename = nullptr;
  const char* output_filename = nullptr;

  if (argc >= 2) checkpoint_path = argv[1];
  else error_usage();
  for (int i = 2; i < argc; i += 2) {
    if (i + 1 >= argc || argv[i][0] != '-' || strlen(argv[i]) != 2) error_usage();
    const char* v = argv[i + 1];
    switch (argv[i][1]) {
      case 't': temperature = (float)atof(v); break;
      case 'p': topp = (float)atof(v); break;
      case 's': rng_seed = (unsigned long long)atoi(v); break;
      case 'n': steps = atoi(v); break;
      case 'i': prompt = v; break;
      case 'z': tokenizer_path = v; break;
      case 'm': mode = v; break;
      case 'y': break;  // chat system prompt (chat mode is disabled in the reference)
      case 'f': input_filename = v; break;
      case 'o': output_filename = v; break;
      case 'b': batch = atoi(v); break;
      case 'g': greedy_test = atoi(v); break;
      default: error_usage();
    }
  }
  if (rng_seed <= 0) rng_seed = (unsigned int)time(nullptr);
  if (temperature < 0.0) temperature = 0.0;
  if (topp < 0.0 || 1.0 < topp) topp = 0.9;
  if (steps < 0) steps = 0;
  if (batch < 1) batch = 1;

  ModelFile model;
  open_model(model, checkpoint_path);
  if (steps == 0 || steps > model.cfg.seq_len) steps = model.cfg.seq_len;
  const int V = model.cfg.vocab_size;
  thallama_tokenizer* tok = thallama_tokenizer_load(tokenizer_path, V);
  if (!tok) {
    fprintf(stderr, "couldn't load %s\n", tokenizer_path);
    exit(EXIT_FAILURE);
  }
  thallama_sampler* smp = thallama_sampler_create(V, temperature, topp, rng_seed);

  if (strcmp(mode, "generate") == 0) {
    RepPath rp;
    double rs;
    std::vector<Replica> reps = replicate(model, 1, 1, 1, &rp, &rs);
    generate(model.cfg, reps[0], tok, smp, prompt, steps);
    release(reps);
  } else if (strcmp(mode, "chat") == 0) {
    // chat() is commented out in the reference's main (src/llama.cpp:1590)
  } else if (strcmp(mode, "test") == 0) {
    steps = model.cfg.seq_len;
    // THALLAMA_TEST_STEPS=T (not in the reference, which always decodes to seq_len in test mode):
    // each request to position T - 1 at most (bench.py's 256-position request workload)
    if (getenv("THALLAMA_TEST_STEPS") && atoi(getenv("THALLAMA_TEST_STEPS")) > 1 &&
        atoi(getenv("THALLAMA_TEST_STEPS")) < steps)
      steps = atoi(getenv("THALLAMA_TEST_STEPS"));
    if (!input_filename || !output_filename) error_usage();
    const int max_token_len = thallama_tokenizer_max_token_length(tok);
    printf("max_token_len: %d, max_seq_len: %d\n", max_token_len, steps);
    thallama_requests* req = thallama_requests_read(input_filename, max_token_len, steps);
    if (!req) {
      fprintf(stderr, "cannot open the file: %s\n", input_filename);
      exit(EXIT_FAILURE);
    }
    if (greedy_test) thallama_requests_set_sampling(req, 0.0f, 0.9f);
    printf("requests size = %lu B\n",
           (unsigned long)(((size_t)thallama_requests_count(req) * max_token_len * steps + 1) * 2));
    int n_dev = 0;
    HIP_OK(hipGetDeviceCount(&n_dev));
    // one worker (replica) per GPU like the reference; THALLAMA_REPLICAS=N runs N workers over
    // the GPUs there are (a rehearsal of an N-GPU run: the worker split, the per-replica decoders)
    const char* rep_env = getenv("THALLAMA_REPLICAS");
    const int n_rep = rep_env && atoi(rep_env) > 0 ? atoi(rep_env) : n_dev;
    // THALLAMA_PASSES=P (not in the reference; bench.py): serve the request file P times on the
    // same resident weights, one "pass i: ..." line each; the output file is the last pass's
    const char* pass_env = getenv("THALLAMA_PASSES");
    int passes = pass_env && atoi(pass_env) > 0 ? atoi(pass_env) : 1;
    // THALLAMA_PASS_BUDGET_S=S (bench.py): no pass starts once the passes so far took S seconds of
    // serving (the last pass run is then the one whose output file is written)
    const char* budget_env = getenv("THALLAMA_PASS_BUDGET_S");
    const double pass_budget = budget_env ? atof(budget_env) : 0.0;
    double served_s = 0.0;
    fprintf(stderr, "\n DATA PARALLELISM \n");
    fprintf(stderr, "\n Num Devices %d\n", n_rep);
    fprintf(stderr, "\n Batch Size %d\n", batch);
    const long load_start = time_in_ms();
    RepPath rp;
    double rep_s = 0.0;
    std::vector<Replica> reps = replicate(model, n_dev, n_rep, batch, &rp, &rep_s);
    const char* how = rp == RepPath::rccl ? "RCCL broadcast" : rp == RepPath::peer ? "peer copies"
                      : rp == RepPath::upload ? "uploads" : "no copies";
    fprintf(stdout, "replication: %s to %d replica(s) on %d GPU(s) in %f s\n", rep_name(rp), n_rep, n_dev, rep_s);
    for (int w = 0; w < n_rep; ++w)
      fprintf(stdout, "worker %d: device %d cpu %d\n", w, reps[w].dev, reps[w].cpu);
    fprintf(stdout, "\nLoad model time (1 %s + %s to %d GPUs): %f\n", model.synth ? "on-device synthesis" : "upload",
            how, n_dev, (double)(time_in_ms() - load_start) / 1000);

    for (int pass = 0; pass < passes; ++pass) {
      if (pass > 0) {  // a fresh copy of the requests (the scheduler fills in their outputs)
        thallama_requests_free(req);
        req = thallama_requests_read(input_filename, max_token_len, steps);
        if (!req) exit(EXIT_FAILURE);
        if (greedy_test) thallama_requests_set_sampling(req, 0.0f, 0.9f);
      }
      const long start = time_in_ms();
      long long num_gen_tokens = 0;
      std::vector<long long> w_tok((size_t)n_rep, 0);
      std::vector<double> w_sec((size_t)n_rep, 0.0);
      std::vector<int> w_req((size_t)n_rep, 0);
      std::vector<float*> w_lg((size_t)n_rep);
      for (int w = 0; w < n_rep; ++w) w_lg[w] = reps[w].logits_h;
      const int st = thallama_serve_requests_stats(req, tokenizer_path, V, n_rep, batch, replica_step,
                                                   getenv("THALLAMA_HOST_ARGMAX") ? nullptr : replica_argmax,
                                                   replica_prefill, &reps, &num_gen_tokens, w_tok.data(), w_sec.data(),
                                                   w_req.data(), w_lg.data());
      const long end = time_in_ms();
      if (st != 0) {
        fprintf(stderr, "test mode failed (%d)\n", st);
        exit(EXIT_FAILURE);
      }
      if (passes > 1)
        fprintf(stdout, "pass %d: tokens %lld seconds %f\n", pass, num_gen_tokens, (double)(end - start) / 1000);
      served_s += (double)(end - start) / 1000;
      if (pass_budget > 0.0 && served_s >= pass_budget && pass + 1 < passes) {
        fprintf(stdout, "pass budget: %d of %d passes in %f s (THALLAMA_PASS_BUDGET_S=%g)\n", pass + 1, passes,
                served_s, pass_budget);
        passes = pass + 1;
      }
      for (int w = 0; w < n_rep; ++w)  // per GPU (worker): its tokens, requests and busy time
        fprintf(stdout, "pass %d worker %d device %d: tokens %lld requests %d seconds %f\n", pass, w, reps[w].dev,
                w_tok[w], w_req[w], w_sec[w]);
      if (pass + 1 < passes) continue;
      fprintf(stdout, "Total achieved token: %lld\n", num_gen_tokens);
      fprintf(stdout, "elapsed time(s): %f, achieved throughput(tok/s): %f\n", (double)(end - start) / 1000,
              num_gen_tokens / (double)(end - start) * 1000);
    }
    if (thallama_requests_write(req, output_filename) != 0) {
      fprintf(stderr, "cannot write output file: %s\n", input_filename);
      exit(EXIT_FAILURE);
    }
    thallama_requests_free(req);
    release(reps);
  } else {
    fprintf(stderr, "unknown mode: %s\n", mode);
    error_usage();
  }
  thallama_sampler_free(smp);
  thallama_tokenizer_free(tok);
  close_model(model);
  fprintf(stdout, "total elapsed time(s): %lf\n", (double)(time_in_ms() - total_start) / 1000);
  return 0;
}
