// host.cpp — the reference CLI's host side (tokenizer, sampler, request files, test-mode
// scheduler), behind include/thallama_host.h.  Built CPU-only into lib/libthallama_host.so.
//
// Byte-level parity with src/llama.cpp is the contract (tests/test_host.py pins every function
// against the reference's own tokenizer/sampler code compiled from /root/reference/run.cc, whose
// copies of these functions are identical to src/llama.cpp's):
//   * the same float operations in the same order (compiled with -ffp-contract=off);
//   * libc's qsort with the same comparator for top-p, so ties among equal probabilities
//     come out in the same order as in the reference on the same libc;
//   * libc's sscanf with the reference's "<0x%02hhX>" format for raw-byte pieces.
// Differences are internal only: the vocabulary lookup is a hash map (the llama2 vocabulary
// has no duplicate pieces, so it returns what the reference's bsearch returns), and the BPE
// merge loop caches each adjacent pair's merge candidate instead of re-concatenating every
// pair on every iteration — the merge ORDER (first pair with the strictly highest score) is
// unchanged, so the output ids are identical.
#include <ctype.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <fstream>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/thallama_host.h"

// ------------------------------------------------------------------------------ tokenizer
struct thallama_tokenizer {
  int vocab_size = 0;
  unsigned max_token_length = 0;
  std::vector<std::string> pieces;
  std::vector<float> scores;
  std::unordered_map<std::string, int> ids;  // piece -> id
  char byte_piece[256][2];                   // raw-byte pieces "\xNN"
  int lookup(const std::string& s) const {
    auto it = ids.find(s);
    return it == ids.end() ? -1 : it->second;
  }
};

extern "C" thallama_tokenizer* thallama_tokenizer_load(const char* path, int vocab_size) {
  FILE* f = fopen(path, "rb");
  if (!f) return nullptr;
  auto* t = new thallama_tokenizer();
  t->vocab_size = vocab_size;
  for (int b = 0; b < 256; ++b) {
    t->byte_piece[b][0] = (char)b;
    t->byte_piece[b][1] = '\0';
  }
  bool ok = fread(&t->max_token_length, sizeof(int), 1, f) == 1;
  t->pieces.resize(vocab_size);
  t->scores.resize(vocab_size);
  for (int i = 0; ok && i < vocab_size; ++i) {
    int len = 0;
    ok = fread(&t->scores[i], sizeof(float), 1, f) == 1 && fread(&len, sizeof(int), 1, f) == 1 && len >= 0;
    if (!ok) break;
    std::string s((size_t)len, '\0');
    ok = len == 0 || fread(&s[0], (size_t)len, 1, f) == 1;
    // the reference keeps C strings: a piece ends at its first NUL
    t->pieces[i] = std::string(s.c_str());
  }
  fclose(f);
  if (!ok) {
    delete t;
    return nullptr;
  }
  for (int i = vocab_size - 1; i >= 0; --i) t->ids[t->pieces[i]] = i;  // lowest id wins on duplicates
  return t;
}

extern "C" void thallama_tokenizer_free(thallama_tokenizer* t) { delete t; }
extern "C" int thallama_tokenizer_max_token_length(const thallama_tokenizer* t) { return (int)t->max_token_length; }
extern "C" const char* thallama_tokenizer_piece(const thallama_tokenizer* t, int id) { return t->pieces[id].c_str(); }
extern "C" float thallama_tokenizer_score(const thallama_tokenizer* t, int id) { return t->scores[id]; }

extern "C" int thallama_tokenizer_encode(thallama_tokenizer* t, const char* text, int bos, int eos, int* tokens,
                                         int* n_tokens) {
  if (!text) return -1;
  std::vector<int> tok;
  if (bos) tok.push_back(1);
  if (text[0] != '\0') tok.push_back(t->lookup(" "));  // add_dummy_prefix
  // UTF-8: a codepoint is a non-continuation byte plus at most 3 continuation bytes; a
  // codepoint missing from the vocabulary falls back to its raw bytes (ids 3..258)
  std::string cp;
  for (const char* c = text; *c; ++c) {
    if ((*c & 0xC0) != 0x80) cp.clear();
    cp.push_back(*c);
    if ((c[1] & 0xC0) == 0x80 && cp.size() < 4) continue;
    const int id = t->lookup(cp);
    if (id != -1) {
      tok.push_back(id);
    } else {
      for (unsigned char b : cp) tok.push_back((int)b + 3);
    }
    cp.clear();
  }
  // BPE merges: repeatedly merge the FIRST adjacent pair whose merged piece has the highest
  // score (strictly greater than every earlier candidate, and than -1e10)
  const int n0 = (int)tok.size();
  std::vector<int> cand(n0 > 0 ? n0 : 1, -1);  // merged id of (tok[i], tok[i+1]) or -1
  auto pair_id = [&](int i) {
    if (tok[i] < 0 || tok[i + 1] < 0) return -1;  // (no " " piece: the reference would read out of bounds)
    return t->lookup(t->pieces[tok[i]] + t->pieces[tok[i + 1]]);
  };
  for (int i = 0; i + 1 < n0; ++i) cand[i] = pair_id(i);
  int n = n0;
  while (true) {
    float best = -1e10f;
    int at = -1;
    for (int i = 0; i + 1 < n; ++i)
      if (cand[i] != -1 && t->scores[cand[i]] > best) {
        best = t->scores[cand[i]];
        at = i;
      }
    if (at < 0) break;
    tok[at] = cand[at];
    tok.erase(tok.begin() + at + 1);
    cand.erase(cand.begin() + at + 1);
    --n;
    if (at + 1 < n) cand[at] = pair_id(at);
    else cand[at] = -1;
    if (at > 0) cand[at - 1] = pair_id(at - 1);
  }
  if (eos) tok.push_back(2);
  for (size_t i = 0; i < tok.size(); ++i) tokens[i] = tok[i];
  *n_tokens = (int)tok.size();
  return 0;
}

extern "C" const char* thallama_tokenizer_decode(const thallama_tokenizer* t, int prev_token, int token) {
  const char* piece = t->pieces[token].c_str();
  if (prev_token == 1 && piece[0] == ' ') ++piece;  // sentencepiece strips the space after BOS
  unsigned char byte_val;
  if (sscanf(piece, "<0x%02hhX>", &byte_val) == 1) piece = t->byte_piece[byte_val];
  return piece;
}

extern "C" int thallama_piece_is_safe(const char* piece) {
  if (!piece || piece[0] == '\0') return 0;
  if (piece[1] == '\0') {
    const unsigned char b = (unsigned char)piece[0];
    if (!(isprint(b) || isspace(b))) return 0;
  }
  return 1;
}

// ------------------------------------------------------------------------------ sampler
extern "C" void thallama_softmax(float* x, int n) {  // src/seq.cpp:18-36
  float mx = x[0];
  for (int i = 1; i < n; ++i)
    if (x[i] > mx) mx = x[i];
  float sum = 0.0f;
  for (int i = 0; i < n; ++i) {
    x[i] = expf(x[i] - mx);
    sum += x[i];
  }
  for (int i = 0; i < n; ++i) x[i] /= sum;
}

extern "C" int thallama_sample_argmax(const float* p, int n) {
  int best = 0;
  for (int i = 1; i < n; ++i)
    if (p[i] > p[best]) best = i;
  return best;
}

extern "C" int thallama_sample_mult(const float* p, int n, float coin) {
  float cdf = 0.0f;
  for (int i = 0; i < n; ++i) {
    cdf += p[i];
    if (coin < cdf) return i;
  }
  return n - 1;
}

namespace {
struct ProbIdx {
  float prob;
  int index;
};
int by_prob_desc(const void* a, const void* b) {
  const float pa = ((const ProbIdx*)a)->prob, pb = ((const ProbIdx*)b)->prob;
  return pa > pb ? -1 : (pa < pb ? 1 : 0);
}
int topp_with(const float* p, int n, float topp, float coin, ProbIdx* buf) {
  // candidates below (1-topp)/(n-1) can never be in the nucleus
  const float cutoff = (1.0f - topp) / (n - 1);
  int m = 0;
  for (int i = 0; i < n; ++i)
    if (p[i] >= cutoff) buf[m++] = ProbIdx{p[i], i};
  qsort(buf, m, sizeof(ProbIdx), by_prob_desc);
  float cum = 0.0f;
  int last = m - 1;
  for (int i = 0; i < m; ++i) {
    cum += buf[i].prob;
    if (cum > topp) {
      last = i;
      break;
    }
  }
  const float r = coin * cum;
  float cdf = 0.0f;
  for (int i = 0; i <= last; ++i) {
    cdf += buf[i].prob;
    if (r < cdf) return buf[i].index;
  }
  return buf[last].index;
}
}  // namespace

extern "C" int thallama_sample_topp(const float* p, int n, float topp, float coin) {
  std::vector<ProbIdx> buf((size_t)n);
  return topp_with(p, n, topp, coin, buf.data());
}

extern "C" unsigned int thallama_random_u32(unsigned long long* s) {  // xorshift*
  *s ^= *s >> 12;
  *s ^= *s << 25;
  *s ^= *s >> 27;
  return (unsigned int)((*s * 0x2545F4914F6CDD1Dull) >> 32);
}

extern "C" float thallama_random_f32(unsigned long long* s) { return (thallama_random_u32(s) >> 8) / 16777216.0f; }

struct thallama_sampler {
  int vocab_size;
  float temperature, topp;
  unsigned long long rng;
  std::vector<ProbIdx> buf;
};

extern "C" thallama_sampler* thallama_sampler_create(int vocab_size, float temperature, float topp,
                                                     unsigned long long seed) {
  auto* s = new thallama_sampler{vocab_size, temperature, topp, seed, {}};
  s->buf.resize((size_t)vocab_size);
  return s;
}
extern "C" void thallama_sampler_free(thallama_sampler* s) { delete s; }
extern "C" unsigned long long thallama_sampler_rng_state(const thallama_sampler* s) { return s->rng; }

extern "C" int thallama_sample(thallama_sampler* s, float* logits) {
  if (s->temperature == 0.0f) return thallama_sample_argmax(logits, s->vocab_size);
  for (int i = 0; i < s->vocab_size; ++i) logits[i] /= s->temperature;
  thallama_softmax(logits, s->vocab_size);
  const float coin = thallama_random_f32(&s->rng);
  if (s->topp <= 0 || s->topp >= 1) return thallama_sample_mult(logits, s->vocab_size, coin);
  return topp_with(logits, s->vocab_size, s->topp, coin, s->buf.data());
}

// ------------------------------------------------------------------------------ request files
struct thallama_requests {
  int max_token_len = 0, max_seq_len = 0;
  float temperature = 1.0f, topp = 0.9f;  // the reference's per-request sampler (src/llama.cpp:897-900)
  std::vector<std::string> prompts, outputs;
  size_t cap() const { return (size_t)max_token_len * (size_t)max_seq_len; }
};

extern "C" void thallama_requests_set_sampling(thallama_requests* r, float temperature, float topp) {
  if (!r) return;
  r->temperature = temperature;
  r->topp = topp;
}

extern "C" thallama_requests* thallama_requests_read(const char* path, int max_token_len, int max_seq_len) {
  std::ifstream in(path);
  if (!in.is_open()) return nullptr;
  auto* r = new thallama_requests();
  r->max_token_len = max_token_len;
  r->max_seq_len = max_seq_len;
  std::string line;
  std::getline(in, line);
  const int n = atoi(line.c_str());
  r->prompts.assign(n > 0 ? n : 0, std::string());
  r->outputs.assign(r->prompts.size(), std::string());
  for (int i = 0; i < n && std::getline(in, line); ++i)
    // each request owns max_token_len*max_seq_len bytes in the reference (NUL-terminated)
    r->prompts[i] = line.substr(0, r->cap() > 0 ? r->cap() - 1 : 0);
  return r;
}

extern "C" void thallama_requests_free(thallama_requests* r) { delete r; }
extern "C" int thallama_requests_count(const thallama_requests* r) { return (int)r->prompts.size(); }
extern "C" const char* thallama_requests_prompt(const thallama_requests* r, int i) { return r->prompts[i].c_str(); }
extern "C" const char* thallama_requests_output(const thallama_requests* r, int i) { return r->outputs[i].c_str(); }

extern "C" int thallama_requests_write(const thallama_requests* r, const char* path) {
  std::ofstream out(path);
  if (!out.is_open()) return -1;
  out << r->prompts.size() << "\n";
  for (const auto& g : r->outputs) out << g << "\n";
  return out.good() ? 0 : -1;
}

// ------------------------------------------------------------------------------ scheduler
// test_data_parallelism (src/llama.cpp:891-1083), with the GPU step as a callback.
extern "C" int thallama_serve_requests(thallama_requests* r, const char* tokenizer_path, int vocab_size,
                                       int n_workers, int batch, thallama_step_fn step, void* ctx,
                                       long long* gen_tokens) {
  return thallama_serve_requests_prefill(r, tokenizer_path, vocab_size, n_workers, batch, step, nullptr, ctx,
                                         gen_tokens);
}

extern "C" int thallama_serve_requests_prefill(thallama_requests* r, const char* tokenizer_path, int vocab_size,
                                               int n_workers, int batch, thallama_step_fn step,
                                               thallama_prefill_fn prefill, void* ctx, long long* gen_tokens) {
  return thallama_serve_requests_greedy(r, tokenizer_path, vocab_size, n_workers, batch, step, nullptr, prefill, ctx,
                                        gen_tokens);
}

extern "C" int thallama_serve_requests_greedy(thallama_requests* r, const char* tokenizer_path, int vocab_size,
                                              int n_workers, int batch, thallama_step_fn step,
                                              thallama_argmax_step_fn argmax_step, thallama_prefill_fn prefill,
                                              void* ctx, long long* gen_tokens) {
  return thallama_serve_requests_stats(r, tokenizer_path, vocab_size, n_workers, batch, step, argmax_step, prefill, ctx,
                                       gen_tokens, nullptr, nullptr, nullptr, nullptr);
}

extern "C" int thallama_serve_requests_stats(thallama_requests* r, const char* tokenizer_path, int vocab_size,
                                             int n_workers, int batch, thallama_step_fn step,
                                             thallama_argmax_step_fn argmax_step, thallama_prefill_fn prefill,
                                             void* ctx, long long* gen_tokens, long long* worker_tokens,
                                             double* worker_seconds, int* worker_requests, float* const* logits_bufs) {
  if (!r || n_workers <= 0 || batch <= 0) return -1;
  // greedy sampling is sample_argmax of the logits: the device step may take it (only B ids return)
  const bool on_device = argmax_step && r->temperature == 0.0f;
  if (!on_device && !step) return -1;
  const int n_req = (int)r->prompts.size();
  const int V = vocab_size;
  std::vector<thallama_sampler*> samplers((size_t)n_req);
  for (int i = 0; i < n_req; ++i) samplers[i] = thallama_sampler_create(V, r->temperature, r->topp, 314028ull);
  std::mutex mu;
  int next_req = 0;
  std::atomic<long long> gen{0};
  std::atomic<int> status{0};

  const auto t_start = std::chrono::steady_clock::now();
  auto worker = [&](int w) {
    int served = 0;
    thallama_tokenizer* tok = thallama_tokenizer_load(tokenizer_path, V);
    if (!tok) {
      status = -2;
      return;
    }
    // the step's logits: the caller's buffer for this worker (e.g. pinned host memory the device
    // copies into at the link rate, as the reference's hipHostMalloc'd logits_host), else our own
    std::vector<float> own(on_device || (logits_bufs && logits_bufs[w]) ? 0 : (size_t)batch * V);
    float* const logits = logits_bufs && logits_bufs[w] ? logits_bufs[w] : own.data();
    std::vector<int> next_ids(batch, 0);
    std::vector<int> req(batch, -1), token(batch, 0), pos(batch, 0), steps(batch, 0), n_prompt(batch, 0);
    std::vector<char> done(batch, 0);
    std::vector<std::vector<int>> prompt(batch);
    std::vector<std::string> text(batch);
    long long local = 0;
    while (status == 0) {
      int idle = 0;
      for (int b = 0; b < batch; ++b) {
        if (req[b] != -1) continue;
        {
          std::lock_guard<std::mutex> g(mu);
          req[b] = next_req;
          if (next_req < n_req) ++next_req;
        }
        if (req[b] >= n_req) {
          req[b] = -1;
          ++idle;
          continue;
        }
        fprintf(stderr, "\nDevice %d - seq id %d in batch, Request %d\n", w, b, req[b]);
        text[b].clear();
        const std::string& p = r->prompts[req[b]];
        prompt[b].assign(p.size() + 3, 0);
        thallama_tokenizer_encode(tok, p.c_str(), 1, 0, prompt[b].data(), &n_prompt[b]);
        token[b] = prompt[b][0];
        pos[b] = 0;
        steps[b] = r->max_seq_len;
        done[b] = 0;
        // Batched prompt: the reference feeds prompt tokens 0..n-2 one decode step each,
        // ignoring their logits (src/llama.cpp:1029-1031).  Processing them in one prefill
        // leaves the slot exactly where those steps would: pos = n-1, token = prompt[n-1],
        // the prompt pieces in the text.  Skipped when the prompt itself would end the
        // sequence (a BOS/EOS id past position 0, or longer than max_seq_len).
        const int m = n_prompt[b] - 1;
        bool ok = prefill && m >= 1 && m < steps[b];
        for (int i = 1; ok && i <= m; ++i) ok = prompt[b][i] != 1 && prompt[b][i] != 2;
        if (ok) {
          const int pst = prefill(ctx, w, b, prompt[b].data(), m, 0);
          if (pst < 0) {
            status = pst;
            break;
          }
          if (pst == 0) {
            for (int i = 0; i < m; ++i) {
              const char* piece = thallama_tokenizer_decode(tok, prompt[b][i], prompt[b][i + 1]);
              if (thallama_piece_is_safe(piece)) text[b] += piece;
            }
            token[b] = prompt[b][m];
            pos[b] = m;
          }
        }
      }
      if (status != 0) break;
      if (idle == batch) break;
      const int st = on_device ? argmax_step(ctx, w, batch, token.data(), pos.data(), next_ids.data())
                               : step(ctx, w, batch, token.data(), pos.data(), logits);
      if (st != 0) {
        status = st;
        break;
      }
      for (int b = 0; b < batch; ++b) {
        if (req[b] < 0) continue;
        int next;
        if (pos[b] < n_prompt[b] - 1) next = prompt[b][pos[b] + 1];  // still in the prompt
        else if (on_device) next = next_ids[b];
        else next = thallama_sample(samplers[req[b]], logits + (size_t)b * V);
        pos[b] += 1;
        if (next == 1 || next == 2) {  // BOS / EOS end the sequence
          done[b] = 1;
        } else {
          const char* piece = thallama_tokenizer_decode(tok, token[b], next);
          if (thallama_piece_is_safe(piece)) text[b] += piece;
          token[b] = next;
          if (pos[b] >= steps[b]) done[b] = 1;
        }
      }
      for (int b = 0; b < batch; ++b) {
        if (!done[b] || req[b] < 0) continue;
        text[b] += "\n";  // the reference appends one here, write_outputfile another
        r->outputs[req[b]] = text[b].substr(0, r->cap() > 0 ? r->cap() - 1 : 0);
        fprintf(stderr, "\nThread %d DONE Request %d \n", w, req[b]);
        local += pos[b] - 1;
        ++served;
        req[b] = -1;
        done[b] = 0;
        pos[b] = 0;
        token[b] = 0;
      }
    }
    gen += local;
    // per-worker accounting (one worker = one GPU's replica): its tokens, its requests, and the
    // time from the common start to its last step
    if (worker_tokens) worker_tokens[w] = local;
    if (worker_requests) worker_requests[w] = served;
    if (worker_seconds)
      worker_seconds[w] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count();
    thallama_tokenizer_free(tok);
  };

  std::vector<std::thread> pool;
  for (int w = 0; w < n_workers; ++w) pool.emplace_back(worker, w);
  for (auto& t : pool) t.join();
  for (auto* s : samplers) thallama_sampler_free(s);
  if (gen_tokens) *gen_tokens = gen.load();
  return status.load();
}
