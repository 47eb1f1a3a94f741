// rnnt_model_mi355x.hpp -- rnnt::models::TorchModel (the reference's csrc/rnnt_model.hpp:39-137) on the
// MI355X engine.  A maintainer swaps the include of rnnt_model.hpp for this file; the reference's
// State / PipelineState (metadata.hpp, metadata.cpp), OfflineSUT / ServerSUT (torch_sut.cpp) and QSL stay
// as they are.
//
// The interface is the reference's: TorchModel(model_file); forward / encode / decode(int which, S& state)
// for S = State (Offline, any split_len) or PipelineState (Server).  What it reads from the state:
//   State          f_, f_lens_ / infer_lens_, split_len_ and next() (metadata.cpp:37-86), actual_batch_size_,
//                  batch_size_, max_res_len_; writes f_lens_ = ceil(infer_lens_ / 2) (rnnt_model.hpp:88-89),
//                  res_ and res_idx_ (the result contract QuerySamplesComplete reads, torch_sut.cpp:221-236).
//   PipelineState  additionally finish_idx_ / dequeue_size_ at entry (the slots update() restarted,
//                  metadata.cpp:122-143) and padded_fea_len_; next() gathers each slot's chunks from F_.
// The LSTM / prediction state tensors of the State (pre_hx_, pre_cx_, ..., pre_cg_) are not used: that
// state lives in the engine (int8 h, fp16 c, bf16 / fp32 prediction state in HBM).
//
// Threading (the reference runs INTER = 28 Offline instances, which = index & 1, torch_sut.cpp:115-145):
// every call is re-entrant.  `which` names a CPU socket as in the reference; it selects the half of the
// node's GPUs attached to that socket (all GPUs when there are fewer than two).  encode() leases an engine
// -- its HIP stream, pinned staging and device buffers -- on the least-loaded GPU of that group and
// decode() returns it, so any number of threads may share a GPU: at most engines_per_gpu batches are in
// flight per GPU (the rest wait), and the encoders of one GPU take turns in arrival order, so each batch's
// latency-bound greedy decode runs beside the next batch's encoder (the bench's schedule).
// A PipelineState keeps its engine for its lifetime (its slots' LSTM and greedy state persist in the
// engine between calls, rnnt_engine_encode_stream / decode_stream).
//
// Chunking: the engine runs each slot's whole span of a call in one wavefront encode.  That equals the
// reference's chunk-by-chunk transcription (h / c carried between chunks, rnnt_model.hpp:64-78) when the
// chunks pair frames the same way as the whole utterance, i.e. for even split_len (pinned by the
// split_len = 2 reference fixture, tests/test_oracle_golden.py).  An odd split_len > 0 is rejected.
#pragma once
#include <ATen/ATen.h>
#include <ATen/Parallel.h>
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../../../include/rnnt_mi355x.h"

namespace rnnt {
namespace models {
namespace mi355x {

constexpr int kFeat = 240;         // TRANS_INPUT_SIZE (metadata.hpp:22)
constexpr int kMaxFeaLen = 500;    // MAX_FEA_LEN (metadata.hpp:32)
constexpr int kMaxSymbols = 30;    // MAX_SYMBOLS_PER_STEP (metadata.hpp:30)
constexpr int kRowTile = 256;      // the engine's batch tile: n_pad is a multiple of it
constexpr int32_t kSos = -1;

inline void check(int rc, const char* what) {  // return codes -> exceptions, as TORCH_CHECK would throw
  if (rc < 0) throw std::runtime_error(std::string("TorchModel: ") + what + ": " + rnnt_last_error());
}
inline void hcheck(hipError_t rc, const char* what) {
  if (rc != hipSuccess) throw std::runtime_error(std::string("TorchModel: ") + what + ": " + hipGetErrorString(rc));
}
inline int64_t round_up(int64_t v, int64_t m) { return (v + m - 1) / m * m; }

// S is a Server PipelineState when it has the slot-refill members (metadata.hpp:84-114)
template <class S, class = void>
struct is_pipeline : std::false_type {};
template <class S>
struct is_pipeline<S, std::void_t<decltype(std::declval<S&>().F_), decltype(std::declval<S&>().dequeue_size_)>>
    : std::true_type {};

struct Options {
  std::vector<int> gpus;     // devices to use (default: every visible GPU; env RNNT_GPUS="0,1,...")
  int engines_per_gpu = 4;   // Offline batches in flight per GPU (env RNNT_ENGINES_PER_GPU)
  int sockets = 2;           // `which` values the SUT passes (index & 1, torch_sut.cpp:145)
  bool encode_turns = true;  // encoders of one GPU take turns (env RNNT_ENCODE_TURNS=0 lets them overlap)
};

inline Options options_from_env() {
  Options o;
  if (const char* g = std::getenv("RNNT_GPUS")) {
    for (const char* p = g; *p;) {
      char* end = nullptr;
      const long d = std::strtol(p, &end, 10);
      if (end == p) throw std::runtime_error("TorchModel: bad RNNT_GPUS list");
      o.gpus.push_back((int)d);
      p = *end == ',' ? end + 1 : end;
    }
  } else {
    int n = 0;
    hcheck(hipGetDeviceCount(&n), "hipGetDeviceCount");
    for (int d = 0; d < n; ++d) o.gpus.push_back(d);
  }
  if (o.gpus.empty()) throw std::runtime_error("TorchModel: no GPU");
  if (const char* k = std::getenv("RNNT_ENGINES_PER_GPU")) o.engines_per_gpu = std::max(1, std::atoi(k));
  if (const char* t = std::getenv("RNNT_ENCODE_TURNS")) o.encode_turns = std::atoi(t) != 0;
  return o;
}

// One batch in flight: an engine, its stream and the buffers one call stages through.
struct Slot {
  int device = 0;
  rnnt_engine* e = nullptr;
  hipStream_t st = nullptr;
  int rows = 0, max_frames = 0, max_res = 0;  // engine capacity (rows a multiple of kRowTile)
  bool sticky = false;                        // a PipelineState's engine (slot state lives in it)
  char* host = nullptr;                       // pinned staging: [offsets i64][lens i32][reset i32][features]
  char* dev = nullptr;                        // its device mirror
  size_t cap = 0;
  int32_t* d_res = nullptr;   // [rows][max_res]
  int32_t* d_len = nullptr;   // [rows]
  int32_t* h_len = nullptr;   // pinned [rows]
  int32_t* h_res = nullptr;   // pinned [rows][widest]: the written columns, copied on to the State's res_
  size_t h_res_cap = 0;
  int32_t* d_reset = nullptr; // points into dev (stream calls)
  float* dense = nullptr;     // [T][rows][256] device input of a batch the SUT assembled in pinned memory
  size_t dense_cap = 0;
  int n = 0;                  // rows of the last encode

  void grow(size_t bytes) {
    if (bytes <= cap) return;
    const size_t c = (size_t)round_up((int64_t)std::max(bytes, cap + cap / 2), 1 << 20);
    if (host) hcheck(hipHostFree(host), "hipHostFree");
    if (dev) hcheck(hipFree(dev), "hipFree");
    host = dev = nullptr;
    cap = 0;
    hcheck(hipHostMalloc((void**)&host, c, hipHostMallocDefault), "hipHostMalloc staging");
    hcheck(hipMalloc((void**)&dev, c), "hipMalloc staging");
    cap = c;
  }
  void grow_dense(size_t bytes) {
    if (bytes <= dense_cap) return;
    if (dense) hcheck(hipFree(dense), "hipFree");
    dense = nullptr;
    dense_cap = 0;
    hcheck(hipMalloc((void**)&dense, bytes), "hipMalloc dense input");
    dense_cap = bytes;
  }
  void grow_res(size_t bytes) {
    if (bytes <= h_res_cap) return;
    if (h_res) hcheck(hipHostFree(h_res), "hipHostFree");
    h_res = nullptr;
    h_res_cap = 0;
    const size_t c = (size_t)round_up((int64_t)bytes, 1 << 20);
    hcheck(hipHostMalloc((void**)&h_res, c, hipHostMallocDefault), "hipHostMalloc results");
    h_res_cap = c;
  }
  ~Slot() {  // torn down by ~TorchModel, while the HIP runtime is up
    if (st) (void)hipStreamSynchronize(st);
    if (host) (void)hipHostFree(host);
    if (h_len) (void)hipHostFree(h_len);
    if (h_res) (void)hipHostFree(h_res);
    for (void* p : {(void*)dev, (void*)d_res, (void*)d_len, (void*)dense})
      if (p) (void)hipFree(p);
    if (st) (void)hipStreamDestroy(st);
    if (e) rnnt_engine_destroy(e);
  }
};

// host memory the device can DMA from directly (hipHostMalloc'd / registered); pageable memory is not
inline bool is_pinned_host(const void* p) {
  hipPointerAttribute_t at{};
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();  // pageable: clear the error the query left
    return false;
  }
  return at.type == hipMemoryTypeHost;
}

// One call's input: each slot's frames of this call, packed back to back (the engine's ragged store).
struct Chunk {
  at::Tensor f;     // fp32 [t][rows][C >= 240] (C++ AssembleSamples layout, or one next() chunk)
  at::Tensor lens;  // int32 [rows]: valid frames of each row in this chunk
};

// Host-side time of the calls, summed over threads (seconds): what the SUT thread spends packing the batch
// into pinned memory, copying it to the device, waiting for its GPU's encoder turn, in the encode, and in
// the decode (greedy loop + result copy).
struct CallStats {
  double pack = 0, copy = 0, turn_wait = 0, encode = 0, decode = 0;
  int64_t calls = 0, frames = 0, dense_calls = 0;  // dense: batches DMA'd from the SUT's pinned memory as they are
};

}  // namespace mi355x

class TorchModel {
 public:
  using Options = mi355x::Options;

  // rnnt_model.hpp:41-47.  model_file: the engine file (tools/export_model.py --engine-file) in place of the
  // TorchScript model; engines are created on first use, sized to the batches the SUT sends.
  explicit TorchModel(const std::string& model_file) : TorchModel(model_file, mi355x::options_from_env()) {}
  TorchModel(const std::string& model_file, Options opts) : file_(model_file), opts_(std::move(opts)) {
    for (int d : opts_.gpus) gpus_.emplace_back(new Gpu{d});
  }
  ~TorchModel() {
    std::lock_guard<std::mutex> l(mu_);
    for (auto& g : gpus_) g->slots.clear();
  }
  TorchModel(const TorchModel&) = delete;
  TorchModel& operator=(const TorchModel&) = delete;

  template <class S>
  void forward(int which, S& state) {  // rnnt_model.hpp:56-60
    encode(which, state);
    decode(which, state);
  }

  // rnnt_model.hpp:62-90.  The batch's features (the whole f_, or every chunk next() yields) go to the
  // engine in one staged copy and one wavefront encode; f_lens_ = ceil(infer_lens_ / 2).
  template <class S>
  void encode(int which, S& state) {
    constexpr bool pipe = mi355x::is_pipeline<S>::value;
    if (state.split_len_ > 0 && (state.split_len_ & 1))
      throw std::runtime_error("TorchModel::encode: odd split_len pairs StackTime frames across chunks; use an even one");
    // the slots update() restarted (its masked_fill_ set, metadata.cpp:122-143): read before next() moves them
    std::vector<int32_t> reset;
    if constexpr (pipe) {
      const at::Tensor fi = state.finish_idx_.to(at::kInt).contiguous();
      reset.assign(fi.data_ptr<int32_t>(), fi.data_ptr<int32_t>() + fi.numel());
      if (state.dequeue_size_ == 0) std::fill(reset.begin(), reset.end(), 0);
    }
    std::vector<mi355x::Chunk> chunks;
    if (state.split_len_ > 0) {
      while (state.next()) chunks.push_back({state.f_, state.f_lens_});
      if (chunks.empty()) throw std::runtime_error("TorchModel::encode: the state has no chunk to encode");
    } else {
      chunks.push_back({state.f_, state.infer_lens_});
    }
    const int rows = (int)state.batch_size_;
    const int n = pipe ? rows : (state.actual_batch_size_ > 0 ? std::min<int>(state.actual_batch_size_, rows) : rows);
    // engines hold a multiple of 64 frames, at least MAX_FEA_LEN (the warmup's MAX_WAV_LEN dummy audio makes
    // 501 frames, rnnt_qsl.cpp:140-141; a PipelineState pads to whole chunks, metadata.cpp:98-102)
    int64_t frames = pipe ? (int64_t)state.padded_fea_len_ : 0;
    for (const auto& c : chunks) frames += pipe ? 0 : c.f.size(0);
    const int max_frames = (int)mi355x::round_up(std::max<int64_t>(frames, mi355x::kMaxFeaLen), 64);
    Lease ls = lease(which, &state, pipe, rows, max_frames, (int)state.max_res_len_);
    try {
      run_encode(ls, chunks, n, rows, pipe ? reset.data() : nullptr);
    } catch (...) {
      release(&state, /*failed=*/true);
      throw;
    }
    state.f_lens_ = (state.infer_lens_ + 1).div(2, "floor").to(at::kInt);  // ceil(infer_lens / STACK_TIME_FACTOR)
  }

  // rnnt_model.hpp:92-124: the greedy loop; res_ / res_idx_ as the reference leaves them (res_idx_ =
  // tokens - 1; res_ keeps update()'s SOS fill past each row's tokens).
  template <class S>
  void decode(int which, S& state) {
    (void)which;
    constexpr bool pipe = mi355x::is_pipeline<S>::value;
    Lease ls = find(&state);
    mi355x::Slot& s = *ls.slot;
    const auto t0 = Clock::now();
    try {
      hcheck(hipSetDevice(s.device), "hipSetDevice");
      const int n = s.n;
      if (pipe)
        mi355x::check(rnnt_engine_decode_stream(s.e, s.d_res, s.d_len, s.max_res, s.d_reset, s.st), "rnnt_engine_decode_stream");
      else
        mi355x::check(rnnt_engine_decode(s.e, s.d_res, s.d_len, s.max_res, s.st), "rnnt_engine_decode");
      hcheck(hipMemcpyAsync(s.h_len, s.d_len, sizeof(int32_t) * n, hipMemcpyDeviceToHost, s.st), "copy res_len");
      hcheck(hipStreamSynchronize(s.st), "sync");
      at::Tensor& res = state.res_;
      at::Tensor& res_idx = state.res_idx_;
      if (!res.is_contiguous() || res.scalar_type() != at::kInt || res.size(0) < n || res.size(1) > s.max_res ||
          res_idx.scalar_type() != at::kInt || res_idx.numel() < n)
        throw std::runtime_error("TorchModel::decode: res_ / res_idx_ are not the State's int32 [batch][max_res_len]");
      int32_t widest = 0;
      int32_t* idx = res_idx.data_ptr<int32_t>();
      for (int i = 0; i < n; ++i) {
        const int32_t len = std::min<int32_t>(s.h_len[i], (int32_t)res.size(1));
        idx[i] = len - 1;  // metadata.cpp:59-60; QuerySamplesComplete sends (res_idx_ + 1) * 4 bytes
        widest = std::max(widest, len);
      }
      if (widest > 0) {  // only the written columns travel, through pinned memory (a 2-D copy straight into the
                         // State's pageable res_ goes through the runtime's staging, row by row)
        s.grow_res((size_t)n * widest * sizeof(int32_t));
        hcheck(hipMemcpy2DAsync(s.h_res, (size_t)widest * sizeof(int32_t), s.d_res, (size_t)s.max_res * sizeof(int32_t),
                                (size_t)widest * sizeof(int32_t), (size_t)n, hipMemcpyDeviceToHost, s.st),
               "copy res");
        hcheck(hipStreamSynchronize(s.st), "sync");
        int32_t* rp = res.data_ptr<int32_t>();
        const int64_t pitch = res.size(1);
        for (int i = 0; i < n; ++i) std::memcpy(rp + i * pitch, s.h_res + (size_t)i * widest, sizeof(int32_t) * widest);
      }
    } catch (...) {
      release(&state, true);
      throw;
    }
    release(&state, false);
    std::lock_guard<std::mutex> l(stats_mu_);
    stats_.decode += secs(t0, Clock::now());
  }

  mi355x::CallStats stats(bool reset = false) {
    std::lock_guard<std::mutex> l(stats_mu_);
    const mi355x::CallStats s = stats_;
    if (reset) stats_ = {};
    return s;
  }

  // engines created so far per GPU (for tests and logs)
  std::vector<int> engines_per_gpu() const {
    std::lock_guard<std::mutex> l(mu_);
    std::vector<int> v;
    for (auto& g : gpus_) v.push_back((int)g->slots.size());
    return v;
  }

 private:
  struct Gpu {
    int device;
    std::vector<std::unique_ptr<mi355x::Slot>> slots;  // owned
    std::vector<mi355x::Slot*> idle;
    int transient = 0;  // Offline leases out
    int active = 0;     // every lease out (+ reservations)
    std::mutex turn_mu;  // encoders take turns: a FIFO ticket lock
    std::condition_variable turn_cv;
    uint64_t next_ticket = 0, serving = 0;
  };
  struct Lease {
    Gpu* gpu = nullptr;
    mi355x::Slot* slot = nullptr;
  };

  std::vector<int> group(int which) const {
    const int n = (int)gpus_.size(), k = std::max(1, opts_.sockets);
    std::vector<int> g;
    if (n >= k) {
      const int w = ((which % k) + k) % k;
      for (int i = w * n / k; i < (w + 1) * n / k; ++i) g.push_back(i);
    }
    if (g.empty())
      for (int i = 0; i < n; ++i) g.push_back(i);
    return g;
  }

  // An engine for `key`'s batch: the one it already holds (re-encode, or a PipelineState's own), an idle
  // one on the least-loaded GPU of the socket's group that fits, or a new one.
  Lease lease(int which, const void* key, bool sticky, int rows, int max_frames, int max_res) {
    const int need_rows = (int)mi355x::round_up(std::max(rows, 1), mi355x::kRowTile);
    std::unique_lock<std::mutex> l(mu_);
    auto it = leases_.find(key);
    if (it != leases_.end()) {
      mi355x::Slot* s = it->second.slot;
      if (s->rows < need_rows || s->max_frames < max_frames || s->max_res < max_res)
        throw std::runtime_error("TorchModel::encode: the state's batch outgrew the engine it holds");
      return it->second;
    }
    const std::vector<int> grp = group(which);
    Gpu* g = nullptr;
    lease_cv_.wait(l, [&] {
      g = nullptr;
      for (int i : grp) {
        Gpu* c = gpus_[i].get();
        if (!sticky && c->transient >= opts_.engines_per_gpu) continue;
        if (!g || c->active < g->active) g = c;
      }
      return g != nullptr;
    });
    mi355x::Slot* s = nullptr;
    for (size_t i = 0; i < g->idle.size(); ++i) {
      mi355x::Slot* c = g->idle[i];
      if (c->rows >= need_rows && c->max_frames >= max_frames && c->max_res >= max_res) {
        s = c;
        g->idle.erase(g->idle.begin() + (long)i);
        break;
      }
    }
    if (!sticky) g->transient++;
    g->active++;
    if (!s) {  // create outside the lock (reads the engine file, packs the weights)
      l.unlock();
      std::unique_ptr<mi355x::Slot> ns;
      try {
        ns = make_slot(g->device, need_rows, max_frames, max_res);
      } catch (...) {
        l.lock();
        if (!sticky) g->transient--;
        g->active--;
        lease_cv_.notify_all();
        throw;
      }
      l.lock();
      s = ns.get();
      g->slots.push_back(std::move(ns));
    }
    s->sticky = sticky;
    Lease ls{g, s};
    leases_[key] = ls;
    return ls;
  }

  Lease find(const void* key) {
    std::lock_guard<std::mutex> l(mu_);
    auto it = leases_.find(key);
    if (it == leases_.end()) throw std::runtime_error("TorchModel::decode: no encode of this state to decode");
    return it->second;
  }

  // back to the GPU's idle list after decode (a PipelineState keeps its engine unless a call failed)
  void release(const void* key, bool failed) {
    std::lock_guard<std::mutex> l(mu_);
    auto it = leases_.find(key);
    if (it == leases_.end()) return;
    Lease ls = it->second;
    if (ls.slot->sticky && !failed) return;
    leases_.erase(it);
    if (!ls.slot->sticky) ls.gpu->transient--;
    ls.gpu->active--;
    if (failed) {  // the engine's state is unknown: drop it
      auto& v = ls.gpu->slots;
      v.erase(std::remove_if(v.begin(), v.end(), [&](const std::unique_ptr<mi355x::Slot>& p) { return p.get() == ls.slot; }),
              v.end());
    } else {
      ls.gpu->idle.push_back(ls.slot);
    }
    lease_cv_.notify_all();
  }

  std::unique_ptr<mi355x::Slot> make_slot(int device, int rows, int max_frames, int max_res) {
    auto s = std::make_unique<mi355x::Slot>();
    s->device = device;
    s->rows = rows;
    s->max_frames = max_frames;
    s->max_res = max_res;
    rnnt_opts o{rows, max_frames, max_res};
    mi355x::check(rnnt_engine_create_from_file(file_.c_str(), device, &o, &s->e), "rnnt_engine_create_from_file");
    hcheck(hipSetDevice(device), "hipSetDevice");
    hcheck(hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking), "hipStreamCreate");
    hcheck(hipMalloc((void**)&s->d_res, (size_t)rows * max_res * sizeof(int32_t)), "hipMalloc res");
    hcheck(hipMalloc((void**)&s->d_len, (size_t)rows * sizeof(int32_t)), "hipMalloc res_len");
    hcheck(hipHostMalloc((void**)&s->h_len, (size_t)rows * sizeof(int32_t), hipHostMallocDefault), "hipHostMalloc res_len");
    return s;
  }

  static void hcheck(hipError_t rc, const char* what) { mi355x::hcheck(rc, what); }
  using Clock = std::chrono::steady_clock;
  static double secs(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double>(b - a).count(); }

  // Packs every row's frames of this call into the slot's pinned staging area (row i's frames back to
  // back from offsets[i], only the 240 real channels: AssembleSamples leaves channels 240..255 zero and
  // the engine's layer-0 weights there are zero), one copy to the device, then the encode -- after the
  // GPU's earlier encoders (turns in arrival order).
  // split_len chunks that are consecutive slices of one contiguous batch (State::update's torch::split of f,
  // metadata.cpp:63) -> that batch as one chunk (a non-owning view; the chunks keep it alive for the call)
  static bool merge_adjacent(const std::vector<mi355x::Chunk>& chunks, std::vector<mi355x::Chunk>& out) {
    if (chunks.size() < 2) return false;
    const at::Tensor& f0 = chunks[0].f;
    if (f0.dim() != 3 || f0.scalar_type() != at::kFloat || !f0.is_contiguous() || !f0.device().is_cpu()) return false;
    const int64_t R = f0.size(1), C = f0.size(2);
    const float* next = f0.data_ptr<float>();
    int64_t T = 0;
    at::Tensor lens = at::zeros_like(chunks[0].lens.to(at::kCPU, at::kInt));
    for (const auto& c : chunks) {
      if (c.f.dim() != 3 || c.f.scalar_type() != at::kFloat || !c.f.is_contiguous() || !c.f.device().is_cpu() ||
          c.f.size(1) != R || c.f.size(2) != C || c.f.data_ptr<float>() != next)
        return false;
      next += c.f.size(0) * R * C;
      T += c.f.size(0);
      lens += c.lens.to(at::kCPU, at::kInt);
    }
    out.push_back({at::from_blob(f0.data_ptr<float>(), {T, R, C}, at::kFloat), lens});
    return true;
  }

  void run_encode(const Lease& ls, const std::vector<mi355x::Chunk>& chunks_in, int n, int rows, const int32_t* reset) {
    mi355x::Slot& s = *ls.slot;
    std::vector<mi355x::Chunk> merged;
    const std::vector<mi355x::Chunk>& chunks = !reset && merge_adjacent(chunks_in, merged) ? merged : chunks_in;
    std::vector<at::Tensor> f(chunks.size()), cl(chunks.size());
    for (size_t c = 0; c < chunks.size(); ++c) {
      f[c] = chunks[c].f.to(at::kCPU, at::kFloat).contiguous();
      cl[c] = chunks[c].lens.to(at::kCPU, at::kInt).contiguous();
      if (f[c].dim() != 3 || f[c].size(1) < rows || f[c].size(2) < mi355x::kFeat || cl[c].numel() < rows)
        throw std::runtime_error("TorchModel::encode: features are not [T][batch][C >= 240] with a length per row");
    }
    const int n_pad = (int)mi355x::round_up(std::max(n, 1), mi355x::kRowTile);
    std::vector<int64_t> off(n_pad, 0);
    std::vector<int32_t> len(n_pad, 0);
    int64_t total = 0;
    int T = 1;
    for (int i = 0; i < n; ++i) {
      int64_t li = 0;
      for (size_t c = 0; c < chunks.size(); ++c) {
        const int32_t v = cl[c].data_ptr<int32_t>()[i];
        if (v < 0 || v > f[c].size(0)) throw std::runtime_error("TorchModel::encode: a length exceeds its frames");
        li += v;
      }
      off[i] = total;
      len[i] = (int32_t)li;
      total += li;
      T = std::max<int>(T, (int)li);
    }
    if (T > s.max_frames) throw std::runtime_error("TorchModel::encode: more frames than the engine holds");
    // a whole batch the SUT assembled in pinned memory ([T][rows][256], zero past each length and in
    // channels 240..255, as AssembleSamples leaves it) goes to HBM as it is: one 2-D copy, no packing
    if (!reset && chunks.size() == 1 && f[0].size(2) == 256 && f[0].data_ptr() == chunks[0].f.data_ptr() &&
        mi355x::is_pinned_host(f[0].data_ptr())) {
      run_encode_dense(ls, f[0], len, T, n, n_pad);
      return;
    }
    const size_t o_off = 0, o_len = o_off + sizeof(int64_t) * n_pad, o_rst = o_len + sizeof(int32_t) * n_pad,
                 o_feat = (size_t)mi355x::round_up((int64_t)(o_rst + sizeof(int32_t) * n_pad), 256);
    const size_t bytes = o_feat + (size_t)total * mi355x::kFeat * sizeof(float);
    hcheck(hipSetDevice(s.device), "hipSetDevice");
    hcheck(hipStreamSynchronize(s.st), "sync");  // the staging area's previous copy has landed
    s.grow(bytes);
    std::memcpy(s.host + o_off, off.data(), sizeof(int64_t) * n_pad);
    std::memcpy(s.host + o_len, len.data(), sizeof(int32_t) * n_pad);
    int32_t* hr = (int32_t*)(s.host + o_rst);
    for (int i = 0; i < n_pad; ++i) hr[i] = reset && i < n ? (reset[i] ? 1 : 0) : 0;
    float* feat = (float*)(s.host + o_feat);
    const auto t0 = Clock::now();
    // blocks of 32 rows, frames outer: each frame's 32 source rows are one contiguous run of the
    // frame-major input, and the block writes 32 sequential destination streams (row-by-row packing
    // would touch a new page per 960-byte frame: the rows of one frame are n x 1 KB apart)
    at::parallel_for(0, (n + 31) / 32, 1, [&](int64_t b, int64_t e) {
      for (int64_t blk = b; blk < e; ++blk) {
        const int64_t i0 = blk * 32, i1 = std::min<int64_t>(n, i0 + 32);
        int64_t base[32];
        for (int64_t i = i0; i < i1; ++i) base[i - i0] = off[i];
        for (size_t c = 0; c < chunks.size(); ++c) {
          const int32_t* lc = cl[c].data_ptr<int32_t>();
          const int64_t R = f[c].size(1), C = f[c].size(2);
          int32_t tmax = 0;
          for (int64_t i = i0; i < i1; ++i) tmax = std::max(tmax, lc[i]);
          for (int32_t t = 0; t < tmax; ++t) {
            const float* src = f[c].data_ptr<float>() + (int64_t)t * R * C;
            for (int64_t i = i0; i < i1; ++i)
              if (t < lc[i]) std::memcpy(feat + (base[i - i0] + t) * mi355x::kFeat, src + i * C, mi355x::kFeat * sizeof(float));
          }
          for (int64_t i = i0; i < i1; ++i) base[i - i0] += lc[i];
        }
      }
    });
    const auto t1 = Clock::now();
    hcheck(hipMemcpyAsync(s.dev, s.host, bytes, hipMemcpyHostToDevice, s.st), "copy batch");
    hcheck(hipStreamSynchronize(s.st), "sync");
    const auto t2 = Clock::now();
    const int64_t* d_off = (const int64_t*)(s.dev + o_off);
    const int32_t* d_len = (const int32_t*)(s.dev + o_len);
    s.d_reset = (int32_t*)(s.dev + o_rst);
    const float* store = (const float*)(s.dev + o_feat);
    Gpu& g = *ls.gpu;
    uint64_t ticket = 0;
    if (opts_.encode_turns) {
      std::unique_lock<std::mutex> l(g.turn_mu);
      ticket = g.next_ticket++;
      g.turn_cv.wait(l, [&] { return g.serving == ticket; });
    }
    const auto t3 = Clock::now();
    int rc = 0;
    hipError_t hr_sync = hipSuccess;
    if (reset)
      rc = rnnt_engine_encode_stream(s.e, store, d_off, d_len, len.data(), s.d_reset, T, n, n_pad, s.st);
    else
      rc = rnnt_engine_encode_gather(s.e, store, d_off, d_len, len.data(), T, n, n_pad, nullptr, s.st);
    if (rc == 0) hr_sync = hipStreamSynchronize(s.st);  // the encoder is free again: the next turn may go
    if (opts_.encode_turns) {
      std::lock_guard<std::mutex> l(g.turn_mu);
      g.serving++;
      g.turn_cv.notify_all();
    }
    const auto t4 = Clock::now();
    mi355x::check(rc, reset ? "rnnt_engine_encode_stream" : "rnnt_engine_encode_gather");
    hcheck(hr_sync, "sync");
    s.n = n;
    std::lock_guard<std::mutex> l(stats_mu_);
    stats_.pack += secs(t0, t1);
    stats_.copy += secs(t1, t2);
    stats_.turn_wait += secs(t2, t3);
    stats_.encode += secs(t3, t4);
    stats_.calls++;
    stats_.frames += total;
  }

  void run_encode_dense(const Lease& ls, const at::Tensor& x, const std::vector<int32_t>& len, int T, int n, int n_pad) {
    mi355x::Slot& s = *ls.slot;
    const int64_t R = x.size(1), w = std::min<int64_t>(R, n_pad);
    const size_t row = 256 * sizeof(float), pitch = (size_t)n_pad * row;
    hcheck(hipSetDevice(s.device), "hipSetDevice");
    hcheck(hipStreamSynchronize(s.st), "sync");
    s.grow(sizeof(int32_t) * n_pad);
    s.grow_dense((size_t)T * pitch);
    std::memcpy(s.host, len.data(), sizeof(int32_t) * n_pad);
    const auto t0 = Clock::now();
    hcheck(hipMemcpyAsync(s.dev, s.host, sizeof(int32_t) * n_pad, hipMemcpyHostToDevice, s.st), "copy lens");
    if (w < n_pad)
      hcheck(hipMemset2DAsync((char*)s.dense + w * row, pitch, 0, (size_t)(n_pad - w) * row, (size_t)T, s.st), "zero rows");
    hcheck(hipMemcpy2DAsync(s.dense, pitch, x.data_ptr<float>(), (size_t)R * row, (size_t)w * row, (size_t)T,
                            hipMemcpyHostToDevice, s.st),
           "copy batch");
    hcheck(hipStreamSynchronize(s.st), "sync");
    const auto t1 = Clock::now();
    Gpu& g = *ls.gpu;
    uint64_t ticket = 0;
    if (opts_.encode_turns) {
      std::unique_lock<std::mutex> l(g.turn_mu);
      ticket = g.next_ticket++;
      g.turn_cv.wait(l, [&] { return g.serving == ticket; });
    }
    const auto t2 = Clock::now();
    const int rc = rnnt_engine_encode(s.e, s.dense, (const int32_t*)s.dev, len.data(), T, n, n_pad, nullptr, s.st);
    const hipError_t hs = rc == 0 ? hipStreamSynchronize(s.st) : hipSuccess;
    if (opts_.encode_turns) {
      std::lock_guard<std::mutex> l(g.turn_mu);
      g.serving++;
      g.turn_cv.notify_all();
    }
    const auto t3 = Clock::now();
    mi355x::check(rc, "rnnt_engine_encode");
    hcheck(hs, "sync");
    s.n = n;
    int64_t frames = 0;
    for (int i = 0; i < n; ++i) frames += len[i];
    std::lock_guard<std::mutex> l(stats_mu_);
    stats_.copy += secs(t0, t1);
    stats_.turn_wait += secs(t1, t2);
    stats_.encode += secs(t2, t3);
    stats_.calls++;
    stats_.frames += frames;
    stats_.dense_calls++;
  }

  std::string file_;
  Options opts_;
  std::vector<std::unique_ptr<Gpu>> gpus_;
  mutable std::mutex mu_;
  std::condition_variable lease_cv_;
  std::unordered_map<const void*, Lease> leases_;
  mutable std::mutex stats_mu_;
  mi355x::CallStats stats_;
};

}  // namespace models
}  // namespace rnnt
