// rnnt_processor_mi355x.hpp -- rnnt::models::AudioProcessor (the reference's csrc/rnnt_processor.hpp:15-58) on
// the MI355X featurizer, for the SUT's WAV=true path (launch_sut.sh:53-55, run.sh STAGE=5).  A maintainer
// swaps the include of rnnt_processor.hpp for this file; OfflineSUT / ServerSUT call it unchanged:
//   processor_.forward(which, x, x_lens, pad_batch_size_)      (torch_sut.cpp:196-200, 446-447)
// x: the QSL's AssembleSamples(processor = true) batch, fp32 [N][max_wav_len] zero-padded audio (rnnt_qsl.cpp:
// 163-179); x_lens: samples per row.  Returns what the TorchScript processor returns (features.py:185-252):
// features [N_out][256][T] fp32 -- normalised per utterance and channel, zero past each row's frames, in
// channels 240..255 and in rows N..N_out-1, N_out = N rounded up to 32 when pad_batch_size -- and their
// lengths int32 [N_out].  The SUT permutes them to [T][N_out][256] (torch_sut.cpp:200); the tensor returned
// here is a permuted view of a pinned [T][N_out][256] host buffer, so that permute gives back a contiguous
// pinned tensor and TorchModel::encode DMAs it to HBM as it is (rnnt_model_mi355x.hpp).
//
// The model file is the processor file tools/export_model.py --processor-file writes (window and mel
// filterbank, rnnt_featurizer_create_from_file) instead of the TorchScript processor.  Threading as
// TorchModel: `socket` selects the half of the node's GPUs on that socket; every call leases a featurizer
// (stream, pinned staging, device buffers) on the least-loaded GPU of the group.
#pragma once
#include <ATen/ATen.h>
#include <ATen/Parallel.h>
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "../../../include/rnnt_mi355x.h"
#include "rnnt_model_mi355x.hpp"

namespace rnnt {
namespace models {

class AudioProcessor {
 public:
  explicit AudioProcessor(const std::string& filename) : AudioProcessor(filename, mi355x::options_from_env()) {}
  AudioProcessor(const std::string& filename, mi355x::Options opts)
      : file_(filename), opts_(std::move(opts)), out_pool_(std::make_shared<OutPool>()) {
    for (int d : opts_.gpus) gpus_.emplace_back(new Gpu{d});
  }
  ~AudioProcessor() {
    std::lock_guard<std::mutex> l(mu_);
    for (auto& g : gpus_) g->slots.clear();
  }
  AudioProcessor(const AudioProcessor&) = delete;
  AudioProcessor& operator=(const AudioProcessor&) = delete;

  // rnnt_processor.hpp:28-37 (no socket: the first socket's GPUs)
  std::tuple<at::Tensor, at::Tensor> forward(at::Tensor& wav, at::Tensor& wav_lens, bool pad_batch_size) {
    return forward(0, wav, wav_lens, pad_batch_size);
  }

  // rnnt_processor.hpp:39-50
  std::tuple<at::Tensor, at::Tensor> forward(int socket, at::Tensor& wav, at::Tensor& wav_lens, bool pad_batch_size) {
    const at::Tensor x = wav.to(at::kCPU, at::kFloat).contiguous();
    const at::Tensor xl = wav_lens.to(at::kCPU, at::kInt).contiguous();
    if (x.dim() != 2 || xl.numel() != x.size(0)) throw std::runtime_error("AudioProcessor: wav is not [N][samples]");
    const int n = (int)x.size(0);
    const int n_out = pad_batch_size ? (n + 31) / 32 * 32 : std::max(n, 1);
    const int32_t* lens = xl.data_ptr<int32_t>();
    std::vector<int64_t> off(std::max(n, 1), 0);
    int64_t total = 0;
    int T = 1;
    for (int i = 0; i < n; ++i) {
      if (lens[i] < 0 || lens[i] > x.size(1)) throw std::runtime_error("AudioProcessor: a length exceeds its row");
      off[i] = total;
      total += lens[i];
      T = std::max<int>(T, (int)rnnt_featurizer_frames(lens[i]));
    }
    Slot& s = lease(socket);
    struct Release {
      AudioProcessor* p;
      Slot* s;
      ~Release() { p->release(s); }
    } rel{this, &s};
    mi355x::hcheck(hipSetDevice(s.device), "hipSetDevice");
    // staging: [offsets i64 n][lens i32 n][pad][samples]
    const size_t o_len = sizeof(int64_t) * off.size(), o_wav = (size_t)mi355x::round_up((int64_t)(o_len + sizeof(int32_t) * off.size()), 256);
    const size_t bytes = o_wav + (size_t)total * sizeof(float);
    s.stage.grow(bytes);
    std::memcpy(s.stage.host, off.data(), o_len);
    if (n) std::memcpy(s.stage.host + o_len, lens, sizeof(int32_t) * n);
    float* w = (float*)(s.stage.host + o_wav);
    const float* xs = x.data_ptr<float>();
    const int64_t pitch = x.size(1);
    at::parallel_for(0, n, 16, [&](int64_t b, int64_t e) {  // the rows' audio back to back (the batch's bulk copy)
      for (int64_t i = b; i < e; ++i) std::memcpy(w + off[i], xs + i * pitch, sizeof(float) * lens[i]);
    });
    mi355x::hcheck(hipMemcpyAsync(s.stage.dev, s.stage.host, bytes, hipMemcpyHostToDevice, s.st), "copy wav");
    const size_t fbytes = (size_t)T * n_out * 256 * sizeof(float);
    if (fbytes > s.feats_cap) {
      if (s.feats) mi355x::hcheck(hipFree(s.feats), "hipFree");
      s.feats = nullptr;
      s.feats_cap = 0;
      mi355x::hcheck(hipMalloc((void**)&s.feats, fbytes + (size_t)n_out * 4 + 256), "hipMalloc features");
      s.feats_cap = fbytes;
    }
    int32_t* d_flen = (int32_t*)((char*)s.feats + (size_t)mi355x::round_up((int64_t)fbytes, 256));
    mi355x::check(rnnt_featurizer_run(s.fz, (const float*)(s.stage.dev + o_wav), (const int64_t*)s.stage.dev, 0,
                                      (const int32_t*)(s.stage.dev + o_len), lens, n, n_out, s.feats, d_flen, T, s.st),
                  "rnnt_featurizer_run");
    // features to a pinned host buffer (returned to the pool when the SUT drops the tensor)
    float* host = out_pool_->take(fbytes);
    at::Tensor F = at::from_blob(host, {T, n_out, 256}, [pool = out_pool_](void* p) { pool->give((float*)p); }, at::kFloat);
    at::Tensor fl = at::empty({n_out}, at::kInt);
    mi355x::hcheck(hipMemcpyAsync(host, s.feats, fbytes, hipMemcpyDeviceToHost, s.st), "copy features");
    mi355x::hcheck(hipMemcpyAsync(fl.data_ptr<int32_t>(), d_flen, sizeof(int32_t) * n_out, hipMemcpyDeviceToHost, s.st),
                   "copy lengths");
    mi355x::hcheck(hipStreamSynchronize(s.st), "sync");
    return {F.permute({1, 2, 0}), fl};
  }

 private:
  // pinned host buffers of feature batches, back in the pool once the SUT drops the tensor
  struct OutPool {
    std::mutex mu;
    std::vector<std::pair<float*, size_t>> all, free;  // (buffer, capacity)
    float* take(size_t bytes) {
      {
        std::lock_guard<std::mutex> l(mu);
        for (size_t i = 0; i < free.size(); ++i)
          if (free[i].second >= bytes) {
            float* p = free[i].first;
            free.erase(free.begin() + (long)i);
            return p;
          }
      }
      float* p = nullptr;
      const size_t c = (size_t)mi355x::round_up((int64_t)std::max<size_t>(bytes, 1), 1 << 20);
      mi355x::hcheck(hipHostMalloc((void**)&p, c, hipHostMallocDefault), "hipHostMalloc features");
      std::lock_guard<std::mutex> l(mu);
      all.emplace_back(p, c);
      return p;
    }
    void give(float* p) {
      std::lock_guard<std::mutex> l(mu);
      for (auto& a : all)
        if (a.first == p) {
          free.push_back(a);
          return;
        }
    }
    ~OutPool() {
      for (auto& a : all) (void)hipHostFree(a.first);
    }
  };
  struct Staging {
    char* host = nullptr;
    char* dev = nullptr;
    size_t cap = 0;
    void grow(size_t bytes) {
      if (bytes <= cap) return;
      const size_t c = (size_t)mi355x::round_up((int64_t)std::max(bytes, cap + cap / 2), 1 << 20);
      if (host) mi355x::hcheck(hipHostFree(host), "hipHostFree");
      if (dev) mi355x::hcheck(hipFree(dev), "hipFree");
      host = dev = nullptr;
      cap = 0;
      mi355x::hcheck(hipHostMalloc((void**)&host, c, hipHostMallocDefault), "hipHostMalloc staging");
      mi355x::hcheck(hipMalloc((void**)&dev, c), "hipMalloc staging");
      cap = c;
    }
    ~Staging() {
      if (host) (void)hipHostFree(host);
      if (dev) (void)hipFree(dev);
    }
  };
  struct Slot {
    int device = 0;
    rnnt_featurizer* fz = nullptr;
    hipStream_t st = nullptr;
    Staging stage;
    float* feats = nullptr;
    size_t feats_cap = 0;
    ~Slot() {
      if (st) (void)hipStreamSynchronize(st);
      if (feats) (void)hipFree(feats);
      if (st) (void)hipStreamDestroy(st);
      if (fz) rnnt_featurizer_destroy(fz);
    }
  };
  struct Gpu {
    int device;
    std::vector<std::unique_ptr<Slot>> slots;
    std::vector<Slot*> idle;
    int active = 0;
  };

  Slot& lease(int socket) {
    std::unique_lock<std::mutex> l(mu_);
    const int n = (int)gpus_.size(), k = std::max(1, opts_.sockets);
    Gpu* g = nullptr;
    for (int i = 0; i < n; ++i) {
      const int w = ((socket % k) + k) % k;
      const bool mine = n < k || (i >= w * n / k && i < (w + 1) * n / k);
      if (mine && (!g || gpus_[i]->active < g->active)) g = gpus_[i].get();
    }
    if (!g) g = gpus_[0].get();
    g->active++;
    if (!g->idle.empty()) {
      Slot* s = g->idle.back();
      g->idle.pop_back();
      return *s;
    }
    l.unlock();
    auto s = std::make_unique<Slot>();
    s->device = g->device;
    try {
      mi355x::check(rnnt_featurizer_create_from_file(file_.c_str(), g->device, &s->fz), "rnnt_featurizer_create_from_file");
      mi355x::hcheck(hipSetDevice(g->device), "hipSetDevice");
      mi355x::hcheck(hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking), "hipStreamCreate");
    } catch (...) {
      l.lock();
      g->active--;
      throw;
    }
    l.lock();
    Slot* p = s.get();
    g->slots.push_back(std::move(s));
    return *p;
  }
  void release(Slot* s) {
    std::lock_guard<std::mutex> l(mu_);
    for (auto& g : gpus_)
      if (g->device == s->device) {
        g->idle.push_back(s);
        g->active--;
        return;
      }
  }

  std::string file_;
  mi355x::Options opts_;
  std::vector<std::unique_ptr<Gpu>> gpus_;
  std::mutex mu_;
  std::shared_ptr<OutPool> out_pool_;
};

}  // namespace models
}  // namespace rnnt
