// rnnt_model_mi355x.hpp -- the body of the reference's TorchModel (csrc/rnnt_model.hpp:39-137) on the
// MI355X engine, as a maintainer drops it into the C++ LoadGen SUT.
//
// Compiled and run: csrc/sut/sut_harness.cpp drives it exactly as OfflineSUT::thInstance does
// (state.update -> model.encode -> model.decode -> QuerySamplesComplete, torch_sut.cpp:185-236) and
// tests/test_sut_harness_gpu.py checks the responses against the CPU restatement.
//
// What stays the reference's: the State contract the SUT reads after decode (metadata.hpp:37-81,
// metadata.cpp:37-74) -- res_ host int32 [batch][max_res_len_] filled with SOS (-1) past each row's
// tokens, res_idx_ host int32 [batch] = tokens - 1 (-1 for none), actual_batch_size_ -- and the call
// shapes encode(which, state) / decode(which, state).  What changes: `which` is a GPU index instead
// of a socket (torch_sut.cpp:145), the model file is the engine file tools/export_model.py writes
// (instead of the TorchScript module, rnnt_model.hpp:41-54), and the encoder / decoder state lives
// in the engine, so State keeps only the batch, its lengths and the results.
#pragma once
#include <ATen/ATen.h>
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../include/rnnt_mi355x.h"

namespace rnnt {

enum Params {  // metadata.hpp:19-34
  STACK_TIME_FACTOR = 2,
  SOS = -1,
  BLANK = 28,
  MAX_SYMBOLS_PER_STEP = 30,
  MAX_FEA_LEN = 500,
  PADDED_INPUT_SIZE = 256
};

inline void check(int rc, const char* what) {  // the reference's TORCH_CHECK convention: errors throw
  if (rc < 0) throw std::runtime_error(std::string(what) + ": " + rnnt_last_error());
}
inline void hcheck(hipError_t rc, const char* what) {
  if (rc != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(rc));
}

// State (metadata.hpp:37-81), Offline form: the members the SUT and the model driver touch.
class State {
 public:
  State() = default;
  explicit State(int32_t batch_size, int32_t split_len = -1) { init(batch_size, split_len); }
  void init(int32_t batch_size, int32_t split_len = -1) {  // metadata.cpp:5-35 (results part)
    batch_size_ = batch_size;
    split_len_ = split_len;
    res_ = at::empty({batch_size_, max_res_len_}, at::kInt);
    res_idx_ = at::empty({batch_size_}, at::kInt);
  }
  // metadata.cpp:37-74: x [T, N_pad, C] fp32 features (AssembleSamples layout), x_lens [N_pad]
  void update(at::Tensor x, at::Tensor x_lens, int32_t split_len = -1, int32_t actual_batch_size = -1) {
    actual_batch_size_ = actual_batch_size < 0 ? (int32_t)x_lens.size(0) : actual_batch_size;
    if (x_lens.size(0) != batch_size_) init((int32_t)x_lens.size(0), split_len);
    split_len_ = split_len;  // chunking is numerically invariant (decoder.py:80-91): the engine walks all T
    res_.fill_(SOS);
    res_idx_.fill_(-1);
    f_ = x;
    f_lens_ = x_lens.to(at::kInt).contiguous();
    infer_lens_ = f_lens_;
    finish_size_ = batch_size_;
  }
  int32_t finish_size_ = 0;
  int32_t actual_batch_size_ = 0;
  int32_t batch_size_ = 0;
  int32_t split_len_ = -1;
  int32_t padded_fea_len_ = MAX_FEA_LEN;
  int32_t max_res_len_ = MAX_FEA_LEN / 2 * MAX_SYMBOLS_PER_STEP;  // metadata.hpp:58-59
  at::Tensor f_, f_lens_, infer_lens_;
  at::Tensor res_, res_idx_;
};

namespace models {

class TorchModel {
 public:
  // model_file: the engine file (tools/export_model.py --engine-file, rnnt_amd.weights.save_engine_file),
  // one engine per GPU (rnnt_model.hpp:41-47 kept one TorchScript clone per socket)
  TorchModel(const std::string& model_file, int n_gpus = 1, int max_batch = 4096) {
    rnnt_opts opts{max_batch, MAX_FEA_LEN, MAX_FEA_LEN / 2 * MAX_SYMBOLS_PER_STEP};
    gpus_.resize(n_gpus);
    for (int g = 0; g < n_gpus; ++g) {
      Gpu& d = gpus_[g];
      d.max_batch = max_batch;
      check(rnnt_engine_create_from_file(model_file.c_str(), g, &opts, &d.e), "rnnt_engine_create_from_file");
      hcheck(hipSetDevice(g), "hipSetDevice");
      hcheck(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking), "hipStreamCreate");
      const size_t rows = (size_t)round_up(max_batch, 256);
      hcheck(hipMalloc(&d.x, (size_t)MAX_FEA_LEN * rows * PADDED_INPUT_SIZE * sizeof(float)), "hipMalloc x");
      hcheck(hipMalloc(&d.lens, rows * sizeof(int32_t)), "hipMalloc lens");
      hcheck(hipMalloc(&d.res, rows * (size_t)opts.max_res * sizeof(int32_t)), "hipMalloc res");
      hcheck(hipMalloc(&d.res_len, rows * sizeof(int32_t)), "hipMalloc res_len");
    }
  }
  ~TorchModel() {
    for (Gpu& d : gpus_) {
      if (d.stream) (void)hipStreamSynchronize(d.stream);
      for (void* p : {(void*)d.x, (void*)d.lens, (void*)d.res, (void*)d.res_len})
        if (p) (void)hipFree(p);
      if (d.stream) (void)hipStreamDestroy(d.stream);
      rnnt_engine_destroy(d.e);
    }
  }
  TorchModel(const TorchModel&) = delete;
  TorchModel& operator=(const TorchModel&) = delete;

  template <class T>
  void forward(int which, T& state) {  // rnnt_model.hpp:56-60
    encode(which, state);
    decode(which, state);
  }

  // rnnt_model.hpp:62-90: the whole transcription; state.f_lens_ becomes ceil(infer_lens / 2)
  template <class T>
  void encode(int which, T& state) {
    Gpu& d = gpus_.at(which);
    const at::Tensor x = state.f_.to(at::kFloat).contiguous();
    const int64_t Tn = x.size(0), n_rows = x.size(1), C = x.size(2);
    const int n = state.actual_batch_size_;
    if (Tn > MAX_FEA_LEN || n_rows > d.max_batch || C > PADDED_INPUT_SIZE || n > n_rows)
      throw std::runtime_error("TorchModel::encode: batch exceeds the engine (T <= 500, N <= max_batch, C <= 256)");
    const int n_pad = (int)round_up(std::max<int64_t>(n_rows, 1), 256);  // the engine's batch tile
    hcheck(hipSetDevice(which), "hipSetDevice");
    // AssembleSamples' [T][N_pad][C] host batch -> the engine's [T][n_pad][256] device input: zero the
    // whole input (pad rows and channels), then each frame's rows as one 2-D copy
    hcheck(hipMemsetAsync(d.x, 0, (size_t)Tn * n_pad * PADDED_INPUT_SIZE * sizeof(float), d.stream), "memset x");
    for (int64_t t = 0; t < Tn; ++t)
      hcheck(hipMemcpy2DAsync(d.x + (size_t)t * n_pad * PADDED_INPUT_SIZE, PADDED_INPUT_SIZE * sizeof(float),
                              x.data_ptr<float>() + (size_t)t * n_rows * C, C * sizeof(float), C * sizeof(float),
                              (size_t)n_rows, hipMemcpyHostToDevice, d.stream),
             "copy x");
    std::vector<int32_t> lens(n_pad, 0);
    const at::Tensor il = state.infer_lens_.to(at::kInt).contiguous();
    std::memcpy(lens.data(), il.data_ptr<int32_t>(), sizeof(int32_t) * std::min<int64_t>(il.numel(), n_rows));
    hcheck(hipMemcpyAsync(d.lens, lens.data(), sizeof(int32_t) * n_pad, hipMemcpyHostToDevice, d.stream), "copy lens");
    hcheck(hipStreamSynchronize(d.stream), "sync");  // `lens` is a host temporary
    check(rnnt_engine_encode(d.e, d.x, d.lens, lens.data(), (int)Tn, n, n_pad, nullptr, d.stream), "rnnt_engine_encode");
    state.f_lens_ = ((state.infer_lens_ + 1) / STACK_TIME_FACTOR).to(at::kInt);  // ceil(len / 2)
  }

  // rnnt_model.hpp:92-124: the greedy loop; results in the State contract (res_ SOS-filled, res_idx_)
  template <class T>
  void decode(int which, T& state) {
    Gpu& d = gpus_.at(which);
    const int n = state.actual_batch_size_;
    const int max_res = state.max_res_len_;
    hcheck(hipSetDevice(which), "hipSetDevice");
    check(rnnt_engine_decode(d.e, d.res, d.res_len, max_res, d.stream), "rnnt_engine_decode");
    std::vector<int32_t> len(n);
    hcheck(hipMemcpyAsync(len.data(), d.res_len, sizeof(int32_t) * n, hipMemcpyDeviceToHost, d.stream), "copy res_len");
    hcheck(hipStreamSynchronize(d.stream), "sync");
    int32_t widest = 0;
    int32_t* idx = state.res_idx_.template data_ptr<int32_t>();
    for (int i = 0; i < n; ++i) {
      idx[i] = len[i] - 1;  // metadata.cpp:59-60 / torch_sut.cpp:224: response size = (res_idx_ + 1) * 4
      widest = std::max(widest, len[i]);
    }
    if (widest > 0)  // only the written columns travel; the rest of res_ keeps update()'s SOS fill
      hcheck(hipMemcpy2DAsync(state.res_.template data_ptr<int32_t>(), (size_t)state.res_.size(1) * sizeof(int32_t),
                              d.res, (size_t)max_res * sizeof(int32_t), (size_t)widest * sizeof(int32_t), n,
                              hipMemcpyDeviceToHost, d.stream),
             "copy res");
    hcheck(hipStreamSynchronize(d.stream), "sync");
  }

 private:
  static int64_t round_up(int64_t v, int64_t m) { return (v + m - 1) / m * m; }
  struct Gpu {
    rnnt_engine* e = nullptr;
    hipStream_t stream = nullptr;
    int max_batch = 0;
    float* x = nullptr;
    int32_t* lens = nullptr;
    int32_t* res = nullptr;
    int32_t* res_len = nullptr;
  };
  std::vector<Gpu> gpus_;
};

}  // namespace models
}  // namespace rnnt
