// sut_state.hpp -- the SUT-side batch state the reference's model driver is handed, restated for the
// harness (test infrastructure, not part of the drop-in): rnnt::State (Offline, metadata.hpp:37-81,
// metadata.cpp:5-95) and rnnt::PipelineState (Server slot refill, metadata.hpp:84-114,
// metadata.cpp:97-194), with the members, their dtypes and the update() / next() protocol the reference
// SUT and TorchModel use.  In the reference build these classes come from metadata.hpp and
// rnnt_model_mi355x.hpp is compiled against them unchanged; restating them here lets the harness drive
// the model through exactly that protocol (split_len chunking, slot refill) without LoadGen.
#pragma once
#include <ATen/ATen.h>
#include <ATen/Parallel.h>

#include <algorithm>
#include <cstdint>
#include <tuple>
#include <vector>

namespace rnnt {

namespace dims {  // metadata.hpp:19-34
constexpr int32_t kPreLayers = 2, kPostLayers = 3, kHidden = 1024, kPredLayers = 2, kPredHidden = 320;
constexpr int32_t kSos = -1, kMaxSymbols = 30, kMaxFeaLen = 500, kPaddedInput = 256, kInput = 240;
}  // namespace dims

struct Sample {  // mlperf::QuerySample
  uint64_t id;
  uint64_t index;
};

class State {
 public:
  State() = default;
  State(int32_t batch_size, int32_t split_len = -1) {
    init(batch_size, split_len);
    const int32_t block = at::get_num_threads() * 16;  // metadata.hpp:43 (integer division, as there)
    padded_batch_size_ = batch_size_ / block * block;
  }
  virtual ~State() = default;

  // metadata.cpp:5-35: allocate per batch size (contents undefined until update)
  void init(int32_t batch_size, int32_t split_len = -1) {
    clear();
    batch_size_ = batch_size;
    split_len_ = split_len;
    if (split_len_ > 0) split_lens_ = at::full({batch_size_}, split_len_, at::kInt);
    for (int32_t l = 0; l < dims::kPreLayers; ++l) {
      pre_hx_.push_back(at::empty({batch_size_, dims::kHidden}, at::kChar));
      pre_cx_.push_back(at::empty({batch_size_, dims::kHidden}, at::kHalf));
    }
    for (int32_t l = 0; l < dims::kPostLayers; ++l) {
      post_hx_.push_back(at::empty({batch_size_, dims::kHidden}, at::kChar));
      post_cx_.push_back(at::empty({batch_size_, dims::kHidden}, at::kHalf));
    }
    pre_g_ = at::full({1, batch_size_}, dims::kSos, at::kInt);
    for (int32_t l = 0; l < dims::kPredLayers; ++l) {
      pre_hg_.push_back(at::empty({batch_size_, dims::kPredHidden}, at::kBFloat16));
      pre_cg_.push_back(at::empty({batch_size_, dims::kPredHidden}, at::kFloat));
    }
    res_ = at::empty({batch_size_, max_res_len_}, at::kInt);
    res_idx_ = at::empty({batch_size_}, at::kInt);
  }

  // metadata.cpp:37-74: a new batch; re-allocates when the padded batch changes size.  Whole-batch
  // mode hands f over at once; split mode cuts it along time into split_len_-frame views for next().
  void update(at::Tensor x, at::Tensor x_lens, int32_t split_len = -1, int32_t actual_batch_size = -1) {
    actual_batch_size_ = actual_batch_size;
    if (x_lens.size(0) != batch_size_) init((int32_t)x_lens.size(0), split_len);
    for (auto* v : {&pre_hx_, &pre_cx_, &post_hx_, &post_cx_})
      for (auto& t : *v) t.zero_();
    pre_g_.fill_(dims::kSos);
    for (auto* v : {&pre_hg_, &pre_cg_})
      for (auto& t : *v) t.zero_();
    res_.fill_(dims::kSos);
    res_idx_.fill_(-1);
    if (split_len_ <= 0) {
      f_ = x;
      f_lens_ = x_lens;
      infer_lens_ = x_lens;
      finish_size_ = batch_size_;
      return;
    }
    f_split_ = at::split(x, split_len_);
    infer_lens_ = x_lens;
    remain_lens_ = x_lens.clone();
    split_idx_ = 0;
    finish_size_ = 0;
  }

  // metadata.cpp:76-86: the next time chunk while some row has frames left
  bool next() {
    if (finish_size_ == batch_size_) return false;
    f_lens_ = at::min(split_lens_, remain_lens_);
    f_ = f_split_[split_idx_++];
    remain_lens_ -= f_lens_;
    finish_idx_ = remain_lens_.le(0);
    finish_size_ = (int32_t)finish_idx_.count_nonzero().item<int64_t>();
    return true;
  }

  void clear() {  // metadata.cpp:88-95
    for (auto* v : {&pre_hx_, &pre_cx_, &post_hx_, &post_cx_, &pre_hg_, &pre_cg_}) v->clear();
  }

  int32_t finish_size_ = 0;
  int32_t actual_batch_size_ = 0;
  int32_t padded_batch_size_ = 0;
  int32_t batch_size_ = 0;
  int32_t split_len_ = -1;
  int32_t padded_fea_len_ = dims::kMaxFeaLen;
  int32_t max_res_len_ = padded_fea_len_ / 2 * dims::kMaxSymbols;
  at::Tensor split_lens_;
  std::vector<at::Tensor> f_split_;
  at::Tensor f_, f_lens_;
  std::vector<at::Tensor> pre_hx_, pre_cx_, post_hx_, post_cx_;
  at::Tensor pre_g_;
  std::vector<at::Tensor> pre_hg_, pre_cg_;
  at::Tensor res_, res_idx_;
  at::Tensor finish_idx_, remain_lens_, infer_lens_;
  int32_t split_idx_ = 0;
};

// Server: batch_size_ slots; finished slots are refilled from the dequeued samples, unfinished ones
// continue where the last call stopped.  Like the reference, it redeclares finish_size_ (and an unused
// tensor split_idx_), hiding State's.
class PipelineState : public State {
 public:
  using Entry = std::tuple<Sample, at::Tensor, at::Tensor>;  // (sample, features [T][1][256], length [1])
  PipelineState(int32_t batch_size, int32_t split_len, int32_t response_size)
      : finish_size_(batch_size), response_size_(response_size) {
    init(batch_size, split_len);
    const int32_t block = at::get_num_threads() * 16;
    padded_batch_size_ = batch_size_ / block * block;
  }

  // metadata.cpp:97-109: T padded to a whole number of chunks, the result rows sized to match
  void init(int32_t batch_size, int32_t split_len = -1) {
    if (split_len > 0) {
      padded_fea_len_ = (dims::kMaxFeaLen + split_len - 1) / split_len * split_len;
      max_res_len_ = padded_fea_len_ / 2 * dims::kMaxSymbols;
    }
    State::init(batch_size, split_len);
    F_ = at::empty({padded_fea_len_, batch_size_, dims::kPaddedInput}, at::kFloat);
    F_lens_ = at::empty({batch_size_}, at::kInt);
    infer_lens_ = at::empty({batch_size_}, at::kInt);
    remain_lens_ = at::zeros({batch_size_}, at::kInt);
    finish_idx_ = at::full({batch_size_}, true, at::kBool);
  }

  // metadata.cpp:111-169: restart the finished slots' state, place the dequeued samples in them
  void update(std::vector<Entry>& dequeued, std::vector<Sample>& samples, int32_t dequeue_size, int32_t split_len) {
    (void)split_len;  // fixed at construction, as in the reference
    dequeue_size_ = dequeue_size;
    const bool* fin = finish_idx_.data_ptr<bool>();
    if (dequeue_size_ != 0) {
      for (int32_t i = 0; i < batch_size_; ++i) {
        if (!fin[i]) continue;
        for (auto* v : {&pre_hx_, &pre_cx_, &post_hx_, &post_cx_, &pre_hg_, &pre_cg_})
          for (auto& t : *v) t[i].zero_();
        pre_g_[0][i] = dims::kSos;
        res_idx_[i] = -1;
      }
    }
    int32_t* Fl = F_lens_.data_ptr<int32_t>();
    int32_t* rem = remain_lens_.data_ptr<int32_t>();
    for (int32_t i = 0; i < batch_size_; ++i)
      if (fin[i]) Fl[i] = 0;
    for (int32_t i = 0, j = 0; i < batch_size_ && j < dequeue_size; ++i) {
      if (!fin[i]) continue;
      const at::Tensor& f = std::get<1>(dequeued[j]);
      const int32_t len = (int32_t)std::get<2>(dequeued[j]).item<int64_t>();
      Fl[i] = len;
      rem[i] = len;
      if (len > 0) F_.narrow(0, 0, len).select(1, i).copy_(f.narrow(0, 0, len).reshape({len, -1}));
      samples[i] = std::get<0>(dequeued[j]);
      ++j;
    }
    padded_size_ = batch_size_ - remain_size_ - dequeue_size;
    if (split_len_ > 0) {
      infer_lens_.zero_();
      finish_size_ = padded_size_;
      stop_size_ = std::min(batch_size_, padded_size_ + response_size_);
    } else {
      f_ = F_;
      f_lens_ = F_lens_;
      infer_lens_ = F_lens_;
      finish_idx_.fill_(true);
      finish_size_ = batch_size_;
    }
  }

  // metadata.cpp:171-194: the next split_len frames of every slot (from where it stopped), until enough
  // slots have finished for a response
  bool next() {
    if (finish_size_ >= stop_size_) {
      remain_size_ = batch_size_ - finish_size_;
      return false;
    }
    f_lens_ = at::min(split_lens_, remain_lens_);
    const int32_t* rem = remain_lens_.data_ptr<int32_t>();
    const int32_t* Fl = F_lens_.data_ptr<int32_t>();
    std::vector<at::Tensor> cols;
    cols.reserve(batch_size_);
    for (int32_t i = 0; i < batch_size_; ++i) {
      const int64_t begin = rem[i] == 0 ? 0 : (int64_t)(Fl[i] - rem[i]);
      cols.push_back(F_.narrow(0, begin, split_len_).select(1, i));
    }
    f_ = at::stack(cols, 1);
    remain_lens_ -= f_lens_;
    infer_lens_ += f_lens_;
    finish_idx_ = remain_lens_.le(0);
    finish_size_ = (int32_t)finish_idx_.count_nonzero().item<int64_t>();
    return true;
  }

  int32_t finish_size_;
  int32_t response_size_;
  int32_t stop_size_ = 0;
  int32_t remain_size_ = 0;
  int32_t dequeue_size_ = 0;
  int32_t padded_size_ = 0;
  at::Tensor F_, F_lens_;
  at::Tensor split_idx_, eos_idx_;
};

}  // namespace rnnt
