// sut_harness.cpp -- drives the TorchModel replacement (rnnt_model_mi355x.hpp) the way the reference's SUT
// drives TorchModel, with the reference's own State protocol (restated in sut_state.hpp), for tests and
// throughput runs.  No LoadGen: "QuerySamplesComplete" writes (query position, bytes, payload) records.
//
// --scenario offline (OfflineSUT, torch_sut.cpp:88-236): the query is sorted longest first
//   (RNNTQuerySampleLibrary::Sort, rnnt_qsl.cpp:104-133); --threads instances, instance `index` calling
//   the model with which = index & 1 (torch_sut.cpp:145), each with its own State(batch, split_len):
//   warm up (dummy N(0,1) batches of MAX_FEA_LEN frames, torch_sut.cpp:124-138), then repeatedly take up
//   to --batch samples off the shared queue under the mutex (:167-182), AssembleSamples into
//   [T][N_pad][256] (rnnt_qsl.cpp:150-188; N_pad a multiple of 32, the intent of torch_sut.cpp:203, whose
//   integer division floors), state.update(x, x_lens, split_len, actual_batch_size), model.encode,
//   model.decode, and answer each sample with (res_[i], (res_idx_[i] + 1) * 4 bytes) (:221-236).
// --scenario server (ServerSUT, torch_sut.cpp:238-571, no audio processor): one producer assembles
//   --pro-batch samples at a time and queues each as ([T][1][256], length) (:436-461); --threads consumers,
//   each with a PipelineState(batch, split_len, response) (:470-540): dequeue up to finish_size_ samples,
//   state.update, model.encode, model.decode, answer every slot with finish_idx_ && F_lens_ > 0 (:542-571).
//
//   rnnt_sut_harness --engine F --feats F --lens F [--query F] [--scenario offline|server] [--threads K]
//                    [--batch B] [--split-len L] [--response R] [--pro-batch P] [--warmup W] [--intra C]
//                    --out F
// --feats: fp32 [sum(lens)][240], the samples' frames back to back; --lens: int32 [N]; --query: int32 QSL
// indices (default 0..N-1).  --pinned 1: each instance assembles its batches into a reused pinned buffer
// (a SUT choice the reference does not make; the model then DMAs the batch as it is instead of packing
// it).  --preassemble 1 (Offline, features): every batch is assembled before the timed region, so the
// line is the model's own rate with the SUT's batches ready.  WAV mode (--processor F --wav F --wav-lens F: fp32 16 kHz audio back to back, int32 samples per
// utterance): AssembleSamples gathers audio and the AudioProcessor drop-in (rnnt_processor_mi355x.hpp)
// featurizes each batch on the GPU before the model, as the SUT does with WAV=true (torch_sut.cpp:192-200,
// 442-461).  Prints one JSON line.
#include <link.h>
#include <limits.h>
#include <stdlib.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <deque>
#include <fstream>
#include <iostream>
#include <list>
#include <map>
#include <numeric>
#include <set>
#include <thread>

#include "rnnt_model_mi355x.hpp"
#include "rnnt_processor_mi355x.hpp"
#include "sut_state.hpp"

namespace {

template <class T>
std::vector<T> read_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary | std::ios::ate);
  if (!f) throw std::runtime_error("cannot open " + path);
  const std::streamsize bytes = f.tellg();
  if (bytes % (std::streamsize)sizeof(T)) throw std::runtime_error("ragged file " + path);
  std::vector<T> v((size_t)bytes / sizeof(T));
  f.seekg(0);
  f.read(reinterpret_cast<char*>(v.data()), bytes);
  if (f.gcount() != bytes) throw std::runtime_error("short read " + path);
  return v;
}

// distinct files mapped as a HIP runtime (two would mean two HIP runtimes: torch's and the system's)
int hip_runtimes() {
  std::set<std::string> files;
  dl_iterate_phdr(
      [](dl_phdr_info* info, size_t, void* p) {
        const char* name = info->dlpi_name;
        if (name && std::strstr(name, "libamdhip64")) {
          char buf[PATH_MAX];
          static_cast<std::set<std::string>*>(p)->insert(realpath(name, buf) ? buf : name);
        }
        return 0;
      },
      &files);
  return (int)files.size();
}

// The QSL: every sample's [len][240] frames in host memory (LoadSamplesToRam).
struct Qsl {
  bool pinned = false;  // assemble into pinned host memory (--pinned 1)
  // WAV mode (--wav / --wav-lens / --processor): each sample's 16 kHz audio back to back
  std::vector<float> wav;
  std::vector<int32_t> wav_lens;
  std::vector<int64_t> wav_first;
  // RNNTQuerySampleLibrary::AssembleSamples, processor mode (rnnt_qsl.cpp:163-179): zeros [N][max len] + audio
  std::pair<at::Tensor, at::Tensor> assemble_wav(const std::vector<int64_t>& idx) const {
    const int64_t n = (int64_t)idx.size();
    int32_t L = 1;
    for (int64_t i : idx) L = std::max(L, wav_lens[i]);
    at::Tensor x = at::zeros({n, L}, at::kFloat);
    at::Tensor xl = at::empty({n}, at::kInt);
    for (int64_t i = 0; i < n; ++i) {
      xl.data_ptr<int32_t>()[i] = wav_lens[idx[i]];
      std::memcpy(x.data_ptr<float>() + i * L, wav.data() + wav_first[idx[i]], sizeof(float) * wav_lens[idx[i]]);
    }
    return {x, xl};
  }
  std::vector<float> feats;
  std::vector<int32_t> lens;
  std::vector<int64_t> first;  // first frame row of each sample
  int max_len = 0;
  at::Tensor sample(int64_t idx) const {  // [len][240] view (x_set_[index])
    return at::from_blob(const_cast<float*>(feats.data()) + first[idx] * rnnt::dims::kInput,
                         {lens[idx], rnnt::dims::kInput}, at::kFloat);
  }
  // RNNTQuerySampleLibrary::AssembleSamples, features mode (rnnt_qsl.cpp:150-188): x [T_max][padded][256]
  // zero except each sample's frames in channels 0..239.  `buf` (optional, per thread) is reused across
  // batches: only what the samples do not overwrite is zeroed, instead of a fresh zero-filled tensor per
  // batch (whose page faults and fill would dominate a large batch's host time)
  std::pair<at::Tensor, at::Tensor> assemble(const std::vector<int64_t>& idx, int64_t padded, at::Tensor* buf = nullptr) const {
    const int64_t n = (int64_t)idx.size();
    constexpr int64_t C = rnnt::dims::kPaddedInput, I = rnnt::dims::kInput;
    int32_t T = 0;
    for (int64_t i : idx) T = std::max(T, lens[i]);
    at::Tensor x;
    if (buf) {
      const int64_t need = (int64_t)T * padded * C;
      if (!buf->defined() || buf->numel() < need) {
        if (pinned) {  // a SUT assembling into pinned memory: the model DMAs the batch as it is
          void* p = nullptr;
          if (hipHostMalloc(&p, (size_t)std::max<int64_t>(need, 1) * sizeof(float), hipHostMallocDefault) != hipSuccess)
            throw std::runtime_error("hipHostMalloc of the assembly buffer failed");
          *buf = at::from_blob(p, {std::max<int64_t>(need, 1)}, [](void* q) { (void)hipHostFree(q); }, at::kFloat);
        } else {
          *buf = at::empty({std::max<int64_t>(need, 1)}, at::kFloat);
        }
      }
      x = buf->narrow(0, 0, need).view({T, padded, C});
    } else {
      x = at::zeros({T, padded, C}, at::kFloat);
    }
    at::Tensor x_lens = at::zeros({padded}, at::kInt);
    float* xp = x.data_ptr<float>();
    int32_t* lp = x_lens.data_ptr<int32_t>();
    for (int64_t i = 0; i < n; ++i) lp[i] = lens[idx[i]];
    // blocks of 32 rows, frames outer (each frame's rows are one contiguous run of x)
    at::parallel_for(0, (padded + 31) / 32, 1, [&](int64_t b, int64_t e) {
      for (int64_t blk = b; blk < e; ++blk) {
        const int64_t i0 = blk * 32, i1 = std::min<int64_t>(padded, i0 + 32);
        for (int32_t t = 0; t < T; ++t) {
          for (int64_t i = i0; i < i1; ++i) {
            const int32_t L = i < n ? lens[idx[i]] : 0;
            float* dst = xp + ((int64_t)t * padded + i) * C;
            if (t < L) {
              std::memcpy(dst, feats.data() + (first[idx[i]] + t) * I, I * sizeof(float));
              if (buf) std::memset(dst + I, 0, (C - I) * sizeof(float));
            } else if (buf) {
              std::memset(dst, 0, C * sizeof(float));
            }
          }
        }
      }
    });
    return {x, x_lens};
  }
};

// "QuerySamplesComplete": records + the State contract per answered row: res_idx_ in range and, for a State
// (Offline), SOS past the row's tokens (update() refills res_ per batch, metadata.cpp:59).  A PipelineState
// only resets res_idx_ when it refills a slot (metadata.cpp:142), so past a Server row's tokens res_ may
// hold the slot's previous utterance, in the reference as here; nothing reads it.
struct Responder {
  bool check_fill = true;
  std::mutex mu;
  std::ofstream out;
  int64_t responses = 0, bad_fill = 0, bad_idx = 0;
  std::chrono::steady_clock::time_point last;
  void complete(const rnnt::Sample& s, const at::Tensor& res_row, int32_t res_len, int32_t max_res) {
    const int32_t* row = res_row.data_ptr<int32_t>();
    int fill_bad = 0;
    for (int32_t j = std::max(res_len, 0); check_fill && j < max_res; ++j)
      if (row[j] != rnnt::dims::kSos) {
        fill_bad = 1;
        break;
      }
    const int32_t id = (int32_t)s.id, size = std::max(res_len, 0) * 4;
    std::lock_guard<std::mutex> l(mu);
    if (res_len < 0 || res_len > max_res) ++bad_idx;
    bad_fill += fill_bad;
    out.write(reinterpret_cast<const char*>(&id), 4);
    out.write(reinterpret_cast<const char*>(&size), 4);
    out.write(reinterpret_cast<const char*>(row), size);
    ++responses;
    last = std::chrono::steady_clock::now();
  }
};

struct Args {
  std::map<std::string, std::string> kv;
  std::string get(const std::string& k, const std::string& d = "") const {
    auto it = kv.find(k);
    return it == kv.end() ? d : it->second;
  }
  int num(const std::string& k, int d) const { return std::atoi(get(k, std::to_string(d)).c_str()); }
};

int usage(const char* argv0) {
  std::fprintf(stderr,
               "usage: %s --engine F --feats F --lens F --out F [--query F] [--scenario offline|server] [--threads K]\n"
               "          [--batch B] [--split-len L] [--response R] [--pro-batch P] [--warmup W] [--intra C] [--progress S]\n"
               "          [--pinned 0|1] [--preassemble 0|1] [--check-fill 0|1]\n"
               "   or (WAV=true) --wav F --wav-lens F --processor F in place of --feats / --lens\n",
               argv0);
  return 2;
}

using Clock = std::chrono::steady_clock;

rnnt::models::AudioProcessor* g_processor = nullptr;  // WAV mode (--processor)

// the first exception of any instance thread, rethrown by main (an escaping one would terminate)
std::mutex g_err_mu;
std::exception_ptr g_err;
bool failed() {
  std::lock_guard<std::mutex> l(g_err_mu);
  return (bool)g_err;
}
template <class F>
void guarded(F f) {
  try {
    f();
  } catch (...) {
    std::lock_guard<std::mutex> l(g_err_mu);
    if (!g_err) g_err = std::current_exception();
  }
}

// OfflineSUT::thInstance (torch_sut.cpp:140-219)
// --preassemble 1: the query's batches assembled before the timed region (instance i assembles batches
// i, i + threads, ...), then taken in order from a shared counter -- what the model sustains when the SUT
// has its batches ready (the harness's own measurement; the reference assembles inside the loop)
struct Preassembled {
  std::vector<std::vector<rnnt::Sample>> samples;
  std::vector<std::pair<at::Tensor, at::Tensor>> batch;
  std::atomic<size_t> next{0};
};

void offline_instance(int index, rnnt::models::TorchModel& model, const Qsl& qsl, std::list<rnnt::Sample>& queue,
                      std::mutex& qmu, Responder& resp, int bs, int split_len, int warmup, int intra,
                      std::atomic<int>& warm, std::atomic<bool>& go, std::atomic<int64_t>& batches,
                      Preassembled* pre, int threads) {
  const int which = index & 1;
  if (intra > 0) at::set_num_threads(intra);  // this instance's team (the reference pins INTRA threads, :143-149)
  at::Tensor xbuf;
  if (pre)
    for (size_t j = (size_t)index; j < pre->samples.size(); j += (size_t)threads) {
      std::vector<int64_t> idx;
      for (const auto& smp : pre->samples[j]) idx.push_back((int64_t)smp.index);
      const int64_t n = (int64_t)idx.size();
      at::Tensor buf;  // a buffer of its own per batch (pinned with --pinned 1)
      pre->batch[j] = qsl.assemble(idx, (n + 31) / 32 * 32, &buf);
    }
  for (int i = 0; i < warmup; ++i) {  // OfflineSUT::warmup (:124-138), GenerateDummySamples (rnnt_qsl.cpp:136-147)
    rnnt::State ws(bs, split_len);
    at::Tensor x, x_lens;
    if (g_processor) {
      at::Tensor w = at::randn({bs, 240000}), wl = at::full({bs}, 240000, at::kInt);  // MAX_WAV_LEN
      std::tie(x, x_lens) = g_processor->forward(which, w, wl, /*pad_batch_size=*/true);
      x = x.permute({2, 0, 1}).contiguous();
    } else {
      x = at::randn({bs, rnnt::dims::kPaddedInput, rnnt::dims::kMaxFeaLen}).permute({2, 0, 1}).contiguous();
      x_lens = at::full({bs}, rnnt::dims::kMaxFeaLen, at::kInt);
    }
    ws.update(x, x_lens, split_len);
    model.forward(which, ws);
  }
  warm++;
  while (!go) std::this_thread::yield();
  rnnt::State state(bs, split_len);
  while (true) {
    std::vector<rnnt::Sample> samples;
    if (pre) {
      const size_t j = pre->next++;
      if (j >= pre->samples.size()) break;
      samples = pre->samples[j];
      const int n = (int)samples.size();
      at::Tensor x = pre->batch[j].first, x_lens = pre->batch[j].second;
      state.update(x, x_lens, split_len, n);
      model.encode(which, state);
      model.decode(which, state);
      const at::Tensor res_lens = state.res_idx_ + 1;
      for (int i = 0; i < n; ++i)
        resp.complete(samples[i], state.res_[i], res_lens.data_ptr<int32_t>()[i], state.max_res_len_);
      // (the batch's memory is kept until the run ends: freeing pinned memory synchronises the device)
      batches++;
      continue;
    }
    {
      std::lock_guard<std::mutex> l(qmu);
      if (queue.empty()) break;
      const size_t k = std::min(queue.size(), (size_t)bs);
      auto it = queue.begin();
      std::advance(it, k);
      samples.assign(queue.begin(), it);
      queue.erase(queue.begin(), it);
    }
    std::vector<int64_t> idx(samples.size());
    for (size_t i = 0; i < samples.size(); ++i) idx[i] = (int64_t)samples[i].index;
    const int n = (int)samples.size();
    at::Tensor x, x_lens;
    if (g_processor) {  // torch_sut.cpp:192-200: AssembleSamples (audio), processor, permute to [T][N][C]
      auto [w, wl] = qsl.assemble_wav(idx);
      std::tie(x, x_lens) = g_processor->forward(which, w, wl, /*pad_batch_size=*/true);
      x = x.permute({2, 0, 1}).contiguous();
    } else {
      std::tie(x, x_lens) = qsl.assemble(idx, (n + 31) / 32 * 32, &xbuf);
    }
    state.update(x, x_lens, split_len, n);
    model.encode(which, state);
    model.decode(which, state);
    const at::Tensor res_lens = state.res_idx_ + 1;
    for (int i = 0; i < n; ++i)
      resp.complete(samples[i], state.res_[i], res_lens.data_ptr<int32_t>()[i], state.max_res_len_);
    batches++;
  }
}

// ServerSUT::thConsumer (torch_sut.cpp:470-540) and QuerySamplesComplete (:542-571)
void server_consumer(int index, rnnt::models::TorchModel& model, std::deque<rnnt::PipelineState::Entry>& processed,
                     std::mutex& pmu, std::atomic<bool>& produced, Responder& resp, int bs, int split_len,
                     int response, int warmup, int intra, std::atomic<int>& warm, std::atomic<bool>& go,
                     std::atomic<int64_t>& batches) {
  const int which = index & 1;
  if (intra > 0) at::set_num_threads(intra);
  for (int i = 0; i < warmup; ++i) {  // ServerSUT::warmup, consumer (:341-346)
    rnnt::State ws(bs, split_len);
    at::Tensor x = at::randn({bs, rnnt::dims::kPaddedInput, rnnt::dims::kMaxFeaLen}).permute({2, 0, 1}).contiguous();
    ws.update(x, at::full({bs}, rnnt::dims::kMaxFeaLen, at::kInt), split_len);
    model.forward(which, ws);
  }
  warm++;
  while (!go) std::this_thread::yield();
  std::vector<rnnt::Sample> samples(bs);
  rnnt::PipelineState state(bs, split_len, response);
  while (true) {
    std::vector<rnnt::PipelineState::Entry> dq;
    int32_t dequeue_size = 0;
    bool finish_dequeue = false;
    while (!finish_dequeue && dequeue_size == 0 && state.finish_size_ != 0) {
      {
        std::lock_guard<std::mutex> l(pmu);
        if (produced && processed.empty()) {  // no new samples left
          finish_dequeue = true;
          break;
        }
        while (!processed.empty() && dequeue_size < state.finish_size_) {  // wait_dequeue_bulk_timed(.., 0)
          dq.push_back(std::move(processed.front()));
          processed.pop_front();
          ++dequeue_size;
        }
      }
      if (state.remain_size_ != 0) break;
      if (dequeue_size == 0) std::this_thread::yield();
    }
    if (finish_dequeue && state.remain_size_ == 0) break;
    state.update(dq, samples, dequeue_size, split_len);
    model.encode(which, state);
    model.decode(which, state);
    const at::Tensor res_lens = state.res_idx_ + 1;
    const bool* fin = state.finish_idx_.data_ptr<bool>();
    const int32_t* Fl = state.F_lens_.data_ptr<int32_t>();
    for (int i = 0; i < bs; ++i)
      if (fin[i] && Fl[i] > 0) resp.complete(samples[i], state.res_[i], res_lens.data_ptr<int32_t>()[i], state.max_res_len_);
    batches++;
  }
}

}  // namespace

int main(int argc, char** argv) {
  if (hip_runtimes() != 1) {
    std::fprintf(stderr, "rnnt_sut_harness: %d HIP runtimes mapped (expected torch's only)\n", hip_runtimes());
    return 3;
  }
  Args a;
  for (int i = 1; i < argc; ++i) {
    const std::string k = argv[i];
    if (k.rfind("--", 0) != 0 || i + 1 >= argc) return usage(argv[0]);
    a.kv[k.substr(2)] = argv[++i];
  }
  const bool wav_mode = !a.get("processor").empty();
  if (a.get("engine").empty() || a.get("out").empty() ||
      (wav_mode ? a.get("wav").empty() || a.get("wav-lens").empty() : a.get("feats").empty() || a.get("lens").empty()))
    return usage(argv[0]);
  try {
    const std::string scenario = a.get("scenario", "offline");
    const int threads = a.num("threads", 1), bs = a.num("batch", 256), split_len = a.num("split-len", -1);
    const int warmup = a.num("warmup", 0), intra = a.num("intra", 0);
    if (threads <= 0 || bs <= 0 || (scenario != "offline" && scenario != "server")) return usage(argv[0]);
    if (intra > 0) at::set_num_threads(intra);
    Qsl qsl;
    qsl.pinned = a.num("pinned", 0) != 0;
    const bool check_fill = a.num("check-fill", 1) != 0;  // 0: throughput lines skip the per-row SOS scan
    if (wav_mode) {  // the sort key is the feature length the processor will produce
      qsl.wav_lens = read_file<int32_t>(a.get("wav-lens"));
      qsl.wav = read_file<float>(a.get("wav"));
      int64_t at_ = 0;
      for (int32_t l : qsl.wav_lens) {
        if (l < 0) throw std::runtime_error("sample length out of range");
        qsl.wav_first.push_back(at_);
        at_ += l;
        qsl.lens.push_back((int32_t)rnnt_featurizer_frames(l));
        qsl.first.push_back(0);
      }
      if ((int64_t)qsl.wav.size() != at_) throw std::runtime_error("wav does not match wav-lens");
    } else {
      qsl.lens = read_file<int32_t>(a.get("lens"));
      qsl.feats = read_file<float>(a.get("feats"));
      int64_t rows = 0;
      for (int32_t l : qsl.lens) {
        if (l < 0 || l > rnnt::dims::kMaxFeaLen) throw std::runtime_error("sample length out of range");
        qsl.first.push_back(rows);
        rows += l;
        qsl.max_len = std::max(qsl.max_len, l);
      }
      if ((int64_t)qsl.feats.size() != rows * rnnt::dims::kInput) throw std::runtime_error("feats do not match lens");
    }
    std::vector<int32_t> query;
    if (!a.get("query").empty()) {
      query = read_file<int32_t>(a.get("query"));
    } else {
      query.resize(qsl.lens.size());
      std::iota(query.begin(), query.end(), 0);
    }
    for (int32_t q : query)
      if (q < 0 || q >= (int32_t)qsl.lens.size()) throw std::runtime_error("query index out of range");

    rnnt::models::TorchModel model(a.get("engine"));
    std::unique_ptr<rnnt::models::AudioProcessor> processor;
    if (wav_mode) {
      processor = std::make_unique<rnnt::models::AudioProcessor>(a.get("processor"));
      g_processor = processor.get();
    }
    Responder resp;
    resp.check_fill = check_fill;
    // progress on stderr every --progress seconds (a long run stays visibly alive)
    const int progress = a.num("progress", 10);
    std::atomic<bool> done{false};
    const Clock::time_point t_start = Clock::now();
    std::thread monitor([&] {
      auto next = t_start;
      while (!done) {
        std::this_thread::sleep_for(std::chrono::milliseconds(100));
        if (progress <= 0 || Clock::now() < next) continue;
        next += std::chrono::seconds(progress);
        int64_t n;
        {
          std::lock_guard<std::mutex> l(resp.mu);
          n = resp.responses;
        }
        const auto cs = model.stats();
        std::fprintf(stderr, "[harness %.0f s] responses %lld, encode calls %lld (pack %.1f s, copy %.1f s, turn wait %.1f s, "
                     "encode %.1f s, decode %.1f s)\n", std::chrono::duration<double>(Clock::now() - t_start).count(),
                     (long long)n, (long long)cs.calls, cs.pack, cs.copy, cs.turn_wait, cs.encode, cs.decode);
      }
    });
    struct Join {
      std::atomic<bool>& d;
      std::thread& t;
      ~Join() {
        d = true;
        t.join();
      }
    } join_monitor{done, monitor};
    resp.out.open(a.get("out"), std::ios::binary);
    std::atomic<int> warm{0};
    std::atomic<bool> go{false};
    std::atomic<int64_t> batches{0};
    std::vector<std::thread> th;
    Clock::time_point t0;
    if (scenario == "offline") {
      // IssueQuery: Sort longest first (stable within a length)
      std::vector<rnnt::Sample> s(query.size());
      for (size_t i = 0; i < query.size(); ++i) s[i] = {(uint64_t)i, (uint64_t)query[i]};
      std::stable_sort(s.begin(), s.end(), [&](const rnnt::Sample& x, const rnnt::Sample& y) {
        return qsl.lens[x.index] > qsl.lens[y.index];
      });
      std::list<rnnt::Sample> queue(s.begin(), s.end());
      std::mutex qmu;
      std::unique_ptr<Preassembled> pre;
      if (a.num("preassemble", 0) != 0) {
        if (wav_mode) throw std::runtime_error("--preassemble is for feature input");
        pre = std::make_unique<Preassembled>();
        for (size_t b = 0; b < s.size(); b += (size_t)bs)
          pre->samples.emplace_back(s.begin() + (long)b, s.begin() + (long)std::min(s.size(), b + (size_t)bs));
        pre->batch.resize(pre->samples.size());
      }
      for (int i = 0; i < threads; ++i)
        th.emplace_back([&, i] {
          guarded([&] {
            offline_instance(i, model, qsl, queue, qmu, resp, bs, split_len, warmup, intra, warm, go, batches, pre.get(),
                             threads);
          });
        });
      while (warm < threads && !failed()) std::this_thread::sleep_for(std::chrono::milliseconds(1));
      model.stats(/*reset=*/true);  // the warmups' calls are not counted
      t0 = Clock::now();
      go = true;
      for (auto& t : th) t.join();
    } else {
      const int response = a.num("response", bs), pro_bs = a.num("pro-batch", 4);
      resp.check_fill = false;
      std::deque<rnnt::PipelineState::Entry> processed;
      std::mutex pmu;
      std::atomic<bool> produced{false};
      for (int i = 0; i < threads; ++i)
        th.emplace_back([&, i] {
          guarded([&] {
            server_consumer(i, model, processed, pmu, produced, resp, bs, split_len, response, warmup, intra, warm,
                            go, batches);
          });
        });
      while (warm < threads && !failed()) std::this_thread::sleep_for(std::chrono::milliseconds(1));
      model.stats(/*reset=*/true);  // the warmups' calls are not counted
      t0 = Clock::now();
      go = true;
      // ServerSUT::thProducer without the audio processor (:436-461): samples in arrival order
      for (size_t s0 = 0; s0 < query.size(); s0 += (size_t)pro_bs) {
        const size_t n = std::min(query.size() - s0, (size_t)pro_bs);
        std::vector<int64_t> idx(n);
        for (size_t i = 0; i < n; ++i) idx[i] = query[s0 + i];
        std::vector<rnnt::PipelineState::Entry> items;
        if (g_processor) {  // :442-461 with the processor: [N][C][T] features, one sample at a time as [T][1][C]
          auto [w, wl] = qsl.assemble_wav(idx);
          auto [f, fl] = g_processor->forward(0, w, wl, /*pad_batch_size=*/false);
          for (size_t i = 0; i < n; ++i)
            items.emplace_back(rnnt::Sample{(uint64_t)(s0 + i), (uint64_t)idx[i]},
                               f.narrow(0, (int64_t)i, 1).permute({2, 0, 1}).contiguous(), fl.narrow(0, (int64_t)i, 1).clone());
        } else {
          auto [x, x_lens] = qsl.assemble(idx, (int64_t)n);
          for (size_t i = 0; i < n; ++i)
            items.emplace_back(rnnt::Sample{(uint64_t)(s0 + i), (uint64_t)idx[i]},
                               x.narrow(1, (int64_t)i, 1).contiguous(), x_lens.narrow(0, (int64_t)i, 1).clone());
        }
        std::lock_guard<std::mutex> l(pmu);
        for (auto& it : items) processed.push_back(std::move(it));
      }
      produced = true;
      for (auto& t : th) t.join();
    }
    if (g_err) std::rethrow_exception(g_err);
    const double secs = std::chrono::duration<double>(resp.last - t0).count();
    const auto per_gpu = model.engines_per_gpu();
    std::cout << "{\"scenario\": \"" << scenario << "\", \"threads\": " << threads << ", \"batch\": " << bs
              << ", \"split_len\": " << split_len << ", \"batches\": " << batches.load() << ", \"responses\": "
              << resp.responses << ", \"bad_sos_fill_rows\": " << resp.bad_fill << ", \"bad_res_idx_rows\": "
              << resp.bad_idx << ", \"seconds\": " << secs << ", \"samples_per_s\": "
              << (secs > 0 ? (double)resp.responses / secs : 0.0) << ", \"engines_per_gpu\": [";
    for (size_t i = 0; i < per_gpu.size(); ++i) std::cout << (i ? ", " : "") << per_gpu[i];
    const auto cs = model.stats();
    std::cout << "], \"model_host_seconds\": {\"pack\": " << cs.pack << ", \"copy\": " << cs.copy
              << ", \"turn_wait\": " << cs.turn_wait << ", \"encode\": " << cs.encode << ", \"decode\": " << cs.decode
              << ", \"encode_calls\": " << cs.calls << ", \"dense_pinned_calls\": " << cs.dense_calls
              << ", \"frames\": " << cs.frames << "}, \"pinned_assembly\": " << (qsl.pinned ? "true" : "false")
              << ", \"preassembled\": " << (a.num("preassemble", 0) != 0 ? "true" : "false")
              << ", \"sos_fill_checked\": " << (resp.check_fill ? "true" : "false") << "}"
              << std::endl;
    return 0;
  } catch (const std::exception& ex) {
    std::fprintf(stderr, "rnnt_sut_harness: %s\n", ex.what());
    return 1;
  }
}
