// sut_harness.cpp -- runs the TorchModel replacement (rnnt_model_mi355x.hpp) the way the reference's
// OfflineSUT::thInstance runs TorchModel (csrc/torch_sut.cpp:140-236), for a test to check:
//   sort the samples longest first (RNNTQuerySampleLibrary::Sort, rnnt_qsl.cpp:104-133), take up to
//   batch_size of them, AssembleSamples into [T_max][N_pad][256] zero-padded fp32 (rnnt_qsl.cpp:150-188,
//   N_pad a multiple of 32 -- the intent of torch_sut.cpp:203, whose integer division floors),
//   state.update(x, x_lens, split_len, actual_batch_size) -> model.encode(which, state) ->
//   model.decode(which, state) -> QuerySamplesComplete: per sample the response is
//   (state.res_[i].data_ptr(), (res_idx_[i] + 1) * 4 bytes) (torch_sut.cpp:221-236).
// No LoadGen here: the "completion" writes (sample index, bytes, payload) records to out_file, and the
// State contract is checked per row (res_idx_ = length - 1, SOS (-1) in every column past it).
//
//   rnnt_sut_harness <engine_file> <feats.bin fp32 [N][T_max][240]> <lens.bin int32 [N]> <N> <T_max>
//                    <batch_size> <out_file>
// Prints one JSON line: batches, responses, rows whose res_ fill or res_idx_ broke the contract.
#include <link.h>
#include <limits.h>
#include <stdlib.h>

#include <cstdio>
#include <fstream>
#include <set>
#include <iostream>
#include <numeric>

#include "rnnt_model_mi355x.hpp"

namespace {
template <class T>
std::vector<T> read_file(const char* path, size_t count) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error(std::string("cannot open ") + path);
  std::vector<T> v(count);
  f.read(reinterpret_cast<char*>(v.data()), (std::streamsize)(count * sizeof(T)));
  if ((size_t)f.gcount() != count * sizeof(T)) throw std::runtime_error(std::string("short file ") + path);
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
}  // namespace

int main(int argc, char** argv) {
  if (hip_runtimes() != 1) {
    std::fprintf(stderr, "rnnt_sut_harness: %d HIP runtimes mapped (expected torch's only)\n", hip_runtimes());
    return 3;
  }
  if (argc != 8) {
    std::fprintf(stderr, "usage: %s engine_file feats.bin lens.bin N T_max batch_size out_file\n", argv[0]);
    return 2;
  }
  try {
    const int N = std::atoi(argv[4]), T_max = std::atoi(argv[5]), bs = std::atoi(argv[6]);
    if (N <= 0 || T_max <= 0 || T_max > rnnt::MAX_FEA_LEN || bs <= 0) throw std::runtime_error("bad N / T_max / batch_size");
    const std::vector<float> feats = read_file<float>(argv[2], (size_t)N * T_max * 240);
    const std::vector<int32_t> lens = read_file<int32_t>(argv[3], (size_t)N);
    for (int32_t l : lens)
      if (l < 0 || l > T_max) throw std::runtime_error("sample length out of range");
    rnnt::models::TorchModel model(argv[1], /*n_gpus=*/1, /*max_batch=*/(bs + 255) / 256 * 256);
    // Sort: longest first, stable (rnnt_qsl.cpp:104-133 buckets by length)
    std::vector<int> order(N);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return lens[a] > lens[b]; });
    std::ofstream out(argv[7], std::ios::binary);
    rnnt::State state(bs);
    int batches = 0, responses = 0, bad_fill = 0, bad_idx = 0;
    for (int s0 = 0; s0 < N; s0 += bs) {
      const int n = std::min(bs, N - s0);
      const int n_pad = (n + 31) / 32 * 32;
      int t_b = 0;
      for (int i = 0; i < n; ++i) t_b = std::max(t_b, lens[order[s0 + i]]);
      t_b = std::max(t_b, 1);
      at::Tensor x = at::zeros({t_b, n_pad, rnnt::PADDED_INPUT_SIZE}, at::kFloat);  // AssembleSamples
      at::Tensor x_lens = at::zeros({n_pad}, at::kInt);
      float* xp = x.data_ptr<float>();
      for (int i = 0; i < n; ++i) {
        const int s = order[s0 + i];
        x_lens.data_ptr<int32_t>()[i] = lens[s];
        for (int t = 0; t < lens[s]; ++t)
          std::memcpy(xp + ((size_t)t * n_pad + i) * rnnt::PADDED_INPUT_SIZE, &feats[((size_t)s * T_max + t) * 240],
                      240 * sizeof(float));
      }
      state.update(x, x_lens, /*split_len=*/-1, n);
      model.encode(0, state);
      model.decode(0, state);
      // QuerySamplesComplete (torch_sut.cpp:221-236)
      const at::Tensor res_lens = state.res_idx_ + 1;
      for (int i = 0; i < n; ++i) {
        const int32_t res_len = res_lens[i].item().toInt();
        const int32_t* row = state.res_[i].data_ptr<int32_t>();
        const int32_t size = res_len * 4;
        if (res_len < 0 || res_len > state.max_res_len_) ++bad_idx;
        for (int j = std::max(res_len, 0); j < state.max_res_len_; ++j)
          if (row[j] != rnnt::SOS) {
            ++bad_fill;
            break;
          }
        const int32_t sid = order[s0 + i];
        out.write(reinterpret_cast<const char*>(&sid), 4);
        out.write(reinterpret_cast<const char*>(&size), 4);
        out.write(reinterpret_cast<const char*>(row), size);
        ++responses;
      }
      ++batches;
    }
    std::cout << "{\"batches\": " << batches << ", \"responses\": " << responses << ", \"bad_sos_fill_rows\": "
              << bad_fill << ", \"bad_res_idx_rows\": " << bad_idx << "}" << std::endl;
    return 0;
  } catch (const std::exception& ex) {
    std::fprintf(stderr, "rnnt_sut_harness: %s\n", ex.what());
    return 1;
  }
}
