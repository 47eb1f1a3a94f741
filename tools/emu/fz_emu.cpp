// fz_emu.cpp -- runs the featurizer's kernels (featurizer.hip: fz_plan, fz_logmel, fz_norm through
// the real rnnt_featurizer_create / rnnt_featurizer_run) on the host emulation of the wave model
// (emu_hip.hpp), with every __shared__ array of fz_logmel_kernel filled with a chosen poison
// pattern when each workgroup starts (EMU_POISON=nan|big|zero|rand).  A kernel that reads an LDS
// word its workgroup has not written produces output that depends on the poison, so two runs with
// different poisons must agree bit for bit; ASan flags any out-of-bounds global access.  Lanes of
// a wave only meet at explicit wave / workgroup barriers here (no implicit lockstep), so a hand-off
// between lanes that relies on lockstep instead of wave_lds_sync also shows up as a difference
// from the float64 restatement (tools/emu/fz_emu_check.py).
// Built by tools/emu/build_fz.sh.  Usage: fz_emu <input.bin> <output.bin>
//   input:  int32 n, int32 n_pad, int32 T_out, float window[320], float fb[80*257], int32 lens[n],
//           float wav[n][max_len] (rows zero padded to max_len = max(lens))
//   output: int32 feat_lens[n_pad], float feats[T_out][n_pad][256]
#include "emu_hip.hpp"

#include <random>
#include <string>
#include <vector>

// the featurizer's kernels see these (emu_fz_poison is called by lane 0 of every fz_logmel
// workgroup before any lane touches LDS: fibers start in lane order and only yield at barriers)
static int g_poison_mode = 0;
static unsigned g_poison_seed = 1;
static void emu_fz_poison(void* p, size_t bytes) {
  uint32_t* w = (uint32_t*)p;
  const size_t n = bytes / 4;
  std::mt19937 rng(g_poison_seed++);
  for (size_t i = 0; i < n; ++i) {
    switch (g_poison_mode) {
      case 0: w[i] = 0x7fc00000u | (rng() & 0x3fffff); break;       // quiet NaNs
      case 1: w[i] = 0x7e967699u; break;                              // 1e38
      case 2: w[i] = 0u; break;                                       // zeros
      default: w[i] = rng(); break;                                   // random bits
    }
  }
}

#include "featurizer_emu.hip.cpp"

int rnnt_internal_fail(int code, const std::string& msg) {
  fprintf(stderr, "featurizer error %d: %s\n", code, msg.c_str());
  return code;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: fz_emu input.bin output.bin\n");
    return 2;
  }
  const char* pm = getenv("EMU_POISON");
  const std::string mode = pm ? pm : "nan";
  g_poison_mode = mode == "nan" ? 0 : mode == "big" ? 1 : mode == "zero" ? 2 : 3;
  FILE* fi = fopen(argv[1], "rb");
  if (!fi) return 2;
  int hdr[3];
  if (fread(hdr, 4, 3, fi) != 3) return 2;
  const int n = hdr[0], n_pad = hdr[1], T_out = hdr[2];
  std::vector<float> window(320), fb(80 * 257);
  std::vector<int32_t> lens(n);
  if (fread(window.data(), 4, 320, fi) != 320 || fread(fb.data(), 4, fb.size(), fi) != fb.size() ||
      fread(lens.data(), 4, n, fi) != (size_t)n)
    return 2;
  int maxl = 1;
  for (int v : lens) maxl = std::max(maxl, v);
  // exact-size "device" buffers: ASan flags any access past them
  float* wav = (float*)malloc((size_t)n * maxl * 4);
  if (fread(wav, 4, (size_t)n * maxl, fi) != (size_t)n * maxl) return 2;
  fclose(fi);
  int32_t* d_lens = (int32_t*)malloc((size_t)n * 4);
  memcpy(d_lens, lens.data(), (size_t)n * 4);
  float* feats = (float*)malloc((size_t)T_out * n_pad * 256 * 4);
  memset(feats, 0xA5, (size_t)T_out * n_pad * 256 * 4);  // the kernels must write every element
  int32_t* flen = (int32_t*)malloc((size_t)n_pad * 4);
  rnnt_featurizer_config cfg{};
  cfg.sample_rate = 16000;
  cfg.n_fft = 512;
  cfg.win_length = 320;
  cfg.hop_length = 160;
  cfg.nfilt = 80;
  cfg.frame_splicing = 3;
  cfg.pad_out_feat = 256;
  cfg.preemph = 0.97f;
  cfg.dither = 1e-5f;
  cfg.log_guard = 1e-20f;
  cfg.norm_eps = 1e-12f;
  rnnt_featurizer* f = nullptr;
  if (rnnt_featurizer_create(&cfg, window.data(), fb.data(), 0, &f)) return 3;
  if (rnnt_featurizer_run(f, wav, nullptr, maxl, d_lens, lens.data(), n, n_pad, feats, flen, T_out, nullptr)) return 3;
  rnnt_featurizer_destroy(f);
  FILE* fo = fopen(argv[2], "wb");
  fwrite(flen, 4, n_pad, fo);
  fwrite(feats, 4, (size_t)T_out * n_pad * 256, fo);
  fclose(fo);
  fprintf(stderr, "fz_emu: %ld workgroups, poison %s\n", emu_workgroups, mode.c_str());
  free(wav);
  free(d_lens);
  free(feats);
  free(flen);
  return 0;
}
