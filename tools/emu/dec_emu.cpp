// dec_emu.cpp -- runs the engine's greedy decode (decoder.hip: launch_dec_xtab +
// launch_greedy_decode, every step kernel) on the host emulation of the wave model
// (emu_hip.hpp) and compares tokens with the oracle (oracle_greedy_decode, bf16 mode).
// Built with AddressSanitizer by tools/emu/build.sh.  Usage: dec_emu [N rows] [Tp] [seed] [server] [blank bias]
// (server: two decode_stream-style calls over halves of the frames, slots kept between them).
#include "emu_hip.hpp"
#include "decoder_emu.hip.cpp"

#include <random>
#include <algorithm>

extern "C" void oracle_greedy_decode(int Tp, int N, const float* f, const int32_t* f_lens, int bf16,
                                     const float* embed, const float* const* pWih, const float* const* pWhh,
                                     const float* const* pbih, const float* const* pbhh, const float* W1t,
                                     const float* W1p, const float* bt, const float* bp, const float* W2,
                                     const float* b2, int32_t* res, int32_t* res_len, int max_res, int32_t* steps);

using namespace rnnt;

static uint16_t f2bf_bits(float f) {  // RNE
  uint32_t u;
  memcpy(&u, &f, 4);
  u += 0x7fff + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}
static float bfr(float f) { return emu_bf2f(f2bf_bits(f)); }
static float bfr_ftz(float f) { return fabsf(f) < 1.17549435e-38f ? copysignf(0.0f, f) : bfr(f); }

template <class T>
static T* dalloc(size_t n) {  // exact-size "device" buffer: ASan flags any access past it
  T* p = (T*)malloc(n * sizeof(T) ? n * sizeof(T) : 1);
  memset(p, 0xA5, n * sizeof(T));
  return p;
}

int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 8;
  const int Tp = argc > 2 ? atoi(argv[2]) : 12;
  const int seed = argc > 3 ? atoi(argv[3]) : 1;
  const bool server = argc > 4 && atoi(argv[4]) != 0;
  const int Npad = (N + 31) / 32 * 32;
  const int max_res = Tp * 30 + 1;
  std::mt19937 rng(seed);
  std::normal_distribution<float> nd(0.0f, 1.0f);
  auto randv = [&](size_t n, float s) {
    std::vector<float> v(n);
    for (auto& x : v) x = bfr(nd(rng) * s);
    return v;
  };
  // torch-layout weights (bf16-exact), oracle inputs
  std::vector<float> embed = randv(28 * P, 0.5f);
  std::vector<float> Wih[2], Whh[2], bih[2], bhh[2];
  for (int l = 0; l < 2; ++l) {
    Wih[l] = randv((size_t)PG4 * P, 0.08f);
    Whh[l] = randv((size_t)PG4 * P, 0.08f);
    bih[l] = randv(PG4, 0.2f);
    bhh[l] = randv(PG4, 0.2f);
  }
  std::vector<float> W1t = randv((size_t)J * H, 0.04f), W1p = randv((size_t)J * P, 0.08f);
  std::vector<float> bt = randv(J, 0.1f), bp = randv(J, 0.1f);
  std::vector<float> W2 = randv((size_t)NLAB * J, 0.15f), b2 = randv(NLAB, 0.3f);
  b2[BLANK] += argc > 5 ? (float)atof(argv[5]) : 1.5f;  // blank bias: mostly blanks, some emissions
  // device layouts (engine.hip's packing: gate-interleaved rows 4u+g, [W_ih | W_hh] natural k)
  uint16_t* d_embed = dalloc<uint16_t>(28 * P);
  for (int i = 0; i < 28 * P; ++i) d_embed[i] = f2bf_bits(embed[i]);
  uint16_t* d_wp[2];
  float *d_bih[2], *d_bhh[2];
  for (int l = 0; l < 2; ++l) {
    d_wp[l] = dalloc<uint16_t>((size_t)PG4 * 640);
    d_bih[l] = dalloc<float>(PG4);
    d_bhh[l] = dalloc<float>(PG4);
    for (int u = 0; u < P; ++u)
      for (int g = 0; g < 4; ++g) {
        const int r = 4 * u + g, tr = g * P + u;
        for (int k = 0; k < P; ++k) {
          d_wp[l][(size_t)r * 640 + k] = f2bf_bits(Wih[l][(size_t)tr * P + k]);
          d_wp[l][(size_t)r * 640 + P + k] = f2bf_bits(Whh[l][(size_t)tr * P + k]);
        }
        d_bih[l][r] = bih[l][tr];
        d_bhh[l][r] = bhh[l][tr];
      }
  }
  uint16_t* d_w1t = dalloc<uint16_t>((size_t)J * H);
  uint16_t* d_w1p = dalloc<uint16_t>((size_t)J * P);
  for (size_t i = 0; i < (size_t)J * H; ++i) d_w1t[i] = f2bf_bits(W1t[i]);
  for (size_t i = 0; i < (size_t)J * P; ++i) d_w1p[i] = f2bf_bits(W1p[i]);
  float* d_bt = dalloc<float>(J);
  float* d_bp = dalloc<float>(J);
  memcpy(d_bt, bt.data(), J * 4);
  memcpy(d_bp, bp.data(), J * 4);
  uint16_t* d_w2 = dalloc<uint16_t>(32 * J);
  float* d_b2 = dalloc<float>(32);
  for (int j = 0; j < 32; ++j) {
    d_b2[j] = j < NLAB ? b2[j] : 0.0f;
    for (int k = 0; k < J; ++k) d_w2[(size_t)j * J + k] = j < NLAB ? f2bf_bits(W2[(size_t)j * J + k]) : 0;
  }
  float* d_xtab = dalloc<float>(29 * PG4);
  DecWeights w{};
  w.embed = d_embed;
  for (int l = 0; l < 2; ++l) {
    w.wp[l] = d_wp[l];
    w.bih_p[l] = d_bih[l];
    w.bhh_p[l] = d_bhh[l];
  }
  w.w1t = d_w1t; w.w1p = d_w1p; w.bt = d_bt; w.bp = d_bp; w.w2 = d_w2; w.b2 = d_b2;
  if (launch_dec_xtab(w, d_xtab, nullptr)) return 2;
  fprintf(stderr, "xtab done (%ld workgroups)\n", emu_workgroups);
  w.xtab = d_xtab;
  // encoder output f [Tp][N][1024] and the joint's encoder half F [Tp][Npad][512] (= joint_trans)
  std::vector<int32_t> flen(Npad, 0);
  std::uniform_int_distribution<int> ld(1, Tp);
  for (int n = 0; n < N; ++n) flen[n] = n == 0 ? Tp : ld(rng);
  std::vector<float> f((size_t)Tp * N * H);
  for (auto& x : f) x = nd(rng);
  float* d_F = dalloc<float>((size_t)Tp * Npad * J);
  {
    std::vector<float> xb(H), wr(H);
    for (int t = 0; t < Tp; ++t)
      for (int n = 0; n < Npad; ++n)
        for (int j = 0; j < J; ++j) {
          float o = 0.0f;
          if (n < N) {
            for (int k = 0; k < H; ++k) {
              xb[k] = bfr_ftz(f[((size_t)t * N + n) * H + k]);
              wr[k] = W1t[(size_t)j * H + k];
            }
            oracle_mfma_bf16_dot(1, H, &bt[j], xb.data(), wr.data(), &o);
          }
          d_F[((size_t)t * Npad + n) * J + j] = o;
        }
  }
  fprintf(stderr, "F done\n");
  int32_t* d_flen = dalloc<int32_t>(Npad);
  memcpy(d_flen, flen.data(), Npad * 4);
  DecArgs a{};
  a.w = w;
  a.F = d_F;
  a.f_lens = d_flen;
  a.hc = dalloc<float>((size_t)Npad * 2 * 4 * P);
  a.G = dalloc<float>((size_t)Npad * J);
  a.PH = dalloc<float>((size_t)Npad * PG4);
#ifdef EMU_HAS_AH
  a.ah0 = dalloc<float>((size_t)Npad * PG4);
  a.ah1 = dalloc<float>((size_t)Npad * PG4);
#endif
  a.res = dalloc<int32_t>((size_t)N * max_res);
  a.res_len = dalloc<int32_t>(N);
  DecState& s = a.s;
  s.time = dalloc<int32_t>(Npad); s.added = dalloc<int32_t>(Npad); s.idx = dalloc<int32_t>(Npad);
  s.preg = dalloc<int32_t>(Npad); s.slot = dalloc<int32_t>(Npad); s.fin = dalloc<int32_t>(Npad);
  s.list = dalloc<int32_t>(2 * (size_t)Npad);
  s.live = dalloc<int4>(2 * (size_t)Npad);
  s.count = dalloc<int32_t>(4);
  s.unfinished = dalloc<int32_t>(4);
  s.pc = dalloc<uint32_t>(8);  // persistent tail decode counters (not emulated: RNNT_EMU builds it out)
  a.N = N;
  a.Npad = Npad;
  a.max_res = max_res;
  a.max_iter = Tp * (MAXSYM + 1) + 2;
  int32_t host_flags[4] = {0, 0, 0, 0};
  hipEvent_t evs[2] = {nullptr, nullptr};
  int steps = 0;
  if (!server) {
    steps = launch_greedy_decode(a, host_flags, evs, nullptr, nullptr);
  } else {  // Server continuous batching: two calls over the two halves of the frames, state carried
    const int T1 = (Tp + 1) / 2;
    int32_t* reset = dalloc<int32_t>(Npad);
    int32_t* cl = dalloc<int32_t>(Npad);
    for (int n = 0; n < Npad; ++n) {
      reset[n] = 1;
      cl[n] = std::min(flen[n], T1);
    }
    a.f_lens = cl;
    a.max_iter = T1 * (MAXSYM + 1) + 2;
    steps = launch_greedy_decode(a, host_flags, evs, nullptr, reset);
    for (int n = 0; n < Npad; ++n) {
      reset[n] = 0;
      cl[n] = std::max(flen[n] - T1, 0);
    }
    a.F = d_F + (size_t)T1 * Npad * J;
    a.max_iter = (Tp - T1) * (MAXSYM + 1) + 2;
    steps += launch_greedy_decode(a, host_flags, evs, nullptr, reset);
  }
  printf("emulated decode: %d steps, %ld workgroups\n", steps, emu_workgroups);
#ifdef EMU_HAS_DEC_CHECK
  printf("bounds checks: %s (0x%x)\n", g_dec_err & 0x7fffffffu ? "FAILED" : "ok", g_dec_err);
#else
  printf("bounds checks: ok (none in this decoder; exact-size buffers only)\n");
#endif
  // oracle
  std::vector<int32_t> ro((size_t)N * max_res), rlo(N), st(2 * N);
  const float* pWih[2] = {Wih[0].data(), Wih[1].data()};
  const float* pWhh[2] = {Whh[0].data(), Whh[1].data()};
  const float* pbih[2] = {bih[0].data(), bih[1].data()};
  const float* pbhh[2] = {bhh[0].data(), bhh[1].data()};
  oracle_greedy_decode(Tp, N, f.data(), flen.data(), 1, embed.data(), pWih, pWhh, pbih, pbhh, W1t.data(), W1p.data(),
                       bt.data(), bp.data(), W2.data(), b2.data(), ro.data(), rlo.data(), max_res, st.data());
  int bad = 0, emitted = 0;
  for (int n = 0; n < N; ++n) {
    emitted += rlo[n];
    if (a.res_len[n] != rlo[n] || memcmp(a.res + (size_t)n * max_res, ro.data() + (size_t)n * max_res, max_res * 4)) {
      if (bad < 5) {
        printf("row %d: len %d vs oracle %d; first tokens", n, a.res_len[n], rlo[n]);
        for (int i = 0; i < 8 && i < max_res; ++i) printf(" %d/%d", a.res[(size_t)n * max_res + i], ro[(size_t)n * max_res + i]);
        printf("\n");
      }
      ++bad;
    }
  }
  printf("rows %d, emitted %d, mismatched rows %d -> %s\n", N, emitted, bad, bad ? "MISMATCH" : "tokens identical");
  return bad ? 1 : 0;
}
