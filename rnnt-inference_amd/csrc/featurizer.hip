// featurizer.hip -- log-mel filterbank front end on gfx950 (the reference's audio processor,
// FilterbankFeatures.forward, datasets/parts/features.py:185-252, run by the C++ SUT through
// AudioProcessor::forward, csrc/rnnt_processor.hpp:29-48, when WAV=true).
//
// Three kernels per batch (DESIGN.md "Featurizer"):
//   fz_plan_kernel    one workgroup: the (utterance, 16-frame chunk) list the next kernel walks
//                     (a compact 1-D grid: no empty workgroups for short utterances);
//   fz_logmel_kernel  one workgroup = 16 STFT frames of one utterance (3 workgroups per CU):
//                       - the chunk's 2720 samples pre-emphasised and reflect-padded into LDS
//                         (intel_mlperf.preemphasis, features.py:196-199);
//                       - one 512-point real FFT per frame as a 256-point complex FFT of
//                         (even, odd) sample pairs: Stockham radix 16 x 16, 16 lanes per frame,
//                         4 frames per wave, one LDS transpose between the two radix-16 passes,
//                         then the real-input split; power + dither^2 (torch.stft center=False
//                         :202-210, power_spectrum :215, :219-220);
//                       - the mel projection [16 frames x 257 bins] x fb^T on
//                         v_mfma_f32_16x16x4f32 over each 16-filter column tile's non-zero bin
//                         span, + 1e-20, log (baddbmm + log, :224-230), written straight to its
//                         spliced position (frame f -> row f/3, channels 80 (f%3) + filter;
//                         frame_splicing :232-235);
//   fz_norm_kernel    one workgroup per utterance: per-channel mean / unbiased variance over the
//                     valid rows (fp64 sums, sequential: deterministic), normalise in place,
//                     zero-fill the time / channel / batch padding (i_layernorm_pad, :239-250).
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rnnt_mi355x.h"
#include "featurizer.hpp"
#include "rnnt_device.hpp"

namespace rnnt {
namespace {

constexpr int NT = 256;                                    // threads per (sub-)workgroup (4 waves)
#ifndef RNNT_FZ_NSUB  // development override (tools/r04_fzdiag.sh variants): 3 = the round-3 workgroup
#define RNNT_FZ_NSUB 1
#endif
constexpr int FZ_NSUB = RNNT_FZ_NSUB;                      // fz_logmel: chunks (4-wave sub-groups) per workgroup
constexpr int SEGC = FZ_HOP * (FZ_CHUNK - 1) + FZ_WIN;     // 2720 samples per chunk
constexpr int WOFF = (FZ_NFFT - FZ_WIN) / 2;               // 96: torch.stft centres the window in n_fft
constexpr int SCR = 17 * 16;                               // 16 x 16 complex transpose, rows padded to 17
constexpr int PROW = 260;                                  // power row (floats, in the frame's scratch)
// z[m] = w y[2m] + i w y[2m+1] is non-zero for m in [48, 208): radix-16 inputs r = 3..12 of lane j
constexpr int R_LO = WOFF / 32, R_HI = (WOFF + FZ_WIN) / 32;  // 3, 13
static_assert(2 * SCR >= PROW, "power row must fit in the frame's scratch");

typedef float floatx4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(fmaf(a.x, b.x, -a.y * b.y), fmaf(a.x, b.y, a.y * b.x));
}

// forward DFT-4 in place
__device__ __forceinline__ void dft4(float2& a, float2& b, float2& c, float2& d) {
  const float2 a0 = cadd(a, c), a1 = csub(a, c), a2 = cadd(b, d);
  const float2 a3 = make_float2(b.y - d.y, d.x - b.x);  // -i (b - d)
  a = cadd(a0, a2);
  b = cadd(a1, a3);
  c = csub(a0, a2);
  d = csub(a1, a3);
}

// forward DFT-16 (4 x 4): X[k1 + 4 k2] ends up in v[4 k1 + k2]
__device__ __forceinline__ void dft16(float2 (&v)[16]) {
#pragma unroll
  for (int n2 = 0; n2 < 4; ++n2) dft4(v[n2], v[4 + n2], v[8 + n2], v[12 + n2]);
  // twiddles W16^(n2 k1) on v[4 k1 + n2]
  const float C1 = 0.92387953251128674f, S1 = 0.38268343236508978f, R2 = 0.70710678118654752f;
  v[5] = cmul(v[5], make_float2(C1, -S1));    // W^1
  v[6] = cmul(v[6], make_float2(R2, -R2));    // W^2
  v[7] = cmul(v[7], make_float2(S1, -C1));    // W^3
  v[9] = cmul(v[9], make_float2(R2, -R2));    // W^2
  v[10] = make_float2(v[10].y, -v[10].x);     // W^4 = -i
  v[11] = cmul(v[11], make_float2(-R2, -R2)); // W^6
  v[13] = cmul(v[13], make_float2(S1, -C1));  // W^3
  v[14] = cmul(v[14], make_float2(-R2, -R2)); // W^6
  v[15] = cmul(v[15], make_float2(-C1, S1));  // W^9
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1) dft4(v[4 * k1], v[4 * k1 + 1], v[4 * k1 + 2], v[4 * k1 + 3]);
}

__device__ __forceinline__ float2 dft16_out(const float2 (&v)[16], int q) { return v[4 * (q & 3) + (q >> 2)]; }

// sample index of the reflect-padded row (torch reflect padding, extended periodically so that
// rows shorter than the pad are defined too)
__device__ __forceinline__ int mirror(int p, int L) {
  if (L == 1) return 0;
  const int period = 2 * (L - 1);
  int m = p % period;
  if (m < 0) m += period;
  return m < L ? m : period - m;
}

// ordering of one wave's LDS writes before its lanes read each other's values
__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ int stft_frames(int L) { return L > 0 ? 1 + L / FZ_HOP : 0; }  // features.py:212

// feature frame t of row n: a [T_out][n_pad][256] batch, or ragged rows of 240 channels
__device__ __forceinline__ float* feat_row(const FzArgs& a, int n, int t) {
  return a.row_off ? a.feats + (size_t)(a.row_off[n] + t) * FZ_FEAT
                   : a.feats + ((size_t)t * a.n_pad + n) * FZ_FEAT_PAD;
}

// (utterance, chunk) of every fz_logmel workgroup: exclusive scan of ceil(F_n / 16), then scatter
__global__ __launch_bounds__(1024) void fz_plan_kernel(FzArgs a) {
  __shared__ int part[1024];
  __shared__ int carry;
  const int tid = threadIdx.x;
  if (tid == 0) carry = 0;
  __syncthreads();
  for (int base = 0; base < a.n; base += 1024) {
    const int n = base + tid;
    const int cnt = n < a.n ? (stft_frames(a.wav_lens[n]) + FZ_CHUNK - 1) / FZ_CHUNK : 0;
    part[tid] = cnt;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {  // inclusive Hillis-Steele scan
      const int v = tid >= off ? part[tid - off] : 0;
      __syncthreads();
      part[tid] += v;
      __syncthreads();
    }
    const int start = carry + part[tid] - cnt;
    for (int c = 0; c < cnt; ++c) a.plan[start + c] = make_int2(n, c);
    __syncthreads();
    if (tid == 1023) carry += part[1023];
    __syncthreads();
  }
}

// A workgroup = FZ_NSUB chunks, one 4-wave sub-group (NT threads) each; other kernels' workgroups
// may share its CU.  This file is compiled WITHOUT packed FP32 VALU (-fno-slp-vectorize, Makefile;
// tests/test_isa_lint.py checks the ISA): with v_pk_add/mul/fma_f32 in the FFT, the results of
// lanes 48-63 of a logmel wave came out wrong in ~8-13 % of the batches whenever decode step
// kernels shared the CU (the corrupted frames follow those lanes when the frame-to-lane map is
// reversed); built without them, 0 in ~100k batches, and no slower.
__global__ __launch_bounds__(NT * FZ_NSUB, 1) void fz_logmel_kernel(FzArgs a) {
  const int sub = threadIdx.x / NT;
  const int gj = blockIdx.x * FZ_NSUB + sub;  // this sub-group's plan entry
  const bool active = gj < a.n_chunks;        // sub-group-uniform: idle ones only meet the barriers
  const int2 job = active ? a.plan[gj] : make_int2(0, 0);
  const int n = job.x;
  const int L = active ? a.wav_lens[n] : 0;
  const int F = stft_frames(L);
  const int f0 = FZ_CHUNK * job.y;

  __shared__ float2 tab[FZ_NFFT];  // W512^t (shared by the sub-groups)
  __shared__ float win[FZ_WIN];
  __shared__ float segs[FZ_NSUB][SEGC];
  __shared__ float2 scrs[FZ_NSUB][NT / 64][4][SCR];
  float* seg = segs[sub];
  float2(*scr)[4][SCR] = scrs[sub];

  const int tid = threadIdx.x % NT, wave = tid >> 6, lane = tid & 63;
  const int slot = lane >> 4, j = lane & 15;  // frame slot in the wave, lane in the frame
  for (int i = threadIdx.x; i < FZ_NFFT; i += NT * FZ_NSUB) tab[i] = a.k.twiddle[i];
  for (int i = threadIdx.x; i < FZ_WIN; i += NT * FZ_NSUB) win[i] = a.k.window[i];
  // pre-emphasised, reflect-padded samples y[160 f0 - 160 + i]: frame f's window covers
  // y[160 f - 160, 160 f + 160) (pad n_fft/2 = 256, window offset 96 inside n_fft); all loads
  // issued before the first use
  if (active) {
    const float* x = a.wav + (a.off ? a.off[n] : (int64_t)n * a.stride);
    const float pc = a.k.preemph;
    const int base = FZ_HOP * f0 - FZ_HOP;
    constexpr int PER = (SEGC + NT - 1) / NT;
    int rr[PER];
    float xv[PER], xm[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int p = base + tid + NT * u;
      rr[u] = (p >= 0 && p < L) ? p : mirror(p, L);
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      xv[u] = x[rr[u]];
      xm[u] = x[max(rr[u] - 1, 0)];
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int i = tid + NT * u;
      if (i < SEGC) seg[i] = rr[u] > 0 ? xv[u] - pc * xm[u] : xv[u];
    }
  }
  __syncthreads();

#ifdef RNNT_FZ_SLOTREV  // development variant (DESIGN 4b diagnosis): lanes 48-63 take frame slot 0, lanes 0-15 slot 3
  const int fslot = 3 - slot;
#else
  const int fslot = slot;
#endif
  float2* sc = scr[wave][fslot];
  if (active) {
    const int fl = 4 * wave + fslot;  // frame in the chunk
    const float* sf = seg + FZ_HOP * fl - WOFF;
    float2 v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (r >= R_LO && r < R_HI) {
        const int i0 = 2 * j + 32 * r;
        v[r] = make_float2(win[i0 - WOFF] * sf[i0], win[i0 + 1 - WOFF] * sf[i0 + 1]);
      } else {
        v[r] = make_float2(0.0f, 0.0f);
      }
    }
    dft16(v);  // pass 1 (Ns = 1): element 16 j + q
#pragma unroll
    for (int q = 0; q < 16; ++q) sc[17 * j + q] = dft16_out(v, q);
    wave_lds_sync();
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = sc[17 * r + j];  // element j + 16 r
#pragma unroll
    for (int r = 1; r < 16; ++r) v[r] = cmul(v[r], tab[2 * r * j]);  // W256^(r j)
    dft16(v);  // pass 2 (Ns = 16): Z[j + 16 q]
    wave_lds_sync();
#pragma unroll
    for (int q = 0; q < 16; ++q) sc[17 * q + j] = dft16_out(v, q);
    wave_lds_sync();
    // X[k] = E + W512^k O with E = (Z[k] + conj Z[256-k]) / 2, O = -i (Z[k] - conj Z[256-k]) / 2
    float pv[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int k = j + 16 * q;
      const int e = (256 - k) & 255;
      const float2 zk = dft16_out(v, q), zm = sc[17 * (e >> 4) + (e & 15)];
      const float2 ev = make_float2(0.5f * (zk.x + zm.x), 0.5f * (zk.y - zm.y));
      const float2 od = make_float2(0.5f * (zk.y + zm.y), -0.5f * (zk.x - zm.x));
      const float2 t = cmul(od, tab[k]);
      const float re = ev.x + t.x, im = ev.y + t.y;
      pv[q] = fmaf(re, re, im * im) + a.k.dither_sq;
    }
    const float nyq = dft16_out(v, 0).x - dft16_out(v, 0).y;  // X[256] = Re Z[0] - Im Z[0]
    wave_lds_sync();  // the frame's Z reads are done: its scratch becomes its power row
    float* prow = reinterpret_cast<float*>(sc);
#pragma unroll
    for (int q = 0; q < 16; ++q) prow[j + 16 * q] = pv[q];
    if (j == 0) prow[FZ_NFFT / 2] = nyq * nyq + a.k.dither_sq;
    if (j >= 1 && j < PROW - FZ_NBIN + 1) prow[FZ_NBIN + j - 1] = 0.0f;
  }
  __syncthreads();
  if (!active) return;
  // mel projection of the 16 frames (rows) on v_mfma_f32_16x16x4f32; log; spliced store
  const float* arow = reinterpret_cast<const float*>(scr[j >> 2][j & 3]) + slot;
  for (int c = 0; c < FZ_MEL_COLS; ++c) {
    if (!((a.k.wave_cols[wave] >> c) & 1)) continue;
    floatx4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
    const float* ar = arow + a.k.col_k0[c];
    const float* bf = a.k.fbB + (size_t)a.k.col_off[c] * 64 + lane;
    const int nst = a.k.col_steps[c];
    for (int s0 = 0; s0 < nst; s0 += 8) {  // fragments fetched 8 steps at a time, then 8 MFMAs
      float av[8], bv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const bool ok = s0 + u < nst;
        av[u] = ok ? ar[4 * (s0 + u)] : 0.0f;
        bv[u] = ok ? bf[64 * (s0 + u)] : 0.0f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv[u], acc, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int f = f0 + 4 * slot + i;  // D row 4 slot + i = frame, column j = filter 16 c + j
      const int t = f / FZ_SPLICE;
      if (f < F && t < a.T_out) feat_row(a, n, t)[FZ_NMEL * (f - FZ_SPLICE * t) + 16 * c + j] = logf(acc[i] + a.k.log_guard);
    }
  }
  // spliced channels of frames past F (the last row's missing 3j+1 / 3j+2 frames) are zero
  if (f0 + FZ_CHUNK >= F && tid < 2 * FZ_NMEL) {
    const int Tn = (F + FZ_SPLICE - 1) / FZ_SPLICE;
    const int q = 1 + tid / FZ_NMEL;
    if (FZ_SPLICE * (Tn - 1) + q >= F && Tn - 1 < a.T_out) feat_row(a, n, Tn - 1)[FZ_NMEL * q + tid % FZ_NMEL] = 0.0f;
  }
}

// per-feature normalisation, one workgroup per row, thread c = channel.  Padded output: the
// row's [T_out] column of the [T_out][n_pad][256] batch, zero past its length and in channels
// 240..255 and rows >= n.  Ragged output (grid n): the row's Tn x 240 frames only.
__global__ __launch_bounds__(NT) void fz_norm_kernel(FzArgs a) {
  const int n = blockIdx.x, c = threadIdx.x;
  const bool ragged = a.row_off != nullptr;
  int Tn = 0;
  if (n < a.n) Tn = (stft_frames(a.wav_lens[n]) + FZ_SPLICE - 1) / FZ_SPLICE;
  Tn = min(Tn, a.T_out);
  if (c == 0) a.feat_lens[n] = Tn;
  const bool live = c < FZ_FEAT;
  if (ragged && !live) return;
  float* col = feat_row(a, n, 0) + c;
  const size_t rs = ragged ? (size_t)FZ_FEAT : (size_t)a.n_pad * FZ_FEAT_PAD;
  const int T_end = ragged ? Tn : a.T_out;
  float mean = 0.0f, rstd = 0.0f;
  if (live && Tn > 0) {
    double s = 0.0, s2 = 0.0;
    int t = 0;
    for (; t + 4 <= Tn; t += 4) {
      float x[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) x[u] = col[(t + u) * rs];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        s += (double)x[u];
        s2 += (double)x[u] * (double)x[u];
      }
    }
    for (; t < Tn; ++t) {
      const double x = (double)col[t * rs];
      s += x;
      s2 += x * x;
    }
    const double m = s / Tn;
    const double var = Tn > 1 ? fmax(s2 - s * m, 0.0) / (double)(Tn - 1) : 0.0;  // unbiased=1
    mean = (float)m;
    rstd = 1.0f / sqrtf((float)var + a.k.eps);
  }
  int t = 0;
  for (; t + 4 <= T_end; t += 4) {
    float x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) x[u] = (live && t + u < Tn) ? col[(t + u) * rs] : 0.0f;
#pragma unroll
    for (int u = 0; u < 4; ++u) col[(t + u) * rs] = (live && t + u < Tn) ? (x[u] - mean) * rstd : 0.0f;
  }
  for (; t < T_end; ++t) col[t * rs] = (live && t < Tn) ? (col[t * rs] - mean) * rstd : 0.0f;
}

}  // namespace

}  // namespace rnnt

// ---------------------------------------------------------------------------- C ABI
using namespace rnnt;

struct rnnt_featurizer {
  int device = 0;
  rnnt_featurizer_config cfg{};
  FzConsts k{};
  std::vector<void*> allocs;
  int2* plan = nullptr;
  size_t plan_cap = 0;  // chunks
  size_t own_cu_lds = 0;  // RNNT_FZ_OWN_CU=1: dynamic LDS that leaves no room for another workgroup on the CU
};

static int fz_fail(int code, const std::string& m) { return rnnt_internal_fail(code, m); }

#define FZCHK(x)                                                                                  \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess) return fz_fail(RNNT_EDEVICE, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

template <class T>
static int fz_upload(rnnt_featurizer* f, const T** dst, const std::vector<T>& h) {
  void* p = nullptr;
  FZCHK(hipMalloc(&p, h.size() * sizeof(T) + 16));
  f->allocs.push_back(p);
  FZCHK(hipMemcpy(p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  *dst = (const T*)p;
  return 0;
}

extern "C" int64_t rnnt_featurizer_frames(int64_t wav_len) {
  if (wav_len <= 0) return 0;
  return (1 + wav_len / FZ_HOP + FZ_SPLICE - 1) / FZ_SPLICE;
}

static size_t own_cu_lds_bytes(int device);

extern "C" int rnnt_featurizer_create(const rnnt_featurizer_config* cfg, const float* window, const float* fb,
                                      int device, rnnt_featurizer** out) {
  if (!cfg || !window || !fb || !out) return fz_fail(RNNT_EINVAL, "null argument");
  *out = nullptr;
  if (cfg->sample_rate != 16000 || cfg->n_fft != FZ_NFFT || cfg->win_length != FZ_WIN ||
      cfg->hop_length != FZ_HOP || cfg->nfilt != FZ_NMEL || cfg->frame_splicing != FZ_SPLICE ||
      cfg->pad_out_feat != FZ_FEAT_PAD)
    return fz_fail(RNNT_EINVAL, "featurizer geometry must be rnnt.toml [input_eval] (16 kHz, n_fft 512, "
                                "win 320, hop 160, 80 filters, splice 3, pad 256)");
  if (!(cfg->norm_eps >= 0.0f) || !(cfg->dither >= 0.0f) || !(cfg->log_guard >= 0.0f))
    return fz_fail(RNNT_EINVAL, "negative dither / log guard / eps");
  DeviceScope dscope(device);
  if (!dscope.ok) return fz_fail(RNNT_EDEVICE, "hipSetDevice failed");
  // fb^T as MFMA B fragments per 16-filter column tile over the tile's non-zero bin span; column
  // tiles dealt to the 4 waves longest first (each wave projects its tiles for every chunk)
  std::vector<float> frag;
  int k0[FZ_MEL_COLS], steps[FZ_MEL_COLS], coff[FZ_MEL_COLS];
  for (int c = 0; c < FZ_MEL_COLS; ++c) {
    int lo = FZ_NBIN, hi = 0;
    for (int m = 16 * c; m < 16 * c + 16; ++m)
      for (int k = 0; k < FZ_NBIN; ++k)
        if (fb[(size_t)m * FZ_NBIN + k] != 0.0f) {
          lo = std::min(lo, k);
          hi = std::max(hi, k + 1);
        }
    if (hi <= lo) lo = hi = 0;
    k0[c] = lo;
    steps[c] = (hi - lo + 3) / 4;
    coff[c] = (int)(frag.size() / 64);
    for (int st = 0; st < steps[c]; ++st)
      for (int l = 0; l < 64; ++l) {
        const int m = 16 * c + (l & 15), k = lo + 4 * st + (l >> 4);
        frag.push_back(k < FZ_NBIN ? fb[(size_t)m * FZ_NBIN + k] : 0.0f);
      }
  }
  int wave_cols[4] = {0, 0, 0, 0}, load[4] = {0, 0, 0, 0};
  {
    int order[FZ_MEL_COLS];
    for (int c = 0; c < FZ_MEL_COLS; ++c) order[c] = c;
    std::sort(order, order + FZ_MEL_COLS, [&](int x, int y) { return steps[x] > steps[y]; });
    for (int i = 0; i < FZ_MEL_COLS; ++i) {
      const int w = (int)(std::min_element(load, load + 4) - load);
      wave_cols[w] |= 1 << order[i];
      load[w] += steps[order[i]];
    }
  }
  std::vector<float2> tw(FZ_NFFT);
  for (int t = 0; t < FZ_NFFT; ++t) {
    const double ang = 2.0 * M_PI * (double)t / (double)FZ_NFFT;
    tw[t] = make_float2((float)cos(ang), (float)-sin(ang));
  }
  auto* f = new rnnt_featurizer;
  f->device = device;
  f->cfg = *cfg;
  int r = 0;
  const float* wptr = nullptr;
  if (!r) r = fz_upload(f, &wptr, std::vector<float>(window, window + FZ_WIN));
  f->k.window = wptr;
  if (frag.empty()) frag.assign(64, 0.0f);
  if (!r) r = fz_upload(f, &f->k.fbB, frag);
  if (!r) r = fz_upload(f, &f->k.twiddle, tw);
  if (r) {
    for (void* p : f->allocs) (void)hipFree(p);
    delete f;
    return r;
  }
  for (int c = 0; c < FZ_MEL_COLS; ++c) {
    f->k.col_k0[c] = k0[c];
    f->k.col_steps[c] = steps[c];
    f->k.col_off[c] = coff[c];
  }
  for (int w = 0; w < 4; ++w) f->k.wave_cols[w] = wave_cols[w];
  f->k.preemph = cfg->preemph;
  f->k.dither_sq = cfg->dither * cfg->dither;
  f->k.log_guard = cfg->log_guard;
  f->k.eps = cfg->norm_eps;
  f->own_cu_lds = own_cu_lds_bytes(device);
  *out = f;
  return 0;
}

extern "C" void rnnt_featurizer_destroy(rnnt_featurizer* f) {
  if (!f) return;
  DeviceScope dscope(f->device);
  for (void* p : f->allocs) (void)hipFree(p);
  if (f->plan) (void)hipFree(f->plan);
  delete f;
}

// RNNT_FZ_OWN_CU=1 (read at rnnt_featurizer_create): each fz_logmel workgroup requests the rest of its CU's
// LDS as unused dynamic LDS, so no other kernel's workgroup shares the CU -- the round-3 guard against the
// lanes-48-63 corruption beside decode workgroups, kept as a runtime switch behind the
// shipped guard (no packed FP32 in any kernel).  Costs occupancy: one 4-wave chunk per CU.
static size_t own_cu_lds_bytes(int device) {
  const char* v = getenv("RNNT_FZ_OWN_CU");
  if (!v || atoi(v) == 0) return 0;
  int per_cu = 0;
  if (hipDeviceGetAttribute(&per_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, device) != hipSuccess)
    return 0;
  hipFuncAttributes fa{};
  if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(fz_logmel_kernel)) != hipSuccess) return 0;
  // all of what is left (any amount over half would do): no workgroup of another kernel fits beside it
  const size_t left = (size_t)per_cu > fa.sharedSizeBytes ? (size_t)per_cu - fa.sharedSizeBytes : 0;
  if (left == 0) return 0;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(fz_logmel_kernel),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)left) != hipSuccess)
    return 0;
  return left;
}

static int launch_logmel(const FzArgs& a, size_t chunks, size_t dyn_lds, hipStream_t st) {
  hipLaunchKernelGGL(fz_logmel_kernel, dim3((unsigned)((chunks + FZ_NSUB - 1) / FZ_NSUB)), dim3(NT * FZ_NSUB),
                     dyn_lds, st, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" size_t rnnt_featurizer_own_cu_lds(const rnnt_featurizer* f) { return f ? f->own_cu_lds : 0; }

// row_off == nullptr: padded [T_out][n_pad][256] output; else ragged rows (n_pad == n)
static int featurizer_run(rnnt_featurizer* f, const float* wav, const int64_t* offsets, int64_t stride,
                          const int32_t* wav_lens, const int32_t* wav_lens_host, int n, int n_pad, float* feats,
                          const int64_t* row_off, int32_t* feat_lens, int T_out, void* stream) {
  if (!offsets && stride <= 0 && n > 0) return fz_fail(RNNT_EINVAL, "need offsets or a positive stride");
  int64_t tmax = 0;
  for (int i = 0; i < n; ++i) {
    if (wav_lens_host[i] < 0) return fz_fail(RNNT_EINVAL, "negative wav length");
    if (!offsets && wav_lens_host[i] > stride) return fz_fail(RNNT_EINVAL, "wav length exceeds the row stride");
    tmax = std::max(tmax, rnnt_featurizer_frames(wav_lens_host[i]));
  }
  if (tmax > T_out) return fz_fail(RNNT_EINVAL, "T_out smaller than the longest utterance's feature frames");
  DeviceScope dscope(f->device);
  if (!dscope.ok) return fz_fail(RNNT_EDEVICE, "hipSetDevice failed");
  size_t chunks = 0;
  for (int i = 0; i < n; ++i)
    if (wav_lens_host[i] > 0) chunks += (size_t)(1 + wav_lens_host[i] / FZ_HOP + FZ_CHUNK - 1) / FZ_CHUNK;
  if (chunks > f->plan_cap) {
    if (f->plan) FZCHK(hipFree(f->plan));
    f->plan = nullptr;
    f->plan_cap = 0;
    FZCHK(hipMalloc((void**)&f->plan, chunks * sizeof(int2)));
    f->plan_cap = chunks;
  }
  FzArgs a{};
  a.k = f->k;
  a.wav = wav;
  a.off = offsets;
  a.stride = stride;
  a.wav_lens = wav_lens;
  a.feats = feats;
  a.row_off = row_off;
  a.feat_lens = feat_lens;
  a.plan = f->plan;
  a.n = n;
  a.n_pad = n_pad;
  a.T_out = T_out;
  hipStream_t st = (hipStream_t)stream;
  a.n_chunks = (int)chunks;
  if (chunks > 0) {
    hipLaunchKernelGGL(fz_plan_kernel, dim3(1), dim3(1024), 0, st, a);
    if (launch_logmel(a, chunks, f->own_cu_lds, st)) return fz_fail(RNNT_EDEVICE, "fz_logmel launch failed");
  }
  if (n_pad > 0) hipLaunchKernelGGL(fz_norm_kernel, dim3(n_pad), dim3(NT), 0, st, a);
  FZCHK(hipGetLastError());
  return 0;
}

extern "C" int rnnt_featurizer_run(rnnt_featurizer* f, const float* wav, const int64_t* offsets, int64_t stride,
                                   const int32_t* wav_lens, const int32_t* wav_lens_host, int n, int n_pad,
                                   float* feats, int32_t* feat_lens, int T_out, void* stream) {
  if (!f || !wav || !wav_lens || !wav_lens_host || !feats || !feat_lens) return fz_fail(RNNT_EINVAL, "null argument");
  if (n < 0 || n_pad < n || n_pad <= 0 || T_out <= 0) return fz_fail(RNNT_EINVAL, "bad n / n_pad / T_out");
  return featurizer_run(f, wav, offsets, stride, wav_lens, wav_lens_host, n, n_pad, feats, nullptr, feat_lens, T_out,
                        stream);
}

extern "C" int rnnt_featurizer_run_rows(rnnt_featurizer* f, const float* wav, const int64_t* offsets, int64_t stride,
                                        const int32_t* wav_lens, const int32_t* wav_lens_host, int n, float* feats,
                                        const int64_t* row_off, int32_t* feat_lens, int max_frames, void* stream) {
  if (!f || !wav || !wav_lens || !wav_lens_host || !feats || !row_off || !feat_lens)
    return fz_fail(RNNT_EINVAL, "null argument");
  if (n < 0 || max_frames <= 0) return fz_fail(RNNT_EINVAL, "bad n / max_frames");
  return featurizer_run(f, wav, offsets, stride, wav_lens, wav_lens_host, n, n, feats, row_off, feat_lens, max_frames,
                        stream);
}
