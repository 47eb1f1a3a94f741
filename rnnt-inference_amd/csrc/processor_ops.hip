// processor_ops.hip -- the audio front end's plugin operators one at a time:
// torch.ops.intel_mlperf.preemphasis / power_spectrum / frame_splicing / i_layernorm_pad, the ops
// the reference's FilterbankFeatures.forward calls between torch.stft, baddbmm and log
// (datasets/parts/features.py:196-250) -- i.e. what its TorchScript processor graph
// (processor_jit.pt, run by csrc/rnnt_processor.hpp:29-48) binds to.  The fused featurizer
// (featurizer.hip) is the throughput path; these give the op-by-op graph the same semantics
// (oracle/featurizer.py restates them; the plugin's own source is absent: parity unpinned).
// All are element-wise / per-column passes over HBM: one launch each, coalesced along the
// contiguous axis, no LDS.
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/rnnt_mi355x.h"
#include "featurizer.hpp"

namespace {

// torch reflect padding index, extended periodically (rows shorter than the pad), as the fused
// featurizer and oracle/featurizer.py mirror_index
__device__ __forceinline__ int mirror_idx(int p, int L) {
  if (L == 1) return 0;
  const int period = 2 * (L - 1);
  int m = p % period;
  if (m < 0) m += period;
  return m < L ? m : period - m;
}

// y[n][p] = pre-emphasised row n at reflect index p - pad (p < len + 2 pad), 0 past it
__global__ void __launch_bounds__(256) op_preemphasis_kernel(const float* __restrict__ x, int64_t stride,
                                                             const int32_t* __restrict__ lens, int L_out, float coeff,
                                                             int pad, float* __restrict__ y) {
  const int n = blockIdx.y, p = blockIdx.x * 256 + threadIdx.x;
  if (p >= L_out) return;
  const int L = lens[n];
  float v = 0.0f;
  if (L > 0 && p < L + 2 * pad) {
    const float* r = x + (size_t)n * stride;
    const int m = mirror_idx(p - pad, L);
    v = m > 0 ? r[m] - coeff * r[m - 1] : r[0];
  }
  y[(size_t)n * L_out + p] = v;
}

// |X|^2 of frames t < frames[n]: x [N][T][bins][2] (re, im) -> y [N][T][bins]
__global__ void __launch_bounds__(256) op_power_spectrum_kernel(const float2* __restrict__ x,
                                                                const int32_t* __restrict__ frames, int T, int bins,
                                                                float* __restrict__ y) {
  const int n = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x, per = (int64_t)T * bins;
  if (i >= per) return;
  const int t = (int)(i / bins);
  float v = 0.0f;
  if (t < frames[n]) {
    const float2 z = x[(size_t)n * per + i];
    v = z.x * z.x + z.y * z.y;
  }
  y[(size_t)n * per + i] = v;
}

// x [N][C][T] -> y [N][C f][To]: y[n][q C + m][t] = x[n][m][f t + q] for frames f t + q < frames[n]
__global__ void __launch_bounds__(256) op_frame_splicing_kernel(const float* __restrict__ x,
                                                                const int32_t* __restrict__ frames, int C, int T,
                                                                int f, int To, float* __restrict__ y) {
  const int n = blockIdx.z, row = blockIdx.y;  // row = q C + m
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= To) return;
  const int q = row / C, m = row % C, s = f * t + q;
  const int F = min(frames[n], T);
  y[((size_t)n * C * f + row) * To + t] = s < F ? x[((size_t)n * C + m) * T + s] : 0.0f;
}

// per (row, channel) over the row's valid frames: (x - mean) / sqrt(var + eps) * w + b, var unbiased
// when asked (one frame: 0), fp64 sums in frame order (deterministic); zero past the length, in
// channels >= C and rows >= N of the [N_out][C_out][T] output
__global__ void __launch_bounds__(256) op_layernorm_pad_kernel(const float* __restrict__ x,
                                                               const float* __restrict__ w,
                                                               const float* __restrict__ b, int wt,
                                                               const int32_t* __restrict__ lens, int N, int C, int T,
                                                               int C_out, float eps, int unbiased,
                                                               float* __restrict__ y, int32_t* __restrict__ lens_out) {
  const int n = blockIdx.y, c = blockIdx.x * 256 + threadIdx.x;
  if (c == 0) lens_out[n] = n < N ? min(lens[n], T) : 0;
  if (c >= C_out) return;
  float* out = y + ((size_t)n * C_out + c) * T;
  const int Tn = (n < N && c < C) ? min(lens[n], T) : 0;
  float mean = 0.0f, rstd = 0.0f;
  if (Tn > 0) {
    const float* col = x + ((size_t)n * C + c) * T;
    double s = 0.0, s2 = 0.0;
    for (int t = 0; t < Tn; ++t) {
      const double v = (double)col[t];
      s += v;
      s2 += v * v;
    }
    const double m = s / Tn;
    const int dof = unbiased ? Tn - 1 : Tn;
    const double var = dof > 0 ? fmax(s2 - s * m, 0.0) / (double)dof : 0.0;
    mean = (float)m;
    rstd = 1.0f / sqrtf((float)var + eps);
    for (int t = 0; t < Tn; ++t) {
      const float wv = t < wt ? w[(size_t)c * wt + t] : 1.0f, bv = t < wt ? b[(size_t)c * wt + t] : 0.0f;
      out[t] = (col[t] - mean) * rstd * wv + bv;
    }
  }
  for (int t = Tn; t < T; ++t) out[t] = 0.0f;
}

int op_fail(int code, const char* m) { return rnnt_internal_fail(code, m); }

int launched(const char* what) {
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? RNNT_OK : op_fail(RNNT_EDEVICE, (std::string(what) + ": " + hipGetErrorString(e)).c_str());
}

}  // namespace

extern "C" int rnnt_op_preemphasis(const float* x, int64_t stride, const int32_t* lens, int n, int L_out, float coeff,
                                   int pad, float* y, void* stream) {
  if (!x || !lens || !y) return op_fail(RNNT_EINVAL, "preemphasis: null argument");
  if (n < 0 || L_out < 0 || pad < 0 || stride < 0) return op_fail(RNNT_EINVAL, "preemphasis: bad shape");
  if (n == 0 || L_out == 0) return RNNT_OK;
  hipLaunchKernelGGL(op_preemphasis_kernel, dim3((L_out + 255) / 256, n), dim3(256), 0, (hipStream_t)stream, x, stride,
                     lens, L_out, coeff, pad, y);
  return launched("preemphasis");
}

extern "C" int rnnt_op_power_spectrum(const float* x, const int32_t* frames, int n, int T, int bins, float* y,
                                      void* stream) {
  if (!x || !frames || !y) return op_fail(RNNT_EINVAL, "power_spectrum: null argument");
  if (n < 0 || T < 0 || bins <= 0) return op_fail(RNNT_EINVAL, "power_spectrum: bad shape");
  const int64_t per = (int64_t)T * bins;
  if (n == 0 || per == 0) return RNNT_OK;
  hipLaunchKernelGGL(op_power_spectrum_kernel, dim3((unsigned)((per + 255) / 256), n), dim3(256), 0,
                     (hipStream_t)stream, (const float2*)x, frames, T, bins, y);
  return launched("power_spectrum");
}

extern "C" int rnnt_op_frame_splicing(const float* x, const int32_t* frames, int n, int C, int T, int factor, float* y,
                                      void* stream) {
  if (!x || !frames || !y) return op_fail(RNNT_EINVAL, "frame_splicing: null argument");
  if (n < 0 || C <= 0 || T < 0 || factor <= 0) return op_fail(RNNT_EINVAL, "frame_splicing: bad shape");
  const int To = (T + factor - 1) / factor;
  if (n == 0 || To == 0) return RNNT_OK;
  hipLaunchKernelGGL(op_frame_splicing_kernel, dim3((To + 255) / 256, C * factor, n), dim3(256), 0,
                     (hipStream_t)stream, x, frames, C, T, factor, To, y);
  return launched("frame_splicing");
}

extern "C" int rnnt_op_layernorm_pad(const float* x, const float* weight, const float* bias, int wt,
                                     const int32_t* lens, int n, int C, int T, int n_out, int C_out, float eps,
                                     int unbiased, float* y, int32_t* lens_out, void* stream) {
  if (!x || !weight || !bias || !lens || !y || !lens_out) return op_fail(RNNT_EINVAL, "i_layernorm_pad: null argument");
  if (n < 0 || C <= 0 || T < 0 || n_out < n || C_out < C || wt < 0) return op_fail(RNNT_EINVAL, "i_layernorm_pad: bad shape");
  if (n_out == 0) return RNNT_OK;
  hipLaunchKernelGGL(op_layernorm_pad_kernel, dim3((C_out + 255) / 256, n_out), dim3(256), 0, (hipStream_t)stream, x,
                     weight, bias, wt, lens, n, C, T, C_out, eps, unbiased, y, lens_out);
  return launched("i_layernorm_pad");
}
