// Audio feature kernels (utils/audio/extraction/extract_features_utils.py).
//
// nstl_autocorr restates extract_overlapping_autocorr + fix_edge_frames_autocorr
// (:54-113): reflect-pad frame_length/2, frames of frame_length every
// hop_length, per-frame DC removal, symmetric Hann (np.hanning), lags
// 0..n_lags by direct products (the reference computes a full 2N-1-lag
// np.correlate and keeps n_lags+1 of them), normalise by lag 0 when non-zero,
// drop lag 0, replicate near-silent edge frames.  One workgroup per frame; the
// windowed frame lives in LDS as f64 (the reference is f64 from the window on).
#include <cmath>

#include "../../include/nstl.h"
#include "common.h"
#include "status.h"

namespace {
constexpr int NT = 256;
constexpr int MAX_FRAME = 4096;

__global__ __launch_bounds__(NT) void autocorr_kernel(const float* y, int64_t n, int L, int hop, int n_lags,
                                                       double* out) {
  __shared__ double w[MAX_FRAME];
  __shared__ double red[NT / 64];
  const int f = blockIdx.x, tid = threadIdx.x;
  const int64_t start = (int64_t)f * hop - L / 2;
  double s = 0.0;
  for (int k = tid; k < L; k += NT) {
    int64_t i = start + k;
    if (i < 0) i = -i;                       // numpy 'reflect' (edge not repeated)
    if (i >= n) i = 2 * (n - 1) - i;
    const double v = (double)y[i];
    w[k] = v;
    s += v;
  }
  s = wave_sum_d(s);
  if ((tid & 63) == 0) red[tid >> 6] = s;
  __syncthreads();
  const double mean = (red[0] + red[1] + red[2] + red[3]) / L;
  // the reference subtracts the mean in float32 (frames are float32 until the
  // float64 window multiplies them)
  const float mean_f = (float)mean;
  for (int k = tid; k < L; k += NT) {
    const float c = (float)w[k] - mean_f;
    const double hann = L > 1 ? 0.5 - 0.5 * cos(2.0 * M_PI * k / (L - 1)) : 1.0;
    w[k] = (double)c * hann;
  }
  __syncthreads();
  __shared__ double ac0;
  for (int lag = tid; lag <= n_lags; lag += NT) {
    double acc = 0.0;
    for (int k = 0; k < L - lag; ++k) acc += w[k] * w[k + lag];
    if (lag == 0) ac0 = acc;
    if (lag > 0) out[(int64_t)f * n_lags + (lag - 1)] = acc;
  }
  __syncthreads();
  if (ac0 != 0.0)
    for (int lag = tid; lag < n_lags; lag += NT) out[(int64_t)f * n_lags + lag] /= ac0;
}

__global__ void autocorr_edges(double* out, int n_frames, int n_lags) {
  // fix_edge_frames_autocorr: replicate a near-all-zero first/last frame
  __shared__ int zero_first, zero_last;
  if (threadIdx.x == 0) {
    zero_first = 1;
    zero_last = 1;
  }
  __syncthreads();
  for (int l = threadIdx.x; l < n_lags; l += blockDim.x) {
    if (fabs(out[l]) >= 1e-7) zero_first = 0;
    if (fabs(out[(int64_t)(n_frames - 1) * n_lags + l]) >= 1e-7) zero_last = 0;
  }
  __syncthreads();
  if (zero_first && n_frames > 1)
    for (int l = threadIdx.x; l < n_lags; l += blockDim.x) out[l] = out[n_lags + l];
  __syncthreads();
  if (zero_last && n_frames > 1)
    for (int l = threadIdx.x; l < n_lags; l += blockDim.x)
      out[(int64_t)(n_frames - 1) * n_lags + l] = out[(int64_t)(n_frames - 2) * n_lags + l];
}
}  // namespace

extern "C" int nstl_autocorr(const float* y, int64_t n_samples, int frame_length, int hop_length, int n_lags,
                             double* out, int n_frames, void* stream) {
  NSTL_CHECK_ARG(y && out && n_samples > frame_length / 2 && frame_length > 1 && frame_length <= MAX_FRAME,
                 "nstl_autocorr: bad sizes");
  NSTL_CHECK_ARG(hop_length > 0 && n_lags > 0 && n_lags < frame_length && n_lags < 512, "nstl_autocorr: bad lags");
  const int64_t padded = n_samples + 2 * (frame_length / 2);
  const int expect = (int)((padded - frame_length) / hop_length + 1);
  NSTL_CHECK_ARG(n_frames == expect, "nstl_autocorr: n_frames %d != %d", n_frames, expect);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(autocorr_kernel, dim3(n_frames), dim3(NT), 0, st, y, n_samples, frame_length, hop_length,
                     n_lags, out);
  NSTL_LAUNCH_CHECK("nstl_autocorr");
  hipLaunchKernelGGL(autocorr_edges, dim3(1), dim3(256), 0, st, out, n_frames, n_lags);
  NSTL_LAUNCH_CHECK("nstl_autocorr edges");
  return 0;
}
