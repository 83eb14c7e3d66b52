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
#include <mutex>
#include <vector>

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

// ============================================================================
// MFCC branch + combined features (extract_features.py:6-46,
// extract_features_utils.py:5-44 -> librosa.feature.mfcc / delta).
//
//   frames  : centre-padded (zeros, n_fft/2 each side) frames of n_fft samples
//             every hop, times the periodic Hann window           [F][kp] f32
//   X       : frames @ DFT basis (cos | sin rows), nstl_gemm f32 MFMA [F][2nb]
//   mel dB  : |X|^2 -> 128 Slaney filters -> 10 log10(max(1e-10, .)) [F][128],
//             running clip-wide max (ordered-int atomicMax)
//   mfcc    : max(dB, max-80) -> DCT-II ortho rows 0..22 (coefficient-major) [23][F]
//   final   : per coefficient CMVN (population std, +1e-10), Savitzky-Golay
//             width-9 deltas (orders 1, 2; mode 'interp' edge fits), mean of
//             frame pairs (odd tail kept) -> out[:, 0:69]; autocorr lags reduced
//             the same way -> out[:, 69:256].
// The librosa algorithm is restated from its published definition (librosa is
// absent from this image): parity for this branch is unpinned, see DESIGN.md.
// ============================================================================
namespace {
constexpr int N_MELS = 128;
constexpr int N_MFCC = 23;
constexpr int N_AC = 187;
constexpr int SG_W = 9;  // delta width

struct FeatTables {
  int dev = -1, sr = 0, n_fft = 0, nb = 0, kp = 0;
  float* basis = nullptr;   // [2nb][kp]: rows 0..nb-1 cos, nb..2nb-1 sin (window in frames)
  float* window = nullptr;  // [n_fft] periodic Hann
  float* mel = nullptr;     // [N_MELS][nb]
  int* band = nullptr;      // [N_MELS][2] first/last+1 non-zero bin
  float* dct = nullptr;     // [N_MFCC][N_MELS]
  float* sg = nullptr;      // [2 orders][SG_W fit positions][SG_W taps]
};

double hz_to_mel(double f) {
  const double f_sp = 200.0 / 3, min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp, logstep = std::log(6.4) / 27.0;
  return f >= min_log_hz ? min_log_mel + std::log(f / min_log_hz) / logstep : f / f_sp;
}
double mel_to_hz(double m) {
  const double f_sp = 200.0 / 3, min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp, logstep = std::log(6.4) / 27.0;
  return m >= min_log_mel ? min_log_hz * std::exp(logstep * (m - min_log_mel)) : f_sp * m;
}

// E[t0][j]: the order-th derivative at position t0 of the least-squares
// polynomial (degree `order`) through samples j = 0..SG_W-1.  Interior outputs
// use t0 = SG_W/2; scipy's mode='interp' edges use the first/last window.
void savgol_table(int order, float* E) {
  const int P = order + 1;
  double G[3][3] = {}, Ginv[3][3] = {};
  for (int a = 0; a < P; ++a)
    for (int b = 0; b < P; ++b)
      for (int t = 0; t < SG_W; ++t) G[a][b] += std::pow((double)t, a + b);
  // invert the (P x P) normal matrix (Gauss-Jordan, P <= 3)
  double M[3][6] = {};
  for (int a = 0; a < P; ++a) {
    for (int b = 0; b < P; ++b) M[a][b] = G[a][b];
    M[a][P + a] = 1.0;
  }
  for (int c = 0; c < P; ++c) {
    int piv = c;
    for (int r = c + 1; r < P; ++r)
      if (std::fabs(M[r][c]) > std::fabs(M[piv][c])) piv = r;
    for (int k = 0; k < 2 * P; ++k) std::swap(M[c][k], M[piv][k]);
    const double d = M[c][c];
    for (int k = 0; k < 2 * P; ++k) M[c][k] /= d;
    for (int r = 0; r < P; ++r)
      if (r != c) {
        const double f = M[r][c];
        for (int k = 0; k < 2 * P; ++k) M[r][k] -= f * M[c][k];
      }
  }
  for (int a = 0; a < P; ++a)
    for (int b = 0; b < P; ++b) Ginv[a][b] = M[a][P + b];
  for (int t0 = 0; t0 < SG_W; ++t0)
    for (int j = 0; j < SG_W; ++j) {
      // coefficient q of the fit = sum_b Ginv[q][b] * j^b * x_j
      double e = 0.0;
      for (int q = order; q < P; ++q) {
        double cq = 0.0;
        for (int b = 0; b < P; ++b) cq += Ginv[q][b] * std::pow((double)j, b);
        double fall = 1.0;  // q! / (q-order)!
        for (int i = 0; i < order; ++i) fall *= (q - i);
        e += cq * fall * std::pow((double)t0, q - order);
      }
      E[t0 * SG_W + j] = (float)e;
    }
}

int upload(void** dst, const void* src, size_t bytes) {
  if (hipMalloc(dst, bytes) != hipSuccess) return nstl::fail((int)hipErrorOutOfMemory, "features: table alloc");
  if (hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice) != hipSuccess)
    return nstl::fail((int)hipErrorUnknown, "features: table upload");
  return 0;
}

// constant tables per (device, sr), built once and kept for the process
int get_tables(int sr, const FeatTables** out) {
  static std::mutex mu;
  static std::vector<FeatTables*> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nstl::fail((int)hipErrorNoDevice, "features: no device");
  std::lock_guard<std::mutex> lock(mu);
  for (auto* t : cache)
    if (t->dev == dev && t->sr == sr) {
      *out = t;
      return 0;
    }
  auto* t = new FeatTables();
  t->dev = dev;
  t->sr = sr;
  t->n_fft = (int)(0.01667 * sr);
  t->nb = t->n_fft / 2 + 1;
  t->kp = (t->n_fft + 3) / 4 * 4;
  const int n_fft = t->n_fft, nb = t->nb, kp = t->kp;
  std::vector<float> basis((size_t)2 * nb * kp, 0.f), win(n_fft), mel((size_t)N_MELS * nb, 0.f), dct(N_MFCC * N_MELS);
  std::vector<int> band(2 * N_MELS);
  for (int k = 0; k < nb; ++k)
    for (int n = 0; n < n_fft; ++n) {
      // exact integer phase reduction keeps the f64 argument small
      const double ph = 2.0 * M_PI * (double)(((int64_t)k * n) % n_fft) / n_fft;
      basis[(size_t)k * kp + n] = (float)std::cos(ph);
      basis[(size_t)(nb + k) * kp + n] = (float)std::sin(ph);
    }
  for (int n = 0; n < n_fft; ++n) win[n] = (float)(0.5 - 0.5 * std::cos(2.0 * M_PI * n / n_fft));
  // librosa.filters.mel(sr, n_fft, n_mels=128, fmin=0, fmax=sr/2, htk=False, norm='slaney')
  std::vector<double> mel_f(N_MELS + 2);
  const double m_lo = hz_to_mel(0.0), m_hi = hz_to_mel(sr / 2.0);
  for (int i = 0; i < N_MELS + 2; ++i) mel_f[i] = mel_to_hz(m_lo + (m_hi - m_lo) * i / (N_MELS + 1));
  for (int i = 0; i < N_MELS; ++i) {
    const double enorm = 2.0 / (mel_f[i + 2] - mel_f[i]);
    int lo = nb, hi = 0;
    for (int b = 0; b < nb; ++b) {
      const double fb = b * ((double)sr / n_fft);
      const double lower = -(mel_f[i] - fb) / (mel_f[i + 1] - mel_f[i]);
      const double upper = (mel_f[i + 2] - fb) / (mel_f[i + 2] - mel_f[i + 1]);
      const double w = std::max(0.0, std::min(lower, upper)) * enorm;
      mel[(size_t)i * nb + b] = (float)w;
      if (w > 0) {
        lo = std::min(lo, b);
        hi = b + 1;
      }
    }
    band[2 * i] = lo < hi ? lo : 0;
    band[2 * i + 1] = hi;
  }
  for (int k = 0; k < N_MFCC; ++k)
    for (int m = 0; m < N_MELS; ++m)
      dct[k * N_MELS + m] = (float)(std::cos(M_PI * k * (2 * m + 1) / (2.0 * N_MELS)) *
                                    std::sqrt((k == 0 ? 1.0 : 2.0) / N_MELS));
  float sg[2 * SG_W * SG_W];
  savgol_table(1, sg);
  savgol_table(2, sg + SG_W * SG_W);
  int rc = upload((void**)&t->basis, basis.data(), basis.size() * 4);
  if (!rc) rc = upload((void**)&t->window, win.data(), win.size() * 4);
  if (!rc) rc = upload((void**)&t->mel, mel.data(), mel.size() * 4);
  if (!rc) rc = upload((void**)&t->band, band.data(), band.size() * 4);
  if (!rc) rc = upload((void**)&t->dct, dct.data(), dct.size() * 4);
  if (!rc) rc = upload((void**)&t->sg, sg, sizeof(sg));
  if (rc) return rc;
  cache.push_back(t);
  *out = t;
  return 0;
}

__global__ __launch_bounds__(256) void stft_frames_kernel(const float* __restrict__ y, int64_t n, int n_fft, int hop,
                                                          int kp, const float* __restrict__ win,
                                                          float* __restrict__ frames) {
  const int f = blockIdx.x;
  const int64_t start = (int64_t)f * hop - n_fft / 2;  // center=True, zero padding
  float* row = frames + (int64_t)f * kp;
  for (int k = threadIdx.x; k < kp; k += 256) {
    const int64_t i = start + k;
    row[k] = (k < n_fft && i >= 0 && i < n) ? y[i] * win[k] : 0.f;
  }
}

__device__ __forceinline__ int ordered_key(float v) {
  const int i = __float_as_int(v);
  return i >= 0 ? i : i ^ 0x7fffffff;
}
__device__ __forceinline__ float from_key(int k) { return __int_as_float(k >= 0 ? k : k ^ 0x7fffffff); }

// one wave per frame: power spectrum -> mel bands -> dB
__global__ __launch_bounds__(256) void mel_db_kernel(const float* __restrict__ X, int F, int nb,
                                                     const float* __restrict__ mel, const int* __restrict__ band,
                                                     float* __restrict__ db, int* __restrict__ max_key) {
  extern __shared__ float pw[];  // [4][nb]
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int f = blockIdx.x * 4 + wave;
  float* p = pw + wave * nb;
  float mx = -INFINITY;
  if (f < F) {
    const float* xr = X + (int64_t)f * 2 * nb;
    for (int b = lane; b < nb; b += 64) {
      const float c = xr[b], s = xr[nb + b];
      p[b] = c * c + s * s;
    }
  }
  __syncthreads();
  if (f < F) {
    for (int m = lane; m < N_MELS; m += 64) {
      const int lo = band[2 * m], hi = band[2 * m + 1];
      const float* w = mel + (int64_t)m * nb;
      float acc = 0.f;
      for (int b = lo; b < hi; ++b) acc = fmaf(w[b], p[b], acc);
      const float v = 10.f * log10f(fmaxf(1e-10f, acc));
      db[(int64_t)f * N_MELS + m] = v;
      mx = fmaxf(mx, v);
    }
  }
  mx = wave_max(mx);
  if (lane == 0 && f < F) atomicMax(max_key, ordered_key(mx));
}

// mfcc[k][f] = sum_m dct[k][m] * max(db[f][m], max_db - 80)
__global__ __launch_bounds__(256) void dct_kernel(const float* __restrict__ db, int F, const float* __restrict__ dct,
                                                  const int* __restrict__ max_key, float* __restrict__ mfcc) {
  __shared__ float tile[64][N_MELS + 1];
  const int f0 = blockIdx.x * 64;
  const float floor_db = from_key(*max_key) - 80.f;
  for (int i = threadIdx.x; i < 64 * N_MELS; i += 256) {
    const int r = i / N_MELS, m = i % N_MELS;
    tile[r][m] = f0 + r < F ? fmaxf(db[(int64_t)(f0 + r) * N_MELS + m], floor_db) : 0.f;
  }
  __syncthreads();
  const int r = threadIdx.x & 63;
  for (int k = threadIdx.x >> 6; k < N_MFCC; k += 4) {
    float acc = 0.f;
    for (int m = 0; m < N_MELS; ++m) acc = fmaf(dct[k * N_MELS + m], tile[r][m], acc);
    if (f0 + r < F) mfcc[(int64_t)k * F + f0 + r] = acc;
  }
}

__device__ __forceinline__ float block_sum_f64(double v, double* red) {
  v = wave_sum_d(v);
  const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[wave] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < nw; ++i) s += red[i];
  return (float)s;
}

// One workgroup per MFCC coefficient: CMVN, deltas, pair reduction -> out.
__global__ __launch_bounds__(1024) void cmvn_delta_reduce_kernel(const float* __restrict__ mfcc, int F,
                                                                 const float* __restrict__ sg, float* __restrict__ out,
                                                                 int64_t ldo, int F60) {
  __shared__ double red[16];
  const int c = blockIdx.x;
  const float* x = mfcc + (int64_t)c * F;
  double s = 0.0;
  for (int i = threadIdx.x; i < F; i += blockDim.x) s += x[i];
  const float mean = (float)(block_sum_f64(s, red) / (double)F);
  double q = 0.0;
  for (int i = threadIdx.x; i < F; i += blockDim.x) {
    const double d = (double)(x[i] - mean);
    q += d * d;
  }
  const float sd = sqrtf(block_sum_f64(q, red) / (float)F);
  const float inv = 1.f / (sd + 1e-10f);
  for (int r = threadIdx.x; r < F60; r += blockDim.x) {
    float v[3] = {0.f, 0.f, 0.f};
    const int j_end = min(2 * r + 2, F);
    for (int j = 2 * r; j < j_end; ++j) {
      const int w0 = min(max(j - SG_W / 2, 0), F - SG_W), t0 = j - w0;
      float d1 = 0.f, d2 = 0.f;
#pragma unroll
      for (int t = 0; t < SG_W; ++t) {
        const float nv = (x[w0 + t] - mean) * inv;
        d1 = fmaf(sg[t0 * SG_W + t], nv, d1);
        d2 = fmaf(sg[SG_W * SG_W + t0 * SG_W + t], nv, d2);
      }
      v[0] += (x[j] - mean) * inv;
      v[1] += d1;
      v[2] += d2;
    }
    const float scale = j_end - 2 * r == 2 ? 0.5f : 1.f;
    float* o = out + (int64_t)r * ldo;
    o[c] = v[0] * scale;
    o[N_MFCC + c] = v[1] * scale;
    o[2 * N_MFCC + c] = v[2] * scale;
  }
}

// autocorr lags [F][n_lags] f64 -> pair means -> out[:, col0 + lag] f32
__global__ __launch_bounds__(256) void reduce_ac_kernel(const double* __restrict__ ac, int F, int n_lags,
                                                        float* __restrict__ out, int64_t ldo, int col0, int F60) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)F60 * n_lags) return;
  const int r = (int)(i / n_lags), l = (int)(i % n_lags);
  const int j = 2 * r;
  const double v = j + 1 < F ? (ac[(int64_t)j * n_lags + l] + ac[(int64_t)(j + 1) * n_lags + l]) / 2.0
                             : ac[(int64_t)j * n_lags + l];
  out[(int64_t)r * ldo + col0 + l] = (float)v;
}

size_t align256(size_t b) { return (b + 255) / 256 * 256; }

struct FeatLayout {
  int n_fft, hop, nb, kp, F, F60;
  size_t frames, X, db, mfcc, ac, key, total;
};

FeatLayout feat_layout(int64_t n_samples, int sr) {
  FeatLayout L;
  L.n_fft = (int)(0.01667 * sr);
  L.hop = L.n_fft / 2;
  L.nb = L.n_fft / 2 + 1;
  L.kp = (L.n_fft + 3) / 4 * 4;
  L.F = L.hop > 0 ? (int)(1 + n_samples / L.hop) : 0;
  L.F60 = (L.F + 1) / 2;
  size_t off = 0;
  L.frames = off; off += align256((size_t)L.F * L.kp * 4);
  L.X = off;      off += align256((size_t)L.F * 2 * L.nb * 4);
  L.db = off;     off += align256((size_t)L.F * N_MELS * 4);
  L.mfcc = off;   off += align256((size_t)L.F * N_MFCC * 4);
  L.ac = off;     off += align256((size_t)L.F * N_AC * 8);
  L.key = off;    off += 256;
  L.total = off;
  return L;
}

__global__ void init_key(int* k) { *k = INT_MIN; }
}  // namespace

extern "C" int64_t nstl_features_workspace_bytes(int64_t n_samples, int sr) {
  return (int64_t)feat_layout(n_samples, sr).total;
}

extern "C" int nstl_features_frames(int64_t n_samples, int sr) { return feat_layout(n_samples, sr).F60; }

extern "C" int nstl_features(const float* y, int64_t n_samples, int sr, float* out, int64_t ld_out, int n_out_frames,
                             void* workspace, int64_t workspace_bytes, void* stream) {
  NSTL_CHECK_ARG(y && out && workspace, "nstl_features: null pointer");
  NSTL_CHECK_ARG(sr >= 8000 && sr <= 192000, "nstl_features: sr %d out of range", sr);
  const FeatLayout L = feat_layout(n_samples, sr);
  NSTL_CHECK_ARG(L.n_fft <= MAX_FRAME && n_samples >= L.n_fft, "nstl_features: %lld samples < one frame",
                 (long long)n_samples);
  // extract_features.py:16-21: fewer than 9 frames is rejected by the caller;
  // the Savitzky-Golay fit needs them as well
  NSTL_CHECK_ARG((n_samples - L.n_fft) / L.hop + 1 >= 9, "nstl_features: fewer than 9 frames");
  NSTL_CHECK_ARG(n_out_frames == L.F60, "nstl_features: n_out_frames %d != %d", n_out_frames, L.F60);
  NSTL_CHECK_ARG(ld_out >= 2 * N_MFCC + N_MFCC + N_AC, "nstl_features: ld_out < 256");
  NSTL_CHECK_ARG(workspace_bytes >= (int64_t)L.total, "nstl_features: workspace too small");
  const FeatTables* T = nullptr;
  if (int rc = get_tables(sr, &T)) return rc;
  hipStream_t st = (hipStream_t)stream;
  char* ws = (char*)workspace;
  float* frames = (float*)(ws + L.frames);
  float* X = (float*)(ws + L.X);
  float* db = (float*)(ws + L.db);
  float* mf = (float*)(ws + L.mfcc);
  double* ac = (double*)(ws + L.ac);
  int* key = (int*)(ws + L.key);

  hipLaunchKernelGGL(stft_frames_kernel, dim3(L.F), dim3(256), 0, st, y, n_samples, L.n_fft, L.hop, L.kp, T->window,
                     frames);
  NSTL_LAUNCH_CHECK("nstl_features frames");
  nstl_gemm_args g = {};
  g.dtype = NSTL_F32; g.c_dtype = NSTL_F32; g.a_kmajor = 1; g.b_kmajor = 1;
  g.A = frames; g.lda = L.kp; g.B = T->basis; g.ldb = L.kp; g.C = X; g.ldc = 2 * L.nb;
  g.M = L.F; g.N = 2 * L.nb; g.K = L.kp; g.alpha = 1.f; g.beta = 0.f; g.epilogue = NSTL_EPI_NONE; g.split_k = 1;
  if (int rc = nstl_gemm(&g, stream)) return rc;
  hipLaunchKernelGGL(init_key, dim3(1), dim3(1), 0, st, key);
  hipLaunchKernelGGL(mel_db_kernel, dim3((L.F + 3) / 4), dim3(256), 4 * L.nb * sizeof(float), st, X, L.F, L.nb,
                     T->mel, T->band, db, key);
  NSTL_LAUNCH_CHECK("nstl_features mel");
  hipLaunchKernelGGL(dct_kernel, dim3((L.F + 63) / 64), dim3(256), 0, st, db, L.F, T->dct, key, mf);
  NSTL_LAUNCH_CHECK("nstl_features dct");
  hipLaunchKernelGGL(cmvn_delta_reduce_kernel, dim3(N_MFCC), dim3(1024), 0, st, mf, L.F, T->sg, out, ld_out, L.F60);
  NSTL_LAUNCH_CHECK("nstl_features cmvn");
  if (int rc = nstl_autocorr(y, n_samples, L.n_fft, L.hop, N_AC, ac, L.F, stream)) return rc;
  const int64_t n_red = (int64_t)L.F60 * N_AC;
  hipLaunchKernelGGL(reduce_ac_kernel, dim3((unsigned)((n_red + 255) / 256)), dim3(256), 0, st, ac, L.F, N_AC, out,
                     ld_out, 3 * N_MFCC, L.F60);
  NSTL_LAUNCH_CHECK("nstl_features reduce");
  return 0;
}
