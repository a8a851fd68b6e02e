// variants.hip — the extra ops of the AdaIN ("2") and speaker-embedding-adjust ("_Adjust")
// model variants:
//
//   * whole-tensor moments  x.mean(), x.std()          factory/AutoVC2.py:58-60 (features)
//   * AdaIN                 (x - x.mean())/x.std()*s+m  factory/Norm.py:84-91
//     and the backward of both (one double-precision reduction + one elementwise pass)
//   * per-utterance time sums of a column block: the speaker-embedding gradient of the
//     broadcast concats when the embedding itself is trained (AutoVC_Adjust.py:178-189)
//   * one time step of a frame-major sequence (nn.LSTM output [:, -1, :], Adjust.py:39)
//   * row L2 normalisation  embeds / ||embeds||         factory/Adjust.py:40-42
//
// Everything here is HBM-bound elementwise or reduction work over (B*T, 80) mel-sized
// tensors (2.6 MB at B=64, T=128): grid-stride float4 loads, fp64 partial sums (a
// whole-tensor variance over 655K values in fp32 would lose ~3 digits to cancellation),
// fixed-size partial arrays reduced by one workgroup so the result is deterministic.
#include <algorithm>

#include "common.h"

namespace {

constexpr int RED_BLOCKS = 512;  // partials per reduction (== AVC_MOMENTS_WS / 2 doubles)
constexpr int RED_THREADS = 256;

__device__ __forceinline__ double wave_sum(double v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  return v;
}

// Block-reduce two doubles into (a, b) held by thread 0.
__device__ __forceinline__ void block_sum2(double& a, double& b) {
  __shared__ double sa[RED_THREADS / 64], sb[RED_THREADS / 64];
  a = wave_sum(a);
  b = wave_sum(b);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) {
    sa[w] = a;
    sb[w] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < RED_THREADS / 64; ++i) {
      sa[0] += sa[i];
      sb[0] += sb[i];
    }
    a = sa[0];
    b = sb[0];
  }
}

// mode 0: (sum x, sum x^2)          -> moments
// mode 1: (sum g, sum g*(x-m)/s)    -> AdaIN backward sums, mom = [m, s]
__global__ void __launch_bounds__(RED_THREADS) reduce2_partial(const float* __restrict__ x,
                                                               const float* __restrict__ g, long long n,
                                                               const float* __restrict__ mom, int mode,
                                                               double* __restrict__ part) {
  double a = 0.0, b = 0.0;
  float m = 0.f, rs = 1.f;
  if (mode == 1) {
    m = mom[0];
    rs = 1.f / mom[1];
  }
  const long long n4 = n >> 2;
  const long long stride = (long long)gridDim.x * blockDim.x;
  const f32x4* x4 = reinterpret_cast<const f32x4*>(x);
  const f32x4* g4 = reinterpret_cast<const f32x4*>(g);
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    f32x4 v = x4[i];
    if (mode == 0) {
      for (int k = 0; k < 4; ++k) {
        a += v[k];
        b += (double)v[k] * v[k];
      }
    } else {
      f32x4 d = g4[i];
      for (int k = 0; k < 4; ++k) {
        a += d[k];
        b += (double)d[k] * ((v[k] - m) * rs);
      }
    }
  }
  for (long long i = (n4 << 2) + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float v = x[i];
    if (mode == 0) {
      a += v;
      b += (double)v * v;
    } else {
      a += g[i];
      b += (double)g[i] * ((v - m) * rs);
    }
  }
  block_sum2(a, b);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = a;
    part[2 * blockIdx.x + 1] = b;
  }
}

// mode 0: out = [mean, std (unbiased, torch.std default)]
// mode 1: out = [S1, S2] as floats (dL/dmu, dL/dsigma of AdaIN)
__global__ void __launch_bounds__(RED_THREADS) reduce2_final(const double* __restrict__ part, int nparts,
                                                             long long n, int mode, float* __restrict__ out) {
  double a = 0.0, b = 0.0;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) {
    a += part[2 * i];
    b += part[2 * i + 1];
  }
  block_sum2(a, b);
  if (threadIdx.x == 0) {
    if (mode == 0) {
      double mean = a / (double)n;
      double var = n > 1 ? (b - a * mean) / (double)(n - 1) : __builtin_nan("");
      out[0] = (float)mean;
      out[1] = (float)sqrt(var > 0.0 ? var : 0.0);
    } else {
      out[0] = (float)a;
      out[1] = (float)b;
    }
  }
}

__global__ void adain_fwd_kernel(const float* __restrict__ x, long long n, const float* __restrict__ mom,
                                 const float* __restrict__ mu, const float* __restrict__ sigma,
                                 float* __restrict__ y) {
  const float m = mom[0];
  const float a = sigma[0] / mom[1];
  const float c = mu[0];
  long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i + 3 < n) {
    f32x4 v = *reinterpret_cast<const f32x4*>(x + i);
    f32x4 r;
    for (int k = 0; k < 4; ++k) r[k] = (v[k] - m) * a + c;
    *reinterpret_cast<f32x4*>(y + i) = r;
  } else {
    for (; i < n; ++i) y[i] = (x[i] - m) * a + c;
  }
}

// dx = alpha*g + beta + gamma*(x - m) (+ acc), the common shape of every whole-tensor
// moment gradient:
//   AdaIN (sums = [S1, S2], sigma):  alpha = sigma/s, beta = -sigma*S1/(n s),
//                                    gamma = -sigma*S2/((n-1) s^2)
//   moments (dmean, dstd):           alpha = 0, beta = dmean/n, gamma = dstd/((n-1) s)
__global__ void affine_grad_kernel(const float* __restrict__ g, const float* __restrict__ x, long long n,
                                   const float* __restrict__ mom, int mode, const float* __restrict__ p0,
                                   const float* __restrict__ p1, const float* __restrict__ acc,
                                   float* __restrict__ dx, float* __restrict__ dmu, float* __restrict__ dsigma) {
  const float m = mom[0], s = mom[1];
  const float nn = (float)n, n1 = (float)(n - 1);
  float alpha, beta, gamma;
  if (mode == 0) {  // AdaIN: p0 = sums [S1, S2], p1 = sigma
    const float sig = p1[0];
    alpha = sig / s;
    beta = -sig * p0[0] / (nn * s);
    gamma = -sig * p0[1] / (n1 * s * s);
  } else {  // moments: p0 = dmean (nullable), p1 = dstd (nullable)
    alpha = 0.f;
    beta = p0 ? p0[0] / nn : 0.f;
    gamma = p1 ? p1[0] / (n1 * s) : 0.f;
  }
  long long i0 = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (mode == 0 && i0 == 0) {
    dmu[0] = p0[0];
    dsigma[0] = p0[1];
  }
  for (long long i = i0; i < n && i < i0 + 4; ++i) {
    float v = beta + gamma * (x[i] - m);
    if (mode == 0) v += alpha * g[i];
    if (acc) v += acc[i];
    dx[i] = v;
  }
}

// out[b][c] (+)= sum_t x[(b*T + t)*ld + c]; one thread per (b, c), T-loop coalesced over c.
__global__ void segsum_kernel(const float* __restrict__ x, long long ld, int B, int T, int C,
                              float* __restrict__ out, int accumulate) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  int b = blockIdx.y;
  if (c >= C) return;
  const float* p = x + (long long)b * T * ld + c;
  float s = 0.f;
  for (int t = 0; t < T; ++t) s += p[(long long)t * ld];
  float* o = out + (long long)b * C + c;
  *o = accumulate ? *o + s : s;
}

// out[b][c] = x[(b*T + t)*C + c]  (scatter = 1: dx[(b*T + t')*C + c] = t' == t ? d[b][c] : 0)
__global__ void step_select_kernel(const float* __restrict__ src, float* __restrict__ dst, int B, int T, int t,
                                   int C, int scatter) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (!scatter) {
    if (i >= (long long)B * C) return;
    int b = (int)(i / C), c = (int)(i % C);
    dst[i] = src[((long long)b * T + t) * C + c];
  } else {
    if (i >= (long long)B * T * C) return;
    int c = (int)(i % C);
    long long f = i / C;
    int b = (int)(f / T), tt = (int)(f % T);
    dst[i] = tt == t ? src[(long long)b * C + c] : 0.f;
  }
}

// One wave per row: y = x / ||x||_2 (norm kept for the backward).
__global__ void __launch_bounds__(256) rownorm_fwd_kernel(const float* __restrict__ x, int R, int C,
                                                          float* __restrict__ y, float* __restrict__ norms) {
  int r = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
  if (r >= R) return;
  const float* p = x + (long long)r * C;
  float s = 0.f;
  for (int c = l; c < C; c += 64) s += p[c] * p[c];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  float nrm = sqrtf(s), inv = 1.f / nrm;
  for (int c = l; c < C; c += 64) y[(long long)r * C + c] = p[c] * inv;
  if (l == 0) norms[r] = nrm;
}

// dx = (dy - y (y . dy)) / ||x||
__global__ void __launch_bounds__(256) rownorm_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ y,
                                                          const float* __restrict__ norms, int R, int C,
                                                          float* __restrict__ dx) {
  int r = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
  if (r >= R) return;
  const long long o = (long long)r * C;
  float d = 0.f;
  for (int c = l; c < C; c += 64) d += y[o + c] * dy[o + c];
  for (int k = 32; k > 0; k >>= 1) d += __shfl_xor(d, k, 64);
  float inv = 1.f / norms[r];
  for (int c = l; c < C; c += 64) dx[o + c] = (dy[o + c] - y[o + c] * d) * inv;
}

// dst[r][c] (row length Cd) = c < C ? src[r*lds + c] : 0, converted to dtype: zero-pads
// (Cd > C) or crops (Cd < C) the columns of a row-major matrix.
template <typename TO>
__global__ void pad_cols_kernel(const float* __restrict__ src, long long lds, TO* __restrict__ dst, int R, int C,
                                int Cd) {
  // rows on grid.y (strided past 65535), four consecutive columns per thread: no 64-bit
  // division per element
  const int c0 = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (c0 >= Cd) return;
  for (int r = blockIdx.y; r < R; r += gridDim.y) {
    const float* s = src + (long long)r * lds;
    TO* d = dst + (long long)r * Cd;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = c0 + k;
      if (c < Cd) d[c] = (TO)(c < C ? s[c] : 0.f);
    }
  }
}

// GELU (erf form, MLPMixer.py:9-14 nn.GELU) forward (bwd = 0: v = gelu(x)) or backward
// (bwd = 1: v = g * gelu'(x)) writing the fp32 result and/or its bf16 GEMM-operand twin in
// the same pass (either pointer may be null), four elements per thread.
__global__ void gelu_twin_kernel(const float* __restrict__ g, const float* __restrict__ x, float* __restrict__ y,
                                 bf16* __restrict__ y16, long long n, int bwd) {
  const long long i0 = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i0 >= n) return;
  float v[4];
  const bool full = i0 + 3 < n;
  if (full) {
    const f32x4 xv = *reinterpret_cast<const f32x4*>(x + i0);
    f32x4 gv = {1.f, 1.f, 1.f, 1.f};
    if (bwd) gv = *reinterpret_cast<const f32x4*>(g + i0);
    for (int k = 0; k < 4; ++k) {
      const float a = xv[k];
      const float cdf = 0.5f * (1.f + erf_nb(a * 0.70710678118654752f));
      v[k] = bwd ? gv[k] * (cdf + a * 0.39894228040143267794f * expf(-0.5f * a * a)) : a * cdf;
    }
    if (y) *reinterpret_cast<f32x4*>(y + i0) = f32x4{v[0], v[1], v[2], v[3]};
    if (y16) *reinterpret_cast<bf16x4*>(y16 + i0) = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
  } else {
    for (long long i = i0; i < n; ++i) {
      const float a = x[i];
      const float cdf = 0.5f * (1.f + erf_nb(a * 0.70710678118654752f));
      const float r = bwd ? g[i] * (cdf + a * 0.39894228040143267794f * expf(-0.5f * a * a)) : a * cdf;
      if (y) y[i] = r;
      if (y16) y16[i] = (bf16)r;
    }
  }
}

inline int blocks_for(long long n, int per) { return (int)((n + per - 1) / per); }

int reduce2(const float* x, const float* g, long long n, const float* mom, int mode, double* ws, float* out,
            hipStream_t s) {
  int nb = (int)std::min<long long>(RED_BLOCKS, std::max<long long>(1, (n + 4 * RED_THREADS - 1) / (4 * RED_THREADS)));
  reduce2_partial<<<nb, RED_THREADS, 0, s>>>(x, g, n, mom, mode, ws);
  reduce2_final<<<1, RED_THREADS, 0, s>>>(ws, nb, n, mode, out);
  return avc_check_launch(mode == 0 ? "avc_moments" : "avc_adain_bwd");
}

}  // namespace

extern "C" size_t avc_moments_ws(void) { return 2 * RED_BLOCKS; }

extern "C" int avc_moments(const float* x, long long n, double* ws, float* out, void* stream) {
  AVC_CHECK_ARG(n > 0 && x && ws && out, "avc_moments: bad arguments (n=%lld)", n);
  AVC_CHECK_ARG(((uintptr_t)x & 15) == 0, "avc_moments: x must be 16-byte aligned");
  return reduce2(x, nullptr, n, nullptr, 0, ws, out, (hipStream_t)stream);
}

extern "C" int avc_moments_bwd(const float* x, long long n, const float* mom, const float* dmean, const float* dstd,
                               const float* acc, float* dx, void* stream) {
  AVC_CHECK_ARG(n > 1 && x && mom && dx, "avc_moments_bwd: bad arguments (n=%lld)", n);
  affine_grad_kernel<<<blocks_for(n, 4 * 256), 256, 0, (hipStream_t)stream>>>(nullptr, x, n, mom, 1, dmean, dstd,
                                                                               acc, dx, nullptr, nullptr);
  return avc_check_launch("avc_moments_bwd");
}

extern "C" int avc_adain_fwd(const float* x, long long n, const float* mom, const float* mu, const float* sigma,
                             float* y, void* stream) {
  AVC_CHECK_ARG(n > 0 && x && mom && mu && sigma && y, "avc_adain_fwd: bad arguments (n=%lld)", n);
  AVC_CHECK_ARG((((uintptr_t)x | (uintptr_t)y) & 15) == 0, "avc_adain_fwd: x, y must be 16-byte aligned");
  adain_fwd_kernel<<<blocks_for(n, 4 * 256), 256, 0, (hipStream_t)stream>>>(x, n, mom, mu, sigma, y);
  return avc_check_launch("avc_adain_fwd");
}

extern "C" int avc_adain_bwd(const float* g, const float* x, long long n, const float* mom, const float* sigma,
                             double* ws, float* sums, float* dx, float* dmu, float* dsigma, void* stream) {
  AVC_CHECK_ARG(n > 1 && g && x && mom && sigma && ws && sums && dx && dmu && dsigma,
                "avc_adain_bwd: bad arguments (n=%lld)", n);
  AVC_CHECK_ARG((((uintptr_t)x | (uintptr_t)g) & 15) == 0, "avc_adain_bwd: x, g must be 16-byte aligned");
  hipStream_t s = (hipStream_t)stream;
  int rc = reduce2(x, g, n, mom, 1, ws, sums, s);
  if (rc) return rc;
  affine_grad_kernel<<<blocks_for(n, 4 * 256), 256, 0, s>>>(g, x, n, mom, 0, sums, sigma, nullptr, dx, dmu, dsigma);
  return avc_check_launch("avc_adain_bwd");
}

extern "C" int avc_segsum(const float* x, long long ld, int B, int T, int C, float* out, int accumulate,
                          void* stream) {
  AVC_CHECK_ARG(B > 0 && T > 0 && C > 0 && ld >= C, "avc_segsum: bad shape B=%d T=%d C=%d ld=%lld", B, T, C, ld);
  dim3 grid((C + 255) / 256, B);
  segsum_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(x, ld, B, T, C, out, accumulate);
  return avc_check_launch("avc_segsum");
}

extern "C" int avc_step_select(const float* src, float* dst, int B, int T, int t, int C, int scatter, void* stream) {
  AVC_CHECK_ARG(B > 0 && T > 0 && C > 0 && t >= 0 && t < T, "avc_step_select: bad shape B=%d T=%d t=%d C=%d", B, T,
                t, C);
  long long n = scatter ? (long long)B * T * C : (long long)B * C;
  step_select_kernel<<<blocks_for(n, 256), 256, 0, (hipStream_t)stream>>>(src, dst, B, T, t, C, scatter);
  return avc_check_launch("avc_step_select");
}

extern "C" int avc_rownorm_fwd(const float* x, int R, int C, float* y, float* norms, void* stream) {
  AVC_CHECK_ARG(R > 0 && C > 0, "avc_rownorm_fwd: bad shape R=%d C=%d", R, C);
  rownorm_fwd_kernel<<<(R + 3) / 4, 256, 0, (hipStream_t)stream>>>(x, R, C, y, norms);
  return avc_check_launch("avc_rownorm_fwd");
}

extern "C" int avc_rownorm_bwd(const float* dy, const float* y, const float* norms, int R, int C, float* dx,
                               void* stream) {
  AVC_CHECK_ARG(R > 0 && C > 0, "avc_rownorm_bwd: bad shape R=%d C=%d", R, C);
  rownorm_bwd_kernel<<<(R + 3) / 4, 256, 0, (hipStream_t)stream>>>(dy, y, norms, R, C, dx);
  return avc_check_launch("avc_rownorm_bwd");
}

// dst[r][c] += src[r*lds + c] for c < C (row length C): a padded product's crop accumulated into a
// gradient in one pass
__global__ void crop_add_kernel(const float* __restrict__ src, long long lds, float* __restrict__ dst, int R, int C) {
  const int c0 = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (c0 >= C) return;
  for (int r = blockIdx.y; r < R; r += gridDim.y) {
    const float* s = src + (long long)r * lds;
    float* d = dst + (long long)r * C;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (c0 + k < C) d[c0 + k] += s[c0 + k];
  }
}

extern "C" int avc_crop_add(const float* src, long long lds, float* dst, int R, int C, void* stream) {
  AVC_CHECK_ARG(src && dst && R > 0 && C > 0 && lds >= C, "avc_crop_add: bad shape R=%d C=%d", R, C);
  const dim3 grid((unsigned)((C + 1023) / 1024), (unsigned)std::min(R, 65535));
  crop_add_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(src, lds, dst, R, C);
  return avc_check_launch("avc_crop_add");
}

extern "C" int avc_pad_cols(const float* src, long long lds, void* dst, int dtype, int R, int C, int Cd,
                            void* stream) {
  AVC_CHECK_ARG(src && dst && R > 0 && C > 0 && Cd > 0 && lds >= C, "avc_pad_cols: bad shape R=%d C=%d Cd=%d", R,
                C, Cd);
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((unsigned)((Cd + 1023) / 1024), (unsigned)std::min(R, 65535));
  if (dtype == AVC_BF16)
    pad_cols_kernel<bf16><<<grid, 256, 0, s>>>(src, lds, reinterpret_cast<bf16*>(dst), R, C, Cd);
  else
    pad_cols_kernel<float><<<grid, 256, 0, s>>>(src, lds, reinterpret_cast<float*>(dst), R, C, Cd);
  return avc_check_launch("avc_pad_cols");
}

extern "C" int avc_gelu_twin(const float* g, const float* x, float* y, void* y16, long long n, int bwd,
                             void* stream) {
  AVC_CHECK_ARG(x && (y || y16) && n > 0 && (!bwd || g), "avc_gelu_twin: bad arguments (n=%lld)", n);
  AVC_CHECK_ARG((((uintptr_t)x | (uintptr_t)y | (uintptr_t)g) & 15) == 0 && ((uintptr_t)y16 & 7) == 0,
                "avc_gelu_twin: unaligned operand");
  gelu_twin_kernel<<<blocks_for(n, 4 * 256), 256, 0, (hipStream_t)stream>>>(g, x, y, reinterpret_cast<bf16*>(y16), n,
                                                                             bwd);
  return avc_check_launch("avc_gelu_twin");
}
