// bn.hip — BatchNorm1d (training mode) + activation, forward and backward, on
// frame-major [M][C] activations (M = B*T frames).
//
// Replaces nn.BatchNorm1d.forward/backward at factory/AutoVC.py:38,91,138,154,169 and the
// F.relu / torch.tanh that follow (AutoVC.py:51,107,175).  Batch statistics come from
// the producing GEMM's epilogue (gemm.hip bn_partial: per 128-row tile (sum, M2)); they
// are merged here with Chan's parallel-variance formula, so no extra pass over the
// activations is needed on the forward.
#include "common.h"

namespace {

constexpr int PTILE = 128;  // rows per partial (must match gemm.hip BM)

__global__ void bn_finalize_kernel(const float* partial, int M, int C, const float* gamma, const float* beta,
                                   float* rmean, float* rvar, long long* nbt, float momentum, float eps,
                                   float* mean_out, float* rstd_out, float* scale, float* shift) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.x == 0 && threadIdx.x == 0 && nbt) *nbt += 1;
  if (c >= C) return;
  const int nt = (M + PTILE - 1) / PTILE;
  double n = 0.0, mean = 0.0, m2 = 0.0;
  for (int t = 0; t < nt; ++t) {
    double nb = (double)min(PTILE, M - t * PTILE);
    double sb = partial[((long long)t * C + c) * 2 + 0];
    double qb = partial[((long long)t * C + c) * 2 + 1];
    double mb = sb / nb;
    double tot = n + nb;
    double d = mb - mean;
    mean += d * nb / tot;
    m2 += qb + d * d * n * nb / tot;
    n = tot;
  }
  double var = m2 / n;
  float rstd = (float)(1.0 / sqrt(var + (double)eps));
  float g = gamma ? gamma[c] : 1.f;
  float b = beta ? beta[c] : 0.f;
  mean_out[c] = (float)mean;
  rstd_out[c] = rstd;
  scale[c] = g * rstd;
  shift[c] = b - (float)mean * g * rstd;
  if (rmean) {
    double unb = n > 1.0 ? m2 / (n - 1.0) : var;
    rmean[c] = (1.f - momentum) * rmean[c] + momentum * (float)mean;
    rvar[c] = (1.f - momentum) * rvar[c] + momentum * (float)unb;
  }
}

__global__ void bn_eval_kernel(const float* rmean, const float* rvar, const float* gamma, const float* beta, int C,
                               float eps, float* mean_out, float* rstd_out, float* scale, float* shift) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float rstd = 1.f / sqrtf(rvar[c] + eps);
  float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
  mean_out[c] = rmean[c];
  rstd_out[c] = rstd;
  scale[c] = g * rstd;
  shift[c] = b - rmean[c] * g * rstd;
}

// plain stats pass (for inputs not produced by avc_gemm): one block per 128-row tile x 256 cols
__global__ void bn_stats_kernel(const float* y, long long ld, int M, int C, float* partial) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  int r0 = blockIdx.y * PTILE;
  if (c >= C) return;
  int r1 = min(M, r0 + PTILE);
  float s = 0.f;
  for (int r = r0; r < r1; ++r) s += y[(long long)r * ld + c];
  float mean = s / (float)(r1 - r0);
  float q = 0.f;
  for (int r = r0; r < r1; ++r) {
    float d = y[(long long)r * ld + c] - mean;
    q += d * d;
  }
  partial[((long long)blockIdx.y * C + c) * 2 + 0] = s;
  partial[((long long)blockIdx.y * C + c) * 2 + 1] = q;
}

__global__ void bn_apply_kernel(const float* __restrict__ y, const float* __restrict__ scale,
                                const float* __restrict__ shift, const float* __restrict__ res, float* __restrict__ out,
                                long long total4, int C, int act) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total4) return;
  long long e = i * 4;
  int c = (int)(e % C);
  f32x4 v = *reinterpret_cast<const f32x4*>(y + e);
  f32x4 sc = *reinterpret_cast<const f32x4*>(scale + c);
  f32x4 sh = *reinterpret_cast<const f32x4*>(shift + c);
  f32x4 o;
#pragma unroll
  for (int k = 0; k < 4; ++k) o[k] = act_fwd(v[k] * sc[k] + sh[k], act);
  if (res) {
    f32x4 r = *reinterpret_cast<const f32x4*>(res + e);
    o += r;
  }
  *reinterpret_cast<f32x4*>(out + e) = o;
}

__global__ void bn_apply1_kernel(const float* __restrict__ y, const float* __restrict__ scale,
                                 const float* __restrict__ shift, const float* __restrict__ res, float* __restrict__ out,
                                 long long total, int C, int act) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = (int)(i % C);
  float o = act_fwd(y[i] * scale[c] + shift[c], act);
  out[i] = res ? o + res[i] : o;
}

// backward reduce: per (row block of RB rows, 64 channels) partial sums of dz, dz*yhat, yhat.
constexpr int RB = 128;
__global__ void bn_bwd_reduce_kernel(const float* __restrict__ dA, const float* __restrict__ a,
                                     const float* __restrict__ y, const float* __restrict__ mean,
                                     const float* __restrict__ rstd, int M, int C, int act, float* ws) {
  __shared__ float red[3][4][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int r0 = blockIdx.y * RB;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f;
  if (c < C) {
    const float mu = mean[c], rs = rstd[c];
    const int r1 = min(M, r0 + RB);
    for (int r = r0 + rl; r < r1; r += 4) {
      long long idx = (long long)r * C + c;
      float dz = act_bwd_from_out(dA[idx], a[idx], act);
      float yh = (y[idx] - mu) * rs;
      s0 += dz;
      s1 += dz * yh;
      s2 += yh;
    }
  }
  red[0][rl][cl] = s0;
  red[1][rl][cl] = s1;
  red[2][rl][cl] = s2;
  __syncthreads();
  if (rl == 0 && c < C) {
    float* p = ws + ((long long)blockIdx.y * C + c) * 3;
    p[0] = red[0][0][cl] + red[0][1][cl] + red[0][2][cl] + red[0][3][cl];
    p[1] = red[1][0][cl] + red[1][1][cl] + red[1][2][cl] + red[1][3][cl];
    p[2] = red[2][0][cl] + red[2][1][cl] + red[2][2][cl] + red[2][3][cl];
  }
}

__global__ void bn_bwd_finalize_kernel(const float* ws, int nrb, int M, int C, const float* gamma,
                                       const float* rstd, float* coef, float* dgamma, float* dbeta, float* dbias,
                                       int acc) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s0 = 0, s1 = 0, s2 = 0;
  for (int b = 0; b < nrb; ++b) {
    const float* p = ws + ((long long)b * C + c) * 3;
    s0 += p[0];
    s1 += p[1];
    s2 += p[2];
  }
  const float g = gamma ? gamma[c] : 1.f;
  const float k1 = g * rstd[c];
  const float invn = 1.f / (float)M;
  coef[c * 3 + 0] = k1;
  coef[c * 3 + 1] = (float)s0 * invn;
  coef[c * 3 + 2] = (float)s1 * invn;
  const float gb = -k1 * (float)(s1 * s2) * invn;
  if (dgamma) dgamma[c] = acc ? dgamma[c] + (float)s1 : (float)s1;
  if (dbeta) dbeta[c] = acc ? dbeta[c] + (float)s0 : (float)s0;
  if (dbias) dbias[c] = acc ? dbias[c] + gb : gb;
}

__global__ void bn_bwd_apply_kernel(const float* __restrict__ dA, const float* __restrict__ a,
                                    const float* __restrict__ y, const float* __restrict__ mean,
                                    const float* __restrict__ rstd, const float* __restrict__ coef, long long total4,
                                    int C, int act, float* __restrict__ dy) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total4) return;
  long long e = i * 4;
  int c = (int)(e % C);
  f32x4 g = *reinterpret_cast<const f32x4*>(dA + e);
  f32x4 av = *reinterpret_cast<const f32x4*>(a + e);
  f32x4 yv = *reinterpret_cast<const f32x4*>(y + e);
  f32x4 o;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float* cf = coef + (c + k) * 3;
    float dz = act_bwd_from_out(g[k], av[k], act);
    float yh = (yv[k] - mean[c + k]) * rstd[c + k];
    o[k] = cf[0] * (dz - cf[1] - yh * cf[2]);
  }
  *reinterpret_cast<f32x4*>(dy + e) = o;
}

__global__ void bn_bwd_apply1_kernel(const float* __restrict__ dA, const float* __restrict__ a,
                                     const float* __restrict__ y, const float* __restrict__ mean,
                                     const float* __restrict__ rstd, const float* __restrict__ coef, long long total,
                                     int C, int act, float* __restrict__ dy) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = (int)(i % C);
  const float* cf = coef + c * 3;
  const float dz = act_bwd_from_out(dA[i], a[i], act);
  const float yh = (y[i] - mean[c]) * rstd[c];
  dy[i] = cf[0] * (dz - cf[1] - yh * cf[2]);
}

// column sums: partial per 128-row block, then finalize
__global__ void colsum_partial_kernel(const float* x, long long ld, int M, int N, float* ws) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int r0 = blockIdx.y * RB;
  float s = 0.f;
  if (c < N) {
    const int r1 = min(M, r0 + RB);
    for (int r = r0 + rl; r < r1; r += 4) s += x[(long long)r * ld + c];
  }
  red[rl][cl] = s;
  __syncthreads();
  if (rl == 0 && c < N) ws[(long long)blockIdx.y * N + c] = red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl];
}

__global__ void colsum_final_kernel(const float* ws, int nrb, int N, float* out, int accumulate) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= N) return;
  float s = 0.f;
  for (int b = 0; b < nrb; ++b) s += ws[(long long)b * N + c];
  out[c] = accumulate ? out[c] + s : s;
}

}  // namespace

extern "C" int avc_bn_finalize(const float* partial, int M, int C, const float* gamma, const float* beta,
                               float* running_mean, float* running_var, long long* nbt, float momentum, float eps,
                               float* mean, float* rstd, float* scale, float* shift, void* stream) {
  AVC_CHECK_ARG(partial && mean && rstd && scale && shift && M > 0 && C > 0, "avc_bn_finalize: bad args");
  bn_finalize_kernel<<<cdiv(C, 256), 256, 0, as_stream(stream)>>>(partial, M, C, gamma, beta, running_mean,
                                                                   running_var, nbt, momentum, eps, mean, rstd,
                                                                   scale, shift);
  return avc_check_launch("avc_bn_finalize");
}

extern "C" int avc_bn_eval(const float* running_mean, const float* running_var, const float* gamma, const float* beta,
                           int C, float eps, float* mean, float* rstd, float* scale, float* shift, void* stream) {
  AVC_CHECK_ARG(running_mean && running_var && mean && rstd && scale && shift, "avc_bn_eval: bad args");
  bn_eval_kernel<<<cdiv(C, 256), 256, 0, as_stream(stream)>>>(running_mean, running_var, gamma, beta, C, eps, mean,
                                                               rstd, scale, shift);
  return avc_check_launch("avc_bn_eval");
}

extern "C" int avc_bn_stats(const float* y, long long ld, int M, int C, float* partial, void* stream) {
  AVC_CHECK_ARG(y && partial && M > 0 && C > 0 && ld >= C, "avc_bn_stats: bad args");
  dim3 grid(cdiv(C, 256), cdiv(M, PTILE));
  bn_stats_kernel<<<grid, 256, 0, as_stream(stream)>>>(y, ld, M, C, partial);
  return avc_check_launch("avc_bn_stats");
}

extern "C" int avc_bn_apply(const float* y, const float* scale, const float* shift, const float* residual, float* out,
                            int M, int C, int act, void* stream) {
  AVC_CHECK_ARG(y && scale && shift && out && C > 0, "avc_bn_apply: bad args");
  const long long total = (long long)M * C;
  if (total == 0) return 0;
  if (C % 4 == 0)
    bn_apply_kernel<<<cdiv(total / 4, 256), 256, 0, as_stream(stream)>>>(y, scale, shift, residual, out, total / 4, C,
                                                                        act);
  else
    bn_apply1_kernel<<<cdiv(total, 256), 256, 0, as_stream(stream)>>>(y, scale, shift, residual, out, total, C, act);
  return avc_check_launch("avc_bn_apply");
}

extern "C" size_t avc_bn_bwd_ws(int M, int C) { return (size_t)cdiv(M, RB) * C * 3 + (size_t)C * 3; }

extern "C" int avc_bn_bwd(const float* dA, const float* a, const float* y, const float* mean, const float* rstd,
                          const float* gamma, int M, int C, int act, float* dy, float* dgamma, float* dbeta,
                          float* dbias, int accumulate, float* ws, void* stream) {
  AVC_CHECK_ARG(dA && a && y && mean && rstd && dy && ws && C > 0, "avc_bn_bwd: bad args");
  hipStream_t s = as_stream(stream);
  const int nrb = cdiv(M, RB);
  dim3 grid(cdiv(C, 64), nrb);
  bn_bwd_reduce_kernel<<<grid, 256, 0, s>>>(dA, a, y, mean, rstd, M, C, act, ws);
  float* coef = ws + (size_t)nrb * C * 3;
  bn_bwd_finalize_kernel<<<cdiv(C, 256), 256, 0, s>>>(ws, nrb, M, C, gamma, rstd, coef, dgamma, dbeta, dbias,
                                                       accumulate);
  const long long total = (long long)M * C;
  if (C % 4 == 0)
    bn_bwd_apply_kernel<<<cdiv(total / 4, 256), 256, 0, s>>>(dA, a, y, mean, rstd, coef, total / 4, C, act, dy);
  else
    bn_bwd_apply1_kernel<<<cdiv(total, 256), 256, 0, s>>>(dA, a, y, mean, rstd, coef, total, C, act, dy);
  return avc_check_launch("avc_bn_bwd");
}

extern "C" size_t avc_colsum_ws(int M, int N) { return (size_t)cdiv(M, RB) * N; }

extern "C" int avc_colsum(const float* x, long long ld, int M, int N, float* out, int accumulate, float* ws,
                          void* stream) {
  AVC_CHECK_ARG(x && out && ws && ld >= N, "avc_colsum: bad args");
  hipStream_t s = as_stream(stream);
  const int nrb = cdiv(M, RB);
  colsum_partial_kernel<<<dim3(cdiv(N, 64), nrb), 256, 0, s>>>(x, ld, M, N, ws);
  colsum_final_kernel<<<cdiv(N, 256), 256, 0, s>>>(ws, nrb, N, out, accumulate);
  return avc_check_launch("avc_colsum");
}
