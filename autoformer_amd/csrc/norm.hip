// norm.hip — the MetaFormer (MetaConv / MetaPool) building blocks on frame-major data.
//
// Replaces: GroupNorm(1, C) (factory/Norm.py:53-60, used at MetaConv.py:23,35),
// nn.LayerNorm + GELU inside MLPMixer (MLPMixer.py:16-33), the Pooling token mixer
// AvgPool1d(3, 1, 1, count_include_pad=False)(x) - x (MetaPool.py:7-15), and einops'
// Rearrange('b c (h p1) (w p2) -> b (h w) (p1 p2 c)') (MLPMixer.py:73-75).
#include "common.h"

#include <algorithm>

namespace {

constexpr int NT = 256;

__device__ __forceinline__ float block_sum(float v, float* red) {
  v = warp_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
  return s;
}

// ---------------------------------------------------------------- GroupNorm(1 group)
// one block per sample; the sample is S = L*C contiguous elements, channel = idx % C
__global__ void gn_stats_kernel(const float* x, long long S, float eps, float* mean, float* rstd) {
  __shared__ float red[16];
  const float* xs = x + (long long)blockIdx.x * S;
  float s = 0.f;
  for (long long i = threadIdx.x; i < S; i += blockDim.x) s += xs[i];
  const float mu = block_sum(s, red) / (float)S;
  float q = 0.f;
  for (long long i = threadIdx.x; i < S; i += blockDim.x) {
    const float d = xs[i] - mu;
    q += d * d;
  }
  const float var = block_sum(q, red) / (float)S;
  if (threadIdx.x == 0) {
    mean[blockIdx.x] = mu;
    rstd[blockIdx.x] = 1.f / sqrtf(var + eps);
  }
}

__global__ void gn_apply_kernel(const float* x, long long S, int C, const float* gamma, const float* beta,
                                const float* mean, const float* rstd, float* y, long long total) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int b = (int)(i / S), c = (int)(i % C);
  y[i] = (x[i] - mean[b]) * rstd[b] * (gamma ? gamma[c] : 1.f) + (beta ? beta[c] : 0.f);
}

// per-sample sums of g = dy*gamma and g*xhat
__global__ void gn_bwd_sample_kernel(const float* dy, const float* x, const float* gamma, const float* mean,
                                     const float* rstd, long long S, int C, float* ws) {
  __shared__ float red[16];
  const long long o = (long long)blockIdx.x * S;
  const float mu = mean[blockIdx.x], rs = rstd[blockIdx.x];
  float s0 = 0.f, s1 = 0.f;
  for (long long i = threadIdx.x; i < S; i += blockDim.x) {
    const float g = dy[o + i] * (gamma ? gamma[(int)(i % C)] : 1.f);
    s0 += g;
    s1 += g * (x[o + i] - mu) * rs;
  }
  const float t0 = block_sum(s0, red);
  const float t1 = block_sum(s1, red);
  if (threadIdx.x == 0) {
    ws[2 * blockIdx.x] = t0 / (float)S;
    ws[2 * blockIdx.x + 1] = t1 / (float)S;
  }
}

__global__ void gn_bwd_dx_kernel(const float* dy, const float* x, const float* gamma, const float* mean,
                                 const float* rstd, const float* ws, long long S, int C, float* dx, long long total) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int b = (int)(i / S), c = (int)(i % C);
  const float rs = rstd[b];
  const float g = dy[i] * (gamma ? gamma[c] : 1.f);
  const float xh = (x[i] - mean[b]) * rs;
  dx[i] = rs * (g - ws[2 * b] - xh * ws[2 * b + 1]);
}

// per-channel partial sums of dy*xhat and dy over 128-row blocks of the (B*L, C) view
__global__ void gn_bwd_param_kernel(const float* dy, const float* x, const float* mean, const float* rstd, int L,
                                    int M, int C, float* ws) {
  __shared__ float red[2][4][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl, r0 = blockIdx.y * 128;
  float s0 = 0.f, s1 = 0.f;
  if (c < C) {
    for (int r = r0 + rl; r < min(M, r0 + 128); r += 4) {
      const int b = r / L;
      const long long i = (long long)r * C + c;
      s0 += dy[i] * (x[i] - mean[b]) * rstd[b];
      s1 += dy[i];
    }
  }
  red[0][rl][cl] = s0;
  red[1][rl][cl] = s1;
  __syncthreads();
  if (rl == 0 && c < C) {
    float* p = ws + ((long long)blockIdx.y * C + c) * 2;
    p[0] = red[0][0][cl] + red[0][1][cl] + red[0][2][cl] + red[0][3][cl];
    p[1] = red[1][0][cl] + red[1][1][cl] + red[1][2][cl] + red[1][3][cl];
  }
}

// Sum of the per-row-block (a, b) partials of 64 channels: 1024 threads = 64 channels x 16 row
// groups, each group with PF partial rows' loads in flight before it adds any (a channel per
// thread walking all partials serially was ~900 dependent loads at the mixer's 118K rows:
// 61 us per call, 2.1 ms of the MetaConv step), then the 16 groups reduced through LDS.
constexpr int PGR = 16, PF = 8;
__global__ void __launch_bounds__(1024) pair_final_kernel(const float* ws, int nrb, int C, float* da, float* db,
                                                          int acc) {
  __shared__ float red[2][PGR][64];
  const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  float s0 = 0.f, s1 = 0.f;
  if (c < C) {
    for (int i0 = grp; i0 < nrb; i0 += PGR * PF) {
      float x0[PF], x1[PF];
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        const int i = i0 + u * PGR;
        const long long o = ((long long)(i < nrb ? i : 0) * C + c) * 2;
        x0[u] = i < nrb ? ws[o] : 0.f;
        x1[u] = i < nrb ? ws[o + 1] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        s0 += x0[u];
        s1 += x1[u];
      }
    }
  }
  red[0][grp][cl] = s0;
  red[1][grp][cl] = s1;
  __syncthreads();
  if (grp == 0 && c < C) {
    s0 = s1 = 0.f;
#pragma unroll
    for (int g = 0; g < PGR; ++g) {
      s0 += red[0][g][cl];
      s1 += red[1][g][cl];
    }
    if (da) da[c] = acc ? da[c] + s0 : s0;
    if (db) db[c] = acc ? db[c] + s1 : s1;
  }
}

// Multi-block per-sample reductions (S % 4 == 0, 16-B aligned): a sample is split over NS blocks
// (B x NS ~ 1024 blocks instead of B = 64 blocks of one sample each), each writing a partial that a
// one-block finalize merges.  Statistics: (count, sum, M2 about the chunk mean), merged by Chan's
// formula; backward: the chunk sums of g = dy * gamma and g * xhat.
__device__ __forceinline__ float block_sum256(float v, float* red) {
  v = warp_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

__global__ void __launch_bounds__(256) gn_stats_part_kernel(const float* x, long long S, int chunk, float* part) {
  __shared__ float red[4];
  const int b = blockIdx.y, k = blockIdx.x;
  const long long c0 = (long long)k * chunk, c1 = min(S, c0 + chunk);
  const f32x4* xs = reinterpret_cast<const f32x4*>(x + (long long)b * S);
  float s = 0.f;
  for (long long i = c0 / 4 + threadIdx.x; i < c1 / 4; i += 256) {
    const f32x4 v = xs[i];
    s += v[0] + v[1] + v[2] + v[3];
  }
  const float n = (float)(c1 > c0 ? c1 - c0 : 0);
  const float sum = block_sum256(s, red);
  const float mu = n > 0.f ? sum / n : 0.f;
  float q = 0.f;
  for (long long i = c0 / 4 + threadIdx.x; i < c1 / 4; i += 256) {
    const f32x4 d = xs[i] - mu;
    q += d[0] * d[0] + d[1] * d[1] + d[2] * d[2] + d[3] * d[3];
  }
  const float m2 = block_sum256(q, red);
  if (threadIdx.x == 0) {
    float* p = part + ((long long)b * gridDim.x + k) * 3;
    p[0] = n;
    p[1] = sum;
    p[2] = m2;
  }
}

__global__ void gn_stats_final_kernel(const float* part, int B, int NS, long long S, float eps, float* mean,
                                      float* rstd) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float* p = part + (long long)b * NS * 3;
  double tot = 0.0;
  for (int k = 0; k < NS; ++k) tot += p[3 * k + 1];
  const double mu = tot / (double)S;
  double m2 = 0.0;
  for (int k = 0; k < NS; ++k) {
    const double n = p[3 * k];
    if (n > 0.0) {
      const double d = p[3 * k + 1] / n - mu;
      m2 += p[3 * k + 2] + n * d * d;
    }
  }
  mean[b] = (float)mu;
  rstd[b] = (float)(1.0 / sqrt(m2 / (double)S + (double)eps));
}

__global__ void __launch_bounds__(256) gn_bwd_sample_part_kernel(const float* dy, const float* x, const float* gamma,
                                                                 const float* mean, const float* rstd, long long S,
                                                                 int C, int chunk, float* part) {
  __shared__ float red[4];
  const int b = blockIdx.y, k = blockIdx.x;
  const long long c0 = (long long)k * chunk, c1 = min(S, c0 + chunk);
  const long long o = (long long)b * S;
  const float mu = mean[b], rs = rstd[b];
  float s0 = 0.f, s1 = 0.f;
  for (long long i4 = c0 / 4 + threadIdx.x; i4 < c1 / 4; i4 += 256) {
    const long long i = 4 * i4;
    const int c = (int)(i % C);
    f32x4 g = *reinterpret_cast<const f32x4*>(dy + o + i);
    if (gamma) g *= *reinterpret_cast<const f32x4*>(gamma + c);
    const f32x4 xh = (*reinterpret_cast<const f32x4*>(x + o + i) - mu) * rs;
    s0 += g[0] + g[1] + g[2] + g[3];
    s1 += g[0] * xh[0] + g[1] * xh[1] + g[2] * xh[2] + g[3] * xh[3];
  }
  const float t0 = block_sum256(s0, red);
  const float t1 = block_sum256(s1, red);
  if (threadIdx.x == 0) {
    float* p = part + ((long long)b * gridDim.x + k) * 2;
    p[0] = t0;
    p[1] = t1;
  }
}

__global__ void gn_bwd_sample_final_kernel(const float* part, int B, int NS, long long S, float* ws) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float t0 = 0.f, t1 = 0.f;
  for (int k = 0; k < NS; ++k) {
    t0 += part[((long long)b * NS + k) * 2];
    t1 += part[((long long)b * NS + k) * 2 + 1];
  }
  ws[2 * b] = t0 / (float)S;
  ws[2 * b + 1] = t1 / (float)S;
}

__global__ void gn_bwd_dx_v_kernel(const float* dy, const float* x, const float* gamma, const float* mean,
                                   const float* rstd, const float* ws, long long S, int C, float* dx,
                                   long long total4) {
  const long long i4 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i4 >= total4) return;
  const long long i = 4 * i4;
  const int b = (int)(i / S), c = (int)(i % C);
  const float rs = rstd[b];
  f32x4 g = *reinterpret_cast<const f32x4*>(dy + i);
  if (gamma) g *= *reinterpret_cast<const f32x4*>(gamma + c);
  const f32x4 xh = (*reinterpret_cast<const f32x4*>(x + i) - mean[b]) * rs;
  *reinterpret_cast<f32x4*>(dx + i) = rs * (g - ws[2 * b] - xh * ws[2 * b + 1]);
}

// ---------------------------------------------------------------- LayerNorm over rows of D
// one wave per row
__global__ void ln_fwd_kernel(const float* x, int R, int D, const float* gamma, const float* beta, float eps, float* y,
                              float* mean, float* rstd) {
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6), l = threadIdx.x & 63;
  if (row >= R) return;
  const float* xr = x + (long long)row * D;
  float s = 0.f;
  for (int i = l; i < D; i += 64) s += xr[i];
  const float mu = warp_sum(s) / (float)D;
  float q = 0.f;
  for (int i = l; i < D; i += 64) {
    const float d = xr[i] - mu;
    q += d * d;
  }
  const float rs = 1.f / sqrtf(warp_sum(q) / (float)D + eps);
  float* yr = y + (long long)row * D;
  for (int i = l; i < D; i += 64) yr[i] = (xr[i] - mu) * rs * (gamma ? gamma[i] : 1.f) + (beta ? beta[i] : 0.f);
  if (l == 0) {
    mean[row] = mu;
    rstd[row] = rs;
  }
}

__global__ void ln_bwd_dx_kernel(const float* dy, const float* x, const float* gamma, const float* mean,
                                 const float* rstd, int R, int D, float* dx) {
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6), l = threadIdx.x & 63;
  if (row >= R) return;
  const long long o = (long long)row * D;
  const float mu = mean[row], rs = rstd[row];
  float s0 = 0.f, s1 = 0.f;
  for (int i = l; i < D; i += 64) {
    const float g = dy[o + i] * (gamma ? gamma[i] : 1.f);
    s0 += g;
    s1 += g * (x[o + i] - mu) * rs;
  }
  const float m0 = warp_sum(s0) / (float)D, m1 = warp_sum(s1) / (float)D;
  for (int i = l; i < D; i += 64) {
    const float g = dy[o + i] * (gamma ? gamma[i] : 1.f);
    dx[o + i] = rs * (g - m0 - (x[o + i] - mu) * rs * m1);
  }
}

__global__ void ln_bwd_param_kernel(const float* dy, const float* x, const float* mean, const float* rstd, int R, int D,
                                    float* ws) {
  __shared__ float red[2][4][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl, r0 = blockIdx.y * 128;
  float s0 = 0.f, s1 = 0.f;
  if (c < D) {
    for (int r = r0 + rl; r < min(R, r0 + 128); r += 4) {
      const long long i = (long long)r * D + c;
      s0 += dy[i] * (x[i] - mean[r]) * rstd[r];
      s1 += dy[i];
    }
  }
  red[0][rl][cl] = s0;
  red[1][rl][cl] = s1;
  __syncthreads();
  if (rl == 0 && c < D) {
    float* p = ws + ((long long)blockIdx.y * D + c) * 2;
    p[0] = red[0][0][cl] + red[0][1][cl] + red[0][2][cl] + red[0][3][cl];
    p[1] = red[1][0][cl] + red[1][1][cl] + red[1][2][cl] + red[1][3][cl];
  }
}

// Vectorised forms (D % 4 == 0, 16-B aligned rows, D <= 256 * NV): one wave per row holds the
// row in registers (NV float4 per lane), so x is read from HBM once; outputs fp32 and / or bf16.
template <int NV>
__global__ void __launch_bounds__(256) ln_fwd_v_kernel(const float* x, int R, int D, const float* gamma,
                                                       const float* beta, float eps, float* y, bf16* y16, float* mean,
                                                       float* rstd) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63, D4 = D >> 2;
  if (row >= R) return;
  const f32x4* xr = reinterpret_cast<const f32x4*>(x + (long long)row * D);
  f32x4 v[NV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c4 = l + 64 * i;
    v[i] = c4 < D4 ? xr[c4] : f32x4{0.f, 0.f, 0.f, 0.f};
    s += v[i][0] + v[i][1] + v[i][2] + v[i][3];
  }
  const float mu = warp_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
    if (l + 64 * i < D4) {
      const f32x4 d = v[i] - mu;
      q += d[0] * d[0] + d[1] * d[1] + d[2] * d[2] + d[3] * d[3];
    }
  const float rs = 1.f / sqrtf(warp_sum(q) / (float)D + eps);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c4 = l + 64 * i;
    if (c4 >= D4) continue;
    const f32x4 g = gamma ? reinterpret_cast<const f32x4*>(gamma)[c4] : f32x4{1.f, 1.f, 1.f, 1.f};
    const f32x4 b = beta ? reinterpret_cast<const f32x4*>(beta)[c4] : f32x4{0.f, 0.f, 0.f, 0.f};
    const f32x4 o = (v[i] - mu) * rs * g + b;
    const long long off = (long long)row * D + 4 * c4;
    if (y) *reinterpret_cast<f32x4*>(y + off) = o;
    if (y16) *reinterpret_cast<bf16x4*>(y16 + off) = bf16x4{(bf16)o[0], (bf16)o[1], (bf16)o[2], (bf16)o[3]};
  }
  if (l == 0) {
    mean[row] = mu;
    rstd[row] = rs;
  }
}

// LayerNorm backward, dx and the parameter partials in one pass: 16 waves x lrb rows per block,
// each wave one row at a time (dy and x rows in registers); dx = rs (g - mean g - xh mean(g xh))
// (+ dres, the residual branch's gradient: the add after the norm folded in) to fp32 and / or
// bf16; per-lane column partials of dy*xh and dy summed over the block's rows, reduced through
// LDS into one (a, b) partial row per block for pair_final_kernel.
constexpr int LRB = 64;  // minimum rows per block (lrb grows with R so that pair_final sums <= ~512 rows)
template <int NV>
__global__ void __launch_bounds__(1024) ln_bwd_v_kernel(const float* dy, const float* x, const float* gamma,
                                                        const float* mean, const float* rstd, int R, int D,
                                                        const float* dres, float* dx, bf16* dx16, float* ws,
                                                        float* rsum, int lrb) {
  __shared__ f32x4 red[2][16][64 * NV];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, D4 = D >> 2;
  f32x4 pa[NV], pb[NV], gm[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    pa[i] = pb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int c4 = l + 64 * i;
    gm[i] = (gamma && c4 < D4) ? reinterpret_cast<const f32x4*>(gamma)[c4] : f32x4{1.f, 1.f, 1.f, 1.f};
  }
  const int r1 = min(R, (int)blockIdx.x * lrb + lrb);
  for (int row = blockIdx.x * lrb + w; row < r1; row += 16) {
    const long long o = (long long)row * D;
    const float mu = mean[row], rs = rstd[row];
    f32x4 dv[NV], xh[NV];
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c4 = l + 64 * i;
      if (c4 < D4) {
        dv[i] = reinterpret_cast<const f32x4*>(dy + o)[c4];
        xh[i] = (reinterpret_cast<const f32x4*>(x + o)[c4] - mu) * rs;
      } else {
        dv[i] = xh[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      const f32x4 g = dv[i] * gm[i], gx = g * xh[i];
      s0 += g[0] + g[1] + g[2] + g[3];
      s1 += gx[0] + gx[1] + gx[2] + gx[3];
      pa[i] += dv[i] * xh[i];
      pb[i] += dv[i];
    }
    const float m0 = warp_sum(s0) / (float)D, m1 = warp_sum(s1) / (float)D;
    float rsv = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c4 = l + 64 * i;
      if (c4 >= D4) continue;
      f32x4 d = rs * (dv[i] * gm[i] - m0 - xh[i] * m1);
      if (dres) d += reinterpret_cast<const f32x4*>(dres + o)[c4];
      if (dx) reinterpret_cast<f32x4*>(dx + o)[c4] = d;
      if (dx16) *reinterpret_cast<bf16x4*>(dx16 + o + 4 * c4) = bf16x4{(bf16)d[0], (bf16)d[1], (bf16)d[2], (bf16)d[3]};
      rsv += d[0] + d[1] + d[2] + d[3];
    }
    if (rsum) {  // the row's sum of dx (a later bias gradient over the transposed layout)
      rsv = warp_sum(rsv);
      if (l == 0) rsum[row] = rsv;
    }
  }
  if (!ws) return;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    red[0][w][l + 64 * i] = pa[i];
    red[1][w][l + 64 * i] = pb[i];
  }
  __syncthreads();
  // thread t: column quad c4 = t % (64 NV), quantity t / (64 NV)
  for (int t = threadIdx.x; t < 2 * 64 * NV; t += 1024) {
    const int qn = t / (64 * NV), c4 = t - qn * 64 * NV;
    if (c4 >= D4) continue;
    f32x4 a = red[qn][0][c4];
#pragma unroll
    for (int k = 1; k < 16; ++k) a += red[qn][k][c4];
    float* p = ws + ((long long)blockIdx.x * D + 4 * c4) * 2 + qn;
#pragma unroll
    for (int e = 0; e < 4; ++e) p[2 * e] = a[e];
  }
}

// GroupNorm apply, 4 channels per thread (C % 4 == 0): fp32 and / or the bf16 operand twin
__global__ void gn_apply_v_kernel(const float* x, long long S, int C, const float* gamma, const float* beta,
                                  const float* mean, const float* rstd, float* y, bf16* y16, long long total4) {
  const long long i4 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i4 >= total4) return;
  const long long i = 4 * i4;
  const int b = (int)(i / S), c = (int)(i % C);
  const f32x4 g = gamma ? *reinterpret_cast<const f32x4*>(gamma + c) : f32x4{1.f, 1.f, 1.f, 1.f};
  const f32x4 bt = beta ? *reinterpret_cast<const f32x4*>(beta + c) : f32x4{0.f, 0.f, 0.f, 0.f};
  const f32x4 o = (*reinterpret_cast<const f32x4*>(x + i) - mean[b]) * rstd[b] * g + bt;
  if (y) *reinterpret_cast<f32x4*>(y + i) = o;
  if (y16) *reinterpret_cast<bf16x4*>(y16 + i) = bf16x4{(bf16)o[0], (bf16)o[1], (bf16)o[2], (bf16)o[3]};
}

// ---------------------------------------------------------------- GELU (exact, erf) backward
__global__ void gelu_bwd_kernel(const float* g, const float* x, float* dx, long long n) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float v = x[i];
  const float cdf = 0.5f * (1.f + erf_nb(v * 0.70710678118654752f));
  const float pdf = 0.39894228040143267794f * expf(-0.5f * v * v);
  dx[i] = g[i] * (cdf + v * pdf);
}

// ---------------------------------------------------------------- Pooling token mixer
// frame-major x (B, L, C): y[t] = mean(x[t-1..t+1] inside [0, L)) - x[t]
__global__ void pool3_kernel(const float* x, float* y, int L, int C, long long total, int backward) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = (int)(i % C);
  const long long f = i / C;
  const int t = (int)(f % L);
  const long long base = (f - t) * C + c;  // frame 0 of this utterance, channel c
  float s = 0.f;
  if (!backward) {
    int n = 0;
    for (int d = -1; d <= 1; ++d) {
      const int tt = t + d;
      if (tt >= 0 && tt < L) {
        s += x[base + (long long)tt * C];
        ++n;
      }
    }
    y[i] = s / (float)n - x[i];
  } else {
    // x = dy; every output window containing t contributes dy[t'] / count(t')
    for (int d = -1; d <= 1; ++d) {
      const int tt = t + d;
      if (tt >= 0 && tt < L) {
        const int cnt = 1 + (tt > 0) + (tt < L - 1);
        s += x[base + (long long)tt * C] / (float)cnt;
      }
    }
    y[i] = s - x[i];
  }
}

// ---------------------------------------------------------------- MLP-Mixer patchify
// image rows = channel axis (C = H*ps), cols = frame axis (L = W*ps) of frame-major nf (B, L, C):
// P[b][h*W + w][p1*ps + p2] = nf[b][w*ps + p2][h*ps + p1]
template <typename TO>
__global__ void patchify_kernel(const float* nf, TO* P, int L, int C, int ps, long long total, int backward) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int W = L / ps, pp = ps * ps;
  const int e = (int)(i % pp);
  const long long pt = i / pp;
  const int np = (C / ps) * W;
  const int b = (int)(pt / np), patch = (int)(pt % np);
  const int h = patch / W, w = patch % W, p1 = e / ps, p2 = e % ps;
  const long long src = ((long long)b * L + (w * ps + p2)) * C + (h * ps + p1);
  if (!backward) P[i] = (TO)nf[src];
  else P[src] = (TO)nf[i];  // scatter back: P is the frame-major gradient, nf the patch gradient
}

// ---------------------------------------------------------------- batched transpose (+accumulate)
// dst[b][c][r] (+)= src[b][r][c] for r < R; dst rows are ld (>= R) long and r in [R, ld) is written
// 0 (the zero-padded patch count of the MLP-Mixer operands).  dst (fp32) and / or dst16 (bf16,
// the GEMM operand) -- one pass instead of a transpose followed by a pad / convert pass.
template <typename TS>
__global__ void btranspose_kernel(const TS* src, float* dst, bf16* dst16, int R, int C, int ld, int acc) {
  __shared__ float tile[32][33];
  const long long off = (long long)blockIdx.z * R * C, doff = (long long)blockIdx.z * C * ld;
  const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int y = ty; y < 32; y += 8) {
    const int r = r0 + y, c = c0 + tx;
    tile[y][tx] = (r < R && c < C) ? (float)src[off + (long long)r * C + c] : 0.f;
  }
  __syncthreads();
  for (int y = ty; y < 32; y += 8) {
    const int c = c0 + y, r = r0 + tx;
    if (c < C && r < ld) {
      const long long o = doff + (long long)c * ld + r;
      float v = tile[tx][y];
      if (dst) {
        if (acc) v += dst[o];
        dst[o] = v;
      }
      if (dst16) dst16[o] = (bf16)v;
    }
  }
}

// 64 x 64 tiles with 16-B loads (4 source columns) and 16-B fp32 / 8-B bf16 stores (4 output
// columns = 4 source rows): interior tiles of sources with C % 4 == 0 and outputs with ld % 4 == 0
// (16-B aligned bases); other tiles take the 32 x 32 element form above
template <typename TS>
__global__ void __launch_bounds__(256) btranspose64_kernel(const TS* src, float* dst, bf16* dst16, int R, int C,
                                                           int ld, int acc) {
  __shared__ float tile[64][65];
  const long long off = (long long)blockIdx.z * R * C, doff = (long long)blockIdx.z * C * ld;
  const int c0 = blockIdx.x * 64, r0 = blockIdx.y * 64;
  const int t = threadIdx.x, q = t & 15, rr = t >> 4;  // 16 quads per row, 16 rows per pass
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int r = r0 + rr + 16 * p, c = c0 + 4 * q;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (r < R && c < C) {
      if constexpr (sizeof(TS) == 4) {
        v = *reinterpret_cast<const f32x4*>(src + off + (long long)r * C + c);
      } else {
        const bf16x4 h = *reinterpret_cast<const bf16x4*>(src + off + (long long)r * C + c);
        v = f32x4{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) tile[rr + 16 * p][4 * q + k] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int cl = rr + 16 * p, c = c0 + cl, r = r0 + 4 * q;  // output row c, columns r .. r+3
    if (c >= C || r >= ld) continue;
    f32x4 v = {tile[4 * q][cl], tile[4 * q + 1][cl], tile[4 * q + 2][cl], tile[4 * q + 3][cl]};
    const long long o = doff + (long long)c * ld + r;
    if (dst) {
      if (acc) v += *reinterpret_cast<const f32x4*>(dst + o);
      *reinterpret_cast<f32x4*>(dst + o) = v;
    }
    if (dst16) *reinterpret_cast<bf16x4*>(dst16 + o) = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
  }
}

}  // namespace

#define GRID1(n) dim3(cdiv((n), 256)), dim3(256), 0, as_stream(stream)

static bool a16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }
static bool a8(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 7) == 0; }


extern "C" size_t avc_norm_ws(int rows, int C) { return (size_t)cdiv(rows, 64) * C * 2 + 1024; }

// samples split into NS chunks of >= 4096 elements, ~1024 blocks in all
static int gn_splits(int B, long long S) {
  long long ns = 1024 / B;
  if (ns < 1) ns = 1;
  const long long cap = S / 4096;
  if (ns > cap) ns = cap > 0 ? cap : 1;
  return (int)ns;
}

extern "C" int avc_group_norm_fwd2(const float* x, int B, long long S, int C, const float* gamma, const float* beta,
                                   float eps, float* y, void* y16, float* mean, float* rstd, float* ws,
                                   void* stream) {
  AVC_CHECK_ARG(x && (y || y16) && mean && rstd && B > 0 && S > 0 && C > 0 && S % C == 0,
                "avc_group_norm_fwd: bad args");
  hipStream_t s = as_stream(stream);
  const int ns = gn_splits(B, S);
  if (ws && S % 4 == 0 && a16(x) && ns > 1) {
    const int chunk = (int)(((S + ns - 1) / ns + 3) / 4 * 4);
    gn_stats_part_kernel<<<dim3(ns, B), 256, 0, s>>>(x, S, chunk, ws);
    gn_stats_final_kernel<<<cdiv(B, 64), 64, 0, s>>>(ws, B, ns, S, eps, mean, rstd);
  } else {
    gn_stats_kernel<<<B, 1024, 0, s>>>(x, S, eps, mean, rstd);
  }
  const long long total = (long long)B * S;
  bf16* o16 = static_cast<bf16*>(y16);
  if (C % 4 == 0 && a16(x) && a16(y) && a8(o16) && a16(gamma) && a16(beta)) {
    gn_apply_v_kernel<<<GRID1(total / 4)>>>(x, S, C, gamma, beta, mean, rstd, y, o16, total / 4);
  } else {
    AVC_CHECK_ARG(y && !y16, "avc_group_norm_fwd: the bf16 twin needs C %% 4 == 0 and aligned data");
    gn_apply_kernel<<<GRID1(total)>>>(x, S, C, gamma, beta, mean, rstd, y, total);
  }
  return avc_check_launch("avc_group_norm_fwd");
}

extern "C" int avc_group_norm_fwd(const float* x, int B, long long S, int C, const float* gamma, const float* beta,
                                  float eps, float* y, float* mean, float* rstd, void* stream) {
  return avc_group_norm_fwd2(x, B, S, C, gamma, beta, eps, y, nullptr, mean, rstd, nullptr, stream);
}

extern "C" int avc_group_norm_bwd(const float* dy, const float* x, const float* gamma, const float* mean,
                                  const float* rstd, int B, long long S, int C, float* dx, float* dgamma, float* dbeta,
                                  int accumulate, float* ws, void* stream) {
  AVC_CHECK_ARG(dy && x && mean && rstd && dx && ws && S % C == 0, "avc_group_norm_bwd: bad args");
  hipStream_t s = as_stream(stream);
  const int L = (int)(S / C), M = B * L;
  const int nrb = cdiv(M, 128);
  float* wsamp = ws + (size_t)nrb * C * 2;
  const long long total = (long long)B * S;
  const int ns = gn_splits(B, S);
  if (C % 4 == 0 && a16(dy) && a16(x) && a16(dx) && a16(gamma)) {
    float* part = wsamp + 2 * B;  // avc_norm_ws leaves room: nrb*C*2 + 2B + 2*B*ns << rows/64*C*2
    const int chunk = (int)(((S + ns - 1) / ns + 3) / 4 * 4);
    gn_bwd_sample_part_kernel<<<dim3(ns, B), 256, 0, s>>>(dy, x, gamma, mean, rstd, S, C, chunk, part);
    gn_bwd_sample_final_kernel<<<cdiv(B, 64), 64, 0, s>>>(part, B, ns, S, wsamp);
    gn_bwd_dx_v_kernel<<<cdiv(total / 4, 256), 256, 0, s>>>(dy, x, gamma, mean, rstd, wsamp, S, C, dx, total / 4);
  } else {
    gn_bwd_sample_kernel<<<B, 1024, 0, s>>>(dy, x, gamma, mean, rstd, S, C, wsamp);
    gn_bwd_dx_kernel<<<cdiv(total, 256), 256, 0, s>>>(dy, x, gamma, mean, rstd, wsamp, S, C, dx, total);
  }
  if (dgamma || dbeta) {
    gn_bwd_param_kernel<<<dim3(cdiv(C, 64), nrb), 256, 0, s>>>(dy, x, mean, rstd, L, M, C, ws);
    pair_final_kernel<<<cdiv(C, 64), 1024, 0, s>>>(ws, nrb, C, dgamma, dbeta, accumulate);
  }
  return avc_check_launch("avc_group_norm_bwd");
}

extern "C" int avc_layer_norm_fwd2(const float* x, int R, int D, const float* gamma, const float* beta, float eps,
                                   float* y, void* y16, float* mean, float* rstd, void* stream) {
  AVC_CHECK_ARG(x && (y || y16) && mean && rstd && R > 0 && D > 0, "avc_layer_norm_fwd: bad args");
  hipStream_t s = as_stream(stream);
  bf16* o16 = static_cast<bf16*>(y16);
  const bool v = D % 4 == 0 && D <= 512 && a16(x) && a16(y) && a8(o16) && a16(gamma) && a16(beta);
  if (v && D <= 256) ln_fwd_v_kernel<1><<<cdiv(R, 4), 256, 0, s>>>(x, R, D, gamma, beta, eps, y, o16, mean, rstd);
  else if (v) ln_fwd_v_kernel<2><<<cdiv(R, 4), 256, 0, s>>>(x, R, D, gamma, beta, eps, y, o16, mean, rstd);
  else {
    AVC_CHECK_ARG(y && !y16, "avc_layer_norm_fwd: the bf16 output needs D %% 4 == 0, D <= 512, aligned rows");
    ln_fwd_kernel<<<cdiv(R, 4), 256, 0, s>>>(x, R, D, gamma, beta, eps, y, mean, rstd);
  }
  return avc_check_launch("avc_layer_norm_fwd");
}

extern "C" int avc_layer_norm_fwd(const float* x, int R, int D, const float* gamma, const float* beta, float eps,
                                  float* y, float* mean, float* rstd, void* stream) {
  return avc_layer_norm_fwd2(x, R, D, gamma, beta, eps, y, nullptr, mean, rstd, stream);
}

extern "C" int avc_layer_norm_bwd2(const float* dy, const float* x, const float* gamma, const float* mean,
                                   const float* rstd, int R, int D, const float* dres, float* dx, void* dx16,
                                   float* row_sum, float* dgamma, float* dbeta, int accumulate, float* ws,
                                   void* stream) {
  AVC_CHECK_ARG(dy && x && mean && rstd && (dx || dx16) && ws && R > 0 && D > 0, "avc_layer_norm_bwd: bad args");
  hipStream_t s = as_stream(stream);
  bf16* o16 = static_cast<bf16*>(dx16);
  const bool v = D % 4 == 0 && D <= 512 && a16(dy) && a16(x) && a16(dx) && a8(o16) && a16(gamma) && a16(dres);
  if (v) {
    const bool par = dgamma || dbeta;
    // enough blocks for the chip, few enough partial rows for one pair_final pass
    const int lrb = std::max(LRB, (cdiv(R, 512) + 15) / 16 * 16), nrb = cdiv(R, lrb);
    if (D <= 256)
      ln_bwd_v_kernel<1><<<nrb, 1024, 0, s>>>(dy, x, gamma, mean, rstd, R, D, dres, dx, o16, par ? ws : nullptr,
                                              row_sum, lrb);
    else
      ln_bwd_v_kernel<2><<<nrb, 1024, 0, s>>>(dy, x, gamma, mean, rstd, R, D, dres, dx, o16, par ? ws : nullptr,
                                              row_sum, lrb);
    if (par) pair_final_kernel<<<cdiv(D, 64), 1024, 0, s>>>(ws, nrb, D, dgamma, dbeta, accumulate);
    return avc_check_launch("avc_layer_norm_bwd");
  }
  AVC_CHECK_ARG(dx && !dx16 && !dres && !row_sum,
                "avc_layer_norm_bwd: dres / bf16 output / row sums need D %% 4 == 0, D <= 512, aligned rows");
  return avc_layer_norm_bwd(dy, x, gamma, mean, rstd, R, D, dx, dgamma, dbeta, accumulate, ws, stream);
}

extern "C" int avc_layer_norm_bwd(const float* dy, const float* x, const float* gamma, const float* mean,
                                  const float* rstd, int R, int D, float* dx, float* dgamma, float* dbeta,
                                  int accumulate, float* ws, void* stream) {
  AVC_CHECK_ARG(dy && x && mean && rstd && dx && ws, "avc_layer_norm_bwd: bad args");
  hipStream_t s = as_stream(stream);
  ln_bwd_dx_kernel<<<cdiv(R, 4), 256, 0, s>>>(dy, x, gamma, mean, rstd, R, D, dx);
  if (dgamma || dbeta) {
    const int nrb = cdiv(R, 128);
    ln_bwd_param_kernel<<<dim3(cdiv(D, 64), nrb), 256, 0, s>>>(dy, x, mean, rstd, R, D, ws);
    pair_final_kernel<<<cdiv(D, 64), 1024, 0, s>>>(ws, nrb, D, dgamma, dbeta, accumulate);
  }
  return avc_check_launch("avc_layer_norm_bwd");
}

extern "C" int avc_gelu_bwd(const float* g, const float* x, float* dx, long long n, void* stream) {
  AVC_CHECK_ARG(g && x && dx, "avc_gelu_bwd: null");
  if (n == 0) return 0;
  gelu_bwd_kernel<<<GRID1(n)>>>(g, x, dx, n);
  return avc_check_launch("avc_gelu_bwd");
}

extern "C" int avc_pool3_mixer(const float* x, float* y, int B, int L, int C, int backward, void* stream) {
  AVC_CHECK_ARG(x && y && x != y, "avc_pool3_mixer: bad args");
  const long long total = (long long)B * L * C;
  pool3_kernel<<<GRID1(total)>>>(x, y, L, C, total, backward);
  return avc_check_launch("avc_pool3_mixer");
}

extern "C" int avc_patchify(const float* src, float* dst, int B, int L, int C, int ps, int backward, void* stream) {
  AVC_CHECK_ARG(src && dst && ps > 0 && L % ps == 0 && C % ps == 0, "avc_patchify: L and C must divide by patch");
  const long long total = (long long)B * L * C;
  patchify_kernel<float><<<GRID1(total)>>>(src, dst, L, C, ps, total, backward);
  return avc_check_launch("avc_patchify");
}

extern "C" int avc_patchify16(const float* src, void* dst, int B, int L, int C, int ps, void* stream) {
  AVC_CHECK_ARG(src && dst && ps > 0 && L % ps == 0 && C % ps == 0, "avc_patchify16: L and C must divide by patch");
  const long long total = (long long)B * L * C;
  patchify_kernel<bf16><<<GRID1(total)>>>(src, static_cast<bf16*>(dst), L, C, ps, total, 0);
  return avc_check_launch("avc_patchify16");
}

extern "C" int avc_transpose_batched(const float* src, float* dst, int B, int R, int C, int accumulate, void* stream) {
  AVC_CHECK_ARG(src && dst && src != dst, "avc_transpose_batched: bad args");
  if (C % 4 == 0 && R % 4 == 0 && a16(src) && a16(dst)) {
    dim3 g64(cdiv(C, 64), cdiv(R, 64), B);
    btranspose64_kernel<float><<<g64, 256, 0, as_stream(stream)>>>(src, dst, nullptr, R, C, R, accumulate);
    return avc_check_launch("avc_transpose_batched");
  }
  dim3 g(cdiv(C, 32), cdiv(R, 32), B);
  btranspose_kernel<float><<<g, 256, 0, as_stream(stream)>>>(src, dst, nullptr, R, C, R, accumulate);
  return avc_check_launch("avc_transpose_batched");
}

extern "C" int avc_transpose_batched2(const void* src, int src_dtype, float* dst, void* dst16, int B, int R, int C,
                                      int ld, int accumulate, void* stream) {
  AVC_CHECK_ARG(src && (dst || dst16) && (const void*)src != (const void*)dst && ld >= R && (!accumulate || dst) &&
                    (src_dtype == AVC_F32 || src_dtype == AVC_BF16),
                "avc_transpose_batched2: bad args");
  // rows r in [R, ld) of the output are zero: the 64-row tiles read zeros past R, so ld % 4 == 0 keeps
  // every 4-column output group inside one tile and the vector path applies
  const bool v64 = C % 4 == 0 && ld % 4 == 0 && a16(src) && a16(dst) && a8(dst16);
  if (v64) {
    dim3 g64(cdiv(C, 64), cdiv(ld, 64), B);
    if (src_dtype == AVC_BF16)
      btranspose64_kernel<bf16><<<g64, 256, 0, as_stream(stream)>>>(static_cast<const bf16*>(src), dst,
                                                                    reinterpret_cast<bf16*>(dst16), R, C, ld,
                                                                    accumulate);
    else
      btranspose64_kernel<float><<<g64, 256, 0, as_stream(stream)>>>(static_cast<const float*>(src), dst,
                                                                     reinterpret_cast<bf16*>(dst16), R, C, ld,
                                                                     accumulate);
    return avc_check_launch("avc_transpose_batched2");
  }
  dim3 g(cdiv(C, 32), cdiv(ld, 32), B);
  if (src_dtype == AVC_BF16)
    btranspose_kernel<bf16><<<g, 256, 0, as_stream(stream)>>>(static_cast<const bf16*>(src), dst,
                                                              reinterpret_cast<bf16*>(dst16), R, C, ld, accumulate);
  else
    btranspose_kernel<float><<<g, 256, 0, as_stream(stream)>>>(static_cast<const float*>(src), dst,
                                                               reinterpret_cast<bf16*>(dst16), R, C, ld, accumulate);
  return avc_check_launch("avc_transpose_batched2");
}
