// norm.hip — the MetaFormer (MetaConv / MetaPool) building blocks on frame-major data.
//
// Replaces: GroupNorm(1, C) (factory/Norm.py:53-60, used at MetaConv.py:23,35),
// nn.LayerNorm + GELU inside MLPMixer (MLPMixer.py:16-33), the Pooling token mixer
// AvgPool1d(3, 1, 1, count_include_pad=False)(x) - x (MetaPool.py:7-15), and einops'
// Rearrange('b c (h p1) (w p2) -> b (h w) (p1 p2 c)') (MLPMixer.py:73-75).
#include "common.h"

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

// ---------------------------------------------------------------- GELU (exact, erf) backward
__global__ void gelu_bwd_kernel(const float* g, const float* x, float* dx, long long n) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float v = x[i];
  const float cdf = 0.5f * (1.f + erff(v * 0.70710678118654752f));
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
__global__ void patchify_kernel(const float* nf, float* P, int L, int C, int ps, long long total, int backward) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int W = L / ps, pp = ps * ps;
  const int e = (int)(i % pp);
  const long long pt = i / pp;
  const int np = (C / ps) * W;
  const int b = (int)(pt / np), patch = (int)(pt % np);
  const int h = patch / W, w = patch % W, p1 = e / ps, p2 = e % ps;
  const long long src = ((long long)b * L + (w * ps + p2)) * C + (h * ps + p1);
  if (!backward) P[i] = nf[src];
  else P[src] = nf[i];  // scatter back: P is the frame-major gradient, nf the patch gradient
}

// ---------------------------------------------------------------- batched transpose (+accumulate)
// dst[b][c][r] (+)= src[b][r][c] for r < R; dst rows are ld (>= R) long and r in [R, ld) is written
// 0 (the zero-padded patch count of the MLP-Mixer operands).  dst (fp32) and / or dst16 (bf16,
// the GEMM operand) -- one pass instead of a transpose followed by a pad / convert pass.
__global__ void btranspose_kernel(const float* src, float* dst, bf16* dst16, int R, int C, int ld, int acc) {
  __shared__ float tile[32][33];
  const long long off = (long long)blockIdx.z * R * C, doff = (long long)blockIdx.z * C * ld;
  const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int y = ty; y < 32; y += 8) {
    const int r = r0 + y, c = c0 + tx;
    tile[y][tx] = (r < R && c < C) ? src[off + (long long)r * C + c] : 0.f;
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

}  // namespace

#define GRID1(n) dim3(cdiv((n), 256)), dim3(256), 0, as_stream(stream)

extern "C" size_t avc_norm_ws(int rows, int C) { return (size_t)cdiv(rows, 128) * C * 2 + 1024; }

extern "C" int avc_group_norm_fwd(const float* x, int B, long long S, int C, const float* gamma, const float* beta,
                                  float eps, float* y, float* mean, float* rstd, void* stream) {
  AVC_CHECK_ARG(x && y && mean && rstd && B > 0 && S > 0 && C > 0 && S % C == 0, "avc_group_norm_fwd: bad args");
  gn_stats_kernel<<<B, 1024, 0, as_stream(stream)>>>(x, S, eps, mean, rstd);
  const long long total = (long long)B * S;
  gn_apply_kernel<<<GRID1(total)>>>(x, S, C, gamma, beta, mean, rstd, y, total);
  return avc_check_launch("avc_group_norm_fwd");
}

extern "C" int avc_group_norm_bwd(const float* dy, const float* x, const float* gamma, const float* mean,
                                  const float* rstd, int B, long long S, int C, float* dx, float* dgamma, float* dbeta,
                                  int accumulate, float* ws, void* stream) {
  AVC_CHECK_ARG(dy && x && mean && rstd && dx && ws && S % C == 0, "avc_group_norm_bwd: bad args");
  hipStream_t s = as_stream(stream);
  const int L = (int)(S / C), M = B * L;
  const int nrb = cdiv(M, 128);
  float* wsamp = ws + (size_t)nrb * C * 2;
  gn_bwd_sample_kernel<<<B, 1024, 0, s>>>(dy, x, gamma, mean, rstd, S, C, wsamp);
  const long long total = (long long)B * S;
  gn_bwd_dx_kernel<<<cdiv(total, 256), 256, 0, s>>>(dy, x, gamma, mean, rstd, wsamp, S, C, dx, total);
  if (dgamma || dbeta) {
    gn_bwd_param_kernel<<<dim3(cdiv(C, 64), nrb), 256, 0, s>>>(dy, x, mean, rstd, L, M, C, ws);
    pair_final_kernel<<<cdiv(C, 64), 1024, 0, s>>>(ws, nrb, C, dgamma, dbeta, accumulate);
  }
  return avc_check_launch("avc_group_norm_bwd");
}

extern "C" int avc_layer_norm_fwd(const float* x, int R, int D, const float* gamma, const float* beta, float eps,
                                  float* y, float* mean, float* rstd, void* stream) {
  AVC_CHECK_ARG(x && y && mean && rstd && R > 0 && D > 0, "avc_layer_norm_fwd: bad args");
  ln_fwd_kernel<<<cdiv(R, 4), 256, 0, as_stream(stream)>>>(x, R, D, gamma, beta, eps, y, mean, rstd);
  return avc_check_launch("avc_layer_norm_fwd");
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
  patchify_kernel<<<GRID1(total)>>>(src, dst, L, C, ps, total, backward);
  return avc_check_launch("avc_patchify");
}

extern "C" int avc_transpose_batched(const float* src, float* dst, int B, int R, int C, int accumulate, void* stream) {
  AVC_CHECK_ARG(src && dst && src != dst, "avc_transpose_batched: bad args");
  dim3 g(cdiv(C, 32), cdiv(R, 32), B);
  btranspose_kernel<<<g, 256, 0, as_stream(stream)>>>(src, dst, nullptr, R, C, R, accumulate);
  return avc_check_launch("avc_transpose_batched");
}

extern "C" int avc_transpose_batched2(const float* src, float* dst, void* dst16, int B, int R, int C, int ld,
                                      int accumulate, void* stream) {
  AVC_CHECK_ARG(src && (dst || dst16) && (const void*)src != (const void*)dst && ld >= R && (!accumulate || dst),
                "avc_transpose_batched2: bad args");
  dim3 g(cdiv(C, 32), cdiv(ld, 32), B);
  btranspose_kernel<<<g, 256, 0, as_stream(stream)>>>(src, dst, reinterpret_cast<bf16*>(dst16), R, C, ld, accumulate);
  return avc_check_launch("avc_transpose_batched2");
}
