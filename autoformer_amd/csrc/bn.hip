// bn.hip — BatchNorm1d (training mode) + activation, forward and backward, on
// frame-major [M][C] activations (M = B*T frames).
//
// Replaces nn.BatchNorm1d.forward/backward at factory/AutoVC.py:38,91,138,154,169 and the
// F.relu / torch.tanh that follow (AutoVC.py:51,107,175).  Batch statistics come from
// the producing GEMM's epilogue (gemm.hip bn_partial: per 128-row tile (sum, M2)); they
// are merged here with Chan's parallel-variance formula, so no extra pass over the
// activations is needed on the forward.
#include "common.h"
#include "bn_internal.h"

#include <atomic>
#include <mutex>
#include <type_traits>

namespace {

using namespace avcbn;

constexpr int PTILE = 128;  // rows per partial (must match gemm.hip BM)

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// One block per 64 channels; 4 row-groups of 64 threads stride over the per-tile partials
// (independent loads, no serial chain).  Merge = two passes over the partials:
//   mean = sum_t s_t / n;   M2 = sum_t [ q_t + n_t (s_t / n_t - mean)^2 ]   (Chan, parallel form)
// 256-thread blocks: a 1024-thread finalize block needs 16 free wave slots on one CU and waits
// behind the side stream's weight-gradient GEMMs (measured 14.8 us per backward finalize in the
// C2 step); 4 row groups x 64 channels start anywhere (FG, strided_sums: bn_internal.h)

__global__ void __launch_bounds__(256) bn_finalize_kernel(const float* __restrict__ partial, int M, int C,
                                                          const float* gamma, const float* beta, float* rmean,
                                                          float* rvar, long long* nbt, float momentum, float eps,
                                                          float* mean_out, float* rstd_out, float* scale,
                                                          float* shift) {
  __shared__ float red[FG * 64];
  const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  if (blockIdx.x == 0 && threadIdx.x == 0 && nbt) *nbt += 1;
  const int nt = (M + PTILE - 1) / PTILE;
  const bool cv = c < C;
  float mean, m2;
  chan_merge<16, false>(partial, nt, C, c, cv, grp, FG, cl, 64, M, PTILE, red, mean, m2);
  if (grp != 0 || !cv) return;
  const float n = (float)M;
  const float var = m2 / n;
  const float rstd = 1.f / sqrtf(var + eps);
  const float g = gamma ? gamma[c] : 1.f;
  const float b = beta ? beta[c] : 0.f;
  mean_out[c] = mean;
  rstd_out[c] = rstd;
  scale[c] = g * rstd;
  shift[c] = b - mean * g * rstd;
  if (rmean) {
    const float unb = n > 1.f ? m2 / (n - 1.f) : var;
    rmean[c] = (1.f - momentum) * rmean[c] + momentum * mean;
    rvar[c] = (1.f - momentum) * rvar[c] + momentum * unb;
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

// plain stats pass (for inputs not produced by avc_gemm, e.g. the Discriminator's LeakyReLU
// outputs): per 128-row tile and channel (sum, M2).  256 threads = 64 channels x 4 row groups of
// 32 rows; a thread loads its 32 values together into registers, the tile mean comes from the
// four groups' sums through LDS, and M2 from the same registers (one pass over memory; the
// previous one-thread-per-column form walked 2 x 128 dependent loads: 38 us per call at C = 44)
__global__ void __launch_bounds__(256) bn_stats_kernel(const float* __restrict__ y, long long ld, int M, int C,
                                                       float* __restrict__ partial) {
  __shared__ float red[2][4][64];
  const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int r0 = blockIdx.y * PTILE, n = min(M - r0, PTILE);
  const bool cv = c < C;
  float v[32];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const int r = grp * 32 + i;
    v[i] = (cv && r < n) ? y[(long long)(r0 + r) * ld + c] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < 32; ++i) s += v[i];
  red[0][grp][cl] = s;
  __syncthreads();
  const float tot = (red[0][0][cl] + red[0][1][cl]) + (red[0][2][cl] + red[0][3][cl]);
  const float mean = tot / (float)n;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const float d = v[i] - mean;
    q += grp * 32 + i < n ? d * d : 0.f;
  }
  red[1][grp][cl] = q;
  __syncthreads();
  if (grp == 0 && cv) {
    partial[((long long)blockIdx.y * C + c) * 2 + 0] = tot;
    partial[((long long)blockIdx.y * C + c) * 2 + 1] = (red[1][0][cl] + red[1][1][cl]) + (red[1][2][cl] + red[1][3][cl]);
  }
}

// typed loads: activations / gradients stored fp32 or bf16 (bf16 compute mode keeps the
// conv outputs y, the BN outputs and their gradients in bf16 -- half the bytes of every pass)
__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ f32x4 ld4(const bf16* p) {
  const bf16x4 v = *reinterpret_cast<const bf16x4*>(p);
  return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
}
__device__ __forceinline__ float ld1(const float* p) { return *p; }
__device__ __forceinline__ float ld1(const bf16* p) { return (float)*p; }
__device__ __forceinline__ void st4(float* o32, bf16* o16, long long e, f32x4 o) {
  if (o32) *reinterpret_cast<f32x4*>(o32 + e) = o;
  if (o16) *reinterpret_cast<bf16x4*>(o16 + e) = bf16x4{(bf16)o[0], (bf16)o[1], (bf16)o[2], (bf16)o[3]};
}

template <typename TY>
__global__ void bn_apply_kernel(const TY* __restrict__ y, const float* __restrict__ scale,
                                const float* __restrict__ shift, const float* __restrict__ res, float* __restrict__ out,
                                bf16* __restrict__ out16, long long total4, int C, int act) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total4) return;
  long long e = i * 4;
  int c = (int)(e % C);
  f32x4 v = ld4(y + e);
  f32x4 sc = *reinterpret_cast<const f32x4*>(scale + c);
  f32x4 sh = *reinterpret_cast<const f32x4*>(shift + c);
  f32x4 o;
#pragma unroll
  for (int k = 0; k < 4; ++k) o[k] = act_fwd(v[k] * sc[k] + sh[k], act);
  if (res) o += *reinterpret_cast<const f32x4*>(res + e);
  st4(out, out16, e, o);
}


template <typename TY>
__global__ void bn_apply1_kernel(const TY* __restrict__ y, const float* __restrict__ scale,
                                 const float* __restrict__ shift, const float* __restrict__ res, float* __restrict__ out,
                                 bf16* __restrict__ out16, long long total, int C, int act) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = (int)(i % C);
  float o = act_fwd(ld1(y + i) * scale[c] + shift[c], act);
  o = res ? o + res[i] : o;
  if (out) out[i] = o;
  if (out16) out16[i] = (bf16)o;
}

// Backward finalize of one 64-channel strip by one 256-thread block (4 row groups reduce the
// per-row-block partials in parallel): apply coefficients + dgamma / dbeta / conv-bias gradient.
// Backward finalize, stand-alone: 16 channels x 16 row groups per block (32 blocks at C = 512, 8
// partial rows per thread at 128 row blocks).  The 64-channel x 4-group form of the GEMM epilogue
// (bwd_finalize_cols) as its own launch ran 8 blocks x 32 rows per thread in 9.9 us per call
// beside the side stream's GEMMs, this one 6.0 us (profiles/r3_bn_bwd_forms_ab.txt)
__global__ void __launch_bounds__(256) bn_bwd_finalize16_kernel(const float* __restrict__ ws, int nrb, int M, int C,
                                                                BwdFin f) {
  __shared__ float red[3][16][17];
  const int cl = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f;
  if (c < C)
    for (int b0 = grp; b0 < nrb; b0 += 16 * 8) {
      float x[8][3];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int b = b0 + 16 * u;
        const float* p = ws + ((long long)(b < nrb ? b : 0) * C + c) * 3;
#pragma unroll
        for (int v = 0; v < 3; ++v) x[u][v] = b < nrb ? p[v] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        s0 += x[u][0];
        s1 += x[u][1];
        s2 += x[u][2];
      }
    }
  red[0][grp][cl] = s0;
  red[1][grp][cl] = s1;
  red[2][grp][cl] = s2;
  __syncthreads();
  if (threadIdx.x >= 16 || c >= C) return;
  float t0 = 0.f, t1 = 0.f, t2 = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    t0 += red[0][i][cl];
    t1 += red[1][i][cl];
    t2 += red[2][i][cl];
  }
  bwd_finalize_store(c, t0, t1, t2, M, C, f);
}

void launch_bwd_finalize(const float* ws, int nrb, int M, int C, const BwdFin& f, hipStream_t s) {
  bn_bwd_finalize16_kernel<<<cdiv(C, 16), 256, 0, s>>>(ws, nrb, M, C, f);
}

// backward reduce: per (64-row block, 64 channels) partial sums of dz, dz*yhat, yhat.
// 256 threads = 16 channel quads (4 channels, one 16-B fp32 / 8-B bf16 load) x 16 row lanes;
// the 4 rows of a lane are loaded together (independent loads in flight).
constexpr int RB = 64;
// 64-row sub-blocks per block of the vectorised reduce.  4 (256 rows, 4x fewer partials for the
// finalize) measured slower in the C2 step: 15.6 + 6.9 us vs 11.6 + 8.5 us per BN backward
constexpr int RBN = 1;

// dz = dA * act'(.): from the stored activation output a (FROM_PRE = false) or from the
// pre-activation z = yhat*gamma + beta recomputed from y (FROM_PRE = true: one fewer
// activation-sized read in each of the two passes)
template <bool FROM_PRE>
__device__ __forceinline__ float bn_dz(float g, float av, float yh, float gm, float bt, int act) {
  return FROM_PRE ? act_bwd_from_pre(g, yh * gm + bt, act) : act_bwd_from_out(g, av, act);
}

template <bool FROM_PRE, typename TD, typename TY>
__global__ void __launch_bounds__(256) bn_bwd_reduce_kernel(const TD* __restrict__ dA, const float* __restrict__ a,
                                                            const TY* __restrict__ y,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ rstd,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta, int M, int C, int act,
                                                            float* ws) {
  __shared__ float red[3][16][65];
  const int cq = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int c = blockIdx.x * 64 + cq * 4;
  const int r0 = blockIdx.y * RB * RBN;
  f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0, s2 = s0;
  if (c < C) {
    const f32x4 mu = *reinterpret_cast<const f32x4*>(mean + c);
    const f32x4 rs = *reinterpret_cast<const f32x4*>(rstd + c);
    f32x4 gm = {1.f, 1.f, 1.f, 1.f}, bt = {0.f, 0.f, 0.f, 0.f};
    if (FROM_PRE) {
      if (gamma) gm = *reinterpret_cast<const f32x4*>(gamma + c);
      if (beta) bt = *reinterpret_cast<const f32x4*>(beta + c);
    }
#pragma unroll 2
    for (int sub = 0; sub < RBN; ++sub) {
      const int rs0 = r0 + sub * RB + rl;
      f32x4 g[4], av[4], yv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = rs0 + 16 * i;
        const long long idx = (long long)(r < M ? r : 0) * C + c;
        g[i] = ld4(dA + idx);
        if (!FROM_PRE) av[i] = ld4(a + idx);
        yv[i] = ld4(y + idx);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (rs0 + 16 * i >= M) continue;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float yh = (yv[i][k] - mu[k]) * rs[k];
          const float dz = bn_dz<FROM_PRE>(g[i][k], FROM_PRE ? 0.f : av[i][k], yh, gm[k], bt[k], act);
          s0[k] += dz;
          s1[k] += dz * yh;
          s2[k] += yh;
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    red[0][rl][cq * 4 + k] = s0[k];
    red[1][rl][cq * 4 + k] = s1[k];
    red[2][rl][cq * 4 + k] = s2[k];
  }
  __syncthreads();
  if (threadIdx.x < 192) {
    const int q = threadIdx.x >> 6, cl = threadIdx.x & 63;
    const int cc = blockIdx.x * 64 + cl;
    if (cc < C) {
      float t = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) t += red[q][i][cl];
      ws[((long long)blockIdx.y * C + cc) * 3 + q] = t;
    }
  }
}

// scalar variant (C % 4 != 0): 64 channels x 4 row lanes
template <bool FROM_PRE, typename TD, typename TY>
__global__ void __launch_bounds__(256) bn_bwd_reduce1_kernel(const TD* __restrict__ dA, const float* __restrict__ a,
                                                             const TY* __restrict__ y,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ rstd,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ beta, int M, int C, int act,
                                                             float* ws) {
  __shared__ float red[3][4][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int r0 = blockIdx.y * RB;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f;
  if (c < C) {
    const float mu = mean[c], rs = rstd[c];
    const float gm = (FROM_PRE && gamma) ? gamma[c] : 1.f, bt = (FROM_PRE && beta) ? beta[c] : 0.f;
    const int r1 = min(M, r0 + RB);
    for (int r = r0 + rl; r < r1; r += 4) {
      const long long idx = (long long)r * C + c;
      const float yh = (ld1(y + idx) - mu) * rs;
      const float dz = bn_dz<FROM_PRE>(ld1(dA + idx), FROM_PRE ? 0.f : a[idx], yh, gm, bt, act);
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
    float v[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) v[q] = red[q][0][cl] + red[q][1][cl] + red[q][2][cl] + red[q][3][cl];
#pragma unroll
    for (int q = 0; q < 3; ++q) p[q] = v[q];
  }
}


// Row-strip form of the backward apply pass: a 256-thread block = 64 channel quads (a 256-channel
// strip) x 4 row lanes, each lane RPT rows, so the six planar per-channel constants are loaded
// once per RPT rows instead of once per 4 elements (the one-quad-per-thread form spends six 16-B
// constant loads per 8-B element load).  All RPT rows' loads are issued before any is used.
// RPT 4 measured best (10.9-11.1 us per 8192 x 512 bf16 call against 13.6 for the one-quad form;
// RPT 8 no better in the step, profiles/r3_bn_bwd_forms_ab.txt).  The forward apply, two
// constants per quad, measured slower in this form (8.6 vs 6.1 us at RPT 8: fewer waves in
// flight) and keeps the one-quad form.
template <int RPT, bool FROM_PRE, typename TD, typename TY>
__global__ void __launch_bounds__(256) bn_bwd_apply_rows_kernel(const TD* __restrict__ dA, const float* __restrict__ a,
                                                                const TY* __restrict__ y,
                                                                const float* __restrict__ coef, int M, int C, int act,
                                                                float* __restrict__ dy, bf16* __restrict__ dy16) {
  const int c = (blockIdx.x * 64 + (threadIdx.x & 63)) * 4;
  if (c >= C) return;
  const int r0 = blockIdx.y * 4 * RPT + (threadIdx.x >> 6);
  const f32x4 k1 = *reinterpret_cast<const f32x4*>(coef + c);
  const f32x4 m1 = *reinterpret_cast<const f32x4*>(coef + C + c);
  const f32x4 m2 = *reinterpret_cast<const f32x4*>(coef + 2 * C + c);
  const f32x4 mu = *reinterpret_cast<const f32x4*>(coef + 3 * C + c);
  const f32x4 rs = *reinterpret_cast<const f32x4*>(coef + 4 * C + c);
  f32x4 bt = {0.f, 0.f, 0.f, 0.f};
  if (FROM_PRE) bt = *reinterpret_cast<const f32x4*>(coef + 5 * C + c);
  f32x4 g[RPT], yv[RPT], av[RPT];
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int r = r0 + 4 * i;
    const long long e = (long long)(r < M ? r : 0) * C + c;
    g[i] = ld4(dA + e);
    yv[i] = ld4(y + e);
    if (!FROM_PRE) av[i] = ld4(a + e);
  }
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int r = r0 + 4 * i;
    if (r >= M) break;
    f32x4 o;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float yc = yv[i][k] - mu[k];
      const float dz = FROM_PRE ? act_bwd_from_pre(g[i][k], yc * k1[k] + bt[k], act)
                                : act_bwd_from_out(g[i][k], av[i][k], act);
      o[k] = k1[k] * (dz - m1[k] - yc * rs[k] * m2[k]);
    }
    st4(dy, dy16, (long long)r * C + c, o);
  }
}

template <bool FROM_PRE, typename TD, typename TY>
void launch_bwd_apply_rows(const TD* dp, const float* a, const TY* yp, const float* coef, int M, int C, int act,
                           float* dy, bf16* d16, hipStream_t s) {
  bn_bwd_apply_rows_kernel<4, FROM_PRE, TD, TY><<<dim3(cdiv(C / 4, 64), cdiv(M, 16)), 256, 0, s>>>(dp, a, yp, coef, M,
                                                                                                C, act, dy, d16);
}

template <bool FROM_PRE, typename TD, typename TY>
__global__ void bn_bwd_apply1_kernel(const TD* __restrict__ dA, const float* __restrict__ a,
                                     const TY* __restrict__ y, const float* __restrict__ coef, long long total,
                                     int C, int act, float* __restrict__ dy, bf16* __restrict__ dy16) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = (int)(i % C);
  const float yc = ld1(y + i) - coef[3 * C + c], k1 = coef[c];
  const float g = ld1(dA + i);
  const float dz = FROM_PRE ? act_bwd_from_pre(g, yc * k1 + coef[5 * C + c], act) : act_bwd_from_out(g, a[i], act);
  const float o = k1 * (dz - coef[C + c] - yc * coef[4 * C + c] * coef[2 * C + c]);
  if (dy) dy[i] = o;
  if (dy16) dy16[i] = (bf16)o;
}

// column sums: partial per strip of rpb rows (a multiple of 64; vectorised like bn_bwd_reduce when
// N % 4 == 0 and ld % 4 == 0, scalar otherwise), then a parallel finalize over the strips.  The
// strips are sized for ~1024 partial blocks, so the finalize reads at most a few hundred rows
// (64-row strips had left it a serial 1849-row loop per column on the mixer's 118336-row sums).
template <bool V4>
__global__ void __launch_bounds__(256) colsum_partial_kernel(const float* __restrict__ x, long long ld, int M, int N,
                                                             int rpb, float* ws) {
  __shared__ float red[16][65];
  const int cq = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int r0 = blockIdx.y * rpb, r1 = min(M, r0 + rpb);
  if constexpr (V4) {
    const int c = blockIdx.x * 64 + cq * 4;
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    if (c < N) {
      for (int rb = r0; rb < r1; rb += 64) {
        f32x4 v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = rb + rl + 16 * i;
          v[i] = *reinterpret_cast<const f32x4*>(x + (long long)(r < r1 ? r : r0) * ld + c);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (rb + rl + 16 * i < r1) s += v[i];
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) red[rl][cq * 4 + k] = s[k];
  } else {
    // 16 channels x 16 row lanes, each thread 4 channels strided by 16
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = blockIdx.x * 64 + cq + 16 * k;
      float s = 0.f;
      if (c < N)
        for (int r = r0 + rl; r < r1; r += 16) s += x[(long long)r * ld + c];
      red[rl][cq + 16 * k] = s;
    }
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    const int c = blockIdx.x * 64 + threadIdx.x;
    if (c < N) {
      float t = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) t += red[i][threadIdx.x];
      ws[(long long)blockIdx.y * N + c] = t;
    }
  }
}

__global__ void __launch_bounds__(256) colsum_final_kernel(const float* __restrict__ ws, int nrb, int N, float* out,
                                                            float* out2, int accumulate) {
  __shared__ float red[FG][64];
  const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  float sv[1] = {0.f};
  if (c < N) strided_sums<1, false, 32>(ws, nrb, N, c, grp, sv);
  float s = sv[0];
  red[grp][cl] = s;
  __syncthreads();
  if (grp != 0 || c >= N) return;
  s = 0.f;
#pragma unroll
  for (int i = 0; i < FG; ++i) s += red[i][cl];
  out[c] = accumulate ? out[c] + s : s;
  if (out2) out2[c] = accumulate ? out2[c] + s : s;  // b_ih and b_hh take the same gradient
}

}  // namespace

extern "C" int avc_bn_finalize(const float* partial, int M, int C, const float* gamma, const float* beta,
                               float* running_mean, float* running_var, long long* nbt, float momentum, float eps,
                               float* mean, float* rstd, float* scale, float* shift, void* stream) {
  AVC_CHECK_ARG(partial && mean && rstd && scale && shift && M > 0 && C > 0, "avc_bn_finalize: bad args");
  bn_finalize_kernel<<<cdiv(C, 64), 256, 0, as_stream(stream)>>>(partial, M, C, gamma, beta, running_mean,
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
  dim3 grid(cdiv(C, 64), cdiv(M, PTILE));
  bn_stats_kernel<<<grid, 256, 0, as_stream(stream)>>>(y, ld, M, C, partial);
  return avc_check_launch("avc_bn_stats");
}

unsigned* avc_counter_slots(int n, hipStream_t s) {
  constexpr unsigned POOL = 1u << 16;
  constexpr int MAXD = 64;
  static std::mutex mu;
  static std::atomic<unsigned*> pool[MAXD];
  static std::atomic<unsigned> next[MAXD];
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAXD || n <= 0 || (unsigned)n > POOL) {
    avc_set_error("avc_counter_slots: no device / bad size");
    return nullptr;
  }
  if (!pool[dev].load(std::memory_order_acquire)) {
    std::lock_guard<std::mutex> lk(mu);
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (!pool[dev].load() && hipStreamIsCapturing(s, &st) == hipSuccess && st == hipStreamCaptureStatusNone) {
      unsigned* p = nullptr;
      if (hipMalloc(&p, POOL * sizeof(unsigned)) == hipSuccess &&
          hipMemset(p, 0, POOL * sizeof(unsigned)) == hipSuccess && hipDeviceSynchronize() == hipSuccess)
        pool[dev].store(p, std::memory_order_release);
    }
  }
  unsigned* base = pool[dev].load(std::memory_order_acquire);
  if (!base) {
    avc_set_error("avc_counter_slots: counter pool not created (first use inside a stream capture? run one "
                  "eager step first)");
    return nullptr;
  }
  return base + avc_ring_reserve(next[dev], (unsigned)n, POOL);
}

unsigned avc_ring_reserve(std::atomic<unsigned>& cursor, unsigned n, unsigned pool) {
  unsigned cur = cursor.load(std::memory_order_relaxed);
  for (;;) {
    const unsigned b = cur & (pool - 1u);
    const bool wrap = b + n > pool;
    const unsigned start = wrap ? 0u : b;
    const unsigned nxt = cur + (wrap ? pool - b : 0u) + n;  // modulo 2^32: pool divides it
    if (cursor.compare_exchange_weak(cur, nxt, std::memory_order_relaxed)) return start;
  }
}

// Host-only test hook of the ring reservation (tests/test_abi.py): no device, no HIP call.
extern "C" unsigned avc_ring_reserve_test(unsigned* cursor, unsigned n, unsigned pool) {
  std::atomic<unsigned> c(*cursor);
  const unsigned r = avc_ring_reserve(c, n, pool);
  *cursor = c.load();
  return r;
}

float* avc_zero_slots(int n, hipStream_t s) {
  constexpr unsigned POOL = 1u << 23;  // 32 MB of floats per device
  constexpr int MAXD = 64;
  static std::mutex mu;
  static std::atomic<float*> pool[MAXD];
  static std::atomic<unsigned> next[MAXD];
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAXD || n <= 0 || (unsigned)n > POOL) {
    avc_set_error("avc_zero_slots: no device / bad size");
    return nullptr;
  }
  if (!pool[dev].load(std::memory_order_acquire)) {
    std::lock_guard<std::mutex> lk(mu);
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (!pool[dev].load() && hipStreamIsCapturing(s, &st) == hipSuccess && st == hipStreamCaptureStatusNone) {
      float* p = nullptr;
      if (hipMalloc(&p, POOL * sizeof(float)) == hipSuccess && hipMemset(p, 0, POOL * sizeof(float)) == hipSuccess &&
          hipDeviceSynchronize() == hipSuccess)
        pool[dev].store(p, std::memory_order_release);
    }
  }
  float* base = pool[dev].load(std::memory_order_acquire);
  if (!base) return nullptr;  // (the caller falls back to its direct form)
  const unsigned n64 = ((unsigned)n + 63u) & ~63u;  // 256-B aligned regions
  return base + avc_ring_reserve(next[dev], n64, POOL);
}

namespace {
// dtype dispatch of the typed BN kernels: F(TY) / F(TD, TY) with float or bf16 pointers
template <typename Fn>
void with_type(int dt, Fn&& fn) {
  if (dt == AVC_BF16) fn(static_cast<const bf16*>(nullptr));
  else fn(static_cast<const float*>(nullptr));
}
}  // namespace

extern "C" int avc_bn_apply(const void* y, int y_dtype, const float* scale, const float* shift,
                            const float* residual, float* out, void* out_bf16, int M, int C, int act, void* stream) {
  bf16* o16 = reinterpret_cast<bf16*>(out_bf16);
  AVC_CHECK_ARG(y && scale && shift && (out || o16) && C > 0 && (y_dtype == AVC_F32 || y_dtype == AVC_BF16),
                "avc_bn_apply: bad args");
  const long long total = (long long)M * C;
  if (total == 0) return 0;
  hipStream_t s = as_stream(stream);
  const bool v4 = C % 4 == 0;
  with_type(y_dtype, [&](auto tag) {
    using TY = std::remove_const_t<std::remove_pointer_t<decltype(tag)>>;
    const TY* yp = static_cast<const TY*>(y);
    if (v4)
      bn_apply_kernel<TY><<<cdiv(total / 4, 256), 256, 0, s>>>(yp, scale, shift, residual, out, o16, total / 4, C,
                                                              act);
    else
      bn_apply1_kernel<TY><<<cdiv(total, 256), 256, 0, s>>>(yp, scale, shift, residual, out, o16, total, C, act);
  });
  return avc_check_launch("avc_bn_apply");
}

extern "C" size_t avc_bn_bwd_ws(int M, int C) { return (size_t)cdiv(M, RB) * C * 3 + (size_t)C * 6 + 4; }

extern "C" int avc_bn_bwd(const void* dA, int dA_dtype, const float* a, const void* y, int y_dtype,
                          const float* mean, const float* rstd, const float* gamma, const float* beta, int M, int C,
                          int act, float* dy, void* dy_bf16, float* dgamma, float* dbeta, float* dbias,
                          int accumulate, float* ws, void* stream) {
  bf16* d16 = reinterpret_cast<bf16*>(dy_bf16);
  AVC_CHECK_ARG(dA && y && mean && rstd && (dy || d16) && ws && C > 0 &&
                    (dA_dtype == AVC_F32 || dA_dtype == AVC_BF16) && (y_dtype == AVC_F32 || y_dtype == AVC_BF16),
                "avc_bn_bwd: bad args");
  hipStream_t s = as_stream(stream);
  const bool pre = a == nullptr;  // activation derivative from the recomputed pre-activation
  // 4-wide loads: 8-B (bf16) / 16-B (fp32) aligned rows
  auto al = [](const void* p, int dt) { return (reinterpret_cast<uintptr_t>(p) & (dt == AVC_BF16 ? 7 : 15)) == 0; };
  const bool v4 = C % 4 == 0 && al(dA, dA_dtype) && al(y, y_dtype) && (pre || aligned16(a)) &&
                  (!gamma || aligned16(gamma)) && (!beta || aligned16(beta)) && (!dy || aligned16(dy)) &&
                  (!d16 || al(d16, AVC_BF16));
  const int nrb = cdiv(M, v4 ? RB * RBN : RB);
  dim3 grid(cdiv(C, 64), nrb);
  // per-channel apply constants, planar [6][C], 16-B aligned
  const size_t coff = ((size_t)nrb * C * 3 + 3) & ~(size_t)3;
  float* coef = ws + coff;
  const long long total = (long long)M * C;
  const BwdFin fin{gamma, beta, mean, rstd, coef, dgamma, dbeta, dbias, accumulate};
  with_type(dA_dtype, [&](auto dtag) {
    using TD = std::remove_const_t<std::remove_pointer_t<decltype(dtag)>>;
    with_type(y_dtype, [&](auto ytag) {
      using TY = std::remove_const_t<std::remove_pointer_t<decltype(ytag)>>;
      const TD* dp = static_cast<const TD*>(dA);
      const TY* yp = static_cast<const TY*>(y);
      if (v4) {
        if (pre) bn_bwd_reduce_kernel<true, TD, TY><<<grid, 256, 0, s>>>(dp, a, yp, mean, rstd, gamma, beta, M, C, act, ws);
        else bn_bwd_reduce_kernel<false, TD, TY><<<grid, 256, 0, s>>>(dp, a, yp, mean, rstd, gamma, beta, M, C, act, ws);
      } else {
        if (pre) bn_bwd_reduce1_kernel<true, TD, TY><<<grid, 256, 0, s>>>(dp, a, yp, mean, rstd, gamma, beta, M, C, act, ws);
        else bn_bwd_reduce1_kernel<false, TD, TY><<<grid, 256, 0, s>>>(dp, a, yp, mean, rstd, gamma, beta, M, C, act, ws);
      }
      launch_bwd_finalize(ws, nrb, M, C, fin, s);
      if (v4) {
        if (pre) launch_bwd_apply_rows<true>(dp, a, yp, coef, M, C, act, dy, d16, s);
        else launch_bwd_apply_rows<false>(dp, a, yp, coef, M, C, act, dy, d16, s);
      } else {
        if (pre)
          bn_bwd_apply1_kernel<true, TD, TY><<<cdiv(total, 256), 256, 0, s>>>(dp, a, yp, coef, total, C, act, dy, d16);
        else
          bn_bwd_apply1_kernel<false, TD, TY><<<cdiv(total, 256), 256, 0, s>>>(dp, a, yp, coef, total, C, act, dy, d16);
      }
    });
  });
  return avc_check_launch("avc_bn_bwd");
}

int avcbn::bn_bwd_reduce_finalize(const void* dA, int dA_dtype, const void* y, int y_dtype, int M, int C, int act,
                                  float* ws, const BwdFin& fin, hipStream_t s) {
  auto al = [](const void* p, int dt) { return (reinterpret_cast<uintptr_t>(p) & (dt == AVC_BF16 ? 7 : 15)) == 0; };
  const bool v4 = C % 4 == 0 && al(dA, dA_dtype) && al(y, y_dtype) && (!fin.gamma || aligned16(fin.gamma)) &&
                  (!fin.beta || aligned16(fin.beta));
  const int nrb = cdiv(M, v4 ? RB * RBN : RB);
  dim3 grid(cdiv(C, 64), nrb);
  with_type(dA_dtype, [&](auto dtag) {
    using TD = std::remove_const_t<std::remove_pointer_t<decltype(dtag)>>;
    with_type(y_dtype, [&](auto ytag) {
      using TY = std::remove_const_t<std::remove_pointer_t<decltype(ytag)>>;
      const TD* dp = static_cast<const TD*>(dA);
      const TY* yp = static_cast<const TY*>(y);
      if (v4)
        bn_bwd_reduce_kernel<true, TD, TY><<<grid, 256, 0, s>>>(dp, nullptr, yp, fin.mean, fin.rstd, fin.gamma, fin.beta,
                                                                M, C, act, ws);
      else
        bn_bwd_reduce1_kernel<true, TD, TY><<<grid, 256, 0, s>>>(dp, nullptr, yp, fin.mean, fin.rstd, fin.gamma,
                                                                 fin.beta, M, C, act, ws);
      launch_bwd_finalize(ws, nrb, M, C, fin, s);
    });
  });
  return avc_check_launch("bn_bwd_reduce_finalize");
}

extern "C" int avc_bn_bwd_apply(const void* dA, int dA_dtype, const void* y, int y_dtype, const float* coef, int M,
                                int C, int act, float* dy, void* dy_bf16, void* stream) {
  bf16* d16 = reinterpret_cast<bf16*>(dy_bf16);
  AVC_CHECK_ARG(dA && y && coef && (dy || d16) && M > 0 && C > 0 && (dA_dtype == AVC_F32 || dA_dtype == AVC_BF16) &&
                    (y_dtype == AVC_F32 || y_dtype == AVC_BF16) && aligned16(coef),
                "avc_bn_bwd_apply: bad args");
  hipStream_t s = as_stream(stream);
  auto al = [](const void* p, int dt) { return (reinterpret_cast<uintptr_t>(p) & (dt == AVC_BF16 ? 7 : 15)) == 0; };
  const bool v4 = C % 4 == 0 && al(dA, dA_dtype) && al(y, y_dtype) && (!dy || aligned16(dy)) &&
                  (!d16 || al(d16, AVC_BF16));
  const long long total = (long long)M * C;
  with_type(dA_dtype, [&](auto dtag) {
    using TD = std::remove_const_t<std::remove_pointer_t<decltype(dtag)>>;
    with_type(y_dtype, [&](auto ytag) {
      using TY = std::remove_const_t<std::remove_pointer_t<decltype(ytag)>>;
      const TD* dp = static_cast<const TD*>(dA);
      const TY* yp = static_cast<const TY*>(y);
      if (v4)
        launch_bwd_apply_rows<true>(dp, static_cast<const float*>(nullptr), yp, coef, M, C, act, dy, d16, s);
      else
        bn_bwd_apply1_kernel<true, TD, TY><<<cdiv(total, 256), 256, 0, s>>>(dp, nullptr, yp, coef, total, C, act, dy,
                                                                           d16);
    });
  });
  return avc_check_launch("avc_bn_bwd_apply");
}

extern "C" size_t avc_colsum_ws(int M, int N) { return (size_t)cdiv(M, RB) * N; }

extern "C" int avc_colsum(const float* x, long long ld, int M, int N, float* out, float* out2, int accumulate,
                          float* ws, void* stream) {
  AVC_CHECK_ARG(x && out && ws && ld >= N, "avc_colsum: bad args");
  hipStream_t s = as_stream(stream);
  // row strips of rpb rows: ~1024 partial blocks in all (nrb <= cdiv(M, RB), the workspace bound)
  const int ncb = cdiv(N, 64), target = 1024 / ncb > 1 ? 1024 / ncb : 1;
  const int rpb = M > 0 ? RB * cdiv(cdiv(M, RB), target) : RB, nrb = cdiv(M, rpb);
  if (N % 4 == 0 && ld % 4 == 0 && aligned16(x))
    colsum_partial_kernel<true><<<dim3(ncb, nrb), 256, 0, s>>>(x, ld, M, N, rpb, ws);
  else
    colsum_partial_kernel<false><<<dim3(ncb, nrb), 256, 0, s>>>(x, ld, M, N, rpb, ws);
  colsum_final_kernel<<<cdiv(N, 64), 256, 0, s>>>(ws, nrb, N, out, out2, accumulate);
  return avc_check_launch("avc_colsum");
}
