// bn_internal.h — BatchNorm backward pieces shared by bn.hip and the GEMM epilogue
// (gemm_internal.h: the backward reduction of the PRODUCING layer's BatchNorm computed in the
// epilogue of the data-gradient GEMM that produces dL/d(activation)).
#pragma once
#include "common.h"

namespace avcbn {

constexpr int FG = 4;  // row groups of the finalize reductions (256 threads = 64 channels x 4)
constexpr int FU = 8;   // partial rows per thread loaded together (independent loads in flight)

// sum over b = grp, grp + FG, ... < nrb of NV consecutive floats at ws[(b*ld + c)*NV + v]:
// FU rows' loads are issued before any is added (one memory latency per FU*FG rows, not per row)
template <int NV, bool SC1 = false, int FUN = FU>  // SC1: partials handed over within the launch
__device__ __forceinline__ void strided_sums(const float* __restrict__ ws, int nrb, long long ld, int c, int grp,
                                             float (&out)[NV]) {
#pragma unroll
  for (int v = 0; v < NV; ++v) out[v] = 0.f;
  for (int b0 = grp; b0 < nrb; b0 += FG * FUN) {
    float x[FUN][NV];
#pragma unroll
    for (int u = 0; u < FUN; ++u) {
      const int b = b0 + u * FG;
      const float* p = ws + ((long long)(b < nrb ? b : 0) * ld + c) * NV;
#pragma unroll
      for (int v = 0; v < NV; ++v) x[u][v] = b < nrb ? (SC1 ? ld_sc1(p + v) : p[v]) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < FUN; ++u)
#pragma unroll
      for (int v = 0; v < NV; ++v) out[v] += x[u][v];
  }
}

struct BwdFin {
  const float* gamma;
  const float* beta;
  const float* mean;
  const float* rstd;
  float* coef;
  float* dgamma;
  float* dbeta;
  float* dbias;
  int acc;
};

// Channel c's apply constants (planar coef[6][C]) and parameter gradients from its three column
// sums over all rows: s0 = sum dz, s1 = sum dz*yhat, s2 = sum yhat.
// SC1: the coefficients are read within the launch (the fused apply of the halo conv): write-through
template <bool SC1 = false>
__device__ __forceinline__ void bwd_finalize_store(int c, float s0, float s1, float s2, int M, int C, const BwdFin& f) {
  const float g = f.gamma ? f.gamma[c] : 1.f;
  const float rs = f.rstd[c], mu = f.mean[c];
  const float k1 = g * rs;
  const float invn = 1.f / (float)M;
  const float m1 = s0 * invn, m2 = s1 * invn;
  // planar per-channel constants of the apply pass (one 16-B load per plane per 4 channels):
  //   yhat = (y - mu)*rs,  z = (y - mu)*k1 + beta,  dy = k1*(dz - m1 - yhat*m2)
  if (SC1) {
    st_sc1(f.coef + c, k1);
    st_sc1(f.coef + C + c, m1);
    st_sc1(f.coef + 2 * C + c, m2);
  } else {
    f.coef[c] = k1;
    f.coef[C + c] = m1;
    f.coef[2 * C + c] = m2;
  }
  f.coef[3 * C + c] = mu;
  f.coef[4 * C + c] = rs;
  f.coef[5 * C + c] = f.beta ? f.beta[c] : 0.f;
  const float gb = -k1 * s1 * s2 * invn;
  if (f.dgamma) f.dgamma[c] = f.acc ? f.dgamma[c] + s1 : s1;
  if (f.dbeta) f.dbeta[c] = f.acc ? f.dbeta[c] + s0 : s0;
  if (f.dbias) f.dbias[c] = f.acc ? f.dbias[c] + gb : gb;
}

// BatchNorm backward finalize of channels c0 .. c0+nc-1 (nc <= 64) from per-row-block partials
// ws[(b*C + c)*3 + {0,1,2}] = (sum dz, sum dz*yhat, sum yhat), b < nrb: the planar apply
// constants coef[6][C] and the parameter gradients.  256 threads (64 channels x FG row
// groups); red: 3*FG*64 floats of LDS.  Every thread of the block calls it.
template <bool SC1, int FUN = 32>  // FUN: partial rows per thread in flight (registers: 3*FUN)
__device__ __forceinline__ void bwd_finalize_cols(const float* ws, int nrb, int M, int C, int c0, int nc,
                                                  const BwdFin& f, float* red) {
  const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int c = c0 + cl;
  const bool cv = cl < nc && c < C;
  float sv[3] = {0.f, 0.f, 0.f};
  if (cv) strided_sums<3, SC1, FUN>(ws, nrb, C, c, grp, sv);
  __syncthreads();  // red may alias LDS the caller just read
  red[(0 * FG + grp) * 64 + cl] = sv[0];
  red[(1 * FG + grp) * 64 + cl] = sv[1];
  red[(2 * FG + grp) * 64 + cl] = sv[2];
  __syncthreads();
  if (grp != 0 || !cv) return;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < FG; ++i) {
    s0 += red[(0 * FG + i) * 64 + cl];
    s1 += red[(1 * FG + i) * 64 + cl];
    s2 += red[(2 * FG + i) * 64 + cl];
  }
  bwd_finalize_store(c, s0, s1, s2, M, C, f);
}

// The same reduction as a stand-alone pass over (dA, y) (bn.hip reduce kernels + finalize):
// fallback of avc_gemm_bnb when the GEMM does not run on an epilogue that computes it.
int bn_bwd_reduce_finalize(const void* dA, int dA_dtype, const void* y, int y_dtype, int M, int C, int act,
                           float* ws, const BwdFin& fin, hipStream_t s);

}  // namespace avcbn
