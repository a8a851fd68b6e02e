// gemm_internal.h — device-side GEMM argument structs and the shared MFMA epilogue used by
// the LDS-tiled kernels in gemm.hip and gemm_nt.hip (internal to libautovc_hip.so).
#pragma once
#include "common.h"
#include "bn_internal.h"

namespace avcg {

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int BM = 128;                    // rows per workgroup tile (BN partial-stat tiles follow it)
constexpr int FBK = 64;                    // K per LDS stage of the fast kernels

struct OpDev {
  const void* ptr;
  long long ld, bstride;
  int dtype, win, vec, taps, pad, t_out, t_in, chans, rows;
  FastDiv tdiv;
  FastDiv cdv;  // window: divide a K index by chans
};

struct GemmArgs {
  int M, N, K, batch, split_k, klen;
  OpDev a, b;
  float* c;
  bf16* c16;
  const float* res;
  long long ldc, cbs;
  const float* bias;
  int accumulate, atomic;
  float* bn_partial;
  int cperm;     // 0, or taps: column n = tap*chans + ch is stored at ch*taps + tap (conv weight layout)
  FastDiv cpd;   // divide a column by chans = N / cperm
  int c16_act;         // avc_gemm_desc.c_bf16_act: C16 holds GELU(C) (ring kernels only)
  const void* agrad;   // avc_gemm_desc.act_grad_of: C *= GELU'(agrad[o]) (ring kernels only)
  int agrad16;         // agrad is bf16
  bf16* c16pre;        // avc_gemm_desc.c_pre_bf16: pre-activation C in bf16 (ring kernels only)
  int ctr;             // avc_gemm_desc.c_trans_rows: C(m, n) stored at ((m / ctr) * N + n) * ctr + m % ctr
  float* csum;         // avc_gemm_desc.col_sum: csum[n] += column sums of the stored C (ring kernels only)
  int csum_n;
  // csum_ws != null: the ring kernels add their tile sums into csum_ws[slot][n] (slot = row tile %
  // csum_slots, self-zeroing pool memory) and one reduce pass adds the slots into csum -- the same
  // column's atomics from every row tile had serialised at one address (up to 924 per column)
  float* csum_ws;
  int csum_slots;
  const float* rbias;  // per-(utterance, edge class) row bias (avc_gemm_desc.row_bias), nullable
  int rb_t, rb_pad;
  FastDiv rb_div;      // divide a row by rb_t
  // BatchNorm finalize by the last row tile of each column tile (bn_cnt != null, bn_partial set):
  // mean / rstd / scale / shift and the running statistics of the tile's columns (avc_gemm_bn)
  unsigned* bn_cnt;
  const float* bn_gamma;
  const float* bn_beta;
  float* bn_rmean;
  float* bn_rvar;
  long long* bn_nbt;
  float* bn_mean;
  float* bn_rstd;
  float* bn_scale;
  float* bn_shift;
  float bn_momentum, bn_eps;
  int bn_nupd;
  int bn_rows;  // rows per bn_partial statistics tile: 0 = BM (128); the one-utterance conv tile: T
  // BatchNorm BACKWARD reduction of the layer that produced this GEMM's output gradient
  // (bnb_ws != null, avc_gemm_bnb): per 128-row tile and column (sum dz, sum dz*yhat,
  // sum yhat) with dz = C * act'(z), z = (y - mean)*rstd*gamma + beta recomputed from the
  // producer's stored conv output y; the last row tile of each column tile finalizes them
  const void* bnb_y;
  int bnb_ydt, bnb_act;
  float* bnb_ws;
  unsigned* bnb_cnt;
  avcbn::BwdFin bnb_fin;
  // split-K without atomics (TT kernels, sk_ws != null): per-stream workspace of split_k partial
  // tiles per output tile and one self-resetting arrival counter per output tile (splitk_last)
  float* sk_ws;
  unsigned* sk_cnt;
  int zero_c;  // C still needs the zero fill of an atomic split-K (deferred to the TT dispatch)
};

// Split-K without atomics (sk_ws != null): every split stores its NF accumulator fragments in
// register order (16 B per lane, write-through sc1, so no fence) into slot ks of its output tile's
// workspace and arrives on the tile's counter; the split that arrives last adds the S slots in
// split order (sc1 loads, its own slot included) so the sum does not depend on which split
// finishes last (deterministic, unlike the atomics), and returns true to run the
// plain epilogue.  The others return false.  Replaces the zero fill of C plus S x M x N float
// atomics (~1.3 TB/s chip-wide, MI355X_MICROARCH.md) with S x M x N write-through stores and
// (S-1) x M x N loads by the last splits.
template <int NF>
__device__ __forceinline__ bool splitk_last(const GemmArgs& g, f32x4* acc, int tile, int ks) {
  constexpr int SC1 = 16;  // buffer-instruction cache-policy bits: sc1
  const int S = g.split_k, nth = blockDim.x, tid = threadIdx.x;
  float* base = g.sk_ws + (long long)tile * S * NF * nth * 4;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, S * NF * nth * 16, 0x00020000);
#pragma unroll
  for (int f = 0; f < NF; ++f)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[f]), rs, ((ks * NF + f) * nth + tid) * 16, 0,
                                           SC1);
  if (!arrive_last(g.sk_cnt + tile, (unsigned)S)) return false;
  f32x4 sum[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) sum[f] = f32x4{0.f, 0.f, 0.f, 0.f};
  // its own slot is re-read too (acc is dead after the stores: VGPRs); the loads of slot s + 1 are
  // in flight while slot s is added, one memory round trip per slot instead of two
  u32x4 v[2][NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) v[0][f] = __builtin_amdgcn_raw_buffer_load_b128(rs, (f * nth + tid) * 16, 0, SC1);
  for (int s = 0; s < S; s += 2) {
    if (s + 1 < S) {
#pragma unroll
      for (int f = 0; f < NF; ++f)
        v[1][f] = __builtin_amdgcn_raw_buffer_load_b128(rs, (((s + 1) * NF + f) * nth + tid) * 16, 0, SC1);
    }
#pragma unroll
    for (int f = 0; f < NF; ++f) sum[f] += __builtin_bit_cast(f32x4, v[0][f]);
    if (s + 1 < S) {
      if (s + 2 < S) {
#pragma unroll
        for (int f = 0; f < NF; ++f)
          v[0][f] = __builtin_amdgcn_raw_buffer_load_b128(rs, (((s + 2) * NF + f) * nth + tid) * 16, 0, SC1);
      }
#pragma unroll
      for (int f = 0; f < NF; ++f) sum[f] += __builtin_bit_cast(f32x4, v[1][f]);
    }
  }
#pragma unroll
  for (int f = 0; f < NF; ++f) acc[f] = sum[f];
  return true;
}

// Last-arriving row tile of a column tile: merge the per-row-tile (sum, M2) partials of columns
// n0 .. n0+BN_-1 (Chan's parallel form, two passes over the L2/MALL-resident partials) and
// publish the BatchNorm coefficients -- the separate finalize launch of the forward is gone.
template <int BN_>
__device__ __forceinline__ void bn_finalize_cols(const GemmArgs& g, int n0, float* red) {
  const int nthr = blockDim.x, ng = nthr / BN_;
  const int tid = threadIdx.x, cl = tid % BN_, grp = tid / BN_;
  const int col = n0 + cl;
  const bool cv = col < g.N && grp < ng;
  const int tr = g.bn_rows ? g.bn_rows : BM;
  const int nt = (g.M + tr - 1) / tr;
  const float n = (float)g.M;
  float mean, m2;
  chan_merge<64 / (256 / BN_), true>(g.bn_partial, nt, g.N, col, cv, grp, ng, cl, BN_, g.M, tr, red, mean, m2);
  if (grp == 0 && col < g.N) {
    const float var = m2 / n;
    const float rstd = 1.f / sqrtf(var + g.bn_eps);
    const float ga = g.bn_gamma ? g.bn_gamma[col] : 1.f;
    const float be = g.bn_beta ? g.bn_beta[col] : 0.f;
    // write-through: the fused apply's workgroups read scale / shift within the launch (ld_sc1)
    st_sc1(g.bn_mean + col, mean);
    st_sc1(g.bn_rstd + col, rstd);
    st_sc1(g.bn_scale + col, ga * rstd);
    st_sc1(g.bn_shift + col, be - mean * ga * rstd);
    if (g.bn_rmean) {
      const float unb = n > 1.f ? m2 / (n - 1.f) : var;
      float rm = g.bn_rmean[col], rv = g.bn_rvar[col];
      for (int k = 0; k < g.bn_nupd; ++k) {
        rm = (1.f - g.bn_momentum) * rm + g.bn_momentum * mean;
        rv = (1.f - g.bn_momentum) * rv + g.bn_momentum * unb;
      }
      g.bn_rmean[col] = rm;
      g.bn_rvar[col] = rv;
    }
  }
  if (tid == 0 && n0 == 0 && g.bn_nbt) *g.bn_nbt += g.bn_nupd;
}

// GELU (erf form, nn.GELU) and its derivative for the fused epilogues
__device__ __forceinline__ float gelu_f(float x) { return 0.5f * x * (1.f + erf_nb(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_grad_f(float x) {
  return 0.5f * (1.f + erf_nb(x * 0.70710678118654752f)) +
         x * 0.39894228040143267794f * __builtin_amdgcn_exp2f(x * x * -0.72134752044448170f);
}

// Column offset of output column `col` (cperm: the Conv1d [Co][Ci][K] layout).
__device__ __forceinline__ long long out_col(const GemmArgs& g, int col) {
  if (!g.cperm) return col;
  const int tap = (int)fdiv((uint32_t)col, g.cpd), ch = col - tap * (int)g.cpd.d;
  return (long long)ch * g.cperm + tap;
}

// Element offset of C(row, col): row-major with the cperm column map, or the transposed blocks of
// avc_gemm_desc.c_trans_rows (C(m, n) at ((m / ctr) * N + n) * ctr + m % ctr)
__device__ __forceinline__ long long out_off(const GemmArgs& g, int row, int col) {
  if (g.ctr) {
    const int b = row / g.ctr;
    return ((long long)b * g.N + col) * g.ctr + (row - b * g.ctr);
  }
  return (long long)row * g.ldc + out_col(g, col);
}

// Row bias of the conv0 fold (avc_gemm_desc.row_bias): rows rbase + 16 i + e, columns cbase + 16 j.
template <int NJ>
__device__ __forceinline__ void add_row_bias(const GemmArgs& g, f32x4 (&acc)[4][NJ], int rbase, int cbase) {
  const int T = g.rb_t, pad = g.rb_pad, ncls = 2 * pad + 1;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = rbase + i * 16 + e;
      if (row >= g.M) continue;
      const int b = (int)fdiv((uint32_t)row, g.rb_div), t = row - b * T;
      const int cls = t < pad ? t : (t >= T - pad ? 2 * pad - (T - 1 - t) : pad);
      const float* rp = g.rbias + (long long)(b * ncls + cls) * g.N;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int col = cbase + j * 16;
        if (col < g.N) acc[i][j][e] += rp[col];
      }
    }
}

// Accumulator layout shared by the fast kernels: 4 waves as 2 (M) x 2 (N); wave (wm, wn) owns
// rows wm*64 + i*16 + 4*(lane>>4) + e and columns wn*BN_/2 + j*16 + (lane&15) of the tile.
// Fused epilogue: bias, residual, accumulate / atomics (split-K, batch-sum), bf16 copy, and
// BatchNorm partial statistics (per 128-row tile: column sum and M2 about the tile mean).
// BNB: the BatchNorm-backward reduction compiled in.  YST: the caller's LDS holds at least
// 8 KiB + 128 x (2*BN_ + 16) bytes, so a bf16 y tile is staged through it with 16-B coalesced
// loads (per-element 2-B buffer loads of y made a fused conv 30 us slower than a plain one)
template <int BN_, bool BNB = true, bool YST = false>
__device__ __forceinline__ void fast_epilogue(const GemmArgs& g, f32x4 (&acc)[4][BN_ / 32], int m0, int n0, int mt,
                                              int bz, int ks, char* smem_raw) {
  constexpr int NJ = BN_ / 32;
  constexpr int WN = BN_ / 2;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int rbase = m0 + wm * 64 + 4 * (lane >> 4);
  const int cbase = n0 + wn * WN + (lane & 15);
  float* C = g.c ? g.c + (long long)bz * g.cbs : nullptr;  // null: bf16-only output
  bf16* C16 = g.c16 ? g.c16 + (long long)bz * g.cbs : nullptr;
  if (g.bias && ks == 0) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int col = cbase + j * 16;
      const float bv = col < g.N ? g.bias[col] : 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i][j] += bv;
    }
  }
  if (g.rbias && ks == 0) add_row_bias<NJ>(g, acc, rbase, cbase);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = rbase + i * 16 + e;
      if (row >= g.M) continue;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int col = cbase + j * 16;
        if (col >= g.N) continue;
        const long long o = out_off(g, row, col);
        float v = acc[i][j][e];
        if (g.res && ks == 0) v += g.res[(long long)bz * g.cbs + o];
        if (g.atomic && !g.sk_ws) {
          atomicAdd(C + o, v);
        } else {
          if (g.accumulate) v += C[o];
          if (C) C[o] = v;
          if (C16) C16[o] = (bf16)v;
        }
      }
    }
  if (g.bn_partial) {
    float* red = reinterpret_cast<float*>(smem_raw);  // [2][BN_] sums, then [2][BN_] M2
    const int cnt = max(1, min(BM, g.M - m0));
    float s[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      float t = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) t += (rbase + i * 16 + e < g.M) ? acc[i][j][e] : 0.f;
      t += __shfl_xor(t, 16, 64);
      t += __shfl_xor(t, 32, 64);
      s[j] = t;
    }
    __syncthreads();
    if (lane < 16) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) red[wm * BN_ + wn * WN + j * 16 + lane] = s[j];
    }
    __syncthreads();
    float qv[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int cl = wn * WN + j * 16 + (lane & 15);
      const float mean = (red[cl] + red[BN_ + cl]) / (float)cnt;
      float t = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = acc[i][j][e] - mean;
          t += (rbase + i * 16 + e < g.M) ? d * d : 0.f;
        }
      t += __shfl_xor(t, 16, 64);
      t += __shfl_xor(t, 32, 64);
      qv[j] = t;
    }
    float* red2 = red + 2 * BN_;
    if (lane < 16) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) red2[wm * BN_ + wn * WN + j * 16 + lane] = qv[j];
    }
    __syncthreads();
    if (tid < BN_) {
      const int cl = tid;
      const int col = n0 + cl;
      if (col < g.N) {
        float* p = g.bn_partial + ((long long)mt * g.N + col) * 2;
        const float s0 = red[cl] + red[BN_ + cl];
        const float s1 = red2[cl] + red2[BN_ + cl];
        // sc1 when another block merges them (bn_cnt): no L2-wide release fence needed
        if (g.bn_cnt) {
          st_sc1(p, s0);
          st_sc1(p + 1, s1);
        } else {
          p[0] = s0;
          p[1] = s1;
        }
      }
    }
    if (g.bn_cnt) {
      const int ntile = (g.M + BM - 1) / BM;
      if (arrive_last(g.bn_cnt + n0 / BN_, (unsigned)ntile)) bn_finalize_cols<BN_>(g, n0, red);
    }
  }
  if (BNB && g.bnb_ws) {
    // BatchNorm backward reduction of the producing layer over this tile's rows (the value the
    // apply pass will read: rounded to bf16 when C is bf16-only)
    float* red = reinterpret_cast<float*>(smem_raw);  // [3][2 wm][BN_], then the finalize's 3*FG*64
    const avcbn::BwdFin& f = g.bnb_fin;
    float s0[NJ], s1[NJ], s2[NJ];
    // y through a buffer resource: 32-bit element offsets (M*ldc < 2^30 checked by the host)
    const bool ybf = g.bnb_ydt == AVC_BF16;
    const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<void*>(g.bnb_y), (short)0, (int)min((long long)g.M * g.ldc * (ybf ? 2 : 4), 0x7fffffffLL), 0x00020000);
    constexpr int YP = 2 * BN_ + 16;  // LDS row pitch of the staged tile (bytes)
    char* ys = smem_raw + 8192;
    const bool yst = YST && ybf && (g.ldc % 8) == 0 && (reinterpret_cast<uintptr_t>(g.bnb_y) & 15) == 0;
    if (yst) {
      // rows m0.., columns n0..n0+BN_-1 as 16-B chunks (8 columns), zero outside [M) x [N)
      constexpr int CPR = BN_ / 8;
      const bf16* yb = reinterpret_cast<const bf16*>(g.bnb_y);
      __syncthreads();  // the caller's last use of LDS is done
      for (int q = tid; q < BM * CPR; q += blockDim.x) {
        const int r = q / CPR, cc = q - r * CPR;
        const int row = m0 + r, col = n0 + cc * 8;
        u32x4 v = {0u, 0u, 0u, 0u};
        if (row < g.M && col < g.N) {
          if (col + 8 <= g.N) {
            v = *reinterpret_cast<const u32x4*>(yb + (long long)row * g.ldc + col);
          } else {
            unsigned short h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            for (int k = 0; k < 8 && col + k < g.N; ++k)
              h[k] = __builtin_bit_cast(unsigned short, yb[(long long)row * g.ldc + col + k]);
            v = u32x4{h[0] | (unsigned)h[1] << 16, h[2] | (unsigned)h[3] << 16, h[4] | (unsigned)h[5] << 16,
                      h[6] | (unsigned)h[7] << 16};
          }
        }
        *reinterpret_cast<u32x4*>(ys + r * YP + cc * 16) = v;
      }
      __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int col = cbase + j * 16;
      const bool cv = col < g.N;
      const float mu = cv ? f.mean[col] : 0.f, rs = cv ? f.rstd[col] : 0.f;
      const float gm = cv && f.gamma ? f.gamma[col] : 1.f, bt = cv && f.beta ? f.beta[col] : 0.f;
      float t0 = 0.f, t1 = 0.f, t2 = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = rbase + i * 16 + e;
          if (!cv || row >= g.M) continue;
          float v = acc[i][j][e];
          if (!C) v = (float)(bf16)v;
          const int o = row * (int)g.ldc + col;
          float yv;
          if (YST && yst)
            yv = __builtin_bit_cast(float, (unsigned)*reinterpret_cast<const unsigned short*>(
                                               ys + (row - m0) * YP + (col - n0) * 2) << 16);
          else
            yv = ybf ? __builtin_bit_cast(float, (unsigned)__builtin_amdgcn_raw_buffer_load_b16(yr, o * 2, 0, 0) << 16)
                     : __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(yr, o * 4, 0, 0));
          const float yh = (yv - mu) * rs;
          const float dz = act_bwd_from_pre(v, yh * gm + bt, g.bnb_act);
          t0 += dz;
          t1 += dz * yh;
          t2 += yh;
        }
      t0 += __shfl_xor(t0, 16, 64);
      t0 += __shfl_xor(t0, 32, 64);
      t1 += __shfl_xor(t1, 16, 64);
      t1 += __shfl_xor(t1, 32, 64);
      t2 += __shfl_xor(t2, 16, 64);
      t2 += __shfl_xor(t2, 32, 64);
      s0[j] = t0;
      s1[j] = t1;
      s2[j] = t2;
      // one column group's y loads at a time: hoisting all of them doubled the kernels' VGPRs
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
    if (lane < 16) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int cl = wn * WN + j * 16 + lane;
        red[(0 * 2 + wm) * BN_ + cl] = s0[j];
        red[(1 * 2 + wm) * BN_ + cl] = s1[j];
        red[(2 * 2 + wm) * BN_ + cl] = s2[j];
      }
    }
    __syncthreads();
    if (tid < BN_) {
      const int col = n0 + tid;
      if (col < g.N) {
        float* p = g.bnb_ws + ((long long)mt * g.N + col) * 3;
#pragma unroll
        for (int q = 0; q < 3; ++q) st_sc1(p + q, red[(q * 2) * BN_ + tid] + red[(q * 2 + 1) * BN_ + tid]);
      }
    }
    if (arrive_last(g.bnb_cnt + n0 / BN_, (g.M + BM - 1) / BM)) {
      const int c1 = min(n0 + BN_, g.N);
      for (int c0 = n0; c0 < c1; c0 += 64)
        avcbn::bwd_finalize_cols<true, 16>(g.bnb_ws, (g.M + BM - 1) / BM, g.M, g.N, c0, min(64, c1 - c0), f, red);
    }
  }
}

// Entry of the NT (both operands K-contiguous, bf16) LDS-DMA pipelined kernel (gemm_nt.hip).
// Returns false when the shape/operands do not qualify (caller falls back).
bool gemm_nt_launch(const GemmArgs& g, hipStream_t s);
// Entry of the halo-reuse Conv1d kernel (5 taps, 'same' padding, bf16; gemm_conv.hip).
bool gemm_conv_launch(const GemmArgs& g, hipStream_t s);
// Entry of the TT (both operands K-strided, bf16) weight-gradient kernel (gemm_tt.hip).
bool gemm_tt_launch(const GemmArgs& g, hipStream_t s);
// launch the zero fill of C when g.zero_c is set (clears it; gemm.hip)
void gemm_zero_c(GemmArgs& g, hipStream_t s);
// per-stream split-K workspace of at least `bytes` (grown, never shrunk; null inside a stream
// capture or on allocation failure: the caller keeps the atomics; gemm_tt.hip)
float* gemm_splitk_ws(size_t bytes, hipStream_t s);
// Entry of the 8-wave deep-ring NT kernel (gemm_ring.hip); false when the shape / operands do
// not qualify or AVC_RING=0.
bool gemm_ring_launch(const GemmArgs& g, hipStream_t s);

}  // namespace avcg
