// lstm.hip — LSTM recurrences (forward and backward) for the AutoVC path.
//
// Replaces the time loops inside nn.LSTM: encoder BiLSTM(512->44, 2 layers)
// (factory/AutoVC.py:43,54-55), decoder lstm1(344->512) (:77,103) and lstm2(512->1024,
// 2 layers) (:96,110).  Gate order i, f, g, o; h0 = c0 = 0; the input projection
// x W_ih^T + b_ih + b_hh is a separate GEMM over all frames (gemm.hip) and arrives here
// as `xproj`.
//
// Two designs, chosen by H:
//  * small H (<= 64, the encoder): batch rows are independent in the recurrence, so one
//    workgroup owns one (utterance, direction) for all T steps.  W_hh lives in registers
//    (one gate row per thread), h/gates in LDS; no inter-workgroup sync at all.
//  * large H (multiple of 128, the decoder): one persistent launch per layer when it fits
//    (bf16, one direction, H in {512, 1024}: lstm_persist_fwd / lstm_persist_bwd below),
//    otherwise one fused kernel per time step.  Each
//    workgroup owns (16*MT utterances) x (8 hidden units, all 4 gates) [forward] or
//    (16*MT utterances) x (16 hidden units) [backward]; the recurrent product runs on
//    MFMA with K split over the 4 waves and operands loaded straight into registers;
//    the cell update is fused into the same kernel's epilogue.  Kernel boundaries are the
//    grid-wide sync (cheaper on gfx950 than a software grid barrier at 256 workgroups,
//    MI355X_MICROARCH.md rows "boundary" vs "barrier-xcd"); the host loop is
//    graph-capturable.
#include <cstdlib>

#include "common.h"

namespace {

// =============================================================== small H: persistent
// The per-step inputs (xproj rows forward; dh, c, c_prev, gates backward) are staged in LDS
// one chunk of SC steps ahead: each thread issues plain loads for chunk k+1 when chunk k
// starts and writes them to the other LDS buffer when it ends, so the T-step dependency chain
// only touches LDS and registers (a one-step prefetch left a global-memory round trip on
// every step of the chain).
constexpr int SC = 16;

template <int HM>
__global__ void __launch_bounds__(256) lstm_small_fwd(const float* __restrict__ xproj, const float* __restrict__ whh,
                                                      int T, int H, int dirs, float* __restrict__ hout,
                                                      float* __restrict__ cout, float* __restrict__ gout) {
  constexpr int GM = 4 * HM, NPF = (SC * GM + 255) / 256;
  const int b = blockIdx.x, d = blockIdx.y, tid = threadIdx.x;
  const int G = 4 * H;
  __shared__ __attribute__((aligned(16))) float hs[HM];
  __shared__ float gs[GM];
  __shared__ float xs[2][SC * GM];
  float w[HM];
  const float* W = whh + (long long)d * G * H;
#pragma unroll
  for (int k = 0; k < HM; ++k) w[k] = (tid < G && k < H) ? W[(long long)tid * H + k] : 0.f;
  if (tid < HM) hs[tid] = 0.f;
  float c = 0.f;
  const long long ldx = (long long)dirs * G, ldh = (long long)dirs * H;
  const int q = tid < G ? tid / H : 0;
  const int t0 = d ? T - 1 : 0, dt = d ? -1 : 1;
  const float* xb = xproj + (long long)b * T * ldx + d * G;
  // chunk element e: step s = k*SC + e/G, gate row e%G
  float pf[NPF];
  auto issue = [&](int k) {
#pragma unroll
    for (int i = 0; i < NPF; ++i) {
      const int e = tid + 256 * i, si = e / G, s = k * SC + si;
      pf[i] = (si < SC && s < T) ? xb[(long long)(t0 + dt * s) * ldx + (e - si * G)] : 0.f;
    }
  };
  auto commit = [&](int buf) {
#pragma unroll
    for (int i = 0; i < NPF; ++i) {
      const int e = tid + 256 * i;
      if (e < SC * G) xs[buf][e] = pf[i];
    }
  };
  const int nch = (T + SC - 1) / SC;
  issue(0);
  commit(0);
  __syncthreads();
  for (int k = 0; k < nch; ++k) {
    if (k + 1 < nch) issue(k + 1);
    const float* xk = xs[k & 1];
    const int ns = min(SC, T - k * SC);
  for (int i = 0; i < ns; ++i) {
    const int t = t0 + dt * (k * SC + i);
    if (tid < G) {
      float acc = xk[i * G + tid];
      const f32x4* h4 = reinterpret_cast<const f32x4*>(hs);
#pragma unroll
      for (int kq = 0; kq < HM / 4; ++kq) {
        f32x4 hv = h4[kq];
        acc += hv[0] * w[4 * kq] + hv[1] * w[4 * kq + 1] + hv[2] * w[4 * kq + 2] + hv[3] * w[4 * kq + 3];
      }
      const float gv = q == 2 ? tanhf(acc) : sigmoidf_(acc);
      gs[tid] = gv;
      gout[((long long)b * T + t) * ldx + d * G + tid] = gv;
    }
    __syncthreads();
    if (tid < H) {
      const float ig = gs[tid], fg = gs[H + tid], gg = gs[2 * H + tid], og = gs[3 * H + tid];
      c = fg * c + ig * gg;
      const float h = og * tanhf(c);
      hs[tid] = h;
      const long long o = ((long long)b * T + t) * ldh + d * H + tid;
      hout[o] = h;
      cout[o] = c;
    }
    __syncthreads();
  }
    if (k + 1 < nch) {
      commit((k + 1) & 1);
      __syncthreads();
    }
  }
}

template <int HM>
__global__ void __launch_bounds__(256) lstm_small_bwd(const float* __restrict__ dhout, const float* __restrict__ call,
                                                      const float* __restrict__ gall, const float* __restrict__ whh,
                                                      int T, int H, int dirs, float* __restrict__ dg) {
  constexpr int RM = 7 * HM, NPF = (SC * RM + 255) / 256;
  const int b = blockIdx.x, d = blockIdx.y, tid = threadIdx.x;
  const int G = 4 * H, R = 7 * H;
  __shared__ float dhs[HM];
  __shared__ float dgs[4 * HM];
  __shared__ float rs[2][SC * RM];  // per step: dh | c | c_prev | i f g o
  // k-role: thread (k = tid>>2, q = tid&3) holds W[q*H + g'][k], g' < H
  const int kk = tid >> 2, qq = tid & 3;
  float wc[HM];
  const float* W = whh + (long long)d * G * H;
#pragma unroll
  for (int g = 0; g < HM; ++g) wc[g] = (kk < H && g < H) ? W[(long long)(qq * H + g) * H + kk] : 0.f;
  if (tid < HM) dhs[tid] = 0.f;
  for (int i = tid; i < 4 * HM; i += 256) dgs[i] = 0.f;
  float dc = 0.f;
  const long long ldg = (long long)dirs * G, ldh = (long long)dirs * H;
  // backward walks opposite to the forward recurrence
  const int t0 = d ? 0 : T - 1, dt = d ? 1 : -1;
  const int fwd_prev = d ? 1 : -1;  // offset of the forward's previous time step
  const float* dhb = dhout + (long long)b * T * ldh + d * H;
  const float* cb = call + (long long)b * T * ldh + d * H;
  const float* gb = gall + (long long)b * T * ldg + d * G;
  // chunk element e: step s = k*SC + e/R, column e%R of the staged row
  float pf[NPF];
  auto issue = [&](int k) {
#pragma unroll
    for (int i = 0; i < NPF; ++i) {
      const int e = tid + 256 * i, si = e / R, col = e - si * R, s = k * SC + si;
      float v = 0.f;
      if (si < SC && s < T) {
        const int t = t0 + dt * s, seg = col / H, u = col - seg * H;
        if (seg == 0) {
          v = dhb[(long long)t * ldh + u];
        } else if (seg == 1) {
          v = cb[(long long)t * ldh + u];
        } else if (seg == 2) {
          const int tp = t + fwd_prev;
          v = (tp >= 0 && tp < T) ? cb[(long long)tp * ldh + u] : 0.f;
        } else {
          v = gb[(long long)t * ldg + (col - 3 * H)];
        }
      }
      pf[i] = v;
    }
  };
  auto commit = [&](int buf) {
#pragma unroll
    for (int i = 0; i < NPF; ++i) {
      const int e = tid + 256 * i;
      if (e < SC * R) rs[buf][e] = pf[i];
    }
  };
  const int nch = (T + SC - 1) / SC;
  issue(0);
  commit(0);
  __syncthreads();
  for (int k = 0; k < nch; ++k) {
    if (k + 1 < nch) issue(k + 1);
    const float* rk = rs[k & 1];
    const int ns = min(SC, T - k * SC);
  for (int i = 0; i < ns; ++i) {
    const int t = t0 + dt * (k * SC + i);
    if (tid < H) {
      const float* row = rk + i * R;
      const float dh = row[tid] + dhs[tid];
      const float c = row[H + tid], cp = row[2 * H + tid];
      const float ig = row[3 * H + tid], fg = row[4 * H + tid], gg = row[5 * H + tid], og = row[6 * H + tid];
      const float tc = tanhf(c);
      const float do_ = dh * tc;
      float dcs = dc + dh * og * (1.f - tc * tc);
      const float di = dcs * gg, dgg = dcs * ig, df = dcs * cp;
      dc = dcs * fg;
      const float a0 = di * ig * (1.f - ig), a1 = df * fg * (1.f - fg), a2 = dgg * (1.f - gg * gg),
                  a3 = do_ * og * (1.f - og);
      const long long og_ = ((long long)b * T + t) * ldg + d * G + tid;
      dg[og_] = a0;
      dg[og_ + H] = a1;
      dg[og_ + 2 * H] = a2;
      dg[og_ + 3 * H] = a3;
      dgs[tid] = a0;
      dgs[H + tid] = a1;
      dgs[2 * H + tid] = a2;
      dgs[3 * H + tid] = a3;
    }
    __syncthreads();
    if (tid < 4 * H) {
      float p = 0.f;
      const float* src = dgs + qq * H;
#pragma unroll
      for (int g = 0; g < HM; ++g) p += (g < H ? src[g] : 0.f) * wc[g];
      p += __shfl_xor(p, 1, 64);
      p += __shfl_xor(p, 2, 64);
      if (qq == 0 && kk < H) dhs[kk] = p;
    }
    __syncthreads();
  }
    if (k + 1 < nch) {
      commit((k + 1) & 1);
      __syncthreads();
    }
  }
}

// =============================================================== large H: per-step kernels
struct StepArgs {
  const float* xproj;  // (B,T,dirs*4H)
  const void* w;       // fwd: dirs x [4H][H]; bwd: dirs x [H][4H]
  float* hout;         // (B,T,dirs*H)
  float* call;         // (B,T,dirs*H)
  float* gall;         // (B,T,dirs*4H) activated gates
  void* hb;            // bf16 ping-pong [2][dirs][B][H] (fwd) / [2][dirs][B][4H] (bwd)
  const float* dhout;  // bwd
  float* dg;           // bwd (B,T,dirs*4H)
  float* dcb;          // bwd [dirs][B][H]
  int B, T, H, dirs, s;
  int dbg;  // diagnostic ablation bits (AVC_LSTM_DEBUG): 1 skip product, 2 skip stores
};

template <bool BF, int MT>
__global__ void __launch_bounds__(256) lstm_step_fwd(StepArgs a) {
  const int H = a.H, G = 4 * H, T = a.T, B = a.B;
  const int d = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int j0 = blockIdx.x * 8, b0 = blockIdx.y * 16 * MT;
  const int t = d ? T - 1 - a.s : a.s;
  const int tp = d ? t + 1 : t - 1;
  const long long ldx = (long long)a.dirs * G, ldh = (long long)a.dirs * H;
  __shared__ float red[4][16 * MT][33];

  // prefetch the epilogue's inputs (independent of the GEMM)
  const int pr = tid >> 3, pj = tid & 7;
  const int pb = b0 + pr;
  const bool pv = pr < 16 * MT && pb < B;
  float px[4] = {0.f, 0.f, 0.f, 0.f}, pcp = 0.f;
  if (pv) {
    const long long ox = ((long long)pb * T + t) * ldx + d * G + j0 + pj;
#pragma unroll
    for (int q = 0; q < 4; ++q) px[q] = a.xproj[ox + q * H];
    if (a.s > 0) pcp = a.call[((long long)pb * T + tp) * ldh + d * H + j0 + pj];
  }

  f32x4 acc[MT][2];
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m][0] = acc[m][1] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (a.s > 0) {
    const int kw = H / 4, kbeg = w * kw;
    const int r16 = lane & 15, kh = lane >> 4;
    if constexpr (BF) {
      const bf16* hp = reinterpret_cast<const bf16*>(a.hb) + ((long long)((a.s - 1) & 1) * a.dirs + d) * B * H;
      const bf16* W = reinterpret_cast<const bf16*>(a.w) + (long long)d * G * H;
      const bf16* arow[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        int b = b0 + m * 16 + r16;
        arow[m] = b < B ? hp + (long long)b * H : nullptr;
      }
      const bf16* brow[2];
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        int col = n * 16 + r16;
        brow[n] = W + (long long)((col >> 3) * H + j0 + (col & 7)) * H;
      }
      const bf16x8 z = {};
#pragma unroll 4
      for (int k0 = kbeg; k0 < kbeg + kw; k0 += 32) {
        const int ko = k0 + 8 * kh;
        bf16x8 af[MT], bfr[2];
#pragma unroll
        for (int m = 0; m < MT; ++m) af[m] = arow[m] ? *reinterpret_cast<const bf16x8*>(arow[m] + ko) : z;
#pragma unroll
        for (int n = 0; n < 2; ++n) bfr[n] = *reinterpret_cast<const bf16x8*>(brow[n] + ko);
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
          for (int n = 0; n < 2; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m], bfr[n], acc[m][n], 0, 0, 0);
      }
    } else {
      const float* W = reinterpret_cast<const float*>(a.w) + (long long)d * G * H;
      const float* arow[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        int b = b0 + m * 16 + r16;
        arow[m] = b < B ? a.hout + ((long long)b * T + tp) * ldh + d * H : nullptr;
      }
      const float* brow[2];
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        int col = n * 16 + r16;
        brow[n] = W + (long long)((col >> 3) * H + j0 + (col & 7)) * H;
      }
#pragma unroll 8
      for (int k0 = kbeg; k0 < kbeg + kw; k0 += 4) {
        float af[MT], bfr[2];
#pragma unroll
        for (int m = 0; m < MT; ++m) af[m] = arow[m] ? arow[m][k0 + kh] : 0.f;
#pragma unroll
        for (int n = 0; n < 2; ++n) bfr[n] = brow[n][k0 + kh];
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
          for (int n = 0; n < 2; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[m], bfr[n], acc[m][n], 0, 0, 0);
      }
    }
  }
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int e = 0; e < 4; ++e) red[w][m * 16 + 4 * (lane >> 4) + e][n * 16 + (lane & 15)] = acc[m][n][e];
  __syncthreads();
  if (pv) {
    float pre[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      pre[q] = px[q] + red[0][pr][q * 8 + pj] + red[1][pr][q * 8 + pj] + red[2][pr][q * 8 + pj] + red[3][pr][q * 8 + pj];
    const float ig = sigmoidf_(pre[0]), fg = sigmoidf_(pre[1]), gg = tanhf(pre[2]), og = sigmoidf_(pre[3]);
    const float c = fg * pcp + ig * gg;
    const float h = og * tanhf(c);
    const int j = j0 + pj;
    const long long oh = ((long long)pb * T + t) * ldh + d * H + j;
    a.hout[oh] = h;
    a.call[oh] = c;
    const long long og_ = ((long long)pb * T + t) * ldx + d * G + j;
    a.gall[og_] = ig;
    a.gall[og_ + H] = fg;
    a.gall[og_ + 2 * H] = gg;
    a.gall[og_ + 3 * H] = og;
    if constexpr (BF) {
      bf16* hn = reinterpret_cast<bf16*>(a.hb) + ((long long)(a.s & 1) * a.dirs + d) * B * H;
      hn[(long long)pb * H + j] = (bf16)h;
    }
  }
}

template <bool BF, int MT>
__global__ void __launch_bounds__(256) lstm_step_bwd(StepArgs a) {
  const int H = a.H, G = 4 * H, T = a.T, B = a.B;
  const int d = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int j0 = blockIdx.x * 16, b0 = blockIdx.y * 16 * MT;
  const int t = d ? a.s : T - 1 - a.s;
  const int tn = d ? t - 1 : t + 1;  // time handled by the previous backward step
  const int tp = d ? t + 1 : t - 1;  // forward's previous time step
  const long long ldg = (long long)a.dirs * G, ldh = (long long)a.dirs * H;
  __shared__ float red[4][16 * MT][17];
  constexpr int PPT = MT;  // (row, unit) pairs per thread: 16*MT*16 / 256

  float pdh[PPT], pc[PPT], pcp[PPT], pg[PPT][4], pdc[PPT];
  int prow[PPT], pjj[PPT];
  bool pv[PPT];
#pragma unroll
  for (int u = 0; u < PPT; ++u) {
    const int p = tid + 256 * u;
    prow[u] = p >> 4;
    pjj[u] = p & 15;
    const int b = b0 + prow[u];
    pv[u] = b < B;
    pdh[u] = pc[u] = pcp[u] = pdc[u] = 0.f;
    pg[u][0] = pg[u][1] = pg[u][2] = pg[u][3] = 0.f;
    if (pv[u]) {
      const int j = j0 + pjj[u];
      const long long oh = ((long long)b * T + t) * ldh + d * H + j;
      pdh[u] = a.dhout[oh];
      pc[u] = a.call[oh];
      if (tp >= 0 && tp < T) pcp[u] = a.call[((long long)b * T + tp) * ldh + d * H + j];
      const long long og_ = ((long long)b * T + t) * ldg + d * G + j;
#pragma unroll
      for (int q = 0; q < 4; ++q) pg[u][q] = a.gall[og_ + q * H];
      if (a.s > 0) pdc[u] = a.dcb[((long long)d * B + b) * H + j];
    }
  }

  f32x4 acc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (a.s > 0) {
    const int kw = G / 4, kbeg = w * kw;
    const int r16 = lane & 15, kh = lane >> 4;
    if constexpr (BF) {
      const bf16* gp = reinterpret_cast<const bf16*>(a.hb) + ((long long)((a.s - 1) & 1) * a.dirs + d) * B * G;
      const bf16* WT = reinterpret_cast<const bf16*>(a.w) + (long long)d * H * G;
      const bf16* arow[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        int b = b0 + m * 16 + r16;
        arow[m] = b < B ? gp + (long long)b * G : nullptr;
      }
      const bf16* brow = WT + (long long)(j0 + r16) * G;
      const bf16x8 z = {};
#pragma unroll 4
      for (int k0 = kbeg; k0 < kbeg + kw; k0 += 32) {
        const int ko = k0 + 8 * kh;
        bf16x8 bfr = *reinterpret_cast<const bf16x8*>(brow + ko);
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          bf16x8 af = arow[m] ? *reinterpret_cast<const bf16x8*>(arow[m] + ko) : z;
          acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr, acc[m], 0, 0, 0);
        }
      }
    } else {
      const float* WT = reinterpret_cast<const float*>(a.w) + (long long)d * H * G;
      const float* arow[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        int b = b0 + m * 16 + r16;
        arow[m] = b < B ? a.dg + ((long long)b * T + tn) * ldg + d * G : nullptr;
      }
      const float* brow = WT + (long long)(j0 + r16) * G;
#pragma unroll 8
      for (int k0 = kbeg; k0 < kbeg + kw; k0 += 4) {
        float bfr = brow[k0 + kh];
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          float af = arow[m] ? arow[m][k0 + kh] : 0.f;
          acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(af, bfr, acc[m], 0, 0, 0);
        }
      }
    }
  }
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int e = 0; e < 4; ++e) red[w][m * 16 + 4 * (lane >> 4) + e][lane & 15] = acc[m][e];
  __syncthreads();
#pragma unroll
  for (int u = 0; u < PPT; ++u) {
    if (!pv[u]) continue;
    const int r = prow[u], jl = pjj[u], b = b0 + r, j = j0 + jl;
    const float dh = pdh[u] + red[0][r][jl] + red[1][r][jl] + red[2][r][jl] + red[3][r][jl];
    const float ig = pg[u][0], fg = pg[u][1], gg = pg[u][2], og = pg[u][3];
    const float tc = tanhf(pc[u]);
    const float do_ = dh * tc;
    const float dcs = pdc[u] + dh * og * (1.f - tc * tc);
    const float di = dcs * gg, dgg = dcs * ig, df = dcs * pcp[u];
    a.dcb[((long long)d * B + b) * H + j] = dcs * fg;
    const float v[4] = {di * ig * (1.f - ig), df * fg * (1.f - fg), dgg * (1.f - gg * gg), do_ * og * (1.f - og)};
    const long long og_ = ((long long)b * T + t) * ldg + d * G + j;
#pragma unroll
    for (int q = 0; q < 4; ++q) a.dg[og_ + q * H] = v[q];
    if constexpr (BF) {
      bf16* gn = reinterpret_cast<bf16*>(a.hb) + ((long long)(a.s & 1) * a.dirs + d) * B * G + (long long)b * G;
#pragma unroll
      for (int q = 0; q < 4; ++q) gn[q * H + j] = (bf16)v[q];
    }
  }
}


// ---------------------------------------------------------------- bf16 step kernels, H known
// Every operand fragment of a wave's K-slice is loaded before the first MFMA, so a step
// pays ONE L2/MALL round trip instead of one per k-step.
template <int H, int MT>
__global__ void __launch_bounds__(256) lstm_step_fwd_bf(StepArgs a) {
  constexpr int G = 4 * H, KW = H / 4, NK = KW / 32;
  const int T = a.T, B = a.B, d = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int j0 = blockIdx.x * 8, b0 = blockIdx.y * 16 * MT;
  const int t = d ? T - 1 - a.s : a.s;
  const int tp = d ? t + 1 : t - 1;
  const long long ldx = (long long)a.dirs * G, ldh = (long long)a.dirs * H;
  __shared__ float red[4][16 * MT][33];
  const int pr = tid >> 3, pj = tid & 7, pb = b0 + pr;
  const bool pv = pr < 16 * MT && pb < B;
  float px[4] = {0.f, 0.f, 0.f, 0.f}, pcp = 0.f;
  if (pv) {
    const long long ox = ((long long)pb * T + t) * ldx + d * G + j0 + pj;
#pragma unroll
    for (int q = 0; q < 4; ++q) px[q] = a.xproj[ox + q * H];
    if (a.s > 0) pcp = a.call[((long long)pb * T + tp) * ldh + d * H + j0 + pj];
  }
  f32x4 acc[MT][2];
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m][0] = acc[m][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (a.s > 0 && !(a.dbg & 1)) {
    const int r16 = lane & 15, ko = w * KW + 8 * (lane >> 4);
    const bf16* hp = reinterpret_cast<const bf16*>(a.hb) + ((long long)((a.s - 1) & 1) * a.dirs + d) * B * H;
    const bf16* W = reinterpret_cast<const bf16*>(a.w) + (long long)d * G * H;
    bf16x8 af[NK][MT], bw[NK][2];
    const bf16x8 z = {};
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int b = b0 + m * 16 + r16;
      const bf16* row = hp + (long long)(b < B ? b : 0) * H + ko;
#pragma unroll
      for (int k = 0; k < NK; ++k) af[k][m] = b < B ? *reinterpret_cast<const bf16x8*>(row + 32 * k) : z;
    }
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const int col = n * 16 + r16;
      const bf16* row = W + (long long)((col >> 3) * H + j0 + (col & 7)) * H + ko;
#pragma unroll
      for (int k = 0; k < NK; ++k) bw[k][n] = *reinterpret_cast<const bf16x8*>(row + 32 * k);
    }
#pragma unroll
    for (int k = 0; k < NK; ++k)
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[k][m], bw[k][n], acc[m][n], 0, 0, 0);
  }
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int e = 0; e < 4; ++e) red[w][m * 16 + 4 * (lane >> 4) + e][n * 16 + (lane & 15)] = acc[m][n][e];
  __syncthreads();
  if (pv && !(a.dbg & 2)) {
    float pre[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      pre[q] = px[q] + red[0][pr][q * 8 + pj] + red[1][pr][q * 8 + pj] + red[2][pr][q * 8 + pj] + red[3][pr][q * 8 + pj];
    const float ig = sigmoidf_(pre[0]), fg = sigmoidf_(pre[1]), gg = tanhf(pre[2]), og = sigmoidf_(pre[3]);
    const float c = fg * pcp + ig * gg;
    const float h = og * tanhf(c);
    const int j = j0 + pj;
    const long long oh = ((long long)pb * T + t) * ldh + d * H + j;
    a.hout[oh] = h;
    a.call[oh] = c;
    const long long og_ = ((long long)pb * T + t) * ldx + d * G + j;
    a.gall[og_] = ig;
    a.gall[og_ + H] = fg;
    a.gall[og_ + 2 * H] = gg;
    a.gall[og_ + 3 * H] = og;
    bf16* hn = reinterpret_cast<bf16*>(a.hb) + ((long long)(a.s & 1) * a.dirs + d) * B * H;
    hn[(long long)pb * H + j] = (bf16)h;
  }
}

// backward: 8 waves split K = 4H; tile 16 utterances x 16 hidden units.
template <int H>
__global__ void __launch_bounds__(512) lstm_step_bwd_bf(StepArgs a) {
  constexpr int G = 4 * H, KW = G / 8, NK = KW / 32;
  const int T = a.T, B = a.B, d = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int j0 = blockIdx.x * 16, b0 = blockIdx.y * 16;
  const int t = d ? a.s : T - 1 - a.s;
  const int tp = d ? t + 1 : t - 1;
  const long long ldg = (long long)a.dirs * G, ldh = (long long)a.dirs * H;
  __shared__ float red[8][16][17];
  const int prow = tid >> 4, pjj = tid & 15, pb = b0 + prow;
  const bool pv = tid < 256 && pb < B;
  float pdh = 0.f, pc = 0.f, pcp = 0.f, pdc = 0.f, pg[4] = {0.f, 0.f, 0.f, 0.f};
  if (pv) {
    const int j = j0 + pjj;
    const long long oh = ((long long)pb * T + t) * ldh + d * H + j;
    pdh = a.dhout[oh];
    pc = a.call[oh];
    if (tp >= 0 && tp < T) pcp = a.call[((long long)pb * T + tp) * ldh + d * H + j];
    const long long og_ = ((long long)pb * T + t) * ldg + d * G + j;
#pragma unroll
    for (int q = 0; q < 4; ++q) pg[q] = a.gall[og_ + q * H];
    if (a.s > 0) pdc = a.dcb[((long long)d * B + pb) * H + j];
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (a.s > 0) {
    const int r16 = lane & 15, ko = w * KW + 8 * (lane >> 4);
    const bf16* gp = reinterpret_cast<const bf16*>(a.hb) + ((long long)((a.s - 1) & 1) * a.dirs + d) * B * G;
    const bf16* WT = reinterpret_cast<const bf16*>(a.w) + (long long)d * H * G;
    const int b = b0 + r16;
    const bf16* arow = gp + (long long)(b < B ? b : 0) * G + ko;
    const bf16* brow = WT + (long long)(j0 + r16) * G + ko;
    bf16x8 af[NK], bw[NK];
    const bf16x8 z = {};
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      af[k] = b < B ? *reinterpret_cast<const bf16x8*>(arow + 32 * k) : z;
      bw[k] = *reinterpret_cast<const bf16x8*>(brow + 32 * k);
    }
#pragma unroll
    for (int k = 0; k < NK; ++k) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[k], bw[k], acc, 0, 0, 0);
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) red[w][4 * (lane >> 4) + e][lane & 15] = acc[e];
  __syncthreads();
  if (pv) {
    const int j = j0 + pjj;
    float dh = pdh;
#pragma unroll
    for (int ww = 0; ww < 8; ++ww) dh += red[ww][prow][pjj];
    const float ig = pg[0], fg = pg[1], gg = pg[2], og = pg[3];
    const float tc = tanhf(pc);
    const float do_ = dh * tc;
    const float dcs = pdc + dh * og * (1.f - tc * tc);
    const float di = dcs * gg, dgg = dcs * ig, df = dcs * pcp;
    a.dcb[((long long)d * B + pb) * H + j] = dcs * fg;
    const float v[4] = {di * ig * (1.f - ig), df * fg * (1.f - fg), dgg * (1.f - gg * gg), do_ * og * (1.f - og)};
    const long long og_ = ((long long)pb * T + t) * ldg + d * G + j;
    bf16* gn = reinterpret_cast<bf16*>(a.hb) + ((long long)(a.s & 1) * a.dirs + d) * B * G + (long long)pb * G;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      a.dg[og_ + q * H] = v[q];
      gn[q * H + j] = (bf16)v[q];
    }
  }
}

// =============================================================== large H: persistent forward
// One launch for all T steps.  Workgroups form NG groups of H/32; group g owns utterance
// rows [8g, 8g+8), member r owns hidden units [32r, 32r+32) and keeps the matching
// 128 rows of W_hh (all four gates) in VGPRs for the whole sequence (wave w = gate w).
// h_t is exchanged inside the group through data-tagged 8-byte granules {tag = step+1,
// two bf16}: one agent-scope (sc1) store per granule, consumers re-read with agent-scope
// loads until every tag matches (MI355X_MICROARCH.md hand-off R2: no flag, no fence).
// Groups are blockIdx % NG: with round-robin dispatch a group sits on one XCD and the
// exchange stays in that XCD's L2 -- a speed assumption only, correctness holds for any
// placement.  Every spin is bounded; on timeout the kernel raises a flag and exits.
constexpr int PRG = 8, PJU = 32;
constexpr unsigned PSPIN = 1u << 22;

struct PersistArgs {
  const float* xproj;
  const bf16* w;
  float* hout;
  bf16* hout16;  // optional bf16 copy of h
  float* call;
  float* gall;
  unsigned long long* xbuf;  // [2][B][H/2] granules, zeroed before launch
  unsigned* flag;            // timeout flag
  unsigned long long* trace;  // diagnostics (avc_lstm_trace), null in production
  int B, T, ng;
};

// Diagnostics: avc_lstm_trace(buf) makes the persistent kernels record the 100 MHz REALTIME
// clock at four points of every step of every workgroup into buf[(wg*T + step)*4 + j]:
// j = 0 step start, 1 exchange complete, 2 recurrent product reduced, 3 step published.
// The stamps go to that buffer only; nothing reads them inside the kernel.
unsigned long long* g_trace = nullptr;

__device__ __forceinline__ void stamp(unsigned long long* tr, int T, int s, int j) {
  if (tr && threadIdx.x == 0) tr[((long long)blockIdx.x * T + s) * 4 + j] = __builtin_amdgcn_s_memrealtime();
}

// Wave 0 polls ONE granule per producing workgroup (lane r reads `src + r*stride`, the
// granule that producer stores last) until all NR tags match, so waiting consumers re-read
// NR words per pass instead of their whole gather (a full-sweep spin by every workgroup kept
// the fabric busy with re-reads of granules that had not changed).  The full sweep that
// follows still checks every tag.  Returns false (flag raised) after a spin timeout.
__device__ __forceinline__ bool probe_producers(const unsigned long long* src, int stride, int NR, unsigned tag,
                                                unsigned* flag) {
  const int lane = threadIdx.x & 63;
  unsigned spins = 0;
  while (true) {
    bool ok = true;
    if (lane < NR)
      ok = (unsigned)(__hip_atomic_load(src + (long long)lane * stride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >>
                      32) == tag;
    if (__all(ok)) return true;
    if (++spins > PSPIN) {
      if (lane == 0) atomicOr(flag, 1u);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

__device__ __forceinline__ unsigned long long granule(unsigned tag, float a, float b) {
  bf16x2 h = {(bf16)a, (bf16)b};
  return ((unsigned long long)tag << 32) | (unsigned long long)__builtin_bit_cast(unsigned, h);
}

// Gather the group's tagged granules of one step into LDS rows of `ap` bf16 pairs
// (row = idx / PER, pair = idx % PER for idx = tid + 256 i).  Loads are issued CH at a time
// unconditionally (all in flight together: a per-granule branch around each load made the
// compiler wait for every load in turn), then matched against the tag; late granules are
// re-read with the whole chunk.  Returns false after a spin timeout (flag raised).
template <int NGR, int PER, int CH>
__device__ __forceinline__ bool gather_granules(const unsigned long long* src, bf16* lds, int ap,
                                                unsigned long long need, unsigned tag, unsigned* flag) {
  const int tid = threadIdx.x;
  unsigned spins = 0;
#pragma unroll
  for (int c0 = 0; c0 < NGR; c0 += CH) {
    while (true) {
      unsigned long long v[CH];
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        const int idx = tid + 256 * (c0 + i), row = idx / PER, c2 = idx - row * PER;
        // rows outside the batch are never needed: read row 0's slot instead (valid memory)
        const int rr = ((need >> (c0 + i)) & 1ull) ? row : 0;
        v[i] = __hip_atomic_load(src + (long long)rr * PER + c2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        const int idx = tid + 256 * (c0 + i), row = idx / PER, c2 = idx - row * PER;
        if (((need >> (c0 + i)) & 1ull) && (unsigned)(v[i] >> 32) == tag) {
          reinterpret_cast<unsigned*>(lds + row * ap)[c2] = (unsigned)v[i];
          need &= ~(1ull << (c0 + i));
        }
      }
      const unsigned long long cm = (CH >= 64 ? ~0ull : ((1ull << CH) - 1ull)) << c0;
      if (!(need & cm)) break;
      if (++spins > PSPIN) {
        atomicOr(flag, 1u);
        return false;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  return true;
}

template <int H>
__global__ void __launch_bounds__(256, 1) lstm_persist_fwd(PersistArgs a) {
  constexpr int G = 4 * H, NK = H / 32, AP = H + 8, H2 = H / 2;
  constexpr int NGR = PRG * H2 / 256;  // granules gathered per thread per step
  __shared__ __attribute__((aligned(16))) bf16 As[16 * AP];
  __shared__ float gs[PRG][4 * PJU + 1];
  __shared__ int quit;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = blockIdx.x % a.ng, r = blockIdx.x / a.ng;
  const int j0 = r * PJU, b0 = g * PRG;
  const int T = a.T, B = a.B;

  bf16x8 wf[2][NK];
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    const bf16* row = a.w + (long long)(w * H + j0 + n * 16 + (lane & 15)) * H + 8 * (lane >> 4);
#pragma unroll
    for (int k = 0; k < NK; ++k) wf[n][k] = *reinterpret_cast<const bf16x8*>(row + 32 * k);
  }
  for (int i = tid; i < 16 * AP / 2; i += 256) reinterpret_cast<unsigned*>(As)[i] = 0u;
  if (tid == 0) quit = 0;
  const int pr = tid >> 5, pu = tid & 31, pb = b0 + pr, pj = j0 + pu;
  const bool pv = pb < B;
  unsigned need0 = 0;  // granules this thread gathers each step (rows inside the batch)
#pragma unroll
  for (int i = 0; i < NGR; ++i)
    if (b0 + (tid + 256 * i) / H2 < B) need0 |= 1u << i;
  float c = 0.f;
  __syncthreads();

  for (int s = 0; s < T; ++s) {
    const int t = s;
    stamp(a.trace, T, s, 0);
    float px[4] = {0.f, 0.f, 0.f, 0.f};
    if (pv) {
      const float* xp = a.xproj + ((long long)pb * T + t) * G + pj;
#pragma unroll
      for (int q = 0; q < 4; ++q) px[q] = xp[q * H];
    }
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    if (s > 0) {
      // ---- gather the group's h_{t-1} (tag == s) into the LDS A tile: wave 0 first waits
      // for every member's last granule (row 0, pair 15 of its 32 units), then all sweep
      const unsigned long long* src = a.xbuf + (long long)((s - 1) & 1) * B * H2 + (long long)b0 * H2;
      if (w == 0 && !probe_producers(src + PJU / 2 - 1, PJU / 2, H / PJU, (unsigned)s, a.flag)) quit = 1;
      __syncthreads();
      if (quit) return;  // block-uniform exit after a spin timeout
      if (!gather_granules<NGR, H2, 16>(src, As, AP, need0, (unsigned)s, a.flag)) quit = 1;
      __syncthreads();
      if (quit) return;
      stamp(a.trace, T, s, 1);
#pragma unroll
      for (int k = 0; k < NK; ++k) {
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(As + (lane & 15) * AP + 32 * k + 8 * (lane >> 4));
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, wf[0][k], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, wf[1][k], acc1, 0, 0, 0);
      }
    }
    if (lane < 32) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        gs[4 * (lane >> 4) + e][w * PJU + (lane & 15)] = acc0[e];
        gs[4 * (lane >> 4) + e][w * PJU + 16 + (lane & 15)] = acc1[e];
      }
    }
    __syncthreads();
    stamp(a.trace, T, s, 2);
    float h = 0.f, ig = 0.f, fg = 0.f, gg = 0.f, og = 0.f;
    if (pv) {
      ig = sigmoidf_(px[0] + gs[pr][pu]);
      fg = sigmoidf_(px[1] + gs[pr][PJU + pu]);
      gg = tanhf(px[2] + gs[pr][2 * PJU + pu]);
      og = sigmoidf_(px[3] + gs[pr][3 * PJU + pu]);
      c = fg * c + ig * gg;
      h = og * tanhf(c);
    }
    const float hn = __shfl_down(h, 1, 64);
    if (pv && !(pu & 1) && s + 1 < T)
      __hip_atomic_store(a.xbuf + (long long)(s & 1) * B * H2 + (long long)pb * H2 + (pj >> 1),
                         granule((unsigned)(s + 1), h, hn), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    stamp(a.trace, T, s, 3);
    if (pv) {
      const long long oh = ((long long)pb * T + t) * H + pj;
      a.hout[oh] = h;
      if (a.hout16) a.hout16[oh] = (bf16)h;
      a.call[oh] = c;
      float* gp = a.gall + ((long long)pb * T + t) * G + pj;
      gp[0] = ig;
      gp[H] = fg;
      gp[2 * H] = gg;
      gp[3 * H] = og;
    }
  }
}

// =============================================================== large H: persistent backward
// One launch for all T steps of dirs == 1 (the decoder LSTMs).  Same decomposition as the
// forward: group g = utterances [8g, 8g+8), member r = hidden units [32r, 32r+32).  The
// recurrent product dh_rec[b][j] = sum_q dG_{t+1}[b][q] W_hh[q][j] runs over all 4H gate
// rows q, so each member keeps W_hh^T[j0..j0+32][0..4H) in VGPRs (wave w = the K-block of
// gate w, 2 x H/32 bf16x8 fragments) and gathers the group's whole dG_{t+1} (8 x 4H bf16)
// into LDS each step from tagged granules {tag = step + 1, two bf16}.  The four waves'
// partial products are summed through LDS; the cell-gradient carry dc stays in a register
// of the thread that owns (b, j) for the whole sequence.  Outputs: dG (fp32) and its bf16
// twin for the input-gradient / weight-gradient GEMMs.  Bounded spins as in the forward.
struct PersistBwdArgs {
  const float* dhout;  // (B,T,H)
  const float* call;   // (B,T,H) cell states
  const float* gall;   // (B,T,4H) activated gates i,f,g,o
  const bf16* wt;      // W_hh^T [H][4H]
  float* dg;           // (B,T,4H)
  bf16* dg16;          // (B,T,4H) or null
  unsigned long long* xbuf;  // [2][B][2H] granules, zeroed before launch
  unsigned* flag;
  unsigned long long* trace;  // diagnostics (avc_lstm_trace), null in production
  int B, T, ng;
};

template <int H>
__global__ void __launch_bounds__(256, 1) lstm_persist_bwd(PersistBwdArgs a) {
  constexpr int G = 4 * H, NK = H / 32, AP = G + 8, G2 = G / 2;
  constexpr int NGR = PRG * G2 / 256;  // granules gathered per thread per step
  static_assert(NGR <= 64, "gather mask is 64 bits");
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16* As = reinterpret_cast<bf16*>(smem_raw);                          // [PRG + 1][AP], row PRG = zeros
  float* red = reinterpret_cast<float*>(smem_raw + (PRG + 1) * AP * 2);  // [4][PRG][PJU + 1]
  int* quit = reinterpret_cast<int*>(red + 4 * PRG * (PJU + 1));
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = blockIdx.x % a.ng, r = blockIdx.x / a.ng;
  const int j0 = r * PJU, b0 = g * PRG;
  const int T = a.T, B = a.B;

  // W_hh^T fragments: B operand of the product, n = unit j0 + 16n + (lane&15), k = gate row
  bf16x8 wf[2][NK];
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    const bf16* row = a.wt + (long long)(j0 + n * 16 + (lane & 15)) * G + w * H + 8 * (lane >> 4);
#pragma unroll
    for (int k = 0; k < NK; ++k) wf[n][k] = *reinterpret_cast<const bf16x8*>(row + 32 * k);
  }
  for (int i = tid; i < (PRG + 1) * AP / 2; i += 256) reinterpret_cast<unsigned*>(As)[i] = 0u;
  if (tid == 0) *quit = 0;
  const int pr = tid >> 5, pu = tid & 31, pb = b0 + pr, pj = j0 + pu;
  const bool pv = pb < B;
  unsigned long long need0 = 0;
#pragma unroll
  for (int i = 0; i < NGR; ++i)
    if (b0 + (tid + 256 * i) / G2 < B) need0 |= 1ull << i;
  // MFMA A rows: 0..7 gathered utterances, 8..15 read the zero row
  const int arow = (lane & 15) < PRG ? (lane & 15) : PRG;
  float dc = 0.f;
  __syncthreads();

  for (int s = 0; s < T; ++s) {
    const int t = T - 1 - s;
    stamp(a.trace, T, s, 0);
    // per-element inputs of this step (independent of the exchange: issued first)
    float dh = 0.f, ct = 0.f, cp = 0.f, gi = 0.f, gf = 0.f, gg = 0.f, go = 0.f;
    if (pv) {
      const long long oh = ((long long)pb * T + t) * H + pj;
      dh = a.dhout[oh];
      ct = a.call[oh];
      cp = t > 0 ? a.call[oh - H] : 0.f;
      const float* gp = a.gall + ((long long)pb * T + t) * G + pj;
      gi = gp[0];
      gf = gp[H];
      gg = gp[2 * H];
      go = gp[3 * H];
    }
    if (s > 0) {
      const unsigned long long* src = a.xbuf + (long long)((s - 1) & 1) * B * G2 + (long long)b0 * G2;
      // wave 0 waits for every member's last granule (row 0, gate o, pair 15), then all sweep
      if (w == 0 && !probe_producers(src + 3 * H / 2 + PJU / 2 - 1, PJU / 2, H / PJU, (unsigned)s, a.flag))
        *quit = 1;
      __syncthreads();
      if (*quit) return;  // block-uniform exit after a spin timeout
      if (!gather_granules<NGR, G2, 16>(src, As, AP, need0, (unsigned)s, a.flag)) *quit = 1;
      __syncthreads();
      if (*quit) return;
      stamp(a.trace, T, s, 1);
      f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      const bf16* ap = As + arow * AP + w * H + 8 * (lane >> 4);
#pragma unroll
      for (int k = 0; k < NK; ++k) {
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(ap + 32 * k);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, wf[0][k], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, wf[1][k], acc1, 0, 0, 0);
      }
      // rows 4*(lane>>4)+e < 8 only for lanes 0..31
      if (lane < 32) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          red[(w * PRG + 4 * (lane >> 4) + e) * (PJU + 1) + (lane & 15)] = acc0[e];
          red[(w * PRG + 4 * (lane >> 4) + e) * (PJU + 1) + 16 + (lane & 15)] = acc1[e];
        }
      }
      __syncthreads();
      stamp(a.trace, T, s, 2);
#pragma unroll
      for (int ww = 0; ww < 4; ++ww) dh += red[(ww * PRG + pr) * (PJU + 1) + pu];
    }
    float v0 = 0.f, v1 = 0.f, v2 = 0.f, v3 = 0.f;
    if (pv) {
      const float tc = tanhf(ct);
      const float dcs = dc + dh * go * (1.f - tc * tc);
      v0 = dcs * gg * gi * (1.f - gi);        // d(pre i)
      v1 = dcs * cp * gf * (1.f - gf);        // d(pre f)
      v2 = dcs * gi * (1.f - gg * gg);        // d(pre g)
      v3 = dh * tc * go * (1.f - go);         // d(pre o)
      dc = dcs * gf;
    }
    const float n0 = __shfl_down(v0, 1, 64), n1 = __shfl_down(v1, 1, 64);
    const float n2 = __shfl_down(v2, 1, 64), n3 = __shfl_down(v3, 1, 64);
    if (pv && !(pu & 1) && s + 1 < T) {
      unsigned long long* dst = a.xbuf + (long long)(s & 1) * B * G2 + (long long)pb * G2 + (pj >> 1);
      const unsigned tag = (unsigned)(s + 1);
      __hip_atomic_store(dst, granule(tag, v0, n0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(dst + H / 2, granule(tag, v1, n1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(dst + H, granule(tag, v2, n2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(dst + 3 * H / 2, granule(tag, v3, n3), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    stamp(a.trace, T, s, 3);
    if (pv) {
      const long long og = ((long long)pb * T + t) * G + pj;
      a.dg[og] = v0;
      a.dg[og + H] = v1;
      a.dg[og + 2 * H] = v2;
      a.dg[og + 3 * H] = v3;
      if (a.dg16) {
        a.dg16[og] = (bf16)v0;
        a.dg16[og + H] = (bf16)v1;
        a.dg16[og + 2 * H] = (bf16)v2;
        a.dg16[og + 3 * H] = (bf16)v3;
      }
    }
  }
}

template <int H>
constexpr size_t persist_bwd_lds() {
  return (size_t)(PRG + 1) * (4 * H + 8) * 2 + (size_t)4 * PRG * (PJU + 1) * 4 + 16;
}

int g_num_cus = -1;
int num_cus() {
  if (g_num_cus < 0) {
    int dev = 0;
    hipDeviceProp_t prop;
    g_num_cus = (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
                    ? prop.multiProcessorCount : 0;
  }
  return g_num_cus;
}

template <int HM>
void launch_small_fwd(dim3 g, hipStream_t s, const float* x, const float* w, int T, int H, int dirs, float* h, float* c,
                      float* gt) {
  lstm_small_fwd<HM><<<g, 256, 0, s>>>(x, w, T, H, dirs, h, c, gt);
}
template <int HM>
void launch_small_bwd(dim3 g, hipStream_t s, const float* dh, const float* c, const float* gt, const float* w, int T,
                      int H, int dirs, float* dg) {
  lstm_small_bwd<HM><<<g, 256, 0, s>>>(dh, c, gt, w, T, H, dirs, dg);
}

}  // namespace

extern "C" int avc_lstm_trace(void* buf) {
  g_trace = reinterpret_cast<unsigned long long*>(buf);
  return 0;
}

extern "C" int avc_lstm_fwd(const float* xproj, const void* w_hh, int wdtype, int B, int T, int H, int dirs, float* h,
                            void* h_bf16, float* c, float* gates, void* hbuf, int compute, void* stream) {
  AVC_CHECK_ARG(xproj && w_hh && h && c && gates && B > 0 && T > 0 && H > 0 && (dirs == 1 || dirs == 2),
                "avc_lstm_fwd: bad args");
  hipStream_t s = as_stream(stream);
  if (H <= 64) {
    AVC_CHECK_ARG(wdtype == AVC_F32, "avc_lstm_fwd: small-H path takes fp32 W_hh");
    dim3 g(B, dirs);
    if (H <= 16) launch_small_fwd<16>(g, s, xproj, (const float*)w_hh, T, H, dirs, h, c, gates);
    else if (H <= 32) launch_small_fwd<32>(g, s, xproj, (const float*)w_hh, T, H, dirs, h, c, gates);
    else if (H <= 48) launch_small_fwd<48>(g, s, xproj, (const float*)w_hh, T, H, dirs, h, c, gates);
    else launch_small_fwd<64>(g, s, xproj, (const float*)w_hh, T, H, dirs, h, c, gates);
    return avc_check_launch("avc_lstm_fwd(small)");
  }
  AVC_CHECK_ARG(H % 128 == 0, "avc_lstm_fwd: H must be <= 64 or a multiple of 128 (got %d)", H);
  const bool bf = compute == AVC_BF16;
  AVC_CHECK_ARG(!bf || (wdtype == AVC_BF16 && hbuf), "avc_lstm_fwd: bf16 compute needs bf16 W_hh and hbuf");
  AVC_CHECK_ARG(bf || wdtype == AVC_F32, "avc_lstm_fwd: fp32 compute needs fp32 W_hh");
  StepArgs a = {};
  static const int dbg = getenv("AVC_LSTM_DEBUG") ? atoi(getenv("AVC_LSTM_DEBUG")) : 0;
  a.dbg = dbg;
  a.xproj = xproj;
  a.w = w_hh;
  a.hout = h;
  a.call = c;
  a.gall = gates;
  a.hb = hbuf;
  a.B = B;
  a.T = T;
  a.H = H;
  a.dirs = dirs;
  const int ng = (B + PRG - 1) / PRG;
  static const bool no_persist = getenv("AVC_LSTM_NO_PERSIST") != nullptr;
  if (bf && dirs == 1 && (H == 1024 || H == 512) && hbuf && !no_persist && ng * (H / PJU) <= num_cus()) {
    // hbuf is the granule scratch (>= 2*B*H/2 u64 + a flag word) in this mode
    PersistArgs p;
    p.xproj = xproj;
    p.w = reinterpret_cast<const bf16*>(w_hh);
    p.hout = h;
    p.hout16 = reinterpret_cast<bf16*>(h_bf16);
    p.call = c;
    p.gall = gates;
    p.xbuf = reinterpret_cast<unsigned long long*>(hbuf);
    p.flag = reinterpret_cast<unsigned*>(p.xbuf + (size_t)2 * B * (H / 2));
    p.trace = g_trace;
    p.B = B;
    p.T = T;
    p.ng = ng;
    (void)hipMemsetAsync(hbuf, 0, ((size_t)2 * B * (H / 2) + 2) * sizeof(unsigned long long), s);
    if (H == 1024) lstm_persist_fwd<1024><<<ng * (H / PJU), 256, 0, s>>>(p);
    else lstm_persist_fwd<512><<<ng * (H / PJU), 256, 0, s>>>(p);
    return avc_check_launch("avc_lstm_fwd(persistent)");
  }
  AVC_CHECK_ARG(h_bf16 == nullptr, "avc_lstm_fwd: the bf16 h copy is produced by the persistent path only");
  const int mt = (H >= 1024 && B > 16) ? 2 : 1;  // 256 workgroups at B = 64
  dim3 g(H / 8, cdiv(B, 16 * mt), dirs);
  for (int st = 0; st < T; ++st) {
    a.s = st;
    if (bf && H == 1024) {
      if (mt == 2) lstm_step_fwd_bf<1024, 2><<<g, 256, 0, s>>>(a);
      else lstm_step_fwd_bf<1024, 1><<<g, 256, 0, s>>>(a);
    } else if (bf && H == 512) {
      if (mt == 2) lstm_step_fwd_bf<512, 2><<<g, 256, 0, s>>>(a);
      else lstm_step_fwd_bf<512, 1><<<g, 256, 0, s>>>(a);
    } else if (bf) {
      if (mt == 2) lstm_step_fwd<true, 2><<<g, 256, 0, s>>>(a);
      else lstm_step_fwd<true, 1><<<g, 256, 0, s>>>(a);
    } else {
      if (mt == 2) lstm_step_fwd<false, 2><<<g, 256, 0, s>>>(a);
      else lstm_step_fwd<false, 1><<<g, 256, 0, s>>>(a);
    }
  }
  return avc_check_launch("avc_lstm_fwd");
}

extern "C" int avc_lstm_bwd(const float* dh_out, const float* h, const float* c, const float* gates, const void* w_hh,
                            const void* w_hh_t, int wdtype, int B, int T, int H, int dirs, float* dgates,
                            void* dgates_bf16, float* dcbuf, void* gbuf, int compute, void* stream) {
  (void)h;
  AVC_CHECK_ARG(dh_out && c && gates && dgates && B > 0 && T > 0 && H > 0 && (dirs == 1 || dirs == 2),
                "avc_lstm_bwd: bad args");
  hipStream_t s = as_stream(stream);
  if (H <= 64) {
    AVC_CHECK_ARG(w_hh && wdtype == AVC_F32, "avc_lstm_bwd: small-H path takes fp32 W_hh");
    dim3 g(B, dirs);
    if (H <= 16) launch_small_bwd<16>(g, s, dh_out, c, gates, (const float*)w_hh, T, H, dirs, dgates);
    else if (H <= 32) launch_small_bwd<32>(g, s, dh_out, c, gates, (const float*)w_hh, T, H, dirs, dgates);
    else if (H <= 48) launch_small_bwd<48>(g, s, dh_out, c, gates, (const float*)w_hh, T, H, dirs, dgates);
    else launch_small_bwd<64>(g, s, dh_out, c, gates, (const float*)w_hh, T, H, dirs, dgates);
    return avc_check_launch("avc_lstm_bwd(small)");
  }
  AVC_CHECK_ARG(H % 128 == 0, "avc_lstm_bwd: H must be <= 64 or a multiple of 128 (got %d)", H);
  AVC_CHECK_ARG(w_hh_t && dcbuf, "avc_lstm_bwd: large-H path needs W_hh^T and dcbuf");
  const bool bf = compute == AVC_BF16;
  AVC_CHECK_ARG(!bf || (wdtype == AVC_BF16 && gbuf), "avc_lstm_bwd: bf16 compute needs bf16 W_hh^T and gbuf");
  const int ng = (B + PRG - 1) / PRG;
  static const bool no_persist = getenv("AVC_LSTM_NO_PERSIST") != nullptr;
  if (bf && dirs == 1 && (H == 1024 || H == 512) && !no_persist && ng * (H / PJU) <= num_cus()) {
    // gbuf is the granule scratch (>= 2*B*2H u64 + a flag word) in this mode
    PersistBwdArgs p;
    p.dhout = dh_out;
    p.call = c;
    p.gall = gates;
    p.wt = reinterpret_cast<const bf16*>(w_hh_t);
    p.dg = dgates;
    p.dg16 = reinterpret_cast<bf16*>(dgates_bf16);
    p.xbuf = reinterpret_cast<unsigned long long*>(gbuf);
    p.flag = reinterpret_cast<unsigned*>(p.xbuf + (size_t)2 * B * (2 * H));
    p.trace = g_trace;
    p.B = B;
    p.T = T;
    p.ng = ng;
    (void)hipMemsetAsync(gbuf, 0, ((size_t)2 * B * (2 * H) + 2) * sizeof(unsigned long long), s);
    if (H == 1024) {
      static bool attr = false;
      if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&lstm_persist_bwd<1024>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)persist_bwd_lds<1024>());
        attr = true;
      }
      lstm_persist_bwd<1024><<<ng * (H / PJU), 256, persist_bwd_lds<1024>(), s>>>(p);
    } else {
      lstm_persist_bwd<512><<<ng * (H / PJU), 256, persist_bwd_lds<512>(), s>>>(p);
    }
    return avc_check_launch("avc_lstm_bwd(persistent)");
  }
  AVC_CHECK_ARG(dgates_bf16 == nullptr, "avc_lstm_bwd: the bf16 dG twin is produced by the persistent path only");
  StepArgs a = {};
  a.w = w_hh_t;
  a.call = const_cast<float*>(c);
  a.gall = const_cast<float*>(gates);
  a.hb = gbuf;
  a.dhout = dh_out;
  a.dg = dgates;
  a.dcb = dcbuf;
  a.B = B;
  a.T = T;
  a.H = H;
  a.dirs = dirs;
  dim3 g(H / 16, cdiv(B, 16), dirs);
  for (int st = 0; st < T; ++st) {
    a.s = st;
    if (bf && H == 1024) lstm_step_bwd_bf<1024><<<g, 512, 0, s>>>(a);
    else if (bf && H == 512) lstm_step_bwd_bf<512><<<g, 512, 0, s>>>(a);
    else if (bf) lstm_step_bwd<true, 1><<<g, 256, 0, s>>>(a);
    else lstm_step_bwd<false, 1><<<g, 256, 0, s>>>(a);
  }
  return avc_check_launch("avc_lstm_bwd");
}
