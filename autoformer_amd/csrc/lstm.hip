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
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <mutex>

#include "common.h"

namespace {

// =============================================================== small H: persistent
// (the encoder BiLSTM, H = 44; no inter-workgroup sync -- design at lstm_small_fwd below)

__device__ __forceinline__ float fsig(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float ftanh(float x) { return 2.f * fsig(2.f * x) - 1.f; }
// FAST (bf16 compute mode): v_exp_f32 / v_rcp_f32 forms; otherwise the IEEE library forms, so
// the fp32 parity mode keeps the reference's activation arithmetic
template <bool FAST>
__device__ __forceinline__ float act_sig(float x) { return FAST ? fsig(x) : sigmoidf_(x); }
template <bool FAST>
__device__ __forceinline__ float act_tanh(float x) { return FAST ? ftanh(x) : tanhf(x); }

// broadcast lane N of each lane quad (DPP quad_perm, no LDS traffic)
template <int N>
__device__ __forceinline__ float quad_bcast(float v) {
  constexpr int ctl = N | (N << 2) | (N << 4) | (N << 6);
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), ctl, 0xf, 0xf, false));
}
// sum over the lane quad (xor 1, then xor 2, as quad_perm)
__device__ __forceinline__ float quad_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xf, 0xf, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xf, 0xf, false));
  return v;
}

// One workgroup = one (utterance, direction) for all T steps: 4 COMPUTE waves + 1 FLUSH wave.
// Compute lane (j, q) = (tid >> 2, tid & 3) owns gate q of hidden unit j.  Per step it
//  * takes its step inputs from a register ring it keeps SD steps ahead with its own global loads
//    (one x-projection element forward; dh, c, c_prev and the unit's four gates backward) -- the
//    loads are unconditional (clamped addresses), so the compiler's vmcnt bookkeeping waits only
//    for the slot being consumed, never for the loads still in flight;
//  * issues ALL its LDS reads of h_{s-1} / dG_{s-1} before the first FMA (one LDS latency per
//    step, not one per 4-wide slice) and runs the product as packed fp32 FMAs (v_pk_fma_f32);
//  * combines the quad's gates with DPP and writes its outputs into an LDS chunk buffer.
// The compute waves issue no stores at all: the flush wave writes each finished chunk of SC steps
// to HBM (fp32, plus an optional bf16 twin for the next GEMMs) while the next chunk runs, so no
// compute wave ever waits on a store.  One workgroup barrier per step orders everything.
constexpr int SNT = 320;  // 4 compute waves + 1 flush wave
constexpr int SD = 4;     // input lead, steps
constexpr int SC = 16;    // output chunk, steps

typedef float f32x2 __attribute__((ext_vector_type(2)));

// Diagnostic timeline (TRACE builds only, avc_lstm_trace): lane 0 of the given wave records the
// 100 MHz realtime clock into tr[(block*Tp + s)*8 + j] once the value `dep` exists (the asm's
// input operand orders the stamp after the code that produces it).
__device__ __forceinline__ void sstamp(unsigned long long* tr, int Tp, int s, int j, float dep) {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : "v"(dep));
  if ((threadIdx.x & 63) == 0)
    tr[((long long)(blockIdx.y * gridDim.x + blockIdx.x) * Tp + s) * 8 + j] = t;
}

constexpr int OOB = 0x7FFFFFF0;  // buffer offset past every buffer here: the store is dropped
typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
typedef unsigned u32x4b_t __attribute__((ext_vector_type(4)));

// Raw buffer resource over `bytes` bytes (0 for a null pointer: every store dropped).  The flush
// wave predicates its stores with it (out-of-range offsets are dropped), so its unrolled flush has
// no branches and every store keeps its own registers: no store waits for an earlier one.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t brsrc(const void* p, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, p ? (int)bytes : 0, 0x00020000);
}

// sum_k w[k] * v[k] over HM/4 float4 LDS slices of v; every slice is read before the first FMA
template <int HM>
__device__ __forceinline__ float dot_lds(const float* __restrict__ v, const f32x2 (&w)[HM / 2]) {
  const f32x4* v4 = reinterpret_cast<const f32x4*>(v);
  f32x4 hv[HM / 4];
#pragma unroll
  for (int k = 0; k < HM / 4; ++k) hv[k] = v4[k];
  // four independent accumulation chains, so no packed FMA waits on its predecessor's result
  f32x2 a[4] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};
#pragma unroll
  for (int k = 0; k < HM / 4; ++k) {
    a[(2 * k) & 3] = __builtin_elementwise_fma(f32x2{hv[k][0], hv[k][1]}, w[2 * k], a[(2 * k) & 3]);
    a[(2 * k + 1) & 3] = __builtin_elementwise_fma(f32x2{hv[k][2], hv[k][3]}, w[2 * k + 1], a[(2 * k + 1) & 3]);
  }
  const f32x2 t = (a[0] + a[1]) + (a[2] + a[3]);
  return t[0] + t[1];
}

// dot_lds with the h slices already in registers (the forward issues its deferred LDS writes between the
// reads and the FMAs)
template <int HM>
__device__ __forceinline__ float dot_regs(const f32x4 (&hv)[HM / 4], const f32x2 (&w)[HM / 2]) {
  f32x2 a[4] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};
#pragma unroll
  for (int k = 0; k < HM / 4; ++k) {
    a[(2 * k) & 3] = __builtin_elementwise_fma(f32x2{hv[k][0], hv[k][1]}, w[2 * k], a[(2 * k) & 3]);
    a[(2 * k + 1) & 3] = __builtin_elementwise_fma(f32x2{hv[k][2], hv[k][3]}, w[2 * k + 1], a[(2 * k + 1) & 3]);
  }
  const f32x2 t = (a[0] + a[1]) + (a[2] + a[3]);
  return t[0] + t[1];
}

// Forward.  T is padded to a multiple of SC with ghost steps that are never written out.
template <int HM, bool FAST, bool TRACE>
__global__ void __launch_bounds__(SNT) lstm_small_fwd(const float* __restrict__ xproj, const float* __restrict__ whh,
                                                      int T, int H, int dirs, float* __restrict__ hout,
                                                      bf16* __restrict__ hout16, float* __restrict__ cout,
                                                      float* __restrict__ gout, unsigned long long* tr) {
  constexpr int GM = 4 * HM;
  const int b = blockIdx.x, d = blockIdx.y, tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int G = 4 * H;
  __shared__ __attribute__((aligned(16))) float hs[2][HM];
  __shared__ __attribute__((aligned(16))) float gst[2][SC][GM];  // output chunks
  __shared__ __attribute__((aligned(16))) float hst[2][SC][HM], cst[2][SC][HM];
  const long long ldx = (long long)dirs * G, ldh = (long long)dirs * H;
  const int t0 = d ? T - 1 : 0, dt = d ? -1 : 1;
  const int Tp = (T + SC - 1) / SC * SC;

  const int j = tid >> 2, q = tid & 3, row = q * H + j;
  const bool act = w < 4 && j < H;
  f32x2 wv[HM / 2];
  float c = 0.f, ring[SD];
  // this lane's x-projection element of step sn (clamped: the surplus lanes / steps load a valid
  // element that is never used)
  const float* xl = xproj + (long long)b * T * ldx + d * G + min(row, G - 1);
  auto xload = [&](int sn) { return xl[(long long)(t0 + dt * min(sn, T - 1)) * ldx]; };
  // flush chunk k (steps k*SC .. k*SC+SC-1) from buffer k & 1 (flush wave): fully unrolled,
  // branch-free buffer stores (gates as 16-B chunks)
  const __amdgpu_buffer_rsrc_t gr = brsrc(gout, (long long)gridDim.x * T * ldx * 4);
  const __amdgpu_buffer_rsrc_t hr = brsrc(hout, (long long)gridDim.x * T * ldh * 4);
  const __amdgpu_buffer_rsrc_t cr = brsrc(cout, (long long)gridDim.x * T * ldh * 4);
  const __amdgpu_buffer_rsrc_t h16r = brsrc(hout16, (long long)gridDim.x * T * ldh * 2);
  auto flush = [&](int k) {
    const int kb = k & 1;
#pragma unroll
    for (int it = 0; it < SC * GM / 4 / 64; ++it) {
      const int idx = it * 64 + lane, i = idx / (GM / 4), c4 = idx % (GM / 4), st = k * SC + i;
      const bool ok = 4 * c4 < G && st < T;
      const long long o = ((long long)b * T + t0 + dt * st) * ldx + d * G + 4 * c4;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4b_t, *reinterpret_cast<const f32x4*>(&gst[kb][i][4 * c4])),
                                             gr, ok ? (int)(o * 4) : OOB, 0, 0);
    }
    if (H % 4 == 0) {  // h, c as 16-B chunks, the bf16 h twin as 8-B chunks
#pragma unroll
      for (int it = 0; it < (SC * HM / 4 + 63) / 64; ++it) {
        const int idx = it * 64 + lane, i = min(idx / (HM / 4), SC - 1), u4 = idx % (HM / 4), st = k * SC + i;
        const bool ok = idx < SC * HM / 4 && 4 * u4 < H && st < T;
        const long long o = ((long long)b * T + t0 + dt * st) * ldh + d * H + 4 * u4;
        const f32x4 hv = *reinterpret_cast<const f32x4*>(&hst[kb][i][4 * u4]);
        const f32x4 cv = *reinterpret_cast<const f32x4*>(&cst[kb][i][4 * u4]);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4b_t, hv), hr, ok ? (int)(o * 4) : OOB, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4b_t, cv), cr, ok ? (int)(o * 4) : OOB, 0, 0);
        const bf16x4 h16 = {(bf16)hv[0], (bf16)hv[1], (bf16)hv[2], (bf16)hv[3]};
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, h16), h16r, ok ? (int)(o * 2) : OOB, 0, 0);
      }
    } else {
#pragma unroll
      for (int it = 0; it < SC * HM / 64; ++it) {
        const int idx = it * 64 + lane, i = idx / HM, u = idx % HM, st = k * SC + i;
        const bool ok = u < H && st < T;
        const long long o = ((long long)b * T + t0 + dt * st) * ldh + d * H + u;
        const float hv = hst[kb][i][u], cv = cst[kb][i][u];
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, hv), hr, ok ? (int)(o * 4) : OOB, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, cv), cr, ok ? (int)(o * 4) : OOB, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (bf16)hv), h16r,
                                              ok ? (int)(o * 2) : OOB, 0, 0);
      }
    }
  };
  if (w < 4) {
    const float* W = whh + (long long)d * G * H + (long long)min(row, G - 1) * H;
#pragma unroll
    for (int k = 0; k < HM / 2; ++k)
      wv[k] = f32x2{(act && 2 * k < H) ? W[2 * k] : 0.f, (act && 2 * k + 1 < H) ? W[2 * k + 1] : 0.f};
    if (tid < 2 * HM) hs[tid / HM][tid % HM] = 0.f;
  }
#pragma unroll
  for (int r = 0; r < SD; ++r) ring[r] = xload(r);
  __syncthreads();

  // the chunk-buffer writes of step s (gates, h, c for the flush wave) are issued during step s + 1, after
  // that step's h reads: the barrier's LDS wait then covers the h_{s+1} write alone, and the deferred writes
  // complete under the next step's FMAs.  The flush of chunk k - 1 moves one step later accordingly.
  float pgv = 0.f, phv = 0.f, pcv = 0.f;
  for (int k = 0; k * SC < Tp; ++k) {
#pragma unroll
    for (int i = 0; i < SC; ++i) {
      const int s = k * SC + i;
      if (w == 4 && k > 0 && i == 1) flush(k - 1);
      // the ring advances in every wave (the flush wave's loads are harmless and unused): a ring
      // slot written only inside the role branch would need a copy at the branch join, and that
      // copy waits for the load just issued
      const float xv = ring[i % SD];
      ring[i % SD] = xload(s + SD);
      if (TRACE && w == 0) sstamp(tr, Tp, s, 0, 0.f);
      if (w < 4) {
        f32x4 hv[HM / 4];
        {
          const f32x4* v4 = reinterpret_cast<const f32x4*>(hs[s & 1]);
#pragma unroll
          for (int kk = 0; kk < HM / 4; ++kk) hv[kk] = v4[kk];
        }
        __builtin_amdgcn_sched_barrier(0);
        if (s > 0 && act) {  // step s - 1's chunk entries (buffer / row of that step)
          const int pb = i > 0 ? (k & 1) : ((k - 1) & 1), pi = i > 0 ? i - 1 : SC - 1;
          gst[pb][pi][row] = pgv;
          if (q == 0) hst[pb][pi][j] = phv;
          else if (q == 1) cst[pb][pi][j] = pcv;
        }
        __builtin_amdgcn_sched_barrier(0);
        const float pre = (act ? xv : 0.f) + dot_regs<HM>(hv, wv);
        if (TRACE && w == 0) sstamp(tr, Tp, s, 1, pre);
        float gv;
        if (FAST) {  // tanh(x) = 2 sig(2x) - 1: one exp + rcp for all four gate lanes
          const float sg = fsig((q == 2 ? 2.f : 1.f) * pre);
          gv = q == 2 ? 2.f * sg - 1.f : sg;
        } else {
          gv = q == 2 ? act_tanh<FAST>(pre) : act_sig<FAST>(pre);
        }
        const float ig = quad_bcast<0>(gv), fg = quad_bcast<1>(gv), gg = quad_bcast<2>(gv), og = quad_bcast<3>(gv);
        c = fg * c + ig * gg;
        const float h = og * act_tanh<FAST>(c);
        if (TRACE && w == 0) sstamp(tr, Tp, s, 2, h);
        if (act && q == 0) hs[(s + 1) & 1][j] = h;
        pgv = gv;
        phv = h;
        pcv = c;
      }
      if (TRACE && w < 4) sstamp(tr, Tp, s, w == 0 ? 3 : 4 + w, 0.f);
      __syncthreads();
    }
  }
  if (w < 4 && act) {  // the last step's chunk entries
    gst[(Tp / SC - 1) & 1][SC - 1][row] = pgv;
    if (q == 0) hst[(Tp / SC - 1) & 1][SC - 1][j] = phv;
    else if (q == 1) cst[(Tp / SC - 1) & 1][SC - 1][j] = pcv;
  }
  __syncthreads();
  if (w == 4) flush(Tp / SC - 1);
}

// Backward: compute lane (j, q) holds column j of gate block q (wc[g] = W[q*H + g][j]) and sums
// dG_{s-1}[q*H + g] * wc[g] over g; the quad's four partial sums (DPP xor steps) give dh_rec[j].
// Its ring holds dh, c, c_prev and the four gates of unit j for the next SD steps.
template <int HM, bool FAST, bool TRACE>
__global__ void __launch_bounds__(SNT) lstm_small_bwd(const float* __restrict__ dhout, const float* __restrict__ call,
                                                      const float* __restrict__ gall, const float* __restrict__ whh,
                                                      int T, int H, int dirs, float* __restrict__ dg,
                                                      bf16* __restrict__ dg16, unsigned long long* tr) {
  constexpr int GM = 4 * HM;
  const int b = blockIdx.x, d = blockIdx.y, tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int G = 4 * H;
  __shared__ __attribute__((aligned(16))) float dgs[2][GM];  // dG of a step, block q at q*HM
  __shared__ __attribute__((aligned(16))) float ost[2][SC][GM];  // output chunks (block q at q*H)
  const long long ldg = (long long)dirs * G, ldh = (long long)dirs * H;
  // backward walks opposite to the forward recurrence
  const int t0 = d ? 0 : T - 1, dt = d ? 1 : -1;
  const int fwd_prev = d ? 1 : -1;  // offset of the forward's previous time step
  const int Tp = (T + SC - 1) / SC * SC;

  const int j = tid >> 2, q = tid & 3, jc = min(j, H - 1);
  const bool act = w < 4 && j < H;
  f32x2 wc[HM / 2];
  float dc = 0.f;
  struct In {
    float dh, c, cp, i, f, g, o;
  };
  In ring[SD];
  const float* dhb = dhout + (long long)b * T * ldh + d * H + jc;
  const float* cb = call + (long long)b * T * ldh + d * H + jc;
  const float* gb = gall + (long long)b * T * ldg + d * G + jc;
  auto fetch = [&](int sn) {  // unconditional loads; c_prev past the sequence start is zeroed at use
    const int t = t0 + dt * min(sn, T - 1), tp = min(max(t + fwd_prev, 0), T - 1);
    In v;
    v.dh = dhb[(long long)t * ldh];
    v.c = cb[(long long)t * ldh];
    v.cp = cb[(long long)tp * ldh];
    const float* g = gb + (long long)t * ldg;
    v.i = g[0];
    v.f = g[H];
    v.g = g[2 * H];
    v.o = g[3 * H];
    return v;
  };
  const __amdgpu_buffer_rsrc_t dgr = brsrc(dg, (long long)gridDim.x * T * ldg * 4);
  const __amdgpu_buffer_rsrc_t dg16r = brsrc(dg16, (long long)gridDim.x * T * ldg * 2);
  auto flush = [&](int k) {  // fully unrolled, branch-free buffer stores (see the forward)
    const int kb = k & 1;
#pragma unroll
    for (int it = 0; it < SC * GM / 4 / 64; ++it) {
      const int idx = it * 64 + lane, i = idx / (GM / 4), c4 = idx % (GM / 4), st = k * SC + i;
      const bool ok = 4 * c4 < G && st < T;
      const long long o = ((long long)b * T + t0 + dt * st) * ldg + d * G + 4 * c4;
      const f32x4 v = *reinterpret_cast<const f32x4*>(&ost[kb][i][4 * c4]);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4b_t, v), dgr, ok ? (int)(o * 4) : OOB, 0, 0);
      const bf16x4 v16 = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, v16), dg16r, ok ? (int)(o * 2) : OOB, 0, 0);
    }
  };
  if (w < 4) {
    const float* W = whh + (long long)d * G * H;
#pragma unroll
    for (int k = 0; k < HM / 2; ++k)
      wc[k] = f32x2{(act && 2 * k < H) ? W[(long long)(q * H + 2 * k) * H + j] : 0.f,
                    (act && 2 * k + 1 < H) ? W[(long long)(q * H + 2 * k + 1) * H + j] : 0.f};
    for (int i = tid; i < 2 * GM; i += 256) dgs[i / GM][i % GM] = 0.f;
  }
#pragma unroll
  for (int r = 0; r < SD; ++r) ring[r] = fetch(r);
  __syncthreads();

  for (int k = 0; k * SC < Tp; ++k) {
    if (w == 4 && k > 0) flush(k - 1);
#pragma unroll
    for (int i = 0; i < SC; ++i) {
      const int s = k * SC + i;
      const In in = ring[i % SD];  // advanced in every wave (see the forward)
      ring[i % SD] = fetch(s + SD);
      if (TRACE && (w == 0 || w == 4)) sstamp(tr, Tp, s, w == 0 ? 0 : 4, 0.f);
      if (w < 4) {
        // recurrent part dh_rec[j] = sum_{q', g} dG_{s-1}[q'*H + g] W[q'*H + g][j]: this lane sums
        // gate block q (entries past H meet zero weights), the quad adds the four blocks
        const float p = dot_lds<HM>(dgs[(s + 1) & 1] + q * HM, wc);
        const float dh = (act ? in.dh : 0.f) + quad_sum(p);
        if (TRACE && w == 0) sstamp(tr, Tp, s, 1, dh);
        if (act) {
          const float cp = s == T - 1 ? 0.f : in.cp;  // the forward's c_{-1} = 0
          const float tc = act_tanh<FAST>(in.c);
          const float dcs = dc + dh * in.o * (1.f - tc * tc);
          const float v = q == 0 ? dcs * in.g * in.i * (1.f - in.i)
                        : q == 1 ? dcs * cp * in.f * (1.f - in.f)
                        : q == 2 ? dcs * in.i * (1.f - in.g * in.g)
                                 : dh * tc * in.o * (1.f - in.o);
          dc = dcs * in.f;
          dgs[s & 1][q * HM + j] = v;  // gate blocks HM apart: 16-B aligned slices, zero tails
          ost[k & 1][i][q * H + j] = v;
        }
        if (TRACE && w == 0) sstamp(tr, Tp, s, 2, dc);
      }
      if (TRACE && (w == 0 || w == 4)) sstamp(tr, Tp, s, w == 0 ? 3 : 5, 0.f);
      __syncthreads();
    }
  }
  if (w == 4) flush(Tp / SC - 1);
}

// =============================================================== small H on MFMA (bf16 compute)
// The encoder BiLSTM (H = 44, AutoVC.py:43,54-55) with its recurrent product on the 4x4x4 bf16
// MFMA (v_mfma_f32_4x4x4_16b_bf16: 16 independent 4x4 blocks per instruction, K = 4 each).  One
// workgroup = 4 utterances (the 4 columns of every block) x one direction; lane l of a wave is
// block l >> 2, column l & 3 (tools/probes/mfma4x4_probe.hip verified the lane map on gfx950:
// A row i / B column j / D column j of block b in lane 4b + i / 4b + j / 4b + j, D row i in
// accumulator register i; 12.7 cycles per dependent MFMA, 8.5 independent).
//
// Forward: block b of compute wave w is hidden unit u = 16w + b and its 4 ROWS are that unit's
// gates i, f, g, o (A = W_hh rows, bf16, in VGPRs for the whole sequence); the B operand is
// h_{s-1} of the block's 4 utterances (bf16, LDS, the same 8 bytes for all 16 blocks).  After
// H/4 MFMAs lane (b, j) holds the four pre-activation gates of cell (u, utterance j) in its four
// accumulator registers: the cell update is lane-local (no DPP, no LDS between the product and
// the cell), one cell per lane, 3 waves for H = 44, and each lane stores its own outputs.
// Backward: dh_rec[u] = sum_r dG[r] W[r][u] over the 4H gate rows r.  Block b = (unit quad ug,
// gate block kq) = (b & 3, b >> 2): its 4 rows are units 16w + 4ug + i, its K runs over gate block
// kq's H rows, so the four blocks kq of a unit quad hold partial sums that two lane exchanges
// (xor 32, xor 16) reduce, each lane keeping the sum of register kq: cell (16w + 4ug + kq, j).
//
// Measured against the packed-FMA kernels above (profiles/r6_bilstm_mfma_ab.txt, B=64, T=128):
// forward 0.585 vs 0.457 us per step, backward 0.727 vs 0.504.  The product is no shorter than the
// FMA dot (0.20 us: LDS read + 11 chained MFMAs), and a lane now activates four gates and tanh(c)
// instead of one gate + tanh(c) (cell 0.22 vs 0.085 us): 64 cells per wave is 4x the
// transcendental work per lane of the one-utterance-per-workgroup form.  Off by default
// (avc_lstm_set_small_mfma / AVC_BILSTM_MFMA=1 select it).
typedef short s16x4 __attribute__((ext_vector_type(4)));
constexpr int MU = 4;   // utterances per workgroup (block columns)
constexpr int MSD = 8;  // input lead, steps (register ring)

__device__ __forceinline__ f32x4 mfma4(s16x4 a, s16x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_4x4x4bf16_1k(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ s16x4 bf4(float a, float b, float c, float d) {
  return __builtin_bit_cast(s16x4, bf16x4{(bf16)a, (bf16)b, (bf16)c, (bf16)d});
}

// Forward.  KC = H / 4 K-chunks, NW = ceil(H / 16) waves.
template <int KC, int NW, bool TRACE>
__global__ void __launch_bounds__(NW * 64) lstm_mfma_fwd(const float* __restrict__ xproj, const float* __restrict__ whh,
                                                         int B, int T, int dirs, float* __restrict__ hout,
                                                         bf16* __restrict__ hout16, float* __restrict__ cout,
                                                         float* __restrict__ gout, unsigned long long* tr) {
  constexpr int H = 4 * KC, G = 4 * H;
  const int d = blockIdx.y, tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int b0 = blockIdx.x * MU;
  __shared__ __attribute__((aligned(16))) bf16 hs[2][MU][H];  // h_{s-1}, the B operand
  const long long ldx = (long long)dirs * G, ldh = (long long)dirs * H;
  const int t0 = d ? T - 1 : 0, dt = d ? -1 : 1;
  const int nu = min(MU, B - b0);  // utterances of this workgroup

  const int j = lane & 3, u = 16 * w + (lane >> 2);
  const bool cell = u < H && j < nu;
  const int bi = b0 + min(j, nu - 1), uc = min(u, H - 1);
  s16x4 wa[KC];
  {  // A: row (lane & 3) = gate of block (lane >> 2) = unit u
    const float* W = whh + (long long)d * G * H + (long long)((lane & 3) * H + uc) * H;
#pragma unroll
    for (int c = 0; c < KC; ++c)
      wa[c] = u < H ? bf4(W[4 * c], W[4 * c + 1], W[4 * c + 2], W[4 * c + 3]) : s16x4{0, 0, 0, 0};
  }
  for (int i = tid; i < 2 * MU * H; i += blockDim.x) (&hs[0][0][0])[i] = (bf16)0.f;
  const float* xl = xproj + (long long)bi * T * ldx + d * G + uc;
  auto xload = [&](int sn) {
    const float* p = xl + (long long)(t0 + dt * min(sn, T - 1)) * ldx;
    return f32x4{p[0], p[H], p[2 * H], p[3 * H]};
  };
  f32x4 ring[MSD];
#pragma unroll
  for (int r = 0; r < MSD; ++r) ring[r] = xload(r);
  float c = 0.f;
  __syncthreads();

  for (int s0 = 0; s0 < T; s0 += MSD) {
#pragma unroll
    for (int r = 0; r < MSD; ++r) {
      const int s = s0 + r;
      if (s >= T) break;
      const f32x4 xv = ring[r];
      ring[r] = xload(s + MSD);
      if (TRACE && w == 0) sstamp(tr, T, s, 0, 0.f);
      const bf16* hr = &hs[s & 1][j][0];
      f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0;
#pragma unroll
      for (int k = 0; k < KC; ++k) {
        const s16x4 hb = *reinterpret_cast<const s16x4*>(hr + 4 * k);
        if (k & 1) a1 = mfma4(wa[k], hb, a1);
        else a0 = mfma4(wa[k], hb, a0);
      }
      const f32x4 pre = a0 + a1 + xv;
      if (TRACE && w == 0) sstamp(tr, T, s, 1, pre[0]);
      const float ig = fsig(pre[0]), fg = fsig(pre[1]), gg = ftanh(pre[2]), og = fsig(pre[3]);
      c = fg * c + ig * gg;
      const float h = og * ftanh(c);
      if (cell) {
        hs[(s + 1) & 1][j][u] = (bf16)h;
        const long long t = t0 + dt * s, oh = ((long long)bi * T + t) * ldh + d * H + u;
        float* gp = gout + ((long long)bi * T + t) * ldx + d * G + u;
        gp[0] = ig;
        gp[H] = fg;
        gp[2 * H] = gg;
        gp[3 * H] = og;
        hout[oh] = h;
        cout[oh] = c;
        if (hout16) hout16[oh] = (bf16)h;
      }
      if (TRACE && w == 0) sstamp(tr, T, s, 2, h);
      __syncthreads();
    }
  }
}

// Backward.  Same workgroup shape; see the block comment above for the lane map.
template <int KC, int NW, bool TRACE>
__global__ void __launch_bounds__(NW * 64) lstm_mfma_bwd(const float* __restrict__ dhout, const float* __restrict__ call,
                                                         const float* __restrict__ gall, const float* __restrict__ whh,
                                                         int B, int T, int dirs, float* __restrict__ dg,
                                                         bf16* __restrict__ dg16, unsigned long long* tr) {
  constexpr int H = 4 * KC, G = 4 * H;
  const int d = blockIdx.y, tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int b0 = blockIdx.x * MU;
  __shared__ __attribute__((aligned(16))) bf16 gs[2][MU][G];  // dG_{s-1}, the B operand
  const long long ldg = (long long)dirs * G, ldh = (long long)dirs * H;
  const int t0 = d ? 0 : T - 1, dt = d ? 1 : -1;  // opposite to the forward recurrence
  const int fwd_prev = d ? 1 : -1;                // offset of the forward's previous time step
  const int nu = min(MU, B - b0);

  const int j = lane & 3, kq = lane >> 4, u = 16 * w + ((lane >> 2) & 3) * 4 + kq;
  const bool cell = u < H && j < nu;
  const int bi = b0 + min(j, nu - 1), uc = min(u, H - 1);
  s16x4 wa[KC];
  {  // A: block (lane >> 2) = (unit quad, gate block kq), row (lane & 3): unit 16w + (lane & 15)
    const int ua = 16 * w + (lane & 15);
    const float* W = whh + (long long)d * G * H + (long long)(kq * H) * H + min(ua, H - 1);
#pragma unroll
    for (int c = 0; c < KC; ++c)
      wa[c] = ua < H ? bf4(W[(4 * c) * H], W[(4 * c + 1) * H], W[(4 * c + 2) * H], W[(4 * c + 3) * H])
                     : s16x4{0, 0, 0, 0};
  }
  for (int i = tid; i < 2 * MU * G; i += blockDim.x) (&gs[0][0][0])[i] = (bf16)0.f;
  struct In {
    float dh, c, cp, i, f, g, o;
  };
  const float* dhb = dhout + (long long)bi * T * ldh + d * H + uc;
  const float* cb = call + (long long)bi * T * ldh + d * H + uc;
  const float* gb = gall + (long long)bi * T * ldg + d * G + uc;
  auto fetch = [&](int sn) {  // unconditional loads; c_prev past the sequence start is zeroed at use
    const int t = t0 + dt * min(sn, T - 1), tp = min(max(t + fwd_prev, 0), T - 1);
    In v;
    v.dh = dhb[(long long)t * ldh];
    v.c = cb[(long long)t * ldh];
    v.cp = cb[(long long)tp * ldh];
    const float* g = gb + (long long)t * ldg;
    v.i = g[0];
    v.f = g[H];
    v.g = g[2 * H];
    v.o = g[3 * H];
    return v;
  };
  In ring[MSD];
#pragma unroll
  for (int r = 0; r < MSD; ++r) ring[r] = fetch(r);
  float dc = 0.f;
  const bool hi = kq & 2, lo = kq & 1;
  __syncthreads();

  for (int s0 = 0; s0 < T; s0 += MSD) {
#pragma unroll
    for (int r = 0; r < MSD; ++r) {
      const int s = s0 + r;
      if (s >= T) break;
      const In in = ring[r];
      ring[r] = fetch(s + MSD);
      if (TRACE && w == 0) sstamp(tr, T, s, 0, 0.f);
      const bf16* gr = &gs[s & 1][j][kq * H];
      f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0;
#pragma unroll
      for (int k = 0; k < KC; ++k) {
        const s16x4 gb4 = *reinterpret_cast<const s16x4*>(gr + 4 * k);
        if (k & 1) a1 = mfma4(wa[k], gb4, a1);
        else a0 = mfma4(wa[k], gb4, a0);
      }
      const f32x4 v = a0 + a1;
      // sum the four gate blocks kq (lanes xor 16, xor 32); this lane keeps register kq
      const float k0 = hi ? v[2] : v[0], k1 = hi ? v[3] : v[1];
      const float r0 = __shfl_xor(hi ? v[0] : v[2], 32, 64), r1 = __shfl_xor(hi ? v[1] : v[3], 32, 64);
      const float e0 = k0 + r0, e1 = k1 + r1;
      const float rec = (lo ? e1 : e0) + __shfl_xor(lo ? e0 : e1, 16, 64);
      if (TRACE && w == 0) sstamp(tr, T, s, 1, rec);
      const float dh = in.dh + rec;
      const float cp = s == T - 1 ? 0.f : in.cp;  // the forward's c_{-1} = 0
      const float tc = ftanh(in.c);
      const float dcs = dc + dh * in.o * (1.f - tc * tc);
      const float di = dcs * in.g * in.i * (1.f - in.i), df = dcs * cp * in.f * (1.f - in.f);
      const float dgg = dcs * in.i * (1.f - in.g * in.g), dob = dh * tc * in.o * (1.f - in.o);
      dc = dcs * in.f;
      if (cell) {
        bf16* gn = &gs[(s + 1) & 1][j][u];
        gn[0] = (bf16)di;
        gn[H] = (bf16)df;
        gn[2 * H] = (bf16)dgg;
        gn[3 * H] = (bf16)dob;
        const long long o = ((long long)bi * T + t0 + dt * s) * ldg + d * G + u;
        dg[o] = di;
        dg[o + H] = df;
        dg[o + 2 * H] = dgg;
        dg[o + 3 * H] = dob;
        if (dg16) {
          dg16[o] = (bf16)di;
          dg16[o + H] = (bf16)df;
          dg16[o + 2 * H] = (bf16)dgg;
          dg16[o + 3 * H] = (bf16)dob;
        }
      }
      if (TRACE && w == 0) sstamp(tr, T, s, 2, dc);
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
  if (a.s > 0) {
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

// =============================================================== large H: persistent recurrences
// One launch for all T steps of a dirs == 1 layer (decoder lstm1 H=512, lstm2 H=1024).
// Workgroups form NG groups of H/32 members; group g owns utterance rows [8g, 8g+8), member r
// owns hidden units [32r, 32r+32) and keeps the matching W_hh slice in VGPRs for the whole
// sequence.  Every step each member needs the whole group's previous output (forward h_{t-1}:
// 8 x H bf16; backward dG_{t+1}: 8 x 4H bf16), handed over inside the launch by the
// write-through form of MI355X_MICROARCH.md "Valid forms" (table row 1):
//   producer: its tile is staged in LDS, wave 0 stores it with 16-B sc1 (write-through)
//             buffer stores, waits s_waitcnt vmcnt(0), then lane 0 stores the member's flag
//             = step + 1 (agent-scope relaxed atomic store = an sc1 store);
//   consumer: wave 0 polls the group's flags with sc1 loads until every member reached the
//             step, the workgroup barrier releases the other waves, and every thread loads its
//             16-B chunks with sc1 buffer loads (L1 bypassed; every handed-off byte is stored
//             and loaded sc1, so no acquire fence).
// Compared with 8-byte {tag, 2 x bf16} granules this moves half the bytes per consumer with
// 16-B accesses, and a waiting consumer re-reads only the flag words.  The payload is
// double-buffered by step parity: a member publishes step s+1 only after consuming step s-1
// from every member, so no slot is overwritten while it is read.  Flags are monotone step
// tags zeroed before every launch; every spin is bounded (timeout -> ctl[0] raised, exit).
// Groups are blockIdx % NG: with round-robin dispatch a group shares one XCD -- a speed
// assumption only, correctness holds for any placement.
//
// Scratch (hbuf forward / gbuf backward):
//   u32 ctl[4] (ctl[0] = timeout flag) | u32 flags[NG][64] | pad to 256 B | bf16 payload [2][B][W]
// with W = H (forward) or 4H (backward); only ctl + flags are zeroed per launch.
constexpr int PRG = 8, PJU = 32, PFL = 64;
constexpr unsigned PSPIN = 1u << 22;
constexpr int AUX_SC1 = 16;  // buffer-instruction cache-policy bits: sc1
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) unsigned gu32;

constexpr size_t px_ctl_bytes(int ng) { return 16 + (size_t)ng * PFL * 4; }
constexpr size_t px_payload_off(int ng) { return (px_ctl_bytes(ng) + 255) & ~(size_t)255; }

struct PersistArgs {
  const float* xproj;  // (B, T/seg, 4H): row b*(T/seg) + t/seg is step t's input projection
  const bf16* w;
  float* hout;
  bf16* hout16;  // optional bf16 copy of h
  float* call;
  float* gall;
  unsigned* ctl;              // scratch: ctl[0] timeout flag, flags from word 4
  bf16* pay;                  // payload [2][B][H]
  unsigned long long* trace;  // diagnostics (avc_lstm_trace), null in production
  unsigned* fault;            // process fault word (avc_set_fault_word), bit 0 on a spin timeout; nullable
  unsigned spin;              // spin bound per wait (PSPIN unless avc_lstm_set_spin / AVC_LSTM_SPIN)
  int nap;                    // granule form: s_sleep(1)s between failed sweeps (0)
  int B, T, ng;
  int seg;                    // frames sharing one xproj row: 1, or T/nc for the lstm1 code fold
};

// Diagnostics: avc_lstm_trace(buf) makes the persistent kernels record the 100 MHz REALTIME
// clock at four points of every step of every workgroup into buf[(wg*T + step)*4 + j]:
// j = 0 step start, 1 exchange complete, 2 recurrent product reduced, 3 step published.
// The stamps go to that buffer only; nothing reads them inside the kernel.
unsigned long long* g_trace = nullptr;

__device__ __forceinline__ void stamp(unsigned long long* tr, int T, int s, int j) {
  if (tr && threadIdx.x == 0) tr[((long long)blockIdx.x * T + s) * 4 + j] = __builtin_amdgcn_s_memrealtime();
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* p, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

// Wave 0: poll the NR flag words of the group (one lane each, sc1 loads, s_sleep between
// passes) until every member has published step `tag`.  false = spin timeout: the launch's
// ctl[0] and the process fault word (when registered) get bit 0, so the host sees the
// failure at its next fault check instead of training on the unfinished outputs.
__device__ __forceinline__ bool poll_flags(unsigned* flags, int NR, unsigned tag, unsigned* ctl, unsigned* fault,
                                           unsigned spin) {
  const int lane = threadIdx.x & 63;
  gu32* f = (gu32*)flags;
  unsigned spins = 0;
  if (spin == 0) {  // injected timeout (avc_lstm_set_spin(~0u)): fail without polling
    if (lane == 0) {
      atomicOr(ctl, 1u);
      if (fault) atomicOr(fault, 1u);
    }
    return false;
  }
  while (true) {
    bool ok = true;
    if (lane < NR) ok = __hip_atomic_load(f + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= tag;
    if (__all(ok)) return true;
    if (++spins > spin) {
      if (lane == 0) {
        atomicOr(ctl, 1u);
        if (fault) atomicOr(fault, 1u);
      }
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// Wave 0, after its write-through payload stores: drain them, then raise the member's flag.
__device__ __forceinline__ void raise_flag(unsigned* flags, int r, unsigned tag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if ((threadIdx.x & 63) == 0)
    __hip_atomic_store((gu32*)flags + r, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Every thread: copy the group's `rows` payload rows of W bf16 (parity slot `slot`) into the
// LDS tile (row stride ap), 16-B sc1 loads, NCH chunks per thread, all in flight together.
// Every thread of the NT-thread workgroup: copy the group's `rows` payload rows of W bf16
// (parity slot row0) into the LDS tile (row stride ap), 16-B sc1 loads, NCH chunks per
// thread, all in flight together.
template <int W, int NCH, int NT>
__device__ __forceinline__ void load_group(__amdgpu_buffer_rsrc_t pay, int row0, int rows, bf16* lds, int ap) {
  constexpr int CPR = W / 8;
  const int tid = threadIdx.x;
  u32x4_t v[NCH];
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int ch = tid + NT * i, row = ch / CPR, col = ch - row * CPR;
    v[i] = row < rows ? __builtin_amdgcn_raw_buffer_load_b128(pay, ((row0 + row) * W + col * 8) * 2, 0, AUX_SC1)
                      : u32x4_t{0u, 0u, 0u, 0u};
  }
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int ch = tid + NT * i, row = ch / CPR, col = ch - row * CPR;
    // NCH is rounded up when NT does not divide the tile (H = 768): skip the overhang
    if (NCH * NT == PRG * CPR || row < PRG) *reinterpret_cast<u32x4_t*>(lds + row * ap + col * 8) = v[i];
  }
}

// Granule form (MI355X_MICROARCH.md "Valid forms", R2; cdna_hip_programming.md G16 recipe):
// the payload IS the flag.  Each 8-byte granule {u32 data = 2 bf16, u32 tag = step + 1} is
// written by one sc1 store (two granules per 16-B store, whose 8-B halves land untorn), so
// the producer needs no drain and no flag, and a consumer needs no flag poll before loading:
// every thread re-reads its own 16-B chunks (sc1, L1 bypassed) until both tags match, then
// stages the data in LDS.  Twice the bytes of the bf16 payload, one fabric round trip fewer
// on both sides.  Chunks I0 .. I0+NCH-1 of the thread (chunk = 2 granules = 4 values; a row
// of W values has W/4 chunks).  false = spin timeout (ctl[0] / fault word raised).
template <int W, int NCH, int I0, int NT>
__device__ __forceinline__ bool sweep_group(__amdgpu_buffer_rsrc_t pay, int row0, int rows, bf16* lds, int ap,
                                            unsigned tag, unsigned spin, unsigned* ctl, unsigned* fault,
                                            int nap) {
  constexpr int CPR = W / 4;
  const int tid = threadIdx.x;
  u32x4_t v[NCH];
  bool ok[NCH];
#pragma unroll
  for (int i = 0; i < NCH; ++i) ok[i] = (tid + NT * (I0 + i)) / CPR >= rows;
  if (spin == 0) {  // injected timeout (avc_lstm_set_spin(~0u)): fail without reading
    if ((threadIdx.x & 63) == 0) {
      atomicOr(ctl, 1u);
      if (fault) atomicOr(fault, 1u);
    }
    return false;
  }
  for (unsigned spins = 0;; ++spins) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int ch = tid + NT * (I0 + i), row = ch / CPR, col = ch - row * CPR;
      if (!ok[i]) v[i] = __builtin_amdgcn_raw_buffer_load_b128(pay, ((row0 + row) * (W / 2) + col * 2) * 8, 0, AUX_SC1);
    }
    bool all = true;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      ok[i] = ok[i] || (v[i][1] == tag && v[i][3] == tag);
      all = all && ok[i];
    }
    if (__all(all)) break;
    if (spins >= spin) {
      if ((threadIdx.x & 63) == 0) {
        atomicOr(ctl, 1u);
        if (fault) atomicOr(fault, 1u);
      }
      return false;
    }
    for (int k = 0; k < nap; ++k) __builtin_amdgcn_s_sleep(1);  // back-off between passes
    asm volatile("" ::: "memory");  // the re-reads are real loads, never hoisted
  }
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int ch = tid + NT * (I0 + i), row = ch / CPR, col = ch - row * CPR;
    if (row < rows) {
      typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
      *reinterpret_cast<u32x2_t*>(lds + row * ap + col * 4) = u32x2_t{v[i][0], v[i][2]};
    }
  }
  return true;
}

// One 16-B sc1 store of two granules: values (d0, d1) = 4 bf16 at granule index gi (even).
__device__ __forceinline__ void store_granules(__amdgpu_buffer_rsrc_t pay, long long gi, unsigned d0, unsigned d1,
                                               unsigned tag) {
  __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{d0, tag, d1, tag}, pay, (int)(gi * 8), 0, AUX_SC1);
}

// acc_n += A . W_n over NK K-blocks of 32: A rows (16 per lane group) are read from LDS at
// `a` + 32k, W fragments live in registers; A fragments are read up to eight K-blocks ahead.
template <int NK>
__device__ __forceinline__ void mfma_rows(const bf16* a, const bf16x8 (&wf)[2][NK], f32x4& acc0, f32x4& acc1) {
  // K-blocks per fragment batch: the largest divisor of NK up to 8 (NK = 12 at H = 768)
  constexpr int KG = NK % 8 == 0 ? 8 : NK % 6 == 0 ? 6 : NK % 4 == 0 ? 4 : NK < 8 ? NK : 1;
#pragma unroll
  for (int k0 = 0; k0 < NK; k0 += KG) {
    bf16x8 af[KG];
#pragma unroll
    for (int i = 0; i < KG; ++i) af[i] = *reinterpret_cast<const bf16x8*>(a + 32 * (k0 + i));
#pragma unroll
    for (int i = 0; i < KG; ++i) {
      acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], wf[0][k0 + i], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], wf[1][k0 + i], acc1, 0, 0, 0);
    }
  }
}

// Workgroups of PNT = 512 threads: eight waves, two per SIMD.  Wave w takes gate (w & 3) and
// half (w >> 2) of the K range, so it holds 128 registers of W fragments instead of 256 and
// the SIMD's two waves hide each other's LDS fragment reads under MFMAs (with four waves of
// 256 W registers the compiler had one A-fragment register left and waited on every read).
// Threads 0..255 own the (utterance, unit) cells of the element-wise stages.
constexpr int PNT = 512;

template <int H, bool GR>
__global__ void __launch_bounds__(PNT, 1) lstm_persist_fwd(PersistArgs a) {
  constexpr int G = 4 * H, NKH = H / 64, AP = H + 8, KH = H / 2;
  constexpr int NCH = (PRG * H / 8 + PNT - 1) / PNT;  // 16-B payload chunks per thread per step
  constexpr int NCG = PRG * H / 4 / PNT;              // granule form: 16-B chunks per thread
  static_assert(!GR || NCG * PNT * 4 == PRG * H, "granule chunks must tile the group payload");
  __shared__ __attribute__((aligned(16))) bf16 As[16 * AP];
  __shared__ __attribute__((aligned(16))) bf16 hs16[PRG * PJU];
  __shared__ float gs[2][PRG][4 * PJU + 1];
  __shared__ float outs[6 * PRG * PJU];  // the step's h, c, i, f, g, o per (utterance, unit) cell
  __shared__ int quit;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, gq = w & 3, kh = w >> 2;
  const int g = blockIdx.x % a.ng, r = blockIdx.x / a.ng;
  const int j0 = r * PJU, b0 = g * PRG;
  const int T = a.T, B = a.B, rows = min(PRG, B - b0);
  const __amdgpu_buffer_rsrc_t pay = rsrc_of(a.pay, (long long)2 * B * H * (GR ? 4 : 2));
  unsigned* flags = a.ctl + 4 + g * PFL;

  // W_hh rows of gate gq for units j0 + 16n + (lane & 15), K half kh
  bf16x8 wf[2][NKH];
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    const bf16* row = a.w + (long long)(gq * H + j0 + n * 16 + (lane & 15)) * H + kh * KH + 8 * (lane >> 4);
#pragma unroll
    for (int k = 0; k < NKH; ++k) wf[n][k] = *reinterpret_cast<const bf16x8*>(row + 32 * k);
  }
  for (int i = tid; i < 16 * AP / 2; i += PNT) reinterpret_cast<unsigned*>(As)[i] = 0u;
  if (tid == 0) quit = 0;
  const int pr = (tid >> 5) & (PRG - 1), pu = tid & 31, pb = b0 + pr, pj = j0 + pu;
  const bool pv = tid < PRG * PJU && pb < B;
  float c = 0.f;
  __syncthreads();

  for (int s = 0; s < T; ++s) {
    const int t = s;
    stamp(a.trace, T, s, 0);
    float px[4] = {0.f, 0.f, 0.f, 0.f};
    if (pv) {
      const float* xp = a.xproj + ((long long)pb * (T / a.seg) + t / a.seg) * G + pj;
#pragma unroll
      for (int q = 0; q < 4; ++q) px[q] = xp[q * H];
    }
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    if (s > 0) {
      // ---- the group's h_{t-1} -> LDS A tile (rows past the batch stay zero)
      if constexpr (GR) {
        if (!sweep_group<H, NCG, 0, PNT>(pay, ((s - 1) & 1) * B + b0, rows, As, AP, (unsigned)s, a.spin, a.ctl,
                                         a.fault, a.nap))
          quit = 1;
        __syncthreads();
        if (quit) return;
      } else {
        if (w == 0 && !poll_flags(flags, H / PJU, (unsigned)s, a.ctl, a.fault, a.spin)) quit = 1;
        __syncthreads();
        if (quit) return;  // block-uniform exit after a spin timeout
        load_group<H, NCH, PNT>(pay, ((s - 1) & 1) * B + b0, rows, As, AP);
        __syncthreads();
      }
      stamp(a.trace, T, s, 1);
      mfma_rows<NKH>(As + (lane & 15) * AP + kh * KH + 8 * (lane >> 4), wf, acc0, acc1);
    }
    if (lane < 32) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        gs[kh][4 * (lane >> 4) + e][gq * PJU + (lane & 15)] = acc0[e];
        gs[kh][4 * (lane >> 4) + e][gq * PJU + 16 + (lane & 15)] = acc1[e];
      }
    }
    __syncthreads();
    stamp(a.trace, T, s, 2);
    float h = 0.f, ig = 0.f, fg = 0.f, gg = 0.f, og = 0.f;
    if (pv) {
      ig = fsig(px[0] + gs[0][pr][pu] + gs[1][pr][pu]);
      fg = fsig(px[1] + gs[0][pr][PJU + pu] + gs[1][pr][PJU + pu]);
      gg = ftanh(px[2] + gs[0][pr][2 * PJU + pu] + gs[1][pr][2 * PJU + pu]);
      og = fsig(px[3] + gs[0][pr][3 * PJU + pu] + gs[1][pr][3 * PJU + pu]);
      c = fg * c + ig * gg;
      h = og * ftanh(c);
    }
    // ---- publish h_t (8 x 32 bf16 tile via LDS; wave 0 stores 4 chunks per row, then the
    // flag) while waves 4..7 write the step's outputs, staged in LDS, to HBM: the publishing
    // wave issues nothing but the hand-off, so its drain waits for the payload alone
    if (tid < PRG * PJU) {
      hs16[pr * PJU + pu] = (bf16)h;
      float* o = outs + tid;
      o[0] = h;
      o[PRG * PJU] = c;
      o[2 * PRG * PJU] = ig;
      o[3 * PRG * PJU] = fg;
      o[4 * PRG * PJU] = gg;
      o[5 * PRG * PJU] = og;
    }
    __syncthreads();
    if (w == 0) {
      if (s + 1 < T) {
        if constexpr (GR) {
          // 8 lanes per row, two granules (4 units) each: the stores are the publication
          const int row = lane >> 3, c4 = lane & 7;
          if (row < rows) {
            const unsigned* hv = reinterpret_cast<const unsigned*>(hs16 + row * PJU + c4 * 4);
            store_granules(pay, ((long long)((s & 1) * B + b0 + row) * H + j0 + c4 * 4) / 2, hv[0], hv[1],
                           (unsigned)(s + 1));
          }
        } else {
          if (lane < 4 * rows) {
            const int row = lane >> 2, c8 = lane & 3;
            const u32x4_t v = *reinterpret_cast<const u32x4_t*>(hs16 + row * PJU + c8 * 8);
            __builtin_amdgcn_raw_buffer_store_b128(v, pay, (((s & 1) * B + b0 + row) * H + j0 + c8 * 8) * 2, 0,
                                                   AUX_SC1);
          }
          raise_flag(flags, r, (unsigned)(s + 1));
        }
      }
    } else if (w >= 4) {
      const int cell = tid - PRG * PJU, ob = b0 + (cell >> 5), oj = j0 + (cell & 31);
      if (ob < B) {
        const float* o = outs + cell;
        const long long oh = ((long long)ob * T + t) * H + oj;
        a.hout[oh] = o[0];
        if (a.hout16) a.hout16[oh] = (bf16)o[0];
        a.call[oh] = o[PRG * PJU];
        float* gp = a.gall + ((long long)ob * T + t) * G + oj;
        gp[0] = o[2 * PRG * PJU];
        gp[H] = o[3 * PRG * PJU];
        gp[2 * H] = o[4 * PRG * PJU];
        gp[3 * H] = o[5 * PRG * PJU];
      }
    }
    stamp(a.trace, T, s, 3);
  }
}

// Backward: same groups and members.  The recurrent product dh_rec[b][j] = sum_q
// dG_{t+1}[b][q] W_hh[q][j] runs over all 4H gate rows q, so each member keeps
// W_hh^T[j0..j0+32][0..4H) in registers (wave w = half (w >> 2) of the K-block of gate
// (w & 3), 2 x H/64 bf16x8 fragments) and loads the group's whole dG_{t+1} (8 x 4H bf16) into
// LDS each step.  The eight waves' partial products are summed through LDS; the cell-gradient
// carry dc stays in a register of the thread that owns (b, j) for the whole sequence.
// Outputs: dG (fp32) and its bf16 twin for the input-gradient / weight-gradient GEMMs.
struct PersistBwdArgs {
  const float* dhout;  // (B,T,H)
  const float* call;   // (B,T,H) cell states
  const float* gall;   // (B,T,4H) activated gates i,f,g,o
  const bf16* wt;      // W_hh^T [H][4H]
  float* dg;           // (B,T,4H)
  bf16* dg16;          // (B,T,4H) or null
  float* sc;           // (B, T/seg, 4H) dG summed over each seg-frame segment, or null
  bf16* sc16;          // its bf16 twin, or null
  unsigned* ctl;       // scratch: ctl[0] timeout flag, flags from word 4
  bf16* pay;           // payload [2][B][4H]
  unsigned long long* trace;  // diagnostics (avc_lstm_trace), null in production
  unsigned* fault;            // as PersistArgs
  unsigned spin;
  int nap;
  int B, T, ng;
  int seg;  // frames per sc row (the lstm1 code fold: T/nc)
};

template <int H, bool GR>
__global__ void __launch_bounds__(PNT, 1) lstm_persist_bwd(PersistBwdArgs a) {
  constexpr int G = 4 * H, NKH = H / 64, AP = G + 8, KH = H / 2, NW = PNT / 64;
  constexpr int NCH = (PRG * G / 8 + PNT - 1) / PNT;  // 16-B payload chunks per thread per step
  constexpr int NCG = PRG * G / 4 / PNT;              // granule form: 16-B chunks per thread
  static_assert(!GR || (NCG * PNT * 4 == PRG * G && NCG % 2 == 0), "granule chunks must tile the payload");
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16* As = reinterpret_cast<bf16*>(smem_raw);                          // [PRG + 1][AP], row PRG = zeros
  float* red = reinterpret_cast<float*>(smem_raw + (PRG + 1) * AP * 2);  // [NW][PRG][PJU + 1]
  bf16* ds16 = reinterpret_cast<bf16*>(red + NW * PRG * (PJU + 1));      // [PRG][4 * PJU] publish tile
  float* outs = reinterpret_cast<float*>(ds16 + PRG * 4 * PJU);         // [4][PRG * PJU] dG of the step
  int* quit = reinterpret_cast<int*>(outs + 4 * PRG * PJU);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, gq = w & 3, kh = w >> 2;
  const int g = blockIdx.x % a.ng, r = blockIdx.x / a.ng;
  const int j0 = r * PJU, b0 = g * PRG;
  const int T = a.T, B = a.B, rows = min(PRG, B - b0);
  const __amdgpu_buffer_rsrc_t pay = rsrc_of(a.pay, (long long)2 * B * G * (GR ? 4 : 2));
  unsigned* flags = a.ctl + 4 + g * PFL;

  // W_hh^T fragments: B operand of the product, n = unit j0 + 16n + (lane&15), k = gate row
  bf16x8 wf[2][NKH];
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    const bf16* row = a.wt + (long long)(j0 + n * 16 + (lane & 15)) * G + gq * H + kh * KH + 8 * (lane >> 4);
#pragma unroll
    for (int k = 0; k < NKH; ++k) wf[n][k] = *reinterpret_cast<const bf16x8*>(row + 32 * k);
  }
  for (int i = tid; i < (PRG + 1) * AP / 2; i += PNT) reinterpret_cast<unsigned*>(As)[i] = 0u;
  if (tid == 0) *quit = 0;
  const int pr = (tid >> 5) & (PRG - 1), pu = tid & 31, pb = b0 + pr, pj = j0 + pu;
  const bool pv = tid < PRG * PJU && pb < B;
  // MFMA A rows: 0..7 loaded utterances, 8..15 read the zero row
  const int arow = (lane & 15) < PRG ? (lane & 15) : PRG;
  float dc = 0.f;
  float ssum[4] = {0.f, 0.f, 0.f, 0.f};  // waves 4..7: the cell's dG over the current segment
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
      f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      if constexpr (GR) {
        // two half sweeps keep the in-flight chunk registers at NCG / 2 per thread
        const int row0 = ((s - 1) & 1) * B + b0;
        if (!sweep_group<G, NCG / 2, 0, PNT>(pay, row0, rows, As, AP, (unsigned)s, a.spin, a.ctl, a.fault,
                                             a.nap) ||
            !sweep_group<G, NCG / 2, NCG / 2, PNT>(pay, row0, rows, As, AP, (unsigned)s, a.spin, a.ctl, a.fault,
                                                    a.nap))
          *quit = 1;
        __syncthreads();
        if (*quit) return;
      } else {
        if (w == 0 && !poll_flags(flags, H / PJU, (unsigned)s, a.ctl, a.fault, a.spin)) *quit = 1;
        __syncthreads();
        if (*quit) return;  // block-uniform exit after a spin timeout
        load_group<G, NCH, PNT>(pay, ((s - 1) & 1) * B + b0, rows, As, AP);
        __syncthreads();
      }
      stamp(a.trace, T, s, 1);
      mfma_rows<NKH>(As + arow * AP + gq * H + kh * KH + 8 * (lane >> 4), wf, acc0, acc1);
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
      for (int ww = 0; ww < NW; ++ww) dh += red[(ww * PRG + pr) * (PJU + 1) + pu];
    }
    float v0 = 0.f, v1 = 0.f, v2 = 0.f, v3 = 0.f;
    if (pv) {
      const float tc = ftanh(ct);
      const float dcs = dc + dh * go * (1.f - tc * tc);
      v0 = dcs * gg * gi * (1.f - gi);        // d(pre i)
      v1 = dcs * cp * gf * (1.f - gf);        // d(pre f)
      v2 = dcs * gi * (1.f - gg * gg);        // d(pre g)
      v3 = dh * tc * go * (1.f - go);         // d(pre o)
      dc = dcs * gf;
    }
    // ---- publish dG_t (8 x (4 gates x 32 units) bf16 tile via LDS; wave 0 stores 16 chunks
    // per row, 2 per lane, then the flag) while waves 4..7 write dG to HBM from LDS
    if (tid < PRG * PJU) {
      bf16* dsr = ds16 + pr * (4 * PJU) + pu;
      dsr[0] = (bf16)v0;
      dsr[PJU] = (bf16)v1;
      dsr[2 * PJU] = (bf16)v2;
      dsr[3 * PJU] = (bf16)v3;
      float* o = outs + tid;
      o[0] = v0;
      o[PRG * PJU] = v1;
      o[2 * PRG * PJU] = v2;
      o[3 * PRG * PJU] = v3;
    }
    __syncthreads();
    if (w == 0) {
      if (s + 1 < T) {
        if constexpr (GR) {
          // 32 two-granule chunks (4 values) per row: 8 rows x 4 gates x 8 chunks, 4 per lane
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int ch = lane + 64 * i, row = ch >> 5, q = (ch >> 3) & 3, c4 = ch & 7;
            if (row < rows) {
              const unsigned* dv = reinterpret_cast<const unsigned*>(ds16 + row * (4 * PJU) + q * PJU + c4 * 4);
              store_granules(pay, ((long long)((s & 1) * B + b0 + row) * G + q * H + j0 + c4 * 4) / 2, dv[0], dv[1],
                             (unsigned)(s + 1));
            }
          }
        } else {
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const int ch = lane + 64 * i, row = ch >> 4, q = (ch >> 2) & 3, c8 = ch & 3;
            if (row < rows) {
              const u32x4_t v = *reinterpret_cast<const u32x4_t*>(ds16 + row * (4 * PJU) + q * PJU + c8 * 8);
              __builtin_amdgcn_raw_buffer_store_b128(v, pay,
                                                     (((s & 1) * B + b0 + row) * G + q * H + j0 + c8 * 8) * 2, 0,
                                                     AUX_SC1);
            }
          }
          raise_flag(flags, r, (unsigned)(s + 1));
        }
      }
    } else if (w >= 4) {
      const int cell = tid - PRG * PJU, ob = b0 + (cell >> 5), oj = j0 + (cell & 31);
      if (ob < B) {
        const float* o = outs + cell;
        const long long og = ((long long)ob * T + t) * G + oj;
        if (a.dg) {
#pragma unroll
          for (int q = 0; q < 4; ++q) a.dg[og + q * H] = o[q * PRG * PJU];
        }
        if (a.dg16) {
#pragma unroll
          for (int q = 0; q < 4; ++q) a.dg16[og + q * H] = (bf16)o[q * PRG * PJU];
        }
        if (a.sc) {  // segment sums (frames t .. t + seg - 1, taken in reverse) for the code fold
#pragma unroll
          for (int q = 0; q < 4; ++q) ssum[q] += o[q * PRG * PJU];
          if (t % a.seg == 0) {
            const long long os = ((long long)ob * (T / a.seg) + t / a.seg) * G + oj;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              a.sc[os + q * H] = ssum[q];
              if (a.sc16) a.sc16[os + q * H] = (bf16)ssum[q];
              ssum[q] = 0.f;
            }
          }
        }
      }
    }
    stamp(a.trace, T, s, 3);
  }
}

// =============================================================== two stacked layers, one launch
// Decoder lstm2 (nn.LSTM(512 -> 1024, num_layers=2), AutoVC.py:96,110) forward as a layer
// WAVEFRONT: tick k runs layer 0 at step k and layer 1 at step k - 1, so both layers share one
// hand-off per tick -- T + 1 hand-offs instead of 2T -- and layer 1's input projection
// h0_t W_ih1^T happens inside the recurrence (no separate 8192 x 4096 x 1024 GEMM).
// Register budget forces the shape: three H x 4H bf16 matrices (W_hh0, W_ih1, W_hh1) live in
// VGPRs, replicated once per utterance group, so groups are 16 utterances (a full MFMA tile, no
// padding rows: ceil(B/16) groups x H/16 members = 256 workgroups at B = 64, H = 1024) and a
// member owns 16 hidden units of EACH layer: 3 x 64 gate columns x H = 192 VGPRs per thread.
// Per tick every member needs the group's h0_{k-1} and h1_{k-2} (16 x H bf16 each) in LDS;
// wave w = (gate pair w & 1, K quarter w >> 1) multiplies each A fragment it reads against six
// weight fragments (P0 = h0 W_hh0^T, P1 = h0 W_ih1^T + h1 W_hh1^T for its two gates), so every
// A element is read from LDS once per tick; the four K quarters meet in LDS.  Thread tid is
// the cell (layer tid >> 8, utterance (tid >> 4) & 15, unit tid & 15).  Hand-off: the
// write-through flag form above, one flag per member per tick covering both layers' tiles.
struct Persist2Args {
  const float* xproj;  // (B,T,4H) layer-0 input projection incl. b_ih0 + b_hh0
  const bf16* w0;      // W_hh0 [4H][H]
  const bf16* wi1;     // W_ih1 [4H][H]
  const bf16* w1;      // W_hh1 [4H][H]
  const float* bias1;  // b_ih1 + b_hh1 (4H)
  float* hout[2];
  bf16* hout16[2];
  float* call[2];
  float* gall[2];
  unsigned* ctl;
  bf16* pay;  // [layer][2 parities][B][H]
  unsigned long long* trace;
  unsigned* fault;
  unsigned spin;
  int B, T, ng;
};

constexpr int QRG = 16, QJU = 16;  // utterances per group, units per member and layer
constexpr int NLW = 4;             // W_hh1 fragments per wave kept in LDS instead of VGPRs

template <int H>
constexpr size_t persist2_lds() {
  return (size_t)2 * QRG * (H + 8) * 2 + (size_t)4 * 2 * 4 * QRG * QJU * 4 + (size_t)2 * QRG * QJU * 2 +
         (size_t)8 * NLW * 64 * 16 + (size_t)6 * 512 * 4 + 16;
}

// Waves 1..7: the staged outputs of tick kp (all 512 cells) to HBM.  (16-B value-major stores
// of the same bytes measured slower per tick: 5.18 vs 4.99 us.)
template <int H>
__device__ __forceinline__ void lstm2_store_outputs(const Persist2Args& a, const float* outs, int kp, int b0, int j0) {
  constexpr int G = 4 * H;
  for (int cell = threadIdx.x - 64; cell < 2 * QRG * QJU; cell += PNT - 64) {
    const int L = cell >> 8, cb = b0 + ((cell >> 4) & 15), cj = j0 + (cell & 15);
    const int t = L == 0 ? kp : kp - 1;
    if (!(L == 0 ? kp < a.T : kp >= 1) || cb >= a.B) continue;
    const float* o = outs + cell;
    const long long oh = ((long long)cb * a.T + t) * H + cj;
    a.hout[L][oh] = o[0];
    a.hout16[L][oh] = (bf16)o[0];
    a.call[L][oh] = o[PNT];
    float* gpo = a.gall[L] + ((long long)cb * a.T + t) * G + cj;
    gpo[0] = o[2 * PNT];
    gpo[H] = o[3 * PNT];
    gpo[2 * H] = o[4 * PNT];
    gpo[3 * H] = o[5 * PNT];
  }
}

template <int H, int SB, int LB, bool OS>
__global__ void __launch_bounds__(PNT, 1) lstm2_persist_fwd(Persist2Args a) {
  constexpr int G = 4 * H, AP = H + 8, NR = H / QJU, NKQ = H / 128;  // k-blocks per K quarter
  constexpr int NCH = 2 * QRG * H / 8 / PNT;                          // 16-B chunks per thread
  static_assert(NCH * PNT * 8 == 2 * QRG * H && NR <= 64, "two-layer tiling");
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16* As = reinterpret_cast<bf16*>(smem_raw);                          // [2 layers][16][AP]
  float* red = reinterpret_cast<float*>(smem_raw + 2 * QRG * AP * 2);    // [kq][L][q][16][16]
  bf16* hs16 = reinterpret_cast<bf16*>(red + 4 * 2 * 4 * QRG * QJU);     // [L][16][16] publish tile
  // the tick's outputs (h, c, i, f, g, o per cell), stored to HBM by waves 1..7 during the NEXT
  // tick (after its products), so they never queue in front of wave 0's hand-off
  float* outs = reinterpret_cast<float*>(reinterpret_cast<char*>(hs16 + 2 * QRG * QJU) + (size_t)8 * NLW * 64 * 16);
  int* quit = reinterpret_cast<int*>(outs + 6 * PNT);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, gp = w & 1, kq = w >> 1;
  const int g = blockIdx.x % a.ng, r = blockIdx.x / a.ng;
  const int j0 = r * QJU, b0 = g * QRG;
  const int T = a.T, B = a.B, rows = min(QRG, B - b0);
  const __amdgpu_buffer_rsrc_t pay = rsrc_of(a.pay, (long long)4 * B * H * 2);
  unsigned* flags = a.ctl + 4 + g * PFL;

  // weight fragments (B operand): gate q = 2gp + i, unit j0 + (lane & 15), k-block kq*NKQ + k.
  // The last NLW W_hh1 fragments of gate 2gp+1 live in LDS (wl, per wave and lane): with all 48
  // in VGPRs the compiler spilled two to scratch and waited on their reload every tick.
  bf16x8 f0[2][NKQ], fi[2][NKQ], f1a[NKQ], f1b[NKQ - NLW];  // W_hh1: gate 2gp (a), 2gp + 1 (b)
  bf16x8* wl = reinterpret_cast<bf16x8*>(hs16 + 2 * QRG * QJU) + (w * NLW) * 64 + lane;  // [w][NLW][64]
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const long long ro = (long long)((2 * gp + i) * H + j0 + (lane & 15)) * H + kq * NKQ * 32 + 8 * (lane >> 4);
#pragma unroll
    for (int k = 0; k < NKQ; ++k) {
      f0[i][k] = *reinterpret_cast<const bf16x8*>(a.w0 + ro + 32 * k);
      fi[i][k] = *reinterpret_cast<const bf16x8*>(a.wi1 + ro + 32 * k);
      const bf16x8 v1 = *reinterpret_cast<const bf16x8*>(a.w1 + ro + 32 * k);
      if (i == 0) f1a[k] = v1;
      else if (k < NKQ - NLW) f1b[k < NKQ - NLW ? k : 0] = v1;
      else wl[(k - (NKQ - NLW)) * 64] = v1;
    }
  }
  for (int i = tid; i < 2 * QRG * AP / 2; i += PNT) reinterpret_cast<unsigned*>(As)[i] = 0u;
  if (tid == 0) *quit = 0;
  // cell of this thread
  const int L = tid >> 8, cr = (tid >> 4) & 15, cu = tid & 15, cb = b0 + cr, cj = j0 + cu;
  const bool cv = cb < B;
  float c = 0.f;
  __syncthreads();

  for (int k = 0; k <= T; ++k) {
    const int t = L == 0 ? k : k - 1;  // this thread's step
    const bool act = L == 0 ? k < T : k >= 1;
    if (k < T) stamp(a.trace, T, k, 0);
    // gate inputs besides the recurrent products: layer 0 the x projection of its step (loaded
    // ahead of the exchange), layer 1 its bias (L1-resident re-loads)
    float px[4] = {0.f, 0.f, 0.f, 0.f};
    if (act && cv) {
      const float* xp = L == 0 ? a.xproj + ((long long)cb * T + t) * G + cj : a.bias1 + cj;
#pragma unroll
      for (int q = 0; q < 4; ++q) px[q] = xp[q * H];
    }
    f32x4 p0[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    f32x4 p1[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    if (k > 0) {
      if (w == 0 && !poll_flags(flags, NR, (unsigned)k, a.ctl, a.fault, a.spin)) *quit = 1;
      __syncthreads();
      if (*quit) return;  // block-uniform exit after a spin timeout
      // h0_{k-1} -> As[0], h1_{k-2} -> As[1] (k >= 2); rows past the batch stay zero
      // (NCH / LB chunks in flight per batch: the weight fragments leave few registers)
      const int slot = (k - 1) & 1;
#pragma unroll
      for (int hf = 0; hf < LB; ++hf) {
        u32x4_t v[NCH / LB];
#pragma unroll
        for (int i = 0; i < NCH / LB; ++i) {
          const int ch = tid + PNT * (hf * NCH / LB + i), l = ch / (QRG * H / 8), rem = ch - l * (QRG * H / 8),
                    row = rem / (H / 8), col = rem - row * (H / 8);
          v[i] = row < rows && (l == 0 || k >= 2)
                     ? __builtin_amdgcn_raw_buffer_load_b128(pay, (((l * 2 + slot) * B + b0 + row) * H + col * 8) * 2,
                                                             0, AUX_SC1)
                     : u32x4_t{0u, 0u, 0u, 0u};
        }
        // OS: the previous tick's outputs leave while this tick's payload loads are in flight
        if (OS && hf == 0 && w > 0) lstm2_store_outputs<H>(a, outs, k - 1, b0, j0);
#pragma unroll
        for (int i = 0; i < NCH / LB; ++i) {
          const int ch = tid + PNT * (hf * NCH / LB + i), l = ch / (QRG * H / 8), rem = ch - l * (QRG * H / 8),
                    row = rem / (H / 8), col = rem - row * (H / 8);
          *reinterpret_cast<u32x4_t*>(As + (l * QRG + row) * AP + col * 8) = v[i];
        }
      }
      __syncthreads();
      if (k < T) stamp(a.trace, T, k, 1);
      const bf16* a0p = As + (lane & 15) * AP + kq * NKQ * 32 + 8 * (lane >> 4);
      const bf16* a1p = a0p + QRG * AP;
#pragma unroll
      for (int kk = 0; kk < NKQ; ++kk) {
        const bf16x8 x0 = *reinterpret_cast<const bf16x8*>(a0p + 32 * kk);
        const bf16x8 x1 = *reinterpret_cast<const bf16x8*>(a1p + 32 * kk);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          p0[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, f0[i][kk], p0[i], 0, 0, 0);
          p1[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, fi[i][kk], p1[i], 0, 0, 0);
          const bf16x8 wb = i == 0                ? f1a[kk]
                            : kk < NKQ - NLW      ? f1b[kk < NKQ - NLW ? kk : 0]
                                                  : wl[(kk - (NKQ - NLW)) * 64];
          p1[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1, wb, p1[i], 0, 0, 0);
        }
        // SB > 0: at most SB k-blocks of A fragments in flight (the weights hold 184 VGPRs)
        if (SB > 0 && kk % SB == SB - 1) __builtin_amdgcn_sched_barrier(0);
      }
    }
    // K-quarter partials -> LDS: red[((kq * 2 + L) * 4 + q) * 256 + row * 16 + unit]
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float* d0 = red + ((kq * 2 + 0) * 4 + 2 * gp + i) * (QRG * QJU) + (lane & 15);
      float* d1 = red + ((kq * 2 + 1) * 4 + 2 * gp + i) * (QRG * QJU) + (lane & 15);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        d0[(4 * (lane >> 4) + e) * QJU] = p0[i][e];
        d1[(4 * (lane >> 4) + e) * QJU] = p1[i][e];
      }
    }
    if (!OS && k > 0 && w > 0) lstm2_store_outputs<H>(a, outs, k - 1, b0, j0);
    __syncthreads();
    if (k < T) stamp(a.trace, T, k, 2);
    float pre[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float s = px[q];
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) s += red[((kk * 2 + L) * 4 + q) * (QRG * QJU) + cr * QJU + cu];
      pre[q] = s;
    }
    const float ig = fsig(pre[0]), fg = fsig(pre[1]), gg = ftanh(pre[2]), og = fsig(pre[3]);
    float h = 0.f;
    if (act) {
      c = fg * c + ig * gg;
      h = og * ftanh(c);
    }
    hs16[(L * QRG + cr) * QJU + cu] = (bf16)h;
    outs[tid] = h;
    outs[PNT + tid] = c;
    outs[2 * PNT + tid] = ig;
    outs[3 * PNT + tid] = fg;
    outs[4 * PNT + tid] = gg;
    outs[5 * PNT + tid] = og;
    __syncthreads();
    // ---- publish h0_k and h1_{k-1} (wave 0: lanes 0..31 layer 0, 32..63 layer 1; 16 B each),
    // needed by tick k + 1 (none after tick T - 1); the other waves store their outputs meanwhile
    if (w == 0 && k < T) {
      const int l = lane >> 5, row = (lane >> 1) & 15, half = lane & 1;
      if (row < rows) {
        const u32x4_t v = *reinterpret_cast<const u32x4_t*>(hs16 + (l * QRG + row) * QJU + half * 8);
        __builtin_amdgcn_raw_buffer_store_b128(v, pay, (((l * 2 + (k & 1)) * B + b0 + row) * H + j0 + half * 8) * 2, 0,
                                               AUX_SC1);
      }
      raise_flag(flags, r, (unsigned)(k + 1));
    }
    if (k < T) stamp(a.trace, T, k, 3);
  }
  if (w > 0) lstm2_store_outputs<H>(a, outs, T, b0, j0);  // the last tick's (staged above its barrier)
}

// =============================================================== two stacked layers, backward
// Decoder lstm2 backward as a layer WAVEFRONT (the forward's mirror): tick k runs layer 1 at step
// T-1-k and layer 0 at step T-k, so one hand-off per tick serves both layers, and layer 1's input
// gradient dX1 = dG1 W_ih1 -- layer 0's upstream gradient -- is formed inside the recurrence (no
// 8192 x 1024 x 4096 GEMM between two single-layer launches).  Tick k hands over dG1 and dG0 of
// tick k-1 (2 x 16 x 4H bf16 = 256 KB per consumer); member r owns units j0..j0+15 of EACH layer:
//   dh1_t  = dG1_{t+1} W_hh1[:, j] + dL/dh1_t (upstream)
//   dh0_t' = dG0_{t'+1} W_hh0[:, j] + dG1_{t'} W_ih1[:, j]       (t' = t + 1: dG1_{t'} = the same payload)
// so each member keeps three 4H x 16 slices (W_hh1^T, W_ih1^T, W_hh0^T rows j0..) as MFMA B fragments:
// 40 in VGPRs and 8 per wave in LDS.  The payload does not fit the LDS as one A tile: it is staged
// in four 64 KB K-chunks (both layers' 16 rows x 1024 gate rows), the loads of chunk c + 1 in flight
// under chunk c's products; wave w takes k-blocks 4w .. 4w+3 of every chunk, and the eight waves'
// partial 16 x 16 products meet in LDS.  Thread tid is the cell (layer tid >> 8, utterance
// (tid >> 4) & 15, unit tid & 15); dc stays in its register.  Hand-off: the forward's write-through
// flag form, one flag per member per tick for both layers' tiles.
struct Persist2BwdArgs {
  const float* dhout1;  // (B,T,H) dL/dh of the top layer's output
  const float* call[2];  // (B,T,H) cell states of layer 0 / 1
  const float* gall[2];  // (B,T,4H) activated gates
  const bf16* wt0;       // W_hh0^T [H][4H]
  const bf16* wti1;      // W_ih1^T [H][4H]
  const bf16* wt1;       // W_hh1^T [H][4H]
  float* dg[2];          // (B,T,4H) dL/d(pre-activation gates); nullable (bf16 twin only)
  bf16* dg16[2];
  float* dbp;            // [layer][group][4H] per-group bias-gradient partials (sum of dG over the group's
                         // utterances and steps); nullable
  unsigned* ctl;
  bf16* pay;  // [layer][2 parities][B][4H]
  unsigned long long* trace;
  unsigned* fault;
  unsigned spin;
  int B, T, ng;
  int opt;  // bits: 1 = dG stores after a barrier behind the flag (the launch sets 1), 2 = no bf16 twin
};

constexpr int BKC = 1024, BNC = 4, BCP = BKC + 8, BNLW = 3;  // K-chunk, chunks, LDS pitch, W_hh0 frags in LDS

// two chunk tiles (LDS-DMA double buffer; the wave partials and the publish tile reuse the first after
// the last chunk), then the LDS-resident weight fragments
template <int H>
constexpr size_t persist2_bwd_lds() {
  return (size_t)2 * 2 * QRG * BCP * 2 + (size_t)8 * BNLW * 64 * 16 + 16;
}

__device__ __attribute__((aligned(16))) unsigned g_zero16_l2[4] = {0u, 0u, 0u, 0u};
typedef __attribute__((address_space(3))) void* l2_lds_ptr;
typedef const __attribute__((address_space(1))) void* l2_gbl_ptr;
// 16-B LDS fragment read as inline asm: the compiler's waitcnt pass would otherwise wait for every
// LDS-DMA in flight (the next chunk's) before it
__device__ __forceinline__ bf16x8 l2_ds_read16(unsigned addr) {
  u32x4_t v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr) : "memory");
  return __builtin_bit_cast(bf16x8, v);
}

template <int H>
__global__ void __launch_bounds__(PNT, 1) lstm2_persist_bwd(Persist2BwdArgs a) {
  constexpr int G = 4 * H, NR = H / QJU, KPW = BKC / 32 / 8, NF0 = BNC * KPW - BNLW;
  constexpr int CB = 2 * QRG * BCP * 2;  // bytes of one chunk tile
  static_assert(G == BNC * BKC && 2 * QRG * 2 == 8 * 8 && NR <= 64 && NF0 > 0, "wavefront tiling");
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  float* red = reinterpret_cast<float*>(smem_raw);                     // [w][L][16][16] (in tile 0)
  bf16* ds16 = reinterpret_cast<bf16*>(red + 8 * 2 * QRG * QJU);       // [L][16][4 gates x 16] (in tile 0)
  bf16x8* wlb = reinterpret_cast<bf16x8*>(smem_raw + 2 * CB);          // [w][BNLW][64]
  int* quit = reinterpret_cast<int*>(wlb + 8 * BNLW * 64);
  static_assert((8 * 2 * QRG * QJU * 4 + 2 * QRG * 4 * QJU * 2) <= CB, "partials fit a chunk tile");
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = blockIdx.x % a.ng, r = blockIdx.x / a.ng;
  const int j0 = r * QJU, b0 = g * QRG;
  const int T = a.T, B = a.B, rows = min(QRG, B - b0);
  const __amdgpu_buffer_rsrc_t pay = rsrc_of(a.pay, (long long)4 * B * G * 2);
  unsigned* flags = a.ctl + 4 + g * PFL;

  // B fragments: column n = unit j0 + (lane & 15), k = gate row c*BKC + (w*KPW + i)*32 + 8*(lane >> 4)
  bf16x8 f1[BNC][KPW], fi[BNC][KPW], f0[NF0];
  bf16x8* wl = wlb + (w * BNLW) * 64 + lane;
  {
    const long long ro = (long long)(j0 + (lane & 15)) * G + 8 * (lane >> 4);
#pragma unroll
    for (int c = 0; c < BNC; ++c)
#pragma unroll
      for (int i = 0; i < KPW; ++i) {
        const long long o = ro + c * BKC + (w * KPW + i) * 32;
        f1[c][i] = *reinterpret_cast<const bf16x8*>(a.wt1 + o);
        fi[c][i] = *reinterpret_cast<const bf16x8*>(a.wti1 + o);
        const bf16x8 v0 = *reinterpret_cast<const bf16x8*>(a.wt0 + o);
        const int idx = c * KPW + i;
        if (idx < NF0) f0[idx < NF0 ? idx : 0] = v0;
        else wl[(idx - NF0) * 64] = v0;
      }
  }
  // this wave's 8 LDS-DMA fills per chunk: q = 8w + i -> layer q >> 5, row (q >> 1) & 15, half q & 1
  // (1 KiB = 512 gate rows): wave-uniform bases + the lane's 16-B offset; rows past the batch read
  // the zero granule
  const long long slot_el = (long long)B * G;  // parity slot stride (elements)
  auto issue = [&](int c, int slot) {
    char* tile = smem_raw + (c & 1) * CB;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int q = 8 * w + i, l = q >> 5, row = (q >> 1) & 15, half = q & 1;
      const bf16* src = row < rows ? a.pay + ((long long)(l * 2 + slot) * B + b0 + row) * G + c * BKC + half * 512 +
                                         lane * 8
                                   : reinterpret_cast<const bf16*>(g_zero16_l2);
      __builtin_amdgcn_global_load_lds((l2_gbl_ptr)src, (l2_lds_ptr)(tile + ((l * QRG + row) * BCP + half * 512) * 2),
                                       16, 0, AUX_SC1);
    }
  };
  if (tid == 0) *quit = 0;
  const int L = tid >> 8, cr = (tid >> 4) & 15, cu = tid & 15, cb = b0 + cr, cj = j0 + cu;
  const bool cv = cb < B;
  const unsigned aoff = (unsigned)(((lane & 15) * BCP + w * KPW * 32 + 8 * (lane >> 4)) * 2);
  float dc = 0.f;
  float sb0 = 0.f, sb1 = 0.f, sb2 = 0.f, sb3 = 0.f;  // this cell's dG summed over its steps (dbp)
  __syncthreads();

  for (int k = 0; k <= T; ++k) {
    const int t = L == 1 ? T - 1 - k : T - k;  // this thread's step
    const bool act = (L == 1 ? k < T : k >= 1) && cv;
    if (k < T) stamp(a.trace, T, k, 0);
    // per-cell inputs of this step (independent of the exchange: issued first)
    float dhu = 0.f, ct = 0.f, cp = 0.f, gi = 0.f, gf = 0.f, gg = 0.f, go = 0.f;
    if (act) {
      const long long oh = ((long long)cb * T + t) * H + cj;
      if (L == 1) dhu = a.dhout1[oh];
      ct = a.call[L][oh];
      cp = t > 0 ? a.call[L][oh - H] : 0.f;
      const float* gp = a.gall[L] + ((long long)cb * T + t) * G + cj;
      gi = gp[0];
      gf = gp[H];
      gg = gp[2 * H];
      go = gp[3 * H];
    }
    f32x4 p1 = {0.f, 0.f, 0.f, 0.f}, p0 = {0.f, 0.f, 0.f, 0.f};
    if (k > 0) {
      if (w == 0 && !poll_flags(flags, NR, (unsigned)k, a.ctl, a.fault, a.spin)) *quit = 1;
      __syncthreads();
      if (*quit) return;  // block-uniform exit after a spin timeout
      if (k < T) stamp(a.trace, T, k, 1);
      const int slot = (k - 1) & 1;
      issue(0, slot);
      issue(1, slot);
#pragma unroll
      for (int c = 0; c < BNC; ++c) {
        // this wave's fills of chunk c have landed (the next chunk's 8 may be in flight), then
        // every wave's
        if (c < BNC - 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_barrier" ::: "memory");
        const unsigned base = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)(smem_raw + (c & 1) * CB) + aoff;
        // XB k-blocks of A fragments at a time (the weight fragments hold ~180 VGPRs)
        constexpr int XB = 1;
#pragma unroll
        for (int i2 = 0; i2 < KPW; i2 += XB) {
          bf16x8 x0[XB], x1[XB];
#pragma unroll
          for (int i = 0; i < XB; ++i) {
            x0[i] = l2_ds_read16(base + 64 * (i2 + i));
            x1[i] = l2_ds_read16(base + QRG * BCP * 2 + 64 * (i2 + i));
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int i = 0; i < XB; ++i) {
            const int idx = c * KPW + i2 + i;
            const bf16x8 wb = idx < NF0 ? f0[idx < NF0 ? idx : 0] : wl[(idx >= NF0 ? idx - NF0 : 0) * 64];
            p1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1[i], f1[c][i2 + i], p1, 0, 0, 0);
            p0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1[i], fi[c][i2 + i], p0, 0, 0, 0);
            p0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0[i], wb, p0, 0, 0, 0);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        asm volatile("s_barrier" ::: "memory");  // every wave is done reading this tile
        if (c + 2 < BNC) issue(c + 2, slot);
      }
    }
    // wave partials -> LDS: red[((w * 2 + L) * 16 + row) * 16 + unit]
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      red[((w * 2 + 0) * QRG + 4 * (lane >> 4) + e) * QJU + (lane & 15)] = p0[e];
      red[((w * 2 + 1) * QRG + 4 * (lane >> 4) + e) * QJU + (lane & 15)] = p1[e];
    }
    __syncthreads();
    if (k < T) stamp(a.trace, T, k, 2);
    float dh = dhu;
#pragma unroll
    for (int ww = 0; ww < 8; ++ww) dh += red[((ww * 2 + L) * QRG + cr) * QJU + cu];
    float v0 = 0.f, v1 = 0.f, v2 = 0.f, v3 = 0.f;
    if (act) {
      const float tc = ftanh(ct);
      const float dcs = dc + dh * go * (1.f - tc * tc);
      v0 = dcs * gg * gi * (1.f - gi);  // d(pre i)
      v1 = dcs * cp * gf * (1.f - gf);  // d(pre f)
      v2 = dcs * gi * (1.f - gg * gg);  // d(pre g)
      v3 = dh * tc * go * (1.f - go);   // d(pre o)
      dc = dcs * gf;
      sb0 += v0;
      sb1 += v1;
      sb2 += v2;
      sb3 += v3;
    }
    bf16* dsr = ds16 + (L * QRG + cr) * (4 * QJU) + cu;
    dsr[0] = (bf16)v0;
    dsr[QJU] = (bf16)v1;
    dsr[2 * QJU] = (bf16)v2;
    dsr[3 * QJU] = (bf16)v3;
    __syncthreads();
    // ---- publish dG1_{t1} and dG0_{t0} (needed by tick k + 1; none after tick T - 1): wave 0, four
    // 16-B chunks per lane (2 layers x 16 rows x 8 chunks), then the flag
    if (w == 0 && k < T) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ch = lane + 64 * i, l = ch >> 7, row = (ch >> 3) & 15, q8 = ch & 7;
        if (row < rows) {
          const u32x4_t pv = *reinterpret_cast<const u32x4_t*>(ds16 + (l * QRG + row) * (4 * QJU) + q8 * 8);
          __builtin_amdgcn_raw_buffer_store_b128(
              pv, pay, (((l * 2 + (k & 1)) * B + b0 + row) * G + (q8 >> 1) * H + j0 + (q8 & 1) * 8) * 2, 0, AUX_SC1);
        }
      }
      raise_flag(flags, r, (unsigned)(k + 1));
    }
    if (a.opt & 1) __syncthreads();  // every wave's stores behind wave 0's flag
    if (act) {  // (wave 0 issues these after its flag: they stay off the hand-off's vmcnt wait)
      const long long og = ((long long)cb * T + t) * G + cj;
      if (a.dg[L]) {
        float* d = a.dg[L] + og;
        d[0] = v0;
        d[H] = v1;
        d[2 * H] = v2;
        d[3 * H] = v3;
      }
      if (a.dg16[L] && !(a.opt & 2)) {
        bf16* d16 = a.dg16[L] + og;
        d16[0] = (bf16)v0;
        d16[H] = (bf16)v1;
        d16[2 * H] = (bf16)v2;
        d16[3 * H] = (bf16)v3;
      }
    }
    if (k < T) stamp(a.trace, T, k, 3);
  }
  if (a.dbp) {
    // the bias gradients' share of this member: dG summed over the group's 16 utterances (LDS, in
    // row order) and T steps (registers, in step order), one plain store per (layer, gate, unit) --
    // deterministic, and the fp32 dG (B x T x 4H per layer) need not be stored for a column sum
    float* sb = red;  // [L][q][16 rows][16 units] = 8 KiB of chunk tile 0
    __syncthreads();  // the last tick's reads of red / ds16 are done
    sb[((L * 4 + 0) * QRG + cr) * QJU + cu] = sb0;
    sb[((L * 4 + 1) * QRG + cr) * QJU + cu] = sb1;
    sb[((L * 4 + 2) * QRG + cr) * QJU + cu] = sb2;
    sb[((L * 4 + 3) * QRG + cr) * QJU + cu] = sb3;
    __syncthreads();
    if (tid < 2 * 4 * QJU) {
      const int l = tid >> 6, q = (tid >> 4) & 3, u = tid & 15;
      float sum = 0.f;
#pragma unroll
      for (int rr = 0; rr < QRG; ++rr) sum += sb[((l * 4 + q) * QRG + rr) * QJU + u];
      a.dbp[((long long)l * a.ng + g) * G + q * H + j0 + u] = sum;
    }
  }
}

template <int H>
constexpr size_t persist_bwd_lds() {
  return (size_t)(PRG + 1) * (4 * H + 8) * 2 + (size_t)(PNT / 64) * PRG * (PJU + 1) * 4 + (size_t)PRG * 4 * PJU * 2 +
         (size_t)4 * PRG * PJU * 4 + 16;
}

// ---------------------------------------------------------------- host-side launch state
// Everything below is process-wide and set up under std::call_once / a mutex: forward calls
// come from the Python thread, backward calls from PyTorch's autograd device thread.
constexpr int MAXDEV = 64;

int num_cus() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAXDEV) return 0;
  static std::once_flag once[MAXDEV];
  static int cus[MAXDEV];
  std::call_once(once[dev], [dev] {
    hipDeviceProp_t prop;
    cus[dev] = hipGetDeviceProperties(&prop, dev) == hipSuccess ? prop.multiProcessorCount : 0;
  });
  return cus[dev];
}

std::atomic<unsigned*> g_fault[MAXDEV];  // per-device fault word (avc_set_fault_word)
std::atomic<unsigned> g_spin{0};         // 0 = PSPIN (or AVC_LSTM_SPIN)

unsigned* fault_word() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAXDEV) return nullptr;
  return g_fault[dev].load(std::memory_order_acquire);
}

unsigned spin_bound() {
  static const unsigned env = [] {
    const char* v = getenv("AVC_LSTM_SPIN");
    return v ? (unsigned)strtoul(v, nullptr, 10) : 0u;
  }();
  const unsigned s = g_spin.load(std::memory_order_relaxed);
  if (s == ~0u) return 0;  // injected timeout: every wait fails at once (fault-path tests)
  return s ? s : env ? env : PSPIN;
}

// Dynamic-LDS attribute of the persistent backward kernels, set once per (kernel, device).
template <int H, bool GR>
void set_bwd_lds_attr() {
  int dev = 0;
  (void)hipGetDevice(&dev);
  static std::once_flag once[MAXDEV];
  std::call_once(once[dev & (MAXDEV - 1)], [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&lstm_persist_bwd<H, GR>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)persist_bwd_lds<H>());
  });
}

// Hand-off form.  Default (measured): granules where a consumer's granule
// payload is at most 16 KB -- the forward at H <= 512 (lstm1: 2.24 -> 1.74 us per step) --
// and the flag form above that (H = 1024 forward 3.08 vs 3.26 us, backward 4.03 vs 4.43 us:
// the doubled payload fetch costs more than the drain and the flag round trip it saves).
// (round 6: the granule form for the lstm1 backward too, H = 512, 64 KB granule payload per consumer: C2 5.53-5.55
// vs 5.50 ms, profiles/r6_gran_bwd512_ab.txt)
bool gran(bool bwd, int H) { return !bwd && (size_t)PRG * H * 4 <= 16384; }
int nap() { return 0; }  // s_sleep(1)s between the granule form's failed sweeps (none measured best)

template <int H>
const void* persist_fn(bool bwd) {
  if (bwd) {
    if (gran(true, H)) {
      set_bwd_lds_attr<H, true>();
      return reinterpret_cast<const void*>(&lstm_persist_bwd<H, true>);
    }
    set_bwd_lds_attr<H, false>();
    return reinterpret_cast<const void*>(&lstm_persist_bwd<H, false>);
  }
  return gran(false, H) ? reinterpret_cast<const void*>(&lstm_persist_fwd<H, true>)
                     : reinterpret_cast<const void*>(&lstm_persist_fwd<H, false>);
}

// Co-residency of a persistent grid: every workgroup must be resident at once (the members
// wait on each other), so the launch is taken only when the occupancy API admits `grid`
// workgroups over the device's CUs.  Cached per (kernel, device).
bool fits_resident(const void* fn, int threads, size_t lds, int grid) {
  static std::mutex mu;
  struct Entry {
    const void* fn;
    int dev;
    int blocks;
  };
  static Entry cache[64];
  static int n = 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  int blocks = -1;
  {
    std::lock_guard<std::mutex> g(mu);
    for (int i = 0; i < n; ++i)
      if (cache[i].fn == fn && cache[i].dev == dev) blocks = cache[i].blocks;
    if (blocks < 0) {
      int nb = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, threads, lds) != hipSuccess) nb = 0;
      (void)hipGetLastError();
      blocks = nb;
      if (n < 64) cache[n++] = Entry{fn, dev, nb};
    }
  }
  return (long long)blocks * num_cus() >= grid;
}

bool no_persist_env() {
  static const bool v = getenv("AVC_LSTM_NO_PERSIST") != nullptr;
  return v;
}

// Whether the one-launch persistent recurrence applies (the same test the launches make).
bool persistent_path(int B, int H, int dirs, bool bf, bool bwd) {
  if (!bf || dirs != 1 || !(H == 1024 || H == 768 || H == 512) || no_persist_env()) return false;
  const int ng = (B + PRG - 1) / PRG, grid = ng * (H / PJU);
  if (grid > num_cus()) return false;
  const void* fn = H == 1024 ? persist_fn<1024>(bwd) : H == 768 ? persist_fn<768>(bwd) : persist_fn<512>(bwd);
  const size_t lds = !bwd ? 0
                     : H == 1024 ? persist_bwd_lds<1024>()
                     : H == 768  ? persist_bwd_lds<768>()
                                 : persist_bwd_lds<512>();
  return fits_resident(fn, PNT, lds, grid);
}

template <int H>
void launch_persist_bwd(dim3 grid, hipStream_t s, bool gr, const PersistBwdArgs& p) {
  if (gr) lstm_persist_bwd<H, true><<<grid, PNT, persist_bwd_lds<H>(), s>>>(p);
  else lstm_persist_bwd<H, false><<<grid, PNT, persist_bwd_lds<H>(), s>>>(p);
}

// The one-launch persistent forward (persistent_path() true): hbuf = control words + flags +
// the [2][B][H] payload (layout above); xproj row b*(T/seg) + t/seg feeds step t.
int persist_fwd(const float* xproj, int seg, const void* w_hh, int B, int T, int H, float* h, void* h_bf16, float* c,
                float* gates, void* hbuf, hipStream_t s, const char* what) {
  const int ng = (B + PRG - 1) / PRG;
  PersistArgs p;
  p.xproj = xproj;
  p.w = reinterpret_cast<const bf16*>(w_hh);
  p.hout = h;
  p.hout16 = reinterpret_cast<bf16*>(h_bf16);
  p.call = c;
  p.gall = gates;
  p.ctl = reinterpret_cast<unsigned*>(hbuf);
  p.pay = reinterpret_cast<bf16*>(reinterpret_cast<char*>(hbuf) + px_payload_off(ng));
  p.trace = g_trace;
  p.fault = fault_word();
  p.spin = spin_bound();
  p.nap = nap();
  p.B = B;
  p.T = T;
  p.ng = ng;
  p.seg = seg;
  const bool gr = gran(false, H);
  // flag form: only ctl + flags are polled; granule form: every tag of the payload too
  if (avc_zero_async(hbuf, gr ? px_payload_off(ng) + (size_t)8 * B * H : px_ctl_bytes(ng), s)) return -1;
  const dim3 grid(ng * (H / PJU));
  if (H == 1024) gr ? lstm_persist_fwd<1024, true><<<grid, PNT, 0, s>>>(p) : lstm_persist_fwd<1024, false><<<grid, PNT, 0, s>>>(p);
  else if (H == 768) gr ? lstm_persist_fwd<768, true><<<grid, PNT, 0, s>>>(p) : lstm_persist_fwd<768, false><<<grid, PNT, 0, s>>>(p);  // Adjust.py:30
  else gr ? lstm_persist_fwd<512, true><<<grid, PNT, 0, s>>>(p) : lstm_persist_fwd<512, false><<<grid, PNT, 0, s>>>(p);
  return avc_check_launch(what);
}

// The persistent backward (persistent_path() true); gbuf = control words + flags + the
// [2][B][4H] payload.  dg (fp32) and dg16 nullable; sc / sc16 (nullable): dG summed over
// each seg-frame segment.
int persist_bwd(const float* dh_out, const float* c, const float* gates, const void* w_hh_t, int B, int T, int H,
                float* dg, void* dg16, float* sc, void* sc16, int seg, void* gbuf, hipStream_t s, const char* what) {
  const int ng = (B + PRG - 1) / PRG;
  PersistBwdArgs p;
  p.dhout = dh_out;
  p.call = c;
  p.gall = gates;
  p.wt = reinterpret_cast<const bf16*>(w_hh_t);
  p.dg = dg;
  p.dg16 = reinterpret_cast<bf16*>(dg16);
  p.sc = sc;
  p.sc16 = reinterpret_cast<bf16*>(sc16);
  p.ctl = reinterpret_cast<unsigned*>(gbuf);
  p.pay = reinterpret_cast<bf16*>(reinterpret_cast<char*>(gbuf) + px_payload_off(ng));
  p.trace = g_trace;
  p.fault = fault_word();
  p.spin = spin_bound();
  p.nap = nap();
  p.B = B;
  p.T = T;
  p.ng = ng;
  p.seg = seg;
  const bool gr = gran(true, H);
  if (avc_zero_async(gbuf, gr ? px_payload_off(ng) + (size_t)32 * B * H : px_ctl_bytes(ng), s)) return -1;
  // (persistent_path set the dynamic-LDS attributes)
  const dim3 grid(ng * (H / PJU));
  if (H == 1024) launch_persist_bwd<1024>(grid, s, gr, p);
  else if (H == 768) launch_persist_bwd<768>(grid, s, gr, p);
  else launch_persist_bwd<512>(grid, s, gr, p);
  return avc_check_launch(what);
}

template <int HM>
void launch_small_fwd(dim3 g, hipStream_t s, bool fast, const float* x, const float* w, int T, int H, int dirs,
                      float* h, bf16* h16, float* c, float* gt) {
  if (g_trace) lstm_small_fwd<HM, true, true><<<g, SNT, 0, s>>>(x, w, T, H, dirs, h, h16, c, gt, g_trace);
  else if (fast) lstm_small_fwd<HM, true, false><<<g, SNT, 0, s>>>(x, w, T, H, dirs, h, h16, c, gt, nullptr);
  else lstm_small_fwd<HM, false, false><<<g, SNT, 0, s>>>(x, w, T, H, dirs, h, h16, c, gt, nullptr);
}
template <int HM>
void launch_small_bwd(dim3 g, hipStream_t s, bool fast, const float* dh, const float* c, const float* gt,
                      const float* w, int T, int H, int dirs, float* dg, bf16* dg16) {
  if (g_trace) lstm_small_bwd<HM, true, true><<<g, SNT, 0, s>>>(dh, c, gt, w, T, H, dirs, dg, dg16, g_trace);
  else if (fast) lstm_small_bwd<HM, true, false><<<g, SNT, 0, s>>>(dh, c, gt, w, T, H, dirs, dg, dg16, nullptr);
  else lstm_small_bwd<HM, false, false><<<g, SNT, 0, s>>>(dh, c, gt, w, T, H, dirs, dg, dg16, nullptr);
}

// The MFMA form of the encoder BiLSTM (lstm_mfma_fwd / _bwd): bf16 compute, H in {16, 32, 44, 48, 64}.
// Off by default (slower, see the kernels); avc_lstm_set_small_mfma(1) or AVC_BILSTM_MFMA=1 selects it.
std::atomic<int> g_small_mfma{-1};
bool small_mfma(int H, bool fast) {
  int on = g_small_mfma.load(std::memory_order_relaxed);
  if (on < 0) on = getenv("AVC_BILSTM_MFMA") ? atoi(getenv("AVC_BILSTM_MFMA")) != 0 : 0;
  return on && fast && (H == 16 || H == 32 || H == 44 || H == 48 || H == 64);
}
template <int KC>
void launch_mfma_fwd(hipStream_t s, const float* x, const float* w, int B, int T, int dirs, float* h, bf16* h16,
                     float* c, float* gt) {
  constexpr int NW = (4 * KC + 15) / 16;
  const dim3 g(cdiv(B, MU), dirs);
  if (g_trace) lstm_mfma_fwd<KC, NW, true><<<g, NW * 64, 0, s>>>(x, w, B, T, dirs, h, h16, c, gt, g_trace);
  else lstm_mfma_fwd<KC, NW, false><<<g, NW * 64, 0, s>>>(x, w, B, T, dirs, h, h16, c, gt, nullptr);
}
template <int KC>
void launch_mfma_bwd(hipStream_t s, const float* dh, const float* c, const float* gt, const float* w, int B, int T,
                     int dirs, float* dg, bf16* dg16) {
  constexpr int NW = (4 * KC + 15) / 16;
  const dim3 g(cdiv(B, MU), dirs);
  if (g_trace) lstm_mfma_bwd<KC, NW, true><<<g, NW * 64, 0, s>>>(dh, c, gt, w, B, T, dirs, dg, dg16, g_trace);
  else lstm_mfma_bwd<KC, NW, false><<<g, NW * 64, 0, s>>>(dh, c, gt, w, B, T, dirs, dg, dg16, nullptr);
}

}  // namespace

extern "C" int avc_lstm_small_mfma(int H, int compute) { return small_mfma(H, compute == AVC_BF16) ? 1 : 0; }
extern "C" int avc_lstm_set_small_mfma(int mode) {
  g_small_mfma.store(mode < 0 ? -1 : (mode ? 1 : 0), std::memory_order_relaxed);
  return 0;
}

unsigned* avc_fault_ptr() { return fault_word(); }

extern "C" int avc_lstm_trace(void* buf) {
  g_trace = reinterpret_cast<unsigned long long*>(buf);
  return 0;
}

extern "C" int avc_set_fault_word(void* word) {
  int dev = 0;
  AVC_CHECK_ARG(hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < MAXDEV, "avc_set_fault_word: no device");
  g_fault[dev].store(reinterpret_cast<unsigned*>(word), std::memory_order_release);
  return 0;
}

extern "C" int avc_lstm_set_spin(unsigned spins) {
  g_spin.store(spins, std::memory_order_relaxed);
  return 0;
}

// Two-layer wavefront forward (lstm2_persist_fwd): shape, compute mode and residency.
#define L2FN(LB, OS) reinterpret_cast<const void*>(&lstm2_persist_fwd<1024, 2, LB, OS>)
bool persist2_path(int B, int H, int In1, bool bf) {
  if (!bf || H != 1024 || In1 != H || no_persist_env() || getenv("AVC_LSTM2_OFF")) return false;
  const int ng = (B + QRG - 1) / QRG, grid = ng * (H / QJU);
  if (grid > num_cus()) return false;
  static std::once_flag once[MAXDEV];
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::call_once(once[dev & (MAXDEV - 1)], [] {
    for (const void* f : {L2FN(1, false), L2FN(2, false), L2FN(1, true), L2FN(2, true)})
      (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)persist2_lds<1024>());
  });
  return fits_resident(L2FN(2, false), PNT, persist2_lds<1024>(), grid);
}

extern "C" int avc_lstm2_persistent(int B, int H, int in1, int compute) {
  return persist2_path(B, H, in1, compute == AVC_BF16) ? 1 : 0;
}

extern "C" size_t avc_lstm2_scratch_bytes(int B, int H) {
  if (B <= 0 || H <= 0) return 0;
  return px_payload_off((B + QRG - 1) / QRG) + (size_t)8 * B * H;
}

extern "C" int avc_lstm2_fwd(const float* xproj0, const void* w_hh0, const void* w_ih1, const void* w_hh1,
                             const float* bias1, int B, int T, int H, float* h0, void* h0_bf16, float* c0,
                             float* gates0, float* h1, void* h1_bf16, float* c1, float* gates1, void* buf,
                             void* stream) {
  AVC_CHECK_ARG(xproj0 && w_hh0 && w_ih1 && w_hh1 && bias1 && h0 && h0_bf16 && c0 && gates0 && h1 && h1_bf16 && c1 &&
                    gates1 && buf && B > 0 && T > 0,
                "avc_lstm2_fwd: bad args");
  AVC_CHECK_ARG(persist2_path(B, H, H, true), "avc_lstm2_fwd: shape B=%d H=%d not supported (see avc_lstm2_persistent)",
                B, H);
  hipStream_t s = as_stream(stream);
  const int ng = (B + QRG - 1) / QRG;
  Persist2Args p;
  p.xproj = xproj0;
  p.w0 = reinterpret_cast<const bf16*>(w_hh0);
  p.wi1 = reinterpret_cast<const bf16*>(w_ih1);
  p.w1 = reinterpret_cast<const bf16*>(w_hh1);
  p.bias1 = bias1;
  p.hout[0] = h0;
  p.hout[1] = h1;
  p.hout16[0] = reinterpret_cast<bf16*>(h0_bf16);
  p.hout16[1] = reinterpret_cast<bf16*>(h1_bf16);
  p.call[0] = c0;
  p.call[1] = c1;
  p.gall[0] = gates0;
  p.gall[1] = gates1;
  p.ctl = reinterpret_cast<unsigned*>(buf);
  p.pay = reinterpret_cast<bf16*>(reinterpret_cast<char*>(buf) + px_payload_off(ng));
  p.trace = g_trace;
  p.fault = fault_word();
  p.spin = spin_bound();
  p.B = B;
  p.T = T;
  p.ng = ng;
  if (avc_zero_async(buf, px_ctl_bytes(ng), s)) return -1;
  // scheduling fence every 2 k-blocks of the product (without one the compiler hoists the A
  // fragment reads and spills weight fragments); payload loads in 2 batches, the previous tick's
  // outputs stored after the products (1 batch, or the stores under the payload loads: slower)
  const dim3 grid(ng * (H / QJU));
  lstm2_persist_fwd<1024, 2, 2, false><<<grid, PNT, persist2_lds<1024>(), s>>>(p);
  return avc_check_launch("avc_lstm2_fwd");
}

// Two-layer wavefront backward (lstm2_persist_bwd): shape, compute mode and residency.
bool persist2_bwd_path(int B, int H, bool bf) {
  if (!bf || H != 1024 || no_persist_env() || getenv("AVC_LSTM2_OFF")) return false;
  const int ng = (B + QRG - 1) / QRG, grid = ng * (H / QJU);
  if (grid > num_cus()) return false;
  static std::once_flag once[MAXDEV];
  int dev = 0;
  (void)hipGetDevice(&dev);
  const void* fn = reinterpret_cast<const void*>(&lstm2_persist_bwd<1024>);
  std::call_once(once[dev & (MAXDEV - 1)], [fn] {
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)persist2_bwd_lds<1024>());
  });
  return fits_resident(fn, PNT, persist2_bwd_lds<1024>(), grid);
}

extern "C" int avc_lstm2_bwd_persistent(int B, int H, int compute) {
  return persist2_bwd_path(B, H, compute == AVC_BF16) ? 1 : 0;
}

extern "C" size_t avc_lstm2_bwd_scratch_bytes(int B, int H) {
  if (B <= 0 || H <= 0) return 0;
  return px_payload_off((B + QRG - 1) / QRG) + (size_t)32 * B * H;  // [2 layers][2 parities][B][4H] bf16
}

extern "C" int avc_lstm2_bwd(const float* dh1, const float* c0, const float* gates0, const float* c1,
                             const float* gates1, const void* w_hh0_t, const void* w_ih1_t, const void* w_hh1_t, int B,
                             int T, int H, float* dg0, void* dg0_bf16, float* dg1, void* dg1_bf16, void* buf,
                             float* db_part, void* stream) {
  AVC_CHECK_ARG(dh1 && c0 && gates0 && c1 && gates1 && w_hh0_t && w_ih1_t && w_hh1_t && (dg0 || dg0_bf16) &&
                    (dg1 || dg1_bf16) && buf && B > 0 && T > 0,
                "avc_lstm2_bwd: bad args");
  AVC_CHECK_ARG(persist2_bwd_path(B, H, true), "avc_lstm2_bwd: shape B=%d H=%d not supported (see avc_lstm2_bwd_persistent)",
                B, H);
  hipStream_t s = as_stream(stream);
  const int ng = (B + QRG - 1) / QRG;
  Persist2BwdArgs p;
  p.dhout1 = dh1;
  p.call[0] = c0;
  p.call[1] = c1;
  p.gall[0] = gates0;
  p.gall[1] = gates1;
  p.wt0 = reinterpret_cast<const bf16*>(w_hh0_t);
  p.wti1 = reinterpret_cast<const bf16*>(w_ih1_t);
  p.wt1 = reinterpret_cast<const bf16*>(w_hh1_t);
  p.dg[0] = dg0;
  p.dg[1] = dg1;
  p.dg16[0] = reinterpret_cast<bf16*>(dg0_bf16);
  p.dg16[1] = reinterpret_cast<bf16*>(dg1_bf16);
  p.dbp = db_part;
  p.ctl = reinterpret_cast<unsigned*>(buf);
  p.pay = reinterpret_cast<bf16*>(reinterpret_cast<char*>(buf) + px_payload_off(ng));
  p.trace = g_trace;
  p.fault = fault_word();
  p.spin = spin_bound();
  p.B = B;
  p.T = T;
  p.ng = ng;
  p.opt = 1;  // the dG stores behind a barrier after the flag (payload-as-output, bit 4: measured slower,
              // profiles/r6_lstm2_bwd_payload_out.txt)
  if (avc_zero_async(buf, px_ctl_bytes(ng), s)) return -1;
  lstm2_persist_bwd<1024><<<dim3(ng * (H / QJU)), PNT, persist2_bwd_lds<1024>(), s>>>(p);
  return avc_check_launch("avc_lstm2_bwd");
}

extern "C" size_t avc_lstm_bwd_scratch_bytes(int B, int H, int dirs) {
  if (B <= 0 || H <= 0 || dirs <= 0) return 0;
  // per-step ping-pong (16 dirs B H) or control words + the [2][B][4H] granule payload (32 B H)
  return std::max((size_t)16 * dirs * B * H, (size_t)32 * B * H + 8192);
}

extern "C" int avc_lstm_persistent(int B, int H, int dirs, int compute, int backward) {
  return persistent_path(B, H, dirs, compute == AVC_BF16, backward != 0) ? 1 : 0;
}

extern "C" int avc_lstm_fwd(const float* xproj, const void* w_hh, int wdtype, int B, int T, int H, int dirs, float* h,
                            void* h_bf16, float* c, float* gates, void* hbuf, int compute, void* stream) {
  AVC_CHECK_ARG(xproj && w_hh && h && c && gates && B > 0 && T > 0 && H > 0 && (dirs == 1 || dirs == 2),
                "avc_lstm_fwd: bad args");
  hipStream_t s = as_stream(stream);
  if (H <= 64) {
    AVC_CHECK_ARG(wdtype == AVC_F32, "avc_lstm_fwd: small-H path takes fp32 W_hh");
    const bool fast = compute == AVC_BF16;  // fp32 weights and state either way; fast activations in bf16 mode
    bf16* h16 = reinterpret_cast<bf16*>(h_bf16);
    if (small_mfma(H, fast)) {
      const float* w = (const float*)w_hh;
      switch (H) {
        case 16: launch_mfma_fwd<4>(s, xproj, w, B, T, dirs, h, h16, c, gates); break;
        case 32: launch_mfma_fwd<8>(s, xproj, w, B, T, dirs, h, h16, c, gates); break;
        case 44: launch_mfma_fwd<11>(s, xproj, w, B, T, dirs, h, h16, c, gates); break;
        case 48: launch_mfma_fwd<12>(s, xproj, w, B, T, dirs, h, h16, c, gates); break;
        default: launch_mfma_fwd<16>(s, xproj, w, B, T, dirs, h, h16, c, gates); break;
      }
      return avc_check_launch("avc_lstm_fwd(small, mfma)");
    }
    dim3 g(B, dirs);
    if (H <= 16) launch_small_fwd<16>(g, s, fast, xproj, (const float*)w_hh, T, H, dirs, h, h16, c, gates);
    else if (H <= 32) launch_small_fwd<32>(g, s, fast, xproj, (const float*)w_hh, T, H, dirs, h, h16, c, gates);
    else if (H <= 48) launch_small_fwd<48>(g, s, fast, xproj, (const float*)w_hh, T, H, dirs, h, h16, c, gates);
    else launch_small_fwd<64>(g, s, fast, xproj, (const float*)w_hh, T, H, dirs, h, h16, c, gates);
    return avc_check_launch("avc_lstm_fwd(small)");
  }
  AVC_CHECK_ARG(H % 128 == 0, "avc_lstm_fwd: H must be <= 64 or a multiple of 128 (got %d)", H);
  const bool bf = compute == AVC_BF16;
  AVC_CHECK_ARG(!bf || (wdtype == AVC_BF16 && hbuf), "avc_lstm_fwd: bf16 compute needs bf16 W_hh and hbuf");
  AVC_CHECK_ARG(bf || wdtype == AVC_F32, "avc_lstm_fwd: fp32 compute needs fp32 W_hh");
  StepArgs a = {};
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
  if (hbuf && persistent_path(B, H, dirs, bf, false))
    return persist_fwd(xproj, 1, w_hh, B, T, H, h, h_bf16, c, gates, hbuf, s, "avc_lstm_fwd(persistent)");
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
    const bool fast = compute == AVC_BF16;
    bf16* dg16 = reinterpret_cast<bf16*>(dgates_bf16);
    if (small_mfma(H, fast)) {
      const float* w = (const float*)w_hh;
      switch (H) {
        case 16: launch_mfma_bwd<4>(s, dh_out, c, gates, w, B, T, dirs, dgates, dg16); break;
        case 32: launch_mfma_bwd<8>(s, dh_out, c, gates, w, B, T, dirs, dgates, dg16); break;
        case 44: launch_mfma_bwd<11>(s, dh_out, c, gates, w, B, T, dirs, dgates, dg16); break;
        case 48: launch_mfma_bwd<12>(s, dh_out, c, gates, w, B, T, dirs, dgates, dg16); break;
        default: launch_mfma_bwd<16>(s, dh_out, c, gates, w, B, T, dirs, dgates, dg16); break;
      }
      return avc_check_launch("avc_lstm_bwd(small, mfma)");
    }
    dim3 g(B, dirs);
    if (H <= 16) launch_small_bwd<16>(g, s, fast, dh_out, c, gates, (const float*)w_hh, T, H, dirs, dgates, dg16);
    else if (H <= 32) launch_small_bwd<32>(g, s, fast, dh_out, c, gates, (const float*)w_hh, T, H, dirs, dgates, dg16);
    else if (H <= 48) launch_small_bwd<48>(g, s, fast, dh_out, c, gates, (const float*)w_hh, T, H, dirs, dgates, dg16);
    else launch_small_bwd<64>(g, s, fast, dh_out, c, gates, (const float*)w_hh, T, H, dirs, dgates, dg16);
    return avc_check_launch("avc_lstm_bwd(small)");
  }
  AVC_CHECK_ARG(H % 128 == 0, "avc_lstm_bwd: H must be <= 64 or a multiple of 128 (got %d)", H);
  AVC_CHECK_ARG(w_hh_t && dcbuf, "avc_lstm_bwd: large-H path needs W_hh^T and dcbuf");
  const bool bf = compute == AVC_BF16;
  AVC_CHECK_ARG(!bf || (wdtype == AVC_BF16 && gbuf), "avc_lstm_bwd: bf16 compute needs bf16 W_hh^T and gbuf");
  if (persistent_path(B, H, dirs, bf, true))
    return persist_bwd(dh_out, c, gates, w_hh_t, B, T, H, dgates, dgates_bf16, nullptr, nullptr, 1, gbuf, s,
                       "avc_lstm_bwd(persistent)");
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

extern "C" int avc_lstm_fwd_fold(const float* pcode, int nc, const void* w_hh, int B, int T, int H, float* h,
                                 void* h_bf16, float* c, float* gates, void* hbuf, void* stream) {
  AVC_CHECK_ARG(pcode && w_hh && h && h_bf16 && c && gates && hbuf && B > 0 && T > 0 && nc > 0 && T % nc == 0,
                "avc_lstm_fwd_fold: bad args");
  AVC_CHECK_ARG(persistent_path(B, H, 1, true, false), "avc_lstm_fwd_fold: B=%d H=%d is not on the persistent path",
                B, H);
  return persist_fwd(pcode, T / nc, w_hh, B, T, H, h, h_bf16, c, gates, hbuf, as_stream(stream),
                     "avc_lstm_fwd_fold");
}

extern "C" int avc_lstm_bwd_fold(const float* dh_out, const float* c, const float* gates, const void* w_hh_t, int B,
                                 int T, int H, int nc, float* dgates, void* dgates_bf16, float* s_code,
                                 void* s_code_bf16, void* gbuf, void* stream) {
  AVC_CHECK_ARG(dh_out && c && gates && w_hh_t && dgates_bf16 && s_code && gbuf && B > 0 && T > 0 && nc > 0 &&
                    T % nc == 0,
                "avc_lstm_bwd_fold: bad args");
  AVC_CHECK_ARG(persistent_path(B, H, 1, true, true), "avc_lstm_bwd_fold: B=%d H=%d is not on the persistent path",
                B, H);
  return persist_bwd(dh_out, c, gates, w_hh_t, B, T, H, dgates, dgates_bf16, s_code, s_code_bf16, T / nc, gbuf,
                     as_stream(stream), "avc_lstm_bwd_fold");
}
