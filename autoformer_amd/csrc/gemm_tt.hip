// gemm_tt.hip — bf16 "TT" GEMM (both operands K-strided) fed by LDS DMA: the weight-gradient
// shape C[M][N] = sum_k A[k][M] B[k][N], k = frames.
//
// Serves every weight gradient of the path: dW of each Conv1d (dy^T . im2col(x), with the
// frame window on B: factory/Norm.py:21-28), dW_ih / dW_hh of the LSTMs (dG^T . x and
// dG^T . h_{t-1}, the latter a one-frame shift window: AutoVC.py:43,77,96) and the linear
// projection (Norm.py:40-50).
//
// Both operands are stored frame-major, so a K-tile is 64 frame rows x 128 columns: it is
// copied global -> LDS row by row with global_load_lds_dwordx4 (256-B rows, 16-B chunks
// XOR-swizzled as chunk ^ (((row&3)<<2) | ((row>>2)&3)) via the source address) and the
// MFMA fragments, which need 8 consecutive frames per lane, are read with the gfx950
// transposing LDS read ds_read_b64_tr_b16 (cdna_hip_programming.md §5.5 T10, layout (b):
// conflict-free for the 16x16x32 operands).  128 x 128 tile, BK = 64, 4 waves as 2 x 2,
// 2 LDS stages, counted vmcnt + raw barrier, shared fused epilogue (gemm_internal.h).
#include <algorithm>
#include <map>
#include <mutex>

#include "gemm_internal.h"

namespace avcg {
namespace {

__device__ __attribute__((aligned(16))) unsigned int g_zero16_tt[4] = {0u, 0u, 0u, 0u};

constexpr int TROW = 256;          // LDS bytes per frame row of a 128-column tile
constexpr int TSTAGE_OP = FBK * TROW;  // one operand's K-tile: 16 KiB

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef const __attribute__((address_space(1))) void* gbl_ptr_t;
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4* lds_s4_ptr;

__device__ __forceinline__ void glds16(const void* src, char* lds) {
  __builtin_amdgcn_global_load_lds((gbl_ptr_t)src, (lds_ptr_t)lds, 16, 0, 0);
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void raw_barrier() { asm volatile("s_barrier" ::: "memory"); }

__device__ __forceinline__ int tswz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }

// One K-strided operand: tile of 64 frame rows x 128 columns [col0, col0 + 128), loaded by NW
// waves.  Wave w, instruction i covers rows 4*(NW*i + w) .. +4; lane L writes row +(L>>4), slot
// L&15, holding global chunk (L&15) ^ tswz(row) = (L&15) ^ (((L>>4)<<2) | (w&3)) (NW is a
// multiple of 4): one fixed column per lane.
template <bool WIN, int NW = 4>
struct TtLoader {
  static constexpr int NI = 16 / NW;
  const bf16* base;
  int col_ok;          // this lane's 8 columns lie inside the operand
  int coff;            // element offset of the lane's column inside a frame row
  int tap;             // window: tap of the lane's column
  long long ld;
  int pad, t_in, t_out;
  FastDiv tdiv;

  __device__ __forceinline__ void init(const OpDev& o, int col0, int bz) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    base = reinterpret_cast<const bf16*>(o.ptr) + (long long)bz * o.bstride;
    const int ch = (lane & 15) ^ (((lane >> 4) << 2) | (w & 3));
    const int col = col0 + 8 * ch;
    col_ok = col < o.rows;
    ld = o.ld;
    pad = o.pad;
    t_in = o.t_in;
    t_out = o.t_out;
    tdiv = o.tdiv;
    if (WIN) {
      tap = col_ok ? (int)fdiv((uint32_t)col, o.cdv) : 0;
      coff = col - tap * o.chans;
    } else {
      tap = 0;
      coff = col;
    }
  }

  __device__ __forceinline__ void issue(char* lds_tile, int kbase, int kend) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int r = 4 * (NW * i + w) + (lane >> 4);
      const int k = kbase + r;
      bool ok = col_ok && k < kend;
      long long frame = k;
      if (WIN) {
        const int b = (int)fdiv((uint32_t)(ok ? k : 0), tdiv);
        const int t2 = k - b * t_out + tap - pad;
        ok = ok && t2 >= 0 && t2 < t_in;
        frame = (long long)b * t_in + t2;
      }
      const void* src = ok ? (const void*)(base + frame * ld + coff) : (const void*)g_zero16_tt;
      glds16(src, lds_tile + 4 * (NW * i + w) * TROW);
    }
  }
};

// Per-lane byte offsets of the two transposed reads (frames +0..3 and +4..7 of the lane's
// 8-frame group) of 16-column block `blk` (= first chunk / 2) inside a 64-frame tile, k-sub 0.
__device__ __forceinline__ void tr_offsets(int chunk0, int& o0, int& o1) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, ql = lane & 15, q = ql >> 2, p = ql & 3;
  const int r0 = 8 * g + q, r1 = 8 * g + 4 + q;
  o0 = r0 * TROW + 16 * ((chunk0 + (p >> 1)) ^ tswz(r0)) + 8 * (p & 1);
  o1 = r1 * TROW + 16 * ((chunk0 + (p >> 1)) ^ tswz(r1)) + 8 * (p & 1);
}

__device__ __forceinline__ bf16x8 tr_frag(const char* tile, int o0, int o1) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_ptr)(tile + o0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_ptr)(tile + o1));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// The same fragment read issued as inline asm.  hipcc treats ds_read_tr16_b64 (the builtin) as
// possibly aliasing any in-flight LDS DMA and waits `vmcnt(0)` before it -- which drains the
// prefetch just issued and serialises every K-tile behind its own global load.  The asm form
// is invisible to that bookkeeping: the caller orders it after the landed stage (counted vmcnt
// + barrier) and waits for the reads itself (tr_wait) before the MFMAs use them.
__device__ __forceinline__ unsigned lds_addr(const char* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
__device__ __forceinline__ bf16x8 tr_frag_asm(const char* tile, int o0, int o1) {
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x4 lo, hi;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(lds_addr(tile + o0)));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(hi) : "v"(lds_addr(tile + o1)));
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}
__device__ __forceinline__ void tr_wait() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);  // nothing (an MFMA on the read registers) moves above the wait
}

template <bool WINB>
__global__ void __launch_bounds__(256, 2) gemm_tt_kernel(GemmArgs g) {
  constexpr int BN_ = 128, NJ = 4;
  constexpr int STAGE = 2 * TSTAGE_OP;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const int tid = threadIdx.x, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q = nwg >> 3, rr = nwg & 7, xcd = bid & 7;
  const int lid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
  const int nN = (g.N + BN_ - 1) / BN_, nM = (g.M + BM - 1) / BM;
  const int z = lid / (nN * nM);
  const int rem = lid - z * nN * nM;
  const int mt = rem / nN, nt = rem - mt * nN;
  const int m0 = mt * BM, n0 = nt * BN_;
  const int bz = z / g.split_k, ks = z - bz * g.split_k;
  const int kbeg = ks * g.klen;
  const int kend = min(g.K, kbeg + g.klen);
  const int nkt = kend > kbeg ? (kend - kbeg + FBK - 1) / FBK : 0;

  TtLoader<false> la;
  TtLoader<WINB> lb;
  la.init(g.a, m0, bz);
  lb.init(g.b, n0, bz);

  f32x4 acc[4][NJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  int ao0[4], ao1[4], bo0[NJ], bo1[NJ];
#pragma unroll
  for (int i = 0; i < 4; ++i) tr_offsets(wm * 8 + 2 * i, ao0[i], ao1[i]);
#pragma unroll
  for (int j = 0; j < NJ; ++j) tr_offsets(wn * 8 + 2 * j, bo0[j], bo1[j]);

  if (nkt > 0) {
    la.issue(smem_raw, kbeg, kend);
    lb.issue(smem_raw + TSTAGE_OP, kbeg, kend);
  }
  for (int kt = 0; kt < nkt; ++kt) {
    wait_vm<0>();
    raw_barrier();
    if (kt + 1 < nkt) {
      char* st = smem_raw + ((kt + 1) & 1) * STAGE;
      la.issue(st, kbeg + (kt + 1) * FBK, kend);
      lb.issue(st + TSTAGE_OP, kbeg + (kt + 1) * FBK, kend);
    }
    const char* As = smem_raw + (kt & 1) * STAGE;
    const char* Bs = As + TSTAGE_OP;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int ko = h * 32 * TROW;
      bf16x8 af[4], bfr[NJ];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = tr_frag_asm(As + ko, ao0[i], ao1[i]);
#pragma unroll
      for (int j = 0; j < NJ; ++j) bfr[j] = tr_frag_asm(Bs + ko, bo0[j], bo1[j]);
      tr_wait();
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }
  __syncthreads();
  if (g.sk_ws && !splitk_last<4 * NJ>(g, &acc[0][0], rem, ks)) return;  // (batch 1: z = ks)
  fast_epilogue<BN_, false>(g, acc, m0, n0, mt, bz, ks, smem_raw);  // (weight gradients: no BN-backward epilogue)
}

template <bool WINB>
void launch(const GemmArgs& g, int nblocks, hipStream_t s) {
  const size_t lds = 2 * 2 * (size_t)TSTAGE_OP;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_tt_kernel<WINB>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  gemm_tt_kernel<WINB><<<nblocks, 256, lds, s>>>(g);
}

bool ok16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// ------------------------------------------------------------------ halo form of the conv dW
// dW[co][tap*Ci + ci] = sum_f dy[f][co] . x[f + tap - pad][ci] for a 5-tap 'same' Conv1d whose
// utterance length is a multiple of the 64-frame K-tile (so a K-tile never spans utterances).
// The window operand above fetches a 64 x 128 tile of x per (tap, 128-channel) column block --
// five copies of the same rows shifted by one.  Here a workgroup owns 128 output channels x
// (5 taps x 32 input channels): per K-tile it stages the dy tile (64 x 128, as above) and ONE
// x halo tile of 68 frames x 32 channels (64-B rows), and tap k reads the halo k rows down.
// Halo rows outside the tile's utterance are loaded as zeros, which is exactly the conv
// padding.  Transposed reads (ds_read_b64_tr_b16) of the 64-B rows use the chunk swizzle
// chunk ^ ((row >> 2) & 2): the two 16-lane groups of a half read rows 8 apart, which then
// take the two different 32-B halves of the row -- conflict-free.
constexpr int HROW = 64;                 // bytes per halo row (32 channels)
constexpr int HROWS = 128;               // halo rows reserved: 2 glds of 16 rows per wave
constexpr int HB_BYTES = HROWS * HROW;   // 8 KiB
constexpr int HSTAGE = TSTAGE_OP + HB_BYTES;

__device__ __forceinline__ int hswz(int row) { return (row >> 2) & 2; }

__device__ __forceinline__ bf16x8 tr_frag_h(const char* tile, int rlo, int chunk0, int p) {
  const int rhi = rlo + 4;
  const int olo = rlo * HROW + 16 * ((chunk0 + (p >> 1)) ^ hswz(rlo)) + 8 * (p & 1);
  const int ohi = rhi * HROW + 16 * ((chunk0 + (p >> 1)) ^ hswz(rhi)) + 8 * (p & 1);
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_ptr)(tile + olo));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_ptr)(tile + ohi));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ bf16x8 tr_frag_h_asm(const char* tile, int rlo, int chunk0, int p) {
  const int rhi = rlo + 4;
  const int olo = rlo * HROW + 16 * ((chunk0 + (p >> 1)) ^ hswz(rlo)) + 8 * (p & 1);
  const int ohi = rhi * HROW + 16 * ((chunk0 + (p >> 1)) ^ hswz(rhi)) + 8 * (p & 1);
  return tr_frag_asm(tile, olo, ohi);
}

template <int NST>
__global__ void __launch_bounds__(256, 2) gemm_tt_halo_kernel(GemmArgs g) {
  constexpr int TAPS = 5, CW = 32, P = NST - 1, LPT = 6;  // glds per thread per K-tile: 4 dy + 2 halo
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];

  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q8 = nwg >> 3, rr = nwg & 7, xcd = bid & 7;
  const int lid = (xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8) + (bid >> 3);
  const OpDev& X = g.b;
  const int chans = X.chans, pad = X.pad, T = X.t_out;
  const int nC = chans / CW, nM = (g.M + BM - 1) / BM;
  const int ks = lid / (nC * nM);
  const int rem = lid - ks * nC * nM;
  const int mt = rem / nC, ct = rem - mt * nC;
  const int m0 = mt * BM, c0 = ct * CW;
  // K-tiles follow the utterance grid: utterance u has tpu tiles of FBK frames, the last one
  // partial when T % FBK != 0 (its dy rows past the utterance load as zeros), so a tile never
  // spans two utterances and one halo copy serves all five taps.  Split ks takes tiles
  // [tb, te) of the (K / T) * tpu.
  const int tpu = (T + FBK - 1) / FBK;
  const int ntiles = (g.K / T) * tpu;
  const int tps = (ntiles + g.split_k - 1) / g.split_k;
  const int tb = min(ntiles, ks * tps), te = min(ntiles, tb + tps);
  const int nkt = te - tb;
  auto tile = [&](int j, int& fend, int& u0) {
    const int u = j / tpu;
    u0 = u * T;
    const int f0 = u0 + (j - u * tpu) * FBK;
    fend = min(f0 + FBK, u0 + T);
    return f0;
  };

  TtLoader<false> la;
  la.init(g.a, m0, 0);
  // halo loader: instruction i (0, 1) of wave w writes rows 16*(2w + i) + (lane >> 2), slot lane & 3
  const bf16* xb = reinterpret_cast<const bf16*>(X.ptr);
  const long long ldx = X.ld;
  int hrow[2], hchk[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    hrow[i] = 16 * (2 * wid + i) + (lane >> 2);
    hchk[i] = 8 * ((lane & 3) ^ hswz(hrow[i]));
  }
  // the K-tile at frame f0 of the utterance [u0, u0 + T); halo rows outside it load as zeros
  auto issue_halo = [&](char* st, int f0, int u0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int f = f0 - pad + hrow[i];
      const bool ok = hrow[i] < FBK + TAPS - 1 && f >= u0 && f < u0 + T;
      const void* src = ok ? (const void*)(xb + (long long)f * ldx + c0 + hchk[i]) : (const void*)g_zero16_tt;
      glds16(src, st + (2 * wid + i) * 1024);
    }
  };
  auto issue_tile = [&](char* st, int j) {
    int fend, u0;
    const int f0 = tile(j, fend, u0);
    la.issue(st, f0, fend);
    issue_halo(st + TSTAGE_OP, f0, u0);
  };

  f32x4 acc[4][TAPS];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int k = 0; k < TAPS; ++k) acc[i][k] = f32x4{0.f, 0.f, 0.f, 0.f};
  int ao0[4], ao1[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) tr_offsets(wm * 8 + 2 * i, ao0[i], ao1[i]);
  const int grp = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;

#pragma unroll
  for (int p = 0; p < P; ++p)
    if (p < nkt) issue_tile(smem_raw + p * HSTAGE, tb + p);
  for (int kt = 0; kt < nkt; ++kt) {
    const int ahead = min(P - 1, nkt - 1 - kt);  // K-tiles allowed to stay in flight
    if constexpr (P >= 2) {
      if (ahead >= 1) wait_vm<LPT>();
      else wait_vm<0>();
    } else {
      wait_vm<0>();
    }
    raw_barrier();
    if (kt + P < nkt) issue_tile(smem_raw + ((kt + P) % NST) * HSTAGE, tb + kt + P);
    const char* As = smem_raw + (kt % NST) * HSTAGE;
    const char* Hs = As + TSTAGE_OP;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      // all 18 fragment reads of the K-half in flight before the 20 MFMAs: one LDS latency
      // per K-half instead of one per tap
      bf16x8 af[4], bfr[TAPS];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = tr_frag_asm(As + h * 32 * TROW, ao0[i], ao1[i]);
#pragma unroll
      for (int k = 0; k < TAPS; ++k) bfr[k] = tr_frag_h_asm(Hs, h * 32 + 8 * grp + qq + k, 2 * wn, pp);
      tr_wait();
#pragma unroll
      for (int k = 0; k < TAPS; ++k)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc[i][k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[k], acc[i][k], 0, 0, 0);
    }
  }
  if (g.sk_ws && !splitk_last<4 * TAPS>(g, &acc[0][0], rem, ks)) return;
  // epilogue: row m0 + wm*64 + 16i + 4*(lane>>4) + e, column tap*chans + c0 + 16*wn + (lane & 15)
  const int rbase = m0 + wm * 64 + 4 * (lane >> 4);
  const int cl = c0 + 16 * wn + (lane & 15);
  // (16-B vector path: C 16-B aligned and its rows a multiple of 4 floats apart; else per element)
  if (g.cperm == TAPS && (!g.atomic || g.sk_ws) && (reinterpret_cast<uintptr_t>(g.c) & 15) == 0 && (g.ldc & 3) == 0) {
    // Straight into the Conv1d [Co][Ci][K] layout: the tile's (32 channels x 5 taps) of a row are
    // ONE contiguous 640-B run there, so each 64-row half is staged through LDS ([64][CPW] floats)
    // and stored as 16-B row chunks (per-element stores 20 B apart had cost more than the
    // separate unpack pass they replace)
    constexpr int CPW = CW * TAPS + 4;  // 164: 16-B rows, row groups 4 apart land 16 banks apart
    float* st = reinterpret_cast<float*>(smem_raw);
    const int lc = (16 * wn + (lane & 15)) * TAPS;
#pragma unroll
    for (int ph = 0; ph < 2; ++ph) {
      __syncthreads();  // the K loop's last fragment reads / the previous half's row reads are done
      if (wm == ph) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int k = 0; k < TAPS; ++k) st[(i * 16 + 4 * (lane >> 4) + e) * CPW + lc + k] = acc[i][k][e];
      }
      __syncthreads();
      constexpr int C4 = CW * TAPS / 4;  // 40 16-B chunks per row
      for (int q = tid; q < 64 * C4; q += 256) {
        const int r = q / C4, c4 = q - r * C4;
        const int row = m0 + ph * 64 + r;
        if (row >= g.M) continue;
        f32x4 v = *reinterpret_cast<const f32x4*>(st + r * CPW + 4 * c4);
        f32x4* cp = reinterpret_cast<f32x4*>(g.c + (long long)row * g.ldc + (long long)c0 * TAPS + 4 * c4);
        if (g.accumulate) v += *cp;
        *cp = v;
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = rbase + i * 16 + e;
      if (row >= g.M) continue;
#pragma unroll
      for (int k = 0; k < TAPS; ++k) {
        float* cp = g.c + (long long)row * g.ldc + (g.cperm ? (long long)cl * TAPS + k : (long long)k * chans + cl);
        const float v = acc[i][k][e];
        if (g.atomic && !g.sk_ws) atomicAdd(cp, v);
        else *cp = g.accumulate ? *cp + v : v;
      }
    }
}

template <int NST>
void launch_halo(const GemmArgs& g, hipStream_t s) {
  const size_t lds = NST * (size_t)HSTAGE;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_tt_halo_kernel<NST>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  const int nb = ((g.M + BM - 1) / BM) * (g.b.chans / 32) * g.split_k;
  gemm_tt_halo_kernel<NST><<<nb, 256, lds, s>>>(g);
}

}  // namespace

float* gemm_splitk_ws(size_t bytes, hipStream_t s) {
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, std::pair<float*, size_t>> ws;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess || hipStreamIsCapturing(s, &st) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(mu);
  auto& e = ws[{dev, s}];
  if (e.second >= bytes) return e.first;
  if (st != hipStreamCaptureStatusNone) return nullptr;  // no allocation inside a capture
  // grow: the old buffer may still be read by this stream's queued kernels, so it is kept (a
  // stream grows a few times per process: the largest weight gradient it runs)
  float* p = nullptr;
  const size_t want = std::max(bytes, (size_t)32 << 20);
  if (hipMalloc(&p, want) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  e = {p, want};
  return p;
}

bool gemm_tt_launch(const GemmArgs& g0, hipStream_t s) {
  // AVC_TT_SPLITK=n: split-K reduced without atomics up to n splits (default 8); 0 = every split-K
  // product by atomics into the zeroed C (the pre-round-5 form)
  static const int fix_max = [] {
    const char* e = getenv("AVC_TT_SPLITK");
    return e ? atoi(e) : 8;
  }();
  const bool fix_on = fix_max > 1;
  GemmArgs ga = g0;
  const GemmArgs& g = ga;
  // the split-K reduction without atomics: `tiles` output tiles of `tile_bytes` each
  auto fixup = [&](int tiles, size_t tile_bytes) {
    // the last split's reduction takes ~one memory round trip per split: past SK_MAX splits the
    // atomics win (AVC_TT_SPLITK=n sets the bound; tools/tt_bench.py)
    if (!fix_on || g.split_k <= 1 || g.split_k > fix_max || g.batch != 1 || !g.c || g.bias || g.res ||
        g.bn_partial || g.rbias)
      return;
    const size_t bytes = (size_t)tiles * g.split_k * tile_bytes;
    if (bytes > ((size_t)1 << 30)) return;
    float* w = gemm_splitk_ws(bytes, s);
    unsigned* c = w ? avc_counter_slots(tiles, s) : nullptr;
    if (!c) return;
    ga.sk_ws = w;
    ga.sk_cnt = c;
    ga.zero_c = 0;
  };
  if (g.klen % FBK || g.M % 8 || g.N % 8) return false;
  for (const OpDev* o : {&g.a, &g.b})
    if (o->dtype != AVC_BF16 || !ok16(o->ptr) || o->ld % 8 || o->bstride % 8) return false;
  if (g.a.win) return false;
  if (g.b.win && g.b.chans % 8) return false;
  const OpDev& x = g.b;
  if (x.win && x.taps == 5 && x.t_in == x.t_out && 2 * x.pad == x.taps - 1 && x.chans % 32 == 0 &&
      g.K % x.t_out == 0 && g.batch == 1 && g.N == x.taps * x.chans && !g.res && !g.c16 && !g.bias && !g.bn_partial) {
    fixup(((g.M + BM - 1) / BM) * (x.chans / 32), (size_t)BM * 32 * x.taps * 4);
    gemm_zero_c(ga, s);
    launch_halo<2>(g, s);  // two LDS stages (three measured no faster)
    return true;
  }
  fixup(((g.M + BM - 1) / BM) * ((g.N + 127) / 128), (size_t)BM * 128 * 4);
  gemm_zero_c(ga, s);
  const int nb = ((g.M + BM - 1) / BM) * ((g.N + 127) / 128) * g.batch * g.split_k;
  if (g.b.win) launch<true>(g, nb, s);
  else launch<false>(g, nb, s);
  return true;
}

}  // namespace avcg
