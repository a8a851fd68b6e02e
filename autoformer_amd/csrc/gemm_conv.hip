// gemm_conv.hip — Conv1d (stride 1, 'same' padding) as an implicit GEMM that stages each
// input tile ONCE for all taps.
//
// C[m][n] = sum_{tap, c} X[frame(m) + tap - pad][c] . W[n][tap*C + c]: the Conv1d forward
// (X = activation, W = Wf[co][tap][ci]) and data gradient (X = dy, W = Wd[ci][tap'][co],
// flipped taps) of factory/Norm.py:21-28 (ConvNorm), i.e. every 512-channel convolution of the
// AutoVC encoder / decoder / postnet (AutoVC.py:21-179) and the MetaConv blocks.
//
// gemm_nt streams the im2col window: K runs over (tap, channel) and the same input rows are
// fetched again for every tap.  Here a stage covers CBK = 32 channels of ALL taps: the
// 128-frame tile plus its taps-1 halo rows (132 rows x 64 B) is copied to LDS once, the five
// weight slices (5 x 64 rows x 64 B) beside it, and tap k reads the halo shifted by k rows.
// Bytes per stage per MFMA drop by 2.1x against the window stream, which is what bounds these
// shapes (one or two 128-row tiles per CU, LDS-DMA latency ~1.1 us per fill).  Rows whose
// shifted frame leaves the utterance read zeros (a per-lane, per-tap predicate on the A
// fragment: a halo row can be valid for one output row and padding for another when a tile
// spans two utterances).
//
// 128 x 64 tile, 4 waves (2 x 2, each 64 x 32), 16x16x32 bf16 MFMA, two LDS stages of 32 KiB
// so two workgroups share a CU (measured on the AutoVC convs: 33 us per 8192x512x2560 conv vs
// 50 us with four stages at one workgroup per CU, 40 us for the window stream), global_load_lds_dwordx4 (16 B per lane, no register staging) into
// 64-B rows XOR-swizzled by 16-B chunk (chunk ^ ((row >> 1) & 3), applied on the source
// address), counted vmcnt + raw barrier, shared fused epilogue (gemm_internal.h: bias, BN
// partial statistics, bf16 twin, accumulate, residual).
#include "gemm_internal.h"

namespace avcg {
namespace {

__device__ __attribute__((aligned(16))) unsigned int g_zero16_cv[4] = {0u, 0u, 0u, 0u};

constexpr int CBK = 32;                 // channels per stage
constexpr int CROW = CBK * 2;           // 64-B LDS rows
constexpr int CBN = 64;                 // output columns per tile
constexpr int AROWS = 192;              // halo rows reserved per stage: 3 glds per thread
constexpr int CA_BYTES = AROWS * CROW;  // 12 KiB

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef const __attribute__((address_space(1))) void* gbl_ptr_t;

__device__ __forceinline__ void glds16(const void* src, char* lds) {
  __builtin_amdgcn_global_load_lds((gbl_ptr_t)src, (lds_ptr_t)lds, 16, 0, 0);
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void raw_barrier() { asm volatile("s_barrier" ::: "memory"); }

__device__ __forceinline__ int cswz(int row) { return (row >> 1) & 3; }

template <int TAPS>
struct ConvCfg {
  static constexpr int B_BYTES = TAPS * CBN * CROW;
  static constexpr int STAGE = CA_BYTES + B_BYTES;
  static constexpr int BI = TAPS * CBN / 16 / 4;  // weight glds per thread per stage
  static constexpr int LPT = 3 + BI;              // glds per thread per stage
  static_assert(TAPS * CBN % 64 == 0, "weight rows must split over four waves");
  static_assert(BM + TAPS - 1 <= AROWS, "halo does not fit");
};

template <int TAPS, int CNST>
__global__ void __launch_bounds__(256, 2) gemm_conv_kernel(GemmArgs g) {
  using Cfg = ConvCfg<TAPS>;
  constexpr int STAGE = Cfg::STAGE, LPT = Cfg::LPT, BI = Cfg::BI, P = CNST - 1;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  // XCD-aware bijective remap (as gemm_nt_kernel)
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q = nwg >> 3, rr = nwg & 7, xcd = bid & 7;
  const int lid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
  const int nN = (g.N + CBN - 1) / CBN;
  const int mt = lid / nN, nt = lid - mt * nN;
  const int m0 = mt * BM, n0 = nt * CBN;

  const OpDev& A = g.a;
  const OpDev& Bo = g.b;
  const bf16* xa = reinterpret_cast<const bf16*>(A.ptr);
  const bf16* wb = reinterpret_cast<const bf16*>(Bo.ptr);
  const int pad = A.pad, T = A.t_out, chans = A.chans;
  const long long lda = A.ld, ldb = Bo.ld;
  const int nst = chans / CBK;

  // ---- loader: halo row hr = 16*(3*wid + i) + (lane >> 2), slot lane & 3
  long long aoff[3];
  bool aok[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int hr = 16 * (3 * wid + i) + (lane >> 2);
    const int f = m0 - pad + hr;
    aok[i] = hr < BM + TAPS - 1 && f >= 0 && f < g.M;
    aoff[i] = (long long)(aok[i] ? f : 0) * lda + 8 * ((lane & 3) ^ cswz(hr));
  }
  // weight row wr = 16*((wid*BI + i) % 4) + (lane >> 2) of tap (wid*BI + i) / 4
  long long boff[BI];
  bool bok[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int ins = wid * BI + i, tap = ins >> 2, wr = 16 * (ins & 3) + (lane >> 2);
    const int n = n0 + wr;
    bok[i] = n < g.N;
    boff[i] = (long long)(bok[i] ? n : 0) * ldb + (long long)tap * chans + 8 * ((lane & 3) ^ cswz(wr));
  }
  auto issue = [&](int st, int cs) {
    char* base = smem_raw + st * STAGE;
    const int c0 = cs * CBK;
#pragma unroll
    for (int i = 0; i < 3; ++i)
      glds16(aok[i] ? (const void*)(xa + aoff[i] + c0) : (const void*)g_zero16_cv, base + (3 * wid + i) * 1024);
#pragma unroll
    for (int i = 0; i < BI; ++i)
      glds16(bok[i] ? (const void*)(wb + boff[i] + c0) : (const void*)g_zero16_cv,
             base + CA_BYTES + (wid * BI + i) * 1024);
  };

  // ---- fragment addressing and the per-tap validity of this lane's four A rows
  const int fr = lane & 15, ch = lane >> 4;
  int arow[4];
  unsigned vmask = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    arow[i] = wm * 64 + i * 16 + fr;
    const int m = min(m0 + arow[i], g.M - 1);
    const int b = (int)fdiv((uint32_t)m, A.tdiv);
    const int t = m - b * T;
#pragma unroll
    for (int k = 0; k < TAPS; ++k) {
      const int t2 = t + k - pad;
      if (t2 >= 0 && t2 < T) vmask |= 1u << (i * 8 + k);
    }
  }
  int bfo[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int r = wn * 32 + j * 16 + fr;
    bfo[j] = CA_BYTES + r * CROW + 16 * (ch ^ cswz(r));
  }

  f32x4 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int p = 0; p < P; ++p)
    if (p < nst) issue(p, p);

  for (int cs = 0; cs < nst; ++cs) {
    const int ahead = min(P - 1, nst - 1 - cs);
    if constexpr (P >= 3) {
      if (ahead >= 2) wait_vm<2 * LPT>();
      else if (ahead == 1) wait_vm<LPT>();
      else wait_vm<0>();
    } else if constexpr (P == 2) {
      if (ahead >= 1) wait_vm<LPT>();
      else wait_vm<0>();
    } else {
      wait_vm<0>();
    }
    raw_barrier();
    if (cs + P < nst) issue((cs + P) % CNST, cs + P);
    const char* st = smem_raw + (cs % CNST) * STAGE;
#pragma unroll
    for (int k = 0; k < TAPS; ++k) {
      bf16x8 af[4], bfr[2];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = arow[i] + k;
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(st + r * CROW + 16 * (ch ^ cswz(r)));
        af[i] = ((vmask >> (i * 8 + k)) & 1u) ? v : bf16x8{};
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(st + k * CBN * CROW + bfo[j]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }
  __syncthreads();  // last wait was vmcnt(0); every fragment read done before the epilogue reuses LDS
  fast_epilogue<CBN>(g, acc, m0, n0, mt, 0, 0, smem_raw);
}

template <int TAPS, int CNST>
void launch(const GemmArgs& g, int nblocks, hipStream_t s) {
  const size_t lds = (size_t)CNST * ConvCfg<TAPS>::STAGE;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_conv_kernel<TAPS, CNST>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  gemm_conv_kernel<TAPS, CNST><<<nblocks, 256, lds, s>>>(g);
}

bool ok16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

bool gemm_conv_launch(const GemmArgs& g, hipStream_t s) {
  // AVC_CONV_HALO: 0 = off (window stream through gemm_nt), 2 / 3 / 4 = LDS stages
  static const int mode = getenv("AVC_CONV_HALO") ? atoi(getenv("AVC_CONV_HALO")) : 2;
  if (!mode) return false;
  const OpDev& a = g.a;
  const OpDev& b = g.b;
  if (!a.win || a.taps != 5 || a.t_in != a.t_out || 2 * a.pad != a.taps - 1) return false;
  if (a.chans % CBK || g.K != a.taps * a.chans || g.batch != 1 || g.split_k != 1) return false;
  if (a.dtype != AVC_BF16 || b.dtype != AVC_BF16 || b.win) return false;
  if (!ok16(a.ptr) || !ok16(b.ptr) || a.ld % 8 || b.ld % 8) return false;
  const int nb = ((g.M + BM - 1) / BM) * ((g.N + CBN - 1) / CBN);
  if (mode == 3) launch<5, 3>(g, nb, s);
  else if (mode == 4) launch<5, 4>(g, nb, s);
  else launch<5, 2>(g, nb, s);
  return true;
}

}  // namespace avcg
