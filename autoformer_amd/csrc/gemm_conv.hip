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

// CBK channels per stage (LDS rows of 2*CBK bytes), CBN output columns per tile, 128-row tiles,
// 4 waves (2 along M, 2 along N).  Every wave issues the same number of glds per
// stage (the counted vmcnt waits assume it), so the halo and weight instruction counts are
// rounded up to a multiple of the wave count; the extra rows load zeros.
template <int TAPS, int CBK, int CBN>
struct ConvCfg {
  static constexpr int NW = 4;                    // waves per workgroup
  static constexpr int TM = 128;                  // tile rows
  static constexpr int ROW = 2 * CBK;             // bytes per LDS row
  static constexpr int CPR = ROW / 16;            // 16-B chunks per row
  static constexpr int RPI = 1024 / ROW;          // rows per glds wave-instruction
  static constexpr int AI = ((TM + TAPS - 1 + RPI - 1) / RPI + NW - 1) / NW * NW;  // halo instructions
  static constexpr int A_BYTES = AI * 1024;
  static constexpr int BROWS = TAPS * CBN;        // weight rows actually used
  static constexpr int BI = ((BROWS + RPI - 1) / RPI + NW - 1) / NW * NW;           // weight instructions
  static constexpr int B_BYTES = BI * 1024;
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int LPT = AI / NW + BI / NW;   // glds per thread per stage
  static constexpr int NJ = CBN / 32;
  static_assert(CBN % 32 == 0 && (CBK == 32 || CBK == 64), "tile shape");
  // slot of chunk c in row r (XOR swizzle on the 16-B chunk index)
  __device__ static __forceinline__ int swz(int r) { return (r >> 1) & (CPR - 1); }
};

// BNB: the BatchNorm-backward epilogue compiled in (only the instances launched with bnb: its
// code in every conv instance cost 20 % of the conv time, measured)
template <int TAPS, int NST, int CBK, int CBN, bool BNB>
__global__ void __launch_bounds__(256, 2) gemm_conv_kernel(GemmArgs g) {
  using C = ConvCfg<TAPS, CBK, CBN>;
  constexpr int NW = C::NW, TM = C::TM;
  constexpr int STAGE = C::STAGE, LPT = C::LPT, AI4 = C::AI / NW, BI4 = C::BI / NW, P = NST - 1;
  constexpr int ROW = C::ROW, CPR = C::CPR, RPI = C::RPI, NJ = C::NJ, KB = CBK / 32;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  // XCD-aware bijective remap (as gemm_nt_kernel)
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q = nwg >> 3, rr = nwg & 7, xcd = bid & 7;
  const int lid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
  const int nN = (g.N + CBN - 1) / CBN;
  const int mt = lid / nN, nt = lid - mt * nN;
  const int m0 = mt * TM, n0 = nt * CBN;

  const OpDev& A = g.a;
  const OpDev& Bo = g.b;
  const bf16* xa = reinterpret_cast<const bf16*>(A.ptr);
  const bf16* wb = reinterpret_cast<const bf16*>(Bo.ptr);
  const int pad = A.pad, T = A.t_out, chans = A.chans;
  const long long lda = A.ld, ldb = Bo.ld;
  const int nst = chans / CBK;

  // ---- loader: instruction ins writes LDS [ins*1KiB, +1KiB) = rows RPI*ins + lane / CPR,
  // slot lane % CPR, which holds global chunk slot ^ swz(row)
  const int lrow = lane / CPR, lslot = lane % CPR;
  long long aoff[AI4];
  bool aok[AI4];
#pragma unroll
  for (int i = 0; i < AI4; ++i) {
    const int hr = RPI * (AI4 * wid + i) + lrow;
    const int f = m0 - pad + hr;
    aok[i] = hr < TM + TAPS - 1 && f >= 0 && f < g.M;
    aoff[i] = (long long)(aok[i] ? f : 0) * lda + 8 * (lslot ^ C::swz(hr));
  }
  long long boff[BI4];
  bool bok[BI4];
#pragma unroll
  for (int i = 0; i < BI4; ++i) {
    const int ins = wid * BI4 + i, wr = RPI * ins + lrow, tap = wr / CBN, n = n0 + (wr - tap * CBN);
    bok[i] = n < g.N && wr < C::BROWS;
    boff[i] = (long long)(bok[i] ? n : 0) * ldb + (long long)tap * chans + 8 * (lslot ^ C::swz(wr));
  }
  auto issue = [&](int st, int cs) {
    char* base = smem_raw + st * STAGE;
    const int c0 = cs * CBK;
#pragma unroll
    for (int i = 0; i < AI4; ++i)
      glds16(aok[i] ? (const void*)(xa + aoff[i] + c0) : (const void*)g_zero16_cv, base + (AI4 * wid + i) * 1024);
#pragma unroll
    for (int i = 0; i < BI4; ++i)
      glds16(bok[i] ? (const void*)(wb + boff[i] + c0) : (const void*)g_zero16_cv,
             base + C::A_BYTES + (wid * BI4 + i) * 1024);
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
  int brow[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) brow[j] = wn * (CBN / 2) + j * 16 + fr;

  f32x4 acc[4][NJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

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
    if (cs + P < nst) issue((cs + P) % NST, cs + P);
    const char* st = smem_raw + (cs % NST) * STAGE;
    // fragments of tap k+1 are read while tap k's MFMAs run (two register sets), so the LDS
    // latency is exposed once per stage rather than once per tap
    bf16x8 af[2][4], bfr[2][NJ];
    auto read_tap = [&](int k, int kb, int slot) {
      const int cc = 4 * kb + ch;  // this lane's 16-B chunk of K block kb
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = arow[i] + k;
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(st + r * ROW + 16 * (cc ^ C::swz(r)));
        af[slot][i] = ((vmask >> (i * 8 + k)) & 1u) ? v : bf16x8{};
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int r = k * CBN + brow[j];
        bfr[slot][j] = *reinterpret_cast<const bf16x8*>(st + C::A_BYTES + r * ROW + 16 * (cc ^ C::swz(r)));
      }
    };
    read_tap(0, 0, 0);
#pragma unroll
    for (int kk = 0; kk < TAPS * KB; ++kk) {
      const int slot = kk & 1;
      if (kk + 1 < TAPS * KB) read_tap((kk + 1) / KB, (kk + 1) % KB, slot ^ 1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[slot][i], bfr[slot][j], acc[i][j], 0, 0, 0);
    }
  }
  __syncthreads();  // last wait was vmcnt(0); every fragment read done before the epilogue reuses LDS
  fast_epilogue<CBN, BNB, true>(g, acc, m0, n0, mt, 0, 0, smem_raw);
}

template <int NST, int CBK, int CBN, bool BNB = false>
void launch(const GemmArgs& g, hipStream_t s) {
  using C = ConvCfg<5, CBK, CBN>;
  const size_t lds = (size_t)NST * C::STAGE;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_conv_kernel<5, NST, CBK, CBN, BNB>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  const int nb = ((g.M + C::TM - 1) / C::TM) * ((g.N + CBN - 1) / CBN);
  gemm_conv_kernel<5, NST, CBK, CBN, BNB><<<nb, 64 * C::NW, lds, s>>>(g);
}

bool ok16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

bool gemm_conv_launch(const GemmArgs& g, hipStream_t s) {
  // stages, channels, columns -- measured (tools/gemm_census.py, a stage / channel / column sweep in
  // round 2): two 32-KiB stages, 32 channels, 64 columns -- two workgroups per CU -- beat 64-channel
  // stages (44-47 us) and three or four stages at one workgroup per CU (50-69 us) on 8192x512x2560
  static const int cfg[3] = {2, 32, 64};
  const OpDev& a = g.a;
  const OpDev& b = g.b;
  if (!a.win || a.taps != 5 || a.t_in != a.t_out || 2 * a.pad != a.taps - 1) return false;
  if (g.K != a.taps * a.chans || g.batch != 1 || g.split_k != 1) return false;
  if (a.dtype != AVC_BF16 || b.dtype != AVC_BF16 || b.win) return false;
  if (!ok16(a.ptr) || !ok16(b.ptr) || a.ld % 8 || b.ld % 8) return false;
  int ns = cfg[0], bk = cfg[1], bn = cfg[2];
  if (a.chans % bk) bk = 32;  // 32-channel stages for channel counts that are not 64-multiples
  if (a.chans % bk) return false;
  if (bk == 32 && bn == 32) bn = 64;
  if (g.bnb_ws) {  // the BN-backward epilogue is instantiated for the default configuration only
    if (bk != 32) return false;
    launch<2, 32, 64, true>(g, s);
    return true;
  }
  // (round 3 measured 256-row tiles of this kernel -- eight waves, one workgroup per CU, three
  // 48-KiB stages -- no faster, profiles/r3_conv_tile_ab.txt; round 4 removed that form: the
  // eight-wave halo conv is gemm_ring.hip's conv_ring_kernel)
#define CONV_CASE(NS, BK, BN)                  \
  if (ns == NS && bk == BK && bn == BN) {      \
    launch<NS, BK, BN>(g, s);                  \
    return true;                               \
  }
  CONV_CASE(2, 32, 64) CONV_CASE(3, 32, 64) CONV_CASE(4, 32, 64) CONV_CASE(2, 64, 32) CONV_CASE(3, 64, 32)
  CONV_CASE(2, 64, 64)
#undef CONV_CASE
  if (bk == 32) {
    launch<2, 32, 64>(g, s);
    return true;
  }
  return false;
}

}  // namespace avcg
