// gemm_nt.hip — bf16 "NT" GEMM (both operands K-contiguous) fed by LDS DMA.
//
// C[M][N] = A[M][K] . B[N][K]^T, fp32 accumulate, with the frame-window A operand of the conv
// path (im2col addressing: row -> (utterance, frame), K -> (tap, channel), zero outside the
// utterance) and the shared fused epilogue (gemm_internal.h).  Serves the Conv1d forward and
// data-gradient GEMMs and the LSTM input projections (factory/Norm.py:21-28,
// AutoVC.py:43,77,96) once their operands are bf16.
//
// Structure (cdna_hip_programming.md §5): 128 x BN_ tile, BK = 64, 4 waves as 2x2, each wave
// 64 x BN_/2 of 16x16x32 MFMAs.  Operands go global -> LDS with global_load_lds_dwordx4
// (16 B per lane, no register staging), NST LDS stages, NST-1 tiles in flight: a counted
// `s_waitcnt vmcnt` + raw s_barrier per K-tile, never vmcnt(0) inside the loop.  LDS rows
// are 128 B, XOR-swizzled by 16-B chunk (chunk ^= (row >> 1) & 7) on the SOURCE address so
// the ds_read_b128 fragment reads are bank-conflict free.  Padding / tails read a 16-B
// zero granule instead of branching.
#include "gemm_internal.h"

namespace avcg {
namespace {

__device__ __attribute__((aligned(16))) unsigned int g_zero16[4] = {0u, 0u, 0u, 0u};

constexpr int ROWB = FBK * 2;  // 128-byte LDS rows

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

// One operand's tile loader: R rows x 64 K per stage = R/32 glds per thread.  Instruction i
// of wave w covers tile rows (4i + w)*8 .. +8; lane L writes row +(L>>3), 16-B slot L&7,
// which holds global K-chunk (L&7) ^ swz(row) — swz(row) = (row>>1)&7 = (4*(w&1) + (L>>4))&7
// for every i, so each lane has one fixed chunk.
template <int R, bool WIN>
struct NtLoader {
  static constexpr int NI = R / 32;
  const bf16* base;
  long long roff[NI];  // element offset of the row (non-window) / of the row's frame (window)
  int tt[NI];          // window: frame within the utterance
  int rok[NI];
  int kc;              // this lane's K offset inside the 64-wide tile
  int ld, pad, t_in, chans;

  __device__ __forceinline__ void init(const OpDev& o, int row0, int bz) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    base = reinterpret_cast<const bf16*>(o.ptr) + (long long)bz * o.bstride;
    kc = 8 * ((lane & 7) ^ ((4 * (w & 1) + (lane >> 4)) & 7));
    ld = (int)o.ld;
    pad = o.pad;
    t_in = o.t_in;
    chans = o.chans;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int r = row0 + (4 * i + w) * 8 + (lane >> 3);
      rok[i] = r < o.rows;
      const int rr = rok[i] ? r : 0;
      if (WIN) {
        const int b = (int)fdiv((uint32_t)rr, o.tdiv);
        tt[i] = rr - b * o.t_out;
        roff[i] = (long long)(b * o.t_in + tt[i]) * o.ld;
      } else {
        tt[i] = 0;
        roff[i] = (long long)rr * o.ld;
      }
    }
  }

  // issue the R/32 glds of K-tile starting at kbase into the stage's LDS image
  __device__ __forceinline__ void issue(char* lds_tile, int kbase, int kend, const FastDiv& cdv) {
    const int w = threadIdx.x >> 6;
    const int k = kbase + kc;
    const bool kok = k < kend;
    int tap = 0, cc = k;
    if (WIN) {
      tap = (int)fdiv((uint32_t)k, cdv);
      cc = k - tap * chans;
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      bool ok = kok && rok[i];
      long long off;
      if (WIN) {
        const int t2 = tt[i] + tap - pad;
        ok = ok && t2 >= 0 && t2 < t_in;
        off = roff[i] + (long long)(tap - pad) * ld + cc;
      } else {
        off = roff[i] + k;
      }
      const void* src = ok ? (const void*)(base + off) : (const void*)g_zero16;
      glds16(src, lds_tile + (4 * i + w) * 8 * ROWB);
    }
  }
};

// BNB: the BatchNorm-backward epilogue compiled in (only for launches with bnb)
template <int BN_, int NST, bool WIN, bool BNB>
__global__ void __launch_bounds__(256, 1) gemm_nt_kernel(GemmArgs g) {
  constexpr int NJ = BN_ / 32, WN = BN_ / 2;
  constexpr int A_BYTES = BM * ROWB, STAGE = (BM + BN_) * ROWB;
  constexpr int LPT = BM / 32 + BN_ / 32;  // glds per thread per K-tile
  constexpr int P = NST - 1;               // tiles in flight
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  // XCD-aware bijective remap (as gemm_fast_kernel)
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

  NtLoader<BM, WIN> la;
  NtLoader<BN_, false> lb;
  la.init(g.a, m0, bz);
  lb.init(g.b, n0, bz);
  const FastDiv cdv = g.a.cdv;

  f32x4 acc[4][NJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment addresses: row (lane&15) of each 16-row block, logical chunk (kk/8 + lane/16)
  // stored at chunk ^ ((row>>1)&7) = chunk ^ ((lane&15)>>1)
  const int frow = lane & 15, sw = frow >> 1;
  const int ch0 = ((lane >> 4) ^ sw) << 4, ch1 = ((4 + (lane >> 4)) ^ sw) << 4;
  const int aoff = (wm * 64 + frow) * ROWB, boff = A_BYTES + (wn * WN + frow) * ROWB;

#pragma unroll
  for (int p = 0; p < P; ++p)
    if (p < nkt) {
      char* st = smem_raw + p * STAGE;
      la.issue(st, kbeg + p * FBK, kend, cdv);
      lb.issue(st + A_BYTES, kbeg + p * FBK, kend, cdv);
    }

  for (int kt = 0; kt < nkt; ++kt) {
    const int ahead = min(P - 1, nkt - 1 - kt);  // tiles allowed to stay in flight
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
    if (kt + P < nkt) {
      char* st = smem_raw + ((kt + P) % NST) * STAGE;
      la.issue(st, kbeg + (kt + P) * FBK, kend, cdv);
      lb.issue(st + A_BYTES, kbeg + (kt + P) * FBK, kend, cdv);
    }
    const char* st = smem_raw + (kt % NST) * STAGE;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int co = h ? ch1 : ch0;
      bf16x8 af[4], bfr[NJ];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const bf16x8*>(st + aoff + i * 16 * ROWB + co);
#pragma unroll
      for (int j = 0; j < NJ; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(st + boff + j * 16 * ROWB + co);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }
  __syncthreads();  // every glds retired (last wait was vmcnt(0)) and every fragment read done
  fast_epilogue<BN_, BNB, true>(g, acc, m0, n0, mt, bz, ks, smem_raw);
}

template <int BN_, int NST, bool WIN, bool BNB = false>
void launch(const GemmArgs& g, int nblocks, hipStream_t s) {
  const size_t lds = (size_t)NST * (BM + BN_) * ROWB;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_nt_kernel<BN_, NST, WIN, BNB>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  gemm_nt_kernel<BN_, NST, WIN, BNB><<<nblocks, 256, lds, s>>>(g);
}

bool ok16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

bool operand_ok(const OpDev& o, bool allow_win) {
  if (o.dtype != AVC_BF16 || !ok16(o.ptr) || o.ld % 8 || o.bstride % 8) return false;
  if (o.win && (!allow_win || o.chans % 8)) return false;
  return true;
}


}  // namespace

bool gemm_nt_launch(const GemmArgs& g, hipStream_t s) {
  if (g.K % 8 || g.klen % FBK) return false;
  if (!operand_ok(g.a, true) || !operand_ok(g.b, false)) return false;
  int bn = -1, nst = 2;
  const long long t128 = (long long)((g.M + BM - 1) / BM) * ((g.N + 127) / 128) * g.batch * g.split_k;
  // measured (tools/gemm_census.py, a tile / stage sweep in round 2): more resident
  // workgroups beat deeper stages on these shapes, so 2 stages; 128-wide tiles when there are
  // >= 4 of them per CU, or for long-K wide products (8192x1024x4096: 75 vs 98 us)
  if (bn != 64 && bn != 128) bn = (g.N > 64 && (t128 >= 1024 || (g.N >= 1024 && g.K >= 2048))) ? 128 : 64;
  if (nst < 2 || nst > 4) nst = 2;
  const int nb = ((g.M + BM - 1) / BM) * ((g.N + bn - 1) / bn) * g.batch * g.split_k;
  const bool win = g.a.win != 0;
  if (g.bnb_ws) {  // BN-backward epilogue: two-stage instances only
    if (bn == 128) {
      if (win) launch<128, 2, true, true>(g, nb, s);
      else launch<128, 2, false, true>(g, nb, s);
    } else {
      if (win) launch<64, 2, true, true>(g, nb, s);
      else launch<64, 2, false, true>(g, nb, s);
    }
    return true;
  }
#define NT_CASE(BNV, NSV)                                   \
  if (bn == BNV && nst == NSV) {                            \
    if (win) launch<BNV, NSV, true>(g, nb, s);              \
    else launch<BNV, NSV, false>(g, nb, s);                 \
    return true;                                            \
  }
  NT_CASE(128, 2) NT_CASE(128, 3) NT_CASE(128, 4) NT_CASE(64, 2) NT_CASE(64, 3) NT_CASE(64, 4)
#undef NT_CASE
  return false;
}

}  // namespace avcg
