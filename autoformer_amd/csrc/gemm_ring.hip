// gemm_ring.hip — bf16 NT GEMM with a deep LDS-DMA ring, eight waves, one workgroup per CU.
//
// C[M][N] = A[M][K] . B[N][K]^T (fp32 accumulate) for the products whose operands are both
// K-contiguous: the MetaConv MLP-Mixer token / channel mixing (factory/MLPMixer.py:58-92,
// factory/MetaConv.py:23-76), the decoder LSTM input projections and data gradients
// (factory/AutoVC.py:96,103,110), and the Conv1d window stream (factory/Norm.py:21-28: A is the
// frame window of the conv input, K = tap x channel, zero outside the utterance).
//
// Why a new kernel: the 4-wave, two-stage kernels of gemm_nt.hip /
// gemm_conv.hip keep ONE LDS-DMA fill in flight per workgroup and two workgroups per CU; their
// times match the ≈25 GB/s-per-CU fill rate of that regime (MI355X_MICROARCH.md
// "ldsdma-fill"), not the MFMA rate.  Here:
//   * one 512-thread workgroup per CU, 8 waves as 2 (M) x 4 (N), so every SIMD holds two waves
//     that cover each other's LDS-read latency (MI355X_MICROARCH.md "Two waves per SIMD");
//   * a ring of NST K-steps (BK = 64, 128-B LDS rows) with NST-1 K-steps of fills in flight
//     ACROSS the barrier: a counted `s_waitcnt vmcnt` + raw `s_barrier` per K-step, never
//     vmcnt(0) inside the loop (cdna_hip_programming.md §5 "Pipelining across barriers");
//     every wave issues the same number of `global_load_lds_dwordx4` per K-step (the counts
//     assume it), rows beyond the operand read a 16-B zero granule;
//   * 128 x 128 (4 slots, 3 in flight), 256 x 128 (3 slots) or 256 x 256 tiles (2 slots; half
//     the operand bytes per FLOP of a 128 x 128 tile);
//   * XOR-swizzled 16-B chunks (chunk ^ ((row >> 1) & 7), applied on the SOURCE address, the
//     LDS image stays lane-linear), conflict-free ds_read_b128 fragment reads;
//   * XCD-aware bijective block remap, then grouped tile order (GM row tiles per group) so the
//     workgroups an XCD runs together share A row panels and B column panels in its L2;
//   * all LDS in ONE __shared__ array (a second __shared__ object can make hipcc drain vmcnt
//     before every K-step's first ds_read: cdna_hip_programming.md §5 item 4(a)); the
//     last-arriver flag of the BN finalize lives in that array too.
// Epilogue: bias, conv0-fold row bias, residual, accumulate / split-K atomics, fp32 C and / or
// bf16 twin, conv weight-layout permutation, BatchNorm partial statistics per 128-row tile and
// the finalize by the last-arriving row tile (the semantics of gemm_internal.h:fast_epilogue).
#include <algorithm>
#include <type_traits>

#include "gemm_internal.h"

namespace avcg {
namespace {

__device__ __attribute__((aligned(16))) unsigned int g_zero16_rg[4] = {0u, 0u, 0u, 0u};

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef const __attribute__((address_space(1))) void* gbl_ptr_t;

constexpr int RROW = 128;  // bytes per LDS row (64 bf16 of K)
constexpr int RBK = 64;    // K per ring slot
constexpr int RNT = 512;   // threads per workgroup

__device__ __forceinline__ void glds16(const void* src, char* lds) {
  __builtin_amdgcn_global_load_lds((gbl_ptr_t)src, (lds_ptr_t)lds, 16, 0, 0);
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void raw_barrier() { asm volatile("s_barrier" ::: "memory"); }

// LDS byte address of a pointer into the kernel's dynamic LDS array
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
// 16-B fragment read issued as inline asm: hipcc's waitcnt pass does not track it, so the caller
// places counted `s_waitcnt lgkmcnt` (+ sched_barrier, cdna_hip_programming.md §5.4 rule 18)
template <int OFF>
__device__ __forceinline__ bf16x8 ds_read16(unsigned addr) {
  u32x4 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF) : "memory");
  return __builtin_bit_cast(bf16x8, v);
}
// N reads at BASE, BASE + STRIDE, ... bytes from addr into d[0..N)
template <int N, int STRIDE, int BASE = 0>
__device__ __forceinline__ void ds_read_n(bf16x8* d, unsigned addr) {
  if constexpr (N > 0) {
    d[0] = ds_read16<BASE>(addr);
    ds_read_n<N - 1, STRIDE, BASE + STRIDE>(d + 1, addr);
  }
}
template <int N>
__device__ __forceinline__ void wait_lgkm() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// R rows x 64 K of one operand per slot: R/64 glds per thread.  Instruction i of wave w covers
// slot rows (8i + w)*8 .. +8; lane L writes row +(L>>3), 16-B slot L&7, which holds global K
// chunk (L&7) ^ ((row>>1)&7) = (L&7) ^ ((4*(w&1) + (L>>4)) & 7) for every i.
template <int R, bool WIN>
struct RingLoader {
  static constexpr int NI = R / 64;
  const bf16* base;
  long long roff[NI];  // element offset of the row (plain) / of the row's frame (window)
  int tt[NI];          // window: frame within the utterance
  bool rok[NI];
  int kc;              // this lane's K offset inside the 64-wide slot
  int ld, pad, t_in, chans;
  const void* zp;      // the 16-B zero granule, held in VGPRs (see init)

  __device__ __forceinline__ void init(const OpDev& o, int row0, int bz) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    base = reinterpret_cast<const bf16*>(o.ptr) + (long long)bz * o.bstride;
    // the zero granule's address pinned in a VGPR pair once: referenced per glds, hipcc had
    // re-materialised it from the GOT (s_getpc + s_load + lgkmcnt(0)) before every fill under
    // SGPR pressure
    zp = (const void*)g_zero16_rg;
    asm volatile("" : "+v"(zp));
    kc = 8 * ((lane & 7) ^ ((4 * (w & 1) + (lane >> 4)) & 7));
    ld = (int)o.ld;
    pad = o.pad;
    t_in = o.t_in;
    chans = o.chans;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int r = row0 + (8 * i + w) * 8 + (lane >> 3);
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

  __device__ __forceinline__ void issue(char* lds, int kbase, int kend, const FastDiv& cdv) {
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
      glds16(ok ? (const void*)(base + off) : zp, lds + (8 * i + w) * 8 * RROW);
    }
  }
};

// "last arrival" on a counter with the flag in the kernel's one LDS array (see header)
__device__ __forceinline__ bool ring_arrive_last(unsigned* cnt, unsigned arrivals, unsigned mine, unsigned* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(cnt, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool last = old + mine == arrivals;
    if (last) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = last ? 1u : 0u;
  }
  __syncthreads();
  return *flag != 0;
}

template <int BM_, int BN_>
__device__ __forceinline__ void ring_store16(f32x4 (&v)[BM_ / 32][BN_ / 64], bf16* out, long long ld, int N, int m0,
                                             int n0, int mlim, char* smem_raw) {
  constexpr int TWM = BM_ / 2, TWN = BN_ / 4, NJ = TWN / 16, RP = TWN + 4, MI = TWM / 16, NCH = (MI + 3) / 4;
  constexpr int L8 = TWN / 8, R8 = 64 / L8;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 2, wn = wid & 3;
  float* reg = reinterpret_cast<float*>(smem_raw) + wid * 64 * RP;
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    const int rlim = min(mlim, m0 + wm * TWM + min(TWM, ch * 64 + 64));
#pragma unroll
    for (int ii = 0; ii < 4; ++ii)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (ch * 4 + ii < MI) reg[(ii * 16 + 4 * (lane >> 4) + e) * RP + j * 16 + (lane & 15)] = v[ch * 4 + ii][j][e];
    __syncthreads();
#pragma unroll
    for (int it = 0; it < 64 / R8; ++it) {
      const int lr = it * R8 + lane / L8, c8 = lane % L8;
      const int row = m0 + wm * TWM + ch * 64 + lr, col = n0 + wn * TWN + 8 * c8;
      if (row >= rlim || col >= N) continue;
      const f32x4 v0 = *reinterpret_cast<const f32x4*>(reg + lr * RP + 8 * c8);
      const f32x4 v1 = *reinterpret_cast<const f32x4*>(reg + lr * RP + 8 * c8 + 4);
      bf16* o = out + (long long)row * ld + col;
      if (col + 7 < N && (ld & 7) == 0) {
        *reinterpret_cast<bf16x8*>(o) = bf16x8{(bf16)v0[0], (bf16)v0[1], (bf16)v0[2], (bf16)v0[3],
                                               (bf16)v1[0], (bf16)v1[1], (bf16)v1[2], (bf16)v1[3]};
      } else {
        for (int k = 0; k < 8 && col + k < N; ++k) o[k] = (bf16)(k < 4 ? v0[k] : v1[k - 4]);
      }
    }
    __syncthreads();
  }
}

// LDS bytes the staged stores need (ring_store_tile): per wave 64 rows x (TWN + 4) fp32
template <int BM_, int BN_>
constexpr size_t ring_epi_lds() {
  return (size_t)8 * 64 * (BN_ / 4 + 4) * 4;
}

// where a row tile's column sums go: its slot of the self-zeroing workspace, or csum itself
__device__ __forceinline__ float* csum_dst(const GemmArgs& g, int row_tile, int lim) {
  return g.csum_ws ? g.csum_ws + (long long)(row_tile % g.csum_slots) * lim : g.csum;
}

// Stores of the 2 x 4 wave layout's accumulators (wave (wm, wn) owns rows m0 + wm*TWM + i*16 +
// 4*(lane>>4) + e and columns n0 + wn*TWN + j*16 + (lane&15)): each wave stages 64-row chunks of
// its tile in its own LDS region and stores them row-contiguous, 16 B per lane (fp32 C) / 8 B
// (bf16), with the residual, accumulate and GELU epilogues applied per 4-column vector and their
// uniform conditions tested once per vector, not per element (the per-element form carried ~1,800
// uniform branches per 256 x 256 tile: 60 -> 90 us on the 8192 x 4096 x 512 projection).
// Column tails and row strides that are not 16-B multiples take the per-element path.
// Rows >= mlim are not stored (g.M, or the end of a one-utterance conv tile); a wave's rows go in
// 64-row chunks, the last one partial when TWM % 64 != 0 (the 192-row conv tile: 64 + 32).
template <int BM_, int BN_>
__device__ __forceinline__ void ring_store_tile(const GemmArgs& g, f32x4 (&acc)[BM_ / 32][BN_ / 64], int m0, int n0,
                                                int bz, int ks, char* smem_raw, int mlim) {
  constexpr int TWM = BM_ / 2, TWN = BN_ / 4, NJ = TWN / 16, RP = TWN + 4, NIT = TWN / 4;
  constexpr int MI = TWM / 16, NCH = (MI + 3) / 4;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 2, wn = wid & 3;
  float* reg = reinterpret_cast<float*>(smem_raw) + wid * 64 * RP;
  float* C = g.c ? g.c + (long long)bz * g.cbs : nullptr;
  bf16* C16 = g.c16 ? g.c16 + (long long)bz * g.cbs : nullptr;
  const float* res = (g.res && ks == 0) ? g.res + (long long)bz * g.cbs : nullptr;
  // GELU-backward input, fp32 or bf16 (avc_gemm_desc.act_grad_dtype)
  const float* agr = (g.agrad && !g.agrad16) ? static_cast<const float*>(g.agrad) + (long long)bz * g.cbs : nullptr;
  const bf16* agr16 = (g.agrad && g.agrad16) ? static_cast<const bf16*>(g.agrad) + (long long)bz * g.cbs : nullptr;
  bf16* P16 = g.c16pre ? g.c16pre + (long long)bz * g.cbs : nullptr;  // bf16 pre-activation
  const bool vec = (g.ldc & 3) == 0 && (reinterpret_cast<uintptr_t>(C) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(C16) & 7) == 0 && (reinterpret_cast<uintptr_t>(res) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(agr) & 15) == 0 && (reinterpret_cast<uintptr_t>(agr16) & 7) == 0 &&
                   (reinterpret_cast<uintptr_t>(P16) & 7) == 0;
  const bool acc_c = g.accumulate != 0, gelu16 = g.c16_act != 0;
  float* csum = g.csum;
  if (g.ctr) {
    // transposed blocks (avc_gemm_desc.c_trans_rows): a lane stores 4 consecutive ROWS of one
    // column (contiguous in C, ctr % 4 == 0), consecutive lanes consecutive row quads
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      const int rlim = min(mlim, m0 + wm * TWM + min(TWM, ch * 64 + 64));
#pragma unroll
      for (int ii = 0; ii < 4; ++ii)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (ch * 4 + ii < MI) reg[(ii * 16 + 4 * (lane >> 4) + e) * RP + j * 16 + (lane & 15)] = acc[ch * 4 + ii][j][e];
      __syncthreads();
#pragma unroll 4
      for (int it = 0; it < NIT; ++it) {
        const int q = it * 64 + lane, r4 = q & 15, cl = q >> 4;
        const int row = m0 + wm * TWM + ch * 64 + 4 * r4, col = n0 + wn * TWN + cl;
        if (row >= rlim || col >= g.N) continue;
        f32x4 v = {reg[(4 * r4) * RP + cl], reg[(4 * r4 + 1) * RP + cl], reg[(4 * r4 + 2) * RP + cl],
                   reg[(4 * r4 + 3) * RP + cl]};
        const long long o = out_off(g, row, col);
        if (res) v += *reinterpret_cast<const f32x4*>(res + o);
        if (acc_c) v += *reinterpret_cast<const f32x4*>(C + o);
        *reinterpret_cast<f32x4*>(C + o) = v;
      }
      __syncthreads();
    }
    return;
  }
  if (!C && !res && !acc_c && !agr && (g.ldc & 7) == 0 && (reinterpret_cast<uintptr_t>(C16) & 15) == 0 &&
      (reinterpret_cast<uintptr_t>(P16) & 15) == 0 && (reinterpret_cast<uintptr_t>(agr16) & 15) == 0) {
    // bf16 outputs only (the MLP-Mixer GELU forward / backward, bf16-only C): 8 columns per lane,
    // 16-B stores (8-B bf16 vectors had cost 665 -> 708 us on the 22016 x 7424 x 1856 product)
    constexpr int L8 = TWN / 8, R8 = 64 / L8;
    f32x4 cs0 = {0.f, 0.f, 0.f, 0.f}, cs1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      const int rlim = min(mlim, m0 + wm * TWM + min(TWM, ch * 64 + 64));
#pragma unroll
      for (int ii = 0; ii < 4; ++ii)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (ch * 4 + ii < MI) reg[(ii * 16 + 4 * (lane >> 4) + e) * RP + j * 16 + (lane & 15)] = acc[ch * 4 + ii][j][e];
      __syncthreads();
      // the GELU-backward input is read G4 iterations at a time by UNCONDITIONAL loads (row and
      // column clamped into the tensor: ldc == N, N % 8 == 0 on this path), so the G4 loads are in
      // flight together; a load inside the bounds branch had been waited for at the branch join,
      // one 16-B load per wave in flight at a time (+180-220 us on the 327 MB pre-activations)
      constexpr int G4 = 64 / R8 < 4 ? 64 / R8 : 4;
      for (int it0 = 0; it0 < 64 / R8; it0 += G4) {
        bf16x8 hv[G4];
        if (agr16) {
#pragma unroll
          for (int k = 0; k < G4; ++k) {
            const int r = min(m0 + wm * TWM + ch * 64 + (it0 + k) * R8 + lane / L8, g.M - 1);
            const int cc = min(n0 + wn * TWN + 8 * (lane % L8), g.N - 8);
            hv[k] = *reinterpret_cast<const bf16x8*>(agr16 + (long long)r * g.ldc + cc);
          }
        }
#pragma unroll
        for (int k4 = 0; k4 < G4; ++k4) {
          const int it = it0 + k4;
          const int lr = it * R8 + lane / L8, c8 = lane % L8;
          const int row = m0 + wm * TWM + ch * 64 + lr, col = n0 + wn * TWN + 8 * c8;
          if (row >= rlim || col >= g.N) continue;
          f32x4 v0 = *reinterpret_cast<const f32x4*>(reg + lr * RP + 8 * c8);
          f32x4 v1 = *reinterpret_cast<const f32x4*>(reg + lr * RP + 8 * c8 + 4);
          const long long o = (long long)row * g.ldc + col;
          if (col + 7 < g.N) {
            if (agr16) {
              const bf16x8 h = hv[k4];
#pragma unroll
              for (int k = 0; k < 4; ++k) {
                v0[k] *= gelu_grad_f((float)h[k]);
                v1[k] *= gelu_grad_f((float)h[4 + k]);
              }
            }
            if (csum) {
              cs0 += v0;
              cs1 += v1;
            }
            if (P16)
              *reinterpret_cast<bf16x8*>(P16 + o) = bf16x8{(bf16)v0[0], (bf16)v0[1], (bf16)v0[2], (bf16)v0[3],
                                                           (bf16)v1[0], (bf16)v1[1], (bf16)v1[2], (bf16)v1[3]};
            if (C16) {
              if (gelu16) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                  v0[k] = gelu_f(v0[k]);
                  v1[k] = gelu_f(v1[k]);
                }
              }
              *reinterpret_cast<bf16x8*>(C16 + o) = bf16x8{(bf16)v0[0], (bf16)v0[1], (bf16)v0[2], (bf16)v0[3],
                                                           (bf16)v1[0], (bf16)v1[1], (bf16)v1[2], (bf16)v1[3]};
            }
          } else {
            for (int k = 0; k < 8 && col + k < g.N; ++k) {
              float x = k < 4 ? v0[k] : v1[k - 4];
              if (agr16) x *= gelu_grad_f((float)agr16[o + k]);
              if (P16) P16[o + k] = (bf16)x;
              if (csum) {
                if (k < 4) cs0[k] += x;
                else cs1[k - 4] += x;
              }
              if (C16) C16[o + k] = (bf16)(gelu16 ? gelu_f(x) : x);
            }
          }
        }
      }
      __syncthreads();
    }
    if (csum) {
      // lanes sharing this lane's 8 columns: lane + k * L8
#pragma unroll
      for (int sh = L8; sh < 64; sh *= 2)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          cs0[k] += __shfl_xor(cs0[k], sh, 64);
          cs1[k] += __shfl_xor(cs1[k], sh, 64);
        }
      if (lane < L8) {
        const int col = n0 + wn * TWN + 8 * lane;
        const int lim = g.csum_n > 0 ? g.csum_n : g.N;
        float* dst = csum_dst(g, m0 / BM_ + bz, lim);
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (col + k < lim) atomicAdd(dst + col + k, k < 4 ? cs0[k] : cs1[k - 4]);
      }
    }
    return;
  }
  // column-sum epilogue: lane's 4 columns are the same for every iteration (64 % (TWN/4) == 0)
  f32x4 cs = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
      const int rlim = min(mlim, m0 + wm * TWM + min(TWM, ch * 64 + 64));
    // this wave's rows ch*64 .. +64 -> its LDS region (the region is the wave's own: the read below
    // only needs the wave's LDS writes retired, which the barrier also guarantees)
#pragma unroll
    for (int ii = 0; ii < 4; ++ii)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (ch * 4 + ii < MI) reg[(ii * 16 + 4 * (lane >> 4) + e) * RP + j * 16 + (lane & 15)] = acc[ch * 4 + ii][j][e];
    __syncthreads();
#pragma unroll 4
    for (int it = 0; it < NIT; ++it) {
      const int q = it * 64 + lane, lr = q / (TWN / 4), c4 = q - lr * (TWN / 4);
      const int row = m0 + wm * TWM + ch * 64 + lr, col = n0 + wn * TWN + 4 * c4;
      if (row >= rlim || col >= g.N) continue;
      f32x4 v = *reinterpret_cast<const f32x4*>(reg + lr * RP + 4 * c4);
      const long long o = (long long)row * g.ldc + col;
      if (vec && col + 3 < g.N) {
        if (res) v += *reinterpret_cast<const f32x4*>(res + o);
        if (acc_c) v += *reinterpret_cast<const f32x4*>(C + o);
        if (agr || agr16) {
          f32x4 x;
          if (agr) {
            x = *reinterpret_cast<const f32x4*>(agr + o);
          } else {
            const bf16x4 h = *reinterpret_cast<const bf16x4*>(agr16 + o);
            x = f32x4{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
          }
          v = f32x4{v[0] * gelu_grad_f(x[0]), v[1] * gelu_grad_f(x[1]), v[2] * gelu_grad_f(x[2]),
                    v[3] * gelu_grad_f(x[3])};
        }
        if (C) *reinterpret_cast<f32x4*>(C + o) = v;
        if (P16) *reinterpret_cast<bf16x4*>(P16 + o) = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
        if (csum) cs += v;
        if (C16) {
          const f32x4 w = gelu16 ? f32x4{gelu_f(v[0]), gelu_f(v[1]), gelu_f(v[2]), gelu_f(v[3])} : v;
          *reinterpret_cast<bf16x4*>(C16 + o) = bf16x4{(bf16)w[0], (bf16)w[1], (bf16)w[2], (bf16)w[3]};
        }
      } else {
        for (int k = 0; k < 4 && col + k < g.N; ++k) {
          float x = v[k];
          if (res) x += res[o + k];
          if (acc_c) x += C[o + k];
          if (agr) x *= gelu_grad_f(agr[o + k]);
          if (agr16) x *= gelu_grad_f((float)agr16[o + k]);
          if (C) C[o + k] = x;
          if (P16) P16[o + k] = (bf16)x;
          if (csum) cs[k] += x;
          if (C16) C16[o + k] = (bf16)(gelu16 ? gelu_f(x) : x);
        }
      }
    }
    __syncthreads();  // the region is rewritten by the next chunk / reused by the BN epilogue
  }
  if (csum) {
    // lanes sharing this lane's 4 columns: lane + k * (TWN/4)
#pragma unroll
    for (int sh = TWN / 4; sh < 64; sh *= 2)
#pragma unroll
      for (int k = 0; k < 4; ++k) cs[k] += __shfl_xor(cs[k], sh, 64);
    if (lane < TWN / 4) {
      const int col = n0 + wn * TWN + 4 * lane;
      const int lim = g.csum_n > 0 ? g.csum_n : g.N;
      float* dst = csum_dst(g, m0 / BM_ + bz, lim);
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (col + k < lim) atomicAdd(dst + col + k, cs[k]);
    }
  }
}

// BatchNorm BACKWARD reduction of the layer that produced this data-gradient GEMM's output
// (avc_gemm_bnb on the halo conv ring: C = dL/da of the producing conv + BN + act layer, whose
// stored conv output y, statistics and affine parameters come in g.bnb_*): per column of this
// 128 x 128 tile, over its rows, (sum dz, sum dz*yhat, sum yhat) with yhat = (y - mean)*rstd and
// dz = C * act'(yhat*gamma + beta) -- C rounded to bf16 first when only the bf16 C is stored (the
// value the apply pass reads) -- into the 128-row-tile partials; the last-arriving row tile of the
// column tile reduces them into the apply constants coef[6][N] and the parameter gradients
// (avcbn::bwd_finalize_store).  The separate reduce + finalize launches of the BN backward
// (bn.hip) are gone.  y (bf16, the bf16 step's conv output) is staged through LDS as 16-B rows.
// y prefetch of the tile: 4 x 16 B per thread, issued at kernel start into registers so it lands
// under the K loop (a load-then-store loop in the epilogue had serialised four HBM round trips)
constexpr int BNB_YQ = 128 * 16 / RNT;  // 16-B chunks per thread (128 rows x 16 chunks of 8 bf16)
// LDS offset of the staged y tile (128 rows x 272 B + flag): below the C staging (ring_epi_lds),
// above the partial sums, so the 2-stage conv ring's 98 KiB hold it
constexpr int BNB_YS_LO = 8 * 1024;
__device__ __forceinline__ int bnb_ys(const GemmArgs&) { return BNB_YS_LO; }
__device__ __forceinline__ void ring_bnb_prefetch(const GemmArgs& g, int m0, int n0, u32x4 (&yv)[BNB_YQ]) {
  const bf16* yb = static_cast<const bf16*>(g.bnb_y);
  // unconditional loads at clamped addresses (N % 8 == 0 on this path), zeroed after: a load inside
  // a bounds branch is waited for at the branch join
#pragma unroll
  for (int k = 0; k < BNB_YQ; ++k) {
    const int q = threadIdx.x + k * RNT, r = q >> 4, cc = q & 15;
    const int row = m0 + r, col = n0 + cc * 8;
    yv[k] = *reinterpret_cast<const u32x4*>(yb + (long long)min(row, g.M - 1) * g.ldc + min(col, g.N - 8));
  }
  // (rows / columns outside the tensor are zeroed where the values are written to LDS: a select
  // here would be a use, and hipcc would wait for the loads right away)
}

__device__ __forceinline__ bool ring_bnb_epilogue(const GemmArgs& g, f32x4 (&acc)[4][2], int m0, int n0,
                                                  char* smem_raw, const u32x4* yv) {
  constexpr int BN_ = 128, NJ = 2, FGR = 4;  // 512 threads = 128 columns x 4 row groups (finalize)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 2, wn = wid & 3;
  const int rbase = m0 + wm * 64 + 4 * (lane >> 4);
  const int cbase = n0 + wn * 32 + (lane & 15);
  const avcbn::BwdFin& f = g.bnb_fin;
  float* red = reinterpret_cast<float*>(smem_raw);  // [3][2 wm][BN_] / the finalize's [3][FGR][BN_]
  constexpr int YP = 2 * BN_ + 16;                  // LDS row pitch of the staged y tile (bytes)
  // above the staged stores' LDS (ring_epi_lds: 72 KiB): the fused apply reads y again after them
  char* ys = smem_raw + bnb_ys(g);
  unsigned* flag = reinterpret_cast<unsigned*>(ys + 128 * YP);
  __syncthreads();  // the K loop's fragment reads are done with the LDS
#pragma unroll
  for (int k = 0; k < BNB_YQ; ++k) {
    const int q = tid + k * RNT, r = q >> 4, cc = q & 15;
    const bool in = m0 + r < g.M && n0 + cc * 8 < g.N;
    *reinterpret_cast<u32x4*>(ys + r * YP + cc * 16) = in ? yv[k] : u32x4{0u, 0u, 0u, 0u};
  }
  __syncthreads();
  const bool round16 = g.c == nullptr;
  float s0[NJ], s1[NJ], s2[NJ];
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
        if (round16) v = (float)(bf16)v;
        const float yf = __builtin_bit_cast(
            float, (unsigned)*reinterpret_cast<const unsigned short*>(ys + (row - m0) * YP + (col - n0) * 2) << 16);
        const float yh = (yf - mu) * rs;
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
  }
  if (lane < 16) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int cl = wn * 32 + j * 16 + lane;
      red[(0 * 2 + wm) * BN_ + cl] = s0[j];
      red[(1 * 2 + wm) * BN_ + cl] = s1[j];
      red[(2 * 2 + wm) * BN_ + cl] = s2[j];
    }
  }
  __syncthreads();
  const int mt = m0 / 128;
  if (tid < BN_) {
    const int col = n0 + tid;
    if (col < g.N) {
      float* p = g.bnb_ws + ((long long)mt * g.N + col) * 3;
#pragma unroll
      for (int q = 0; q < 3; ++q) st_sc1(p + q, red[(q * 2) * BN_ + tid] + red[(q * 2 + 1) * BN_ + tid]);
    }
  }
  const int nrb = (g.M + 127) / 128;
  return ring_arrive_last(g.bnb_cnt + n0 / BN_, (unsigned)nrb, 1u, flag);
}

// the last-arriving row tile of a column tile: the apply constants and parameter gradients of its
// 128 columns from every row tile's partials (after this workgroup's C stores are issued, so their
// drain overlaps these loads)
__device__ __forceinline__ void ring_bnb_finalize(const GemmArgs& g, int n0, char* smem_raw) {
  constexpr int BN_ = 128, FGR = 4;
  const int tid = threadIdx.x;
  const avcbn::BwdFin& f = g.bnb_fin;
  float* red = reinterpret_cast<float*>(smem_raw);
  const int nrb = (g.M + 127) / 128;
  {
    // 128 columns x FGR row groups, the partials handed over within the launch (sc1 loads)
    const int cl = tid & (BN_ - 1), grp = tid >> 7;
    const int c = n0 + cl;
    const bool cv = c < g.N;
    float sv[3] = {0.f, 0.f, 0.f};
    // 16 partial rows per thread in flight (a sequential loop of sc1 loads had cost ~25 us per conv)
    static_assert(FGR == avcbn::FG, "row groups of strided_sums");
    if (cv) avcbn::strided_sums<3, true, 16>(g.bnb_ws, nrb, g.N, c, grp, sv);
    __syncthreads();
    red[(0 * FGR + grp) * BN_ + cl] = sv[0];
    red[(1 * FGR + grp) * BN_ + cl] = sv[1];
    red[(2 * FGR + grp) * BN_ + cl] = sv[2];
    __syncthreads();
    if (grp == 0 && cv) {
      float a0 = 0.f, a1 = 0.f, a2 = 0.f;
#pragma unroll
      for (int k = 0; k < FGR; ++k) {
        a0 += red[(0 * FGR + k) * BN_ + cl];
        a1 += red[(1 * FGR + k) * BN_ + cl];
        a2 += red[(2 * FGR + k) * BN_ + cl];
      }
      avcbn::bwd_finalize_store(c, a0, a1, a2, g.M, g.N, f);
    }
  }
}

// Epilogue for the 2 x 4 wave layout (see ring_store_tile): bias and conv0-fold row bias in the
// accumulators, the staged stores, then the BatchNorm partial statistics / finalize.
// BNB: compile the BN-backward reduction (128 x 128 only; yv = the y tile prefetched at kernel start)
// mlim < 0: g.M; the one-utterance conv tile passes the end of its utterance.  BM_ == 192 (that tile)
// computes ONE BatchNorm statistics tile of g.bn_rows rows (both wave rows); otherwise 128-row ones.
template <int BM_, int BN_, bool BNB = false>
__device__ __forceinline__ void ring_epilogue(const GemmArgs& g, f32x4 (&acc)[BM_ / 32][BN_ / 64], int m0, int n0,
                                              int bz, int ks, char* smem_raw, const u32x4* yv = nullptr,
                                              int mlim = -1) {
  constexpr int TWM = BM_ / 2, TWN = BN_ / 4, MI = TWM / 16, NJ = TWN / 16;
  if (mlim < 0) mlim = g.M;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 2, wn = wid & 3;
  const int rbase = m0 + wm * TWM + 4 * (lane >> 4);
  const int cbase = n0 + wn * TWN + (lane & 15);
  if (g.bias && ks == 0) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int col = cbase + j * 16;
      const float bv = col < g.N ? g.bias[col] : 0.f;
#pragma unroll
      for (int i = 0; i < MI; ++i) acc[i][j] += bv;
    }
  }
  if (g.rbias && ks == 0) {
    const int T = g.rb_t, pad = g.rb_pad, ncls = 2 * pad + 1;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = rbase + i * 16 + e;
        if (row >= mlim) continue;
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
  bool bnb_last = false;
  if constexpr (BNB && BM_ == 128 && BN_ == 128) {
    // before the C stores, so the last-arrival wait covers the partials only
    if (g.bnb_ws) bnb_last = ring_bnb_epilogue(g, acc, m0, n0, smem_raw, yv);
  }
  ring_store_tile<BM_, BN_>(g, acc, m0, n0, bz, ks, smem_raw, mlim);
  if constexpr (BNB && BM_ == 128 && BN_ == 128) {
    if (bnb_last) {
      __syncthreads();  // the staged stores are done with the LDS
      ring_bnb_finalize(g, n0, smem_raw);
    }
  }
  if (g.bn_partial) {
    // per 128-row statistics tile: column sum and M2 about the tile mean (Chan's form, merged by
    // the finalize).  Waves w with (w's rows)/128 == h contribute to tile h of this workgroup.
    constexpr bool UTT = BM_ == 192;              // one statistics tile of g.bn_rows rows
    constexpr int NH = UTT ? 1 : BM_ / 128;       // statistics tiles per workgroup tile
    constexpr int WPT = UTT ? 2 : 128 / TWM;      // waves (along M) per statistics tile
    const int srows = UTT ? g.bn_rows : 128;
    float* red = reinterpret_cast<float*>(smem_raw);  // [2][BN_] sums, then [2][BN_] M2
    float* red2 = red + 2 * BN_;
    unsigned* flag = reinterpret_cast<unsigned*>(red2 + 2 * BN_);
    const int h = wm / WPT;
    const int cnt = max(1, min(srows, mlim - (m0 + srows * h)));
    float s[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      float t = 0.f;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) t += (rbase + i * 16 + e < mlim) ? acc[i][j][e] : 0.f;
      t += __shfl_xor(t, 16, 64);
      t += __shfl_xor(t, 32, 64);
      s[j] = t;
    }
    __syncthreads();  // the main loop's last fragment reads of LDS are done
    if (lane < 16) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) red[wm * BN_ + wn * TWN + j * 16 + lane] = s[j];
    }
    __syncthreads();
    float qv[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int cl = wn * TWN + j * 16 + (lane & 15);
      float tot = 0.f;
#pragma unroll
      for (int w = 0; w < WPT; ++w) tot += red[(h * WPT + w) * BN_ + cl];
      const float mean = tot / (float)cnt;
      float t = 0.f;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = acc[i][j][e] - mean;
          t += (rbase + i * 16 + e < mlim) ? d * d : 0.f;
        }
      t += __shfl_xor(t, 16, 64);
      t += __shfl_xor(t, 32, 64);
      qv[j] = t;
    }
    if (lane < 16) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) red2[wm * BN_ + wn * TWN + j * 16 + lane] = qv[j];
    }
    __syncthreads();
    const int mt0 = m0 / srows;
    if (tid < NH * BN_) {
      const int hh = tid / BN_, cl = tid - hh * BN_;
      const int col = n0 + cl;
      if (col < g.N && m0 + srows * hh < g.M) {
        float s0 = 0.f, s1 = 0.f;
#pragma unroll
        for (int w = 0; w < WPT; ++w) {
          s0 += red[(hh * WPT + w) * BN_ + cl];
          s1 += red2[(hh * WPT + w) * BN_ + cl];
        }
        float* p = g.bn_partial + ((long long)(mt0 + hh) * g.N + col) * 2;
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
      const int ntile = (g.M + srows - 1) / srows;
      const int mine = min(NH, ntile - mt0);
      unsigned* cnt = g.bn_cnt + n0 / BN_;
      if (ring_arrive_last(cnt, (unsigned)ntile, (unsigned)mine, flag)) bn_finalize_cols<BN_>(g, n0, red);
    }
  }
}

template <int BM_, int BN_, int NST, bool WIN>
__global__ void __launch_bounds__(RNT, 2) gemm_ring_kernel(GemmArgs g, int gm) {
  constexpr int TWM = BM_ / 2, TWN = BN_ / 4, MI = TWM / 16, NJ = TWN / 16;
  constexpr int A_BYTES = BM_ * RROW, STAGE = (BM_ + BN_) * RROW;
  constexpr int LPT = BM_ / 64 + BN_ / 64;  // glds per thread per K-step
  constexpr int P = NST - 1;                // K-steps in flight
  static_assert(NST >= 2 && NST <= 4, "ring depth");
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 2, wn = wid & 3;

  // XCD-aware bijective remap (blocks b, b+8, ... share an XCD) ...
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q = nwg >> 3, rr = nwg & 7, xcd = bid & 7;
  const int lid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
  // ... then grouped order: gm row tiles x all column tiles per group, row tile fastest
  const int nN = (g.N + BN_ - 1) / BN_, nM = (g.M + BM_ - 1) / BM_;
  const int z = lid / (nN * nM);
  const int rem = lid - z * nN * nM;
  const int grp = rem / (gm * nN);
  const int fm = grp * gm;
  const int gsz = min(nM - fm, gm);
  const int wi = rem - grp * gm * nN;
  const int mt = fm + wi % gsz, nt = wi / gsz;
  const int m0 = mt * BM_, n0 = nt * BN_;
  const int bz = z / g.split_k, ks = z - bz * g.split_k;
  const int kbeg = ks * g.klen;
  const int kend = min(g.K, kbeg + g.klen);
  const int nkt = kend > kbeg ? (kend - kbeg + RBK - 1) / RBK : 0;

  RingLoader<BM_, WIN> la;
  RingLoader<BN_, false> lb;
  la.init(g.a, m0, bz);
  lb.init(g.b, n0, bz);
  const FastDiv cdv = g.a.cdv;

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment reads: row (lane&15) of each 16-row block, logical chunk 4h + (lane>>4) stored at
  // chunk ^ ((row>>1)&7) = chunk ^ ((lane&15)>>1) (block bases are multiples of 16 rows)
  const int frow = lane & 15, sw = frow >> 1;
  const int ch0 = ((lane >> 4) ^ sw) << 4, ch1 = ((4 + (lane >> 4)) ^ sw) << 4;
  const int aoff = (wm * TWM + frow) * RROW, boff = A_BYTES + (wn * TWN + frow) * RROW;

#pragma unroll
  for (int p = 0; p < P; ++p)
    if (p < nkt) {
      char* st = smem_raw + p * STAGE;
      la.issue(st, kbeg + p * RBK, kend, cdv);
      lb.issue(st + A_BYTES, kbeg + p * RBK, kend, cdv);
    }

  for (int kt = 0; kt < nkt; ++kt) {
    const int ahead = min(P - 1, nkt - 1 - kt);  // K-steps allowed to stay in flight
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
      la.issue(st, kbeg + (kt + P) * RBK, kend, cdv);
      lb.issue(st + A_BYTES, kbeg + (kt + P) * RBK, kend, cdv);
    }
    // One K-step = two 32-deep halves h; fragments read by inline asm with counted waits so that
    // the next group's reads are in flight while the current group's MFMAs issue (hipcc's own
    // schedule re-used one register set and drained lgkmcnt(0) before every MFMA group):
    //   read B(h0), A(h0) rows 0..MI/2, A(h0) rows MI/2..MI | MFMA h0 first half
    //   read B(h1), A(h1) first half                       | MFMA h0 second half
    //   read A(h1) second half                             | MFMA h1 first half | MFMA h1 second half
    constexpr int MH = MI / 2;
    const unsigned st = lds_addr(smem_raw + (kt % NST) * STAGE);
    const unsigned a0 = st + aoff + ch0, a1 = st + aoff + ch1, b0 = st + boff + ch0, b1 = st + boff + ch1;
    bf16x8 af0[MI], bf0[NJ], af1[MI], bf1[NJ];
    auto mfma_rows = [&](const bf16x8* af, const bf16x8* bfr, auto i0c) {
      constexpr int I0 = decltype(i0c)::value;
#pragma unroll
      for (int i = 0; i < MH; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[I0 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[I0 + i], bfr[j], acc[I0 + i][j], 0, 0, 0);
    };
    using Z0 = std::integral_constant<int, 0>;
    using ZH = std::integral_constant<int, MH>;
    ds_read_n<NJ, 16 * RROW>(bf0, b0);
    ds_read_n<MH, 16 * RROW>(af0, a0);
    ds_read_n<MH, 16 * RROW, MH * 16 * RROW>(af0 + MH, a0);
    wait_lgkm<MH>();
    mfma_rows(af0, bf0, Z0{});
    __builtin_amdgcn_sched_barrier(0);
    ds_read_n<NJ, 16 * RROW>(bf1, b1);
    ds_read_n<MH, 16 * RROW>(af1, a1);
    wait_lgkm<NJ + MH>();
    mfma_rows(af0, bf0, ZH{});
    __builtin_amdgcn_sched_barrier(0);
    ds_read_n<MH, 16 * RROW, MH * 16 * RROW>(af1 + MH, a1);
    wait_lgkm<MH>();
    mfma_rows(af1, bf1, Z0{});
    wait_lgkm<0>();
    mfma_rows(af1, bf1, ZH{});
  }
  __syncthreads();  // every glds retired (the last wait was vmcnt(0)) and every fragment read done
  ring_epilogue<BM_, BN_>(g, acc, m0, n0, bz, ks, smem_raw);
}

template <int BM_, int BN_, int NST, bool WIN>
void launch(const GemmArgs& g, int gm, hipStream_t s) {
  const size_t lds = std::max((size_t)NST * (BM_ + BN_) * RROW, ring_epi_lds<BM_, BN_>());
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_ring_kernel<BM_, BN_, NST, WIN>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  const int nb = ((g.M + BM_ - 1) / BM_) * ((g.N + BN_ - 1) / BN_) * g.batch * g.split_k;
  gemm_ring_kernel<BM_, BN_, NST, WIN><<<nb, RNT, lds, s>>>(g, gm);
}

// ---------------------------------------------------------------------------------------------
// Conv1d (5 taps, stride 1, 'same' padding) with the input tile staged ONCE for all taps, in the
// ring form: 128 frames x 128 output columns per workgroup (the one tile that gives each of the
// 256 CUs a tile of the AutoVC 8192 x 512 convs), 8 waves as 2 x 4 (64 x 32 each), stages of
// CBK = 32 channels: the 132-row halo (128 frames + 4, 64-B rows) and the five 128-column weight
// slices (640 rows x 64 B) = 49 KiB per stage, three stages (147 KiB), two in flight.  Tap k
// reads the halo k rows down.  The 49 glds wave-instructions of a stage are dealt over the 8
// waves (wave 0 issues 7, the others 6: the counted waits use each wave's own count).
// ALIGNED (T % 128 == 0): a tile never spans two utterances, so the loader zero-fills the halo
// rows of other utterances and the fragments need no per-lane predicate; otherwise a per-lane,
// per-tap mask zeroes the A fragment rows whose shifted frame leaves the utterance.
// X = activation, W = Wf[co][tap][ci] (forward) or dy and Wd[ci][tap'][co] (data gradient).
// CV_NST: LDS stages of the halo conv ring.  Two (98 KiB) rather than three (147 KiB): alone the
// same time (29.0 vs 28.6 us at 8192 x 512 x 2560), but a side-stream weight-gradient workgroup
// (48 KiB) now fits on a CU beside it, so a backward conv no longer waits for those to drain from
// its CUs: C2 5.78-5.80 -> 5.74-5.75 ms (profiles/r5_conv_ring_slope.txt).  The one-utterance tile
// (CU_NST) and the warp-specialised diagnostic form (WS_NST) keep three.
constexpr int CV_TM = 128, CV_TN = 128, CV_TAPS = 5, CV_CBK = 32, CV_NST = 2, CU_NST = 3;
constexpr int CV_AI = (CV_TM + CV_TAPS - 1 + 15) / 16;  // 9 halo instructions (16 rows of 64 B)
constexpr int CV_BI = CV_TAPS * CV_TN / 16;             // 40 weight instructions
constexpr int CV_TOT = CV_AI + CV_BI;                   // 49
constexpr int CV_LW = (CV_TOT + 7) / 8;                 // 7: instructions of waves < CV_TOT % 8
constexpr int CV_ABYTES = CV_AI * 1024;
constexpr int CV_STAGE = CV_TOT * 1024;

template <int N>
__device__ __forceinline__ void wait_cv(bool full) {
  if (full) wait_vm<N * CV_LW>();
  else wait_vm<N * (CV_LW - 1)>();
}

// ABL (timing diagnostics only, wrong results; tools/ring_ab.py): 1 = no fragment reads / MFMAs
// (the ring's loads alone), 2 = no loads after the prologue (fragment reads + MFMAs alone),
// 3 = the weight slices fetched as 1-KiB contiguous pieces ([Ci/32][K][Co][32] addressing applied
// to the [Co][K][Ci] buffer: the timing of a repacked weight layout), 4 = MFMAs alone (no loads
// after the prologue, fragments read in the first stage only), 5 = fragment reads alone (no loads
// after the prologue, no MFMAs), 6 = production with s_setprio(1) around every MFMA group
template <bool ALIGNED, int ABL = 0, bool BNB = false>
__global__ void __launch_bounds__(RNT, 2) conv_ring_kernel(GemmArgs g, int gm) {
  constexpr int MI = 4, NJ = 2, P = CV_NST - 1;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3;
  const bool full = wid < (CV_TOT % 8 ? CV_TOT % 8 : 8);  // this wave issues CV_LW per stage

  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q = nwg >> 3, rr = nwg & 7, xcd = bid & 7;
  const int lid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
  const int nN = (g.N + CV_TN - 1) / CV_TN, nM = (g.M + CV_TM - 1) / CV_TM;
  const int grp = lid / (gm * nN), fm = grp * gm, gsz = min(nM - fm, gm);
  const int wi = lid - grp * gm * nN;
  const int mt = fm + wi % gsz, nt = wi / gsz;
  const int m0 = mt * CV_TM, n0 = nt * CV_TN;

  const OpDev& A = g.a;
  const OpDev& Bo = g.b;
  const bf16* xa = reinterpret_cast<const bf16*>(A.ptr);
  const bf16* wb = reinterpret_cast<const bf16*>(Bo.ptr);
  const int pad = A.pad, T = A.t_out, chans = A.chans;
  const int nst = chans / CV_CBK;

  // ---- loader: instruction qi = i*8 + wid (i < CV_LW, qi < CV_TOT) writes stage bytes
  // [qi KiB, +1 KiB) = rows 16*qi + (lane>>2) of 64 B, 16-B slot lane&3 holding the global chunk
  // (lane&3) ^ ((row>>1)&3)
  const int b0 = (int)fdiv((uint32_t)m0, A.tdiv);  // utterance of the tile's first row
  // a lane whose row is padding reads the 16-B zero granule at every stage (stride 0): no select
  // in the issue loop, and the granule's address pinned in VGPRs (hipcc had re-loaded it from the
  // GOT, s_load + lgkmcnt(0), before every fill: 30 per stage loop)
  const bf16* zp = reinterpret_cast<const bf16*>(g_zero16_rg);
  asm volatile("" : "+v"(zp));
  const bf16* src[CV_LW];
  long long sst[CV_LW];  // elements per stage
#pragma unroll
  for (int i = 0; i < CV_LW; ++i) {
    const int qi = i * 8 + wid;
    const int lrow = lane >> 2, slot = lane & 3;
    src[i] = zp;
    sst[i] = 0;
    if (qi < CV_AI) {
      const int hr = 16 * qi + lrow;  // halo row
      const int f = m0 - pad + hr;
      bool ok = hr < CV_TM + CV_TAPS - 1 && f >= 0 && f < g.M;
      if (ALIGNED && ok) ok = (int)fdiv((uint32_t)f, A.tdiv) == b0;
      if (ok) {
        src[i] = xa + (long long)f * A.ld + 8 * (slot ^ ((hr >> 1) & 3));
        sst[i] = CV_CBK;
      }
    } else if (qi < CV_TOT) {
      const int wr = 16 * (qi - CV_AI) + lrow;  // weight row = tap * 128 + column
      const int tap = wr / CV_TN, n = n0 + (wr - tap * CV_TN);
      if (n < g.N) {
        if (ABL == 3) {
          src[i] = wb + ((long long)tap * g.N + n) * CV_CBK + 8 * (slot ^ ((wr >> 1) & 3));
          sst[i] = (long long)CV_TAPS * g.N * CV_CBK;
        } else {
          src[i] = wb + (long long)n * Bo.ld + (long long)tap * chans + 8 * (slot ^ ((wr >> 1) & 3));
          sst[i] = CV_CBK;
        }
      }
    }
  }
  auto issue = [&](int stg, int cs) {
    char* base = smem_raw + stg * CV_STAGE;
#pragma unroll
    for (int i = 0; i < CV_LW; ++i) {
      const int qi = i * 8 + wid;
      if (qi < CV_TOT) glds16(src[i] + cs * sst[i], base + qi * 1024);
    }
  };

  // ---- fragments: A row (halo) wm*64 + i*16 + frow + k, chunk (lane>>4) ^ ((row>>1)&3); rows
  // 16 apart share the swizzle, so i is an immediate offset of 1 KiB.  B row k*128 + wn*32 + j*16 +
  // frow: its swizzle is ((frow>>1)&3), the (k, j) part an immediate offset.
  const int frow = lane & 15, kq = lane >> 4;
  int aaddr[CV_TAPS];
#pragma unroll
  for (int k = 0; k < CV_TAPS; ++k) {
    const int r = wm * 64 + frow + k;
    aaddr[k] = r * 64 + 16 * (kq ^ ((r >> 1) & 3));
  }
  const int baddr = CV_ABYTES + (wn * 32 + frow) * 64 + 16 * (kq ^ ((frow >> 1) & 3));
  unsigned vmask = 0xFFFFFFFFu;
  if (!ALIGNED) {
    vmask = 0;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int m = min(m0 + wm * 64 + i * 16 + frow, g.M - 1);
      const int b = (int)fdiv((uint32_t)m, A.tdiv);
      const int t = m - b * T;
#pragma unroll
      for (int k = 0; k < CV_TAPS; ++k) {
        const int t2 = t + k - pad;
        if (t2 >= 0 && t2 < T) vmask |= 1u << (i * 8 + k);
      }
    }
  }

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[2][MI], bfr[2][NJ];
  u32x4 bnb_y[BNB ? BNB_YQ : 1];
  if constexpr (BNB) {
    if (g.bnb_ws) ring_bnb_prefetch(g, m0, n0, bnb_y);
  }

#pragma unroll
  for (int p = 0; p < P; ++p)
    if (p < nst) issue(p, p);

  for (int cs = 0; cs < nst; ++cs) {
    const int ahead = min(P - 1, nst - 1 - cs);
    if (ahead >= 1) wait_cv<1>(full);
    else wait_vm<0>();
    raw_barrier();
    if ((ABL == 0 || ABL == 3 || ABL == 6) && cs + P < nst) issue((cs + P) % CV_NST, cs + P);
    if (ABL == 1) continue;
    const unsigned st = lds_addr(smem_raw + (cs % CV_NST) * CV_STAGE);
    auto read_tap = [&](auto kc, int slot) {
      if (ABL == 4 && cs > 0) return;
      constexpr int k = decltype(kc)::value;
      const unsigned a0 = st + aaddr[k], b0 = st + baddr;
      af[slot][0] = ds_read16<0>(a0);
      af[slot][1] = ds_read16<1024>(a0);
      af[slot][2] = ds_read16<2048>(a0);
      af[slot][3] = ds_read16<3072>(a0);
      bfr[slot][0] = ds_read16<(k * CV_TN) * 64>(b0);
      bfr[slot][1] = ds_read16<(k * CV_TN + 16) * 64>(b0);
    };
    auto mfma_tap = [&](auto kc, int slot) {
      constexpr int k = decltype(kc)::value;
      if (ABL == 5) {  // keep the reads live without MFMAs
#pragma unroll
        for (int i = 0; i < MI; ++i) asm volatile("" ::"v"(af[slot][i]));
#pragma unroll
        for (int j = 0; j < NJ; ++j) asm volatile("" ::"v"(bfr[slot][j]));
        return;
      }
      if (ABL == 6) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const bf16x8 av = (ALIGNED || ((vmask >> (i * 8 + k)) & 1u)) ? af[slot][i] : bf16x8{};
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bfr[slot][j], acc[i][j], 0, 0, 0);
      }
      if (ABL == 6) __builtin_amdgcn_s_setprio(0);
    };
    // Software pipeline with inline-asm fragment reads and counted waits: tap k+1's six reads are
    // in flight while tap k's eight MFMAs issue (the wave waits only for tap k's reads).  Left to
    // itself hipcc re-used one register set and waited lgkmcnt(0) twice per tap -- two exposed
    // LDS round trips per tap, 23.5 us of the conv in its reads + MFMAs alone (tools/ring_ab.py).
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    using I4 = std::integral_constant<int, 4>;
    read_tap(I0{}, 0);
    read_tap(I1{}, 1);
    wait_lgkm<6>();
    mfma_tap(I0{}, 0);
    __builtin_amdgcn_sched_barrier(0);
    read_tap(I2{}, 0);
    wait_lgkm<6>();
    mfma_tap(I1{}, 1);
    __builtin_amdgcn_sched_barrier(0);
    read_tap(I3{}, 1);
    wait_lgkm<6>();
    mfma_tap(I2{}, 0);
    __builtin_amdgcn_sched_barrier(0);
    read_tap(I4{}, 0);
    wait_lgkm<6>();
    mfma_tap(I3{}, 1);
    wait_lgkm<0>();
    mfma_tap(I4{}, 0);
  }
  __syncthreads();
  ring_epilogue<CV_TM, CV_TN, BNB>(g, acc, m0, n0, 0, 0, smem_raw, bnb_y);
}

// ---------------------------------------------------------------------------------------------
// The halo conv with ONE UTTERANCE per row tile (128 < T <= 192, T = 176 for C4 / C5): a 192 x 128
// tile (the 2 x 4 waves own 96 x 32 each, 6 x 2 MFMA blocks) whose rows T .. 191 are computed from
// zero halo rows and never stored, so B = 64 utterances x 4 column tiles = 256 tiles = one round of
// the CUs (the 128-row tiles of conv_ring_kernel number 352 at T = 176: two rounds, no faster than
// gemm_conv.hip).  A stage holds the utterance's T + 4 halo rows (13 fill instructions of 16 rows)
// and the five weight slices (40): 53 KiB, three stages = 159 KiB.  The BatchNorm statistics of the
// forward come as one T-row tile per workgroup (GemmArgs::bn_rows = T, merged by bn_finalize_cols).
constexpr int CU_TM = 192, CU_AI = 13, CU_TOT = CU_AI + CV_BI, CU_LW = (CU_TOT + 7) / 8;
constexpr int CU_ABYTES = CU_AI * 1024, CU_STAGE = CU_TOT * 1024;

template <int N>
__device__ __forceinline__ void wait_cu(bool full) {
  if (full) wait_vm<N * CU_LW>();
  else wait_vm<N * (CU_LW - 1)>();
}

template <int NSTU>
__global__ void __launch_bounds__(RNT, 2) conv_utt_kernel(GemmArgs g, int gm) {
  constexpr int MI = 6, NJ = 2, P = NSTU - 1;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3;
  const bool full = wid < (CU_TOT % 8 ? CU_TOT % 8 : 8);  // this wave issues CU_LW per stage

  const OpDev& A = g.a;
  const OpDev& Bo = g.b;
  const int pad = A.pad, T = A.t_out, chans = A.chans;
  const int nst = chans / CV_CBK;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q = nwg >> 3, rr = nwg & 7, xcd = bid & 7;
  const int lid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
  const int nN = (g.N + CV_TN - 1) / CV_TN, nM = g.M / T;
  const int grp = lid / (gm * nN), fm = grp * gm, gsz = min(nM - fm, gm);
  const int wi = lid - grp * gm * nN;
  const int mt = fm + wi % gsz, nt = wi / gsz;
  const int m0 = mt * T, n0 = nt * CV_TN;
  const bf16* xa = reinterpret_cast<const bf16*>(A.ptr);
  const bf16* wb = reinterpret_cast<const bf16*>(Bo.ptr);

  // loader: instruction qi = i*8 + wid writes stage bytes [qi KiB, +1 KiB): rows 16*qi + (lane>>2)
  // of 64 B; halo rows outside the utterance read the zero granule (stride 0)
  const bf16* zp = reinterpret_cast<const bf16*>(g_zero16_rg);
  asm volatile("" : "+v"(zp));
  const bf16* src[CU_LW];
  long long sst[CU_LW];
#pragma unroll
  for (int i = 0; i < CU_LW; ++i) {
    const int qi = i * 8 + wid;
    const int lrow = lane >> 2, slot = lane & 3;
    src[i] = zp;
    sst[i] = 0;
    if (qi < CU_AI) {
      const int hr = 16 * qi + lrow;
      const int t = hr - pad;  // frame within the utterance
      if (t >= 0 && t < T) {
        src[i] = xa + (long long)(m0 + t) * A.ld + 8 * (slot ^ ((hr >> 1) & 3));
        sst[i] = CV_CBK;
      }
    } else if (qi < CU_TOT) {
      const int wr = 16 * (qi - CU_AI) + lrow;  // weight row = tap * 128 + column
      const int tap = wr / CV_TN, n = n0 + (wr - tap * CV_TN);
      if (n < g.N) {
        src[i] = wb + (long long)n * Bo.ld + (long long)tap * chans + 8 * (slot ^ ((wr >> 1) & 3));
        sst[i] = CV_CBK;
      }
    }
  }
  auto issue = [&](int stg, int cs) {
    char* base = smem_raw + stg * CU_STAGE;
#pragma unroll
    for (int i = 0; i < CU_LW; ++i) {
      const int qi = i * 8 + wid;
      if (qi < CU_TOT) glds16(src[i] + cs * sst[i], base + qi * 1024);
    }
  };

  // fragments: A row (halo) wm*96 + i*16 + frow + k (i an immediate offset of 1 KiB), B row
  // k*128 + wn*32 + j*16 + frow
  const int frow = lane & 15, kq = lane >> 4;
  int aaddr[CV_TAPS];
#pragma unroll
  for (int k = 0; k < CV_TAPS; ++k) {
    const int r = wm * 96 + frow + k;
    aaddr[k] = r * 64 + 16 * (kq ^ ((r >> 1) & 3));
  }
  const int baddr = CU_ABYTES + (wn * 32 + frow) * 64 + 16 * (kq ^ ((frow >> 1) & 3));

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[2][MI], bfr[2][NJ];

#pragma unroll
  for (int p = 0; p < P; ++p)
    if (p < nst) issue(p, p);

  for (int cs = 0; cs < nst; ++cs) {
    const int ahead = min(P - 1, nst - 1 - cs);
    if (ahead >= 1) wait_cu<1>(full);
    else wait_vm<0>();
    raw_barrier();
    if (cs + P < nst) issue((cs + P) % NSTU, cs + P);
    const unsigned st = lds_addr(smem_raw + (cs % NSTU) * CU_STAGE);
    auto read_tap = [&](auto kc, int slot) {
      constexpr int k = decltype(kc)::value;
      const unsigned a0 = st + aaddr[k], b0 = st + baddr;
      af[slot][0] = ds_read16<0>(a0);
      af[slot][1] = ds_read16<1024>(a0);
      af[slot][2] = ds_read16<2048>(a0);
      af[slot][3] = ds_read16<3072>(a0);
      af[slot][4] = ds_read16<4096>(a0);
      af[slot][5] = ds_read16<5120>(a0);
      bfr[slot][0] = ds_read16<(k * CV_TN) * 64>(b0);
      bfr[slot][1] = ds_read16<(k * CV_TN + 16) * 64>(b0);
    };
    auto mfma_tap = [&](int slot) {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[slot][i], bfr[slot][j], acc[i][j], 0, 0, 0);
    };
    // tap k+1's eight reads in flight while tap k's twelve MFMAs issue (conv_ring_kernel's pipeline)
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    using I4 = std::integral_constant<int, 4>;
    read_tap(I0{}, 0);
    read_tap(I1{}, 1);
    wait_lgkm<8>();
    mfma_tap(0);
    __builtin_amdgcn_sched_barrier(0);
    read_tap(I2{}, 0);
    wait_lgkm<8>();
    mfma_tap(1);
    __builtin_amdgcn_sched_barrier(0);
    read_tap(I3{}, 1);
    wait_lgkm<8>();
    mfma_tap(0);
    __builtin_amdgcn_sched_barrier(0);
    read_tap(I4{}, 0);
    wait_lgkm<8>();
    mfma_tap(1);
    wait_lgkm<0>();
    mfma_tap(0);
  }
  __syncthreads();
  ring_epilogue<CU_TM, CV_TN>(g, acc, m0, n0, 0, 0, smem_raw, nullptr, m0 + T);
}

void launch_conv_utt(const GemmArgs& g0, int gm, hipStream_t s) {
  GemmArgs g = g0;
  g.bn_rows = g.a.t_out;  // one statistics tile per utterance
  // three LDS stages (two: 106 KiB, room for a side-stream workgroup beside it -- measured no faster,
  // profiles/r5_conv_ring_slope.txt)
  const size_t lds = std::max((size_t)CU_NST * CU_STAGE, ring_epi_lds<CU_TM, CV_TN>());
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_utt_kernel<CU_NST>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  const int nb = (g.M / g.a.t_out) * ((g.N + CV_TN - 1) / CV_TN);
  conv_utt_kernel<CU_NST><<<nb, RNT, lds, s>>>(g, gm);
}

template <bool ALIGNED, int ABL = 0, bool BNB = false>
void launch_conv(const GemmArgs& g, int gm, hipStream_t s) {
  const size_t lds = std::max((size_t)CV_NST * CV_STAGE, ring_epi_lds<CV_TM, CV_TN>());
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_ring_kernel<ALIGNED, ABL, BNB>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  const int nb = ((g.M + CV_TM - 1) / CV_TM) * ((g.N + CV_TN - 1) / CV_TN);
  conv_ring_kernel<ALIGNED, ABL, BNB><<<nb, RNT, lds, s>>>(g, gm);
}

bool ok16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

bool operand_ok(const OpDev& o, bool allow_win) {
  if (o.dtype != AVC_BF16 || !ok16(o.ptr) || o.ld % 8 || o.bstride % 8) return false;
  if (o.win && (!allow_win || o.chans % 8)) return false;
  return true;
}

// AVC_RING = "BM,BN,NST[,GM]" forces a configuration (benchmarking), "0" disables the kernel;
// AVC_RING_WIN = 0 leaves the conv window operands to gemm_conv.hip, 1 lets forced configurations
// stream them as im2col windows, 2 (default) puts aligned 5-tap convs on the halo ring kernel.  avc_gemm_set_ring() sets the
// same at run time (A/B tools in one process).
struct RingCfg {
  int mode = -1;  // -1 auto, 0 off, 1 forced
  int bm = 0, bn = 0, nst = 0, gm = 8, win = 2;
  int abl = 0;  // timing ablations of the halo conv (win 3 / 4 through avc_gemm_set_ring)
  bool utt = true;  // one-utterance conv tiles for 128 < T <= 192 (win 10 through avc_gemm_set_ring: off)
};
RingCfg init_cfg() {
  RingCfg r;
  if (const char* e = getenv("AVC_RING")) {
    int a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    const int n = sscanf(e, "%d,%d,%d,%d", &a0, &a1, &a2, &a3);
    if (n >= 1 && a0 <= 0) r.mode = a0 < 0 ? -1 : 0;
    if (n >= 3) {
      r.mode = 1;
      r.bm = a0;
      r.bn = a1;
      r.nst = a2;
    }
    if (n >= 4 && a3 > 0) r.gm = a3;
  }
  if (const char* e = getenv("AVC_RING_WIN")) r.win = atoi(e);
  return r;
}
RingCfg g_ring = init_cfg();

}  // namespace

thread_local int g_ring_last = 0;  // avc_gemm_ring_last
bool gemm_ring_launch_(const GemmArgs& g, hipStream_t s);

bool gemm_ring_launch(const GemmArgs& g, hipStream_t s) {
  g_ring_last = 0;
  const bool r = gemm_ring_launch_(g, s);
  return r;
}

int ring_num_cus() {
  static int n = [] {
    int dev = 0;
    hipDeviceProp_t p;
    return (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&p, dev) == hipSuccess) ? p.multiProcessorCount
                                                                                                : 0;
  }();
  return n;
}

bool gemm_ring_launch_(const GemmArgs& g_in, hipStream_t s) {
  const RingCfg& c = g_ring;
  const GemmArgs& g = g_in;
  if (c.mode == 0 || (g.a.win && !c.win)) return false;
  if (g.K % 8 || g.klen % RBK || g.atomic || g.cperm) return false;  // (no atomic / cperm stores)
  if (g.ctr && ((reinterpret_cast<uintptr_t>(g.c) & 15) || (reinterpret_cast<uintptr_t>(g.res) & 15) ||
                (g.cbs & 3)))
    return false;  // the transposed stores are 16-B vectors
  if (!operand_ok(g.a, true) || !operand_ok(g.b, false)) return false;
  const long long units = (long long)g.batch * g.split_k;
  const bool win = g.a.win != 0;
  // 5-tap 'same' convs on 32-channel stages: the halo form (win == 2), utterance-aligned tiles only
  // unless forced (T % 128 != 0 leaves 1.4 tiles per CU at B=64 T=176, where the 128 x 64 tiles of
  // gemm_conv.hip spread better -- tools/ring_ab.py, profiles/r4_ring_ab.txt)
  const OpDev& a = g.a;
  const bool halo = win && c.win == 2 && a.taps == CV_TAPS && a.t_in == a.t_out && 2 * a.pad == a.taps - 1 &&
                    g.K == a.taps * a.chans && a.chans % CV_CBK == 0 && g.batch == 1 && g.split_k == 1 && !g.b.win &&
                    (c.mode == 1 || (a.t_out % CV_TM == 0 && g.N >= 128));
  // the BatchNorm-backward reduction epilogue (avc_gemm_bnb) exists on the halo conv tile only, for a
  // bf16 y (ring_bnb_epilogue)
  if (g.bnb_ws && !(halo && g.bnb_ydt == AVC_BF16 && g.N % 8 == 0 && g.ldc % 8 == 0 &&
                    (reinterpret_cast<uintptr_t>(g.bnb_y) & 15) == 0 && !g.c16_act && !g.agrad && !g.csum))
    return false;
  // one utterance per row tile (T = 176 of C4 / C5): the 192-row tile, when every epilogue it has is
  // one the 2 x 4 ring epilogue covers (no BN-backward / GELU / column-sum / transposed stores) and
  // the forward BatchNorm statistics are finalized in the kernel (their tiles are T rows, which
  // only bn_finalize_cols is told)
  const int T = a.t_out;
  const bool utt = win && c.win == 2 && c.mode != 1 && a.taps == CV_TAPS && a.t_in == T && 2 * a.pad == a.taps - 1 &&
                   g.K == a.taps * a.chans && a.chans % CV_CBK == 0 && g.batch == 1 && g.split_k == 1 && !g.b.win &&
                   T > CV_TM && T <= CU_TM && g.M % T == 0 && g.N >= 128 && !g.bnb_ws && !g.c16_act && !g.agrad &&
                   !g.csum && !g.ctr && (!g.bn_partial || g.bn_cnt) && !c.abl && c.utt;
  if (utt) {
    launch_conv_utt(g, c.gm, s);
    g_ring_last = 3;
    return true;
  }
  if (halo) {
    if (c.abl == 1) launch_conv<true, 1>(g, c.gm, s);
    else if (c.abl == 2) launch_conv<true, 2>(g, c.gm, s);
    else if (c.abl == 3) launch_conv<true, 3>(g, c.gm, s);
    else if (c.abl == 4) launch_conv<true, 4>(g, c.gm, s);
    else if (c.abl == 5) launch_conv<true, 5>(g, c.gm, s);
    else if (c.abl == 6) launch_conv<true, 6>(g, c.gm, s);
    else if (g.bnb_ws) {  // the BN-backward reduction epilogue (8-wave tile only)
      if (a.t_out % CV_TM == 0) launch_conv<true, 0, true>(g, c.gm, s);
      else launch_conv<false, 0, true>(g, c.gm, s);
    } else if (a.t_out % CV_TM == 0) launch_conv<true>(g, c.gm, s);
    else launch_conv<false>(g, c.gm, s);
    g_ring_last = 2;
    return true;
  }
  int bm, bn, nst;
  if (c.mode == 1) {
    bm = c.bm;
    bn = c.bn;
    nst = c.nst;
  } else {
    // Tile choice by a wave-quantised cost model: a configuration runs occ workgroups per CU, so
    // a product costs ceil(tiles / (256 occ)) rounds of BM*BN*K work at the configuration's per-flop
    // efficiency (1 : 0.85 : 0.75 for 256x256 / 256x128 / 128x128, fitted to the per-call census
    // of the C2 / C4 steps, tools/gemm_census.py --ring-ab, profiles/r4_gemm_census_*.txt).  Every
    // plain bf16 NN product of those steps ran as fast or faster on the chosen ring tile than on
    // gemm_nt.hip.  Conv windows: the generic window stream only for channel counts the halo form
    // cannot take (344 / 88 / 80 channels) and N <= 512, where it measured faster than
    // gemm_conv.hip; the rest stay on gemm_conv.hip.
    if (win && (g.N > 512 || a.chans % CV_CBK == 0)) return false;
    // 128x128x2 (64 KB of LDS) runs TWO workgroups per CU, one's epilogue under the other's K loop:
    // 512 concurrent tiles at efficiency 0.47, 0.38 under the GELU-backward epilogue (its extra
    // operand stream) -- fitted to the same census with that tile forced (profiles/r4_gemm_census_x2_c*.txt)
    struct Opt {
      int bm, bn, nst, occ;
      double eff;
    };
    const Opt opts[4] = {{256, 256, 2, 1, 1.0}, {256, 128, 3, 1, 0.85}, {128, 128, 4, 1, 0.75},
                         {128, 128, 2, 2, g.agrad ? 0.38 : 0.47}};
    double best = 0;
    bm = 0;
    bn = 0;
    nst = 0;
    for (const Opt& o : opts) {
      const long long tiles = (long long)((g.M + o.bm - 1) / o.bm) * ((g.N + o.bn - 1) / o.bn) * units;
      const long long slots = 256ll * o.occ;
      const double cost = (double)((tiles + slots - 1) / slots) * o.bm * o.bn / o.eff;
      if (!bm || cost < best * 0.999) {
        best = cost;
        bm = o.bm;
        bn = o.bn;
        nst = o.nst;
      }
    }
  }
#define RING_CASE(BMV, BNV, NSV)                       \
  if (bm == BMV && bn == BNV && nst == NSV) {          \
    if (win) launch<BMV, BNV, NSV, true>(g, c.gm, s);  \
    else launch<BMV, BNV, NSV, false>(g, c.gm, s);     \
    g_ring_last = 1;                                   \
    return true;                                       \
  }
  RING_CASE(256, 256, 2) RING_CASE(256, 128, 3) RING_CASE(128, 128, 4) RING_CASE(128, 128, 3)
  RING_CASE(128, 256, 3) RING_CASE(256, 128, 2) RING_CASE(128, 128, 2)  // (128x128x2: 64 KB, two per CU)
#undef RING_CASE
  return false;
}

}  // namespace avcg

extern "C" int avc_gemm_ring_last(void) { return avcg::g_ring_last; }

// Benchmarking hook (tools/ring_ab.py): mode -1 auto, 0 off, 1 forced (bm, bn, nst); gm row
// tiles per group (<= 0 keeps it); win: as AVC_RING_WIN.
extern "C" int avc_gemm_set_ring(int mode, int bm, int bn, int nst, int gm, int win) {
  avcg::g_ring.mode = mode;
  avcg::g_ring.bm = bm;
  avcg::g_ring.bn = bn;
  avcg::g_ring.nst = nst;
  if (gm > 0) avcg::g_ring.gm = gm;
  avcg::g_ring.win = win >= 3 ? 2 : win;
  // 3: loads only, 4: reads + MFMAs only, 5: contiguous weight pieces, 7: MFMAs only, 8: reads only,
  // 9: s_setprio around the MFMA groups (timing ablations of the halo conv)
  avcg::g_ring.abl = (win >= 3 && win <= 5) ? win - 2 : (win >= 7 && win <= 9) ? win - 3 : 0;
  // 10: the halo convs without the one-utterance tile (T = 176 back on gemm_conv.hip); any other
  // value restores the default
  avcg::g_ring.utt = win != 10;
  return 0;
}
