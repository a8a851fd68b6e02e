// gemm.hip — LDS-tiled MFMA GEMM with frame-window (im2col / time-shift) operand
// addressing and fused epilogues (bias, accumulate, split-K atomics, BatchNorm batch
// statistics).  gfx950 only.
//
// Replaces the implicit cuDNN/cuBLAS calls behind nn.Conv1d (factory/Norm.py:21-28),
// nn.Linear (Norm.py:40-50) and nn.LSTM's input projections (AutoVC.py:43,77,96), plus
// every weight/data-gradient GEMM of their backward.
//
// Tile 128x128x32, 256 threads = 4 waves in a 2x2 grid, each wave 64x64 = 4x4 MFMA
// 16x16 tiles.  Operands are staged global -> registers -> LDS (register staging lets
// the loader apply the conv window / zero padding and the fp32->bf16 conversion), LDS is
// double-buffered with one barrier per K-tile.
#include <cstdio>
#include <cstdlib>

#include "gemm_internal.h"

namespace {

using namespace avcg;
constexpr int BN = 128, BK = 32, NT = 256;

template <bool BF>
struct Traits;
template <>
struct Traits<true> {
  typedef bf16 T;
  static constexpr int LDK = BK + 8;  // 80-byte rows
};
template <>
struct Traits<false> {
  typedef float T;
  static constexpr int LDK = BK + 4;  // 144-byte rows
};

__device__ __forceinline__ float ld1(const void* p, long long idx, int dtype) {
  return dtype == AVC_F32 ? reinterpret_cast<const float*>(p)[idx] : (float)reinterpret_cast<const bf16*>(p)[idx];
}

// window split of a (tap, c) index
__device__ __forceinline__ void split_tap(int x, const OpDev& o, int& tap, int& c) {
  tap = 0;
  for (int j = 1; j < o.taps; ++j) tap += (x >= j * o.chans);
  c = x - tap * o.chans;
}

// K-major operand: thread owns rows (tid>>3)+32i, k offset (tid&7)*4.
struct KMajorState {
  int rowok[4];
  long long rowbase[4];  // plain: r*ld ; window: (b*t_in + t) frame index
  int tt[4];             // window: t
};

__device__ __forceinline__ void kmajor_init(const OpDev& o, int row0, int tid, KMajorState& s) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int r = row0 + (tid >> 3) + 32 * i;
    s.rowok[i] = r < o.rows;
    if (o.win) {
      uint32_t b = fdiv((uint32_t)r, o.tdiv);
      int t = r - (int)b * o.t_out;
      s.tt[i] = t;
      s.rowbase[i] = (long long)b * o.t_in + t;
    } else {
      s.tt[i] = 0;
      s.rowbase[i] = (long long)r * o.ld;
    }
  }
}

__device__ __forceinline__ f32x4 kmajor_elem_load(const OpDev& o, const KMajorState& s, int i, int k, int K,
                                                  long long boff) {
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  if (o.vec) {
    if (!s.rowok[i] || k >= K) return v;
    long long idx;
    if (o.win) {
      int tap, c;
      split_tap(k, o, tap, c);
      int t2 = s.tt[i] + tap - o.pad;
      if (t2 < 0 || t2 >= o.t_in) return v;
      idx = (s.rowbase[i] + tap - o.pad) * o.ld + c;
    } else {
      idx = s.rowbase[i] + k;
    }
    return load4(o.ptr, idx + boff, o.dtype);
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    int kk = k + e;
    if (!s.rowok[i] || kk >= K) continue;
    long long idx;
    if (o.win) {
      int tap, c;
      split_tap(kk, o, tap, c);
      int t2 = s.tt[i] + tap - o.pad;
      if (t2 < 0 || t2 >= o.t_in) continue;
      idx = (s.rowbase[i] + tap - o.pad) * o.ld + c;
    } else {
      idx = s.rowbase[i] + kk;
    }
    v[e] = ld1(o.ptr, idx + boff, o.dtype);
  }
  return v;
}

// K-strided operand: thread owns rows row0+(tid&31)*4 .. +3 and k (tid>>5)*4+j.
struct KStridedState {
  int r;  // first of 4 rows
  int tap, c;
};

__device__ __forceinline__ void kstrided_init(const OpDev& o, int row0, int tid, KStridedState& s) {
  s.r = row0 + (tid & 31) * 4;
  if (o.win) {
    split_tap(s.r, o, s.tap, s.c);
  } else {
    s.tap = 0;
    s.c = s.r;
  }
}

__device__ __forceinline__ f32x4 kstrided_load(const OpDev& o, const KStridedState& s, int k, int K, long long boff) {
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  if (k >= K) return v;
  long long fr = k;
  if (o.vec && o.win) {
    uint32_t b = fdiv((uint32_t)k, o.tdiv);
    int t = k - (int)b * o.t_out;
    int t2 = t + s.tap - o.pad;
    if (t2 < 0 || t2 >= o.t_in) return v;
    fr = (long long)b * o.t_in + t2;
  } else {
    fr = k;
  }
  if (o.vec) {
    if (s.r >= o.rows) return v;
    return load4(o.ptr, fr * o.ld + s.c + boff, o.dtype);
  }
  // scalar path (odd sizes): every element resolves its own (tap, c) and frame.
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    int rr = s.r + e;
    if (rr >= o.rows) continue;
    long long idx;
    if (o.win) {
      int tap2, c2;
      split_tap(rr, o, tap2, c2);
      uint32_t b = fdiv((uint32_t)k, o.tdiv);
      int t3 = k - (int)b * o.t_out + tap2 - o.pad;
      if (t3 < 0 || t3 >= o.t_in) continue;
      idx = ((long long)b * o.t_in + t3) * o.ld + c2;
    } else {
      idx = (long long)k * o.ld + rr;
    }
    v[e] = ld1(o.ptr, idx + boff, o.dtype);
  }
  return v;
}

template <bool BF>
__device__ __forceinline__ void store4(typename Traits<BF>::T* dst, f32x4 v) {
  if constexpr (BF) {
    bf16x4 h = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
    *reinterpret_cast<bf16x4*>(dst) = h;
  } else {
    *reinterpret_cast<f32x4*>(dst) = v;
  }
}

template <bool KS>
struct Loader {
  KMajorState km;
  KStridedState ks;
  f32x4 v[4];

  __device__ __forceinline__ void init(const OpDev& o, int row0, int tid) {
    if constexpr (KS) kstrided_init(o, row0, tid, ks);
    else kmajor_init(o, row0, tid, km);
  }
  __device__ __forceinline__ void load(const OpDev& o, int k0, int kend, int tid, long long boff) {
    if constexpr (KS) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = kstrided_load(o, ks, k0 + (tid >> 5) * 4 + j, kend, boff);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = kmajor_elem_load(o, km, i, k0 + (tid & 7) * 4, kend, boff);
    }
  }
  template <bool BF>
  __device__ __forceinline__ void write(typename Traits<BF>::T* lds, int tid) {
    constexpr int LDK = Traits<BF>::LDK;
    if constexpr (KS) {
      const int r = (tid & 31) * 4, kq = (tid >> 5) * 4;
#pragma unroll
      for (int ri = 0; ri < 4; ++ri) {
        f32x4 w = {v[0][ri], v[1][ri], v[2][ri], v[3][ri]};
        store4<BF>(lds + (r + ri) * LDK + kq, w);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) store4<BF>(lds + ((tid >> 3) + 32 * i) * LDK + (tid & 7) * 4, v[i]);
    }
  }
};

template <bool BF, bool AKS, bool BKS>
__global__ void __launch_bounds__(NT) gemm_generic_kernel(GemmArgs g) {
  typedef typename Traits<BF>::T T;
  constexpr int LDK = Traits<BF>::LDK;
  constexpr int TILE = (BM + BN) * LDK;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* smem = reinterpret_cast<T*>(smem_raw);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
  const int bz = blockIdx.z / g.split_k, ks = blockIdx.z % g.split_k;
  const int kbeg = ks * g.klen;
  const int kend = min(g.K, kbeg + g.klen);
  const long long aoff = (long long)bz * g.a.bstride, boff = (long long)bz * g.b.bstride;

  Loader<AKS> la;
  Loader<BKS> lb;
  la.init(g.a, m0, tid);
  lb.init(g.b, n0, tid);

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nkt = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  if (nkt > 0) {
    la.load(g.a, kbeg, kend, tid, aoff);
    lb.load(g.b, kbeg, kend, tid, boff);
    la.template write<BF>(smem, tid);
    lb.template write<BF>(smem + BM * LDK, tid);
  }
  __syncthreads();

  for (int kt = 0; kt < nkt; ++kt) {
    T* As = smem + (kt & 1) * TILE;
    T* Bs = As + BM * LDK;
    const bool more = kt + 1 < nkt;
    if (more) {
      la.load(g.a, kbeg + (kt + 1) * BK, kend, tid, aoff);
      lb.load(g.b, kbeg + (kt + 1) * BK, kend, tid, boff);
    }
    if constexpr (BF) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(As + (wm * 64 + i * 16 + (lane & 15)) * LDK + 8 * (lane >> 4));
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + (wn * 64 + j * 16 + (lane & 15)) * LDK + 8 * (lane >> 4));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int kk = 0; kk < BK; kk += 4) {
        float af[4], bfr[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = As[(wm * 64 + i * 16 + (lane & 15)) * LDK + kk + (lane >> 4)];
#pragma unroll
        for (int j = 0; j < 4; ++j) bfr[j] = Bs[(wn * 64 + j * 16 + (lane & 15)) * LDK + kk + (lane >> 4)];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
    if (more) {
      T* An = smem + ((kt + 1) & 1) * TILE;
      la.template write<BF>(An, tid);
      lb.template write<BF>(An + BM * LDK, tid);
    }
    __syncthreads();
  }

  // ---------------------------------------------------------------- epilogue
  const int rbase = m0 + wm * 64 + 4 * (lane >> 4);
  const int cbase = n0 + wn * 64 + (lane & 15);
  float* C = g.c + (long long)bz * g.cbs;
  if (g.bias && ks == 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int col = cbase + j * 16;
      float bv = col < g.N ? g.bias[col] : 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i][j] += bv;
    }
  }
  if (g.rbias && ks == 0) add_row_bias<4>(g, acc, rbase, cbase);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      int row = rbase + i * 16 + e;
      if (row >= g.M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        int col = cbase + j * 16;
        if (col >= g.N) continue;
        float* p = C + out_off(g, row, col);
        float v = acc[i][j][e];
        if (g.res && ks == 0) v += g.res[(long long)bz * g.cbs + out_off(g, row, col)];
        if (g.atomic) atomicAdd(p, v);
        else if (g.accumulate) *p += v;
        else *p = v;
      }
    }

  if (g.bn_partial) {
    // Per-column (sum, M2 about the tile mean) over this tile's valid rows.
    float* red = reinterpret_cast<float*>(smem_raw);  // [2][BN]
    const int cnt = min(BM, g.M - m0);
    float s[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
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
      for (int j = 0; j < 4; ++j) red[wm * BN + wn * 64 + j * 16 + lane] = s[j];
    }
    __syncthreads();
    float mean[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int cl = wn * 64 + j * 16 + (lane & 15);
      mean[j] = (red[cl] + red[BN + cl]) / (float)cnt;
    }
    float q[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float t = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float d = acc[i][j][e] - mean[j];
          t += (rbase + i * 16 + e < g.M) ? d * d : 0.f;
        }
      t += __shfl_xor(t, 16, 64);
      t += __shfl_xor(t, 32, 64);
      q[j] = t;
    }
    __syncthreads();
    float* red2 = red + 2 * BN;
    if (lane < 16) {
#pragma unroll
      for (int j = 0; j < 4; ++j) red2[wm * BN + wn * 64 + j * 16 + lane] = q[j];
    }
    __syncthreads();
    if (tid < BN) {
      int col = n0 + tid;
      if (col < g.N) {
        float* p = g.bn_partial + ((long long)blockIdx.y * g.N + col) * 2;
        p[0] = red[tid] + red[BN + tid];
        p[1] = red2[tid] + red2[BN + tid];
      }
    }
  }
}

__global__ void zero2d_kernel(float* c, long long ldc, long long cbs, int M, int N) {
  long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  long long total = (long long)M * N;
  if (idx >= total) return;
  int r = (int)(idx / N), col = (int)(idx % N);
  c[(long long)blockIdx.y * cbs + (long long)r * ldc + col] = 0.f;
}

}  // namespace

// the zero fill of C before an atomic split-K / batch sum (deferred to here for the TT dispatch)
void avcg::gemm_zero_c(GemmArgs& g, hipStream_t s) {
  if (!g.zero_c) return;
  g.zero_c = 0;
  const long long tot = (long long)g.M * g.N;
  dim3 zg(cdiv(tot, 256), g.cbs == 0 ? 1 : g.batch);
  zero2d_kernel<<<zg, 256, 0, s>>>(g.c, g.ldc, g.cbs, g.M, g.N);
}

namespace {

bool aligned4(const void* p, int dtype) {
  uintptr_t a = reinterpret_cast<uintptr_t>(p);
  return dtype == AVC_F32 ? (a % 16 == 0) : (a % 8 == 0);
}

int make_op(const avc_operand& o, int rows, int K, OpDev& d, const char* name) {
  AVC_CHECK_ARG(o.ptr != nullptr, "avc_gemm: operand %s is null", name);
  AVC_CHECK_ARG(o.dtype == AVC_F32 || o.dtype == AVC_BF16, "avc_gemm: operand %s bad dtype", name);
  d.ptr = o.ptr;
  d.ld = o.ld;
  d.bstride = o.batch_stride;
  d.dtype = o.dtype;
  d.win = o.taps > 0;
  d.taps = o.taps > 0 ? o.taps : 1;
  d.pad = o.pad;
  d.t_out = o.t_out > 0 ? o.t_out : 1;
  d.t_in = o.t_in > 0 ? o.t_in : 1;
  d.chans = o.chans > 0 ? o.chans : 1;
  d.rows = rows;
  d.tdiv = make_fastdiv((uint32_t)d.t_out);
  d.cdv = make_fastdiv((uint32_t)d.chans);
  if (d.win) {
    AVC_CHECK_ARG(o.t_out > 0 && o.t_in > 0 && o.chans > 0, "avc_gemm: operand %s window needs t_out/t_in/chans", name);
    int span = d.taps * d.chans;
    AVC_CHECK_ARG(span == (o.kstrided ? rows : K), "avc_gemm: operand %s taps*chans=%d != split dim %d", name, span,
                  o.kstrided ? rows : K);
  }
  int contig = o.kstrided ? rows : K;
  d.vec = (o.ld % 4 == 0) && (contig % 4 == 0) && (o.batch_stride % 4 == 0) && aligned4(o.ptr, o.dtype) &&
          (!d.win || d.chans % 4 == 0);
  return 0;
}


// ============================================================================ fast path
// bf16 MFMA, operands whose contiguous dimension is a multiple of 4 elements.  Loads are
// raw buffer loads: a padding / out-of-range element gets an offset past num_records and
// the hardware returns zeros, so the loader has no branches and all loads of a K-tile are
// in flight together (the generic kernel above serialises them behind exec-masked
// branches).  BK = 64, 2 LDS stages, 2 workgroups per CU, XCD-aware tile order.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
constexpr int FLDK = FBK + 8;  // 144-byte LDS rows
constexpr unsigned FINVALID = 0x7FFFFFF0u;

__device__ __forceinline__ unsigned pk2(float a, float b) {
  bf16x2 h = {(bf16)a, (bf16)b};
  return __builtin_bit_cast(unsigned, h);
}
__device__ __forceinline__ unsigned short lo16(unsigned x) { return (unsigned short)(x & 0xFFFFu); }
__device__ __forceinline__ unsigned short hi16(unsigned x) { return (unsigned short)(x >> 16); }
__device__ __forceinline__ unsigned join16(unsigned short a, unsigned short b) { return (unsigned)a | ((unsigned)b << 16); }

template <int DT>
struct RawT;
template <>
struct RawT<AVC_BF16> {
  typedef u32x2 T;
  static constexpr int ES = 2;
  static __device__ __forceinline__ T load(__amdgpu_buffer_rsrc_t r, unsigned off) {
    return __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0);
  }
  // 4 elements as two packed bf16 pairs
  static __device__ __forceinline__ u32x2 pack(T v) { return v; }
};
template <>
struct RawT<AVC_F32> {
  typedef u32x4 T;
  static constexpr int ES = 4;
  static __device__ __forceinline__ T load(__amdgpu_buffer_rsrc_t r, unsigned off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
  }
  static __device__ __forceinline__ u32x2 pack(T v) {
    return u32x2{pk2(__uint_as_float(v[0]), __uint_as_float(v[1])), pk2(__uint_as_float(v[2]), __uint_as_float(v[3]))};
  }
};

template <int R, bool KS, int DT>
struct FLoader {
  static constexpr int NV = R * FBK / 1024;  // 4-element vectors per thread per K-tile
  static constexpr int NB = NV / 4;          // k-strided: 4x4 blocks per thread
  typedef typename RawT<DT>::T Raw;
  Raw raw[NV];
  __amdgpu_buffer_rsrc_t rsrc;
  // k-major state
  int frame[NV], tt[NV], rok[NV], kq;
  // k-strided state
  int rq[NB > 0 ? NB : 1], kb[NB > 0 ? NB : 1], tap, c, rowok;

  __device__ __forceinline__ void init(const OpDev& o, int row0, int tid, long long boff) {
    const char* base = reinterpret_cast<const char*>(o.ptr) + boff * RawT<DT>::ES;
    rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), (short)0, (int)FINVALID, 0x00020000);
    if constexpr (!KS) {
      kq = (tid & 15) * 4;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int r = row0 + (tid >> 4) + 16 * i;
        rok[i] = r < o.rows;
        if (o.win) {
          const int b = (int)fdiv((uint32_t)r, o.tdiv);
          tt[i] = r - b * o.t_out;
          frame[i] = b * o.t_in + tt[i];
        } else {
          tt[i] = 0;
          frame[i] = r;
        }
      }
    } else {
      constexpr int RQ = R / 4;
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int bi = tid + 256 * j;
        rq[j] = bi % RQ;
        kb[j] = (bi / RQ) * 4;
      }
      const int r = row0 + rq[0] * 4;  // NB > 1 only when RQ divides 256: same rq for every j
      rowok = r < o.rows;
      if (o.win) {
        tap = 0;
        for (int j = 1; j < o.taps; ++j) tap += (r >= j * o.chans);
        c = r - tap * o.chans;
      } else {
        tap = 0;
        c = r;
      }
    }
  }

  __device__ __forceinline__ void load(const OpDev& o, int kbase, int kend) {
    if constexpr (!KS) {
      const int k = kbase + kq;
      int tp = 0, cc = k;
      if (o.win) {
        for (int j = 1; j < o.taps; ++j) tp += (k >= j * o.chans);
        cc = k - tp * o.chans;
      }
      const bool kok = k < kend;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int t2 = tt[i] + tp - o.pad;
        const bool ok = kok && rok[i] && (!o.win || (t2 >= 0 && t2 < o.t_in));
        const unsigned elem = (unsigned)(frame[i] + tp - o.pad) * (unsigned)o.ld + (unsigned)cc;
        raw[i] = RawT<DT>::load(rsrc, ok ? elem * RawT<DT>::ES : FINVALID);
      }
    } else {
#pragma unroll
      for (int j = 0; j < NB; ++j) {
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int k = kbase + kb[j] + jj;
          unsigned elem;
          bool ok = rowok && k < kend;
          if (o.win) {
            const int b = (int)fdiv((uint32_t)k, o.tdiv);
            const int t2 = k - b * o.t_out + tap - o.pad;
            ok = ok && t2 >= 0 && t2 < o.t_in;
            elem = (unsigned)(b * o.t_in + t2) * (unsigned)o.ld + (unsigned)c;
          } else {
            elem = (unsigned)k * (unsigned)o.ld + (unsigned)c;
          }
          raw[4 * j + jj] = RawT<DT>::load(rsrc, ok ? elem * RawT<DT>::ES : FINVALID);
        }
      }
    }
  }

  __device__ __forceinline__ void write(bf16* lds, int tid) {
    if constexpr (!KS) {
#pragma unroll
      for (int i = 0; i < NV; ++i)
        *reinterpret_cast<u32x2*>(lds + ((tid >> 4) + 16 * i) * FLDK + kq) = RawT<DT>::pack(raw[i]);
    } else {
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        u32x2 p[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) p[jj] = RawT<DT>::pack(raw[4 * j + jj]);
        // p[jj] = rows (r0 r1 | r2 r3) at k = kb+jj  ->  row ri: k0..k3
        const u32x2 r0 = {join16(lo16(p[0][0]), lo16(p[1][0])), join16(lo16(p[2][0]), lo16(p[3][0]))};
        const u32x2 r1 = {join16(hi16(p[0][0]), hi16(p[1][0])), join16(hi16(p[2][0]), hi16(p[3][0]))};
        const u32x2 r2 = {join16(lo16(p[0][1]), lo16(p[1][1])), join16(lo16(p[2][1]), lo16(p[3][1]))};
        const u32x2 r3 = {join16(hi16(p[0][1]), hi16(p[1][1])), join16(hi16(p[2][1]), hi16(p[3][1]))};
        bf16* d = lds + (rq[j] * 4) * FLDK + kb[j];
        *reinterpret_cast<u32x2*>(d) = r0;
        *reinterpret_cast<u32x2*>(d + FLDK) = r1;
        *reinterpret_cast<u32x2*>(d + 2 * FLDK) = r2;
        *reinterpret_cast<u32x2*>(d + 3 * FLDK) = r3;
      }
    }
  }
};

template <int BN_, bool AKS, bool BKS, int ADT, int BDT>
__global__ void __launch_bounds__(256, 2) gemm_fast_kernel(GemmArgs g) {
  constexpr int NJ = BN_ / 32;  // 16-wide MFMA column tiles per wave
  constexpr int WN = BN_ / 2;   // wave tile columns
  constexpr int TILE = (BM + BN_) * FLDK;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16* smem = reinterpret_cast<bf16*>(smem_raw);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  // XCD-aware bijective remap: blocks that share an A row-panel run on one XCD's L2.
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

  FLoader<BM, AKS, ADT> la;
  FLoader<BN_, BKS, BDT> lb;
  la.init(g.a, m0, tid, (long long)bz * g.a.bstride);
  lb.init(g.b, n0, tid, (long long)bz * g.b.bstride);

  f32x4 acc[4][NJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nkt = kend > kbeg ? (kend - kbeg + FBK - 1) / FBK : 0;
  if (nkt > 0) {
    la.load(g.a, kbeg, kend);
    lb.load(g.b, kbeg, kend);
    la.write(smem, tid);
    lb.write(smem + BM * FLDK, tid);
  }
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const bf16* As = smem + (kt & 1) * TILE;
    const bf16* Bs = As + BM * FLDK;
    const bool more = kt + 1 < nkt;
    if (more) {
      la.load(g.a, kbeg + (kt + 1) * FBK, kend);
      lb.load(g.b, kbeg + (kt + 1) * FBK, kend);
    }
#pragma unroll
    for (int kk = 0; kk < FBK; kk += 32) {
      bf16x8 af[4], bfr[NJ];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(As + (wm * 64 + i * 16 + (lane & 15)) * FLDK + kk + 8 * (lane >> 4));
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + (wn * WN + j * 16 + (lane & 15)) * FLDK + kk + 8 * (lane >> 4));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      bf16* An = smem + ((kt + 1) & 1) * TILE;
      la.write(An, tid);
      lb.write(An + BM * FLDK, tid);
    }
    __syncthreads();
  }

  fast_epilogue<BN_, !AKS && !BKS>(g, acc, m0, n0, mt, bz, ks, smem_raw);  // bnb: non-TT layouts only
}

template <int BN_, bool AKS, bool BKS, int ADT, int BDT>
void launch_fast(const GemmArgs& g, int nblocks, hipStream_t s) {
  const size_t lds = 2 * (BM + BN_) * FLDK * sizeof(bf16);
  static bool attr = false;  // > 64 KiB of dynamic LDS must be opted into once per kernel
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_fast_kernel<BN_, AKS, BKS, ADT, BDT>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  gemm_fast_kernel<BN_, AKS, BKS, ADT, BDT><<<nblocks, 256, lds, s>>>(g);
}

template <int BN_, bool AKS, bool BKS>
void launch_fast_dt(const GemmArgs& g, int nblocks, hipStream_t s) {
  const bool af = g.a.dtype == AVC_F32, bfl = g.b.dtype == AVC_F32;
  if (af && bfl) launch_fast<BN_, AKS, BKS, AVC_F32, AVC_F32>(g, nblocks, s);
  else if (af) launch_fast<BN_, AKS, BKS, AVC_F32, AVC_BF16>(g, nblocks, s);
  else if (bfl) launch_fast<BN_, AKS, BKS, AVC_BF16, AVC_F32>(g, nblocks, s);
  else launch_fast<BN_, AKS, BKS, AVC_BF16, AVC_BF16>(g, nblocks, s);
}

template <int BN_>
void launch_fast_layout(const GemmArgs& g, bool aks, bool bks, int nblocks, hipStream_t s) {
  if (!aks && !bks) launch_fast_dt<BN_, false, false>(g, nblocks, s);
  else if (!aks && bks) launch_fast_dt<BN_, false, true>(g, nblocks, s);
  else if (aks && !bks) launch_fast_dt<BN_, true, false>(g, nblocks, s);
  else launch_fast_dt<BN_, true, true>(g, nblocks, s);
}

bool fits32(const OpDev& o, int rows, int K, bool ks) {
  // largest element offset the 32-bit buffer addressing can see
  long long frames = o.win ? (long long)((ks ? K : rows) / (o.t_out > 0 ? o.t_out : 1) + 1) * o.t_in : (ks ? K : rows);
  long long span = frames * o.ld + (ks ? rows : K) + o.ld;
  return span * (o.dtype == AVC_F32 ? 4 : 2) < (long long)FINVALID - 64;
}

}  // namespace

static int bn_finalize_after(const GemmArgs& g, const avc_bn_fin* f, void* stream) {
  for (int k = 0; k < f->nupd; ++k)
    if (avc_bn_finalize(g.bn_partial, g.M, g.N, f->gamma, f->beta, f->running_mean, f->running_var,
                        f->num_batches_tracked, f->momentum, f->eps, f->mean, f->rstd, f->scale, f->shift, stream))
      return -1;
  return 0;
}

// avc_gemm_bnb off the fused epilogue: the same reduction as a pass over the GEMM's output
static int bnb_after(const avc_gemm_desc* d, const avc_bnb_args* bb, hipStream_t s) {
  const avcbn::BwdFin fin{bb->gamma, bb->beta, bb->mean, bb->rstd, bb->coef, bb->dgamma, bb->dbeta, bb->dbias,
                          bb->accumulate};
  AVC_CHECK_ARG(d->ldc == d->N, "avc_gemm_bnb: the unfused fallback needs ldc == N");
  const void* out = d->c ? (const void*)d->c : d->c_bf16;
  return avcbn::bn_bwd_reduce_finalize(out, d->c ? AVC_F32 : AVC_BF16, bb->y, bb->y_dtype, d->M, d->N, bb->act, bb->ws,
                                       fin, s);
}

// The BatchNorm apply outputs of avc_gemm_bn / avc_gemm_bnb when the GEMM's epilogue did not write
// them (every kernel but the halo conv ring): the apply passes after the statistics
static int bn_apply_after(const avc_gemm_desc* d, const avc_bn_fin* f, const avc_bnb_args* bb, hipStream_t s) {
  const void* y = d->c ? (const void*)d->c : d->c_bf16;
  const int ydt = d->c ? AVC_F32 : AVC_BF16;
  if (f && f->apply_bf16)
    return avc_bn_apply(y, ydt, f->scale, f->shift, nullptr, nullptr, f->apply_bf16, d->M, d->N, f->apply_act, s);
  if (bb && bb->dy_bf16)
    return avc_bn_bwd_apply(y, ydt, bb->y, bb->y_dtype, bb->coef, d->M, d->N, bb->act, nullptr, bb->dy_bf16, s);
  return 0;
}

// The fused GELU / column-sum epilogues (avc_gemm_desc.c_bf16_act / act_grad_of / col_sum) exist in
// the ring kernels only; the other kernels store the plain product (fp32 C and / or bf16: the
// pre-activation slot, or the bf16 C itself when there is no fp32 C) and one pass follows.
struct GeluPost {
  int act = 0;
  const void* agrad = nullptr;
  int agrad16 = 0;
  bf16* c16 = nullptr;
  bf16* pre16 = nullptr;
  float* csum = nullptr;
  int csum_n = 0;
};
static GeluPost strip_gelu(GemmArgs& g) {
  GeluPost p;
  p.csum = g.csum;
  p.csum_n = g.csum_n;
  g.csum = nullptr;
  if (g.c16_act) {  // product -> c (fp32) and the bf16 pre-activation slot; c16 = GELU(that) after
    p.act = g.c16_act;
    p.c16 = g.c16;
    p.pre16 = g.c16pre;
    g.c16 = g.c16pre;
  } else if (g.agrad) {  // product -> c, or (no fp32 C) the bf16 C; scaled by GELU' after
    p.agrad = g.agrad;
    p.agrad16 = g.agrad16;
    p.c16 = g.c16;
    if (g.c) g.c16 = nullptr;
  }
  g.c16_act = 0;
  g.agrad = nullptr;
  g.c16pre = nullptr;
  return p;
}
// act: c16[i] = GELU(src[i]) (and pre16[i] = src[i] in bf16 when given); else c[i] / c16[i] =
// src[i] * GELU'(agr[i]) (src may alias either)
template <typename TS>
__global__ void gelu_post_kernel(const TS* src, const void* agr, int agr16, float* c, bf16* c16, long long n,
                                 int act, bf16* pre16) {
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    float x = (float)src[i];
    if (act) {
      c16[i] = (bf16)gelu_f(x);
      if (pre16) pre16[i] = (bf16)x;
      continue;
    }
    x *= gelu_grad_f(agr16 ? (float)static_cast<const bf16*>(agr)[i] : static_cast<const float*>(agr)[i]);
    if (c) c[i] = x;
    if (c16) c16[i] = (bf16)x;
  }
}
// column sums of C (rows ldc apart) added into out[n], n < nc: 256 columns x 64 rows per block
template <typename T>
__global__ void colsum_atomic_kernel(const T* c, long long ldc, int M, int nc, float* out) {
  const int col = blockIdx.x * 256 + threadIdx.x, r0 = blockIdx.y * 64;
  if (col >= nc) return;
  float s = 0.f;
  for (int r = r0; r < min(M, r0 + 64); ++r) s += (float)c[(long long)r * ldc + col];
  atomicAdd(out + col, s);
}
// the slotted column sums (GemmArgs::csum_ws) into csum, leaving the slots zeroed for the next user
__global__ void colsum_slots_kernel(float* ws, int slots, int nc, float* csum) {
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col >= nc) return;
  float s = 0.f;
  for (int k = 0; k < slots; ++k) {
    s += ws[(long long)k * nc + col];
    ws[(long long)k * nc + col] = 0.f;
  }
  csum[col] += s;
}
// write_pre: the product kernel wrote fp32 C only (generic kernel): the bf16 pre-activation slot of a
// fused GELU is filled here from C
static int gelu_after(const GemmArgs& g, const GeluPost& p, hipStream_t s, bool write_pre = false) {
  const long long n = (long long)g.M * g.N * g.batch;
  const int blocks = (int)(n / 256 + 1 < 8192 ? n / 256 + 1 : 8192);
  if (p.act || p.agrad) {
    if (g.c) gelu_post_kernel<float><<<blocks, 256, 0, s>>>(g.c, p.agrad, p.agrad16, p.agrad ? g.c : nullptr, p.c16, n,
                                                           p.act, write_pre ? p.pre16 : nullptr);
    else gelu_post_kernel<bf16><<<blocks, 256, 0, s>>>(p.act ? p.pre16 : p.c16, p.agrad, p.agrad16, nullptr, p.c16, n,
                                                       p.act, nullptr);
    if (avc_check_launch("avc_gemm(gelu)")) return -1;
  }
  if (p.csum) {
    const int nc = p.csum_n > 0 ? p.csum_n : g.N, rows = g.M * g.batch;
    const dim3 grid(cdiv(nc, 256), cdiv(rows, 64));
    if (g.c) colsum_atomic_kernel<float><<<grid, 256, 0, s>>>(g.c, g.ldc, rows, nc, p.csum);
    else colsum_atomic_kernel<bf16><<<grid, 256, 0, s>>>(p.c16 ? p.c16 : g.c16, g.ldc, rows, nc, p.csum);
    return avc_check_launch("avc_gemm(col_sum)");
  }
  return 0;
}

static int gemm_impl(const avc_gemm_desc* d, const avc_bn_fin* f, void* stream, const avc_bnb_args* bb = nullptr) {
  AVC_CHECK_ARG(d != nullptr, "avc_gemm: null desc");
  AVC_CHECK_ARG(d->M >= 0 && d->N >= 0 && d->K >= 0, "avc_gemm: negative dims");
  if (d->M == 0 || d->N == 0) return 0;
  AVC_CHECK_ARG(d->c != nullptr || d->c_bf16 != nullptr, "avc_gemm: null C");
  GemmArgs g;
  g.M = d->M;
  g.N = d->N;
  g.K = d->K;
  g.batch = d->batch > 0 ? d->batch : 1;
  g.split_k = d->split_k > 1 ? d->split_k : 1;
  if (make_op(d->a, d->M, d->K, g.a, "A")) return -1;
  if (make_op(d->b, d->N, d->K, g.b, "B")) return -1;
  // A batch of products that share B (no B batch stride) with contiguous A and C batches is ONE
  // product of batch*M rows: one tile grid without a per-batch row-tile remainder (the MetaConv
  // token-mixing products, 64 x 344 rows: 3 x 128-row tiles per utterance -> 172 for all)
  if (g.batch > 1 && g.split_k == 1 && !d->a.kstrided && !g.a.win && d->b.batch_stride == 0 && d->ldc > 0 &&
      d->a.batch_stride == (long long)d->M * d->a.ld && d->c_batch_stride == (long long)d->M * d->ldc &&
      (long long)d->M * g.batch < (1ll << 30)) {
    g.M = d->M * g.batch;
    g.a.rows = g.M;
    g.a.bstride = 0;
    g.batch = 1;
  }
  int kl = (d->K + g.split_k - 1) / g.split_k;
  kl = ((kl + BK - 1) / BK) * BK;
  g.klen = kl > 0 ? kl : BK;
  g.c = d->c;
  g.c16 = reinterpret_cast<bf16*>(d->c_bf16);
  g.res = d->residual;
  g.ldc = d->ldc;
  g.cbs = d->c_batch_stride;
  g.bias = d->bias;
  g.accumulate = d->accumulate;
  // split-K partials, or a batch whose outputs all land in one C (c_batch_stride == 0: a sum
  // over the batch, e.g. a weight gradient of a per-utterance product), accumulate atomically
  g.atomic = g.split_k > 1 || (g.batch > 1 && d->c_batch_stride == 0);
  g.bn_partial = d->bn_partial;
  g.cperm = d->cperm > 1 ? d->cperm : 0;
  AVC_CHECK_ARG(!g.cperm || (d->N % g.cperm == 0 && !g.bias && !g.res && !g.c16 && !g.bn_partial),
                "avc_gemm: cperm needs N %% taps == 0 and no bias / residual / bf16 / BN epilogue");
  g.cpd = make_fastdiv(g.cperm ? (uint32_t)(d->N / g.cperm) : 1u);
  g.c16_act = d->c_bf16_act;
  g.agrad = d->act_grad_of;
  g.agrad16 = d->act_grad_dtype == AVC_BF16;
  g.c16pre = reinterpret_cast<bf16*>(d->c_pre_bf16);
  g.csum = d->col_sum;
  g.csum_n = d->col_sum_n;
  g.csum_ws = nullptr;
  g.csum_slots = 1;
  g.ctr = d->c_trans_rows;
  AVC_CHECK_ARG(g.ctr == 0 || (g.ctr > 0 && g.ctr % 4 == 0 && d->M % g.ctr == 0 && d->ldc == d->N && d->c &&
                               !d->a.kstrided && !d->b.kstrided &&
                               !d->c_bf16 && !d->cperm && !d->bn_partial && !bb &&
                               !g.c16_act && !g.agrad && !g.csum && !d->row_bias && g.split_k == 1 &&
                               (g.batch == 1 || d->c_batch_stride == (long long)d->M * d->N)),
                "avc_gemm: c_trans_rows needs rows %% 4 == 0 dividing M, an fp32 C with ldc == N and no bf16 / BN / "
                "GELU / col_sum / row-bias / cperm / split-K / batch-sum epilogue");
  AVC_CHECK_ARG(d->act_grad_dtype == AVC_F32 || d->act_grad_dtype == AVC_BF16, "avc_gemm: bad act_grad_dtype");
  AVC_CHECK_ARG(!g.csum || (!d->accumulate && g.split_k == 1 && !d->cperm &&
                            (g.batch == 1 || d->c_batch_stride == (long long)d->M * d->ldc) &&
                            d->col_sum_n >= 0 && d->col_sum_n <= d->N && !(g.c16_act && !d->c)),
                "avc_gemm: col_sum needs no accumulate / split-K / batch sum / cperm, col_sum_n <= N (and an fp32 "
                "C with c_bf16_act)");
  AVC_CHECK_ARG(g.c16_act == 0 || g.c16_act == AVC_ACT_GELU, "avc_gemm: c_bf16_act must be 0 or AVC_ACT_GELU");
  AVC_CHECK_ARG(!g.c16pre || g.c16_act, "avc_gemm: c_pre_bf16 needs c_bf16_act");
  AVC_CHECK_ARG(!(g.c16_act && g.agrad), "avc_gemm: c_bf16_act and act_grad_of are exclusive");
  AVC_CHECK_ARG(!(g.c16_act || g.agrad) ||
                    (d->ldc == d->N && (g.batch == 1 || d->c_batch_stride == (long long)d->M * d->N) &&
                     !d->accumulate && g.split_k == 1 &&
                     !d->cperm && !d->bn_partial && !bb && (!g.agrad || !d->residual) &&
                     (!g.c16_act || (d->c_bf16 && (d->c || g.c16pre)))),
                "avc_gemm: the fused GELU epilogues need ldc == N, no accumulate / split-K / batch sum / cperm / BN "
                "epilogues (act_grad_of: no residual; c_bf16_act: c_bf16 and c or c_pre_bf16 set)");
  g.rbias = d->row_bias;
  g.rb_t = d->rb_t;
  g.rb_pad = d->rb_pad;
  g.rb_div = make_fastdiv(d->row_bias && d->rb_t > 0 ? (uint32_t)d->rb_t : 1u);
  AVC_CHECK_ARG(!g.rbias || (d->rb_t > 2 * d->rb_pad && d->rb_pad >= 0 && d->M % d->rb_t == 0 && !g.cperm &&
                             g.batch == 1 && !d->a.kstrided && !d->b.kstrided),
                "avc_gemm: row_bias needs rb_t > 2 rb_pad, M %% rb_t == 0, batch 1, no cperm, non-K-strided operands");
  g.bn_cnt = nullptr;
  g.bn_rows = 0;
  g.bnb_ws = nullptr;
  g.bnb_cnt = nullptr;
  g.bnb_y = nullptr;
  g.bnb_ydt = AVC_F32;
  g.bnb_act = 0;
  g.bnb_fin = avcbn::BwdFin{};
  AVC_CHECK_ARG(!(f && f->apply_bf16) || (d->ldc == d->N && g.batch == 1 && !d->residual),
                "avc_gemm_bn: apply_bf16 needs ldc == N, batch 1, no residual");
  AVC_CHECK_ARG(!(bb && bb->dy_bf16) || d->ldc == d->N, "avc_gemm_bnb: dy_bf16 needs ldc == N");
  if (f) {
    AVC_CHECK_ARG(g.bn_partial && f->mean && f->rstd && f->scale && f->shift && f->nupd >= 1 &&
                      (!f->running_mean == !f->running_var),
                  "avc_gemm_bn: needs bn_partial, mean / rstd / scale / shift, nupd >= 1");
    g.bn_gamma = f->gamma;
    g.bn_beta = f->beta;
    g.bn_rmean = f->running_mean;
    g.bn_rvar = f->running_var;
    g.bn_nbt = f->num_batches_tracked;
    g.bn_mean = f->mean;
    g.bn_rstd = f->rstd;
    g.bn_scale = f->scale;
    g.bn_shift = f->shift;
    g.bn_momentum = f->momentum;
    g.bn_eps = f->eps;
    g.bn_nupd = f->nupd;
  }
  AVC_CHECK_ARG(!(g.bn_partial && (g.split_k > 1 || g.batch > 1 || d->accumulate)),
                "avc_gemm: bn_partial needs split_k == 1, batch == 1, accumulate == 0");
  AVC_CHECK_ARG(g.c || (!g.atomic && !d->accumulate && !g.cperm),
                "avc_gemm: a bf16-only C (c == NULL) cannot accumulate, split K, sum a batch or permute");
  hipStream_t s = as_stream(stream);
  AVC_CHECK_ARG(!(g.res && g.atomic && g.batch > 1 && d->c_batch_stride == 0),
                "avc_gemm: residual with a batch-summed output is not supported");
  const bool bf = d->compute == AVC_BF16;
  const bool aks = d->a.kstrided != 0, bks = d->b.kstrided != 0;
  g.sk_ws = nullptr;
  g.sk_cnt = nullptr;
  g.zero_c = g.atomic && !d->accumulate;
  // a TT product may reduce its split-K partials without atomics (gemm_tt_launch): its zero fill
  // waits for that decision; every other path zeroes now
  if (!(bf && aks && bks)) gemm_zero_c(g, s);
  if (bf && g.a.vec && g.b.vec && fits32(g.a, g.M, g.K, aks) && fits32(g.b, g.N, g.K, bks)) {
    // re-split K in units of the fast kernel's BK
    int klf = (d->K + g.split_k - 1) / g.split_k;
    g.klen = ((klf + FBK - 1) / FBK) * FBK;
    if (g.klen <= 0) g.klen = FBK;
    if (f) {  // the BN finalize rides on the fast kernels' epilogue (one counter per 64 columns)
      g.bn_cnt = avc_counter_slots(cdiv(g.N, 32), s);  // one per column tile (tiles >= 32 columns)
      if (!g.bn_cnt) return -1;
    }
    const bool bnb_fused = bb && !aks && !bks;  // every non-TT fast kernel runs fast_epilogue
    if (bnb_fused) {
      g.bnb_ws = bb->ws;
      g.bnb_y = bb->y;
      g.bnb_ydt = bb->y_dtype;
      g.bnb_act = bb->act;
      g.bnb_fin = avcbn::BwdFin{bb->gamma, bb->beta, bb->mean, bb->rstd, bb->coef, bb->dgamma, bb->dbeta, bb->dbias,
                                bb->accumulate};
      g.bnb_cnt = avc_counter_slots(cdiv(g.N, 32), s);  // one per column tile (tiles >= 32 columns)
      if (!g.bnb_cnt) return -1;
    }
    const char* what = "avc_gemm(fast)";
    GeluPost post;
    if (g.csum && (long long)g.M * g.batch >= 4096) {
      const int nc = g.csum_n > 0 ? g.csum_n : g.N;
      g.csum_slots = 32;
      g.csum_ws = avc_zero_slots(g.csum_slots * nc, s);  // null: the direct atomics
    }
    const bool ring = !aks && !bks && gemm_ring_launch(g, s);
    if (ring) what = "avc_gemm(ring)";
    else post = strip_gelu(g);  // the other kernels have no GELU epilogue: a pass after them
    if (ring) {
    } else if (!aks && !bks && gemm_conv_launch(g, s)) what = "avc_gemm(conv)";
    else if (!aks && !bks && gemm_nt_launch(g, s)) what = "avc_gemm(nt)";
    else if (aks && bks && gemm_tt_launch(g, s)) what = "avc_gemm(tt)";
    else {
      gemm_zero_c(g, s);
      const long long t128 = (long long)cdiv(g.M, BM) * cdiv(g.N, 128) * g.batch * g.split_k;
      const bool narrow = g.N <= 64 || t128 < 384;
      const int nb = narrow ? cdiv(g.M, BM) * cdiv(g.N, 64) * g.batch * g.split_k : (int)t128;
      if (narrow) launch_fast_layout<64>(g, aks, bks, nb, s);
      else launch_fast_layout<128>(g, aks, bks, nb, s);
    }
    if (avc_check_launch(what)) return -1;
    if (ring && g.csum_ws) {
      const int nc = g.csum_n > 0 ? g.csum_n : g.N;
      colsum_slots_kernel<<<cdiv(nc, 256), 256, 0, s>>>(g.csum_ws, g.csum_slots, nc, g.csum);
      if (avc_check_launch("avc_gemm(col_sum slots)")) return -1;
    }
    if (gelu_after(g, post, s)) return -1;
    if (bb && !bnb_fused && bnb_after(d, bb, s)) return -1;
    if (f && !g.bn_cnt && bn_finalize_after(g, f, stream)) return -1;
    return bn_apply_after(d, f, bb, s);
  }
  gemm_zero_c(g, s);
  const GeluPost post = strip_gelu(g);
  // the generic kernel writes fp32 C only: a bf16 output is produced afterwards from C by the GELU
  // pass (fused GELU / GELU' epilogues), so C must exist and a plain bf16 twin is refused
  AVC_CHECK_ARG(!g.c16 || post.c16, "avc_gemm: c_bf16 output needs the fast path (bf16 compute, vectorisable operands)");
  AVC_CHECK_ARG(g.c != nullptr,
                "avc_gemm: a bf16-only output (no fp32 c) needs the fast path (bf16 compute, vectorisable operands)");
  g.c16 = nullptr;  // written by gelu_after from C
  static const bool trace_generic = getenv("AVC_GEMM_TRACE") != nullptr;
  if (trace_generic && bf)
    fprintf(stderr, "avc_gemm generic: M=%d N=%d K=%d batch=%d split=%d aks=%d bks=%d avec=%d bvec=%d awin=%d chans=%d\n",
            g.M, g.N, g.K, g.batch, g.split_k, (int)aks, (int)bks, (int)g.a.vec, (int)g.b.vec, (int)g.a.win,
            g.a.chans);
  dim3 grid(cdiv(g.N, BN), cdiv(g.M, BM), g.batch * g.split_k);
  size_t lds = bf ? 2 * (BM + BN) * Traits<true>::LDK * sizeof(bf16) : 2 * (BM + BN) * Traits<false>::LDK * sizeof(float);
#define AVC_GEMM_LAUNCH(BFV, A, B) gemm_generic_kernel<BFV, A, B><<<grid, NT, lds, s>>>(g)
  if (bf) {
    if (!aks && !bks) AVC_GEMM_LAUNCH(true, false, false);
    else if (!aks && bks) AVC_GEMM_LAUNCH(true, false, true);
    else if (aks && !bks) AVC_GEMM_LAUNCH(true, true, false);
    else AVC_GEMM_LAUNCH(true, true, true);
  } else {
    if (!aks && !bks) AVC_GEMM_LAUNCH(false, false, false);
    else if (!aks && bks) AVC_GEMM_LAUNCH(false, false, true);
    else if (aks && !bks) AVC_GEMM_LAUNCH(false, true, false);
    else AVC_GEMM_LAUNCH(false, true, true);
  }
#undef AVC_GEMM_LAUNCH
  if (avc_check_launch("avc_gemm")) return -1;
  if (gelu_after(g, post, s, true)) return -1;
  if (bb && bnb_after(d, bb, s)) return -1;
  if (f && bn_finalize_after(g, f, stream)) return -1;  // generic kernels: finalize launch(es) after the GEMM
  return bn_apply_after(d, f, bb, s);
}

extern "C" int avc_gemm(const avc_gemm_desc* d, void* stream) { return gemm_impl(d, nullptr, stream); }

extern "C" size_t avc_gemm_bnb_ws(int M, int N) {
  // fused: cdiv(M, 128) row tiles; fallback pass: cdiv(M, 64) row blocks; 3 sums each
  return (size_t)cdiv(M, 64) * N * 3;
}

extern "C" int avc_gemm_bnb(const avc_gemm_desc* d, const avc_bnb_args* bb, void* stream) {
  AVC_CHECK_ARG(d != nullptr && bb != nullptr, "avc_gemm_bnb: null args");
  AVC_CHECK_ARG(bb->y && bb->mean && bb->rstd && bb->coef && bb->ws && (bb->y_dtype == AVC_F32 || bb->y_dtype == AVC_BF16),
                "avc_gemm_bnb: needs y, mean, rstd, coef, ws");
  AVC_CHECK_ARG(d->batch <= 1 && d->split_k <= 1 && !d->accumulate && !d->residual && !d->cperm && !d->bias &&
                    !d->bn_partial,
                "avc_gemm_bnb: a plain single product (no split K, batch, accumulate, residual, bias, BN stats)");
  AVC_CHECK_ARG((reinterpret_cast<uintptr_t>(bb->coef) & 15) == 0, "avc_gemm_bnb: coef must be 16-B aligned");
  return gemm_impl(d, nullptr, stream, bb);
}

extern "C" int avc_gemm_bn(const avc_gemm_desc* d, const avc_bn_fin* f, void* stream) {
  AVC_CHECK_ARG(f != nullptr, "avc_gemm_bn: null finalize args");
  return gemm_impl(d, f, stream);
}
