// elem.hip — layout glue, weight repacks, losses and the fused Adam step.
//
// Glue replaces the tensor reshuffles of factory/AutoVC.py: input concat with the
// broadcast speaker embedding (:46-48), code extraction (:56-66) and expansion + concat
// (:197-204).  Losses replace F.mse_loss / F.l1_loss of train.py:85-86,94 and Adam
// replaces torch.optim.Adam (train.py:49,99).
#include <cstdarg>
#include <cstdio>

#include "common.h"

static thread_local char g_err[512] = "";

void avc_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int avc_check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    avc_set_error("%s: %s", what, hipGetErrorString(e));
    return -2;
  }
  return 0;
}

extern "C" int avc_abi_version(void) { return AVC_ABI_VERSION; }
extern "C" const char* avc_last_error(void) { return g_err; }

namespace {

__global__ void enc_concat_kernel(const float* mel, long long mel_ld, const float* emb, float* out, int B, int T,
                                  int nm, int de) {
  const int C = nm + de;
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  long long total = (long long)B * T * C;
  if (i >= total) return;
  int c = (int)(i % C);
  long long f = i / C;
  int b = (int)(f / T);
  out[i] = c < nm ? mel[f * mel_ld + c] : emb[(long long)b * de + (c - nm)];
}

__global__ void codes_gather_kernel(const float* lo, float* codes, int B, int T, int D, int freq) {
  const int nc = T / freq, W = 2 * D;
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)B * nc * W) return;
  int c = (int)(i % W);
  int k = (int)((i / W) % nc);
  int b = (int)(i / ((long long)W * nc));
  int t = c < D ? k * freq + freq - 1 : k * freq;
  codes[i] = lo[((long long)b * T + t) * W + c];
}

__global__ void codes_scatter_kernel(const float* dcodes, float* dlo, int B, int T, int D, int freq) {
  const int nc = T / freq, W = 2 * D;
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)B * T * W) return;
  int c = (int)(i % W);
  int t = (int)((i / W) % T);
  int b = (int)(i / ((long long)W * T));
  int k = t / freq, r = t - k * freq;
  bool hit = c < D ? (r == freq - 1) : (r == 0);
  dlo[i] = hit ? dcodes[((long long)b * nc + k) * W + c] : 0.f;
}

__global__ void dec_concat_kernel(const float* codes, const float* emb, float* out, int B, int T, int nc, int cd,
                                  int de) {
  const int C = cd + de;
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)B * T * C) return;
  int c = (int)(i % C);
  int t = (int)((i / C) % T);
  int b = (int)(i / ((long long)C * T));
  const int rep = T / nc;
  out[i] = c < cd ? codes[((long long)b * nc + t / rep) * cd + c] : emb[(long long)b * de + (c - cd)];
}

// The decoder LSTM's input projection folded per code and per utterance:
//   out[b*T + t][g] = pc[b*nc + t/rep][g] + pe[b][g]      (rep = T / nc, float4 over g)
// pc = codes . W_ih[:, :cd]^T (one row per code), pe = c_trg . W_ih[:, cd:]^T + b (one row per
// utterance): W_ih . cat(code_expand, c_trg) + b without the (B*T, cd+de) concat or its GEMM.
__global__ void expand_codes_kernel(const f32x4* __restrict__ pc, const f32x4* __restrict__ pe, f32x4* __restrict__ out,
                                    int T, int nc, int G4, long long n4) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  const int g = (int)(i % G4);
  const long long r = i / G4;
  const int t = (int)(r % T), b = (int)(r / T);
  const int rep = T / nc;
  out[i] = pc[((long long)b * nc + t / rep) * G4 + g] + pe[(long long)b * G4 + g];
}

// out[b*nc + j][k] = k < cd ? codes[b][j*cd + k] : emb[b][k - cd], bf16 (avc_code_cat)
__global__ void code_cat_kernel(const float* __restrict__ codes, const float* __restrict__ emb, bf16* __restrict__ out,
                                int nc, int cd, int de, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int C = cd + de;
  const int k = (int)(i % C);
  const long long r = i / C;  // b*nc + j
  const long long b = r / nc;
  out[i] = (bf16)(k < cd ? codes[r * cd + k] : emb[b * de + (k - cd)]);
}

__global__ void dec_concat_bwd_kernel(const float* dout, float* dcodes, int B, int T, int nc, int cd, int de) {
  const int C = cd + de;
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)B * nc * cd) return;
  int c = (int)(i % cd);
  int k = (int)((i / cd) % nc);
  int b = (int)(i / ((long long)cd * nc));
  const int rep = T / nc;
  float s = 0.f;
  for (int t = k * rep; t < (k + 1) * rep; ++t) s += dout[((long long)b * T + t) * C + c];
  dcodes[i] = s;
}

template <typename T>
__device__ __forceinline__ void put(void* dst, long long i, float v);
template <>
__device__ __forceinline__ void put<float>(void* dst, long long i, float v) {
  reinterpret_cast<float*>(dst)[i] = v;
}
template <>
__device__ __forceinline__ void put<bf16>(void* dst, long long i, float v) {
  reinterpret_cast<bf16*>(dst)[i] = (bf16)v;
}

__device__ __forceinline__ void putd(void* dst, long long i, float v, int dtype) {
  if (dtype == AVC_F32) put<float>(dst, i, v);
  else put<bf16>(dst, i, v);
}

__global__ void conv_pack_kernel(const float* w, void* out, int dtype, int Co, int Ci, int K, int mode) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  long long total = (long long)Co * Ci * K;
  if (i >= total) return;
  // i indexes the SOURCE W[co][ci][k]
  int k = (int)(i % K);
  int ci = (int)((i / K) % Ci);
  int co = (int)(i / ((long long)K * Ci));
  long long o = mode == 0 ? ((long long)co * K + k) * Ci + ci : ((long long)ci * K + (K - 1 - k)) * Co + co;
  putd(out, o, w[i], dtype);
}

// Weight-pack units, LDS-staged where the layout changes, 256 threads (round 6: the per-element forms
// scattered 2-B stores Ci or K*Co elements apart -- ~64 B of memory traffic per stored bf16 -- and the
// batched repack ran at ~1 TB/s, 225 us beside the encoder backward for the decoder's weights).  Every
// unit keeps 16 independent loads per thread in flight and needs at most PK_BUF floats of LDS (17 KiB,
// so a pack workgroup still fits beside a conv ring workgroup).  W[co][ci][k] fp32 ->
//   mode 0, Wf[co][k][ci]:     unit = 4 output x 64 input channels (K <= 16; 4 runs of 64*K floats in,
//                              4*K runs of 64 out);
//   mode 1, Wd[ci][K-1-k][co]: unit = 32 output x 16 input channels (K <= 8; 32 runs of 16*K floats in,
//                              16*K runs of 32 out).
constexpr int PK_KMAX_F = 16, PK_KMAX_D = 8, PK_BUF = 64 * 65;
__host__ __device__ constexpr long long conv_pack_units(int Co, int Ci, int mode) {
  return mode == 0 ? (long long)((Co + 3) / 4) * ((Ci + 63) / 64) : (long long)((Co + 31) / 32) * ((Ci + 15) / 16);
}
__device__ void conv_pack_unit(const float* __restrict__ w, void* out, int dtype, int Co, int Ci, int K, int mode,
                               long long u, float* buf) {
  const int tid = threadIdx.x;
  if (mode == 0) {
    const int ncb = (Ci + 63) / 64;
    const int co0 = (int)(u / ncb) * 4, ci0 = (int)(u % ncb) * 64;
    const int n = 4 * 64 * K;
    for (int e = tid; e < n; e += 256) {
      const int r = e / (64 * K), rem = e - r * 64 * K;  // rem = ci_l * K + k
      const int cil = rem / K, k = rem - cil * K;
      const int co = co0 + r, ci = ci0 + cil;
      buf[(r * K + k) * 65 + cil] = (co < Co && ci < Ci) ? w[((long long)co * Ci + ci0) * K + rem] : 0.f;
    }
    __syncthreads();
    for (int e = tid; e < n; e += 256) {
      const int r = e / (64 * K), rem = e - r * 64 * K;  // rem = k * 64 + ci_l
      const int k = rem >> 6, cil = rem & 63;
      const int co = co0 + r, ci = ci0 + cil;
      if (co < Co && ci < Ci) putd(out, ((long long)co * K + k) * Ci + ci, buf[(r * K + k) * 65 + cil], dtype);
    }
  } else {
    const int ncb = (Ci + 15) / 16;
    const int co0 = (int)(u / ncb) * 32, ci0 = (int)(u % ncb) * 16;
    const int n = 32 * 16 * K;
    for (int e = tid; e < n; e += 256) {
      const int r = e / (16 * K), rem = e - r * 16 * K;  // row r = co_l, rem = ci_l * K + k
      const int co = co0 + r, ci = ci0 + rem / K;
      buf[rem * 33 + r] = (co < Co && ci < Ci) ? w[((long long)co * Ci + ci0) * K + rem] : 0.f;
    }
    __syncthreads();
    for (int e = tid; e < n; e += 256) {
      const int q = e >> 5, col = e & 31;  // q = ci_l * K + k
      const int cil = q / K, k = q - cil * K;
      const int ci = ci0 + cil, co = co0 + col;
      if (co < Co && ci < Ci) putd(out, ((long long)ci * K + (K - 1 - k)) * Co + co, buf[q * 33 + col], dtype);
    }
  }
  __syncthreads();  // buf is reused by the caller's next unit
}

__global__ void __launch_bounds__(256) conv_pack_tiled_kernel(const float* w, void* out, int dtype, int Co, int Ci,
                                                              int K, int mode) {
  __shared__ float buf[PK_BUF];
  const long long nu = conv_pack_units(Co, Ci, mode);
  for (long long u = blockIdx.x; u < nu; u += gridDim.x) conv_pack_unit(w, out, dtype, Co, Ci, K, mode, u, buf);
}

__global__ void conv_grad_unpack_kernel(const float* dwf, float* dw, int Co, int Ci, int K, int acc) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  long long total = (long long)Co * Ci * K;
  if (i >= total) return;
  int k = (int)(i % K);
  int ci = (int)((i / K) % Ci);
  int co = (int)(i / ((long long)K * Ci));
  float v = dwf[((long long)co * K + k) * Ci + ci];
  dw[i] = acc ? dw[i] + v : v;
}

__global__ void convert_kernel(const float* src, void* dst, int dtype, long long n) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) putd(dst, i, src[i], dtype);
}

__global__ void transpose_kernel(const float* src, void* dst, int dtype, int R, int C, long long ldo) {
  __shared__ float tile[32][33];
  int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 32 x 8
  for (int y = ty; y < 32; y += 8) {
    int r = r0 + y, c = c0 + tx;
    tile[y][tx] = (r < R && c < C) ? src[(long long)r * C + c] : 0.f;
  }
  __syncthreads();
  for (int y = ty; y < 32; y += 8) {
    int c = c0 + y, r = r0 + tx;  // dst[c][r]
    if (c < C && r < R) putd(dst, (long long)c * ldo + r, tile[tx][y], dtype);
  }
}

__global__ void add_kernel(const float* a, const float* b, float* o, long long n) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) o[i] = a[i] + b[i];
}

__global__ void loss_kernel(const float* a, const float* b, long long n, float* out, int mode) {
  __shared__ float red[4];
  float s = 0.f;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    float d = a[i] - b[i];
    s += mode == 0 ? d * d : fabsf(d);
  }
  s = warp_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out, (red[0] + red[1] + red[2] + red[3]) / (float)n);
}

__global__ void loss_grad_kernel(const float* a, const float* b, long long n, const float* dloss, int mode, float* g,
                                 float sign) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float d = a[i] - b[i];
  float f = mode == 0 ? 2.f * d : (d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f));
  g[i] = sign * dloss[0] * f / (float)n;
}

// The loss block of Solver.train (train.py:84-96) in one launch: grid-stride partial sums of
// (x - y1)^2, (x - y2)^2 over n1 and |ca - cb| over n2 (float4 loads when 16-B aligned), block
// partials handed over with write-through stores, the last-arriving block sums them in block
// order (deterministic, no zeroing launch) and writes the three means and the weighted total.
constexpr int VCL_GRID = 256;
__global__ void __launch_bounds__(256) vc_loss_kernel(const float* __restrict__ x, const float* __restrict__ y1,
                                                      const float* __restrict__ y2, long long n1,
                                                      const float* __restrict__ ca, const float* __restrict__ cb,
                                                      long long n2, float lam, float* out, float* ws, unsigned* cnt,
                                                      int vec) {
  __shared__ float red[3][4];
  float s0 = 0.f, s1 = 0.f, s2 = 0.f;
  const long long stride = (long long)gridDim.x * blockDim.x;
  const long long i0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (vec) {
    const long long q1 = n1 / 4;
    for (long long i = i0; i < q1; i += stride) {
      const f32x4 a = reinterpret_cast<const f32x4*>(x)[i];
      const f32x4 d1 = a - reinterpret_cast<const f32x4*>(y1)[i];
      const f32x4 d2 = a - reinterpret_cast<const f32x4*>(y2)[i];
      s0 += d1[0] * d1[0] + d1[1] * d1[1] + d1[2] * d1[2] + d1[3] * d1[3];
      s1 += d2[0] * d2[0] + d2[1] * d2[1] + d2[2] * d2[2] + d2[3] * d2[3];
    }
    for (long long i = 4 * q1 + i0; i < n1; i += stride) {
      const float d1 = x[i] - y1[i], d2 = x[i] - y2[i];
      s0 += d1 * d1;
      s1 += d2 * d2;
    }
  } else {
    for (long long i = i0; i < n1; i += stride) {
      const float d1 = x[i] - y1[i], d2 = x[i] - y2[i];
      s0 += d1 * d1;
      s1 += d2 * d2;
    }
  }
  for (long long i = i0; i < n2; i += stride) s2 += fabsf(ca[i] - cb[i]);
  s0 = warp_sum(s0);
  s1 = warp_sum(s1);
  s2 = warp_sum(s2);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = s0;
    red[1][w] = s1;
    red[2][w] = s2;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    const float* r = red[threadIdx.x];
    st_sc1(ws + (long long)blockIdx.x * 3 + threadIdx.x, r[0] + r[1] + r[2] + r[3]);
  }
  if (!arrive_last(cnt, gridDim.x)) return;
  // thread t loads block t's three partials (all loads in flight at once; a serial loop of
  // agent-scope loads cost 30 us), then a fixed-order tree: deterministic
  float p0 = 0.f, p1 = 0.f, p2 = 0.f;
  if (threadIdx.x < gridDim.x) {
    const float* q = ws + (long long)threadIdx.x * 3;
    p0 = ld_sc1(q);
    p1 = ld_sc1(q + 1);
    p2 = ld_sc1(q + 2);
  }
  p0 = warp_sum(p0);
  p1 = warp_sum(p1);
  p2 = warp_sum(p2);
  __syncthreads();  // red reused
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = p0;
    red[1][w] = p1;
    red[2][w] = p2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float t0 = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    const float t1 = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    const float t2 = red[2][0] + red[2][1] + red[2][2] + red[2][3];
    const float m0 = t0 / (float)n1, m1 = t1 / (float)n1, m2 = n2 > 0 ? t2 / (float)n2 : 0.f;
    out[0] = m0;
    out[1] = m1;
    out[2] = m2;
    out[3] = m0 + m1 + lam * m2;
  }
}

__device__ __forceinline__ float dval(const float* p) { return p ? *p : 0.f; }

__global__ void vc_loss_grad_kernel(const float* __restrict__ x, const float* __restrict__ y1,
                                    const float* __restrict__ y2, long long n1, const float* __restrict__ ca,
                                    const float* __restrict__ cb, long long n2, float lam, const float* d0,
                                    const float* d1, const float* d2, const float* d3, float* g1, float* g2,
                                    float* ga, float* gb) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const float t3 = dval(d3);
  if (i < n1) {
    const float xv = x[i];
    if (g1) g1[i] = (t3 + dval(d0)) * 2.f * (y1[i] - xv) / (float)n1;
    if (g2) g2[i] = (t3 + dval(d1)) * 2.f * (y2[i] - xv) / (float)n1;
  } else if (i < n1 + n2) {
    const long long k = i - n1;
    const float d = ca[k] - cb[k];
    const float v = (lam * t3 + dval(d2)) * (d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f)) / (float)n2;
    if (ga) ga[k] = v;
    if (gb) gb[k] = -v;
  }
}

// Batched weight packing (avc_pack_batch).  The launch is cut into UNITS: a 64 x 64 tile of a
// transpose or a conv tile (staged through LDS so both the fp32 reads and the bf16 writes are
// coalesced), or 4096 elements of anything else (copy / add: float4 along the source; a channel
// slice of the conv0 fold or an oversized conv: scalar, along the destination / source).
// prefix[i] = first unit of op i; a block finds its op by one block-uniform binary search per
// unit (<= 128 ops).
constexpr int PACK_MAX_OPS = 128;

__device__ __forceinline__ void put4(void* dst, long long i, float4 v, int dtype) {
  if (dtype == AVC_F32) {
    *reinterpret_cast<float4*>(reinterpret_cast<float*>(dst) + i) = v;
  } else {
    *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(dst) + i) = bf16x4{(bf16)v.x, (bf16)v.y, (bf16)v.z, (bf16)v.w};
  }
}
__device__ __forceinline__ bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

__global__ void __launch_bounds__(256) pack_batch_kernel(const avc_pack_op* __restrict__ ops,
                                                         const long long* __restrict__ prefix, int nops,
                                                         long long total) {
  __shared__ float buf[PK_BUF];  // the units' staging (a transpose tile is [64][65])
  __shared__ long long pre[PACK_MAX_OPS + 1];
  __shared__ avc_pack_op sops[PACK_MAX_OPS];
  const int tid = threadIdx.x;
  // the op table and its prefix, once per block: the per-unit search then costs LDS reads only
  for (int i = tid; i <= nops; i += 256) pre[i] = prefix[i];
  for (int i = tid; i < nops; i += 256) sops[i] = ops[i];
  __syncthreads();
  for (long long u = blockIdx.x; u < total; u += gridDim.x) {
    int lo = 0, hi = nops;  // largest i with pre[i] <= u
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (pre[mid] <= u) lo = mid;
      else hi = mid;
    }
    const avc_pack_op& op = sops[lo];
    const long long lu = u - pre[lo];
    if (op.kind == AVC_PACK_TRANSPOSE) {  // dst[c*ld + r] = src[r*C + c], src [R][C]; 64 x 64 tile
      const int R = op.d0, C = op.d1, tcn = (C + 63) / 64;
      const int r0 = (int)(lu / tcn) * 64, c0 = (int)(lu % tcn) * 64;
      const bool v4 = (C & 3) == 0 && al16(op.src);
      // load: 64 rows x 16 float4 = 4 per thread (row = q >> 4, col4 = q & 15), 16 B in flight each
      float4 v[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int q = t * 256 + tid, r = r0 + (q >> 4), c = c0 + 4 * (q & 15);
        if (v4 && r < R && c + 3 < C) {
          v[t] = *reinterpret_cast<const float4*>(op.src + (long long)r * C + c);
        } else {
          float e[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) e[k] = (r < R && c + k < C) ? op.src[(long long)r * C + c + k] : 0.f;
          v[t] = float4{e[0], e[1], e[2], e[3]};
        }
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int q = t * 256 + tid, rl = q >> 4, cl = 4 * (q & 15);
        buf[(cl + 0) * 65 + rl] = v[t].x;
        buf[(cl + 1) * 65 + rl] = v[t].y;
        buf[(cl + 2) * 65 + rl] = v[t].z;
        buf[(cl + 3) * 65 + rl] = v[t].w;
      }
      __syncthreads();
      // store: dst rows c0.. (64 of them), 64 consecutive r each: 4 x 4 elements per thread
      const bool s4 = (op.ld_out & 3) == 0 && al16(op.dst);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int q = t * 256 + tid, cl = q >> 4, rl = 4 * (q & 15);
        const int c = c0 + cl, r = r0 + rl;
        if (c >= C) continue;
        // (65-float LDS rows are 4-B aligned only: four scalar reads)
        const float e0 = buf[cl * 65 + rl], e1 = buf[cl * 65 + rl + 1], e2 = buf[cl * 65 + rl + 2],
                    e3 = buf[cl * 65 + rl + 3];
        const long long o = (long long)c * op.ld_out + r;
        if (s4 && r + 3 < R) {
          put4(op.dst, o, float4{e0, e1, e2, e3}, op.out_dtype);
        } else {
          const float e[4] = {e0, e1, e2, e3};
          for (int k = 0; k < 4 && r + k < R; ++k) putd(op.dst, o + k, e[k], op.out_dtype);
        }
      }
      __syncthreads();  // the tile is reused by the next unit
      continue;
    }
    if (op.kind == AVC_PACK_CONV_F && op.d2 <= PK_KMAX_F) {
      conv_pack_unit(op.src, op.dst, op.out_dtype, op.d0, op.d1, op.d2, 0, lu, buf);
      continue;
    }
    if (op.kind == AVC_PACK_CONV_D && op.d2 <= PK_KMAX_D) {
      conv_pack_unit(op.src, op.dst, op.out_dtype, op.d0, op.d1, op.d2, 1, lu, buf);
      continue;
    }
    if (op.kind == AVC_PACK_CONV_SLICE) {  // avc_conv_pack_slice's layouts, one element per thread-step
      const int Co = op.d0, Ci = op.d1, K = op.d2, cpad = op.cpad, cn = op.cn;
      const long long n = (long long)(op.mode == 3 ? cn : Co) * cpad * K;
#pragma unroll 4
      for (int j = 0; j < 16; ++j) {
        const long long i = lu * 4096 + j * 256 + tid;
        if (i >= n) break;
        putd(op.dst, i, slice_val(op.src, Co, Ci, K, op.ci0, cn, cpad, op.mode, i), op.out_dtype);
      }
      continue;
    }
    const bool conv = op.kind == AVC_PACK_CONV_F || op.kind == AVC_PACK_CONV_D;
    const long long n = conv ? (long long)op.d0 * op.d1 * op.d2 : op.d0;
    if (!conv && al16(op.src) && al16(op.dst) && (op.kind != AVC_PACK_ADD || al16(op.src2))) {
      // COPY / ADD: 4096 elements per unit, 4 float4 per thread (and 4 of src2)
      float4 a[4], b[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const long long i = lu * 4096 + (t * 256 + tid) * 4;
        a[t] = i + 3 < n ? *reinterpret_cast<const float4*>(op.src + i) : float4{0.f, 0.f, 0.f, 0.f};
        b[t] = (op.kind == AVC_PACK_ADD && i + 3 < n) ? *reinterpret_cast<const float4*>(op.src2 + i)
                                                      : float4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const long long i = lu * 4096 + (t * 256 + tid) * 4;
        if (i + 3 < n) {
          put4(op.dst, i, float4{a[t].x + b[t].x, a[t].y + b[t].y, a[t].z + b[t].z, a[t].w + b[t].w}, op.out_dtype);
        } else {
          for (long long k = i; k < n && k < i + 4; ++k)
            putd(op.dst, k, op.src[k] + (op.kind == AVC_PACK_ADD ? op.src2[k] : 0.f), op.out_dtype);
        }
      }
      continue;
    }
#pragma unroll 4
    for (int j = 0; j < 16; ++j) {
      const long long i = lu * 4096 + j * 256 + tid;
      if (i >= n) break;
      float v = op.src[i];
      long long o = i;
      if (op.kind == AVC_PACK_ADD) {
        v += op.src2[i];
      } else if (conv) {  // source W[co][ci][k]
        const int K = op.d2, Ci = op.d1;
        const int ii = (int)i, k = ii % K, ci = (ii / K) % Ci, co = ii / (K * Ci);
        o = op.kind == AVC_PACK_CONV_F ? ((long long)co * K + k) * Ci + ci : ((long long)ci * K + (K - 1 - k)) * op.d0 + co;
      }
      putd(op.dst, o, v, op.out_dtype);
    }
  }
}

__global__ void adam_prep_kernel(float* state, float lr, float beta1, float beta2) {
  float step = state[0] + 1.f;
  state[0] = step;
  double bc1 = 1.0 - pow((double)beta1, (double)step);
  double bc2 = 1.0 - pow((double)beta2, (double)step);
  state[1] = (float)(lr / bc1);
  state[2] = (float)sqrt(bc2);
}

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float beta1, float beta2, float eps,
                                          float step_size, float bc2s) {
  m = m + (1.f - beta1) * (g - m);
  v = v * beta2 + (1.f - beta2) * g * g;
  const float denom = sqrtf(v) / bc2s + eps;
  p = p - step_size * (m / denom);
}

__device__ __forceinline__ void adam_vec(float4& p, const float4& g, float4& m, float4& v, float beta1, float beta2,
                                         float eps, float step_size, float bc2s) {
  adam_elem(p.x, g.x, m.x, v.x, beta1, beta2, eps, step_size, bc2s);
  adam_elem(p.y, g.y, m.y, v.y, beta1, beta2, eps, step_size, bc2s);
  adam_elem(p.z, g.z, m.z, v.z, beta1, beta2, eps, step_size, bc2s);
  adam_elem(p.w, g.w, m.w, v.w, beta1, beta2, eps, step_size, bc2s);
}

// 16-B vectors, two per array in flight per thread and iteration (a capped grid beside other kernels
// still keeps enough bytes in flight); the scalar tail / unaligned form does the same per-element math
__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, long long n, float beta1, float beta2, float eps,
                            const float* __restrict__ state, int vec) {
  const float step_size = state[1], bc2s = state[2];
  const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long stride = (long long)gridDim.x * blockDim.x;
  long long done = 0;
  if (vec) {
    float4* p4 = reinterpret_cast<float4*>(p);
    const float4* g4 = reinterpret_cast<const float4*>(g);
    float4* m4 = reinterpret_cast<float4*>(m);
    float4* v4 = reinterpret_cast<float4*>(v);
    const long long n4 = n >> 2;
    long long i = tid;
    for (; i + stride < n4; i += 2 * stride) {
      float4 ga = g4[i], gb = g4[i + stride];
      float4 ma = m4[i], mb = m4[i + stride];
      float4 va = v4[i], vb = v4[i + stride];
      float4 pa = p4[i], pb = p4[i + stride];
      adam_vec(pa, ga, ma, va, beta1, beta2, eps, step_size, bc2s);
      adam_vec(pb, gb, mb, vb, beta1, beta2, eps, step_size, bc2s);
      m4[i] = ma; m4[i + stride] = mb;
      v4[i] = va; v4[i + stride] = vb;
      p4[i] = pa; p4[i + stride] = pb;
    }
    if (i < n4) {
      float4 ga = g4[i], ma = m4[i], va = v4[i], pa = p4[i];
      adam_vec(pa, ga, ma, va, beta1, beta2, eps, step_size, bc2s);
      m4[i] = ma; v4[i] = va; p4[i] = pa;
    }
    done = n4 << 2;
  }
  for (long long i = done + tid; i < n; i += stride) {
    float pi = p[i], mi = m[i], vi = v[i];
    adam_elem(pi, g[i], mi, vi, beta1, beta2, eps, step_size, bc2s);
    m[i] = mi;
    v[i] = vi;
    p[i] = pi;
  }
}

__global__ void act_fwd_kernel(const float* x, float* y, long long n, int act) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = act_fwd(x[i], act);
}

__global__ void act_bwd_kernel(const float* g, const float* yout, float* dx, long long n, int act) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dx[i] = act_bwd_from_out(g[i], yout[i], act);
}

// nn.BCELoss(mean) on probabilities p against a constant target; log clamped at -100
__global__ void bce_kernel(const float* p, long long n, float target, float* out) {
  __shared__ float red[4];
  float s = 0.f;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float lp = fmaxf(logf(p[i]), -100.f), l1p = fmaxf(logf(1.f - p[i]), -100.f);
    s += -(target * lp + (1.f - target) * l1p);
  }
  s = warp_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out, (red[0] + red[1] + red[2] + red[3]) / (float)n);
}

// d BCE / d p (PyTorch: grad * (p - t) / max(p (1 - p), 1e-12) / n), chained through the
// sigmoid that produced p when `through_sigmoid` (dlogit = dp * p (1 - p)).
__global__ void bce_grad_kernel(const float* p, long long n, float target, const float* dloss, float* g,
                                int through_sigmoid) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float pi = p[i];
  float d = dloss[0] * (pi - target) / fmaxf((1.f - pi) * pi, 1e-12f) / (float)n;
  if (through_sigmoid) d *= pi * (1.f - pi);
  g[i] = d;
}

}  // namespace

#define GRID1(n) dim3(cdiv((n), 256)), dim3(256), 0, as_stream(stream)

extern "C" int avc_enc_concat(const float* mel, long long mel_ld, const float* emb, float* out, int B, int T, int nm,
                              int de, void* stream) {
  AVC_CHECK_ARG(mel && emb && out, "avc_enc_concat: null");
  long long n = (long long)B * T * (nm + de);
  enc_concat_kernel<<<GRID1(n)>>>(mel, mel_ld, emb, out, B, T, nm, de);
  return avc_check_launch("avc_enc_concat");
}

extern "C" int avc_codes_gather(const float* lo, float* codes, int B, int T, int D, int freq, void* stream) {
  AVC_CHECK_ARG(lo && codes && freq > 0 && T % freq == 0, "avc_codes_gather: T %% freq must be 0");
  long long n = (long long)B * (T / freq) * 2 * D;
  codes_gather_kernel<<<GRID1(n)>>>(lo, codes, B, T, D, freq);
  return avc_check_launch("avc_codes_gather");
}

extern "C" int avc_codes_scatter(const float* dcodes, float* dlo, int B, int T, int D, int freq, void* stream) {
  AVC_CHECK_ARG(dcodes && dlo && freq > 0 && T % freq == 0, "avc_codes_scatter: T %% freq must be 0");
  long long n = (long long)B * T * 2 * D;
  codes_scatter_kernel<<<GRID1(n)>>>(dcodes, dlo, B, T, D, freq);
  return avc_check_launch("avc_codes_scatter");
}

extern "C" int avc_dec_concat(const float* codes, const float* emb, float* out, int B, int T, int nc, int cd, int de,
                              void* stream) {
  AVC_CHECK_ARG(codes && emb && out && nc > 0 && T % nc == 0, "avc_dec_concat: bad args");
  long long n = (long long)B * T * (cd + de);
  dec_concat_kernel<<<GRID1(n)>>>(codes, emb, out, B, T, nc, cd, de);
  return avc_check_launch("avc_dec_concat");
}

extern "C" int avc_dec_concat_bwd(const float* dout, float* dcodes, int B, int T, int nc, int cd, int de,
                                  void* stream) {
  AVC_CHECK_ARG(dout && dcodes && nc > 0 && T % nc == 0, "avc_dec_concat_bwd: bad args");
  long long n = (long long)B * nc * cd;
  dec_concat_bwd_kernel<<<GRID1(n)>>>(dout, dcodes, B, T, nc, cd, de);
  return avc_check_launch("avc_dec_concat_bwd");
}

extern "C" int avc_expand_codes(const float* pc, const float* pe, float* out, int B, int T, int nc, int G,
                                void* stream) {
  AVC_CHECK_ARG(pc && pe && out && B > 0 && nc > 0 && T % nc == 0 && G % 4 == 0 &&
                    ((reinterpret_cast<uintptr_t>(pc) | reinterpret_cast<uintptr_t>(pe) |
                      reinterpret_cast<uintptr_t>(out)) & 15) == 0,
                "avc_expand_codes: bad args");
  const long long n4 = (long long)B * T * (G / 4);
  expand_codes_kernel<<<GRID1(n4)>>>(reinterpret_cast<const f32x4*>(pc), reinterpret_cast<const f32x4*>(pe),
                                     reinterpret_cast<f32x4*>(out), T, nc, G / 4, n4);
  return avc_check_launch("avc_expand_codes");
}

extern "C" int avc_code_cat(const float* codes, const float* emb, void* out_bf16, int B, int nc, int cd, int de,
                            void* stream) {
  AVC_CHECK_ARG(codes && emb && out_bf16 && B > 0 && nc > 0 && cd > 0 && de > 0, "avc_code_cat: bad args");
  const long long n = (long long)B * nc * (cd + de);
  code_cat_kernel<<<GRID1(n)>>>(codes, emb, reinterpret_cast<bf16*>(out_bf16), nc, cd, de, n);
  return avc_check_launch("avc_code_cat");
}

extern "C" int avc_conv_pack(const float* w, void* out, int dtype, int Co, int Ci, int K, int mode, void* stream) {
  AVC_CHECK_ARG(w && out && (mode == 0 || mode == 1), "avc_conv_pack: bad args");
  long long n = (long long)Co * Ci * K;
  if (K <= (mode == 0 ? PK_KMAX_F : PK_KMAX_D)) {
    const long long nu = conv_pack_units(Co, Ci, mode);
    conv_pack_tiled_kernel<<<(int)std::min<long long>(nu, 2048), 256, 0, as_stream(stream)>>>(w, out, dtype, Co, Ci, K,
                                                                                               mode);
  } else {
    conv_pack_kernel<<<GRID1(n)>>>(w, out, dtype, Co, Ci, K, mode);
  }
  return avc_check_launch("avc_conv_pack");
}

extern "C" int avc_conv_grad_unpack(const float* dwf, float* dw, int Co, int Ci, int K, int acc, void* stream) {
  AVC_CHECK_ARG(dwf && dw, "avc_conv_grad_unpack: null");
  long long n = (long long)Co * Ci * K;
  conv_grad_unpack_kernel<<<GRID1(n)>>>(dwf, dw, Co, Ci, K, acc);
  return avc_check_launch("avc_conv_grad_unpack");
}

extern "C" int avc_convert(const float* src, void* dst, int dtype, long long n, void* stream) {
  AVC_CHECK_ARG(src && dst, "avc_convert: null");
  if (n == 0) return 0;
  convert_kernel<<<GRID1(n)>>>(src, dst, dtype, n);
  return avc_check_launch("avc_convert");
}

extern "C" int avc_transpose(const float* src, void* dst, int dtype, int R, int C, long long ld_dst, void* stream) {
  AVC_CHECK_ARG(src && dst && (ld_dst == 0 || ld_dst >= R), "avc_transpose: bad args");
  if (ld_dst == 0) ld_dst = R;
  dim3 g(cdiv(C, 32), cdiv(R, 32));
  transpose_kernel<<<g, 256, 0, as_stream(stream)>>>(src, dst, dtype, R, C, ld_dst);
  return avc_check_launch("avc_transpose");
}

extern "C" int avc_add(const float* a, const float* b, float* o, long long n, void* stream) {
  AVC_CHECK_ARG(a && b && o, "avc_add: null");
  if (n == 0) return 0;
  add_kernel<<<GRID1(n)>>>(a, b, o, n);
  return avc_check_launch("avc_add");
}

__global__ void zero_words_kernel(unsigned* p, long long n) {
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) p[i] = 0u;
}

int avc_zero_async(void* p, size_t bytes, hipStream_t s) {
  const long long n = (long long)(bytes / 4);
  if (n == 0) return 0;
  zero_words_kernel<<<(int)std::min<long long>(1024, cdiv(n, 256)), 256, 0, s>>>(static_cast<unsigned*>(p), n);
  return avc_check_launch("avc_zero_async");
}

static int loss_launch(const float* a, const float* b, long long n, float* out, int mode, void* stream) {
  AVC_CHECK_ARG(a && b && out && n > 0, "avc loss: bad args");
  if (avc_zero_async(out, sizeof(float), as_stream(stream))) return -1;
  // 256 blocks: enough loads in flight for the 655 K mel values, and 256 same-word atomicAdds
  // (≈12 ns each at the L2) instead of 1024
  int grid = (int)std::min<long long>(256, cdiv(n, 1024));
  loss_kernel<<<grid, 256, 0, as_stream(stream)>>>(a, b, n, out, mode);
  return avc_check_launch("avc loss");
}

extern "C" int avc_mse_loss(const float* a, const float* b, long long n, float* out, void* stream) {
  return loss_launch(a, b, n, out, 0, stream);
}
extern "C" int avc_l1_loss(const float* a, const float* b, long long n, float* out, void* stream) {
  return loss_launch(a, b, n, out, 1, stream);
}

extern "C" int avc_loss_grad(const float* a, const float* b, long long n, const float* dloss, int mode, float* g,
                             float sign, void* stream) {
  AVC_CHECK_ARG(a && b && dloss && g, "avc_loss_grad: null");
  loss_grad_kernel<<<GRID1(n)>>>(a, b, n, dloss, mode, g, sign);
  return avc_check_launch("avc_loss_grad");
}

extern "C" size_t avc_vc_loss_ws(void) { return (size_t)VCL_GRID * 3; }

extern "C" int avc_vc_loss(const float* x, const float* y1, const float* y2, long long n1, const float* ca,
                           const float* cb, long long n2, float lambda_cd, float* out, float* ws, void* stream) {
  AVC_CHECK_ARG(x && y1 && y2 && out && ws && n1 > 0 && n2 >= 0 && (n2 == 0 || (ca && cb)), "avc_vc_loss: bad args");
  hipStream_t s = as_stream(stream);
  unsigned* cnt = avc_counter_slots(1, s);
  if (!cnt) return -1;
  const int vec = (((uintptr_t)x | (uintptr_t)y1 | (uintptr_t)y2) & 15) == 0;
  const int grid = (int)std::min<long long>(VCL_GRID, std::max<long long>(1, cdiv(std::max(n1 / 4, n2), 256)));
  vc_loss_kernel<<<grid, 256, 0, s>>>(x, y1, y2, n1, ca, cb, n2, lambda_cd, out, ws, cnt, vec);
  return avc_check_launch("avc_vc_loss");
}

extern "C" int avc_vc_loss_grad(const float* x, const float* y1, const float* y2, long long n1, const float* ca,
                                const float* cb, long long n2, float lambda_cd, const float* d0, const float* d1,
                                const float* d2, const float* d3, float* g1, float* g2, float* ga, float* gb,
                                void* stream) {
  AVC_CHECK_ARG(x && y1 && y2 && n1 > 0 && n2 >= 0 && (n2 == 0 || (ca && cb)), "avc_vc_loss_grad: bad args");
  const long long n = n1 + n2;
  vc_loss_grad_kernel<<<GRID1(n)>>>(x, y1, y2, n1, ca, cb, n2, lambda_cd, d0, d1, d2, d3, g1, g2, ga, gb);
  return avc_check_launch("avc_vc_loss_grad");
}

extern "C" int avc_pack_batch(const avc_pack_op* ops, const long long* prefix, int nops, long long total,
                              void* stream) {
  AVC_CHECK_ARG(ops && prefix && nops > 0 && nops <= PACK_MAX_OPS && total >= 0, "avc_pack_batch: bad args");
  if (total == 0) return 0;
  const int grid = (int)std::min<long long>(2048, total);
  pack_batch_kernel<<<grid, 256, 0, as_stream(stream)>>>(ops, prefix, nops, total);
  return avc_check_launch("avc_pack_batch");
}

extern "C" int avc_adam_blocks(float* p, const float* g, float* m, float* v, long long n, float lr, float beta1,
                               float beta2, float eps, float* state, int advance, int max_blocks, void* stream) {
  AVC_CHECK_ARG(p && g && m && v && state && max_blocks >= 0, "avc_adam: bad args");
  hipStream_t s = as_stream(stream);
  if (advance) adam_prep_kernel<<<1, 1, 0, s>>>(state, lr, beta1, beta2);
  if (n == 0) return avc_check_launch("avc_adam");
  const int vec = ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(m) |
                    reinterpret_cast<uintptr_t>(v)) & 15) == 0;
  int grid = (int)std::min<long long>(max_blocks > 0 ? max_blocks : 2048, cdiv(n, vec ? 2048 : 256));
  adam_kernel<<<grid, 256, 0, s>>>(p, g, m, v, n, beta1, beta2, eps, state, vec);
  return avc_check_launch("avc_adam");
}

extern "C" int avc_adam(float* p, const float* g, float* m, float* v, long long n, float lr, float beta1, float beta2,
                        float eps, float* state, int advance, void* stream) {
  return avc_adam_blocks(p, g, m, v, n, lr, beta1, beta2, eps, state, advance, 0, stream);
}

extern "C" int avc_act_fwd(const float* x, float* y, long long n, int act, void* stream) {
  AVC_CHECK_ARG(x && y, "avc_act_fwd: null");
  if (n == 0) return 0;
  act_fwd_kernel<<<GRID1(n)>>>(x, y, n, act);
  return avc_check_launch("avc_act_fwd");
}

extern "C" int avc_act_bwd(const float* g, const float* yout, float* dx, long long n, int act, void* stream) {
  AVC_CHECK_ARG(g && yout && dx, "avc_act_bwd: null");
  if (n == 0) return 0;
  act_bwd_kernel<<<GRID1(n)>>>(g, yout, dx, n, act);
  return avc_check_launch("avc_act_bwd");
}

extern "C" int avc_bce_loss(const float* p, long long n, float target, float* out, void* stream) {
  AVC_CHECK_ARG(p && out && n > 0, "avc_bce_loss: bad args");
  if (avc_zero_async(out, sizeof(float), as_stream(stream))) return -1;
  bce_kernel<<<(int)std::min<long long>(1024, cdiv(n, 256)), 256, 0, as_stream(stream)>>>(p, n, target, out);
  return avc_check_launch("avc_bce_loss");
}

extern "C" int avc_bce_grad(const float* p, long long n, float target, const float* dloss, float* g,
                            int through_sigmoid, void* stream) {
  AVC_CHECK_ARG(p && dloss && g, "avc_bce_grad: null");
  bce_grad_kernel<<<GRID1(n)>>>(p, n, target, dloss, g, through_sigmoid);
  return avc_check_launch("avc_bce_grad");
}
