// melgan.hip — the MelGAN vocoder generator (reference melgan/modules.py:88-131, used by
// util/evaluate.py:98 through melgan/interface.py:47-53 MelVocoder.inverse) for the
// conversion path, inference only.
//
// Layout: frame-major [B*L][C] like every other activation of the build.  The convolutions run
// on avc_gemm; what is here is the glue the GEMM operand cannot express:
//
//   * mg_gather      im2col rows of a dilated conv with REFLECTION padding (nn.ReflectionPad1d,
//                    modules.py:76,95,124) and the LeakyReLU(0.2) that precedes every conv of
//                    the generator (modules.py:75,78,108,123), written in the GEMM operand dtype.
//                    (The zero-padded 3-tap window of the transposed convs needs no gather: the
//                    GEMM's window operand reads it in place.)
//   * mg_act         LeakyReLU into a GEMM-operand copy (fp32 and/or bf16).
//   * mg_wn_pack     weight_norm (w = g v / ||v||, torch.nn.utils.weight_norm, dim 0) folded into
//                    the GEMM B-operand pack.  For ConvTranspose1d(k = 2r, stride r, padding
//                    r/2 + r%2) output frame o = j*r + p reads input frames q and q-1,
//                    q = j + (p + pad) / r, taps (p + pad) % r and that + r: the layer is ONE GEMM
//                    over the 3-tap window (j-1, j, j+1) with N = r*Cout (phase-major), whose
//                    [B*L][r*Cout] output IS the upsampled frame-major sequence [B*L*r][Cout].
//   * mg_conv_out    the last ReflectionPad1d(3) + WNConv1d(ngf -> 1, k 7) + Tanh
//                    (modules.py:122-126): one output sample per thread, N = 1 is no GEMM.
#include <algorithm>

#include "common.h"

namespace {

__device__ __forceinline__ float lrelu(float v, float s) { return v >= 0.f ? v : v * s; }

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ f32x4 ld4(const bf16* p) {
  const bf16x4 v = *reinterpret_cast<const bf16x4*>(p);
  return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
}
__device__ __forceinline__ void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
__device__ __forceinline__ void st4(bf16* p, f32x4 v) {
  *reinterpret_cast<bf16x4*>(p) = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
}

// reflect (ReflectionPad1d: -1 -> 1, L -> L-2) or -1 = zero
__device__ __forceinline__ int src_frame(int s, int L, int reflect) {
  if (s >= 0 && s < L) return s;
  if (!reflect) return -1;
  return s < 0 ? -s : 2 * (L - 1) - s;
}

// out[(b*Lo + t)][k*C + c] = act(x[b][src(t + k*dil - pad)][c]), 4 channels per thread
template <typename TI, typename TO>
__global__ void mg_gather_kernel(const TI* __restrict__ x, int B, int L, int C, int taps, int dil, int pad,
                                 int reflect, int act, float slope, TO* __restrict__ out, int Lo) {
  const int C4 = C >> 2;
  const long long total = (long long)B * Lo * taps * C4;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int c4 = (int)(i % C4);
    const long long r = i / C4;
    const int k = (int)(r % taps);
    const long long m = r / taps;
    const int t = (int)(m % Lo), b = (int)(m / Lo);
    const int s = src_frame(t + k * dil - pad, L, reflect);
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (s >= 0) {
      v = ld4(x + ((long long)b * L + s) * C + 4 * c4);
      if (act) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = lrelu(v[e], slope);
      }
    }
    st4(out + m * (long long)taps * C + (long long)k * C + 4 * c4, v);
  }
}

__global__ void mg_act_kernel(const float* __restrict__ x, long long n4, float slope, float* __restrict__ out,
                              bf16* __restrict__ out16) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    f32x4 v = ld4(x + 4 * i);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = lrelu(v[e], slope);
    if (out) st4(out + 4 * i, v);
    if (out16) st4(out16 + 4 * i, v);
  }
}

// ||v[d]|| over the d1*K elements of slice d (one 256-thread block per slice)
__global__ void __launch_bounds__(256) mg_norm_kernel(const float* __restrict__ v, int n, float* __restrict__ norms) {
  __shared__ float red[4];
  const float* p = v + (long long)blockIdx.x * n;
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += p[i] * p[i];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) norms[blockIdx.x] = sqrtf(red[0] + red[1] + red[2] + red[3]);
}

// conv (stride == 0): v [Co][Ci][K] -> out [Co][K*Ci]   (tap-major columns, = mg_gather rows)
// transposed (stride r): v [Ci][Co][2r] -> out [r*Co][3*Ci] polyphase (see header)
template <typename TO>
__global__ void mg_pack_kernel(const float* __restrict__ v, const float* __restrict__ g,
                               const float* __restrict__ norms, int d0, int d1, int K, int stride, int pad,
                               TO* __restrict__ out, const float* __restrict__ bias, float* __restrict__ bias_out) {
  const long long rows = stride ? (long long)stride * d1 : d0;
  const long long cols = stride ? 3LL * d0 : (long long)K * d1;
  const long long total = rows * cols;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long n = i / cols, kk = i % cols;
    float w = 0.f;
    if (!stride) {
      const int co = (int)n, k = (int)(kk / d1), ci = (int)(kk % d1);
      w = g[co] * v[((long long)co * d1 + ci) * K + k] / norms[co];
    } else {
      const int r = stride, p = (int)(n / d1), co = (int)(n % d1);
      const int tap = (int)(kk / d0), ci = (int)(kk % d0);
      const int dl = (p + pad) / r, rho = (p + pad) % r;
      const int k = tap == dl + 1 ? rho : tap == dl ? rho + r : -1;
      if (k >= 0) w = g[ci] * v[((long long)ci * d1 + co) * K + k] / norms[ci];
      if (kk == 0 && bias_out) bias_out[n] = bias ? bias[co] : 0.f;
    }
    out[i] = (TO)w;
  }
}

// audio[b][t] = tanh(bias + sum_k sum_c w[k][c] * lrelu(x[b][reflect(t + k - 3)][c]))
template <int TAPS>
__global__ void __launch_bounds__(256) mg_conv_out_kernel(const float* __restrict__ x, int B, int L, int C,
                                                          const float* __restrict__ w, const float* __restrict__ bias,
                                                          float slope, float* __restrict__ out) {
  extern __shared__ float ws[];  // [TAPS][C]
  for (int i = threadIdx.x; i < TAPS * C; i += blockDim.x) ws[i] = w[i];
  __syncthreads();
  const long long m = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= (long long)B * L) return;
  const int t = (int)(m % L), b = (int)(m / L);
  float acc = bias[0];
#pragma unroll
  for (int k = 0; k < TAPS; ++k) {
    const int s = src_frame(t + k - TAPS / 2, L, 1);
    const float* row = x + ((long long)b * L + s) * C;
    for (int c = 0; c < C; c += 4) {
      const f32x4 v = ld4(row + c);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc += ws[k * C + c + e] * lrelu(v[e], slope);
    }
  }
  out[m] = tanhf(acc);
}

int blocks_for(long long n) { return (int)std::min<long long>((n + 255) / 256, 65535LL * 4); }

}  // namespace

extern "C" int avc_mg_gather(const void* x, int x_dtype, int B, int L, int C, int taps, int dil, int pad, int reflect,
                             int act, float slope, void* out, int out_dtype, void* stream) {
  AVC_CHECK_ARG(x && out && B > 0 && L > 0 && C > 0 && C % 4 == 0 && taps > 0 && dil > 0 && pad >= 0,
                "avc_mg_gather: bad args (C must be a multiple of 4)");
  AVC_CHECK_ARG(!reflect || pad < L, "avc_mg_gather: reflection pad %d needs L > pad (L = %d)", pad, L);
  const int Lo = L + 2 * pad - dil * (taps - 1);
  AVC_CHECK_ARG(Lo > 0, "avc_mg_gather: empty output");
  const long long n = (long long)B * Lo * taps * (C / 4);
  hipStream_t s = as_stream(stream);
  const int nb = blocks_for(n);
  if (x_dtype == AVC_BF16) {
    if (out_dtype == AVC_BF16)
      mg_gather_kernel<bf16, bf16><<<nb, 256, 0, s>>>((const bf16*)x, B, L, C, taps, dil, pad, reflect, act, slope,
                                                      (bf16*)out, Lo);
    else
      mg_gather_kernel<bf16, float><<<nb, 256, 0, s>>>((const bf16*)x, B, L, C, taps, dil, pad, reflect, act, slope,
                                                       (float*)out, Lo);
  } else {
    if (out_dtype == AVC_BF16)
      mg_gather_kernel<float, bf16><<<nb, 256, 0, s>>>((const float*)x, B, L, C, taps, dil, pad, reflect, act, slope,
                                                       (bf16*)out, Lo);
    else
      mg_gather_kernel<float, float><<<nb, 256, 0, s>>>((const float*)x, B, L, C, taps, dil, pad, reflect, act,
                                                        slope, (float*)out, Lo);
  }
  return avc_check_launch("avc_mg_gather");
}

extern "C" int avc_mg_act(const float* x, long long n, float slope, float* out, void* out_bf16, void* stream) {
  AVC_CHECK_ARG(x && (out || out_bf16) && n >= 0 && n % 4 == 0, "avc_mg_act: bad args (n must be a multiple of 4)");
  if (n == 0) return 0;
  mg_act_kernel<<<blocks_for(n / 4), 256, 0, as_stream(stream)>>>(x, n / 4, slope, out,
                                                                   reinterpret_cast<bf16*>(out_bf16));
  return avc_check_launch("avc_mg_act");
}

extern "C" int avc_mg_wn_pack(const float* v, const float* g, const float* bias, int d0, int d1, int K, int stride,
                              int pad, float* norms, void* out, int out_dtype, float* bias_out, void* stream) {
  AVC_CHECK_ARG(v && g && norms && out && d0 > 0 && d1 > 0 && K > 0 && stride >= 0, "avc_mg_wn_pack: bad args");
  AVC_CHECK_ARG(!stride || (K == 2 * stride && pad >= 0 && pad <= stride),
                "avc_mg_wn_pack: transposed pack needs K = 2*stride (got K=%d stride=%d)", K, stride);
  hipStream_t s = as_stream(stream);
  mg_norm_kernel<<<d0, 256, 0, s>>>(v, d1 * K, norms);
  const long long n = stride ? (long long)stride * d1 * 3 * d0 : (long long)d0 * d1 * K;
  if (out_dtype == AVC_BF16)
    mg_pack_kernel<bf16><<<blocks_for(n), 256, 0, s>>>(v, g, norms, d0, d1, K, stride, pad, (bf16*)out, bias, bias_out);
  else
    mg_pack_kernel<float><<<blocks_for(n), 256, 0, s>>>(v, g, norms, d0, d1, K, stride, pad, (float*)out, bias,
                                                        bias_out);
  return avc_check_launch("avc_mg_wn_pack");
}

extern "C" int avc_mg_conv_out(const float* x, int B, int L, int C, int taps, const float* w, const float* bias,
                               float slope, float* out, void* stream) {
  AVC_CHECK_ARG(x && w && bias && out && B > 0 && C > 0 && C % 4 == 0 && taps == 7 && L > taps / 2,
                "avc_mg_conv_out: bad args (7 taps, C %% 4 == 0, L > 3)");
  const long long m = (long long)B * L;
  mg_conv_out_kernel<7><<<(int)((m + 255) / 256), 256, taps * C * sizeof(float), as_stream(stream)>>>(
      x, B, L, C, w, bias, slope, out);
  return avc_check_launch("avc_mg_conv_out");
}
