// fold.hip — the speaker half of the encoder's first convolution, folded out of the frame axis.
//
// Reference: factory/AutoVC.py:46-51 (Encoder.forward): x = cat(mel (B, 80, T), c_org broadcast
// over T (B, 256, T)); conv0 = ConvNorm(336 -> 512, k 5, pad 2) + BN + ReLU.  Because c_org is
// constant over the frames of an utterance, its share of conv0 is
//     y_e[b, t, co] = sum_{k valid at t} sum_ci W[co][80 + ci][k] c_org[b][ci]
//                   = sum_{k valid at t} E[b][k][co],      E = c_org . We  (one B x 5*512 x 256 GEMM)
// where "k valid at t" means 0 <= t + k - pad < T (zero padding): every interior frame sees the
// same five taps, the first / last `pad` frames fewer.  So conv0 runs on the 80 mel channels
// alone (padded to 96 for the 32-channel halo kernels) and the speaker term enters as a
// per-(utterance, edge class) row bias in the GEMM epilogue (avc_gemm_desc.row_bias), before the
// BatchNorm statistics.  The backward mirrors it: dW[co][80 + ci][k] = sum_b Sdy[b][k][co] c[b][ci]
// and dc_org[b][ci] = sum_{k, co} Sdy[b][k][co] W[co][80 + ci][k] with Sdy[b][k][co] the column
// sums of dy over the frames where tap k is valid (avc_conv_edge_colsum) -- K = B GEMMs instead
// of K = B*T.
#include "common.h"

namespace {

__device__ __forceinline__ void put(void* dst, long long i, float v, int dtype) {
  if (dtype == AVC_BF16) reinterpret_cast<bf16*>(dst)[i] = (bf16)v;
  else reinterpret_cast<float*>(dst)[i] = v;
}

// one thread per OUTPUT element (padding written as zeros)
__global__ void conv_pack_slice_kernel(const float* __restrict__ w, void* __restrict__ out, int dtype, int Co, int Ci,
                                       int K, int ci0, int cn, int cpad, int mode) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)(mode == 3 ? cn : Co) * cpad * K;
  if (i >= total) return;
  put(out, i, slice_val(w, Co, Ci, K, ci0, cn, cpad, mode, i), dtype);
}

// S[b][cls][co] = sum_{k valid for cls} E[b][k*Co + co]; cls = 0..pad-1 (t = cls), pad (interior),
// pad+1..2pad (t = T - 2*pad - 1 + cls)
__global__ void conv_edge_table_kernel(const float* __restrict__ E, int B, int Co, int K, int T, int pad,
                                       float* __restrict__ S) {
  const int ncls = 2 * pad + 1;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)B * ncls * Co) return;
  const int co = (int)(i % Co);
  const int cls = (int)((i / Co) % ncls);
  const int b = (int)(i / ((long long)Co * ncls));
  const int t = cls < pad ? cls : (cls == pad ? pad : T - 1 - (2 * pad - cls));
  float s = 0.f;
  for (int k = 0; k < K; ++k) {
    const int src = t + k - pad;
    if (src >= 0 && src < T) s += E[((long long)b * K + k) * Co + co];
  }
  S[i] = s;
}

// out[b][k][c] = sum over frames t of utterance b with 0 <= t + k - pad < T of dy[b*T + t][c]:
// a 256-thread block per (utterance, 64 channels) = 16 channel quads x 16 row lanes sums the
// utterance's frames; then per tap the rows where that tap reads padding (the first / last
// `pad` frames at most) are subtracted.
template <typename TD>
__device__ __forceinline__ f32x4 row4(const TD* p) {
  if constexpr (sizeof(TD) == 2) {
    const bf16x4 h = *reinterpret_cast<const bf16x4*>(p);
    return f32x4{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
  } else {
    return *reinterpret_cast<const f32x4*>(p);
  }
}

template <typename TD>
__global__ void __launch_bounds__(256) conv_edge_colsum_kernel(const TD* __restrict__ dy, int T, int C, int K, int pad,
                                                               float* __restrict__ out) {
  __shared__ f32x4 red[16][16];
  const int cq = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int b = blockIdx.y, c = blockIdx.x * 64 + cq * 4;
  const bool cv = c < C;
  const TD* p = dy + (long long)b * T * C + c;
  f32x4 tot = {0.f, 0.f, 0.f, 0.f};
  if (cv)
    for (int t = rl; t < T; t += 16) tot += row4(p + (long long)t * C);
  red[rl][cq] = tot;
  __syncthreads();
  if (rl < K && cv) {
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 16; ++i) s += red[i][cq];
    const int k = rl;  // frames whose tap-k source lies outside [0, T): t < pad - k and t >= T + pad - k
    for (int t = 0; t < min(T, pad - k); ++t) s -= row4(p + (long long)t * C);
    for (int t = max(0, T + pad - k); t < T; ++t) s -= row4(p + (long long)t * C);
    *reinterpret_cast<f32x4*>(out + ((long long)b * K + k) * C + c) = s;
  }
}

// dw[co][ci0 + ci][k] (+)= dwf[co*ld + k*kstride + ci], ci < cn (dw rows Ci channels wide)
__global__ void conv_grad_unpack_slice_kernel(const float* __restrict__ dwf, long long ld, int kstride,
                                              float* __restrict__ dw, int Co, int Ci, int K, int ci0, int cn, int acc) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)Co * cn * K) return;
  const int k = (int)(i % K);
  const int ci = (int)((i / K) % cn);
  const int co = (int)(i / ((long long)K * cn));
  const float v = dwf[(long long)co * ld + (long long)k * kstride + ci];
  const long long o = ((long long)co * Ci + ci0 + ci) * K + k;
  dw[o] = acc ? dw[o] + v : v;
}

}  // namespace

extern "C" int avc_conv_pack_slice(const float* w, void* out, int dtype, int Co, int Ci, int K, int ci0, int cn,
                                   int cpad, int mode, void* stream) {
  AVC_CHECK_ARG(w && out && Co > 0 && Ci > 0 && K > 0 && ci0 >= 0 && cn > 0 && ci0 + cn <= Ci &&
                    cpad >= (mode == 3 ? Co : cn) && mode >= 0 && mode <= 3 && (dtype == AVC_F32 || dtype == AVC_BF16),
                "avc_conv_pack_slice: bad args");
  const long long n = (long long)(mode == 3 ? cn : Co) * cpad * K;
  conv_pack_slice_kernel<<<cdiv(n, 256), 256, 0, as_stream(stream)>>>(w, out, dtype, Co, Ci, K, ci0, cn, cpad, mode);
  return avc_check_launch("avc_conv_pack_slice");
}

extern "C" int avc_conv_edge_table(const float* E, int B, int Co, int K, int T, int pad, float* S, void* stream) {
  AVC_CHECK_ARG(E && S && B > 0 && Co > 0 && K > 0 && pad >= 0 && T > 2 * pad, "avc_conv_edge_table: bad args");
  const long long n = (long long)B * (2 * pad + 1) * Co;
  conv_edge_table_kernel<<<cdiv(n, 256), 256, 0, as_stream(stream)>>>(E, B, Co, K, T, pad, S);
  return avc_check_launch("avc_conv_edge_table");
}

extern "C" int avc_conv_edge_colsum(const void* dy, int dy_dtype, int B, int T, int C, int K, int pad, float* out,
                                    void* stream) {
  AVC_CHECK_ARG(dy && out && B > 0 && T > 0 && C > 0 && C % 4 == 0 && K > 0 && pad >= 0 &&
                    (dy_dtype == AVC_F32 || dy_dtype == AVC_BF16),
                "avc_conv_edge_colsum: bad args (C %% 4 == 0)");
  AVC_CHECK_ARG(K <= 16, "avc_conv_edge_colsum: K <= 16");
  const dim3 grid(cdiv(C, 64), B);
  if (dy_dtype == AVC_BF16)
    conv_edge_colsum_kernel<bf16><<<grid, 256, 0, as_stream(stream)>>>(static_cast<const bf16*>(dy), T, C, K, pad, out);
  else
    conv_edge_colsum_kernel<float><<<grid, 256, 0, as_stream(stream)>>>(static_cast<const float*>(dy), T, C, K, pad, out);
  return avc_check_launch("avc_conv_edge_colsum");
}

extern "C" int avc_conv_grad_unpack_slice(const float* dwf, long long ld, int kstride, float* dw, int Co, int Ci, int K,
                                          int ci0, int cn, int accumulate, void* stream) {
  AVC_CHECK_ARG(dwf && dw && Co > 0 && K > 0 && cn > 0 && ci0 >= 0 && ci0 + cn <= Ci && kstride >= cn &&
                    ld >= (long long)K * kstride,
                "avc_conv_grad_unpack_slice: bad args");
  const long long n = (long long)Co * cn * K;
  conv_grad_unpack_slice_kernel<<<cdiv(n, 256), 256, 0, as_stream(stream)>>>(dwf, ld, kstride, dw, Co, Ci, K, ci0, cn,
                                                                             accumulate);
  return avc_check_launch("avc_conv_grad_unpack_slice");
}
