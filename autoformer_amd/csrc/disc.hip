// disc.hip — the Discriminator's head: flatten + Linear(1628 -> 1) + Sigmoid, forward and backward.
//
// Reference: factory/Discriminator.py:18-29 (x = flatten(bn2(leaky(conv3(.)))) channel-major, C3 x L3
// = 22 x 74 = 1628 features; dense1 = nn.Linear(1628, 1); sigmoid).  Our activation a3 is bin-major
// ([B][L3][C3], the convs run with the mel bins as frames), so feature f = l*C3 + c of a row reads
// dense1.weight[c*L3 + l]: the permutation is folded into the index instead of a transposed weight
// copy (forward) and a transposed gradient copy (backward).  A GEMV with one output column ran on
// the generic fp32 GEMM as ONE workgroup looping over K (176 us per call in the C5 step,
// gpurun_out/r3s12/breakdown_disc.txt); here one workgroup per utterance reduces its row.
#include "common.h"

namespace {

// one 256-thread block per utterance b: p[b] = sigmoid(bias + sum_{l,c} a[b][l*C + c] w[c*L + l])
__global__ void __launch_bounds__(256) disc_dense_fwd_kernel(const float* __restrict__ a, const float* __restrict__ w,
                                                             const float* __restrict__ bias, int L, int C,
                                                             float* __restrict__ logit, float* __restrict__ p) {
  __shared__ float red[4];
  const int b = blockIdx.x, F = L * C;
  const float* row = a + (long long)b * F;
  float s = 0.f;
  for (int f = threadIdx.x; f < F; f += 256) {
    const int l = f / C, c = f - l * C;
    s += row[f] * w[c * L + l];
  }
  s = warp_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float z = (red[0] + red[1]) + (red[2] + red[3]) + (bias ? bias[0] : 0.f);
    if (logit) logit[b] = z;
    p[b] = 1.f / (1.f + expf(-z));
  }
}

// 256 threads = 64 features x 4 utterance groups: dlogit[b] = dp[b] p[b] (1 - p[b]) (through the
// sigmoid); da[b][f] = dlogit[b] w[c*L + l], dw[c*L + l] = sum_b dlogit[b] a[b][f] (the four groups'
// partial sums meet in LDS); block 0 also writes dbias = sum_b dlogit[b].  B <= 1024.
__global__ void __launch_bounds__(256) disc_dense_bwd_kernel(const float* __restrict__ dp, const float* __restrict__ p,
                                                             const float* __restrict__ a, const float* __restrict__ w,
                                                             int B, int L, int C, float* __restrict__ da,
                                                             float* __restrict__ dw, float* __restrict__ dbias) {
  __shared__ float dl[1024];
  __shared__ float red[4][64];
  for (int b = threadIdx.x; b < B; b += 256) dl[b] = dp[b] * p[b] * (1.f - p[b]);
  __syncthreads();
  const int F = L * C;
  const int fl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int f = blockIdx.x * 64 + fl;
  if (blockIdx.x == 0 && threadIdx.x < 64) {
    float s = 0.f;
    for (int b = threadIdx.x; b < B; b += 64) s += dl[b];
    s = warp_sum(s);
    if (threadIdx.x == 0 && dbias) dbias[0] = s;
  }
  const bool fv = f < F;
  const int l = fv ? f / C : 0, c = fv ? f - l * C : 0;
  const float wf = fv ? w[c * L + l] : 0.f;
  float s = 0.f;
  if (fv)
    for (int b = grp; b < B; b += 4) {
      const long long i = (long long)b * F + f;
      s += dl[b] * a[i];
      if (da) da[i] = dl[b] * wf;
    }
  red[grp][fl] = s;
  __syncthreads();
  if (grp == 0 && fv && dw) dw[c * L + l] = (red[0][fl] + red[1][fl]) + (red[2][fl] + red[3][fl]);
}

}  // namespace

extern "C" int avc_disc_dense_fwd(const float* a, const float* w, const float* bias, int B, int L, int C, float* logit,
                                  float* p, void* stream) {
  AVC_CHECK_ARG(a && w && p && B > 0 && L > 0 && C > 0, "avc_disc_dense_fwd: bad args");
  disc_dense_fwd_kernel<<<B, 256, 0, as_stream(stream)>>>(a, w, bias, L, C, logit, p);
  return avc_check_launch("avc_disc_dense_fwd");
}

extern "C" int avc_disc_dense_bwd(const float* dp, const float* p, const float* a, const float* w, int B, int L, int C,
                                  float* da, float* dw, float* dbias, void* stream) {
  AVC_CHECK_ARG(dp && p && a && w && B > 0 && B <= 1024 && L > 0 && C > 0, "avc_disc_dense_bwd: bad args (B <= 1024)");
  disc_dense_bwd_kernel<<<cdiv((long long)L * C, 64), 256, 0, as_stream(stream)>>>(dp, p, a, w, B, L, C, da, dw,
                                                                                     dbias);
  return avc_check_launch("avc_disc_dense_bwd");
}
