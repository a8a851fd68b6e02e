// Layout / timing probe of v_mfma_f32_4x4x4_16b_bf16 (__builtin_amdgcn_mfma_f32_4x4x4bf16_1k) on
// gfx950: which lane / element of A and B feeds which lane / register of D, and the issue cost of a
// dependent chain (the encoder BiLSTM's recurrent product, lstm.hip lstm_mfma_*).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef short s4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));

__device__ short bf(float x) { unsigned u = __builtin_bit_cast(unsigned, x); return (short)(u >> 16); }

__global__ void probe(float* out, long long* cyc) {
  const int l = threadIdx.x;
  s4 a, b, one;
  for (int e = 0; e < 4; ++e) { a[e] = bf((float)(l + 64 * e)); one[e] = bf(1.f); }
  f4 z = {0.f, 0.f, 0.f, 0.f};
  f4 d1 = __builtin_amdgcn_mfma_f32_4x4x4bf16_1k(a, one, z, 0, 0, 0);  // rows
  f4 d2 = __builtin_amdgcn_mfma_f32_4x4x4bf16_1k(one, a, z, 0, 0, 0);  // columns
  s4 a3, b3;
  for (int e = 0; e < 4; ++e) { a3[e] = bf((float)(e + 1)); b3[e] = bf(e == 2 ? 1.f : 0.f); }
  f4 d3 = __builtin_amdgcn_mfma_f32_4x4x4bf16_1k(a3, b3, z, 0, 0, 0);  // k pairing
  for (int r = 0; r < 4; ++r) {
    out[(0 * 64 + l) * 4 + r] = d1[r];
    out[(1 * 64 + l) * 4 + r] = d2[r];
    out[(2 * 64 + l) * 4 + r] = d3[r];
  }
  // dependent chain timing
  f4 acc = z;
  long long t0 = clock64();
  for (int i = 0; i < 1024; ++i) acc = __builtin_amdgcn_mfma_f32_4x4x4bf16_1k(a3, b3, acc, 0, 0, 0);
  long long t1 = clock64();
  f4 acc2 = z, acc3 = z, acc4 = z;
  long long t2 = clock64();
  for (int i = 0; i < 256; ++i) {
    acc = __builtin_amdgcn_mfma_f32_4x4x4bf16_1k(a3, b3, acc, 0, 0, 0);
    acc2 = __builtin_amdgcn_mfma_f32_4x4x4bf16_1k(a3, b3, acc2, 0, 0, 0);
    acc3 = __builtin_amdgcn_mfma_f32_4x4x4bf16_1k(a3, b3, acc3, 0, 0, 0);
    acc4 = __builtin_amdgcn_mfma_f32_4x4x4bf16_1k(a3, b3, acc4, 0, 0, 0);
  }
  long long t3 = clock64();
  if (l == 0) { cyc[0] = t1 - t0; cyc[1] = t3 - t2; }
  out[3 * 256 + l] = acc[0] + acc2[1] + acc3[2] + acc4[3];
}

int main() {
  float* d; long long* c;
  hipMalloc(&d, 4 * 256 * 4 + 1024); hipMalloc(&c, 16);
  probe<<<1, 64>>>(d, c);
  float h[3 * 256]; long long hc[2];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost); hipMemcpy(hc, c, 16, hipMemcpyDeviceToHost);
  // d1: lane L reg r = 4*laneA + 384 -> laneA(row source); d2 -> laneB(column source)
  printf("lane: rowsrc(reg0..3) | colsrc(reg0..3) | kpair\n");
  for (int l = 0; l < 64; ++l) {
    printf("%2d:", l);
    for (int r = 0; r < 4; ++r) printf(" %3d", (int)((h[(0 * 64 + l) * 4 + r] - 384) / 4));
    printf(" |");
    for (int r = 0; r < 4; ++r) printf(" %3d", (int)((h[(1 * 64 + l) * 4 + r] - 384) / 4));
    printf(" | %g\n", h[(2 * 64 + l) * 4]);
  }
  printf("dependent chain: %.2f cyc/mfma; 4 independent: %.2f cyc/mfma\n", hc[0] / 1024.0, hc[1] / 1024.0);
  return 0;
}
