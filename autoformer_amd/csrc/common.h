// Shared device/host helpers for libautovc_hip.so (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/autovc_hip.h"

typedef __bf16 bf16;
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------ errors
void avc_set_error(const char* fmt, ...);
#define AVC_CHECK_ARG(cond, ...)          \
  do {                                    \
    if (!(cond)) {                        \
      avc_set_error(__VA_ARGS__);         \
      return -1;                          \
    }                                     \
  } while (0)
int avc_check_launch(const char* what);

// ------------------------------------------------------------------ conversions
__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }

// Load 4 consecutive elements of dtype (0 f32, 1 bf16) as floats.
__device__ __forceinline__ f32x4 load4(const void* base, long long idx, int dtype) {
  if (dtype == AVC_F32) {
    return *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(base) + idx);
  } else {
    bf16x4 v = *reinterpret_cast<const bf16x4*>(reinterpret_cast<const bf16*>(base) + idx);
    return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
  }
}

// ------------------------------------------------------------------ fast unsigned division
struct FastDiv {
  uint32_t d, m, s;
};
inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d ? d : 1;
  f.s = 0;
  while ((1ull << f.s) < f.d) f.s++;
  f.m = (uint32_t)((((1ull << 32) * ((1ull << f.s) - f.d)) / f.d) + 1);
  return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  return (uint32_t)(((uint64_t)__umulhi(n, f.m) + n) >> f.s);
}

// ------------------------------------------------------------------ math
__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

__device__ __forceinline__ float act_fwd(float x, int act) {
  switch (act) {
    case AVC_ACT_RELU: return x > 0.f ? x : 0.f;
    case AVC_ACT_TANH: return tanhf(x);
    case AVC_ACT_LEAKY: return x > 0.f ? x : 0.01f * x;
    case AVC_ACT_GELU: return 0.5f * x * (1.f + erff(x * 0.70710678118654752f));
    case AVC_ACT_SIGMOID: return 1.f / (1.f + expf(-x));
    default: return x;
  }
}

// derivative expressed through the activation OUTPUT a (relu/tanh/leaky/none).
__device__ __forceinline__ float act_bwd_from_out(float g, float a, int act) {
  switch (act) {
    case AVC_ACT_RELU: return a > 0.f ? g : 0.f;
    case AVC_ACT_TANH: return g * (1.f - a * a);
    case AVC_ACT_LEAKY: return a > 0.f ? g : 0.01f * g;
    case AVC_ACT_SIGMOID: return g * a * (1.f - a);
    default: return g;
  }
}

// the same derivatives from the pre-activation z (recomputed as yhat*gamma + beta), so the
// BatchNorm backward need not read the activation output
__device__ __forceinline__ float act_bwd_from_pre(float g, float z, int act) {
  switch (act) {
    case AVC_ACT_RELU: return z > 0.f ? g : 0.f;
    case AVC_ACT_TANH: {
      const float t = tanhf(z);
      return g * (1.f - t * t);
    }
    case AVC_ACT_LEAKY: return z > 0.f ? g : 0.01f * g;
    case AVC_ACT_SIGMOID: {
      const float sg = 1.f / (1.f + expf(-z));
      return g * sg * (1.f - sg);
    }
    default: return g;
  }
}

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
static inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }
