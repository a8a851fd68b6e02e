// Shared device/host helpers for libautovc_hip.so (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <atomic>
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
// Zero `bytes` (a multiple of 4) at p with a KERNEL on stream s.  Used instead of hipMemsetAsync for
// everything a later kernel of the same stream depends on: replayed inside a hipGraph after eager
// work, a captured memset node was not reliably complete / visible when the next kernel node ran
// (the persistent recurrences then read the previous replay's flags; tools/graph_fwd_probe.py).
int avc_zero_async(void* p, size_t bytes, hipStream_t s);

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
// erf without branches: the device library's two single-precision pieces (|x| < 1: x + x r(x^2);
// else 1 - exp(-(t + t q(t))), the same minimax coefficients) both evaluated and one selected, the
// exponential as one v_exp_f32.  The library form branches per wave, and a wave of GELU inputs
// straddles |x| = 1, so it ran both pieces plus the exp range fix-ups under exec masks: the
// epilogue's GELU / GELU' was VALU-bound (~40 instructions per element on 163 M elements per
// MLP-Mixer channel product).  Max abs error 7.7e-8 over [-6, 6] (fp64 check).
__device__ __forceinline__ float erf_nb(float x) {
  const float t = fabsf(x), s = x * x;
  float q = fmaf(t, __uint_as_float(0x378e98abu), __uint_as_float(0xb9c68948u));
  q = fmaf(t, q, __uint_as_float(0x3b7cd369u));
  q = fmaf(t, q, __uint_as_float(0xbcc618b2u));
  q = fmaf(t, q, __uint_as_float(0x3dda74e4u));
  q = fmaf(t, q, __uint_as_float(0x3f228afdu));
  q = fmaf(t, q, __uint_as_float(0x3e03c728u));
  const float far = 1.f - __builtin_amdgcn_exp2f(fmaf(t, q, t) * -1.44269504088896341f);
  float r = fmaf(s, __uint_as_float(0xba1345e1u), __uint_as_float(0x3ba10414u));
  r = fmaf(s, r, __uint_as_float(0xbcdac9b8u));
  r = fmaf(s, r, __uint_as_float(0x3de703beu));
  r = fmaf(s, r, __uint_as_float(0xbec09330u));
  r = fmaf(s, r, __uint_as_float(0x3e0375d0u));
  const float near = fmaf(t, r, t);
  return copysignf(t < 1.f ? near : far, x);
}
// Element i of a channel-slice pack of conv weight W [Co][Ci][K] (fp32) -- input channels
// [ci0, ci0 + cn) of the conv0 fold, zero-padded to cpad (avc_conv_pack_slice, avc_pack_batch):
//   mode 0: [Co][K][cpad]   mode 1: [cpad][K-1-k][Co]   mode 2: [K][Co][cpad]
//   mode 3: [cn][K-1-k][cpad] with the OUTPUT channel axis padded to cpad
__device__ __forceinline__ float slice_val(const float* w, int Co, int Ci, int K, int ci0, int cn, int cpad, int mode,
                                           long long i) {
  int co, ci, k;
  if (mode == 3) {
    co = (int)(i % cpad);
    k = K - 1 - (int)((i / cpad) % K);
    ci = (int)(i / ((long long)cpad * K));
    return co < Co ? w[((long long)co * Ci + ci0 + ci) * K + k] : 0.f;
  }
  if (mode == 0) {
    ci = (int)(i % cpad);
    k = (int)((i / cpad) % K);
    co = (int)(i / ((long long)cpad * K));
  } else if (mode == 1) {
    co = (int)(i % Co);
    k = K - 1 - (int)((i / Co) % K);
    ci = (int)(i / ((long long)Co * K));
  } else {
    ci = (int)(i % cpad);
    co = (int)((i / cpad) % Co);
    k = (int)(i / ((long long)cpad * Co));
  }
  return ci < cn ? w[((long long)co * Ci + ci0 + ci) * K + k] : 0.f;
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

__device__ __forceinline__ float act_fwd(float x, int act) {
  switch (act) {
    case AVC_ACT_RELU: return x > 0.f ? x : 0.f;
    case AVC_ACT_TANH: return tanhf(x);
    case AVC_ACT_LEAKY: return x > 0.f ? x : 0.01f * x;
    case AVC_ACT_GELU: return 0.5f * x * (1.f + erf_nb(x * 0.70710678118654752f));
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

// ------------------------------------------------------------------ last-block reductions
// Per-device pool of zeroed arrival counters for "the last block to arrive finalizes"
// reductions (bn.hip).  Returns n consecutive slots, or nullptr with the error recorded (first
// use inside a stream capture, allocation failure).  The last arrival of a launch resets its
// slot to 0, so slots are reused without a reset pass.
unsigned* avc_counter_slots(int n, hipStream_t s);
// Reserve n consecutive slots of a ring of `pool` slots (pool a power of two <= 2^31) through
// the shared cursor.  A request that would cross the end of the ring starts at 0 and the
// cursor moves past the skipped tail AND the request, so the next request starts after it:
// reserved ranges never overlap while fewer than `pool` slots are live (a plain
// fetch_add(n) moved the crossing request to 0 but advanced the cursor by n only).
unsigned avc_ring_reserve(std::atomic<unsigned>& cursor, unsigned n, unsigned pool);
// the process fault word of the current device (avc_set_fault_word; lstm.hip), nullable
unsigned* avc_fault_ptr();
// n floats of a device pool that is all zero between uses: the user leaves its region zeroed
// (a ring like avc_counter_slots; created on first use outside a stream capture)
float* avc_zero_slots(int n, hipStream_t s);

// Agent-coherent (sc1) scalar store / load: the data handed from block to block through an
// arrival counter bypasses the per-XCD L2 on both sides, so no fence (an agent-scope release
// fence writes back the whole L2 on gfx950 -- measured +1 ms per C2 step when every reduce
// block issued one).
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Arrival of a block at counter `cnt` expecting `arrivals` blocks.  Every thread calls it after
// its hand-off stores, which must be st_sc1 stores: they are waited for (vmcnt(0)), one lane
// increments the counter (agent-scope relaxed atomic), and the block that arrives last resets it
// and returns true; it then reads the hand-off data with ld_sc1.
__device__ __forceinline__ bool arrive_last(unsigned* cnt, unsigned arrivals, unsigned mine = 1) {
  __shared__ unsigned s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(cnt, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool last = old + mine == arrivals;
    if (last) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = last ? 1u : 0u;
  }
  __syncthreads();
  return s_last != 0;
}

// 8-byte load of a (sum, M2) pair; SC1: handed over within the launch (agent-coherent load)
template <bool SC1>
__device__ __forceinline__ float2 ld_pair(const float* p) {
  if (SC1) {
    const unsigned long long u =
        __hip_atomic_load(reinterpret_cast<unsigned long long*>(const_cast<float*>(p)), __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_AGENT);
    return make_float2(__uint_as_float((unsigned)u), __uint_as_float((unsigned)(u >> 32)));
  }
  return *reinterpret_cast<const float2*>(p);
}

// Chan's parallel merge of per-tile (sum, M2) pairs at P[(t*ld + col)*2], t < nt, tiles of `tile`
// rows (the last one M - t*tile):  mean = sum_t s_t / M,  M2 = sum_t [q_t + n_t (s_t/n_t - mean)^2].
// Thread (grp < ng, cl < nc) covers tiles grp, grp + ng, ...; its first U tiles are loaded in ONE
// round and kept in registers for both passes (the finalize is latency-bound: one memory round
// instead of one per pass and per 8 tiles); further tiles (nt > ng*U) take extra rounds.  red:
// ng*nc floats of LDS.  Every thread of the block calls it; mean / m2 come back in all of them.
template <int U, bool SC1>
__device__ __forceinline__ void chan_merge(const float* P, int nt, long long ld, int col, bool cv, int grp, int ng,
                                           int cl, int nc, int M, int tile, float* red, float& mean, float& m2) {
  float2 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int t = grp + u * ng;
    v[u] = (cv && t < nt) ? ld_pair<SC1>(P + ((long long)t * ld + col) * 2) : make_float2(0.f, 0.f);
  }
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) s += v[u].x;
  if (cv)
    for (int t = grp + U * ng; t < nt; t += ng) s += ld_pair<SC1>(P + ((long long)t * ld + col) * 2).x;
  const bool act = grp < ng;
  __syncthreads();
  if (act) red[grp * nc + cl] = s;
  __syncthreads();
  float tot = 0.f;
  for (int i = 0; i < ng; ++i) tot += red[i * nc + cl];
  mean = tot / (float)M;
  float q = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int t = grp + u * ng;
    if (cv && t < nt) {
      const float nb = (float)min(tile, M - t * tile);
      const float d = v[u].x / nb - mean;
      q += v[u].y + nb * d * d;
    }
  }
  if (cv)
    for (int t = grp + U * ng; t < nt; t += ng) {
      const float2 w = ld_pair<SC1>(P + ((long long)t * ld + col) * 2);
      const float nb = (float)min(tile, M - t * tile);
      const float d = w.x / nb - mean;
      q += w.y + nb * d * d;
    }
  __syncthreads();
  if (act) red[grp * nc + cl] = q;
  __syncthreads();
  m2 = 0.f;
  for (int i = 0; i < ng; ++i) m2 += red[i * nc + cl];
  __syncthreads();
}
