// Probe: what a cross-stream event record costs the stream it is recorded on.
// Back-to-back ~5 us kernels on one stream, (A) plain, (B) an event record (DisableTiming |
// DisableSystemFence, as events.hip) between every two, (C) the same with a default-flag event,
// (D) the event attached to the kernel's own completion (hipExtLaunchKernelGGL stop event),
// (E) as B with a second stream waiting on every record and running a tiny kernel.
//   hipcc --offload-arch=gfx950 -O2 tools/probes/event_gap.hip -o /tmp/event_gap && /tmp/event_gap
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      printf("%s failed: %s\n", #x, hipGetErrorString(e_));                          \
      return 1;                                                                      \
    }                                                                                \
  } while (0)

__global__ void spin(float* out, long long ticks) {
  const long long t0 = wall_clock64();
  float acc = 0.f;
  while (wall_clock64() - t0 < ticks) acc += 1.f;
  if (acc < 0.f) out[threadIdx.x] = acc;  // never true: keeps the loop
}

__global__ void tiny(float* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] += 1.f;
}

int main() {
  hipStream_t s, s2;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  float* buf;
  CK(hipMalloc(&buf, 4096));
  int rate_khz = 0;
  CK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0));
  const long long ticks = (long long)rate_khz * 5 / 1000;  // ~5 us
  const int N = 400;
  hipEvent_t t0, t1, efast, edef;
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  CK(hipEventCreateWithFlags(&efast, hipEventDisableTiming | hipEventDisableSystemFence));
  CK(hipEventCreateWithFlags(&edef, hipEventDisableTiming));
  for (int mode = 0; mode < 5; ++mode) {
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipStreamSynchronize(s));
      CK(hipEventRecord(t0, s));
      for (int i = 0; i < N; ++i) {
        if (mode == 3) {
          hipExtLaunchKernelGGL(spin, dim3(256), dim3(64), 0, s, nullptr, efast, 0, buf, ticks);
        } else {
          spin<<<256, 64, 0, s>>>(buf, ticks);
          if (mode == 1 || mode == 4) CK(hipEventRecord(efast, s));
          if (mode == 2) CK(hipEventRecord(edef, s));
          if (mode == 4) {
            CK(hipStreamWaitEvent(s2, efast, 0));
            tiny<<<1, 64, 0, s2>>>(buf + 64);
          }
        }
      }
      CK(hipEventRecord(t1, s));
      CK(hipEventSynchronize(t1));
      CK(hipStreamSynchronize(s2));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, t0, t1));
      const char* names[] = {"plain", "record(fast event)", "record(default event)", "ext launch stop event",
                             "record + side wait + tiny"};
      printf("%-28s %7.2f us per kernel\n", names[mode], ms * 1e3 / N);
    }
  }
  return 0;
}
