// Launch-overhead probe (tools only, not part of librps): what a dependent kernel boundary
// costs on the GPU against a hipGraph replay and against a grid-wide barrier inside one
// cooperative launch.  Decides how the small-N SPH frame (a dozen dependent sort launches of
// ~1 us of work each) should be scheduled.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/launch_probe tools/launch_probe.hip
//   ./tools/launch_probe            (on the GPU box)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

__global__ void empty_kernel() {}

// One pass over n entries (a bitonic-pass-sized touch: 8 B read + 8 B written per entry).
__global__ void touch_kernel(uint2* a, unsigned n) {
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    uint2 v = a[i];
    v.x += 1;
    a[i] = v;
  }
}

// Grid barrier: one arrival counter and a generation word in global memory, vector atomics.
// The spin is bounded: a barrier that never completes sets *err and lets the wave go on, so
// the grid always drains.
__device__ void grid_barrier(unsigned* count, unsigned* gen, unsigned nblocks, unsigned* err) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned g = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned arrived =
        __hip_atomic_fetch_add(count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (arrived == nblocks - 1) {
      __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(gen, g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      unsigned spins = 0;
      while (__hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) {
        if (++spins > (1u << 22)) {
          __hip_atomic_fetch_add(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
  }
  __syncthreads();
}

__global__ void coop_kernel(uint2* a, unsigned n, unsigned iters, unsigned* count, unsigned* gen,
                            unsigned* err) {
  for (unsigned it = 0; it < iters; ++it) {
    if (a) {
      for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        uint2 v = a[i];
        v.x += 1;
        a[i] = v;
      }
    }
    grid_barrier(count, gen, gridDim.x, err);
  }
}

static float time_ms(hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
  float ms;
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms;
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const unsigned n = 65536;
  uint2* a;
  CK(hipMalloc(&a, n * sizeof(uint2)));
  CK(hipMemset(a, 0, n * sizeof(uint2)));
  unsigned* sync;
  CK(hipMalloc(&sync, 3 * sizeof(unsigned)));
  CK(hipMemset(sync, 0, 3 * sizeof(unsigned)));
  const int reps = 2000;

  for (int w = 0; w < 200; ++w) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
  CK(hipStreamSynchronize(s));
  CK(hipEventRecord(e0, s));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
  CK(hipEventRecord(e1, s));
  std::printf("{\"probe\": \"empty kernel, stream\", \"us_per_launch\": %.3f}\n", time_ms(s, e0, e1) * 1e3 / reps);

  for (unsigned blocks : {32u, 128u, 256u}) {
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(touch_kernel, dim3(blocks), dim3(256), 0, s, a, n);
    CK(hipEventRecord(e1, s));
    std::printf("{\"probe\": \"touch 64Ki x 8 B, stream\", \"blocks\": %u, \"us_per_launch\": %.3f}\n", blocks,
                time_ms(s, e0, e1) * 1e3 / reps);
  }

  // The same chain captured once and replayed.
  {
    const int len = 100;
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int r = 0; r < len; ++r) hipLaunchKernelGGL(touch_kernel, dim3(256), dim3(256), 0, s, a, n);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < reps / len; ++r) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e1, s));
    std::printf("{\"probe\": \"touch 64Ki x 8 B, graph of %d\", \"us_per_launch\": %.3f}\n", len,
                time_ms(s, e0, e1) * 1e3 / (reps / len * len));
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }

  int dev = 0, coop = 0, cus = 0, per_cu = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, coop_kernel, 256, 0));
  std::printf("{\"cooperative\": %d, \"cus\": %d, \"blocks_per_cu\": %d}\n", coop, cus, per_cu);
  if (!coop || per_cu < 1) return 0;
  for (unsigned blocks : {32u, 128u, 256u}) {
    if (blocks > (unsigned)(cus * per_cu)) continue;
    for (int with_touch = 0; with_touch < 2; ++with_touch) {
      uint2* aa = with_touch ? a : nullptr;
      unsigned iters = 1000;
      unsigned* cnt = sync;
      unsigned* gen = sync + 1;
      unsigned* err = sync + 2;
      void* args[] = {&aa, (void*)&n, &iters, &cnt, &gen, &err};
      CK(hipEventRecord(e0, s));
      CK(hipLaunchCooperativeKernel((const void*)coop_kernel, dim3(blocks), dim3(256), args, 0, s));
      CK(hipEventRecord(e1, s));
      const float ms = time_ms(s, e0, e1);
      unsigned h[3];
      CK(hipMemcpy(h, sync, sizeof(h), hipMemcpyDeviceToHost));
      std::printf("{\"probe\": \"cooperative, grid barrier%s\", \"blocks\": %u, \"us_per_barrier\": %.3f, \"errors\": %u}\n",
                  with_touch ? " + touch" : "", blocks, ms * 1e3 / iters, h[2]);
    }
  }
  return 0;
}
