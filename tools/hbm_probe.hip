// hbm_probe.hip — practical HBM ceilings on this MI355X for the stream kernel's access
// pattern (known-good reference for the roofline fraction; cdna_hip_programming.md §5.4
// rule 10).  Standalone:  hipcc --offload-arch=gfx950 -O3 -o hbm_probe tools/hbm_probe.hip
//   copy      : float4 src -> dst                      (read B, write B)
//   rmw5      : 5 SoA float arrays updated in place    (read 5B/5, write 5B/5) == stream kernel shape
//   read      : float4 sum (one atomic per block)      (read only)
//   write     : float4 fill                            (write only)
// each with plain and nontemporal accesses, one-shot grids, 256-thread blocks.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <utility>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

template <bool NT>
__device__ __forceinline__ f4 ld(const f4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  return *p;
}
template <bool NT>
__device__ __forceinline__ void st(f4* p, f4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

template <bool NT>
__global__ __launch_bounds__(256) void copy_k(const f4* __restrict__ a, f4* __restrict__ b, size_t n4) {
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n4) st<NT>(b + i, ld<NT>(a + i));
}

template <bool NT>
__global__ __launch_bounds__(256) void rmw5_k(f4* a, f4* b, f4* c, f4* d, f4* e, size_t n4, float s) {
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  f4 A = ld<NT>(a + i), B = ld<NT>(b + i), C = ld<NT>(c + i), D = ld<NT>(d + i), E = ld<NT>(e + i);
  st<NT>(a + i, A * s + B);
  st<NT>(b + i, B * s + C);
  st<NT>(c + i, C * s + D);
  st<NT>(d + i, D * s + E);
  st<NT>(e + i, E * s + A);
}

// Out-of-place: 5 input arrays -> 5 output arrays.
template <bool NT>
__global__ __launch_bounds__(256) void copy5_k(const f4* a, const f4* b, const f4* c, const f4* d,
                                               const f4* e, f4* A_, f4* B_, f4* C_, f4* D_, f4* E_,
                                               size_t n4, float s) {
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  f4 A = ld<NT>(a + i), B = ld<NT>(b + i), C = ld<NT>(c + i), D = ld<NT>(d + i), E = ld<NT>(e + i);
  st<NT>(A_ + i, A * s + B);
  st<NT>(B_ + i, B * s + C);
  st<NT>(C_ + i, C * s + D);
  st<NT>(D_ + i, D * s + E);
  st<NT>(E_ + i, E * s + A);
}

// Tiled SoA (AoSoA): tiles of T particles, each tile = 5 contiguous field segments of T
// floats.  One workgroup (256 lanes x 4 particles) covers 1024 particles.
template <bool NT, int T>
__global__ __launch_bounds__(256) void rmw5_tiled_k(f4* base, size_t n4, float s) {
  size_t v = (size_t)blockIdx.x * 256 + threadIdx.x;  // float4 index within the field view
  if (v >= n4) return;
  constexpr size_t T4 = T / 4;
  const size_t tile = v / T4, w = v % T4;
  f4* t = base + tile * 5 * T4 + w;
  f4 A = ld<NT>(t), B = ld<NT>(t + T4), C = ld<NT>(t + 2 * T4), D = ld<NT>(t + 3 * T4), E = ld<NT>(t + 4 * T4);
  st<NT>(t, A * s + B);
  st<NT>(t + T4, B * s + C);
  st<NT>(t + 2 * T4, C * s + D);
  st<NT>(t + 3 * T4, D * s + E);
  st<NT>(t + 4 * T4, E * s + A);
}

// Tiled, U float4 per lane per field (U consecutive 1 KiB wave slices).
template <bool NT, int T, int U>
__global__ __launch_bounds__(256) void rmw5_tiled_u_k(f4* base, size_t n4, float s) {
  constexpr size_t T4 = T / 4;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    size_t v = ((size_t)blockIdx.x * U + u) * 256 + threadIdx.x;
    if (v >= n4) return;
    const size_t tile = v / T4, w = v % T4;
    f4* t = base + tile * 5 * T4 + w;
    f4 A = ld<NT>(t), B = ld<NT>(t + T4), C = ld<NT>(t + 2 * T4), D = ld<NT>(t + 3 * T4), E = ld<NT>(t + 4 * T4);
    st<NT>(t, A * s + B);
    st<NT>(t + T4, B * s + C);
    st<NT>(t + 2 * T4, C * s + D);
    st<NT>(t + 3 * T4, D * s + E);
    st<NT>(t + 4 * T4, E * s + A);
  }
}

// XCD-aware block order: blocks are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md
// "Workgroup dispatch"), so remap b -> a contiguous chunk per XCD (bijection for any G).
__device__ __forceinline__ size_t xcd_block(size_t b, size_t G) {
  const size_t q = G / 8, r = G % 8, x = b % 8, k = b / 8;
  return x * q + (x < r ? x : r) + k;
}

// Tiled, optional XCD remap, optional ping-pong (read src tiles, write dst tiles).
template <bool NT, int T, bool XCD, bool PP>
__global__ __launch_bounds__(256) void rmw5_tiled_x_k(f4* src, f4* dst, size_t n4, float s) {
  const size_t b = XCD ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
  size_t v = b * 256 + threadIdx.x;
  if (v >= n4) return;
  constexpr size_t T4 = T / 4;
  const size_t tile = v / T4, w = v % T4;
  const size_t off = tile * 5 * T4 + w;
  const f4* t = src + off;
  f4* u = (PP ? dst : src) + off;
  f4 A = ld<NT>(t), B = ld<NT>(t + T4), C = ld<NT>(t + 2 * T4), D = ld<NT>(t + 3 * T4), E = ld<NT>(t + 4 * T4);
  st<NT>(u, A * s + B);
  st<NT>(u + T4, B * s + C);
  st<NT>(u + 2 * T4, C * s + D);
  st<NT>(u + 3 * T4, D * s + E);
  st<NT>(u + 4 * T4, E * s + A);
}

// Flat in-place float4 update (one stream, field-agnostic) over the same 5n-float buffer.
template <bool NT>
__global__ __launch_bounds__(256) void flat_rmw_k(f4* a, size_t n4, float s) {
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n4) st<NT>(a + i, ld<NT>(a + i) * s + 1.0f);
}

// Flat, U float4 per lane spaced by the grid's wave slice (loads first, then stores).
template <bool NT, int U>
__global__ __launch_bounds__(256) void flat_rmw_u_k(f4* a, size_t n4, float s) {
  const size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x;
  f4 r[U];
#pragma unroll
  for (int u = 0; u < U; ++u) if (base + u * 256 < n4) r[u] = ld<NT>(a + base + u * 256);
#pragma unroll
  for (int u = 0; u < U; ++u) if (base + u * 256 < n4) st<NT>(a + base + u * 256, r[u] * s + 1.0f);
}

// Expiry layout: tiles of T particles = 4 float segments + one u16 segment (T*18 B).
// x,y,vx,vy read+written, the u16 expiry read (written only where it matches: never here).
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
template <int T, bool EXP>
__global__ __launch_bounds__(256) void rmw4e_k(f4* base, size_t n4, float s, unsigned short key) {
  size_t v = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= n4) return;
  constexpr size_t T4 = T / 4;
  const size_t tile = v / T4, w = v % T4;
  f4* t = base + tile * (EXP ? 18 : 16) * T4 / 4 + w;  // tile stride in f4: T*18/16
  f4 A = __builtin_nontemporal_load(t), B = __builtin_nontemporal_load(t + T4),
     C = __builtin_nontemporal_load(t + 2 * T4), D = __builtin_nontemporal_load(t + 3 * T4);
  bool hit = false;
  if constexpr (EXP) {
    const u16x4* e = reinterpret_cast<const u16x4*>(t - w + 4 * T4) + w;
    u16x4 E = __builtin_nontemporal_load(e);
    hit = E[0] == key || E[1] == key || E[2] == key || E[3] == key;
  }
  if (hit) A = A + 1.0f;
  __builtin_nontemporal_store(A * s + B, t);
  __builtin_nontemporal_store(B * s + C, t + T4);
  __builtin_nontemporal_store(C * s + D, t + 2 * T4);
  __builtin_nontemporal_store(D * s + A, t + 3 * T4);
}

// Tiled, every store depending on its own load only (as flat_rmw_u).
template <int T>
__global__ __launch_bounds__(256) void rmw5_tiled_indep_k(f4* base, size_t n4, float s) {
  size_t v = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= n4) return;
  constexpr size_t T4 = T / 4;
  const size_t tile = v / T4, w = v % T4;
  f4* t = base + tile * 5 * T4 + w;
  f4 A = ld<true>(t), B = ld<true>(t + T4), C = ld<true>(t + 2 * T4), D = ld<true>(t + 3 * T4), E = ld<true>(t + 4 * T4);
  st<true>(t, A * s + 1.0f);
  st<true>(t + T4, B * s + 1.0f);
  st<true>(t + 2 * T4, C * s + 1.0f);
  st<true>(t + 3 * T4, D * s + 1.0f);
  st<true>(t + 4 * T4, E * s + 1.0f);
}

// Tiled with all stores depending on all loads (the particle step's shape).
template <int T>
__global__ __launch_bounds__(256) void rmw5_tiled_all_k(f4* base, size_t n4, float s) {
  size_t v = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= n4) return;
  constexpr size_t T4 = T / 4;
  const size_t tile = v / T4, w = v % T4;
  f4* t = base + tile * 5 * T4 + w;
  f4 A = ld<true>(t), B = ld<true>(t + T4), C = ld<true>(t + 2 * T4), D = ld<true>(t + 3 * T4), E = ld<true>(t + 4 * T4);
  const f4 S = (A + B) + (C + D) + E;
  st<true>(t, A * s + S);
  st<true>(t + T4, B * s + S);
  st<true>(t + 2 * T4, C * s + S);
  st<true>(t + 3 * T4, D * s + S);
  st<true>(t + 4 * T4, E * s + S);
}

// Same with 512-thread workgroups.
template <bool NT, int T>
__global__ __launch_bounds__(512) void rmw5_tiled_b512_k(f4* base, size_t n4, float s) {
  size_t v = (size_t)blockIdx.x * 512 + threadIdx.x;
  if (v >= n4) return;
  constexpr size_t T4 = T / 4;
  const size_t tile = v / T4, w = v % T4;
  f4* t = base + tile * 5 * T4 + w;
  f4 A = ld<NT>(t), B = ld<NT>(t + T4), C = ld<NT>(t + 2 * T4), D = ld<NT>(t + 3 * T4), E = ld<NT>(t + 4 * T4);
  st<NT>(t, A * s + B);
  st<NT>(t + T4, B * s + C);
  st<NT>(t + 2 * T4, C * s + D);
  st<NT>(t + 3 * T4, D * s + E);
  st<NT>(t + 4 * T4, E * s + A);
}

template <bool NT>
__global__ __launch_bounds__(256) void rmw4_k(f4* a, f4* b, f4* c, f4* d, size_t n4, float s) {
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  f4 A = ld<NT>(a + i), B = ld<NT>(b + i), C = ld<NT>(c + i), D = ld<NT>(d + i);
  st<NT>(a + i, A * s + B);
  st<NT>(b + i, B * s + C);
  st<NT>(c + i, C * s + D);
  st<NT>(d + i, D * s + A);
}

template <bool NT>
__global__ __launch_bounds__(256) void read_k(const f4* __restrict__ a, size_t n4, float* out) {
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  float v = 0.f;
  if (i < n4) {
    f4 x = ld<NT>(a + i);
    v = x[0] + x[1] + x[2] + x[3];
  }
  for (int o = 32; o; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0 && v == 12345.678f) atomicAdd(out, v);  // keep the load live
}

template <bool NT>
__global__ __launch_bounds__(256) void write_k(f4* __restrict__ a, size_t n4, float s) {
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n4) st<NT>(a + i, f4{s, s, s, s});
}

int main(int argc, char** argv) {
  const size_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 100000000ull;  // floats per array
  const size_t n4 = n / 4;
  const int reps = 50;
  std::vector<float*> arr(5);
  for (auto& p : arr) {
    CHECK(hipMalloc(&p, n * sizeof(float)));
    CHECK(hipMemset(p, 0, n * sizeof(float)));
  }
  float* out;
  CHECK(hipMalloc(&out, sizeof(float)));
  // 10 GB copy pair: two 2.5 GB buffers (== 5 x 4e8 B of the rmw5 shape split in halves)
  const size_t cbytes = 5 * n * sizeof(float) / 2, c4 = cbytes / 16;
  f4 *ca, *cb;
  CHECK(hipMalloc(&ca, cbytes));
  CHECK(hipMalloc(&cb, cbytes));
  CHECK(hipMemset(ca, 0, cbytes));
  hipEvent_t t0, t1;
  CHECK(hipEventCreate(&t0));
  CHECK(hipEventCreate(&t1));
  auto run = [&](const char* name, double bytes, auto&& launch) {
    for (int w = 0; w < 20; ++w) launch();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(t0));
    for (int r = 0; r < reps; ++r) launch();
    CHECK(hipEventRecord(t1));
    CHECK(hipEventSynchronize(t1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, t0, t1));
    ms /= reps;
    std::printf("%-14s %8.4f ms  %7.0f GB/s  (%.3g B)\n", name, ms, bytes / (ms * 1e-3) / 1e9, bytes);
  };
  const unsigned g = (unsigned)((n4 + 255) / 256), gc = (unsigned)((c4 + 255) / 256);
  f4 *a = (f4*)arr[0], *b = (f4*)arr[1], *c = (f4*)arr[2], *d = (f4*)arr[3], *e = (f4*)arr[4];
  std::vector<float*> arr2(5);
  for (auto& p : arr2) {
    CHECK(hipMalloc(&p, n * sizeof(float)));
    CHECK(hipMemset(p, 0, n * sizeof(float)));
  }
  f4 *a2 = (f4*)arr2[0], *b2 = (f4*)arr2[1], *c2 = (f4*)arr2[2], *d2 = (f4*)arr2[3], *e2 = (f4*)arr2[4];
  f4* tiled = ca;  // 5 n floats fit exactly in the 2.5n-float copy buffer pair? use ca+cb span
  (void)tiled;
  f4* tb;
  CHECK(hipMalloc(&tb, 5 * n * sizeof(float)));
  CHECK(hipMemset(tb, 0, 5 * n * sizeof(float)));
  f4* tb2;
  CHECK(hipMalloc(&tb2, 5 * n * sizeof(float)));
  CHECK(hipMemset(tb2, 0, 5 * n * sizeof(float)));
  const bool only_new = argc > 2;
  for (int round = 0; round < 2; ++round) {
    std::printf("-- round %d (n = %zu floats/array)\n", round, n);
    run("t8192 nt", 40.0 * n, [&] { hipLaunchKernelGGL((rmw5_tiled_k<true, 8192>), dim3(g), dim3(256), 0, 0, tb, n4, 1.0f); });
    run("t8192 xcd", 40.0 * n, [&] { hipLaunchKernelGGL((rmw5_tiled_x_k<true, 8192, true, false>), dim3(g), dim3(256), 0, 0, tb, tb, n4, 1.0f); });
    run("pp8192 nt", 40.0 * n, [&] { hipLaunchKernelGGL((rmw5_tiled_x_k<true, 8192, false, true>), dim3(g), dim3(256), 0, 0, tb, tb2, n4, 1.0f); std::swap(tb, tb2); });
    run("pp8192 xcd", 40.0 * n, [&] { hipLaunchKernelGGL((rmw5_tiled_x_k<true, 8192, true, true>), dim3(g), dim3(256), 0, 0, tb, tb2, n4, 1.0f); std::swap(tb, tb2); });
    run("pp65536 nt", 40.0 * n, [&] { hipLaunchKernelGGL((rmw5_tiled_x_k<true, 65536, false, true>), dim3(g), dim3(256), 0, 0, tb, tb2, n4, 1.0f); std::swap(tb, tb2); });
    run("t8192 b512", 40.0 * n, [&] { hipLaunchKernelGGL((rmw5_tiled_b512_k<true, 8192>), dim3((g + 1) / 2), dim3(512), 0, 0, tb, n4, 1.0f); });
    run("copy5 nt", 40.0 * n, [&] { hipLaunchKernelGGL(copy5_k<true>, dim3(g), dim3(256), 0, 0, a, b, c, d, e, a2, b2, c2, d2, e2, n4, 1.0f); });
    const size_t f4n = 5 * n4;
    const unsigned gf = (unsigned)((f4n + 255) / 256);
    run("flat rmw", 40.0 * n, [&] { hipLaunchKernelGGL(flat_rmw_k<true>, dim3(gf), dim3(256), 0, 0, tb, f4n, 1.0f); });
    run("flat rmw u5", 40.0 * n, [&] { hipLaunchKernelGGL((flat_rmw_u_k<true, 5>), dim3((gf + 4) / 5), dim3(256), 0, 0, tb, f4n, 1.0f); });
    run("flat rmw u4", 40.0 * n, [&] { hipLaunchKernelGGL((flat_rmw_u_k<true, 4>), dim3((gf + 3) / 4), dim3(256), 0, 0, tb, f4n, 1.0f); });
    run("flat copy", 40.0 * n, [&] { hipLaunchKernelGGL(copy_k<true>, dim3(gf), dim3(256), 0, 0, tb, tb2, f4n); std::swap(tb, tb2); });
    run("t1024 indep", 40.0 * n, [&] { hipLaunchKernelGGL((rmw5_tiled_indep_k<1024>), dim3(g), dim3(256), 0, 0, tb, n4, 1.0f); });
    run("t8192 indep", 40.0 * n, [&] { hipLaunchKernelGGL((rmw5_tiled_indep_k<8192>), dim3(g), dim3(256), 0, 0, tb, n4, 1.0f); });
    run("t1024 all", 40.0 * n, [&] { hipLaunchKernelGGL((rmw5_tiled_all_k<1024>), dim3(g), dim3(256), 0, 0, tb, n4, 1.0f); });
    run("t8192 all", 40.0 * n, [&] { hipLaunchKernelGGL((rmw5_tiled_all_k<8192>), dim3(g), dim3(256), 0, 0, tb, n4, 1.0f); });
    run("t1024 nt", 40.0 * n, [&] { hipLaunchKernelGGL((rmw5_tiled_k<true, 1024>), dim3(g), dim3(256), 0, 0, tb, n4, 1.0f); });
    run("t8192 4f+u16", 34.0 * n, [&] { hipLaunchKernelGGL((rmw4e_k<8192, true>), dim3(g), dim3(256), 0, 0, tb, n4, 1.0f, (unsigned short)7); });
    run("t8192 4f", 32.0 * n, [&] { hipLaunchKernelGGL((rmw4e_k<8192, false>), dim3(g), dim3(256), 0, 0, tb, n4, 1.0f, (unsigned short)7); });
    run("t4096 4f+u16", 34.0 * n, [&] { hipLaunchKernelGGL((rmw4e_k<4096, true>), dim3(g), dim3(256), 0, 0, tb, n4, 1.0f, (unsigned short)7); });
    run("t16384 4f+u16", 34.0 * n, [&] { hipLaunchKernelGGL((rmw4e_k<16384, true>), dim3(g), dim3(256), 0, 0, tb, n4, 1.0f, (unsigned short)7); });
    if (only_new) continue;
    run("rmw5 nt", 40.0 * n, [&] { hipLaunchKernelGGL(rmw5_k<true>, dim3(g), dim3(256), 0, 0, a, b, c, d, e, n4, 1.0f); });
    run("t1024 nt", 40.0 * n, [&] { hipLaunchKernelGGL((rmw5_tiled_k<true, 1024>), dim3(g), dim3(256), 0, 0, tb, n4, 1.0f); });
    run("t2048 nt", 40.0 * n, [&] { hipLaunchKernelGGL((rmw5_tiled_k<true, 2048>), dim3(g), dim3(256), 0, 0, tb, n4, 1.0f); });
    run("t4096 nt", 40.0 * n, [&] { hipLaunchKernelGGL((rmw5_tiled_k<true, 4096>), dim3(g), dim3(256), 0, 0, tb, n4, 1.0f); });
    run("t8192 nt", 40.0 * n, [&] { hipLaunchKernelGGL((rmw5_tiled_k<true, 8192>), dim3(g), dim3(256), 0, 0, tb, n4, 1.0f); });
    run("t16384 nt", 40.0 * n, [&] { hipLaunchKernelGGL((rmw5_tiled_k<true, 16384>), dim3(g), dim3(256), 0, 0, tb, n4, 1.0f); });
    run("t65536 nt", 40.0 * n, [&] { hipLaunchKernelGGL((rmw5_tiled_k<true, 65536>), dim3(g), dim3(256), 0, 0, tb, n4, 1.0f); });
    run("t4096 plain", 40.0 * n, [&] { hipLaunchKernelGGL((rmw5_tiled_k<false, 4096>), dim3(g), dim3(256), 0, 0, tb, n4, 1.0f); });
    run("t4096u2 nt", 40.0 * n, [&] { hipLaunchKernelGGL((rmw5_tiled_u_k<true, 4096, 2>), dim3((g + 1) / 2), dim3(256), 0, 0, tb, n4, 1.0f); });
    run("t4096u4 nt", 40.0 * n, [&] { hipLaunchKernelGGL((rmw5_tiled_u_k<true, 4096, 4>), dim3((g + 3) / 4), dim3(256), 0, 0, tb, n4, 1.0f); });
    run("t8192u2 nt", 40.0 * n, [&] { hipLaunchKernelGGL((rmw5_tiled_u_k<true, 8192, 2>), dim3((g + 1) / 2), dim3(256), 0, 0, tb, n4, 1.0f); });
    run("copy nt", 2.0 * cbytes, [&] { hipLaunchKernelGGL(copy_k<true>, dim3(gc), dim3(256), 0, 0, ca, cb, c4); });
  }
  return 0;
}
