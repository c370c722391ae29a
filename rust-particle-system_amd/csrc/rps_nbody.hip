// rps_nbody.hip — all-pairs N-body kernels for gfx950 (build-defined extension, north_star
// C4/C5): float2 source tiles staged through LDS, 8 targets per
// lane as packed f32 pairs, two-level summation, source splits with a fixed-order reduce.
//
// Its own translation unit so it can be compiled with the max-ILP machine scheduler
// (Makefile): the default scheduler serialised the inner loop into dependent chains with
// ~75 hazard s_nops per 32 interactions; max-ILP interleaves the 16 independent chains
// (0 s_nops, 168 VGPRs, 3 waves/SIMD) and runs 3 % faster (tools/ab_nbody.py).
#include <hip/hip_runtime.h>

#include "rps_internal.hpp"

namespace rps {

namespace {

constexpr int kBlock = 256;  // 4 waves of 64

__global__ __launch_bounds__(kBlock) void nbody_pack_kernel(const float* x, const float* y,
                                                            f2* pos, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i < n) pos[i] = f2{x[i], y[i]};
}

__global__ __launch_bounds__(kBlock) void nbody_pad_kernel(f2* pos, uint64_t from, uint64_t to) {
  const uint64_t i = from + (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  // Far-away padding: r2 = 2e36 -> inv^3 underflows to 0, so a pad adds exactly +0.
  if (i < to) pos[i] = f2{1.0e18f, 1.0e18f};
}

constexpr int kTargetsPerLane = 8;
constexpr int kTargetPairs = kTargetsPerLane / 2;

// Each lane owns kTargetsPerLane targets as kTargetPairs float2 pairs (targets t and
// t + kBlock in one pair), so every operation of the interaction except the rsq is one
// v_pk_* instruction covering two targets: per 2 interactions 8 packed ops + 2 v_rsq_f32
// (the FP32-VALU issue floor for this formula).  Per target the arithmetic
// is the scalar formula r2 = dx*dx + (dy*dy + eps2) with explicit FMAs, unchanged.
//
// Source split (blockIdx.y): when the targets alone give too few workgroups to fill 256 CUs
// (small N, or a strong-scaled shard), the sources are cut into gridDim.y contiguous ranges
// of whole LDS tiles; each workgroup writes its raw partial sums to part[split][target] and
// nbody_reduce_kernel adds them in split order (deterministic, no atomics).
__global__ __launch_bounds__(kBlock) void nbody_accel_kernel(const f2* __restrict__ pos,
                                                             uint64_t ns_padded, uint64_t t0,
                                                             uint64_t nt, float eps2, float gm,
                                                             uint64_t split_len,
                                                             f2* __restrict__ part,
                                                             float* __restrict__ ax_out,
                                                             float* __restrict__ ay_out,
                                                             uint64_t* __restrict__ stamps) {
  static_assert(kNbodyTile / 2 == kBlock, "one float2 source pair per lane per tile");
  // Clock stamps (profiled launches only, stamps != nullptr): the workgroup's shader-clock
  // counter and 100-MHz real-time counter at its start and end, so the host can report the
  // clock the chip sustained under this kernel (MI355X_MICROARCH.md, DVFS: in-kernel clock =
  // delta s_memtime / delta s_memrealtime x 100 MHz).  Two reads per workgroup lifetime
  // (~90 ms at 2^22), written to a buffer nothing else reads; no output depends on them.
  uint64_t c0 = 0, r0 = 0;
  if (stamps && threadIdx.x == 0) {
    c0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  __shared__ f4 tile[kNbodyTile / 2];  // pairs of float2 sources
  // Two-level summation: the registers ax/ay sum one tile's 512 contributions, and each
  // lane's running totals live in LDS (tot[2p + c][lane], conflict-free 8-B accesses), added
  // once per tile.  One f32 accumulator over all sources lost ~1e-3 of |a| at 2^22 sources
  // (the error grows with the contributions per sum); per-tile sums keep it near 1e-6 at
  // every N (tools/nbody_diag.py).  Keeping the totals in LDS instead of 16 more VGPRs
  // leaves the inner loop's register budget, and so its schedule, unchanged.
  __shared__ f2 tot[2 * kTargetPairs][kBlock];
  const uint64_t base = (uint64_t)blockIdx.x * kBlock * kTargetsPerLane;
  f2 tx[kTargetPairs], ty[kTargetPairs], ax[kTargetPairs], ay[kTargetPairs];
#pragma unroll
  for (int p = 0; p < kTargetPairs; ++p) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint64_t t = base + threadIdx.x + (uint64_t)(2 * p + h) * kBlock;
      const f2 q = t < nt ? pos[t0 + t] : f2{0.0f, 0.0f};
      tx[p][h] = q[0];
      ty[p][h] = q[1];
    }
    tot[2 * p][threadIdx.x] = f2{0.0f, 0.0f};
    tot[2 * p + 1][threadIdx.x] = f2{0.0f, 0.0f};
  }
  const f2 e2 = {eps2, eps2};
  const f4* src4 = reinterpret_cast<const f4*>(pos);
  const uint64_t s_begin = (uint64_t)blockIdx.y * split_len;
  const uint64_t s_end = s_begin + split_len < ns_padded ? s_begin + split_len : ns_padded;
  // The next tile's sources are loaded into registers while this one is computed.
  f4 next = s_begin < s_end ? src4[(s_begin >> 1) + threadIdx.x] : f4{0.0f, 0.0f, 0.0f, 0.0f};
  for (uint64_t s0 = s_begin; s0 < s_end; s0 += kNbodyTile) {
    __syncthreads();
    tile[threadIdx.x] = next;
    __syncthreads();
    if (s0 + kNbodyTile < s_end) next = src4[((s0 + kNbodyTile) >> 1) + threadIdx.x];
#pragma unroll
    for (int p = 0; p < kTargetPairs; ++p) {
      ax[p] = f2{0.0f, 0.0f};
      ay[p] = f2{0.0f, 0.0f};
    }
#pragma unroll 2
    for (uint32_t q = 0; q < kNbodyTile / 2; ++q) {
      const f4 sp = tile[q];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f2 sx = {sp[2 * h], sp[2 * h]}, sy = {sp[2 * h + 1], sp[2 * h + 1]};
#pragma unroll
        for (int p = 0; p < kTargetPairs; ++p) {
          const f2 dx = sx - tx[p];
          const f2 dy = sy - ty[p];
          const f2 r2 = __builtin_elementwise_fma(dx, dx, __builtin_elementwise_fma(dy, dy, e2));
          const f2 inv = {__builtin_amdgcn_rsqf(r2[0]), __builtin_amdgcn_rsqf(r2[1])};
          const f2 inv3 = (inv * inv) * inv;
          ax[p] = __builtin_elementwise_fma(dx, inv3, ax[p]);
          ay[p] = __builtin_elementwise_fma(dy, inv3, ay[p]);
        }
      }
    }
#pragma unroll
    for (int p = 0; p < kTargetPairs; ++p) {
      tot[2 * p][threadIdx.x] += ax[p];
      tot[2 * p + 1][threadIdx.x] += ay[p];
    }
  }
#pragma unroll
  for (int p = 0; p < kTargetPairs; ++p) {
    ax[p] = tot[2 * p][threadIdx.x];
    ay[p] = tot[2 * p + 1][threadIdx.x];
  }
#pragma unroll
  for (int p = 0; p < kTargetPairs; ++p) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint64_t t = base + threadIdx.x + (uint64_t)(2 * p + h) * kBlock;
      if (t < nt) {
        if (part) {
          part[(uint64_t)blockIdx.y * nt + t] = f2{ax[p][h], ay[p][h]};
        } else {
          ax_out[t] = ax[p][h] * gm;
          ay_out[t] = ay[p][h] * gm;
        }
      }
    }
  }
  if (stamps && threadIdx.x == 0) {
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    const uint64_t wg = (uint64_t)blockIdx.y * gridDim.x + blockIdx.x;
    reinterpret_cast<ulonglong2*>(stamps)[wg] = make_ulonglong2(c1 - c0, r1 - r0);
  }
}

__global__ __launch_bounds__(kBlock) void nbody_reduce_kernel(const f2* __restrict__ part,
                                                              uint32_t splits, uint64_t nt,
                                                              float gm, float* __restrict__ ax_out,
                                                              float* __restrict__ ay_out) {
  const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (t >= nt) return;
  f2 a = part[t];
  for (uint32_t s = 1; s < splits; ++s) a += part[(uint64_t)s * nt + t];
  ax_out[t] = a[0] * gm;
  ay_out[t] = a[1] * gm;
}

__global__ __launch_bounds__(kBlock) void nbody_integrate_kernel(NbodyIntegrateArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= a.n) return;
  float px = a.x[i], py = a.y[i], qx = a.vx[i], qy = a.vy[i];
  qx = qx + a.gx_dt;
  qy = qy + a.gy_dt;
  qx = qx + a.ax[i] * a.dt;
  qy = qy + a.ay[i] * a.dt;
  if (a.drag_on) {
    qx = qx * a.drag_f;
    qy = qy * a.drag_f;
  }
  px = px + qx * a.dt;
  py = py + qy * a.dt;
  wall(a.x_min, a.x_max, a.y_min, a.y_max, a.damping, px, py, qx, qy);
  a.x[i] = px;
  a.y[i] = py;
  a.vx[i] = qx;
  a.vy[i] = qy;
}

inline uint32_t blocks_for(uint64_t n, uint32_t per_block = kBlock) {
  return (uint32_t)((n + per_block - 1) / per_block);
}

}  // namespace

hipError_t launch_nbody_pack(const float* x, const float* y, f2* pos, uint64_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(nbody_pack_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, s, x, y, pos, n);
  return hipGetLastError();
}

hipError_t launch_nbody_pad(f2* pos, uint64_t from, uint64_t to, hipStream_t s) {
  if (to <= from) return hipSuccess;
  hipLaunchKernelGGL(nbody_pad_kernel, dim3(blocks_for(to - from)), dim3(kBlock), 0, s, pos, from,
                     to);
  return hipGetLastError();
}

uint32_t nbody_splits_for(uint64_t nt, uint64_t ns_padded) {
  if (nt == 0) return 1;
  const uint64_t tb = blocks_for(nt, kBlock * kTargetsPerLane);
  const uint64_t tiles = ns_padded / kNbodyTile;
  uint64_t s = (kNbodyMinBlocks + tb - 1) / tb;
  if (s > kNbodyMaxSplits) s = kNbodyMaxSplits;
  if (s > tiles) s = tiles;
  return s < 1 ? 1u : (uint32_t)s;
}

// The split count a launch actually uses: splits of whole tiles, none of them empty.
static uint32_t launch_splits(uint64_t ns_padded, uint32_t splits, uint64_t* split_len) {
  const uint64_t tiles = ns_padded / kNbodyTile;
  if (splits < 1) splits = 1;
  if (splits > tiles) splits = (uint32_t)tiles;
  *split_len = (tiles + splits - 1) / splits * kNbodyTile;
  return (uint32_t)((ns_padded + *split_len - 1) / *split_len);
}

uint64_t nbody_workgroups(uint64_t nt, uint64_t ns_padded, uint32_t splits) {
  uint64_t len;
  return (uint64_t)blocks_for(nt, kBlock * kTargetsPerLane) * launch_splits(ns_padded, splits, &len);
}

hipError_t launch_nbody_accel(const f2* pos, uint64_t ns_padded, uint64_t t0, uint64_t nt,
                              float eps2, float gm, f2* part, uint32_t splits, float* ax,
                              float* ay, uint64_t* stamps, hipStream_t s) {
  if (nt == 0) return hipSuccess;
  uint64_t split_len;
  splits = launch_splits(ns_padded, splits, &split_len);
  f2* p = splits > 1 ? part : nullptr;
  hipLaunchKernelGGL(nbody_accel_kernel, dim3(blocks_for(nt, kBlock * kTargetsPerLane), splits),
                     dim3(kBlock), 0, s, pos, ns_padded, t0, nt, eps2, gm, split_len, p, ax, ay, stamps);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !p) return e;
  hipLaunchKernelGGL(nbody_reduce_kernel, dim3(blocks_for(nt)), dim3(kBlock), 0, s, p, splits, nt, gm,
                     ax, ay);
  return hipGetLastError();
}

hipError_t launch_nbody_integrate(const NbodyIntegrateArgs& a, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  hipLaunchKernelGGL(nbody_integrate_kernel, dim3(blocks_for(a.n)), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

}  // namespace rps
