// rps_kernels.hip — hand-written gfx950 kernels for the per-particle step.
//
// Reference hot path: ParticleComputeNode::run (src/particle_compute.rs:91-195) dispatching
// the five WGSL entry points of assets/compute_shader.wgsl.  Layout and roofline of each
// kernel: DESIGN.md §4-§5.  Built with -ffp-contract=off (see rps_device.hpp).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "rps_internal.hpp"

namespace rps {

namespace {

constexpr int kBlock = 256;  // 4 waves of 64

template <bool NT>
__device__ __forceinline__ f4 ld4(const float* p) {
  if constexpr (NT) {
    return __builtin_nontemporal_load(reinterpret_cast<const f4*>(p));
  } else {
    return *reinterpret_cast<const f4*>(p);
  }
}

template <bool NT>
__device__ __forceinline__ void st4(float* p, f4 v) {
  if constexpr (NT) {
    __builtin_nontemporal_store(v, reinterpret_cast<f4*>(p));
  } else {
    *reinterpret_cast<f4*>(p) = v;
  }
}

// One u16 [next] entry per lane (the quad's earliest expiry).
template <bool NT>
__device__ __forceinline__ uint16_t ldn(const uint16_t* p) {
  if constexpr (NT) {
    return __builtin_nontemporal_load(p);
  } else {
    return *p;
  }
}
template <bool NT>
__device__ __forceinline__ void stn(uint16_t* p, uint16_t v) {
  if constexpr (NT) {
    __builtin_nontemporal_store(v, p);
  } else {
    *p = v;
  }
}

// Four u16 expiries (8 B per lane, 512 B per wave).
typedef uint16_t h4 __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ h4 lde4(const uint16_t* p) {
  if constexpr (NT) {
    return __builtin_nontemporal_load(reinterpret_cast<const h4*>(p));
  } else {
    return *reinterpret_cast<const h4*>(p);
  }
}
template <bool NT>
__device__ __forceinline__ void ste4(uint16_t* p, h4 v) {
  if constexpr (NT) {
    __builtin_nontemporal_store(v, reinterpret_cast<h4*>(p));
  } else {
    *reinterpret_cast<h4*>(p) = v;
  }
}

struct StatsAcc {
  float x0, x1, y0, y1;
  double ke;
  unsigned long long count, respawned;
  __device__ void init() {
    x0 = y0 = __builtin_huge_valf();
    x1 = y1 = -__builtin_huge_valf();
    ke = 0.0;
    count = respawned = 0;
  }
  __device__ void add(float x, float y, float vx, float vy, bool re) {
    x0 = fminf(x0, x);
    x1 = fmaxf(x1, x);
    y0 = fminf(y0, y);
    y1 = fmaxf(y1, y);
    ke += 0.5 * ((double)vx * (double)vx + (double)vy * (double)vy);
    count += 1;
    respawned += re ? 1 : 0;
  }
};

// wave64 butterfly reduction, then the 4 waves of the workgroup through LDS; lane 0 of
// wave 0 writes the workgroup's partial (no atomics: the finalize pass sums partials in a
// fixed order, so the stats are reproducible run to run).
__device__ void block_reduce_stats(StatsAcc acc, StatsPartial* out) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    acc.x0 = fminf(acc.x0, __shfl_xor(acc.x0, off, 64));
    acc.x1 = fmaxf(acc.x1, __shfl_xor(acc.x1, off, 64));
    acc.y0 = fminf(acc.y0, __shfl_xor(acc.y0, off, 64));
    acc.y1 = fmaxf(acc.y1, __shfl_xor(acc.y1, off, 64));
    acc.ke += __shfl_xor(acc.ke, off, 64);
    acc.count += __shfl_xor(acc.count, off, 64);
    acc.respawned += __shfl_xor(acc.respawned, off, 64);
  }
  __shared__ StatsAcc waves[kBlock / 64];
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) waves[wave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    StatsAcc t = waves[0];
#pragma unroll
    for (int w = 1; w < kBlock / 64; ++w) {
      t.x0 = fminf(t.x0, waves[w].x0);
      t.x1 = fmaxf(t.x1, waves[w].x1);
      t.y0 = fminf(t.y0, waves[w].y0);
      t.y1 = fmaxf(t.y1, waves[w].y1);
      t.ke += waves[w].ke;
      t.count += waves[w].count;
      t.respawned += waves[w].respawned;
    }
    StatsPartial p;
    p.bbox[0] = t.x0;
    p.bbox[1] = t.x1;
    p.bbox[2] = t.y0;
    p.bbox[3] = t.y1;
    p.ke = t.ke;
    p.count = t.count;
    p.respawned = t.respawned;
    p._pad = 0;
    out[blockIdx.x] = p;
  }
}

// ---------------------------------------------------------------------------------------
// Streaming step: one fused pass per active step.  SoA x|y|vx|vy read and written
// in place with 16-B vector accesses (4 particles per lane), grid-stride.  32 B/particle
// of x, y, vx, vy read+write; with lifetime +2 B per 64 particles: the group's [next] (its
// earliest expiry), and the group's 64 expiries (one 128-B line) read, and written on
// respawn, only when one is due: 32.03 B per particle plus ~19 % of groups' expiry lines at
// C3.
// ---------------------------------------------------------------------------------------
// NTM: bit 0 = nontemporal loads, bit 1 = nontemporal stores.  Workgroup b takes block b: an
// XCD-contiguous numbering (each XCD one range of tiles) was measured 3 % slower.

// The attractor table inside this launch's kernarg segment (see StreamArgs::att).
template <class Args>
__device__ __forceinline__ att_ptr kernarg_f4(size_t offset) {
  typedef __attribute__((address_space(4))) const char* kchar;
  return (att_ptr)((kchar)__builtin_amdgcn_kernarg_segment_ptr() + offset);
}

// Four particles of one lane (two f2 pairs) through `nsub` steps in registers: per step the
// motion of both pairs, then their lifetimes (step_pair_motion / step_pair_life).
// Eq: the quad's expiries as loaded (meaningful only if `due`); E receives the final ones.
template <bool VERLET, bool LIFETIME>
__device__ __forceinline__ void step_quad(const StreamArgs& a, att_ptr att0, size_t att_stride,
                                          uint32_t nsub, uint64_t step0, uint32_t clock0,
                                          uint64_t gid, f4& X, f4& Y, f4& VX, f4& VY, h4 Eq,
                                          bool due, uint16_t nx, h4& E, bool re[4], bool& any) {
  f2 x[2] = {{X[0], X[1]}, {X[2], X[3]}}, y[2] = {{Y[0], Y[1]}, {Y[2], Y[3]}};
  f2 vx[2] = {{VX[0], VX[1]}, {VX[2], VX[3]}}, vy[2] = {{VY[0], VY[1]}, {VY[2], VY[3]}};
  bool r[4] = {false, false, false, false};
  for (uint32_t sub = 0; sub < nsub; ++sub) {
    step_pair_motion<VERLET, 2>(a, att0 + sub * att_stride, x, y, vx, vy);
    if constexpr (LIFETIME) {
      if (sub == 0) {
        // First use of the expiry load, after the motion: the empty asm makes the load an
        // unconditional instruction the compiler keeps in flight until here (a select on
        // `due` at the load would be turned into a branch around it and force the wait
        // before the motion).  Not due: no expiry equals any of the nsub clocks, so nx
        // stands in for the quad's four (and is never written back).
        asm volatile("" : "+v"(Eq));
        E = due ? Eq : h4{nx, nx, nx, nx};
      }
      // The quad's particles that expire in this step, respawned one per pass of a mask loop:
      // the wave runs one Philox pass whenever any of its 256 particles respawns (rarely two),
      // not one per element slot (four inlined copies, each entered by ~19 % of waves at C3).
      // Each particle's respawn is keyed by its own (gid, step), so the order is immaterial.
      const uint16_t ck = (uint16_t)(clock0 + sub);
      uint32_t m = 0;
#pragma unroll
      for (int c = 0; c < 4; ++c) m |= (E[c] == ck ? 1u : 0u) << c;
      while (m) {
        const uint32_t c = __builtin_ctz(m);
        m &= m - 1u;
        float px, py, qx, qy;
        const uint32_t L = respawn(a, step0 + sub, gid + c, px, py, qx, qy);
#pragma unroll
        for (uint32_t cc = 0; cc < 4; ++cc) {
          if (cc == c) {
            x[cc >> 1][cc & 1] = px;
            y[cc >> 1][cc & 1] = py;
            vx[cc >> 1][cc & 1] = qx;
            vy[cc >> 1][cc & 1] = qy;
            E[cc] = (uint16_t)(ck + L);
            r[cc] = true;
          }
        }
        any = true;
      }
    }
  }
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    X[2 * p] = x[p][0];
    X[2 * p + 1] = x[p][1];
    Y[2 * p] = y[p][0];
    Y[2 * p + 1] = y[p][1];
    VX[2 * p] = vx[p][0];
    VX[2 * p + 1] = vx[p][1];
    VY[2 * p] = vy[p][0];
    VY[2 * p + 1] = vy[p][1];
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) re[c] = r[c];
}

// One particle (n % 4 tails) through `nsub` steps: the pair path with element 1 a copy.
template <bool VERLET, bool LIFETIME>
__device__ __forceinline__ bool step_single(const StreamArgs& a, att_ptr att0, size_t att_stride,
                                            uint32_t nsub, uint64_t step0, uint32_t clock0,
                                            uint64_t gid, float& px, float& py, float& qx,
                                            float& qy, uint16_t& pe, bool& any) {
  f2 x[1] = {{px, px}}, y[1] = {{py, py}}, vx[1] = {{qx, qx}}, vy[1] = {{qy, qy}};
  uint16_t e[2] = {pe, pe};
  bool r0 = false;
  for (uint32_t sub = 0; sub < nsub; ++sub) {
    step_pair_motion<VERLET, 1>(a, att0 + sub * att_stride, x, y, vx, vy);
    bool rr[2];
    step_pair_life<LIFETIME>(a, step0 + sub, clock0 + sub, gid, x[0], y[0], vx[0], vy[0], e, rr, true);
    r0 |= rr[0];
    any |= rr[0];
  }
  px = x[0][0];
  py = y[0][0];
  qx = vx[0][0];
  qy = vy[0][0];
  pe = e[0];
  return r0;
}

// Shared body of the one-step and the temporally fused kernels.
template <bool VERLET, bool LIFETIME, bool STATS, int NTM>
__device__ __forceinline__ void stream_body(const StreamArgs& a, att_ptr att0, size_t att_stride,
                                            uint32_t nsub) {
  constexpr bool NTL = (NTM & 1) != 0, NTS = (NTM & 2) != 0;
  const uint64_t nvec = a.n >> 2;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  const uint64_t tid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint64_t step0 = ((uint64_t)a.step_hi << 32) | a.step_lo;
  StatsAcc acc;
  if constexpr (STATS) acc.init();
  // Wave-uniform trip count (kBlock and the stride are multiples of 64): the lanes of a group
  // fold their quads' next expiries across the 16-lane row after the body, so every lane of
  // the wave takes part in the shuffles; lanes past the last quad skip the body.
  for (uint64_t v = tid; (v & ~63ull) < nvec; v += stride) {
    const bool valid = v < nvec;
    const uint64_t i = v << 2;
    uint16_t nx = 0;
    bool due = false;  // one of the group's expiries falls in this launch's steps (row-uniform)
    uint32_t dn = 0x10000u;  // after the body: (u16)(quad's next expiry - end clock) if due
    if (valid) {
      const uint64_t o = tidx(i);  // 4 consecutive particles never straddle a tile
      // [next] is loaded first: the expiries of a due group are then fetched while the state
      // loads are still in flight (loads return in order).  [next] and the expiries are
      // loaded and stored *temporally* whatever NTM says: their lines stay in L2 between the
      // load and the partial (2-B / 8-B) store, which then leaves as a whole dirty line rather
      // than as a partial write at the memory side (nontemporal: 0.4921 -> 0.4872 ms per C3
      // step, same box, tools/ab_stream.py).
      if constexpr (LIFETIME) nx = ldn<false>(a.next + nidx(i));
      f4 X = ld4<NTL>(a.x + o);
      f4 Y = ld4<NTL>(a.y + o);
      f4 VX = ld4<NTL>(a.vx + o);
      f4 VY = ld4<NTL>(a.vy + o);
      h4 E = {0, 0, 0, 0}, Eq = {0, 0, 0, 0};
      if constexpr (LIFETIME) {
        due = (uint16_t)(nx - (uint16_t)a.clock) < nsub;
        // Every lane issues the expiry load; a lane with nothing due reads the first 8 B of
        // the expiry segment instead (one cached line for the whole wave), so no bytes move
        // for it.
        Eq = *reinterpret_cast<const h4*>(a.exp + (due ? eidx(i) : 0));
      }
      bool re[4], any = false;
      step_quad<VERLET, LIFETIME>(a, att0, att_stride, nsub, step0, a.clock, a.id_offset + i, X, Y,
                                  VX, VY, Eq, due, nx, E, re, any);
      if constexpr (STATS) {
#pragma unroll
        for (int c = 0; c < 4; ++c) acc.add(X[c], Y[c], VX[c], VY[c], re[c]);
      }
      st4<NTS>(a.x + o, X);
      st4<NTS>(a.y + o, Y);
      st4<NTS>(a.vx + o, VX);
      st4<NTS>(a.vy + o, VY);
      if constexpr (LIFETIME) {
        if (any) ste4<false>(a.exp + eidx(i), E);  // expiry written only on respawn
        if (due) {
          const uint16_t c1 = (uint16_t)(a.clock + nsub);
          dn = (uint16_t)(quad_next(E[0], E[1], E[2], E[3], c1) - c1);
        }
      }
    }
    if constexpr (LIFETIME) {
      // The group's next expiry: the nearest of its quads' (lanes past the last quad and
      // groups not due hold 0x10000, which never wins in a due group).
      dn = min(dn, (uint32_t)__shfl_xor((int)dn, 1, 16));
      dn = min(dn, (uint32_t)__shfl_xor((int)dn, 2, 16));
      dn = min(dn, (uint32_t)__shfl_xor((int)dn, 4, 16));
      dn = min(dn, (uint32_t)__shfl_xor((int)dn, 8, 16));
      if (due && (threadIdx.x & 15) == 0) {
        const uint16_t n2 = (uint16_t)(a.clock + nsub + dn);
        if (n2 != nx) stn<false>(a.next + nidx(i), n2);
      }
    }
  }
  // n % 4 tail particles, one per lane of the first threads.
  const uint64_t rem = a.n - (nvec << 2);
  if (tid < rem) {
    const uint64_t i = (nvec << 2) + tid;
    const uint64_t o = tidx(i);
    float x = a.x[o], y = a.y[o], vx = a.vx[o], vy = a.vy[o];
    uint16_t e = LIFETIME ? a.exp[eidx(i)] : 0;
    bool any = false;
    const bool re = step_single<VERLET, LIFETIME>(a, att0, att_stride, nsub, step0, a.clock,
                                                  a.id_offset + i, x, y, vx, vy, e, any);
    a.x[o] = x;
    a.y[o] = y;
    a.vx[o] = vx;
    a.vy[o] = vy;
    if constexpr (LIFETIME) {
      if (any) a.exp[eidx(i)] = e;
    }
    if constexpr (STATS) acc.add(x, y, vx, vy, re);
  }
  if constexpr (STATS) block_reduce_stats(acc, a.partials);
}

template <bool VERLET, bool LIFETIME, bool STATS, int NTM>
// Occupancy is capped at 6 waves/SIMD by the launcher's LDS reservation (launch_stream_t), not
// by register limits: 8 waves are slower than 6 on this stream whatever the VGPR count.
__global__ __launch_bounds__(kBlock) void stream_step_kernel(StreamArgs a) {
  stream_body<VERLET, LIFETIME, STATS, NTM>(a, kernarg_f4<StreamArgs>(offsetof(StreamArgs, att)), 0, 1);
}

// Temporal fusion: the same per-particle step applied nsub times in registers, state read
// and written once.  Particles are independent, so this is bitwise equal to
// nsub separate launches; stats (if any) reduce the final substep's state.
template <bool VERLET, bool LIFETIME, bool STATS, int NTM>
__global__ __launch_bounds__(kBlock) void stream_fused_kernel(FusedArgs fa) {
  stream_body<VERLET, LIFETIME, STATS, NTM>(fa.base, kernarg_f4<FusedArgs>(offsetof(FusedArgs, att)),
                                            kMaxAttractors, fa.nsub);
}

// First level of the fixed-order partial reduction: workgroup b folds partials
// [b*chunk, (b+1)*chunk) so the single-workgroup finalize reads at most 256 entries.
__global__ __launch_bounds__(kBlock) void stats_fold_kernel(const StatsPartial* partials,
                                                            uint32_t count, uint32_t chunk,
                                                            StatsPartial* out) {
  StatsAcc acc;
  acc.init();
  const uint32_t lo = blockIdx.x * chunk;
  const uint32_t hi = min(count, lo + chunk);
  for (uint32_t i = lo + threadIdx.x; i < hi; i += kBlock) {
    const StatsPartial p = partials[i];
    acc.x0 = fminf(acc.x0, p.bbox[0]);
    acc.x1 = fmaxf(acc.x1, p.bbox[1]);
    acc.y0 = fminf(acc.y0, p.bbox[2]);
    acc.y1 = fmaxf(acc.y1, p.bbox[3]);
    acc.ke += p.ke;
    acc.count += p.count;
    acc.respawned += p.respawned;
  }
  block_reduce_stats(acc, out);
}

__global__ __launch_bounds__(kBlock) void stats_finalize_kernel(const StatsPartial* partials,
                                                                uint32_t count, StatsResult* out,
                                                                StatsGlobal* global,
                                                                unsigned long long step) {
  StatsAcc acc;
  acc.init();
  for (uint32_t i = threadIdx.x; i < count; i += kBlock) {
    const StatsPartial p = partials[i];
    acc.x0 = fminf(acc.x0, p.bbox[0]);
    acc.x1 = fmaxf(acc.x1, p.bbox[1]);
    acc.y0 = fminf(acc.y0, p.bbox[2]);
    acc.y1 = fmaxf(acc.y1, p.bbox[3]);
    acc.ke += p.ke;
    acc.count += p.count;
    acc.respawned += p.respawned;
  }
  __shared__ StatsPartial res[1];
  block_reduce_stats(acc, res - blockIdx.x);  // writes res[0]
  __syncthreads();
  if (threadIdx.x == 0) {
    StatsResult r;
    for (int k = 0; k < 4; ++k) r.bbox[k] = res[0].bbox[k];
    r.ke = res[0].ke;
    r.count = res[0].count;
    r.respawned = res[0].respawned;
    r.step = step;
    *out = r;
    if (global) {
      StatsGlobal g;
      g.neg_min_max[0] = -r.bbox[0];
      g.neg_min_max[1] = r.bbox[1];
      g.neg_min_max[2] = -r.bbox[2];
      g.neg_min_max[3] = r.bbox[3];
      g.sums[0] = r.ke;
      g.sums[1] = (double)r.count;
      g.sums[2] = (double)r.respawned;
      *global = g;
    }
  }
}

// ---------------------------------------------------------------------------------------
// AoS <-> SoA (the 32-B Particle of src/particle.rs:20-25)
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void aos_to_soa_kernel(const rps_particle* aos, Fields f,
                                                            Layout L, uint64_t offset, uint64_t n) {
  const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j >= n) return;
  const f4 pv = *reinterpret_cast<const f4*>(&aos[j].position[0]);
  const uint64_t o = lidx(L, offset + j);
  f.x[o] = pv[0];
  f.y[o] = pv[1];
  f.vx[o] = pv[2];
  f.vy[o] = pv[3];
}

__global__ __launch_bounds__(kBlock) void soa_to_aos_kernel(Fields f, Layout L, uint64_t offset,
                                                            rps_particle* aos, uint64_t n,
                                                            float max_energy, int spawn_colour) {
  const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j >= n) return;
  const uint64_t o = lidx(L, offset + j);
  const float qx = f.vx[o], qy = f.vy[o];
  *reinterpret_cast<f4*>(&aos[j].position[0]) = f4{f.x[o], f.y[o], qx, qy};
  const f4 c = spawn_colour ? f4{1.0f, 1.0f, 1.0f, 1.0f} : set_color(qx, qy, max_energy);
  *reinterpret_cast<f4*>(&aos[j].color[0]) = c;
}

// rps_set_config's upload: the 144-B config travels in this launch's kernarg segment and one
// wave copies it to the device config, one dword per lane (ordered on the context stream
// like any kernel; no staging buffer, no copy-engine handoff).
struct ConfigStoreArgs {
  rps_config cfg;
  rps_config* dst;
};
__global__ __launch_bounds__(64) void config_store_kernel(ConfigStoreArgs a) {
  typedef __attribute__((address_space(4))) const uint32_t* kword;
  const uint32_t i = threadIdx.x;
  if (i < sizeof(rps_config) / 4u) {
    const kword src = (kword)((__attribute__((address_space(4))) const char*)__builtin_amdgcn_kernarg_segment_ptr() +
                              offsetof(ConfigStoreArgs, cfg));
    reinterpret_cast<uint32_t*>(a.dst)[i] = src[i];
  }
}

// One field <-> a dense float range (checkpoint / SoA transfers through the layout).
__global__ __launch_bounds__(kBlock) void field_gather_kernel(const float* field, Layout L,
                                                              uint64_t offset, float* out,
                                                              uint64_t n) {
  const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j < n) out[j] = field[lidx(L, offset + j)];
}

__global__ __launch_bounds__(kBlock) void field_scatter_kernel(float* field, Layout L,
                                                               uint64_t offset, const float* in,
                                                               uint64_t n) {
  const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j < n) field[lidx(L, offset + j)] = in[j];
}

// Lifetime field views.  Before the step with lifetime clock c, a particle
// with expiry e has (u16)(e - c) + 1 steps left.  mode 0: life in seconds = steps * dt;
// mode 1: the raw u16 expiry (debug); mode 2: steps left as an exact f32 integer.  Writing
// (life_scatter): mode 0 takes seconds, e = c + life_steps(L) - 1; mode 2 takes steps,
// e = c + clamp(ceil(v), 1, 65535) - 1.
__global__ __launch_bounds__(kBlock) void life_gather_kernel(const uint16_t* exp, Layout L,
                                                             uint64_t offset, float* out, uint64_t n,
                                                             uint32_t clock, float dt, int mode) {
  const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j >= n) return;
  const uint16_t e = exp[lidx(L, offset + j)];
  const float left = (float)((uint32_t)(uint16_t)(e - (uint16_t)clock) + 1u);
  if (mode == 1)
    reinterpret_cast<uint16_t*>(out)[j] = e;
  else
    out[j] = mode == 2 ? left : left * dt;
}

__global__ __launch_bounds__(kBlock) void life_scatter_kernel(uint16_t* exp, Layout L,
                                                              uint64_t offset, const float* in,
                                                              uint64_t n, uint32_t clock, float dt,
                                                              int mode) {
  const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j >= n) return;
  const uint32_t steps = mode == 2 ? life_steps(in[j], 1.0f) : life_steps(in[j], dt);
  exp[lidx(L, offset + j)] = (uint16_t)(clock + steps - 1u);
}

// [next] of groups [g0, g1) from the expiries of their full quads (quad index < nquads) at
// lifetime clock `clock` (after any write of expiries outside the stream kernel: initial
// scatter, lifetime uploads).
__global__ __launch_bounds__(kBlock) void next_rebuild_kernel(const uint16_t* exp, uint16_t* next,
                                                              uint64_t g0, uint64_t g1,
                                                              uint64_t nquads, uint32_t clock) {
  const uint64_t g = g0 + (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (g >= g1) return;
  const uint16_t c = (uint16_t)clock;
  const uint64_t q0 = g << (kGroupLog - 2);
  const uint64_t q1 = min(q0 + (kGroup >> 2), nquads);
  uint16_t best = 0;
  for (uint64_t q = q0; q < q1; ++q) {
    const h4 E = *reinterpret_cast<const h4*>(exp + eidx(q << 2));
    const uint16_t e = quad_next(E[0], E[1], E[2], E[3], c);
    if (q == q0 || (uint16_t)(e - c) < (uint16_t)(best - c)) best = e;
  }
  next[nidx(g << kGroupLog)] = best;
}

// ---------------------------------------------------------------------------------------
// Initial scatter (seeded restatement of src/main.rs:182-216)
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void init_scatter_kernel(InitArgs a) {
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < a.n;
       i += (uint64_t)gridDim.x * kBlock) {
  const uint64_t g = a.id_offset + i;
  const uint64_t o = lidx(a.layout, i);
  const float t = (float)g / a.global_count_f;
  a.f.x[o] = a.x_min + t * (a.x_max - a.x_min);
  uint32_t w[4];
  philox4x32_10((uint32_t)g, (uint32_t)(g >> 32), 0xFFFFFFFFu, 0xFFFFFFFFu, a.key0, a.key1, w);
  const float u1 = (float)((w[0] >> 8) + 1u) * (1.0f / 16777216.0f);
  float c, s;
  sincos_turns(u01(w[1]), c, s);
  const float z = sqrtf(-2.0f * log_unit(u1)) * c;
  const float y_center = (a.y_min + a.y_max) / 2.0f;
  const float y_sd = (a.y_max - a.y_min) * 0.125f;
  float yy = y_center + z * y_sd;
  yy = yy < a.y_min ? a.y_min : yy;
  yy = yy > a.y_max ? a.y_max : yy;
  a.f.y[o] = yy;
  a.f.vx[o] = 0.0f;
  a.f.vy[o] = 0.0f;
  if (a.f.exp)
    a.f.exp[lidx(a.exp_layout, i)] =
        (uint16_t)(a.clock + life_steps(a.life_min + u01(w[2]) * a.life_range, a.dt) - 1u);
  }
}

// ---------------------------------------------------------------------------------------
// SPH: the reference's five passes
// ---------------------------------------------------------------------------------------

// sort_particles, compute_shader.wgsl:470-505: pass (group_width gw, flip = step_index == 0)
// pairs left = h + 2gw*(i/gw), h = i % gw, with right = left + (flip ? 2gw-1-2h : gw) and
// swaps the (key, index) entries when key(left) > key(right).
// Several consecutive passes of one stage in registers.  Passes t..t+K-1 of a stage have
// strides G, G/2, ..., g = G / 2^(K-1) (stride = group_width).  For a residue r < g the
// 2^K entries r + j*g (j < 2^K) of a 2G block are closed under the non-flip passes (stride
// g*2^m pairs j with j + 2^m), and with a flip first pass (pairs h <-> 2G-1-h) the class r
// together with its mirror class g-1-r (2^(K+1) entries, r < g/2) is closed as well.  One
// thread loads its group, applies the K passes in network order (flip first, then
// descending strides) with the reference's compare-swap, and stores it back: the same
// network, the same comparisons, so the same result as K pass-per-dispatch launches.
// `mem` is the lookup (global passes) or the workgroup's LDS tile (local passes).
template <int K, bool FLIP, class T>
__device__ __forceinline__ void sort_group(T mem, uint32_t base, uint32_t r, uint32_t g) {
  constexpr int M = 1 << K;            // entries per residue class
  constexpr int E = FLIP ? 2 * M : M;  // entries per group
  uint2 v[E];
#pragma unroll
  for (int j = 0; j < M; ++j) v[j] = mem[base + r + j * g];
  if constexpr (FLIP) {
#pragma unroll
    for (int j = 0; j < M; ++j) v[M + j] = mem[base + (g - 1u - r) + j * g];
    // flip pass: position r + j*g pairs with 2G-1-(r + j*g) = (g-1-r) + (M-1-j)*g.
#pragma unroll
    for (int j = 0; j < M / 2; ++j) {
      uint2& lo = v[j];  // position < G: the left entry
      uint2& hi = v[M + (M - 1 - j)];
      if (lo.x > hi.x) { const uint2 tmp = lo; lo = hi; hi = tmp; }
      uint2& lo2 = v[M + j];  // mirror class, position (g-1-r) + j*g < G
      uint2& hi2 = v[M - 1 - j];
      if (lo2.x > hi2.x) { const uint2 tmp = lo2; lo2 = hi2; hi2 = tmp; }
    }
  }
  // Non-flip passes, strides g*2^m for m = (FLIP ? K-2 : K-1) down to 0, in each class.
#pragma unroll
  for (int m = (FLIP ? K - 2 : K - 1); m >= 0; --m) {
#pragma unroll
    for (int c = 0; c < E / M; ++c) {
#pragma unroll
      for (int j = 0; j < M; ++j) {
        if (j & (1 << m)) continue;
        uint2& a = v[c * M + j];
        uint2& b = v[c * M + j + (1 << m)];
        if (a.x > b.x) { const uint2 tmp = a; a = b; b = tmp; }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < M; ++j) mem[base + r + j * g] = v[j];
  if constexpr (FLIP) {
#pragma unroll
    for (int j = 0; j < M; ++j) mem[base + (g - 1u - r) + j * g] = v[M + j];
  }
}

// Groups of a (K, flip) chunk in an array of `len` entries, group q -> (base, residue).
// len, G and g are powers of two (a flip chunk has g >= 2), so the split is shifts and masks
// rather than a runtime u32 division per group.
__device__ __forceinline__ uint32_t sort_groups(uint32_t len, uint32_t G, uint32_t g, bool flip) {
  return (len >> (__builtin_ctz(G) + 1)) << (__builtin_ctz(g) - (flip ? 1 : 0));
}
__device__ __forceinline__ void sort_group_at(uint32_t q, uint32_t G, uint32_t g, bool flip,
                                              uint32_t& base, uint32_t& r) {
  const uint32_t lp = __builtin_ctz(g) - (flip ? 1u : 0u);  // log2(groups per 2G block)
  base = (q >> lp) << (__builtin_ctz(G) + 1);
  r = q & ((1u << lp) - 1u);
}

// K global passes of one stage, one group per thread.
template <int K, bool FLIP>
__global__ __launch_bounds__(kBlock) void sph_sort_fused_kernel(uint2* __restrict__ lookup,
                                                                uint32_t p, uint32_t G) {
  const uint32_t g = G >> (K - 1);
  const uint32_t q = blockIdx.x * kBlock + threadIdx.x;
  if (q >= sort_groups(p, G, g, FLIP)) return;
  uint32_t base, r;
  sort_group_at(q, G, g, FLIP, base, r);
  sort_group<K, FLIP>(lookup, base, r, g);
}

constexpr uint32_t kSortTile = 8192;      // entries per workgroup tile (64 KiB of LDS)
constexpr uint32_t kSortLd = 8;           // 16-B tile loads a lane keeps in flight at once
constexpr uint32_t kSortLdBin = 4;        // the same in the bin launch (positions + pad entries)

// LDS view of a sort tile with one pad entry per 32 (256 B, one pass over the 64 banks):
// the small-stride passes have lanes 16-32 B apart, which without padding land on 8 of the
// 32 bank pairs (8-way conflicts); padded they spread over all 32.
struct PaddedTile {
  uint2* p;
  __device__ __forceinline__ uint2& operator[](uint32_t i) const { return p[i + (i >> 5)]; }
};

// bin_particles_in_grid (wgsl:455-468) folded into the first sort launch: entries [0, n)
// get (key, i) from the current positions and offsets[i] <- 0xFFFFFFFF; entries [n, P) keep
// what the previous frame's sort left there (the reference never rewrites them).
struct SortBin {
  const rps_config* cfg;
  const f4* st;  // packed {x, y, vx, vy} per particle
  uint32_t* offsets;
  uint32_t n;
  const uint2* prebuilt;  // bin entries the previous frame's sim wrote (nullptr: from positions)
  bool reset_pre;         // prebuilt entries in particle order (no layout): still reset offsets
};

__device__ __forceinline__ f2 bin_pos(const SortBin& b, uint32_t i) {
  return reinterpret_cast<const f2*>(b.st)[2u * i];
}
__device__ __forceinline__ void bin_reset(const SortBin& b, uint32_t i) {
  b.offsets[i] = 0xFFFFFFFFu;
}
__device__ __forceinline__ uint2 bin_key(const SortBin& b, f2 pos, uint32_t i) {
  bin_reset(b, i);
  if (b.prebuilt) return b.prebuilt[i];  // slot-resident state: (key, slot), keyed by the sim
  const float r = b.cfg->smoothing_radius;
  const int32_t cx = f32_to_i32((pos[0] + b.cfg->screen_bounds[1]) / r);
  const int32_t cy = f32_to_i32((pos[1] + b.cfg->screen_bounds[3]) / r);
  return make_uint2(cell_key(cx, cy, b.cfg->particle_count), i);
}
__device__ __forceinline__ uint2 bin_entry(const SortBin& b, uint32_t i) {
  return bin_key(b, bin_pos(b, i), i);
}

// One register chunk of the passes of `stage` starting at `step` (sort_group: up to KMAX
// passes, flip first: up to KMAX-1) over the `len` entries at `off` of the tile, groups dealt
// to work-items w0, w0 + wn, ...  Returns the number of passes covered.
template <int KMAX>
__device__ __forceinline__ uint32_t sort_chunk(const PaddedTile& s, uint32_t off, uint32_t len,
                                               uint32_t stage, uint32_t step, uint32_t w0,
                                               uint32_t wn, uint32_t cap = 32u) {
  const uint32_t G = 1u << (stage - step);
  const uint32_t left = min(stage - step + 1u, cap);  // passes left in this stage (capped)
  // A flip pass with G = 1 pairs (2i, 2i+1) exactly like a non-flip one.
  const bool flip = step == 0u && G > 1u;
  const uint32_t kf = KMAX > 1 ? (uint32_t)KMAX - 1u : 1u;  // flip chunks: 2^(K+1) entries
  const uint32_t K = flip ? ((G >= (2u << (kf - 1u)) && kf <= left) ? kf : 1u)
                          : (left < (uint32_t)KMAX ? left : (uint32_t)KMAX);
  const uint32_t g = G >> (K - 1u);
  const uint32_t groups = sort_groups(len, G, g, flip);
  for (uint32_t q = w0; q < groups; q += wn) {
    uint32_t b, r;
    sort_group_at(q, G, g, flip, b, r);
    if (flip) {
      if (KMAX >= 4 && K == 3u) sort_group<3, true>(s, off + b, r, g);
      else if (KMAX >= 3 && K == 2u) sort_group<2, true>(s, off + b, r, g);
      else sort_group<1, true>(s, off + b, r, g);
    } else {
      if (KMAX >= 4 && K == 4u) sort_group<4, false>(s, off + b, r, g);
      else if (KMAX >= 3 && K == 3u) sort_group<3, false>(s, off + b, r, g);
      else if (KMAX >= 2 && K == 2u) sort_group<2, false>(s, off + b, r, g);
      else sort_group<1, false>(s, off + b, r, g);
    }
  }
  return K;
}

// A wave's LDS writes visible to its own later LDS reads (any lane): LDS serves one wave's
// instructions in order; the wait and the wavefront fences keep the compiler from moving
// LDS accesses across the point.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Every remaining pass of stages [stage_lo, stage_hi] whose group_width fits one tile:
// a pass with 2*gw <= tile only pairs entries inside aligned blocks of 2*gw, so a tile of
// the array can run it on its own.  Passes go in register chunks (sort_group) of up to KMAX
// (flip first: up to KMAX-1).  Passes whose span 2*gw exceeds a wave's share of the tile
// (64 lanes x one group each) run across the workgroup with a barrier per chunk; the rest
// -- every pass of the early stages and the tail of each later stage -- run inside each
// wave's own span with only wave-level ordering.  Same network, same compare order per pair
// -> identical result to the reference's pass-per-dispatch schedule.
template <bool BIN, int KMAX, uint32_t CAP = kSortTile>
__global__ __launch_bounds__(1024) void sph_sort_local_kernel(
    uint2* __restrict__ lookup, uint32_t tile, uint32_t stage_lo, uint32_t stage_hi,
    uint32_t first_step, SortBin bin, uint32_t vec) {
  __shared__ uint2 lds[CAP + CAP / 32];
  const PaddedTile s{lds};
  const uint32_t base0 = blockIdx.x * tile;
  if (!BIN && vec) {
    // Two entries per lane in 16-B loads, all of a lane's loads issued before its first LDS
    // write: a loop of load -> wait -> write paid one memory round trip per iteration.
    // kSortLd loads per lane cover every (tile, threads) pair launch_sort_local uses
    // (tile <= 16 x threads); the loop after it never runs for those.
    uint4 v[kSortLd];
#pragma unroll
    for (uint32_t k = 0; k < kSortLd; ++k) {
      const uint32_t q = 2u * threadIdx.x + k * 2u * blockDim.x;
      if (q < tile) v[k] = *reinterpret_cast<const uint4*>(lookup + base0 + q);
    }
#pragma unroll
    for (uint32_t k = 0; k < kSortLd; ++k) {
      const uint32_t q = 2u * threadIdx.x + k * 2u * blockDim.x;
      if (q < tile) {
        s[q] = make_uint2(v[k].x, v[k].y);
        s[q + 1u] = make_uint2(v[k].z, v[k].w);
      }
    }
    for (uint32_t q = 2u * threadIdx.x + kSortLd * 2u * blockDim.x; q < tile; q += 2u * blockDim.x) {
      const uint4 w = *reinterpret_cast<const uint4*>(lookup + base0 + q);
      s[q] = make_uint2(w.x, w.y);
      s[q + 1u] = make_uint2(w.z, w.w);
    }
  } else if (vec) {  // the bin launch: every position (or pad entry) load first, then the keys
    // (kSortLdBin, not kSortLd: 8 would take the launch to 93 VGPRs, one 1024-thread block per CU)
    f2 pa[kSortLdBin], pc[kSortLdBin];
    uint4 lk[kSortLdBin];
#pragma unroll
    for (uint32_t k = 0; k < kSortLdBin; ++k) {
      const uint32_t q = 2u * threadIdx.x + k * 2u * blockDim.x;
      const uint32_t gq = base0 + q;
      if (q < tile) {
        if (gq < bin.n) {
          pa[k] = bin_pos(bin, gq);
          if (gq + 1u < bin.n) pc[k] = bin_pos(bin, gq + 1u);
          else lk[k] = *reinterpret_cast<const uint4*>(lookup + gq);
        } else {
          lk[k] = *reinterpret_cast<const uint4*>(lookup + gq);
        }
      }
    }
#pragma unroll
    for (uint32_t k = 0; k < kSortLdBin; ++k) {
      const uint32_t q = 2u * threadIdx.x + k * 2u * blockDim.x;
      const uint32_t gq = base0 + q;
      if (q < tile) {
        uint2 a, c;
        if (gq < bin.n) {
          a = bin_key(bin, pa[k], gq);
          c = gq + 1u < bin.n ? bin_key(bin, pc[k], gq + 1u) : make_uint2(lk[k].z, lk[k].w);
        } else {
          a = make_uint2(lk[k].x, lk[k].y);
          c = make_uint2(lk[k].z, lk[k].w);
        }
        s[q] = a;
        s[q + 1u] = c;
      }
    }
    for (uint32_t q = 2u * threadIdx.x + kSortLdBin * 2u * blockDim.x; q < tile; q += 2u * blockDim.x) {
      const uint32_t gq = base0 + q;
      uint2 a, c;
      if (BIN && gq < bin.n) {
        a = bin_entry(bin, gq);
        c = gq + 1u < bin.n ? bin_entry(bin, gq + 1u) : lookup[gq + 1u];
      } else {
        const uint4 v = *reinterpret_cast<const uint4*>(lookup + gq);
        a = make_uint2(v.x, v.y);
        c = make_uint2(v.z, v.w);
      }
      s[q] = a;
      s[q + 1u] = c;
    }
  } else {
    for (uint32_t q = threadIdx.x; q < tile; q += blockDim.x) {
      const uint32_t gq = base0 + q;
      s[q] = (BIN && gq < bin.n) ? bin_entry(bin, gq) : lookup[gq];
    }
  }
  __syncthreads();
  const uint32_t ws = min(tile, 64u << KMAX);  // one wave's span (blockDim is a multiple of 64)
  const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  uint32_t stage = stage_lo, step = first_step;
  while (stage <= stage_hi) {
    while (step <= stage && (2u << (stage - step)) > ws) {  // cross-wave passes
      step += sort_chunk<KMAX>(s, 0u, tile, stage, step, threadIdx.x, blockDim.x);
      __syncthreads();
    }
    uint32_t last = stage;  // later stages whose whole network is wave-local join in
    while (last < stage_hi && (2u << (last + 1u)) <= ws) ++last;
    for (uint32_t reg = wid; reg < tile / ws; reg += nw) {
      for (uint32_t st = stage, sp = step; st <= last; ++st, sp = 0u) {
        while (sp <= st) {
          sp += sort_chunk<KMAX>(s, reg * ws, ws, st, sp, lane, 64u);
          wave_lds_sync();
        }
      }
    }
    __syncthreads();
    stage = last + 1u;
    step = 0u;
  }
  if (vec) {
    for (uint32_t q = 2u * threadIdx.x; q < tile; q += 2u * blockDim.x) {
      const uint2 a = s[q], c = s[q + 1u];
      *reinterpret_cast<uint4*>(lookup + base0 + q) = make_uint4(a.x, a.y, c.x, c.y);
    }
  } else {
    for (uint32_t q = threadIdx.x; q < tile; q += blockDim.x) lookup[base0 + q] = s[q];
  }
}

// ---------------------------------------------------------------------------------------
// Static-network tail launch.  After a later stage's global passes (strides >= the tile), what
// is left of the stage inside each tile is always the same network: the TLOG non-flip passes
// of strides 2^(TLOG-1), ..., 2, 1.  With the strides known at compile time every LDS address
// is one per-thread base plus an immediate offset (PaddedTile's pad folds into it: padded(e0 +
// j*g) = padded(e0) + j*g + (j*g >> 5) for a group's base aligned to 2G and residue r < g), and
// the first and last register chunks talk to memory directly: the first loads its eight
// entries (strides 2^(TLOG-1..TLOG-3), group r = thread) from the lookup, the last (strides 8,
// 4, 2, 1) is a 16-entry group held by a lane pair, eight consecutive entries per lane, whose
// stride-8 pass exchanges entries across the pair with a DPP move, and stores them.  Two LDS
// sweeps fewer than staging the tile (round 2: load sweep, five chunk sweeps, store sweep).
// Same compare-swaps in the same pass order as the reference's dispatch sequence.
// ---------------------------------------------------------------------------------------
// Compare-swap (lower position first): swap when lo.x > hi.x, equal keys stay.  Independent
// pairs go in batches: every compare first (one mask per pair), then each pair's two
// v_swap_b32 with its mask as EXEC, EXEC restored at the end -- three VALU ops per pair instead
// of a compare and four selects, and no branches (2^22 tail 15.9 -> 13.5 us: the in-tile passes
// are VALU-bound).
__device__ __forceinline__ void cas(uint2& a, uint2& b) {
  uint64_t m, sv;
  asm("v_cmp_gt_u32_e64 %[m], %[ax], %[bx]\n\t"
      "s_mov_b64 %[sv], exec\n\t"
      "s_mov_b64 exec, %[m]\n\t"
      "v_swap_b32 %[ax], %[bx]\n\t"
      "v_swap_b32 %[ay], %[by]\n\t"
      "s_mov_b64 exec, %[sv]"
      : [ax] "+v"(a.x), [bx] "+v"(b.x), [ay] "+v"(a.y), [by] "+v"(b.y), [m] "=&s"(m), [sv] "=&s"(sv));
}
__device__ __forceinline__ void cas2(uint2& a0, uint2& b0, uint2& a1, uint2& b1) {
  uint64_t m0, m1, sv;
  asm("v_cmp_gt_u32_e64 %[m0], %[a0x], %[b0x]\n\t"
      "v_cmp_gt_u32_e64 %[m1], %[a1x], %[b1x]\n\t"
      "s_mov_b64 %[sv], exec\n\t"
      "s_mov_b64 exec, %[m0]\n\t"
      "v_swap_b32 %[a0x], %[b0x]\n\t"
      "v_swap_b32 %[a0y], %[b0y]\n\t"
      "s_mov_b64 exec, %[m1]\n\t"
      "v_swap_b32 %[a1x], %[b1x]\n\t"
      "v_swap_b32 %[a1y], %[b1y]\n\t"
      "s_mov_b64 exec, %[sv]"
      : [a0x] "+v"(a0.x), [b0x] "+v"(b0.x), [a0y] "+v"(a0.y), [b0y] "+v"(b0.y),
        [a1x] "+v"(a1.x), [b1x] "+v"(b1.x), [a1y] "+v"(a1.y), [b1y] "+v"(b1.y),
        [m0] "=&s"(m0), [m1] "=&s"(m1), [sv] "=&s"(sv));
}
__device__ __forceinline__ void cas4(uint2& a0, uint2& b0, uint2& a1, uint2& b1, uint2& a2, uint2& b2,
                                     uint2& a3, uint2& b3) {
  uint64_t m0, m1, m2, m3, sv;
  asm("v_cmp_gt_u32_e64 %[m0], %[a0x], %[b0x]\n\t"
      "v_cmp_gt_u32_e64 %[m1], %[a1x], %[b1x]\n\t"
      "v_cmp_gt_u32_e64 %[m2], %[a2x], %[b2x]\n\t"
      "v_cmp_gt_u32_e64 %[m3], %[a3x], %[b3x]\n\t"
      "s_mov_b64 %[sv], exec\n\t"
      "s_mov_b64 exec, %[m0]\n\t"
      "v_swap_b32 %[a0x], %[b0x]\n\t"
      "v_swap_b32 %[a0y], %[b0y]\n\t"
      "s_mov_b64 exec, %[m1]\n\t"
      "v_swap_b32 %[a1x], %[b1x]\n\t"
      "v_swap_b32 %[a1y], %[b1y]\n\t"
      "s_mov_b64 exec, %[m2]\n\t"
      "v_swap_b32 %[a2x], %[b2x]\n\t"
      "v_swap_b32 %[a2y], %[b2y]\n\t"
      "s_mov_b64 exec, %[m3]\n\t"
      "v_swap_b32 %[a3x], %[b3x]\n\t"
      "v_swap_b32 %[a3y], %[b3y]\n\t"
      "s_mov_b64 exec, %[sv]"
      : [a0x] "+v"(a0.x), [b0x] "+v"(b0.x), [a0y] "+v"(a0.y), [b0y] "+v"(b0.y),
        [a1x] "+v"(a1.x), [b1x] "+v"(b1.x), [a1y] "+v"(a1.y), [b1y] "+v"(b1.y),
        [a2x] "+v"(a2.x), [b2x] "+v"(b2.x), [a2y] "+v"(a2.y), [b2y] "+v"(b2.y),
        [a3x] "+v"(a3.x), [b3x] "+v"(b3.x), [a3y] "+v"(a3.y), [b3y] "+v"(b3.y),
        [m0] "=&s"(m0), [m1] "=&s"(m1), [m2] "=&s"(m2), [m3] "=&s"(m3), [sv] "=&s"(sv));
}

// Entry index of the p-th pair's lower entry in a pass of stride 2^m (bit m cleared).
__device__ __forceinline__ constexpr int pair_lo(int p, int m) {
  return ((p >> m) << (m + 1)) | (p & ((1 << m) - 1));
}

// The non-flip passes of strides g*2^(K-1), ..., g over the 2^K entries v[j] = position
// r + j*g of one group (sort_group's inner loop with M = 2^K).
template <int K>
__device__ __forceinline__ void group_passes(uint2 (&v)[1 << K]) {
#pragma unroll
  for (int m = K - 1; m >= 0; --m) {
    if constexpr (K == 1) {
      cas(v[0], v[1]);
    } else if constexpr (K == 2) {
      const int d = 1 << m, j0 = pair_lo(0, m), j1 = pair_lo(1, m);
      cas2(v[j0], v[j0 + d], v[j1], v[j1 + d]);
    } else {
#pragma unroll
      for (int p = 0; p < (1 << (K - 1)); p += 4) {
        const int d = 1 << m;
        const int j0 = pair_lo(p, m), j1 = pair_lo(p + 1, m), j2 = pair_lo(p + 2, m), j3 = pair_lo(p + 3, m);
        cas4(v[j0], v[j0 + d], v[j1], v[j1 + d], v[j2], v[j2 + d], v[j3], v[j3 + d]);
      }
    }
  }
}

// Padded LDS index offset of the group's entry j (see above).
template <uint32_t G>
__device__ __forceinline__ constexpr uint32_t pad_off(uint32_t j) {
  return j * G + ((j * G) >> 5);
}
__device__ __forceinline__ uint32_t padded(uint32_t e) { return e + (e >> 5); }

// Group i of a thread's 2^LNG in a register chunk: a wave owns the same block of 64 * 2^LNG
// groups as with q = t * 2^LNG + i (so a chunk inside the wave's entries stays wave-local), but
// consecutive lanes take consecutive groups: consecutive LDS entries, no bank conflicts.
template <int LNG>
__device__ __forceinline__ uint32_t chunk_group(uint32_t t, int i) {
  return ((t >> 6) << (6 + LNG)) + ((uint32_t)i << 6) + (t & 63u);
}

// One LDS chunk: passes of strides 2^LG down to 2^(LG-K+1), non-flip, 2^(LE-K) groups per thread
// (2^LE entries, eight by default).
template <int LG, int K, int LE = 3>
__device__ __forceinline__ void lds_chunk(uint2* lds, uint32_t t) {
  constexpr int LGG = LG - K + 1;
  constexpr uint32_t g = 1u << LGG;
  constexpr int NG = 1 << (LE - K);
#pragma unroll
  for (int i = 0; i < NG; ++i) {
    const uint32_t q = chunk_group<LE - K>(t, i);
    const uint32_t e0 = ((q >> LGG) << (LG + 1)) + (q & (g - 1u));
    const uint32_t a = padded(e0);
    uint2 v[1 << K];
#pragma unroll
    for (int j = 0; j < (1 << K); ++j) v[j] = lds[a + pad_off<g>(j)];
    group_passes<K>(v);
#pragma unroll
    for (int j = 0; j < (1 << K); ++j) lds[a + pad_off<g>(j)] = v[j];
  }
}

// The middle chunks: strides 2^LG down to 2^LO, three passes per chunk (the last one fewer);
// a chunk whose span 2G exceeds one wave's 512 entries ends with a workgroup barrier.
template <int LG, int LO>
__device__ __forceinline__ void lds_chunks(uint2* lds, uint32_t t) {
  if constexpr (LG >= LO) {
    constexpr int K = LG - LO + 1 >= 3 ? 3 : LG - LO + 1;
    lds_chunk<LG, K>(lds, t);
    if constexpr ((2 << LG) > 512) __syncthreads();
    else wave_lds_sync();
    lds_chunks<LG - K, LO>(lds, t);
  }
}

// Where the LDS chunks of a tile's in-tile passes stop (log2 of the last LDS stride); the passes
// below run in registers.  Tiles of 8192 entries (16 waves): stride 8 as a DPP exchange across a
// lane pair (tails) and strides 16, 8 across a lane quad (head), measured faster there; smaller
// tiles: every stride down to 8 in LDS, so the lane keeps only 4, 2, 1 (2^20 head 20.0 -> 18.9 us,
// 2^19 13.2 -> 12.6, profiles/r06_sort_stride8_ab.txt; at 2^22 the head went 55.9 -> 56.9).
template <int TLOG>
constexpr int kTailLdsLo = TLOG >= 13 ? 4 : 3;
template <int TLOG>
constexpr int kHeadLdsLo = TLOG >= 13 ? 5 : 3;

// A pass across lanes: entry j of this lane against entry j (REV: 7 - j) of the DPP partner
// (quad_perm CTRL); `left` = this lane holds the lower position of each pair.
template <int CTRL, bool REV>
__device__ __forceinline__ void xlane_pass(uint2 (&v)[8], bool left) {
  uint2 p[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    p[j].x = (uint32_t)__builtin_amdgcn_mov_dpp((int)v[REV ? 7 - j : j].x, CTRL, 0xF, 0xF, false);
    p[j].y = (uint32_t)__builtin_amdgcn_mov_dpp((int)v[REV ? 7 - j : j].y, CTRL, 0xF, 0xF, false);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const bool swap = left ? (v[j].x > p[j].x) : (p[j].x > v[j].x);
    v[j] = swap ? p[j] : v[j];
  }
}
constexpr int kDppXor1 = 0xB1;  // quad_perm [1, 0, 3, 2]
constexpr int kDppXor2 = 0x4E;  // quad_perm [2, 3, 0, 1]
constexpr int kDppRev4 = 0x1B;  // quad_perm [3, 2, 1, 0]

// Quad transpose on pair-index bit B: pair j = (v[2j], v[2j+1]); the pairs whose bit B differs
// from the lane's bit B trade places with the DPP partner's (lane ^ 2^B) pair j ^ 2^B.
template <int B, int CTRL>
__device__ __forceinline__ void quad_swap_bit(uint2 (&v)[8], uint32_t t) {
  const bool hi = (t >> B) & 1u;
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    constexpr int sh = B == 1 ? 0 : 1;  // position of the pair-index bit that is not B
    const int j0 = m << sh, j1 = j0 | (1 << B);  // pairs with bit B = 0 / 1
#pragma unroll
    for (int h = 0; h < 2; ++h) {  // value selects only: a select of array elements spills v
      const uint2 x0 = v[2 * j0 + h], x1 = v[2 * j1 + h];
      const uint32_t ex = hi ? x0.x : x1.x, ey = hi ? x0.y : x1.y;
      const uint32_t rx = (uint32_t)__builtin_amdgcn_mov_dpp((int)ex, CTRL, 0xF, 0xF, false);
      const uint32_t ry = (uint32_t)__builtin_amdgcn_mov_dpp((int)ey, CTRL, 0xF, 0xF, false);
      v[2 * j0 + h] = make_uint2(hi ? rx : x0.x, hi ? ry : x0.y);
      v[2 * j1 + h] = make_uint2(hi ? x1.x : rx, hi ? x1.y : ry);
    }
  }
}

// Store a lane's eight consecutive entries [8t, 8t + 8) of `tile` in whole 64-B segments: the
// lane quad transposes its 16-B pairs, so store i of lane l writes pair l of lane i's eight and
// each store instruction fills one 64-B segment per quad (lane-strided 16-B stores would send
// four partial write requests per segment).  NT: nontemporal stores, for the 8192-entry tiles
// (P >= 2^21) whose lookup outgrows the L2s anyway (2^22 frame 0.8890 -> 0.8855 ms, 2^21
// 0.4885 -> 0.4832, profiles/r05_sort_ntstore_ab.txt); smaller lookups stay cached for the
// next launch.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <bool NT = false>
__device__ __forceinline__ void store_eight(uint2* tile, uint32_t t, uint2 (&v)[8]) {
  quad_swap_bit<1, kDppXor2>(v, t);
  quad_swap_bit<0, kDppXor1>(v, t);
  u32x4* out = reinterpret_cast<u32x4*>(tile + 32u * (t >> 2) + 2u * (t & 3u));
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const u32x4 q{v[2 * i].x, v[2 * i].y, v[2 * i + 1].x, v[2 * i + 1].y};
    if (NT) __builtin_nontemporal_store(q, out + 4 * i);
    else out[4 * i] = q;
  }
}


// The compare-swap of the reference's pass on the entries at positions pa != pb (the lower
// position is the left one).
__device__ __forceinline__ void cas_at(uint2& va, uint32_t pa, uint2& vb, uint32_t pb) {
  uint2& l = pa < pb ? va : vb;
  uint2& r = pa < pb ? vb : va;
  if (l.x > r.x) {
    const uint2 tmp = l;
    l = r;
    r = tmp;
  }
}

// The value at position x after the first TG global passes of stage s (the flip, pairing x with
// its mirror x ^ (2^(s+1) - 1), then for TG = 2 stride 2^(s-1)): the passes of the 2^TG entries
// x's group spans (in TG other tiles), recomputed by every tile of the group; the launch's own
// tile keeps its entry.  The same compare-swaps as the register-fused launch they replace.
template <int TG>
__device__ __forceinline__ uint2 folded_global(uint32_t x, uint32_t s, const uint2 (&e)[1 << TG]) {
  const uint32_t m = (2u << s) - 1u;
  if constexpr (TG == 1) {
    uint2 a = e[0], ma = e[1];
    cas_at(a, x, ma, x ^ m);
    return a;
  } else {
    const uint32_t h = 1u << (s - 1u);
    uint2 a = e[0], b = e[1], ma = e[2], mb = e[3];
    cas_at(a, x, ma, x ^ m);  // flip
    cas_at(b, x ^ h, mb, x ^ h ^ m);
    cas_at(a, x, b, x ^ h);  // stride 2^(s-1)
    cas_at(ma, x ^ m, mb, x ^ m ^ h);
    return a;
  }
}
template <int TG>
__device__ __forceinline__ uint32_t folded_pos(uint32_t x, uint32_t s, int k) {
  const uint32_t m = (2u << s) - 1u, h = TG == 2 ? 1u << (s - 1u) : 0u;
  return (k & 1 ? (TG == 1 ? m : h) : 0u) ^ (k & 2 ? m : 0u) ^ x;
}

// TG > 0: the stage's first TG global passes folded in (stage s = TLOG + TG - 1; one launch
// fewer per such stage: DESIGN.md §5.2).  Every tile of a group reads the others' entries, so
// the launch reads `src` and writes `lookup` (a second buffer: the sort ping-pongs).
template <int TLOG, int TG = 0>
__global__ __launch_bounds__(1u << (TLOG - 3)) __attribute__((amdgpu_waves_per_eu(4))) void sph_sort_tail_kernel(
    uint2* __restrict__ lookup, const uint2* __restrict__ src) {
  static_assert(TLOG >= 10 && TLOG <= 13, "eight entries per thread, 128..1024 threads");
  constexpr uint32_t TILE = 1u << TLOG, NT = TILE / 8;
  __shared__ uint2 lds[TILE + TILE / 32];
  const uint32_t t = threadIdx.x;
  uint2* tile = lookup + (size_t)blockIdx.x * TILE;
  {  // strides TILE/2, TILE/4, TILE/8: group r = t, entries t + j * NT, straight from the lookup
    uint2 v[8];
    if constexpr (TG == 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = tile[t + j * NT];
    } else {
      constexpr uint32_t s = TLOG + TG - 1;
      uint2 e[8][1 << TG];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t x = blockIdx.x * TILE + t + j * NT;
#pragma unroll
        for (int k = 0; k < (1 << TG); ++k) e[j][k] = src[folded_pos<TG>(x, s, k)];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = folded_global<TG>(blockIdx.x * TILE + t + j * NT, s, e[j]);
    }
    group_passes<3>(v);
    const uint32_t a = padded(t);
#pragma unroll
    for (int j = 0; j < 8; ++j) lds[a + pad_off<NT>(j)] = v[j];
  }
  __syncthreads();
  lds_chunks<TLOG - 4, kTailLdsLo<TLOG>>(lds, t);
  {  // strides 8 (DPP across the lane pair (2k, 2k + 1), 8192-entry tiles), 4, 2, 1: the lane's
     // eight consecutive entries [8t, 8t + 8)
    const uint32_t a = padded(8u * t);
    uint2 v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = lds[a + i];
    if constexpr (kTailLdsLo<TLOG> > 3) xlane_pass<kDppXor1, false>(v, (t & 1u) == 0u);
    group_passes<3>(v);
    store_eight<TLOG == 13>(tile, t, v);
  }
}

// ---------------------------------------------------------------------------------------
// Static-network head launch: bin (wgsl:455-468) + every stage whose whole network fits one
// tile (stages 0 .. TLOG-1), eight entries per thread.  Between stages a thread holds its eight
// consecutive entries [8t, 8t + 8) in registers, and lane quads the 32 entries [32k, 32k + 32):
// passes of stride 1, 2, 4 run inside a lane, strides 8 and 16 (and the flips of stages 3
// and 4) across the quad with DPP moves, so stages 0-4 and the last five passes of every later
// stage never touch LDS.  A later stage S writes its entries to LDS once, runs its flip chunk
// (strides 2^S, 2^(S-1)) and its passes of strides 2^(S-2) .. 32 there in register chunks with
// compile-time addresses, and reads its entries back.  The last stage stores them.  Same
// compare-swaps in the same order as the reference's pass-per-dispatch schedule.
// ---------------------------------------------------------------------------------------


// Stages 0-2 (spans 2, 4, 8): inside the lane's eight consecutive entries.
__device__ __forceinline__ void reg_stages012(uint2 (&v)[8]) {
  cas4(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]);  // stage 0: flip G = 1
  cas4(v[0], v[3], v[1], v[2], v[4], v[7], v[5], v[6]);  // stage 1: flip G = 2, then G = 1
  cas4(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]);
  cas4(v[0], v[7], v[1], v[6], v[2], v[5], v[3], v[4]);  // stage 2: flip G = 4, then G = 2, 1
  cas4(v[0], v[2], v[1], v[3], v[4], v[6], v[5], v[7]);
  cas4(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]);
}

// The flip chunk of stage S >= 5 in LDS: the flip pass (G = 2^S) and stride 2^(S-1), on the
// residue class r and its mirror g - 1 - r (g = 2^(S-1), four entries each), thread t = group t.
template <int S>
__device__ __forceinline__ void lds_flip_chunk(uint2* lds, uint32_t t) {
  constexpr uint32_t g = 1u << (S - 1);
  constexpr int LP = S - 2;  // log2(groups per 2G block)
  const uint32_t base = (t >> LP) << (S + 1), r = t & ((1u << LP) - 1u);
  const uint32_t a = padded(base + r), b = padded(base + g - 1u - r);
  uint2 v[8];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[j] = lds[a + pad_off<g>(j)];
    v[4 + j] = lds[b + pad_off<g>(j)];
  }
  // flip: position r + j*g pairs with (g-1-r) + (3-j)*g; then stride g inside each class
  cas4(v[0], v[7], v[1], v[6], v[4], v[3], v[5], v[2]);
  cas4(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    lds[a + pad_off<g>(j)] = v[j];
    lds[b + pad_off<g>(j)] = v[4 + j];
  }
}

template <int SPAN>
__device__ __forceinline__ void lds_sync() {
  if constexpr (SPAN > 512) __syncthreads();
  else wave_lds_sync();
}

// Non-flip strides 2^LG down to 2^LO, register chunks of up to three passes; each chunk is
// followed by the sync its span needs (the register tail reads the lane's own entries next).
template <int LG, int LO>
__device__ __forceinline__ void lds_mid_chunks(uint2* lds, uint32_t t) {
  if constexpr (LG >= LO) {
    constexpr int K = LG - LO + 1 >= 3 ? 3 : LG - LO + 1;
    lds_chunk<LG, K>(lds, t);
    lds_sync<(2 << LG)>();
    lds_mid_chunks<LG - K, LO>(lds, t);
  }
}

// The register tail of a stage: strides 16 (if HI16), 8, 4, 2, 1.
template <bool HI16>
__device__ __forceinline__ void reg_tail(uint2 (&v)[8], uint32_t t) {
  if constexpr (HI16) xlane_pass<kDppXor2, false>(v, (t & 2u) == 0u);
  xlane_pass<kDppXor1, false>(v, (t & 1u) == 0u);
  group_passes<3>(v);
}

template <int S, int TLOG>
__device__ __forceinline__ void head_stages(uint2* lds, uint32_t t, uint2 (&v)[8]) {
  if constexpr (S < TLOG) {
    const uint32_t a = padded(8u * t);
#pragma unroll
    for (int i = 0; i < 8; ++i) lds[a + i] = v[i];
    lds_sync<(2 << S)>();
    lds_flip_chunk<S>(lds, t);
    lds_sync<(2 << S)>();
    lds_mid_chunks<S - 2, kHeadLdsLo<TLOG>>(lds, t);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = lds[a + i];
    if constexpr (kHeadLdsLo<TLOG> > 3) reg_tail<(S >= 6)>(v, t);  // strides 16, 8 by DPP, then 4, 2, 1
    else group_passes<3>(v);                                          // strides 4, 2, 1
    // The next stage's first LDS write goes to this lane's own entries, which only this
    // wave's chunks read in this stage once the last cross-wave chunk's barrier has passed.
    head_stages<S + 1, TLOG>(lds, t, v);
  }
}

// The bin pass for the eight consecutive entries [g0, g0 + 8): the sim's prebuilt (key, slot)
// entries and the pad entries [n, P) as four 16-B loads where the eight are all of one kind,
// positions keyed otherwise; offsets reset as bin_particles_in_grid does (wgsl:467).
__device__ __forceinline__ void bin_load_eight(const uint2* lookup, const SortBin& bin, uint32_t g0, uint2 (&v)[8]) {
  const uint2* src = g0 >= bin.n ? lookup + g0 : bin.prebuilt && g0 + 8u <= bin.n ? bin.prebuilt + g0 : nullptr;
  if (src) {
    const uint4* q = reinterpret_cast<const uint4*>(src);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint4 w = q[i];
      v[2 * i] = make_uint2(w.x, w.y);
      v[2 * i + 1] = make_uint2(w.z, w.w);
    }
    if (g0 < bin.n && bin.reset_pre) {
#pragma unroll
      for (uint32_t k = 0; k < 8; ++k) bin_reset(bin, g0 + k);
    }
    return;
  }
  uint2 raw[8];
#pragma unroll
  for (uint32_t k = 0; k < 8; ++k) {
    const uint32_t gq = g0 + k;
    raw[k] = gq >= bin.n ? lookup[gq] : bin.prebuilt ? bin.prebuilt[gq] : __builtin_bit_cast(uint2, bin_pos(bin, gq));
  }
#pragma unroll
  for (uint32_t k = 0; k < 8; ++k) {
    const uint32_t gq = g0 + k;
    if (gq >= bin.n) {
      v[k] = raw[k];
    } else if (bin.prebuilt) {
      if (bin.reset_pre) bin_reset(bin, gq);
      v[k] = raw[k];
    } else {
      v[k] = bin_key(bin, __builtin_bit_cast(f2, raw[k]), gq);
    }
  }
}

template <int TLOG>
__global__ __launch_bounds__(1u << (TLOG - 3)) __attribute__((amdgpu_waves_per_eu(4))) void sph_sort_head_kernel(uint2* __restrict__ lookup, SortBin bin) {
  static_assert(TLOG >= 10 && TLOG <= 13, "eight entries per thread, 128..1024 threads");
  constexpr uint32_t TILE = 1u << TLOG;
  __shared__ uint2 lds[TILE + TILE / 32];
  const uint32_t t = threadIdx.x;
  const uint32_t base0 = blockIdx.x * TILE;
  uint2 v[8];
  // bin: the lane's eight consecutive entries [8t, 8t + 8) straight from memory (no LDS image:
  // stages 0-4 run in registers), every load first, then the keys
  bin_load_eight(lookup, bin, base0 + 8u * t, v);
  reg_stages012(v);
  xlane_pass<kDppXor1, true>(v, (t & 1u) == 0u);  // stage 3: flip G = 8 (lane pair), then 4, 2, 1
  group_passes<3>(v);
  xlane_pass<kDppRev4, true>(v, (t & 2u) == 0u);  // stage 4: flip G = 16 (lane quad), then 8 ... 1
  reg_tail<false>(v, t);
  head_stages<5, TLOG>(lds, t, v);
  store_eight<TLOG == 13>(lookup + base0, t, v);
}

// ---------------------------------------------------------------------------------------
// Static-network gathered-tile launch: all T >= 5 global passes of one stage (strides 2^s down to
// the local tile 2^lg) in one launch, with the schedule fixed at compile time.  A workgroup gathers the residues r0 .. r0 + W - 1 (and their mirrors g - W - r0
// .. g - 1 - r0) of every class j < 2^T: in tile order tau = 2W j + W c + k the stage's passes
// are the tile's stage T + LW from its flip down to stride 2W.  The flip chunk (flip + the next
// stride) loads its eight entries straight from the lookup, the last chunk stores straight to
// it, the chunks between run in LDS with compile-time addresses.
// ---------------------------------------------------------------------------------------

// A non-flip register chunk read from LDS, stored through `store(tau, entry)`.
template <int LG, int K, int LE, class Store>
__device__ __forceinline__ void lds_chunk_out(const uint2* lds, uint32_t t, Store&& store) {
  constexpr int LGG = LG - K + 1;
  constexpr uint32_t g = 1u << LGG;
  constexpr int NG = 1 << (LE - K);
#pragma unroll
  for (int i = 0; i < NG; ++i) {
    const uint32_t q = chunk_group<LE - K>(t, i);
    const uint32_t e0 = ((q >> LGG) << (LG + 1)) + (q & (g - 1u));
    const uint32_t a = padded(e0);
    uint2 v[1 << K];
#pragma unroll
    for (int j = 0; j < (1 << K); ++j) v[j] = lds[a + pad_off<g>(j)];
    group_passes<K>(v);
#pragma unroll
    for (int j = 0; j < (1 << K); ++j) store(e0 + j * g, v[j]);
  }
}

// Non-flip strides 2^LG down to 2^LO in LDS chunks of up to LE passes, the lowest chunk (up to
// LE passes) left for lds_chunk_out.
template <int LG, int LO, int LE>
__device__ __forceinline__ void gather_mid_chunks(uint2* lds, uint32_t t) {
  constexpr int left = LG - LO + 1;  // passes from 2^LG down to 2^LO
  if constexpr (left > LE) {
    constexpr int K = (left - LE) % LE == 0 ? LE : (left - LE) % LE;
    lds_chunk<LG, K, LE>(lds, t);
    __syncthreads();
    gather_mid_chunks<LG - K, LO, LE>(lds, t);
  }
}

// 2^LE entries per thread: 8, or 16 for the nine-pass stage, whose 16-residue tile of 16 384
// entries would otherwise need 2048 threads (residue groups of 8 instead split every 128-B line
// between two workgroups: twice the L2 reads, 1.5x the HBM bytes, 22.0 us).
template <int T, int LW, int LE>
__global__ __launch_bounds__(1u << (T + LW + 1 - LE)) __attribute__((amdgpu_waves_per_eu(4))) void sph_sort_gather_kernel(
    uint2* __restrict__ lookup, uint32_t s, uint32_t lg) {
  static_assert(T >= 5 && T + LW + 1 - LE <= 10, "at most 1024 threads");
  constexpr int TL = T + LW + 1;  // log2 of the gathered tile
  constexpr int M = 1 << (LE - 1);  // entries per class in the flip chunk
  constexpr uint32_t TT = 1u << TL, W = 1u << LW, gp = TT >> (LE - 1);  // gp: the flip chunk's stride g'
  constexpr int KF = LE - 1;  // passes of the flip chunk (the flip and KF - 1 strides)
  __shared__ uint2 lds[TT + TT / 32];
  const uint32_t g = 1u << lg;
  const uint32_t rgs = lg - LW - 1u;  // log2(residue groups of W in [0, g/2))
  const uint32_t base = (blockIdx.x >> rgs) << (s + 1u);
  const uint32_t r0 = (blockIdx.x & ((1u << rgs) - 1u)) << LW;
  const auto pos = [&](uint32_t tau) {
    const uint32_t j = tau >> (LW + 1), c = (tau >> LW) & 1u, k = tau & (W - 1u);
    return base + j * g + (c ? (g - W - r0 + k) : (r0 + k));
  };
  const uint32_t t = threadIdx.x;
  {  // the flip (G' = TT/2) and strides TT/4 .. gp on class t and its mirror gp - 1 - t, from memory
    uint2 v[2 * M];
#pragma unroll
    for (int j = 0; j < M; ++j) {
      v[j] = lookup[pos(t + j * gp)];
      v[M + j] = lookup[pos(gp - 1u - t + j * gp)];
    }
#pragma unroll
    for (int j = 0; j < M / 2; j += 2)  // flip: position t + j*gp pairs with (gp-1-t) + (M-1-j)*gp
      cas4(v[j], v[2 * M - 1 - j], v[M + j], v[M - 1 - j], v[j + 1], v[2 * M - 2 - j], v[M + j + 1],
           v[M - 2 - j]);
#pragma unroll
    for (int m = KF - 2; m >= 0; --m)  // strides gp * 2^m inside each class
#pragma unroll
      for (int c = 0; c < 2 * M; c += M)
#pragma unroll
        for (int p = 0; p < M / 2; p += 2) {
          const int d = 1 << m, j0 = c + pair_lo(p, m), j1 = c + pair_lo(p + 1, m);
          cas2(v[j0], v[j0 + d], v[j1], v[j1 + d]);
        }
    const uint32_t a = padded(t), b = padded(gp - 1u - t);
#pragma unroll
    for (int j = 0; j < M; ++j) {
      lds[a + pad_off<gp>(j)] = v[j];
      lds[b + pad_off<gp>(j)] = v[M + j];
    }
  }
  __syncthreads();
  gather_mid_chunks<TL - LE, LW + 1, LE>(lds, t);  // strides gp/2 .. 2W, all but the last chunk
  constexpr int KL = T + 1 - LE >= LE ? LE : T + 1 - LE;
  lds_chunk_out<LW + KL, KL, LE>(lds, t, [&](uint32_t tau, uint2 e) { lookup[pos(tau)] = e; });
}

// ---------------------------------------------------------------------------------------
// Compact sort (2^11 <= P <= 2^16, the reference's default N = 50 000 and C1): the same network
// on 4-byte entries key << 16 | payload (key < N <= 2^16, payload < P <= 2^16), compared on the
// high halves only (v_cmp_gt_u32_sdwa WORD_1), so equal keys stay in place exactly as in the
// reference's compare-swap.  One head launch (bin + the stages inside a tile, the schedule of
// sph_sort_head_kernel) and ONE launch per later stage: its T global passes are folded into the
// tail launch for every T (the tiles of a stage's group each recompute the group's passes from
// the other tiles' entries, read from one packed buffer, written to the other), so P = 2^16 is
// five launches instead of nine.  The last launch unpacks into the uint2 lookup.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t cpack(uint2 e) { return (e.x << 16) | (e.y & 0xFFFFu); }
__device__ __forceinline__ uint2 cunpack(uint32_t e) { return make_uint2(e >> 16, e & 0xFFFFu); }

// Compare-swaps on packed entries: every compare first (the keys' high halves by SDWA), then
// each pair's v_swap_b32 with its mask as EXEC (as cas4 on uint2 entries).
__device__ __forceinline__ void ccas(uint32_t& a, uint32_t& b) {
  uint64_t m, sv;
  asm("v_cmp_gt_u32_sdwa %[m], %[a], %[b] src0_sel:WORD_1 src1_sel:WORD_1\n\t"
      "s_mov_b64 %[sv], exec\n\t"
      "s_mov_b64 exec, %[m]\n\t"
      "v_swap_b32 %[a], %[b]\n\t"
      "s_mov_b64 exec, %[sv]"
      : [a] "+v"(a), [b] "+v"(b), [m] "=&s"(m), [sv] "=&s"(sv));
}
__device__ __forceinline__ void ccas2(uint32_t& a0, uint32_t& b0, uint32_t& a1, uint32_t& b1) {
  uint64_t m0, m1, sv;
  asm("v_cmp_gt_u32_sdwa %[m0], %[a0], %[b0] src0_sel:WORD_1 src1_sel:WORD_1\n\t"
      "v_cmp_gt_u32_sdwa %[m1], %[a1], %[b1] src0_sel:WORD_1 src1_sel:WORD_1\n\t"
      "s_mov_b64 %[sv], exec\n\t"
      "s_mov_b64 exec, %[m0]\n\t"
      "v_swap_b32 %[a0], %[b0]\n\t"
      "s_mov_b64 exec, %[m1]\n\t"
      "v_swap_b32 %[a1], %[b1]\n\t"
      "s_mov_b64 exec, %[sv]"
      : [a0] "+v"(a0), [b0] "+v"(b0), [a1] "+v"(a1), [b1] "+v"(b1), [m0] "=&s"(m0), [m1] "=&s"(m1),
        [sv] "=&s"(sv));
}
__device__ __forceinline__ void ccas4(uint32_t& a0, uint32_t& b0, uint32_t& a1, uint32_t& b1, uint32_t& a2,
                                      uint32_t& b2, uint32_t& a3, uint32_t& b3) {
  uint64_t m0, m1, m2, m3, sv;
  asm("v_cmp_gt_u32_sdwa %[m0], %[a0], %[b0] src0_sel:WORD_1 src1_sel:WORD_1\n\t"
      "v_cmp_gt_u32_sdwa %[m1], %[a1], %[b1] src0_sel:WORD_1 src1_sel:WORD_1\n\t"
      "v_cmp_gt_u32_sdwa %[m2], %[a2], %[b2] src0_sel:WORD_1 src1_sel:WORD_1\n\t"
      "v_cmp_gt_u32_sdwa %[m3], %[a3], %[b3] src0_sel:WORD_1 src1_sel:WORD_1\n\t"
      "s_mov_b64 %[sv], exec\n\t"
      "s_mov_b64 exec, %[m0]\n\t"
      "v_swap_b32 %[a0], %[b0]\n\t"
      "s_mov_b64 exec, %[m1]\n\t"
      "v_swap_b32 %[a1], %[b1]\n\t"
      "s_mov_b64 exec, %[m2]\n\t"
      "v_swap_b32 %[a2], %[b2]\n\t"
      "s_mov_b64 exec, %[m3]\n\t"
      "v_swap_b32 %[a3], %[b3]\n\t"
      "s_mov_b64 exec, %[sv]"
      : [a0] "+v"(a0), [b0] "+v"(b0), [a1] "+v"(a1), [b1] "+v"(b1), [a2] "+v"(a2), [b2] "+v"(b2),
        [a3] "+v"(a3), [b3] "+v"(b3), [m0] "=&s"(m0), [m1] "=&s"(m1), [m2] "=&s"(m2), [m3] "=&s"(m3),
        [sv] "=&s"(sv));
}

// group_passes on packed entries.
template <int K>
__device__ __forceinline__ void cgroup_passes(uint32_t (&v)[1 << K]) {
#pragma unroll
  for (int m = K - 1; m >= 0; --m) {
    if constexpr (K == 1) {
      ccas(v[0], v[1]);
    } else if constexpr (K == 2) {
      const int d = 1 << m, j0 = pair_lo(0, m), j1 = pair_lo(1, m);
      ccas2(v[j0], v[j0 + d], v[j1], v[j1 + d]);
    } else {
#pragma unroll
      for (int p = 0; p < (1 << (K - 1)); p += 4) {
        const int d = 1 << m;
        const int j0 = pair_lo(p, m), j1 = pair_lo(p + 1, m), j2 = pair_lo(p + 2, m), j3 = pair_lo(p + 3, m);
        ccas4(v[j0], v[j0 + d], v[j1], v[j1 + d], v[j2], v[j2 + d], v[j3], v[j3 + d]);
      }
    }
  }
}

// xlane_pass on packed entries: one DPP move per entry.
template <int CTRL, bool REV>
__device__ __forceinline__ void cxlane_pass(uint32_t (&v)[8], bool left) {
  uint32_t p[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) p[j] = (uint32_t)__builtin_amdgcn_mov_dpp((int)v[REV ? 7 - j : j], CTRL, 0xF, 0xF, false);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const bool swap = left ? (v[j] >> 16) > (p[j] >> 16) : (p[j] >> 16) > (v[j] >> 16);
    v[j] = swap ? p[j] : v[j];
  }
}

// The LDS chunks of the head and tail (lds_chunk, lds_chunks, lds_flip_chunk, lds_mid_chunks)
// on packed entries; the same padded indices (one pad entry per 32).
template <int LG, int K>
__device__ __forceinline__ void clds_chunk(uint32_t* lds, uint32_t t) {
  constexpr int LGG = LG - K + 1;
  constexpr uint32_t g = 1u << LGG;
  constexpr int NG = 1 << (3 - K);
#pragma unroll
  for (int i = 0; i < NG; ++i) {
    const uint32_t q = chunk_group<3 - K>(t, i);
    const uint32_t e0 = ((q >> LGG) << (LG + 1)) + (q & (g - 1u));
    const uint32_t a = padded(e0);
    uint32_t v[1 << K];
#pragma unroll
    for (int j = 0; j < (1 << K); ++j) v[j] = lds[a + pad_off<g>(j)];
    cgroup_passes<K>(v);
#pragma unroll
    for (int j = 0; j < (1 << K); ++j) lds[a + pad_off<g>(j)] = v[j];
  }
}
template <int LG>
__device__ __forceinline__ void clds_chunks(uint32_t* lds, uint32_t t, bool active = true) {
  if constexpr (LG >= 4) {
    constexpr int K = LG - 3 >= 3 ? 3 : LG - 3;
    if (active) clds_chunk<LG, K>(lds, t);
    lds_sync<(2 << LG)>();  // every wave of the workgroup, active or not
    clds_chunks<LG - K>(lds, t, active);
  }
}
template <int S>
__device__ __forceinline__ void clds_flip_chunk(uint32_t* lds, uint32_t t) {
  constexpr uint32_t g = 1u << (S - 1);
  constexpr int LP = S - 2;
  const uint32_t base = (t >> LP) << (S + 1), r = t & ((1u << LP) - 1u);
  const uint32_t a = padded(base + r), b = padded(base + g - 1u - r);
  uint32_t v[8];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[j] = lds[a + pad_off<g>(j)];
    v[4 + j] = lds[b + pad_off<g>(j)];
  }
  ccas4(v[0], v[7], v[1], v[6], v[4], v[3], v[5], v[2]);
  ccas4(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    lds[a + pad_off<g>(j)] = v[j];
    lds[b + pad_off<g>(j)] = v[4 + j];
  }
}
template <int LG>
__device__ __forceinline__ void clds_mid_chunks(uint32_t* lds, uint32_t t) {
  if constexpr (LG >= 5) {
    constexpr int K = LG - 4 >= 3 ? 3 : LG - 4;
    clds_chunk<LG, K>(lds, t);
    lds_sync<(2 << LG)>();
    clds_mid_chunks<LG - K>(lds, t);
  }
}
template <bool HI16>
__device__ __forceinline__ void creg_tail(uint32_t (&v)[8], uint32_t t) {
  if constexpr (HI16) cxlane_pass<kDppXor2, false>(v, (t & 2u) == 0u);
  cxlane_pass<kDppXor1, false>(v, (t & 1u) == 0u);
  cgroup_passes<3>(v);
}
template <int S, int TLOG>
__device__ __forceinline__ void chead_stages(uint32_t* lds, uint32_t t, uint32_t (&v)[8]) {
  if constexpr (S < TLOG) {
    const uint32_t a = padded(8u * t);
#pragma unroll
    for (int i = 0; i < 8; ++i) lds[a + i] = v[i];
    lds_sync<(2 << S)>();
    clds_flip_chunk<S>(lds, t);
    lds_sync<(2 << S)>();
    clds_mid_chunks<S - 2>(lds, t);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = lds[a + i];
    creg_tail<(S >= 6)>(v, t);
    chead_stages<S + 1, TLOG>(lds, t, v);
  }
}

// A lane's eight consecutive entries [8t, 8t + 8) of the tile at `base`: packed (two 16-B
// stores) or unpacked into the uint2 lookup (four).
template <bool OUT_LOOKUP>
__device__ __forceinline__ void cstore_eight(uint32_t* __restrict__ cout, uint2* __restrict__ lookup, uint32_t base,
                                             uint32_t t, const uint32_t (&v)[8]) {
  if constexpr (OUT_LOOKUP) {
    uint4* o = reinterpret_cast<uint4*>(lookup + base + 8u * t);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint2 lo = cunpack(v[2 * i]), hi = cunpack(v[2 * i + 1]);
      o[i] = make_uint4(lo.x, lo.y, hi.x, hi.y);
    }
  } else {
    uint4* o = reinterpret_cast<uint4*>(cout + base + 8u * t);
    o[0] = make_uint4(v[0], v[1], v[2], v[3]);
    o[1] = make_uint4(v[4], v[5], v[6], v[7]);
  }
}

// Bin + stages [0, TLOG) of one tile (sph_sort_head_kernel's schedule).  Entries [n, P) are the
// previous frame's pad entries, read from the uint2 lookup (keys < N, payloads < P: both fit).
template <int TLOG, bool OUT_LOOKUP>
__global__ __launch_bounds__(1u << (TLOG - 3)) __attribute__((amdgpu_waves_per_eu(4))) void sph_csort_head_kernel(
    uint2* __restrict__ lookup, SortBin bin, uint32_t* __restrict__ cout) {
  static_assert(TLOG >= 11 && TLOG <= 13, "eight entries per thread, 256..1024 threads");
  constexpr uint32_t TILE = 1u << TLOG;
  __shared__ uint32_t lds[TILE + TILE / 32];
  const uint32_t t = threadIdx.x;
  const uint32_t base0 = blockIdx.x * TILE;
  uint32_t v[8];
  {
    uint2 e[8];
    bin_load_eight(lookup, bin, base0 + 8u * t, e);  // the lane's eight entries, no LDS image
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = cpack(e[i]);
  }
  ccas4(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]);  // stages 0-2 (reg_stages012)
  ccas4(v[0], v[3], v[1], v[2], v[4], v[7], v[5], v[6]);
  ccas4(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]);
  ccas4(v[0], v[7], v[1], v[6], v[2], v[5], v[3], v[4]);
  ccas4(v[0], v[2], v[1], v[3], v[4], v[6], v[5], v[7]);
  ccas4(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]);
  cxlane_pass<kDppXor1, true>(v, (t & 1u) == 0u);  // stage 3
  cgroup_passes<3>(v);
  cxlane_pass<kDppRev4, true>(v, (t & 2u) == 0u);  // stage 4
  creg_tail<false>(v, t);
  chead_stages<5, TLOG>(lds, t, v);
  cstore_eight<OUT_LOOKUP>(cout, lookup, base0, t, v);
}

// The values at positions x0 .. x0 + 3 (x0 = 0 mod 4) after the first TG global passes of stage
// s = TLOG + TG - 1 (the flip, then strides 2^(s-1) .. 2^TLOG).  A position x's group is the 2^TG
// positions x ^ (a * mirror) ^ (sum of b_k 2^(s-k)); indexed by u = bits [TLOG, s] of a position,
// the flip pairs u with ~u and the later passes pair u with u ^ 2^b, the lower position (u's bit
// 0) being the left one: the passes are a 2^TG-entry flip stage.  Held at c = u ^ ux (ux = x's u,
// the tile index's low bits, uniform over the workgroup), x is v[0], and each pass's direction is
// one uniform bit of ux (a scalar branch per pass).  The four positions' groups are four
// consecutive entries of each tile of the group (reversed in the mirrored ones): one 16-B load
// per tile.  Only v[0] is kept, so the compiler drops the compare-swaps outside its cone.
__device__ __forceinline__ void cas_keep(uint32_t& l, uint32_t& r) {
  const bool sw = (l >> 16) > (r >> 16);
  const uint32_t nl = sw ? r : l, nr = sw ? l : r;
  l = nl;
  r = nr;
}
template <int TG>
__device__ __forceinline__ uint4 cfold4(const uint32_t* __restrict__ src, uint32_t x0, uint32_t lo) {
  constexpr uint32_t M = 1u << TG;
  const uint32_t s = lo + TG - 1u;
  const uint32_t ux = (x0 >> lo) & (M - 1u);
  const uint32_t lowm = (1u << lo) - 1u;
  const uint32_t hi = x0 & ~((2u << s) - 1u);
  uint32_t v[4][M];
#pragma unroll
  for (uint32_t c = 0; c < M; ++c) {
    const bool mir = c >> (TG - 1);
    const uint32_t low = mir ? (lowm - 3u - (x0 & lowm)) : (x0 & lowm);
    const uint4 w = *reinterpret_cast<const uint4*>(src + (hi | ((ux ^ c) << lo) | low));
    v[0][c] = mir ? w.w : w.x;
    v[1][c] = mir ? w.z : w.y;
    v[2][c] = mir ? w.y : w.z;
    v[3][c] = mir ? w.x : w.w;
  }
  const auto pass = [&](uint32_t dim, bool flip) {
#pragma unroll
    for (uint32_t c = 0; c < M; ++c) {
      if (c & (1u << dim)) continue;
      const uint32_t c1 = flip ? (c ^ (M - 1u)) : (c | (1u << dim));
      if ((ux >> dim) & 1u) {  // c's partner is the left entry
#pragma unroll
        for (int i = 0; i < 4; ++i) cas_keep(v[i][c1], v[i][c]);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) cas_keep(v[i][c], v[i][c1]);
      }
    }
  };
  pass(TG - 1u, true);
#pragma unroll
  for (int b = TG - 2; b >= 0; --b) pass((uint32_t)b, false);
  return make_uint4(v[0][0], v[1][0], v[2][0], v[3][0]);
}

// A later stage s = TLOG + TG - 1 of one tile: its TG global passes (cfold4, four consecutive
// positions per thread and 16-B loads, through LDS to the tail's order) and its in-tile passes
// (sph_sort_tail_kernel's schedule), src -> cout, or the uint2 lookup for the last stage.
// WIDE: twice the threads (TILE / 4), one cfold4 each, so a workgroup has twice the fold loads
// in flight; the tail's in-tile passes then run on the first TILE / 8 threads (whole waves), the
// others only joining the barriers.
template <int TLOG, int TG, bool OUT_LOOKUP, bool WIDE = false>
__global__ __launch_bounds__(1u << (TLOG - (WIDE ? 2 : 3))) __attribute__((amdgpu_waves_per_eu(4))) void sph_csort_stage_kernel(
    const uint32_t* __restrict__ src, uint32_t* __restrict__ cout, uint2* __restrict__ lookup) {
  static_assert(TLOG >= 11 && TLOG <= 13 && TG >= 1 && TG <= 5 && (!WIDE || TLOG <= 12), "compact sort shapes");
  constexpr uint32_t TILE = 1u << TLOG, NT = TILE / 8;
  __shared__ uint32_t lds[TILE + TILE / 32];
  const uint32_t t = threadIdx.x;
  const uint32_t base0 = blockIdx.x * TILE;
#pragma unroll
  for (uint32_t k = 0; k < (WIDE ? 1u : 2u); ++k) {  // the folded entries 4 (t + k NT) .. + 3
    const uint32_t q = 4u * (t + k * NT);
    const uint4 f = cfold4<TG>(src, base0 + q, TLOG);
    lds[padded(q)] = f.x;  // q = 0 mod 4: the four share one pad offset
    lds[padded(q) + 1u] = f.y;
    lds[padded(q) + 2u] = f.z;
    lds[padded(q) + 3u] = f.w;
  }
  __syncthreads();
  const bool active = !WIDE || t < NT;
  if (active) {  // strides TILE/2, TILE/4, TILE/8 on the entries t + j * NT
    const uint32_t a = padded(t);
    uint32_t v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = lds[a + pad_off<NT>(j)];
    cgroup_passes<3>(v);
#pragma unroll
    for (int j = 0; j < 8; ++j) lds[a + pad_off<NT>(j)] = v[j];
  }
  lds_sync<TILE>();
  clds_chunks<TLOG - 4>(lds, t, active);
  if (active) {  // strides 8, 4, 2, 1 (lane pair: stride 8 by DPP)
    const uint32_t a = padded(8u * t);
    uint32_t v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = lds[a + i];
    cxlane_pass<kDppXor1, false>(v, (t & 1u) == 0u);
    cgroup_passes<3>(v);
    cstore_eight<OUT_LOOKUP>(cout, lookup, base0, t, v);
  }
}

// calculate_spatial_lookup_offsets, compute_shader.wgsl:507-525: offsets[key] = the first
// slot of key's run.  The same pass also records ends[key] = one past the run's last slot
// in [0, n): the reference's scan of a run stops at the first slot whose key differs or at
// N (wgsl:233-237), and the sorted prefix [0, N) holds each key's entries contiguously, so
// [offsets[key], ends[key]) is exactly the set of slots it visits, in the same order.
// (ends[] needs no reset: it is read only for keys whose offsets entry this frame set.)
__global__ __launch_bounds__(kBlock) void sph_offsets_kernel(const uint2* __restrict__ lookup,
                                                             uint32_t* __restrict__ offsets,
                                                             uint32_t* __restrict__ ends,
                                                             uint32_t n) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const uint32_t key = lookup[i].x;
  const uint32_t prev = i > 0u ? lookup[i - 1u].x : 0xFFFFFFFFu;
  const uint32_t next = i + 1u < n ? lookup[i + 1u].x : 0xFFFFFFFFu;
  if (key != prev) offsets[key] = i;
  if (key != next || i + 1u == n) ends[key] = i + 1u;
}

// Spatial record layout: cell enumeration (8 x 8 tiles; see the layout kernels below; tall
// tiles measured equal).
constexpr uint32_t kCellOut = 0xFFFFFFFFu;
constexpr uint32_t kCellPending = 0xFFFFFFFEu;  // cellrun entry the fixup resolves by key
constexpr uint32_t kRunScan = 32u;               // longest run a runs-kernel lane measures itself
constexpr uint32_t kRunIdx = 2u;                 // particle indices a run's cell_info records

#ifndef RPS_CELL_TILE_LOG
#define RPS_CELL_TILE_LOG 3  // 8 x 8 cells per tile (4 x 4: equal, 16 x 16: slower)
#endif
#ifndef RPS_CELL_TILE_LOG_X
#define RPS_CELL_TILE_LOG_X RPS_CELL_TILE_LOG
#endif
#ifndef RPS_CELL_TILE_LOG_Y
#define RPS_CELL_TILE_LOG_Y RPS_CELL_TILE_LOG
#endif
// Tile width 2^kCX and height 2^kCY cells.
constexpr uint32_t kCX = RPS_CELL_TILE_LOG_X, kCY = RPS_CELL_TILE_LOG_Y;
constexpr uint32_t kCXM = (1u << kCX) - 1u, kCYM = (1u << kCY) - 1u, kCXY = kCX + kCY;
#ifndef RPS_TILE_COLMAJOR
#define RPS_TILE_COLMAJOR 0  // tiles column by column (slower, below)
#endif
#ifndef RPS_CELL_COLMAJOR
// Cells within a tile column by column: the scans walk a particle's nine runs column by column
// (GRID_OFFSETS, wgsl:200-204), so each column's three runs are adjacent in storage (2^22
// 1.1003 -> 1.0873 ms/frame; tiles column by column too: 1.0968; 16 x 16: 1.0917, 4 x 4: 1.0961).
#define RPS_CELL_COLMAJOR 1
#endif
__device__ __forceinline__ uint32_t grid_enum_xy(const SphGrid& g, uint32_t x, uint32_t y) {
  const uint32_t in_tile = RPS_CELL_COLMAJOR ? (((x & kCXM) << kCY) | (y & kCYM)) : (((y & kCYM) << kCX) | (x & kCXM));
#if RPS_TILE_COLMAJOR
  const uint32_t th = (g.cells >> kCXY) / g.tw;
  return (((x >> kCX) * th + (y >> kCY)) << kCXY) | in_tile;
#else
  return (((y >> kCY) * g.tw + (x >> kCX)) << kCXY) | in_tile;
#endif
}
__device__ __forceinline__ uint32_t grid_enum(const SphGrid& g, int32_t cx, int32_t cy) {
  const uint32_t x = (uint32_t)cx - (uint32_t)g.cx_lo, y = (uint32_t)cy - (uint32_t)g.cy_lo;
  if (x >= g.w || y >= g.h) return kCellOut;
  return grid_enum_xy(g, x, y);
}

// Inverse of grid_enum; false for the padding cells of edge tiles.
__device__ __forceinline__ bool grid_cell(const SphGrid& g, uint32_t e, int32_t& cx, int32_t& cy) {
  const uint32_t tile = e >> kCXY;
#if RPS_TILE_COLMAJOR
  const uint32_t th = (g.cells >> kCXY) / g.tw;
  const uint32_t tx_ = tile / th, ty = tile - tx_ * th;
  const uint32_t tile_rm = ty * g.tw + tx_;  // the same tile in row-major numbering
#else
  const uint32_t ty = tile / g.tw, tile_rm = tile;
#endif
  const uint32_t lo = RPS_CELL_COLMAJOR ? ((e >> kCY) & kCXM) : (e & kCXM);
  const uint32_t hi = RPS_CELL_COLMAJOR ? (e & kCYM) : ((e >> kCX) & kCYM);
  const uint32_t x = ((tile_rm - ty * g.tw) << kCX) + lo, y = (ty << kCY) + hi;
  cx = (int32_t)((uint32_t)g.cx_lo + x);
  cy = (int32_t)((uint32_t)g.cy_lo + y);
  return x < g.w && y < g.h;
}

__constant__ int32_t kGridOff[9][2] = {{-1, -1}, {-1, 0}, {-1, 1}, {0, -1}, {0, 0},
                                       {0, 1},   {1, -1}, {1, 0},  {1, 1}};

// pre_simulation_step part 1 (wgsl:397-405) in lookup order: slot t (of all P) takes
// particle i = lookup[t].y (one 16-B gather of its packed state), applies gravity and
// predicts, and writes slot-ordered records that the later passes read contiguously
// (SphBuffers: pp_s, rec_pv, idx_s, cur_s).  The density and sim passes therefore read a
// complete snapshot.  The reference's per-particle predicted_positions /
// densities buffers are not written on the hot path; launch_sph_debug_views rebuilds them
// from the slot records on readback.  Pad slots repeat some particle and
// write identical values.
// Slot ownership (P != N), two rules:
// - Particle-order frames (no layout, or a layout frame on state in particle order) use
//   SphSlots::owner: {epoch, ~slot} in one u64 per particle, claimed by atomicMax, so the lowest
//   slot of the current active frame wins and an entry of an older frame loses to any claim
//   without a reset pass (a memset launch per frame, 4.7 us at 50 000).
// - Slot-resident layout frames (SphSlots::own_s non-null) own a particle at its unflagged
//   entry: the pad entries carry kPidFlag | index, and own_s[t] marks slot t as the owner;
//   owner[] is neither claimed nor read in those frames.
__device__ __forceinline__ uint64_t owner_tag(const SphSlots& sl, uint32_t t) {
  return ((uint64_t)sl.owner_epoch << 32) | (uint64_t)(0xFFFFFFFFu - t);
}
__device__ __forceinline__ void owner_claim(const SphSlots& sl, uint32_t i, uint32_t t) {
  atomicMax(reinterpret_cast<unsigned long long*>(sl.owner + i), (unsigned long long)owner_tag(sl, t));
}
__device__ __forceinline__ bool owner_is(const SphSlots& sl, uint32_t i, uint32_t t) {
  return sl.own_s ? sl.own_s[t] != 0u : sl.owner[i] == owner_tag(sl, t);
}

// apply_gravity (wgsl:397-400) and the prediction (:402-405) of particle i into slot u.
// `e` is the sort payload: the particle index, or with slot-resident state the particle's slot
// in st (its index then idx_prev[e]).
// A sort payload: the particle index; in a slot-resident frame the particle's slot of the
// previous frame (state st[slot], index idx_prev[slot]); or kPidFlag | index, a stale pad entry
// of a layout frame with P != N (its payload rewritten as the index, since the slot it named is
// gone), whose state sits at the particle's slot of the previous frame (bin_prev[index].y, the
// sim's bin entry) in a resident frame and at the index otherwise.
struct Payload {
  uint32_t state, pid;
};
__device__ __forceinline__ Payload resolve_payload(uint32_t e, const uint32_t* __restrict__ idx_prev,
                                                   const uint2* __restrict__ bin_prev) {
  if (e & kPidFlag) {
    const uint32_t i = e & ~kPidFlag;
    return Payload{bin_prev ? bin_prev[i].y : i, i};
  }
  return Payload{e, idx_prev ? idx_prev[e] : e};
}

__device__ __forceinline__ uint32_t predict_slot(const rps_config* __restrict__ cfg, const f4* __restrict__ st,
                                                 const SphSlots& sl, uint32_t u, uint32_t e,
                                                 const uint32_t* __restrict__ idx_prev = nullptr,
                                                 const uint2* __restrict__ bin_prev = nullptr) {
  const Payload pl = resolve_payload(e, idx_prev, bin_prev);
  const f4 s = st[pl.state];
  const uint32_t i = pl.pid;
  if (sl.own_s) sl.own_s[u] = (e & kPidFlag) ? 0u : 1u;  // P != N, resident: the unflagged entry
  else if (sl.owner) owner_claim(sl, i, u);  // P != N: the lowest slot of particle i owns it
  const float dt = cfg->fixed_delta_time;
  const float qx = s[2] + 0.0f * dt;  // apply_gravity, wgsl:397-400
  const float qy = s[3] + (-cfg->gravity) * dt;
  const float px = s[0] + qx * dt, py = s[1] + qy * dt;  // wgsl:402-405
  sl.pp_s[u] = f2{px, py};
  sl.rec_pv[u] = f4{px, py, qx, qy};
  sl.idx_s[u] = i;
  sl.cur_s[u] = f2{s[0], s[1]};
  return i;
}

__global__ __launch_bounds__(kBlock) void sph_predict_kernel(const rps_config* __restrict__ cfg,
                                                             const uint2* __restrict__ lookup,
                                                             const f4* __restrict__ st,
                                                             SphSlots sl, uint32_t p_slots,
                                                             uint32_t* __restrict__ offsets,
                                                             uint32_t* __restrict__ ends,
                                                             uint32_t n_offsets) {
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= p_slots) return;
  const uint2 e = lookup[t];
  if (t < n_offsets) {  // the offsets pass folded in (active frames): sph_offsets_kernel's body
    const uint32_t prev = t > 0u ? lookup[t - 1u].x : 0xFFFFFFFFu;
    const uint32_t next = t + 1u < n_offsets ? lookup[t + 1u].x : 0xFFFFFFFFu;
    if (e.x != prev) offsets[e.x] = t;
    if (e.x != next || t + 1u == n_offsets) ends[e.x] = t + 1u;
  }
  predict_slot(cfg, st, sl, t, e.y);
}

// The nine runs a particle at predicted position p scans, in the reference's cell order
// (wgsl:223-224 / :277-278), flattened: entry f (0 <= f < total) of their concatenation.
// The non-empty runs go to a per-lane LDS table, entry k = {slot - f of the run's first
// entry, f one past its last}, so walking the flat index costs a compare per entry and an
// LDS read per run boundary (RunCursor).  The 18 offsets/ends loads are issued together; a
// key absent from [0, N) has offsets 0xFFFFFFFF, an empty run.
typedef uint2 RunTable[9][kBlock];  // [run][lane]: consecutive lanes, consecutive banks

__device__ __forceinline__ uint32_t grid_key(int32_t cx, int32_t cy, int o, uint32_t N) {
  return cell_key((int32_t)((uint32_t)cx + (uint32_t)kGridOff[o][0]),
                  (int32_t)((uint32_t)cy + (uint32_t)kGridOff[o][1]), N);
}

// Where a scan finds the run of a neighbour cell: key-indexed {offsets, ends} in lookup order,
// or (spatial layout) the cell-ordered storage runs, found by key (key_run) for lanes whose
// 3 x 3 block leaves the layout's grid.
struct RunBounds {
  const uint32_t* offsets;
  const uint32_t* ends;
  const uint2* cellrun;
  const uint2* run2;
  const uint2* key_cell;
  uint32_t epoch;
  SphGrid g;
  uint32_t* keybits;  // SphLayoutArgs::keybits (the density pass clears it for the next frame)
};

// The storage run of key k in a layout frame: its owner cell's (cellrun), or a listed run's
// (run2); none ({0xFFFFFFFF, 0}) if the key has no run this build (key_cell of another epoch).
__device__ __forceinline__ uint2 key_run(const uint2* __restrict__ key_cell, const uint2* __restrict__ cellrun,
                                         const uint2* __restrict__ run2, uint32_t epoch, uint32_t k) {
  const uint2 kc = key_cell[k];
  if (kc.y != epoch) return make_uint2(0xFFFFFFFFu, 0u);
  return kc.x == kCellOut ? run2[k] : cellrun[kc.x];
}

template <bool LAYOUT>
__device__ __forceinline__ uint32_t nine_runs(const RunBounds& rb, float px, float py, float xoff,
                                              float yoff, float r, uint32_t N, RunTable& runs,
                                              uint32_t* nruns = nullptr) {
  const int32_t cx = f32_to_i32((px + xoff) / r);  // particle_position_to_cell_coord, wgsl:121-130
  const int32_t cy = f32_to_i32((py + yoff) / r);
  uint32_t s[9], e[9];
  if (LAYOUT) {
    const uint32_t x = (uint32_t)cx - (uint32_t)rb.g.cx_lo, y = (uint32_t)cy - (uint32_t)rb.g.cy_lo;
    const bool in = x - 1u < rb.g.w - 2u && y - 1u < rb.g.h - 2u;  // all nine cells in the grid
    if (!__builtin_amdgcn_ballot_w64(!in)) {
#pragma unroll
      for (int o = 0; o < 9; ++o) {
        const uint2 v = rb.cellrun[grid_enum_xy(rb.g, x + (uint32_t)kGridOff[o][0], y + (uint32_t)kGridOff[o][1])];
        s[o] = v.x;
        e[o] = v.y;
      }
    } else {
#pragma unroll
      for (int o = 0; o < 9; ++o) {
        const uint2 v = in ? rb.cellrun[grid_enum_xy(rb.g, x + (uint32_t)kGridOff[o][0],
                                                     y + (uint32_t)kGridOff[o][1])]
                           : key_run(rb.key_cell, rb.cellrun, rb.run2, rb.epoch, grid_key(cx, cy, o, N));
        s[o] = v.x;
        e[o] = v.y;
      }
    }
  } else {
    uint32_t key[9];
#pragma unroll
    for (int o = 0; o < 9; ++o) key[o] = grid_key(cx, cy, o, N);
#pragma unroll
    for (int o = 0; o < 9; ++o) {
      s[o] = rb.offsets[key[o]];
      e[o] = rb.ends[key[o]];
    }
  }
  // A run that starts where the previous non-empty one ends in memory extends its table
  // entry (with the spatial layout a column's three runs usually do): fewer run boundaries
  // for the cursor, the same flat entries.
  uint32_t c = 0, m = 0;
  uint2 last = make_uint2(0u, 0u);
#pragma unroll
  for (int o = 0; o < 9; ++o) {
    if (s[o] < N) {
      const uint32_t len = e[o] - s[o];
      if (m && s[o] == last.x + last.y) {
        last.y += len;
      } else {
        if (m) runs[m - 1u][threadIdx.x] = last;
        last = make_uint2(s[o] - c, c + len);
        ++m;
      }
      c += len;
    }
  }
  if (m) runs[m - 1u][threadIdx.x] = last;
  if (nruns) *nruns = m;
  return c;
}

// The run table in registers (the long scans: every lane looks up entries of one slot's list at
// once, with no chain of LDS reads): slot(f) = f + x of the last run whose start is <= f.
struct RunRegs {
  uint2 r[9];
  uint32_t n;
  __device__ RunRegs(const RunTable& t, uint32_t nr) : n(nr) {
#pragma unroll
    for (int m = 0; m < 9; ++m) r[m] = t[m][threadIdx.x];
  }
  __device__ explicit RunRegs(const uint2* g) {  // a long_table_store record (total in r9.y)
#pragma unroll
    for (int m = 0; m < 9; ++m) r[m] = g[m];
    n = g[9].x;
  }
  __device__ __forceinline__ uint32_t slot(uint32_t f) const {
    uint32_t x = r[0].x;
#pragma unroll
    for (uint32_t m = 1; m < 9; ++m)
      if (m < n && f >= r[m - 1].y) x = r[m].x;
    return f + x;
  }
};

// The in-order sum of a long scan (one wave, one slot): the lanes' terms of the entries that
// count, compacted in entry order into the wave's LDS buffer, then read back by every lane
// (broadcast reads, eight in flight) and added one entry after another -- the particle's own
// order, as v_readlane per entry did at several times the cost.
// Adds the compacted terms buf[0, cnt) to the pair s in order, each a pair (s += w) or, for
// pressure's four-wide terms, two (s += w.xy, then s += w.zw): the reference's fx, fy updates,
// as packed adds (per component IEEE, the same roundings).  Whole groups of eight go unguarded;
// a sum NaN in both components stays NaN whatever follows, so the groups stop there.
__device__ __forceinline__ void long_add(f2& s, const f2& w) { s = s + w; }
__device__ __forceinline__ void long_add(f2& s, const f4& w) {
  s = s + f2{w[0], w[1]};
  s = s + f2{w[2], w[3]};
}
template <class T>
__device__ __forceinline__ void long_sum(const T* buf, uint32_t cnt, f2& s) {
  uint32_t i = 0;
  for (; i + 8u <= cnt && !(s[0] != s[0] && s[1] != s[1]); i += 8u) {
    T w[8];
#pragma unroll
    for (uint32_t j = 0; j < 8u; ++j) w[j] = buf[i + j];
#pragma unroll
    for (uint32_t j = 0; j < 8u; ++j) long_add(s, w[j]);
  }
  if (i < cnt && !(s[0] != s[0] && s[1] != s[1])) {  // the last group
    T w[8];
#pragma unroll
    for (uint32_t j = 0; j < 8u; ++j) w[j] = buf[min(i + j, cnt - 1u)];
#pragma unroll
    for (uint32_t j = 0; j < 8u; ++j)
      if (i + j < cnt) long_add(s, w[j]);
  }
}

template <class T>
__device__ __forceinline__ uint32_t long_compact(T* buf, uint32_t base, bool in, const T& w) {
  const uint64_t m = __builtin_amdgcn_ballot_w64(in);
  const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  if (in) buf[base + below] = w;
  return base + (uint32_t)__builtin_popcountll(m);
}

// Walks the flat index forward: slot(f) for non-decreasing f < total.
struct RunCursor {
  const RunTable& runs;
  uint32_t r = 0;
  uint2 cur;
  __device__ explicit RunCursor(const RunTable& t) : runs(t), cur(t[0][threadIdx.x]) {}
  __device__ __forceinline__ uint32_t slot(uint32_t f) {
    if (f >= cur.y) cur = runs[++r][threadIdx.x];  // runs are non-empty: one step suffices
    return f + cur.x;
  }
  // The same for increasing f that may skip whole runs.
  __device__ __forceinline__ uint32_t slot_skip(uint32_t f) {
    while (f >= cur.y) cur = runs[++r][threadIdx.x];
    return f + cur.x;
  }
};

// Long scans (P != N).  The reference's pad hazard keeps the top P - N entries of
// each frame's sort as stale duplicates that sort back in, so at N = 50 000 the runs of the keys
// near N grow to 150+ entries and a particle near such a cell scans 200+ entries; its lane's
// chain of dependent batches was the density and sim kernels' critical path (5.7x the 65 536
// kernel time for 1.5x the work).  Slots whose nine runs hold more than kLongScan entries (those
// the sim scans without a mask anyway) are appended to a queue by the density kernel and
// computed one slot per WAVE by sph_density_long_kernel and sph_sim_long_kernel: 64 lanes
// load and evaluate 64 consecutive entries at once, and the sums are taken entry by entry in
// the reference's order from the lanes' terms (v_readlane), so every particle's sums are the
// same additions in the same order as in its own lane.
// A particle whose own position is not finite stays in its lane: its sums are NaN from its
// first entry on, and both scans stop after one batch.
constexpr uint32_t kLongSub = 4;  // entries per lane in flight in the long-scan kernels (256 per wave)
__device__ __forceinline__ bool long_scan(const SphSlots& sl, uint32_t total, f2 p) {
  return total > sl.long_min && fabsf(p[0]) < INFINITY && fabsf(p[1]) < INFINITY;
}

// Appends v for every lane with `want` to q (one atomic per wave).
__device__ __forceinline__ uint32_t wave_append(bool want, uint32_t* count, uint4* q, uint4 v) {
  const uint64_t m = __builtin_amdgcn_ballot_w64(want);
  if (!m) return 0u;
  const uint32_t leader = (uint32_t)__builtin_ctzll(m);
  const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  uint32_t base = 0u;
  if (lane == leader) base = atomicAdd(count, (uint32_t)__builtin_popcountll(m));
  base = (uint32_t)__builtin_amdgcn_readlane((int)base, (int)leader);
  const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  if (want) q[base + below] = v;
  return base + below;  // this lane's entry (when it appended)
}

// A queued slot's run table for the long kernels (the density pass has it in LDS): entries 0-8
// the table, entry 9 {runs, total}; the long kernels load it with the queue entry, in place of
// the keys and the 18 offsets/ends (or cellrun) loads and the table build.
__device__ __forceinline__ void long_table_store(const SphSlots& sl, uint32_t k, const RunTable& runs,
                                                 uint32_t nr, uint32_t total) {
  uint2* o = sl.longtab + (size_t)k * kLongTab;
#pragma unroll
  for (uint32_t m = 0; m < 9u; ++m)
    if (m < nr) o[m] = runs[m][threadIdx.x];
  o[9] = make_uint2(nr, total);
}

// Work mapping of the density and sim passes: thread t takes lookup slot t of all P.  Lanes
// of a wave then hold the particles of a few cells and read the same runs together.  Every
// particle's fresh entry is in exactly one slot; pad slots repeat some
// particle, whose recomputation writes the identical value (outputs are separate buffers),
// so the race is benign and results are independent of it.
//
// Neighbour masks.  Only about a third of the 3x3-cell entries lie within the smoothing
// radius; the reference adds nothing for the others (wgsl:246, :299-301, :369).  The
// density pass, which tests every entry anyway, sets bit f of a 128-bit mask per slot for
// each flat entry f within the radius (two u64 words, nbr_mask[w * P + t], one coalesced
// store each).  The sim pass rebuilds the same run table and visits only the set bits, in
// increasing f, for both of its scans: the wave pays the force bodies for the most entries
// any lane has within the radius, not for every entry scanned.  The radius test is the same
// on both sides: the sim's (q - p)^2 sums equal the density's (p - q)^2 sums bit for bit.
// A particle with more than 128 entries in its nine runs scans and tests them as before.
//
// One entry's density_kernel / near_density_kernel terms at squared distance sq (wgsl:176-189,
// :246-250), for an entry within the radius.  Correctly rounded sqrt without the input scaling
// unless a lane of the wave needs it (0 < sq < 2^-96: two particles closer than ~1e-14, only
// ever near the origin): the same bits as sqrtf (tools/sqrt_check.hip, every input), 2^22
// frame 1.2461 -> 1.2358 ms (same box).
__device__ __forceinline__ f2 density_terms(float sq, float r, float dn, float ndn) {
  const float dist = sqrt_rn_wave(sq);
  float k1 = 0.0f, k2 = 0.0f;
  if (!(dist >= r)) {
    const float v = r - dist;
    k1 = (dn * v) * v;
    k2 = ((ndn * v) * v) * v;
  }
  return f2{k1, k2};
}

// The density pass's per-slot outputs: the neighbour mask, and the neighbour halves of
// pressure_term / near_pressure_term (wgsl:323-327), which depend on this particle alone:
// evaluated once here (same ops, same bits) instead of per visiting neighbour in the sim pass.
__device__ __forceinline__ void density_store(const rps_config* __restrict__ cfg, const SphSlots& sl, uint32_t t,
                                              uint32_t p_slots, f2 p, float d, float nd, uint64_t m0, uint64_t m1) {
  sl.nbr_mask[t] = m0;
  sl.nbr_mask[p_slots + t] = m1;
  const float P = (d - cfg->target_density) * cfg->pressure_multiplier;  // wgsl:191-199
  const float Pn = nd * cfg->near_density_multiplier;
  sl.rec_pd[t] = f4{p[0], p[1], P / (d * d), Pn / (d * nd)};
  sl.dens_s[t] = f2{d, nd};
}

// calculate_density, compute_shader.wgsl:207-254: entries summed in run order, kScanBatch
// predicted positions in flight per lane across run boundaries.
template <int kScanBatch, bool LAYOUT>
__global__ __launch_bounds__(kBlock) void sph_density_kernel(const rps_config* __restrict__ cfg,
                                                             RunBounds rb, SphSlots sl, uint32_t p_slots) {
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= p_slots) return;
  const uint32_t N = cfg->particle_count;
  if (LAYOUT && t <= N / 32u) rb.keybits[t] = 0u;  // the fixup has read it; the next runs kernel sets it
  if (sl.owner && t >= N && !owner_is(sl, sl.idx_s[t], t)) return;  // a repeat no scan visits
  const f2 p = sl.pp_s[t];
  const float r = cfg->smoothing_radius, r2 = r * r;
  const float dn = cfg->density_kernel_norm, ndn = cfg->near_density_kernel_norm;
  __shared__ RunTable runs;
  uint32_t nr = 0;
  const uint32_t total = nine_runs<LAYOUT>(rb, p[0], p[1], cfg->screen_bounds[1],
                                   cfg->screen_bounds[3], r, N, runs, &nr);
  RunCursor rc(runs);
  float d = 0.0f, nd = 0.0f;
  uint64_t m0 = 0, m1 = 0;
  // Density and near density both NaN stay NaN whatever is added (payloads aside, DESIGN.md
  // §3.4).  With the particle's own position finite, the entry that made them NaN is another
  // particle's NaN (or infinite) position, already in the mask, and the sim's pressure term for
  // it is NaN in both components: the particle's state ends NaN whatever follows, so the scan
  // stops there (the rest of the mask unset).  An own non-finite position makes both sums NaN at
  // the first entry, its own included, so its mask is what the sim's self-skipping scan needs in
  // full; but with more than 128 entries the sim scans the runs and ignores the mask, so such a
  // particle stops too (at N = 50 000 the NaN particles pile into the key-0 run, which each of
  // them scanned whole: 2 180 entries by frame 70, the kernel's critical path).
  const bool own_finite = fabsf(p[0]) < INFINITY && fabsf(p[1]) < INFINITY;
  if (sl.longq) {  // long scans go to sph_density_long_kernel (see there)
    const bool defer = long_scan(sl, total, p);
    const uint32_t k =
        wave_append(defer, sl.longq_n, sl.longq, make_uint4(t + 1u, __float_as_uint(p[0]), __float_as_uint(p[1]), 0u));
    if (defer) {
      long_table_store(sl, k, runs, nr, total);
      return;
    }
  }
  const bool may_stop = own_finite || total > 128u;
  for (uint32_t f = 0; f < total && !(may_stop && d != d && nd != nd); f += kScanBatch) {
    f2 q[kScanBatch];
#pragma unroll
    for (int u = 0; u < kScanBatch; ++u) q[u] = sl.pp_s[rc.slot(min(f + u, total - 1u))];
#pragma unroll
    for (int u = 0; u < kScanBatch; ++u) {
      if (f + u < total) {
        const float dx = p[0] - q[u][0], dy = p[1] - q[u][1];
        const float sq = dx * dx + dy * dy;
        if (!(sq > r2)) {
          const uint32_t b = f + u;
          if (total <= 128u) {  // otherwise the sim pass scans the runs (masks unused)
            if (b < 64u) m0 |= 1ull << b;
            else m1 |= 1ull << (b - 64u);
          }
          const f2 k = density_terms(sq, r, dn, ndn);
          d = d + k[0];
          nd = nd + k[1];
        }
      }
    }
  }
  density_store(cfg, sl, t, p_slots, p, d, nd, m0, m1);
}

// Lane pairs (small P: one slot per lane leaves a single wave per SIMD, and each wave waits on
// one lane's chain of gathers).  Lanes 2k and 2k + 1 take the same slot: the even lane gathers
// and evaluates flat entries f, f + 2, ..., the odd lane f + 1, f + 3, ...; each lane then takes
// its partner's terms by DPP and BOTH add every entry in the reference's order (entry f + 2u,
// then f + 2u + 1), so the pair holds identical sums, masks and loop conditions: the same
// additions in the same order as one lane, twice the waves and half the chain per lane.
// Generalised to G = 2 or 4 lanes per slot (lane groups): lane `sub` of a group takes entries
// f + G u + sub; every lane adds all G entries of each step in order, taking the others' terms by
// a DPP broadcast inside the group, and the group's "entry counts" flags from one ballot.
template <int G, int K>
__device__ __forceinline__ float grp_bcast(float v) {  // lane K of this lane's group
  constexpr int ctrl = G == 4 ? K * 0x55 : (K ? 0xF5 : 0xA0);  // quad_perm [K,K,K,K] / [K,K,K+2,K+2]
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), ctrl, 0xF, 0xF, false));
}
template <int G>
__device__ __forceinline__ uint32_t grp_flags(bool use) {  // bit k: lane k of the group's flag
  const uint64_t m = __builtin_amdgcn_ballot_w64(use);
  return (uint32_t)(m >> (threadIdx.x & 63u & ~(uint32_t)(G - 1))) & ((1u << G) - 1u);
}

// calculate_density (wgsl:207-254) by lane pairs; otherwise sph_density_kernel.
template <int kScanBatch, bool LAYOUT, int G>
__global__ __launch_bounds__(kBlock) void sph_density2_kernel(const rps_config* __restrict__ cfg,
                                                              RunBounds rb, SphSlots sl, uint32_t p_slots) {
  const uint32_t g = blockIdx.x * kBlock + threadIdx.x;
  const uint32_t t = g / G, par = g % G;
  if (t >= p_slots) return;  // pair-uniform, as every condition below
  const uint32_t N = cfg->particle_count;
  if (LAYOUT && par == 0u && t <= N / 32u) rb.keybits[t] = 0u;
  if (sl.owner && t >= N && !owner_is(sl, sl.idx_s[t], t)) return;
  const f2 p = sl.pp_s[t];
  const float r = cfg->smoothing_radius, r2 = r * r;
  const float dn = cfg->density_kernel_norm, ndn = cfg->near_density_kernel_norm;
  __shared__ RunTable runs;
  uint32_t nr = 0;
  const uint32_t total = nine_runs<LAYOUT>(rb, p[0], p[1], cfg->screen_bounds[1],
                                   cfg->screen_bounds[3], r, N, runs, &nr);
  RunCursor rc(runs);
  float d = 0.0f, nd = 0.0f;
  uint64_t m0 = 0, m1 = 0;
  const bool own_finite = fabsf(p[0]) < INFINITY && fabsf(p[1]) < INFINITY;
  if (sl.longq) {
    const bool defer = long_scan(sl, total, p);
    const uint32_t k = wave_append(defer && par == 0u, sl.longq_n, sl.longq,
                                   make_uint4(t + 1u, __float_as_uint(p[0]), __float_as_uint(p[1]), 0u));
    if (defer) {
      if (par == 0u) long_table_store(sl, k, runs, nr, total);
      return;
    }
  }
  const bool may_stop = own_finite || total > 128u;
  for (uint32_t f = 0; f < total && !(may_stop && d != d && nd != nd); f += G * kScanBatch) {
    f2 q[kScanBatch];
#pragma unroll
    for (int u = 0; u < kScanBatch; ++u) q[u] = sl.pp_s[rc.slot_skip(min(f + G * u + par, total - 1u))];
#pragma unroll
    for (int u = 0; u < kScanBatch; ++u) {
      const uint32_t b = f + G * u + par;  // this lane's entry
      const float dx = p[0] - q[u][0], dy = p[1] - q[u][1];
      const float sq = dx * dx + dy * dy;
      const bool in = b < total && !(sq > r2);
      f2 k = f2{0.0f, 0.0f};
      if (in) k = density_terms(sq, r, dn, ndn);
      const uint32_t fl = grp_flags<G>(in);  // entries f + G u + 0 .. G - 1, in order
      const auto add = [&](float a0, float a1, int kk) {
        if ((fl >> kk) & 1u) {
          d = d + a0;
          nd = nd + a1;
        }
      };
      add(grp_bcast<G, 0>(k[0]), grp_bcast<G, 0>(k[1]), 0);
      add(grp_bcast<G, 1>(k[0]), grp_bcast<G, 1>(k[1]), 1);
      if constexpr (G == 4) {
        add(grp_bcast<G, 2>(k[0]), grp_bcast<G, 2>(k[1]), 2);
        add(grp_bcast<G, 3>(k[0]), grp_bcast<G, 3>(k[1]), 3);
      }
      if (total <= 128u) {
        const uint32_t be = f + G * u;  // a multiple of G: the group's bits in one word
        if (be < 64u) m0 |= (uint64_t)fl << be;
        else m1 |= (uint64_t)fl << (be - 64u);
      }
    }
  }
  if (par == 0u) density_store(cfg, sl, t, p_slots, p, d, nd, m0, m1);
}

// A long scan of the density pass (kLongScan): one queued slot per wave, 64 entries per step.
__global__ __launch_bounds__(kBlock) void sph_density_long_kernel(const rps_config* __restrict__ cfg,
                                                                  SphSlots sl, uint32_t p_slots) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));  // uniform: the queue entry and its table go to SGPRs
  const uint32_t nw = gridDim.x * (kBlock / 64u);
  const float r = cfg->smoothing_radius, r2 = r * r;
  const float dn = cfg->density_kernel_norm, ndn = cfg->near_density_kernel_norm;
  __shared__ f2 terms[kBlock / 64u][64u * kLongSub];
  for (uint32_t k = blockIdx.x * (kBlock / 64u) + wv;; k += nw) {
    const uint4 e = sl.longq[k];
    if (!e.x) break;  // past the last entry
    const uint32_t t = e.x - 1u;
    const f2 p = f2{__uint_as_float(e.y), __uint_as_float(e.z)};
    // The slot's run table as the density pass stored it, in registers: lane l looks up entries
    // l, l + 64, ... directly.
    const uint2* tg = sl.longtab + (size_t)k * kLongTab;
    const RunRegs rr(tg);
    const uint32_t total = tg[9].y;
    float d = 0.0f, nd = 0.0f;
    for (uint32_t f0 = 0; f0 < total; f0 += 64u * kLongSub) {
      f2 q[kLongSub];
#pragma unroll
      for (uint32_t u = 0; u < kLongSub; ++u) q[u] = sl.pp_s[rr.slot(min(f0 + 64u * u + lane, total - 1u))];
      uint32_t cnt = 0;
#pragma unroll
      for (uint32_t u = 0; u < kLongSub; ++u) {
        const float dx = p[0] - q[u][0], dy = p[1] - q[u][1];
        const float sq = dx * dx + dy * dy;
        const f2 kk = density_terms(sq, r, dn, ndn);
        cnt = long_compact(terms[wv], cnt, f0 + 64u * u + lane < total && !(sq > r2), kk);
      }
      wave_lds_sync();
      // entries in increasing f: the lane's order; a sum NaN in both components stays NaN
      f2 dd = f2{d, nd};
      long_sum(terms[wv], cnt, dd);
      d = dd[0];
      nd = dd[1];
      wave_lds_sync();  // the next chunk rewrites the buffer
      if (d != d && nd != nd) break;  // NaN whatever follows (more than 128 entries: no mask)
    }
    if (lane == 0u) density_store(cfg, sl, t, p_slots, p, d, nd, 0ull, 0ull);
  }
}

// Drivers of the sim pass's two scans: body(q) for every entry within the radius that is
// not the particle itself, in the reference's order, q = load(slot).  Self-skip (wgsl:295,
// :365) compares particle indices; with P == N there are no pad entries, every particle owns
// exactly one slot, and the index test is the slot test j != t, which saves the 4-B index
// load per entry (kPads = false).
template <int kScanBatch, bool kPads, class Load, class Body, class Done>
__device__ __forceinline__ void scan_masked(const SphSlots& sl, const RunTable& runs, uint64_t m0,
                                            uint64_t m1, uint32_t self, Load&& load, Body&& body,
                                            Done&& done) {
  RunCursor rc(runs);
  while ((m0 | m1) && !done()) {
    uint32_t fs[kScanBatch], qi[kScanBatch];
    bool live[kScanBatch];
    f4 q[kScanBatch];
#pragma unroll
    for (int u = 0; u < kScanBatch; ++u) {  // the next set bits, lowest first
      live[u] = (m0 | m1) != 0;
      if (m0) {
        fs[u] = (uint32_t)__builtin_ctzll(m0);
        m0 &= m0 - 1u;
      } else if (m1) {
        fs[u] = 64u + (uint32_t)__builtin_ctzll(m1);
        m1 &= m1 - 1u;
      } else {
        fs[u] = u ? fs[u - 1] : 0u;
      }
    }
#pragma unroll
    for (int u = 0; u < kScanBatch; ++u) {
      const uint32_t j = rc.slot_skip(fs[u]);
      q[u] = load(j);
      qi[u] = kPads ? sl.idx_s[j] : j;
    }
#pragma unroll
    for (int u = 0; u < kScanBatch; ++u)
      if (live[u] && qi[u] != self) body(q[u]);
  }
}

template <int kScanBatch, bool kPads, class Load, class Body, class Done>
__device__ __forceinline__ void scan_runs(const SphSlots& sl, const RunTable& runs, uint32_t f0,
                                          uint32_t total, f2 p, float r2, uint32_t self, Load&& load,
                                          Body&& body, Done&& done) {
  RunCursor rc(runs);
  for (uint32_t f = f0; f < total && !done(); f += kScanBatch) {
    f4 q[kScanBatch];
    uint32_t qi[kScanBatch];
#pragma unroll
    for (int u = 0; u < kScanBatch; ++u) {
      const uint32_t j = rc.slot_skip(min(f + u, total - 1u));
      q[u] = load(j);
      qi[u] = kPads ? sl.idx_s[j] : j;
    }
#pragma unroll
    for (int u = 0; u < kScanBatch; ++u) {
      if (f + u < total && qi[u] != self) {
        const float dx = q[u][0] - p[0], dy = q[u][1] - p[1];
        if (!(dx * dx + dy * dy > r2)) body(q[u]);
      }
    }
  }
}

// One entry's pressure_force terms (wgsl:279-334) for an entry within the radius: the
// pressure and near-pressure contributions {x, y, near x, near y}, each the product the
// reference adds (the sums take them in that order).
__device__ __forceinline__ f4 pressure_terms(const f4& q, f2 p, float P_rho2, float Pn_rho2, float r, float dn,
                                             float ndn) {
  const float dx = q[0] - p[0], dy = q[1] - p[1];
  const float dist = sqrt_rn_wave(dx * dx + dy * dy);
  float dirx, diry;
  if (dist > 0.0001f) {
    dirx = dx / dist;
    diry = dy / dist;
  } else {
    dirx = 0.0f;
    diry = 1.0f;
  }
  const float pt = P_rho2 + q[2];    // + Pj / (rj * rj)
  const float npt = Pn_rho2 + q[3];  // + Pnj / (rj * rnj)
  float dk = 0.0f, ndk = 0.0f;
  if (!(dist >= r)) {
    const float v = r - dist;
    dk = (-2.0f * dn) * v;
    ndk = ((-3.0f * ndn) * v) * v;
  }
  return f4{(dirx * pt) * dk, (diry * pt) * dk, (dirx * npt) * ndk, (diry * npt) * ndk};
}

// viscosity_kernel of an entry within the radius (wgsl:336-384): the weight of (v_j - v_i).
__device__ __forceinline__ float viscosity_weight(const f4& q, f2 p, float r, float vn) {
  const float dx = p[0] - q[0], dy = p[1] - q[1];
  const float dist = sqrt_rn_wave(dx * dx + dy * dy);
  float k = 0.0f;
  if (!(dist >= r)) {
    const float v = r * r - dist * dist;
    k = ((vn * v) * v) * v;
  }
  return k;
}

// The sim pass's loop invariants of slot t (its particle i).
struct SimOwn {
  f2 p;
  float P_rho2, Pn_rho2;  // loop-invariant halves of pressure_term and near_pressure_term (wgsl:323-327)
  uint32_t i;
};
__device__ __forceinline__ SimOwn sim_own(const rps_config* __restrict__ cfg, const SphSlots& sl, uint32_t t) {
  const f4 own = sl.rec_pd[t];  // own predicted position (xy) and P / rho^2 (z)
  // own records read once (the masks, densities, current positions: nontemporal, so they do not
  // take the L2 lines the neighbour gathers use; 2^22 frame 0.8950 -> 0.8848 ms, 2^21 0.4920 ->
  // 0.4871); rec_pd / rec_pv lines are the neighbours' too
  const f2 own_d = __builtin_nontemporal_load(sl.dens_s + t);
  const float rho = own_d[0];
  const float Pn = own_d[1] * cfg->near_density_multiplier;
  return SimOwn{f2{own[0], own[1]}, own[2], Pn / (rho * rho), sl.idx_s[t]};
}

// Viscosity applied, Euler (wgsl:392-395), walls (:69-99) and the store of slot t's new state
// (RESIDENT: at the slot, slot-resident state; else at the particle).
template <bool RESIDENT>
__device__ __forceinline__ void sim_finish(const rps_config* __restrict__ cfg, const SphSlots& sl, f4* __restrict__ st,
                                           uint2* __restrict__ bin_next, uint32_t t, uint32_t i, float qx, float qy,
                                           float wx, float wy) {
  const float dt = cfg->fixed_delta_time;
  qx = qx + (wx * cfg->viscocity_strength) * dt;
  qy = qy + (wy * cfg->viscocity_strength) * dt;
  const f2 c = __builtin_nontemporal_load(sl.cur_s + t);
  float ox = c[0] + qx * dt;
  float oy = c[1] + qy * dt;
  wall(cfg->screen_bounds[0], cfg->screen_bounds[1], cfg->screen_bounds[2], cfg->screen_bounds[3],
       cfg->damping_factor, ox, oy, qx, qy);
  if (RESIDENT) {
    // Slot-resident state: the new state at its slot (a coalesced store instead of a 16-B
    // scatter), and the next frame's bin entry of particle i (bin_key's ops on the same
    // position and config), which the next head launch reads in place of the positions.
    st[t] = f4{ox, oy, qx, qy};
    const float r = cfg->smoothing_radius;
    const int32_t cx = f32_to_i32((ox + cfg->screen_bounds[1]) / r);
    const int32_t cy = f32_to_i32((oy + cfg->screen_bounds[3]) / r);
    // a scattered 8-B store (particle order): nontemporal, so it does not take the L2 lines the
    // neighbour gathers use (2^22 frame 0.9035 -> 0.8936 ms, 2^21 0.4964 -> 0.4933)
    __builtin_nontemporal_store((uint64_t)cell_key(cx, cy, cfg->particle_count) | ((uint64_t)t << 32),
                                reinterpret_cast<uint64_t*>(bin_next + i));
  } else {
    st[i] = f4{ox, oy, qx, qy};
    if (bin_next) {  // the next frame's bin entry in particle order (SphBuffers::pkeys)
      const float r = cfg->smoothing_radius;
      const int32_t cx = f32_to_i32((ox + cfg->screen_bounds[1]) / r);
      const int32_t cy = f32_to_i32((oy + cfg->screen_bounds[3]) / r);
      bin_next[i] = make_uint2(cell_key(cx, cy, cfg->particle_count), i);
    }
  }
}

// simulation_step, compute_shader.wgsl:435-453: pressure (:256-334) and viscosity
// (:336-384) against the start-of-pass velocity snapshot (rec_pv.zw), Euler (:392-395) and
// walls (:69-99).  The new packed state of particle i is written in place, st[i]: after the
// predict pass nothing reads st in this frame (the scans read the slot records), so one state
// buffer does; a second one (ping-pong) only added 64 MB at 2^22 to the frame's working set,
// which is what decides whether the scattered 16-B writes merge in the Infinity Cache or go
// to HBM as partial-line writes.  Slots the density pass queued (long scans)
// are left to sph_sim_long_kernel.
template <int kScanBatch, bool kPads, bool LAYOUT>
__device__ __forceinline__ void sim_body(const rps_config* __restrict__ cfg, const RunBounds& rb, const SphSlots& sl,
                                         f4* __restrict__ st, uint2* __restrict__ bin_next, uint32_t p_slots,
                                         uint32_t bid, RunTable& runs) {
  const uint32_t t = bid * kBlock + threadIdx.x;
  if (t >= p_slots) return;
  const SimOwn o = sim_own(cfg, sl, t);
  if (kPads && !owner_is(sl, o.i, t)) return;  // a repeat: its owner slot computes the same state
  const uint32_t self = kPads ? o.i : t;
  const float dt = cfg->fixed_delta_time;
  const float r = cfg->smoothing_radius, r2 = r * r;
  const uint32_t N = cfg->particle_count;
  const float dn = cfg->density_kernel_norm, ndn = cfg->near_density_kernel_norm;
  const float vn = cfg->viscocity_kernel_norm;
  const f2 p = o.p;
  const uint32_t total = nine_runs<LAYOUT>(rb, p[0], p[1], cfg->screen_bounds[1],
                                   cfg->screen_bounds[3], r, N, runs);
  const bool masked = total <= 128u;
  if (sl.longq && long_scan(sl, total, p)) return;  // queued by the density pass
  const uint64_t m0 = masked ? __builtin_nontemporal_load(sl.nbr_mask + t) : 0u,
                 m1 = masked ? __builtin_nontemporal_load(sl.nbr_mask + p_slots + t) : 0u;
  float fx = 0.0f, fy = 0.0f;
  const auto load_pd = [&](uint32_t j) { return sl.rec_pd[j]; };
  const auto pressure = [&](const f4& q) {
    const f4 w = pressure_terms(q, p, o.P_rho2, o.Pn_rho2, r, dn, ndn);
    fx = fx + w[0];
    fy = fy + w[1];
    fx = fx + w[2];
    fy = fy + w[3];
  };
  // A force sum that is NaN in both components stays NaN whatever is added (payloads aside,
  // DESIGN.md §3.4): the scan stops there.  Only a particle whose state ends NaN gets there.
  const auto pressure_nan = [&] { return fx != fx && fy != fy; };
  if (masked)
    scan_masked<kScanBatch, kPads>(sl, runs, m0, m1, self, load_pd, pressure, pressure_nan);
  else
    scan_runs<kScanBatch, kPads>(sl, runs, 0u, total, p, r2, self, load_pd, pressure, pressure_nan);
  const f4 own_pv = sl.rec_pv[t];
  const float qx = own_pv[2] + fx * dt;  // post-gravity velocity (the pre pass, wgsl:397-400)
  const float qy = own_pv[3] + fy * dt;
  float wx = 0.0f, wy = 0.0f;
  const auto load_pv = [&](uint32_t j) { return sl.rec_pv[j]; };
  const auto viscosity = [&](const f4& q) {
    const float k = viscosity_weight(q, p, r, vn);
    wx = wx + (q[2] - qx) * k;
    wy = wy + (q[3] - qy) * k;
  };
  const auto viscosity_nan = [&] { return wx != wx && wy != wy; };
  if (masked)
    scan_masked<kScanBatch, kPads>(sl, runs, m0, m1, self, load_pv, viscosity, viscosity_nan);
  else
    scan_runs<kScanBatch, kPads>(sl, runs, 0u, total, p, r2, self, load_pv, viscosity, viscosity_nan);
  sim_finish<LAYOUT>(cfg, sl, st, bin_next, t, o.i, qx, qy, wx, wy);
}

template <int kScanBatch, bool kPads, bool LAYOUT>
__global__ __launch_bounds__(kBlock) void sph_sim_kernel(const rps_config* __restrict__ cfg,
                                                         RunBounds rb, SphSlots sl, f4* __restrict__ st,
                                                         uint2* __restrict__ bin_next, uint32_t p_slots) {
  __shared__ RunTable runs;
  sim_body<kScanBatch, kPads, LAYOUT>(cfg, rb, sl, st, bin_next, p_slots, blockIdx.x, runs);
}

// Lane-pair drivers of the sim's scans (see sph_density2_kernel): the entries split between the
// lanes of a pair -- masked: the set bits alternately (the even lane the 1st, 3rd, ... of each
// batch's pairs of bits); runs: flat entries f + 2u + par --, each lane evaluating its entries'
// terms (term(q), for entries within the radius that are not the particle itself), and both
// lanes adding every entry's terms in the reference's order through add(terms, use, par).
__device__ __forceinline__ bool pop_bit(uint64_t& m0, uint64_t& m1, uint32_t& f) {
  if (m0) {
    f = (uint32_t)__builtin_ctzll(m0);
    m0 &= m0 - 1u;
    return true;
  }
  if (m1) {
    f = 64u + (uint32_t)__builtin_ctzll(m1);
    m1 &= m1 - 1u;
    return true;
  }
  return false;
}
template <int kScanBatch, bool kPads, int G, class T, class Load, class Term, class Add, class Done>
__device__ __forceinline__ void scan_masked2(const SphSlots& sl, const RunTable& runs, uint64_t m0, uint64_t m1,
                                             uint32_t self, uint32_t par, Load&& load, Term&& term, Add&& add,
                                             Done&& done) {
  RunCursor rc(runs);
  uint32_t prev = 0u;
  while ((m0 | m1) && !done()) {
    uint32_t fs[kScanBatch], qi[kScanBatch];
    bool live[kScanBatch];
    f4 q[kScanBatch];
#pragma unroll
    for (int u = 0; u < kScanBatch; ++u) {  // the next G set bits, lowest first: lane k takes the k-th
      uint32_t first = 0u, mine = 0u;
      bool any = false, got = false;
#pragma unroll
      for (int kk = 0; kk < G; ++kk) {
        uint32_t fb = 0u;
        const bool lb = pop_bit(m0, m1, fb);
        if (kk == 0) {
          any = lb;
          first = fb;
        }
        if ((uint32_t)kk == par) {
          got = lb;
          mine = fb;
        }
      }
      live[u] = got;
      // an idle lane re-reads an entry it may read (the loop runs while lane 0 has one)
      fs[u] = got ? mine : (any ? first : prev);
      prev = fs[u];
    }
#pragma unroll
    for (int u = 0; u < kScanBatch; ++u) {
      const uint32_t j = rc.slot_skip(fs[u]);
      q[u] = load(j);
      qi[u] = kPads ? sl.idx_s[j] : j;
    }
#pragma unroll
    for (int u = 0; u < kScanBatch; ++u) {
      const bool use = live[u] && qi[u] != self;
      T w{};
      if (use) w = term(q[u]);
      add(w, use, par);
    }
  }
}
template <int kScanBatch, bool kPads, int G, class T, class Load, class Term, class Add, class Done>
__device__ __forceinline__ void scan_runs2(const SphSlots& sl, const RunTable& runs, uint32_t total, f2 p, float r2,
                                           uint32_t self, uint32_t par, Load&& load, Term&& term, Add&& add,
                                           Done&& done) {
  RunCursor rc(runs);
  for (uint32_t f = 0; f < total && !done(); f += G * kScanBatch) {
    f4 q[kScanBatch];
    uint32_t qi[kScanBatch];
#pragma unroll
    for (int u = 0; u < kScanBatch; ++u) {
      const uint32_t j = rc.slot_skip(min(f + G * u + par, total - 1u));
      q[u] = load(j);
      qi[u] = kPads ? sl.idx_s[j] : j;
    }
#pragma unroll
    for (int u = 0; u < kScanBatch; ++u) {
      const float dx = q[u][0] - p[0], dy = q[u][1] - p[1];
      const bool use = f + G * u + par < total && qi[u] != self && !(dx * dx + dy * dy > r2);
      T w{};
      if (use) w = term(q[u]);
      add(w, use, par);
    }
  }
}

// simulation_step (wgsl:435-453) by lane pairs; otherwise sph_sim_kernel.
template <int kScanBatch, bool kPads, bool LAYOUT, int G>
__device__ __forceinline__ void sim2_body(const rps_config* __restrict__ cfg, const RunBounds& rb, const SphSlots& sl,
                                          f4* __restrict__ st, uint2* __restrict__ bin_next, uint32_t p_slots,
                                          uint32_t bid, RunTable& runs) {
  const uint32_t g = bid * kBlock + threadIdx.x;
  const uint32_t t = g / G, par = g % G;
  if (t >= p_slots) return;
  const SimOwn o = sim_own(cfg, sl, t);
  if (kPads && !owner_is(sl, o.i, t)) return;
  const uint32_t self = kPads ? o.i : t;
  const float dt = cfg->fixed_delta_time;
  const float r = cfg->smoothing_radius, r2 = r * r;
  const uint32_t N = cfg->particle_count;
  const float dn = cfg->density_kernel_norm, ndn = cfg->near_density_kernel_norm;
  const float vn = cfg->viscocity_kernel_norm;
  const f2 p = o.p;
  const uint32_t total = nine_runs<LAYOUT>(rb, p[0], p[1], cfg->screen_bounds[1],
                                   cfg->screen_bounds[3], r, N, runs);
  const bool masked = total <= 128u;
  if (sl.longq && long_scan(sl, total, p)) return;
  const uint64_t m0 = masked ? __builtin_nontemporal_load(sl.nbr_mask + t) : 0u,
                 m1 = masked ? __builtin_nontemporal_load(sl.nbr_mask + p_slots + t) : 0u;
  float fx = 0.0f, fy = 0.0f;
  const auto load_pd = [&](uint32_t j) { return sl.rec_pd[j]; };
  const auto pterm = [&](const f4& q) { return pressure_terms(q, p, o.P_rho2, o.Pn_rho2, r, dn, ndn); };
  const auto padd = [&](const f4& w, bool use, uint32_t) {
    const uint32_t fl = grp_flags<G>(use);  // the group's entries of this step, lane 0's first
    const auto add = [&](float a, float b, float c, float e, int kk) {
      if ((fl >> kk) & 1u) {
        fx = fx + a;
        fy = fy + b;
        fx = fx + c;
        fy = fy + e;
      }
    };
    add(grp_bcast<G, 0>(w[0]), grp_bcast<G, 0>(w[1]), grp_bcast<G, 0>(w[2]), grp_bcast<G, 0>(w[3]), 0);
    add(grp_bcast<G, 1>(w[0]), grp_bcast<G, 1>(w[1]), grp_bcast<G, 1>(w[2]), grp_bcast<G, 1>(w[3]), 1);
    if constexpr (G == 4) {
      add(grp_bcast<G, 2>(w[0]), grp_bcast<G, 2>(w[1]), grp_bcast<G, 2>(w[2]), grp_bcast<G, 2>(w[3]), 2);
      add(grp_bcast<G, 3>(w[0]), grp_bcast<G, 3>(w[1]), grp_bcast<G, 3>(w[2]), grp_bcast<G, 3>(w[3]), 3);
    }
  };
  const auto pressure_nan = [&] { return fx != fx && fy != fy; };
  if (masked)
    scan_masked2<kScanBatch, kPads, G, f4>(sl, runs, m0, m1, self, par, load_pd, pterm, padd, pressure_nan);
  else
    scan_runs2<kScanBatch, kPads, G, f4>(sl, runs, total, p, r2, self, par, load_pd, pterm, padd, pressure_nan);
  const f4 own_pv = sl.rec_pv[t];
  const float qx = own_pv[2] + fx * dt;
  const float qy = own_pv[3] + fy * dt;
  float wx = 0.0f, wy = 0.0f;
  const auto load_pv = [&](uint32_t j) { return sl.rec_pv[j]; };
  const auto vterm = [&](const f4& q) {
    const float k = viscosity_weight(q, p, r, vn);
    return f2{(q[2] - qx) * k, (q[3] - qy) * k};
  };
  const auto vadd = [&](const f2& w, bool use, uint32_t) {
    const uint32_t fl = grp_flags<G>(use);
    const auto add = [&](float a, float b, int kk) {
      if ((fl >> kk) & 1u) {
        wx = wx + a;
        wy = wy + b;
      }
    };
    add(grp_bcast<G, 0>(w[0]), grp_bcast<G, 0>(w[1]), 0);
    add(grp_bcast<G, 1>(w[0]), grp_bcast<G, 1>(w[1]), 1);
    if constexpr (G == 4) {
      add(grp_bcast<G, 2>(w[0]), grp_bcast<G, 2>(w[1]), 2);
      add(grp_bcast<G, 3>(w[0]), grp_bcast<G, 3>(w[1]), 3);
    }
  };
  const auto viscosity_nan = [&] { return wx != wx && wy != wy; };
  if (masked)
    scan_masked2<kScanBatch, kPads, G, f2>(sl, runs, m0, m1, self, par, load_pv, vterm, vadd, viscosity_nan);
  else
    scan_runs2<kScanBatch, kPads, G, f2>(sl, runs, total, p, r2, self, par, load_pv, vterm, vadd, viscosity_nan);
  if (par == 0u) sim_finish<LAYOUT>(cfg, sl, st, bin_next, t, o.i, qx, qy, wx, wy);
}

template <int kScanBatch, bool kPads, bool LAYOUT, int G>
__global__ __launch_bounds__(kBlock) void sph_sim2_kernel(const rps_config* __restrict__ cfg,
                                                          RunBounds rb, SphSlots sl, f4* __restrict__ st,
                                                          uint2* __restrict__ bin_next, uint32_t p_slots) {
  __shared__ RunTable runs;
  sim2_body<kScanBatch, kPads, LAYOUT, G>(cfg, rb, sl, st, bin_next, p_slots, blockIdx.x, runs);
}

// The sim pass of the density pass's queued slots (kLongScan), one per wave: lane l evaluates
// flat entries l, l + 64, ... of both scans; the sums add the lanes' terms entry by entry
// (long_compact, then every lane reads them back in order).
typedef f4 LongTerms[kBlock / 64u][64u * kLongSub];  // 16 KiB: fits a RunTable's 18 KiB
template <bool kPads, bool LAYOUT>
__device__ __forceinline__ void sim_long_body(const rps_config* __restrict__ cfg, const SphSlots& sl, f4* __restrict__ st, uint2* __restrict__ bin_next,
                                              uint32_t bid, uint32_t nblk, LongTerms& terms) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));  // uniform: the queue entry and its table go to SGPRs
  const uint32_t nw = nblk * (kBlock / 64u);
  const float dt = cfg->fixed_delta_time;
  const float r = cfg->smoothing_radius, r2 = r * r;
  const float dn = cfg->density_kernel_norm, ndn = cfg->near_density_kernel_norm;
  const float vn = cfg->viscocity_kernel_norm;
  if (bid == 0u && threadIdx.x == 0u) *sl.longq_n = 0u;  // the density pass's appends are done
  f4* const tb = terms[wv];
  f2* const tv = reinterpret_cast<f2*>(terms[wv]);
  for (uint32_t k = bid * (kBlock / 64u) + wv;; k += nw) {
    const uint4 e = sl.longq[k];
    if (!e.x) break;  // past the last entry
    if (lane == 0u) sl.longq[k].x = 0u;  // cleared for the next active frame
    const uint32_t t = e.x - 1u;
    const f2 p = f2{__uint_as_float(e.y), __uint_as_float(e.z)};
    const uint2* tg = sl.longtab + (size_t)k * kLongTab;
    const RunRegs rr(tg);
    const uint32_t total = tg[9].y;
    const SimOwn o = sim_own(cfg, sl, t);
    const f4 own_pv = sl.rec_pv[t];
    if (kPads && !owner_is(sl, o.i, t)) continue;  // a repeat (wave-uniform)
    const uint32_t self = kPads ? o.i : t;
    // The entries of both scans: within the radius and not the particle itself (scan_runs);
    // kLongSub per lane in flight, entry f = f0 + 64 u + lane.  Both records of a chunk are
    // gathered together; the viscosity terms need the pressure sums, so a list longer than one
    // chunk gathers its velocity records again after the pressure scan.
    const bool one = total <= 64u * kLongSub;
    const auto gather = [&](uint32_t f0, const f4* rec, f4 (&q)[kLongSub], f4 (&qv)[kLongSub],
                            bool (&in)[kLongSub], bool both) {
      uint32_t j[kLongSub], qi[kLongSub];
#pragma unroll
      for (uint32_t u = 0; u < kLongSub; ++u) j[u] = rr.slot(min(f0 + 64u * u + lane, total - 1u));
#pragma unroll
      for (uint32_t u = 0; u < kLongSub; ++u) {
        q[u] = rec[j[u]];
        if (both) qv[u] = sl.rec_pv[j[u]];
        qi[u] = kPads ? sl.idx_s[j[u]] : j[u];
      }
#pragma unroll
      for (uint32_t u = 0; u < kLongSub; ++u) {
        const float dx = q[u][0] - p[0], dy = q[u][1] - p[1];
        in[u] = f0 + 64u * u + lane < total && qi[u] != self && !(dx * dx + dy * dy > r2);
      }
    };
    f4 qv[kLongSub];
    bool in1[kLongSub];
    float fx = 0.0f, fy = 0.0f;
    for (uint32_t f0 = 0; f0 < total && !(fx != fx && fy != fy); f0 += 64u * kLongSub) {
      f4 q[kLongSub];
      gather(f0, sl.rec_pd, q, qv, in1, one);
      uint32_t cnt = 0;
#pragma unroll
      for (uint32_t u = 0; u < kLongSub; ++u)
        cnt = long_compact(tb, cnt, in1[u], pressure_terms(q[u], p, o.P_rho2, o.Pn_rho2, r, dn, ndn));
      wave_lds_sync();
      f2 ff = f2{fx, fy};
      long_sum(tb, cnt, ff);
      fx = ff[0];
      fy = ff[1];
      wave_lds_sync();
    }
    const float qx = own_pv[2] + fx * dt;
    const float qy = own_pv[3] + fy * dt;
    float wx = 0.0f, wy = 0.0f;
    const auto visc = [&](const f4 (&q)[kLongSub], const bool (&in)[kLongSub]) {
      uint32_t cnt = 0;
#pragma unroll
      for (uint32_t u = 0; u < kLongSub; ++u) {
        const float kw = viscosity_weight(q[u], p, r, vn);
        cnt = long_compact(tv, cnt, in[u], f2{(q[u][2] - qx) * kw, (q[u][3] - qy) * kw});
      }
      wave_lds_sync();
      f2 ww = f2{wx, wy};
      long_sum(tv, cnt, ww);
      wx = ww[0];
      wy = ww[1];
      wave_lds_sync();
    };
    if (one) {
      visc(qv, in1);  // rec_pv's position is rec_pd's: the same entries pass the test
    } else {
      for (uint32_t f0 = 0; f0 < total && !(wx != wx && wy != wy); f0 += 64u * kLongSub) {
        f4 q[kLongSub];
        bool in[kLongSub];
        gather(f0, sl.rec_pv, q, qv, in, false);
        visc(q, in);
      }
    }
    if (lane == 0u) sim_finish<LAYOUT>(cfg, sl, st, bin_next, t, o.i, qx, qy, wx, wy);
  }
}

template <bool kPads, bool LAYOUT>
__global__ __launch_bounds__(kBlock) void sph_sim_long_kernel(const rps_config* __restrict__ cfg,
                                                              SphSlots sl, f4* __restrict__ st,
                                                              uint2* __restrict__ bin_next) {
  __shared__ LongTerms terms;
  sim_long_body<kPads, LAYOUT>(cfg, sl, st, bin_next, blockIdx.x, gridDim.x, terms);
}

// The sim pass in one launch with the long scans (P != N): blocks [0, nlong) take the queued
// slots (sim_long_body), the rest the slots in their lanes or lane pairs.  Neither part reads
// what the other writes (states of disjoint particles; records and densities of the passes
// before), so nothing orders them: the long slots' latency runs beside the main scans instead of
// after them, and the frame loses a launch.
template <int kScanBatch, bool kPads, bool LAYOUT, int G>
__global__ __launch_bounds__(kBlock) void sph_sim_fused_kernel(const rps_config* __restrict__ cfg,
                                                               RunBounds rb, SphSlots sl, f4* __restrict__ st,
                                                               uint2* __restrict__ bin_next, uint32_t p_slots,
                                                               uint32_t nlong) {
  __shared__ RunTable runs;
  if (blockIdx.x < nlong) {
    sim_long_body<kPads, LAYOUT>(cfg, sl, st, bin_next, blockIdx.x, nlong, reinterpret_cast<LongTerms&>(runs));
    return;
  }
  if constexpr (G > 1) sim2_body<kScanBatch, kPads, LAYOUT, G>(cfg, rb, sl, st, bin_next, p_slots, blockIdx.x - nlong, runs);
  else sim_body<kScanBatch, kPads, LAYOUT>(cfg, rb, sl, st, bin_next, p_slots, blockIdx.x - nlong, runs);
}

// predicted_positions / densities (wgsl:58, :61) rebuilt from the slot records for
// rps_read_debug: slot t holds particle idx_s[t]'s values (pads repeat identical ones).
__global__ __launch_bounds__(kBlock) void sph_debug_views_kernel(SphSlots sl, f2* __restrict__ pred,
                                                                 f2* __restrict__ dens,
                                                                 uint32_t p_slots) {
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= p_slots) return;
  const uint32_t i = sl.idx_s[t];
  if (sl.owner && !owner_is(sl, i, t)) return;  // repeats may have skipped the density pass
  pred[i] = sl.pp_s[t];
  dens[i] = sl.dens_s[t];
}

// Cost accounting for rps_sph_frame_cost (not on the frame path): per slot, the entries of
// its particle's nine runs (what the reference's density and sim scans visit,
// wgsl:207-254, :279-384) and how many of them lie within the radius.  One (scanned,
// within) u64 pair per workgroup, summed on the host; integer sums, so order-free.
// Slot-resident state (SphBuffers::bin_next): the bin entries from the state itself, with the
// current config (after rps_set_config), as the sim would have written them.
__global__ __launch_bounds__(kBlock) void sph_rebin_kernel(const rps_config* __restrict__ cfg,
                                                           const f4* __restrict__ st,
                                                           const uint32_t* __restrict__ perm,
                                                           uint2* __restrict__ bin_next, SphSlots sl,
                                                           uint32_t slots) {
  const uint32_t u = blockIdx.x * kBlock + threadIdx.x;
  if (u >= slots) return;
  if (sl.owner && !owner_is(sl, perm[u], u)) return;  // P != N: the state sits at owner slots
  const f4 s = st[u];
  const float r = cfg->smoothing_radius;
  const int32_t cx = f32_to_i32((s[0] + cfg->screen_bounds[1]) / r);
  const int32_t cy = f32_to_i32((s[1] + cfg->screen_bounds[3]) / r);
  bin_next[perm[u]] = make_uint2(cell_key(cx, cy, cfg->particle_count), u);
}
// The state back in particle order.
__global__ __launch_bounds__(kBlock) void sph_materialize_kernel(const f4* __restrict__ st,
                                                                 const uint32_t* __restrict__ perm,
                                                                 f4* __restrict__ dst, SphSlots sl,
                                                                 uint32_t slots) {
  const uint32_t u = blockIdx.x * kBlock + threadIdx.x;
  if (u < slots && (!sl.owner || owner_is(sl, perm[u], u))) dst[perm[u]] = st[u];
}
// Leaving slot-resident state: the lookup's payloads back to particle indices in place -- the
// slots [0, N) name through `perm` (null: already indices) and, with P != N, the pad entries'
// flagged indices -- so the lookup is the reference's spatial_lookup again and no later read
// needs the slot map (rps_read_debug after a download / export / upload).
__global__ __launch_bounds__(kBlock) void sph_lookup_canonical_kernel(uint2* lookup, const uint32_t* __restrict__ perm,
                                                                      uint32_t p) {
  const uint32_t k = blockIdx.x * kBlock + threadIdx.x;
  if (k >= p) return;
  const uint32_t y = lookup[k].y;
  lookup[k].y = (y & kPidFlag) ? y & ~kPidFlag : perm ? perm[y] : y;
}
// The sorted lookup with particle indices as payloads (the reference's spatial_lookup).
__global__ __launch_bounds__(kBlock) void sph_lookup_translate_kernel(const uint2* __restrict__ lookup,
                                                                      const uint32_t* __restrict__ perm,
                                                                      uint2* __restrict__ out, uint32_t p) {
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= p) return;
  const uint2 e = lookup[t];
  out[t] = make_uint2(e.x, (e.y & kPidFlag) ? e.y & ~kPidFlag : perm ? perm[e.y] : e.y);
}
__global__ __launch_bounds__(kBlock) void sph_count_kernel(const rps_config* __restrict__ cfg,
                                                           const uint32_t* __restrict__ offsets,
                                                           const uint32_t* __restrict__ ends,
                                                           const RunBounds rb, bool layout,
                                                           const f2* __restrict__ pp_s,
                                                           uint32_t p_slots,
                                                           unsigned long long* __restrict__ out) {
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  unsigned long long scanned = 0, within = 0;
  if (t < p_slots) {
    const f2 p = pp_s[t];
    const float r = cfg->smoothing_radius, r2 = r * r;
    const uint32_t N = cfg->particle_count;
    const int32_t cx = f32_to_i32((p[0] + cfg->screen_bounds[1]) / r);
    const int32_t cy = f32_to_i32((p[1] + cfg->screen_bounds[3]) / r);
    for (int o = 0; o < 9; ++o) {
      const uint32_t key = grid_key(cx, cy, o, N);
      const uint2 kr = layout ? key_run(rb.key_cell, rb.cellrun, rb.run2, rb.epoch, key)  // storage runs
                              : make_uint2(offsets[key], ends[key]);
      const uint32_t s0 = kr.x, e0 = kr.y;
      if (s0 >= N) continue;
      scanned += e0 - s0;
      for (uint32_t j = s0; j < e0; ++j) {
        const f2 q = pp_s[j];
        const float dx = p[0] - q[0], dy = p[1] - q[1];
        within += !((dx * dx + dy * dy) > r2);
      }
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    scanned += __shfl_xor(scanned, off, 64);
    within += __shfl_xor(within, off, 64);
  }
  __shared__ unsigned long long part[2][kBlock / 64];
  const uint32_t wave = threadIdx.x / 64;
  if ((threadIdx.x & 63u) == 0u) {
    part[0][wave] = scanned;
    part[1][wave] = within;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    unsigned long long v = 0;
    for (uint32_t w = 0; w < kBlock / 64; ++w) v += part[threadIdx.x][w];
    out[2ull * blockIdx.x + threadIdx.x] = v;
  }
}

// ---------------------------------------------------------------------------------------
// Spatial record layout (P == N; DESIGN.md §5 "Record layout").  The slot records are stored
// run by run in a spatial order of the cells instead of the sorted lookup's hash order: a
// key's run (its entries in lookup order) stays contiguous and in order, so every scan visits
// the same entries in the same order as the reference (bitwise), but the runs of neighbouring
// cells sit next to each other, and a cell-ordered table of storage runs (cellrun) replaces
// the scans' key-indexed (hash-random) run bounds:
//   runs kernel (slot order, in place of pass 3): at a run start, the run's length and the
//       cell of its first particle (its owner): cell_info[cell] = {first slot, length tagged
//       with the build's epoch (a stale record needs no reset pass), the first kRunIdx particle
//       indices}; runs whose first particle lies outside the grid (or
//       longer than kRunScan) go to a list (the reference's offsets are rebuilt on readback);
//   block counts (256 cells) and one-workgroup scan: block bases; listed runs after the grid's;
//   write (cell order): each owned run gets the next storage range -> cellrun[cell];
//       then pass 4's prediction for the block's storage range, in storage order; cells
//       owning no run are marked;
//   fixup (cell order): marked cells take their key's run (key_run: through the key's owner
//       recorded by the runs kernel; a key shared by several cells belongs to one of them).
// Cells are enumerated in 8 x 8 tiles (column by column inside a tile), tiles row-major over
// the screen's cell range.

// Exclusive prefix of v over a workgroup of NT threads; *total = the workgroup's sum.
template <uint32_t NT>
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* total) {
  __shared__ uint32_t wsum[NT / 64];
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= (uint32_t)d) x += y;
  }
  if (lane == 63u) wsum[wave] = x;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (uint32_t w = 0; w < NT / 64; ++w) {
    const uint32_t s = wsum[w];
    pre += w < wave ? s : 0u;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return pre + x - v;
}

// Each run's length and owner cell (the layout's replacement for pass 3: the scans find runs
// through cellrun / key_run, and the reference's offsets are rebuilt on debug readback).  Every
// run's last slot also records the run's end by key (run_end), so the scan kernel sizes a
// listed run with one load whatever its length.
__global__ __launch_bounds__(kBlock) void sph_runs_kernel(SphLayoutArgs a, const rps_config* __restrict__ cfg,
                                                          const uint2* __restrict__ lookup,
                                                          const f4* __restrict__ st, uint32_t n,
                                                          const uint2* __restrict__ bin_prev) {
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63u;
  const bool valid = t < n;  // every lane stays for the wave-wide ballots below
  const uint2 e = valid ? lookup[t] : make_uint2(0u, 0u);
  const uint32_t prev = valid && t > 0u ? lookup[t - 1u].x : 0xFFFFFFFFu;
  const uint32_t next = t + 1u < n ? lookup[t + 1u].x : ~e.x;
  if (valid && next != e.x) a.run_end[e.x] = t + 1u;
  const bool start = valid && e.x != prev;
  // The bitmap of keys with a run (the fixup looks a key up only where its bit is set: almost no
  // empty cell's key has a run).  Keys rise along the wave, so lanes sharing a 32-key word are adjacent: an
  // OR-scan within each word's segment, one atomicOr per word and wave.
  {
    const uint32_t word = valid ? e.x >> 5 : 0xFFFFFFFFu;
    uint32_t bits = start ? 1u << (e.x & 31u) : 0u;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint32_t ob = (uint32_t)__shfl_down((int)bits, d, 64);
      const uint32_t ow = (uint32_t)__shfl_down((int)word, d, 64);
      if (lane + d < 64u && ow == word) bits |= ob;
    }
    const uint32_t pw = (uint32_t)__shfl_up((int)word, 1, 64);
    if (valid && bits && (lane == 0u || pw != word)) atomicOr(&a.keybits[word], bits);
  }
  // Run lengths without a walk: a run starting in this wave ends at the wave's next run start
  // or, for the wave's last run, where the 64 slots after the wave first hold another key (one
  // coalesced load per lane; a run reaching past them is longer than kRunScan, so listed).
  const uint64_t starts = __builtin_amdgcn_ballot_w64(start);
  const uint32_t klast = (uint32_t)__builtin_amdgcn_readlane((int)e.x, 63);
  const uint32_t u = t + 64u;  // slot lane of the 64 after the wave
  const bool same = u < n && lookup[u].x == klast;
  const uint64_t other = __builtin_amdgcn_ballot_w64(!same);
  // The payloads of the kRunIdx - 1 slots after this one, from the lanes that loaded them.
  uint32_t nxt[kRunIdx];
#pragma unroll
  for (uint32_t k = 1; k < kRunIdx; ++k) nxt[k] = (uint32_t)__shfl_down((int)e.y, k, 64);
  if (!start) return;
  const uint64_t above = lane == 63u ? 0ull : starts >> (lane + 1u);
  const uint32_t len = above ? (uint32_t)__builtin_ctzll(above) + 1u
                             : min(64u - lane, n - t) + (other ? (uint32_t)__builtin_ctzll(other) : 64u);
  // The cell of the run's first particle, computed as the bin pass did (same state, same
  // ops), so its key is e.x; anything else (never seen) is handled as outside the grid.
  const f4 s = st[resolve_payload(e.y, nullptr, bin_prev).state];
  // The first kRunIdx particle indices (the write pass then needs no lookup gathers for
  // them): from the wave's lanes, loaded only past the wave's end.
  uint32_t idx[kRunIdx];
  idx[0] = e.y;
#pragma unroll
  for (uint32_t k = 1; k < kRunIdx; ++k) idx[k] = k >= len ? 0u : lane + k < 64u ? nxt[k] : lookup[t + k].y;
  const float r = cfg->smoothing_radius;
  const int32_t cx = f32_to_i32((s[0] + cfg->screen_bounds[1]) / r);
  const int32_t cy = f32_to_i32((s[1] + cfg->screen_bounds[3]) / r);
  const uint32_t c = cell_key(cx, cy, cfg->particle_count) == e.x ? grid_enum(a.g, cx, cy) : kCellOut;
  // The key's owner (keys rise along the wave: these stores share few lines), tagged with the
  // build's epoch, so no pass resets key_cell.
  const bool listed = c == kCellOut || len > kRunScan;
  a.key_cell[e.x] = make_uint2(listed ? kCellOut : c, a.epoch);
  if (listed) {
    a.out_runs[atomicAdd(a.n_out, 1u)] = make_uint2(t, 0u);  // placed by the scan kernel
  } else {
    a.cell_info[c] = make_uint4(t, len | a.epoch << 8, idx[0], idx[1]);
  }
}

// The length of the run cell e owns this frame (0: none; a record of another epoch is stale).
__device__ __forceinline__ uint32_t owned_len(const SphLayoutArgs& a, uint32_t v) {
  return v >> 8 == a.epoch ? v & 0xFFu : 0u;
}

// Run lengths owned by each 256-cell block.
__global__ __launch_bounds__(kBlock) void sph_layout_count_kernel(SphLayoutArgs a) {
  const uint32_t e = blockIdx.x * kBlock + threadIdx.x;
  const uint32_t len = owned_len(a, e < a.g.cells ? a.cell_info[e].y : 0u);
  uint32_t tot;
  block_exclusive_scan<kBlock>(len, &tot);
  if (threadIdx.x == 0) a.part[blockIdx.x] = tot;
}

// Block bases from the block sums (one workgroup), then the listed runs (first particle
// outside the grid, or longer than kRunScan) after the grid's, in list order: each one's
// length from run_end, its storage run (run2) and base (out_runs[j].y).  part[nparts] gets the
// grid's total, where the listed runs' storage starts; the write kernel predicts their slots.
__global__ __launch_bounds__(1024) void sph_layout_scan_kernel(SphLayoutArgs a,
                                                               const uint2* __restrict__ lookup,
                                                               uint32_t nparts) {
  const uint32_t m = *a.n_out;
  const uint32_t per = (nparts + 1023u) / 1024u, b0 = threadIdx.x * per;
  uint32_t sum = 0;
  for (uint32_t k = 0; k < per; ++k)
    if (b0 + k < nparts) sum += a.part[b0 + k];
  uint32_t total;
  uint32_t pre = block_exclusive_scan<1024>(sum, &total);
  for (uint32_t k = 0; k < per; ++k)
    if (b0 + k < nparts) {
      const uint32_t v = a.part[b0 + k];
      a.part[b0 + k] = pre;
      pre += v;
    }
  if (threadIdx.x == 0) a.part[nparts] = total;
  uint32_t base = total;
  for (uint32_t c = 0; c < m; c += 1024u) {
    const uint32_t j = c + threadIdx.x;
    uint32_t key = 0, t = 0, len = 0;
    if (j < m) {
      t = a.out_runs[j].x;
      key = lookup[t].x;
      len = a.run_end[key] - t;
    }
    uint32_t tot;
    const uint32_t p = base + block_exclusive_scan<1024>(len, &tot);
    if (j < m) {
      a.run2[key] = make_uint2(p, p + len);
      a.out_runs[j] = make_uint2(t, p);
    }
    base += tot;
  }
}

// Storage runs of a block of 256 cells, and pass 4's prediction (predict_slot) for the
// block's storage range [bases, bases + its run lengths) in storage order: lane k takes
// storage slots k, k + 256, ..., so every lane has the same work whatever the run lengths.
// The cell owning slot k comes from an LDS map the owners fill (slots < kSlotMap; beyond it,
// a binary search over the block's run bases), its particle index from the indices the runs
// kernel recorded (run entries < kRunIdx; beyond them, the lookup).
constexpr uint32_t kSlotMap = 2048;
__global__ __launch_bounds__(kBlock) void sph_layout_write_kernel(SphLayoutArgs a,
                                                                  const rps_config* __restrict__ cfg,
                                                                  uint2* __restrict__ lookup,
                                                                  const f4* __restrict__ st,
                                                                  const uint32_t* __restrict__ idx_prev,
                                                                  const uint2* __restrict__ bin_prev,
                                                                  SphSlots sl, uint32_t N, uint32_t p_slots) {
  __shared__ uint32_t lbase[kBlock], lsrc[kBlock], lidx[kRunIdx][kBlock];
  __shared__ uint8_t lcell[kSlotMap];
  const uint32_t e = blockIdx.x * kBlock + threadIdx.x;
  const bool in = e < a.g.cells;
  const uint4 i0 = in ? a.cell_info[e] : make_uint4(0u, 0u, 0u, 0u);
  const uint32_t len = owned_len(a, i0.y);
  const uint32_t b0 = a.part[blockIdx.x];
  uint32_t tot;
  const uint32_t rel = block_exclusive_scan<kBlock>(len, &tot);
  lbase[threadIdx.x] = rel;
  lsrc[threadIdx.x] = i0.x;
  lidx[0][threadIdx.x] = i0.z;
  lidx[1][threadIdx.x] = i0.w;
  for (uint32_t r = 0; r < len && rel + r < kSlotMap; ++r) lcell[rel + r] = (uint8_t)threadIdx.x;
  if (in) {
    if (len) {
      a.cellrun[e] = make_uint2(b0 + rel, b0 + rel + len);
    } else {
      a.cellrun[e] = make_uint2(kCellPending, 0u);
    }
  }
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < tot; k += kBlock) {
    uint32_t lo;
    if (k < kSlotMap) {
      lo = lcell[k];
    } else {  // the last cell whose base is <= k
      lo = 0;
#pragma unroll
      for (uint32_t step = kBlock / 2; step; step >>= 1)
        if (lbase[lo + step] <= k) lo += step;
    }
    const uint32_t r = k - lbase[lo];
    const uint32_t i = r < kRunIdx ? lidx[r][lo] : lookup[lsrc[lo] + r].y;
    predict_slot(cfg, st, sl, b0 + k, i, idx_prev, bin_prev);
  }
  // The listed runs' slots [part[blocks], N), spread over every thread of the launch (one slot
  // per thread at most once the launch covers N: a clump of many particles in one run costs
  // no lane more than its share); the run of slot k by binary search over their bases.
  const uint32_t m = *a.n_out;
  const uint32_t stride = gridDim.x * kBlock;
  for (uint32_t k = a.part[gridDim.x] + blockIdx.x * kBlock + threadIdx.x; k < N; k += stride) {
    uint32_t lo = 0, hi = m;  // the last listed run whose base is <= k
    while (hi - lo > 1u) {
      const uint32_t mid = (lo + hi) >> 1;
      if (a.out_runs[mid].y <= k) lo = mid;
      else hi = mid;
    }
    const uint2 run = a.out_runs[lo];
    predict_slot(cfg, st, sl, k, lookup[run.x + (k - run.y)].y, idx_prev, bin_prev);
  }
  // P != N: the pad slots [N, P) (never scanned) keep lookup order after the
  // layout's N storage slots; the density and sim passes compute only those that own their
  // particle (one pushed out of [0, N) by stale entries).  These entries are the next frame's
  // stale pads: their payloads become particle indices (kPidFlag), since the slots they name
  // are this frame's (resolve_payload).
  for (uint32_t k = N + blockIdx.x * kBlock + threadIdx.x; k < p_slots; k += stride)
    lookup[k].y = kPidFlag | predict_slot(cfg, st, sl, k, lookup[k].y, idx_prev, bin_prev);
}

// Cells owning no run take their key's storage run (key_run; the owners' cellrun entries are
// complete after the write pass).
// The listed-run count goes back to 0 for the next frame's runs kernel.
__global__ __launch_bounds__(kBlock) void sph_layout_fixup_kernel(SphLayoutArgs a, uint32_t N) {
  const uint32_t c = blockIdx.x * kBlock + threadIdx.x;
  if (c == 0u) *a.n_out = 0u;
  if (c >= a.g.cells) return;
  if (a.cellrun[c].x == kCellPending) {
    int32_t cx, cy;
    grid_cell(a.g, c, cx, cy);
    const uint32_t k = cell_key(cx, cy, N);
    a.cellrun[c] = (a.keybits[k >> 5] >> (k & 31u)) & 1u ? key_run(a.key_cell, a.cellrun, a.run2, a.epoch, k)
                                                         : make_uint2(0xFFFFFFFFu, 0u);
  }
}

inline uint32_t blocks_for(uint64_t n, uint32_t per_block = kBlock) {
  return (uint32_t)((n + per_block - 1) / per_block);
}

}  // namespace

// ---------------------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------------------
// The AQL dispatch packet counts work-items in 32 bits, so grids are capped at 2^31
// work-items (kMaxGridBlocks x 256); kernels that can exceed it loop grid-stride.
constexpr uint64_t kMaxGridBlocks = 1ull << 23;

uint32_t stream_blocks_for(uint64_t n) {
  const uint64_t nvec = n >> 2;
  uint64_t b = (nvec + kBlock - 1) / kBlock;
  if (b == 0) b = 1;
  return (uint32_t)(b > kMaxGridBlocks ? kMaxGridBlocks : b);
}

template <bool V, bool L, bool S, int NTM>
static hipError_t launch_stream_t(const StreamArgs& a, uint32_t grid, hipStream_t s) {
  // An LDS reservation that is never used caps the occupancy at 6 workgroups per CU (6
  // waves/SIMD; 163 840 / 25 000 = 6.55).  The kernels at <= 64 VGPRs (no lifetime, no stats)
  // otherwise run 8 waves/SIMD, and 8 is slower than 6 on the stream (same box, 1e8,
  // tools/ab_stream.py, AB_LIFE=0): 8 waves 0.5051 ms, 7 0.5004, 6 0.4767, 5 0.4766, 4
  // 0.4854.  The C3 kernel (71 VGPRs, 7 waves) is unchanged at 6 (0.4923 vs 0.4924) and
  // slower at 5 (0.5050) and 4 (0.5358); the stats steps (83-91 VGPRs) run 5 either way.
  constexpr uint32_t kStreamLds = 25000;
  hipLaunchKernelGGL((stream_step_kernel<V, L, S, NTM>), dim3(grid), dim3(kBlock), kStreamLds, s, a);
  return hipGetLastError();
}

// Cache policy (stream_nt_default, rps_context.hip): nontemporal stores always; nontemporal
// loads (3) or temporal loads (2, states of 48-576 MiB, which the Infinity Cache partly serves).
template <bool V, bool L, bool S>
static hipError_t launch_stream_nt(const StreamArgs& a, const StreamLaunch& l, hipStream_t s) {
  if (l.nontemporal == 2) return launch_stream_t<V, L, S, 2>(a, l.grid, s);
  return launch_stream_t<V, L, S, 3>(a, l.grid, s);
}

hipError_t launch_stream_step(const StreamArgs& a, const StreamLaunch& l, hipStream_t s) {
  const int sel = (l.verlet ? 4 : 0) | (l.lifetime ? 2 : 0) | (l.stats ? 1 : 0);
  switch (sel) {
    case 0: return launch_stream_nt<false, false, false>(a, l, s);
    case 1: return launch_stream_nt<false, false, true>(a, l, s);
    case 2: return launch_stream_nt<false, true, false>(a, l, s);
    case 3: return launch_stream_nt<false, true, true>(a, l, s);
    case 4: return launch_stream_nt<true, false, false>(a, l, s);
    case 5: return launch_stream_nt<true, false, true>(a, l, s);
    case 6: return launch_stream_nt<true, true, false>(a, l, s);
    default: return launch_stream_nt<true, true, true>(a, l, s);
  }
}

template <bool V, bool L, bool S, int NTM>
static hipError_t launch_fused_t(const FusedArgs& a, uint32_t grid, hipStream_t s) {
  hipLaunchKernelGGL((stream_fused_kernel<V, L, S, NTM>), dim3(grid), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

// Fused variants are built for the NT-load+store policy only (the measured best, §5).
hipError_t launch_stream_fused(const FusedArgs& a, const StreamLaunch& l, hipStream_t s) {
  const int sel = (l.verlet ? 4 : 0) | (l.lifetime ? 2 : 0) | (l.stats ? 1 : 0);
  switch (sel) {
    case 0: return launch_fused_t<false, false, false, 3>(a, l.grid, s);
    case 1: return launch_fused_t<false, false, true, 3>(a, l.grid, s);
    case 2: return launch_fused_t<false, true, false, 3>(a, l.grid, s);
    case 3: return launch_fused_t<false, true, true, 3>(a, l.grid, s);
    case 4: return launch_fused_t<true, false, false, 3>(a, l.grid, s);
    case 5: return launch_fused_t<true, false, true, 3>(a, l.grid, s);
    case 6: return launch_fused_t<true, true, false, 3>(a, l.grid, s);
    default: return launch_fused_t<true, true, true, 3>(a, l.grid, s);
  }
}

hipError_t launch_stats_finalize(const StatsPartial* partials, uint32_t count,
                                 StatsPartial* scratch, StatsResult* out, StatsGlobal* global,
                                 uint64_t step, hipStream_t s) {
  if (count > kStatsFold) {
    const uint32_t chunk = (count + kStatsFold - 1) / kStatsFold;
    const uint32_t blocks = (count + chunk - 1) / chunk;
    hipLaunchKernelGGL(stats_fold_kernel, dim3(blocks), dim3(kBlock), 0, s, partials, count, chunk,
                       scratch);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    partials = scratch;
    count = blocks;
  }
  hipLaunchKernelGGL(stats_finalize_kernel, dim3(1), dim3(kBlock), 0, s, partials, count, out,
                     global, (unsigned long long)step);
  return hipGetLastError();
}

hipError_t launch_aos_to_soa(const rps_particle* aos, Fields f, Layout L, uint64_t offset,
                             uint64_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(aos_to_soa_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, s, aos, f, L, offset, n);
  return hipGetLastError();
}

hipError_t launch_config_store(const rps_config& cfg, rps_config* dst, hipStream_t s) {
  ConfigStoreArgs a;
  a.cfg = cfg;
  a.dst = dst;
  hipLaunchKernelGGL(config_store_kernel, dim3(1), dim3(64), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_soa_to_aos(Fields f, Layout L, uint64_t offset, rps_particle* aos, uint64_t n,
                             float max_energy, int spawn_colour, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(soa_to_aos_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, s, f, L, offset, aos,
                     n, max_energy, spawn_colour);
  return hipGetLastError();
}

hipError_t launch_field_gather(const float* field, Layout L, uint64_t offset, float* out,
                               uint64_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(field_gather_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, s, field, L, offset,
                     out, n);
  return hipGetLastError();
}

hipError_t launch_life_gather(const uint16_t* exp, Layout L, uint64_t offset, float* out,
                              uint64_t n, uint32_t clock, float dt, int mode, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(life_gather_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, s, exp, L, offset,
                     out, n, clock, dt, mode);
  return hipGetLastError();
}

hipError_t launch_life_scatter(uint16_t* exp, Layout L, uint64_t offset, const float* in,
                               uint64_t n, uint32_t clock, float dt, int mode, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(life_scatter_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, s, exp, L, offset,
                     in, n, clock, dt, mode);
  return hipGetLastError();
}

hipError_t launch_field_scatter(float* field, Layout L, uint64_t offset, const float* in,
                                uint64_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(field_scatter_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, s, field, L,
                     offset, in, n);
  return hipGetLastError();
}

hipError_t launch_next_rebuild(const uint16_t* exp, uint16_t* next, uint64_t first, uint64_t n,
                               uint64_t total, uint32_t clock, hipStream_t s) {
  // the groups overlapping particles [first, first + n) that hold a full quad of a shard of
  // `total` particles
  const uint64_t nquads = total >> 2;
  const uint64_t g0 = first >> kGroupLog;
  const uint64_t g1 = std::min((first + n + kGroup - 1) >> kGroupLog, (nquads * 4 + kGroup - 1) >> kGroupLog);
  if (n == 0 || g1 <= g0) return hipSuccess;
  hipLaunchKernelGGL(next_rebuild_kernel, dim3(blocks_for(g1 - g0)), dim3(kBlock), 0, s, exp, next, g0,
                     g1, nquads, clock);
  return hipGetLastError();
}

hipError_t launch_init_scatter(const InitArgs& a, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  const uint64_t b = (a.n + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(init_scatter_kernel, dim3((uint32_t)(b > kMaxGridBlocks ? kMaxGridBlocks : b)),
                     dim3(kBlock), 0, s, a);
  return hipGetLastError();
}



// Launch K global passes of one stage starting at stride G (flip = it is the stage's first).
template <int K>
static hipError_t launch_sort_fused(uint2* lookup, uint32_t P, uint32_t G, bool flip, hipStream_t s) {
  const uint32_t g = G >> (K - 1);
  const uint32_t threads = (P / (2u * G)) * (flip ? g / 2u : g);
  if (flip)
    hipLaunchKernelGGL((sph_sort_fused_kernel<K, true>), dim3(blocks_for(threads)), dim3(kBlock), 0, s,
                       lookup, P, G);
  else
    hipLaunchKernelGGL((sph_sort_fused_kernel<K, false>), dim3(blocks_for(threads)), dim3(kBlock), 0, s,
                       lookup, P, G);
  return hipGetLastError();
}

// Bin + the whole network of a lookup below 2048 entries (one tile of P entries, LDS passes in
// register chunks of two).
static hipError_t launch_sort_small(uint32_t threads, hipStream_t s, uint2* lookup, uint32_t tile,
                                    uint32_t hi, const SortBin& sb) {
  hipLaunchKernelGGL((sph_sort_local_kernel<true, 2>), dim3(1), dim3(threads), 0, s, lookup, tile, 0u, hi, 0u, sb,
                     tile >= 2u ? 1u : 0u);
  return hipGetLastError();
}

// Tile of the compact sort at P entries (2^11 .. 2^16): RPS_SPH_CSORT_TLOG, else by size.
static uint32_t csort_tlog(uint32_t stages, uint32_t forced) {
  uint32_t tl = forced ? forced : (stages <= 13u ? stages : 12u);
  return std::max(11u, std::min(std::min(tl, 13u), stages));
}

// The compact sort (see sph_csort_head_kernel): head + one launch per later stage.
static hipError_t launch_sph_csort(const SphBuffers& b, const SortBin& bin, uint32_t stages, hipStream_t s,
                                   uint32_t* launches) {
  const uint32_t P = b.p;
  const uint32_t tl = csort_tlog(stages, b.csort_tlog);
  const uint32_t tiles = P >> tl, nt = (1u << tl) / 8u;
  uint32_t* const cb[2] = {reinterpret_cast<uint32_t*>(b.sl.nbr_mask),  // dead during the sort
                           reinterpret_cast<uint32_t*>(b.sl.nbr_mask) + P};
  const bool one = stages == tl;
#define RPS_CHEAD(TL)                                                                                         \
  if (one) hipLaunchKernelGGL((sph_csort_head_kernel<TL, true>), dim3(tiles), dim3(nt), 0, s, b.lookup, bin, cb[0]); \
  else hipLaunchKernelGGL((sph_csort_head_kernel<TL, false>), dim3(tiles), dim3(nt), 0, s, b.lookup, bin, cb[0])
  switch (tl) {
    case 11: RPS_CHEAD(11); break;
    case 12: RPS_CHEAD(12); break;
    default: RPS_CHEAD(13); break;
  }
#undef RPS_CHEAD
  hipError_t e = hipGetLastError();
  ++*launches;
  if (e != hipSuccess) return e;
  for (uint32_t stage = tl, k = 0; stage < stages; ++stage, ++k) {
    const uint32_t tg = stage - tl + 1u;
    const bool last = stage + 1u == stages;
    const bool wide = b.csort_wide && tl <= 12u && tg >= b.csort_wide;  // the wide fold pays from 4 folded passes on
    const uint32_t* src = cb[k & 1u];
    uint32_t* dst = cb[(k + 1u) & 1u];
#define RPS_CSTAGE(TL, TG)                                                                                        \
  case TG:                                                                                                        \
    if (wide && last) hipLaunchKernelGGL((sph_csort_stage_kernel<TL, TG, true, (TL <= 12)>), dim3(tiles), dim3(2u * nt), 0, s, src, dst, b.lookup); \
    else if (wide) hipLaunchKernelGGL((sph_csort_stage_kernel<TL, TG, false, (TL <= 12)>), dim3(tiles), dim3(2u * nt), 0, s, src, dst, b.lookup); \
    else if (last) hipLaunchKernelGGL((sph_csort_stage_kernel<TL, TG, true>), dim3(tiles), dim3(nt), 0, s, src, dst, b.lookup); \
    else hipLaunchKernelGGL((sph_csort_stage_kernel<TL, TG, false>), dim3(tiles), dim3(nt), 0, s, src, dst, b.lookup); \
    break
    switch (tl) {
      case 11:
        switch (tg) { RPS_CSTAGE(11, 1); RPS_CSTAGE(11, 2); RPS_CSTAGE(11, 3); RPS_CSTAGE(11, 4); RPS_CSTAGE(11, 5);
          default: return hipErrorInvalidValue; }
        break;
      case 12:
        switch (tg) { RPS_CSTAGE(12, 1); RPS_CSTAGE(12, 2); RPS_CSTAGE(12, 3); RPS_CSTAGE(12, 4);
          default: return hipErrorInvalidValue; }
        break;
      default:
        switch (tg) { RPS_CSTAGE(13, 1); RPS_CSTAGE(13, 2); RPS_CSTAGE(13, 3);
          default: return hipErrorInvalidValue; }
    }
#undef RPS_CSTAGE
    e = hipGetLastError();
    ++*launches;
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// Whether this frame's sort runs compact: 2^11 <= P <= 2^16 and every lookup payload below 2^16.
// Only a resident frame with P != N holds flagged payloads (the pad entries the previous layout
// frame wrote).  Every path that leaves the resident state (a non-layout frame, and
// every particle-order API call: particle and field uploads and downloads, export,
// init_scatter) runs sph_canonical, which unflags them, and sph_frame_begin fails a frame that finds
// slot-resident payloads outside a resident frame (tests/test_gpu_sph.py
// test_sph_init_scatter_leaves_resident_state, test_sph_resident_state_api).
static bool csort_ok(const SphBuffers& b) {
  return b.csort && b.p >= 2048u && b.p <= 65536u && !(b.resident && b.p != b.n);
}

// Passes 1-2 of the frame: bin (folded into the first sort launch) + the bitonic network.
hipError_t launch_sph_sort(const SphBuffers& b, hipStream_t s, uint32_t* passes,
                           uint32_t* launches) {
  const uint32_t P = b.p;
  uint32_t stages = 0;
  while ((1u << stages) < P) ++stages;
  *passes = stages * (stages + 1u) / 2u;
  *launches = 0;
  // Slot-resident state: the previous layout frame's sim wrote the bin entries (key, slot).
  // Without the layout, the previous active frame's sim wrote (key, i) for the current state and
  // config (SphBuffers::pkeys): the head reads them instead of keying the positions.
  const SortBin bin{b.cfg, b.st, b.offsets, b.n, b.resident || b.pkeys ? b.bin_next : nullptr,
                    !b.resident && b.pkeys};
  if (csort_ok(b)) return launch_sph_csort(b, bin, stages, s, launches);
  if (stages == 0) {  // P == 1: nothing to sort, only bin
    hipLaunchKernelGGL((sph_sort_local_kernel<true, 1>), dim3(1), dim3(64), 0, s, b.lookup, 1u, 1u, 0u,
                       0u, bin, 0u);
    ++*launches;
    return hipGetLastError();
  }
  // Tile: P / 256 entries clamped to [2048, 8192] -- one workgroup per CU in the LDS passes
  // once P allows it, and the largest such tile (fewest global passes).  Measured per size
  // (DESIGN.md §5): 2048 up to P = 2^19, 4096 at 2^20, 8192 from 2^21.  A fixed 8192 above
  // 2^18 left half the CUs idle at 2^20 (0.429 -> 0.404 ms/frame) and 2^19 (0.294 -> 0.265).
  const uint32_t tile = std::min(P, std::min(kSortTile, std::max(2048u, P / 256u)));
  uint32_t tile_log = 0;
  while ((1u << tile_log) < tile) ++tile_log;
  const uint32_t tiles = P / tile;
  // Stages whose whole network fits one tile: one launch (with the bin pass).
  const uint32_t first_global_stage = tile_log;  // stage s has 2*2^s = 2^(s+1) span
  const uint32_t lt = std::max(64u, tile >> 2);  // P < 2048: two passes per register chunk
  hipError_t e = hipSuccess;
  switch (tile_log) {  // bin + stages [0, tile_log): the static-network head launch
    case 13: hipLaunchKernelGGL((sph_sort_head_kernel<13>), dim3(tiles), dim3(1024), 0, s, b.lookup, bin); break;
    case 12: hipLaunchKernelGGL((sph_sort_head_kernel<12>), dim3(tiles), dim3(512), 0, s, b.lookup, bin); break;
    case 11: hipLaunchKernelGGL((sph_sort_head_kernel<11>), dim3(tiles), dim3(256), 0, s, b.lookup, bin); break;
    default:  // P < 2048: one tile of P entries
      e = launch_sort_small(lt, s, b.lookup, tile, first_global_stage - 1u, bin);
      if (e != hipSuccess) return e;
  }
  e = hipGetLastError();
  ++*launches;
  if (e != hipSuccess) return e;
  // The first two later stages (one and two global passes) fold those passes into their tail
  // launches, which then read one buffer and write the other (the neighbour masks' buffer,
  // dead during the sort): lookup -> scratch -> lookup.  Tiles up to 4096 entries (same box,
  // ms/frame: 50 000 0.1433 -> 0.1408, 65 536 0.0996 -> 0.0971, 10^6 0.4284 -> 0.4157; with
  // 8192-entry tiles at 2^22 0.9239 -> 0.9255, not kept).  RPS_SPH_SORT_FOLD=0 runs them as
  // register-fused launches.
  const bool fold = b.sort_fold && tile_log <= 12u && stages >= first_global_stage + 2u;
  uint2* const scratch = reinterpret_cast<uint2*>(b.sl.nbr_mask);
  for (uint32_t stage = first_global_stage; stage < stages; ++stage) {
    // Passes whose compare span 2*gw exceeds the tile are global: steps [0, T).  Up to four
    // of them run as one register-fused launch (sph_sort_fused_kernel); three or five per
    // launch were slower.
    uint32_t T = 0;
    while (T <= stage && 2u * (1u << (stage - T)) > tile) ++T;
    uint32_t step = 0;
    if (fold && T <= 2u) {  // T == stage - first_global_stage + 1
      uint2* dst = T == 1u ? scratch : b.lookup;
      const uint2* src = T == 1u ? b.lookup : scratch;
#define RPS_TAIL_FOLD(TL, NTH)                                                                          \
  if (T == 1u) hipLaunchKernelGGL((sph_sort_tail_kernel<TL, 1>), dim3(tiles), dim3(NTH), 0, s, dst, src); \
  else hipLaunchKernelGGL((sph_sort_tail_kernel<TL, 2>), dim3(tiles), dim3(NTH), 0, s, dst, src)
      switch (tile_log) {
        case 13: RPS_TAIL_FOLD(13, 1024); break;
        case 12: RPS_TAIL_FOLD(12, 512); break;
        case 11: RPS_TAIL_FOLD(11, 256); break;
        default: return hipErrorInvalidValue;
      }
#undef RPS_TAIL_FOLD
      e = hipGetLastError();
      ++*launches;
      if (e != hipSuccess) return e;
      continue;
    }
    // Stages with five to nine global passes run them all in one gathered-tile launch
    // (sph_sort_gather_kernel; at T = 5 and 2^22 it also beats the 32-entry register-fused
    // launch, 16.3 us: frame -4.5 us).
    if (step < T && T >= 5u && T <= 9u && tile_log >= 6u) {
      // Residue groups of 16 (whole 128-B lines); eight entries per thread, sixteen at T = 9.
      const uint32_t blocks = (P >> (stage + 1u)) << (tile_log - 5u);
      const uint32_t threads = T == 9u ? 1024u : (32u << T) / 8u;
      switch (T) {
        case 5: hipLaunchKernelGGL((sph_sort_gather_kernel<5, 4, 3>), dim3(blocks), dim3(threads), 0, s, b.lookup, stage, tile_log); break;
        case 6: hipLaunchKernelGGL((sph_sort_gather_kernel<6, 4, 3>), dim3(blocks), dim3(threads), 0, s, b.lookup, stage, tile_log); break;
        case 7: hipLaunchKernelGGL((sph_sort_gather_kernel<7, 4, 3>), dim3(blocks), dim3(threads), 0, s, b.lookup, stage, tile_log); break;
        case 8: hipLaunchKernelGGL((sph_sort_gather_kernel<8, 4, 3>), dim3(blocks), dim3(threads), 0, s, b.lookup, stage, tile_log); break;
        default: hipLaunchKernelGGL((sph_sort_gather_kernel<9, 4, 4>), dim3(blocks), dim3(threads), 0, s, b.lookup, stage, tile_log); break;
      }
      e = hipGetLastError();
      ++*launches;
      if (e != hipSuccess) return e;
      step = T;
    }
    while (step < T) {
      const uint32_t k = T - step < 4u ? T - step : 4u;
      const uint32_t G = 1u << (stage - step);
      const bool flip = step == 0;
      switch (k) {
        case 1: e = launch_sort_fused<1>(b.lookup, P, G, flip, s); break;
        case 2: e = launch_sort_fused<2>(b.lookup, P, G, flip, s); break;
        case 3: e = launch_sort_fused<3>(b.lookup, P, G, flip, s); break;
        default: e = launch_sort_fused<4>(b.lookup, P, G, flip, s); break;
      }
      ++*launches;
      if (e != hipSuccess) return e;
      step += k;
    }
    if (step <= stage) {  // the stage's passes inside each tile: strides tile/2 .. 1
      switch (tile_log) {
        case 13: hipLaunchKernelGGL((sph_sort_tail_kernel<13>), dim3(tiles), dim3(1024), 0, s, b.lookup, b.lookup); break;
        case 12: hipLaunchKernelGGL((sph_sort_tail_kernel<12>), dim3(tiles), dim3(512), 0, s, b.lookup, b.lookup); break;
        case 11: hipLaunchKernelGGL((sph_sort_tail_kernel<11>), dim3(tiles), dim3(256), 0, s, b.lookup, b.lookup); break;
        default: return hipErrorInvalidValue;  // later stages exist only with 2048..8192-entry tiles
      }
      e = hipGetLastError();
      ++*launches;
      if (e != hipSuccess) return e;
    }
  }
  return hipSuccess;
}

hipError_t launch_sph_offsets(const SphBuffers& b, hipStream_t s) {
  hipLaunchKernelGGL(sph_offsets_kernel, dim3(blocks_for(b.n)), dim3(kBlock), 0, s, b.lookup,
                     b.offsets, b.ends, b.n);
  return hipGetLastError();
}

// Entries in flight per lane in the density and sim scans, unless the context forces one
// (SphBuffers::batch_d / batch_s, from RPS_SPH_BATCH[_D|_S] at rps_create): by size, measured
// (DESIGN.md §5).
int sph_batch(bool density, uint32_t p, int forced, bool layout) {
  if (forced == 4 || forced == 6 || forced == 8 || forced == 16) return forced;
  // With the spatial record layout the sim's gathers hit the caches: 4 at 2^22 too (1.1251 ->
  // 1.1018 ms/frame; 8: 1.1607), as below 2^21.
  if (!density && layout) return 4;
  // The sim scan keeps 4 entries in flight up to P = 2^21, where its slot records stay in
  // the caches (2^20 frame 0.404 -> 0.392 ms, 2^21 0.670 -> 0.651), and 6 beyond (2^22: 1.2223
  // ms with 8, 1.2129 with 6 -- 91 VGPRs, 5 waves/SIMD instead of 111 and 4 --, 1.28 with 4,
  // 1.2989 with 12).  The density scan is indifferent (4 or 8 within 0.3 %) and keeps 8.
  if (density) return 8;
  return p > (1u << 21) ? 6 : 4;
}

static RunBounds run_bounds(const SphBuffers& b) {
  return RunBounds{b.offsets, b.ends, b.lay.cellrun, b.lay.run2, b.lay.key_cell, b.lay.epoch, b.lay.g,
                   b.lay.keybits};
}

// Workgroups of the long-scan kernels (4 waves each, a wave per queued slot in turn).
static uint32_t long_blocks(uint32_t p) { return std::min<uint32_t>(blocks_for(p), 512u); }

static hipError_t launch_sph_density(const SphBuffers& b, hipStream_t s) {
  const RunBounds rb = run_bounds(b);
  if (b.p <= b.pair_max_p) {  // lane groups (sph_density2_kernel)
#define RPS_DENSITY2(B, G)                                                                              \
  if (b.layout)                                                                                         \
    hipLaunchKernelGGL((sph_density2_kernel<B, true, G>), dim3(blocks_for(G * b.p)), dim3(kBlock), 0, s, \
                       b.cfg, rb, b.sl, b.p);                                                            \
  else                                                                                                  \
    hipLaunchKernelGGL((sph_density2_kernel<B, false, G>), dim3(blocks_for(G * b.p)), dim3(kBlock), 0, s, \
                       b.cfg, rb, b.sl, b.p)
    if (b.lane_group == 4) {
      if (b.batch_d == 4) { RPS_DENSITY2(4, 4); } else { RPS_DENSITY2(2, 4); }
    } else {
      if (b.batch_d == 8) { RPS_DENSITY2(8, 2); } else { RPS_DENSITY2(4, 2); }
    }
#undef RPS_DENSITY2
  } else {
#define RPS_DENSITY(B)                                                                            \
  if (b.layout)                                                                                   \
    hipLaunchKernelGGL((sph_density_kernel<B, true>), dim3(blocks_for(b.p)), dim3(kBlock), 0, s, \
                       b.cfg, rb, b.sl, b.p);                                               \
  else                                                                                            \
    hipLaunchKernelGGL((sph_density_kernel<B, false>), dim3(blocks_for(b.p)), dim3(kBlock), 0, s, \
                       b.cfg, rb, b.sl, b.p)
    switch (sph_batch(true, b.p, b.batch_d, b.layout)) {
      case 4: RPS_DENSITY(4); break;
      case 16: RPS_DENSITY(16); break;
      default: RPS_DENSITY(8); break;
    }
#undef RPS_DENSITY
  }
  if (b.sl.longq) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(sph_density_long_kernel, dim3(long_blocks(b.p)), dim3(kBlock), 0, s, b.cfg, b.sl, b.p);
  }
  return hipGetLastError();
}

hipError_t launch_sph_pre(const SphBuffers& b, hipStream_t s) {
  // Owners are claimed by the predict pass of active frames only (with the frame's epoch), so
  // after gated frames they still describe the slot records (rps_read_debug's views).
  hipLaunchKernelGGL(sph_predict_kernel, dim3(blocks_for(b.p)), dim3(kBlock), 0, s, b.cfg, b.lookup, b.st,
                     b.sl, b.p, b.offsets, b.ends, b.n);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_sph_density(b, s);
}

bool sph_layout_grid(const rps_config& c, uint32_t cell_cap, SphGrid* g) {
  if (cell_cap == 0) return false;
  const float r = c.smoothing_radius;
  // The cells of positions inside the walls, as the bin pass computes them (+1 cell margin).
  const double x0 = std::floor(((double)c.screen_bounds[0] + c.screen_bounds[1]) / r) - 1.0;
  const double x1 = std::floor(((double)c.screen_bounds[1] + c.screen_bounds[1]) / r) + 1.0;
  const double y0 = std::floor(((double)c.screen_bounds[2] + c.screen_bounds[3]) / r) - 1.0;
  const double y1 = std::floor(((double)c.screen_bounds[3] + c.screen_bounds[3]) / r) + 1.0;
  if (!(x1 >= x0) || !(y1 >= y0) || x0 < -2.0e9 || y0 < -2.0e9 || x1 > 2.0e9 || y1 > 2.0e9) return false;
  const double w = x1 - x0 + 1.0, h = y1 - y0 + 1.0;
  const double tsx = (double)(1u << kCX), tsy = (double)(1u << kCY);
  const double tw = std::ceil(w / tsx), th = std::ceil(h / tsy);
  if (tw * th * tsx * tsy > (double)cell_cap) return false;
  g->cx_lo = (int32_t)x0;
  g->cy_lo = (int32_t)y0;
  g->w = (uint32_t)w;
  g->h = (uint32_t)h;
  g->tw = (uint32_t)tw;
  g->cells = (uint32_t)(tw * th * tsx * tsy);
  return true;
}

hipError_t launch_sph_layout_pre(const SphBuffers& b, hipStream_t s) {
  const SphLayoutArgs& a = b.lay;
  const uint2* bin_prev = b.resident ? b.bin_next : nullptr;  // flagged pad payloads (resolve_payload)
  hipLaunchKernelGGL(sph_runs_kernel, dim3(blocks_for(b.n)), dim3(kBlock), 0, s, a, b.cfg, b.lookup, b.st, b.n,
                     bin_prev);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const uint32_t nparts = blocks_for(a.g.cells);
  hipLaunchKernelGGL(sph_layout_count_kernel, dim3(nparts), dim3(kBlock), 0, s, a);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(sph_layout_scan_kernel, dim3(1), dim3(1024), 0, s, a, b.lookup, nparts);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(sph_layout_write_kernel, dim3(nparts), dim3(kBlock), 0, s, a, b.cfg, b.lookup, b.st,
                     b.resident ? b.idx_prev : nullptr, bin_prev, b.sl, b.n, b.p);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(sph_layout_fixup_kernel, dim3(nparts), dim3(kBlock), 0, s, a, b.n);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  return launch_sph_density(b, s);
}

hipError_t launch_sph_sim(const SphBuffers& b, hipStream_t s) {
  const RunBounds rb = run_bounds(b);
  if (b.sl.longq && b.sim_fuse) {  // P != N: the long scans in the same launch (sph_sim_fused_kernel)
    const uint32_t nlong = long_blocks(b.p);
    const bool pairs = b.p <= b.pair_max_p;
    const uint32_t G = b.lane_group_s == 4 ? 4u : 2u;
    const dim3 g(nlong + (pairs ? blocks_for(G * b.p) : blocks_for(b.p)));
#define RPS_SIMF(B, PR)                                                                                          \
  if (b.layout)                                                                                                  \
    hipLaunchKernelGGL((sph_sim_fused_kernel<B, true, true, PR>), g, dim3(kBlock), 0, s, b.cfg, rb, b.sl, b.st,    \
                       b.bin_next, b.p, nlong);                                                                  \
  else                                                                                                           \
    hipLaunchKernelGGL((sph_sim_fused_kernel<B, true, false, PR>), g, dim3(kBlock), 0, s, b.cfg, rb, b.sl, b.st,   \
                       b.bin_next, b.p, nlong)
    if (pairs && G == 4) {
      // two entries in flight per lane (50 000 0.0750 -> 0.0740 ms/frame, 20 000 0.0507 -> 0.0500)
      if (b.batch_s == 1) { RPS_SIMF(1, 4); } else { RPS_SIMF(2, 4); }
    } else if (pairs) {
      if (b.batch_s == 4) { RPS_SIMF(4, 2); } else { RPS_SIMF(2, 2); }
    } else {
      switch (sph_batch(false, b.p, b.batch_s, b.layout)) {
        case 4: RPS_SIMF(4, 1); break;
        case 6: RPS_SIMF(6, 1); break;
        case 16: RPS_SIMF(16, 1); break;
        default: RPS_SIMF(8, 1); break;
      }
    }
#undef RPS_SIMF
    return hipGetLastError();
  }
#define RPS_SIM(B)                                                                                  \
  if (b.layout && b.p == b.n)                                                                       \
    hipLaunchKernelGGL((sph_sim_kernel<B, false, true>), dim3(blocks_for(b.p)), dim3(kBlock), 0, s, \
                       b.cfg, rb, b.sl, b.st, b.bin_next, b.p);                                           \
  else if (b.layout)                                                                                \
    hipLaunchKernelGGL((sph_sim_kernel<B, true, true>), dim3(blocks_for(b.p)), dim3(kBlock), 0, s, \
                       b.cfg, rb, b.sl, b.st, b.bin_next, b.p);                                           \
  else if (b.p == b.n)                                                                              \
    hipLaunchKernelGGL((sph_sim_kernel<B, false, false>), dim3(blocks_for(b.p)), dim3(kBlock), 0, s, \
                       b.cfg, rb, b.sl, b.st, b.bin_next, b.p);                                           \
  else                                                                                              \
    hipLaunchKernelGGL((sph_sim_kernel<B, true, false>), dim3(blocks_for(b.p)), dim3(kBlock), 0, s, \
                       b.cfg, rb, b.sl, b.st, b.bin_next, b.p)
  if (b.p <= b.pair_max_p) {  // lane groups (sph_sim2_kernel)
#define RPS_SIM2(B, G)                                                                                       \
  {                                                                                                          \
    const dim3 g2(blocks_for(G * b.p));                                                                      \
    if (b.layout && b.p == b.n)                                                                              \
      hipLaunchKernelGGL((sph_sim2_kernel<B, false, true, G>), g2, dim3(kBlock), 0, s, b.cfg, rb, b.sl, b.st, b.bin_next, b.p); \
    else if (b.layout)                                                                                       \
      hipLaunchKernelGGL((sph_sim2_kernel<B, true, true, G>), g2, dim3(kBlock), 0, s, b.cfg, rb, b.sl, b.st, b.bin_next, b.p);  \
    else if (b.p == b.n)                                                                                     \
      hipLaunchKernelGGL((sph_sim2_kernel<B, false, false, G>), g2, dim3(kBlock), 0, s, b.cfg, rb, b.sl, b.st, b.bin_next, b.p); \
    else                                                                                                     \
      hipLaunchKernelGGL((sph_sim2_kernel<B, true, false, G>), g2, dim3(kBlock), 0, s, b.cfg, rb, b.sl, b.st, b.bin_next, b.p); \
  }
    if (b.lane_group_s == 4) {
      if (b.batch_s == 1) { RPS_SIM2(1, 4); } else { RPS_SIM2(2, 4); }
    } else {
      if (b.batch_s == 4) { RPS_SIM2(4, 2); } else { RPS_SIM2(2, 2); }
    }
#undef RPS_SIM2
  } else {
    switch (sph_batch(false, b.p, b.batch_s, b.layout)) {
      case 4: RPS_SIM(4); break;
      case 6: RPS_SIM(6); break;
      case 16: RPS_SIM(16); break;
      default: RPS_SIM(8); break;
    }
  }
#undef RPS_SIM
  if (b.sl.longq) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const dim3 g(long_blocks(b.p));
    if (b.layout)  // long scans exist only with P != N
      hipLaunchKernelGGL((sph_sim_long_kernel<true, true>), g, dim3(kBlock), 0, s, b.cfg, b.sl, b.st, b.bin_next);
    else if (b.p == b.n)
      hipLaunchKernelGGL((sph_sim_long_kernel<false, false>), g, dim3(kBlock), 0, s, b.cfg, b.sl, b.st, b.bin_next);
    else
      hipLaunchKernelGGL((sph_sim_long_kernel<true, false>), g, dim3(kBlock), 0, s, b.cfg, b.sl, b.st, b.bin_next);
  }
  return hipGetLastError();
}

uint32_t sph_count_blocks(uint32_t p_slots) { return blocks_for(p_slots); }

hipError_t launch_sph_count(const SphBuffers& b, unsigned long long* out, hipStream_t s) {
  hipLaunchKernelGGL(sph_count_kernel, dim3(blocks_for(b.p)), dim3(kBlock), 0, s, b.cfg,
                     b.offsets, b.ends, run_bounds(b), b.layout, b.sl.pp_s, b.p, out);
  return hipGetLastError();
}

hipError_t launch_sph_rebin(const SphBuffers& b, const uint32_t* perm, hipStream_t s) {
  hipLaunchKernelGGL(sph_rebin_kernel, dim3(blocks_for(b.p)), dim3(kBlock), 0, s, b.cfg, b.st, perm, b.bin_next,
                     b.sl, b.sl.owner ? b.p : b.n);
  return hipGetLastError();
}
hipError_t launch_sph_materialize(const SphBuffers& b, const f4* st, const uint32_t* perm, f4* dst, hipStream_t s) {
  const uint32_t slots = b.sl.owner ? b.p : b.n;
  hipLaunchKernelGGL(sph_materialize_kernel, dim3(blocks_for(slots)), dim3(kBlock), 0, s, st, perm, dst, b.sl, slots);
  return hipGetLastError();
}
hipError_t launch_sph_lookup_canonical(const SphBuffers& b, const uint32_t* perm, hipStream_t s) {
  if (b.p == b.n && !perm) return hipSuccess;
  hipLaunchKernelGGL(sph_lookup_canonical_kernel, dim3(blocks_for(b.p)), dim3(kBlock), 0, s, b.lookup, perm, b.p);
  return hipGetLastError();
}
hipError_t launch_sph_lookup_translate(const uint2* lookup, const uint32_t* perm, uint2* out, uint32_t p,
                                       hipStream_t s) {
  hipLaunchKernelGGL(sph_lookup_translate_kernel, dim3(blocks_for(p)), dim3(kBlock), 0, s, lookup, perm, out, p);
  return hipGetLastError();
}
hipError_t launch_sph_debug_views(const SphBuffers& b, hipStream_t s) {
  hipLaunchKernelGGL(sph_debug_views_kernel, dim3(blocks_for(b.p)), dim3(kBlock), 0, s, b.sl,
                     b.pred, b.dens, b.p);
  return hipGetLastError();
}

}  // namespace rps
