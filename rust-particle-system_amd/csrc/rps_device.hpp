// rps_device.hpp — per-particle device math for gfx950.
//
// Every function here computes, operation for operation, what assets/compute_shader.wgsl
// (or the build-defined extension spec in DESIGN.md §3.2) prescribes.  The whole library is
// compiled with -ffp-contract=off and without fast-math, so each a*b+c is two IEEE
// roundings and division/sqrt are correctly rounded: results are bit-identical to the CPU
// restatement in oracle/ (which is only a test-side checker; nothing here links it).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rps {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int kMaxAttractors = 8;

// Correctly rounded sqrt for x == 0, x >= 2^-96, +inf and NaN (payload aside): the
// compiler's IEEE sequence without its input scaling for tiny x.  v_sqrt_f32 is within
// 1 ulp; the two FMA residual tests pick the correctly rounded neighbour exactly as that
// sequence does.  Callers take sqrtf for 0 < x < 2^-96 (tools/sqrt_check.hip compares this
// with sqrtf over every non-negative float on the GPU).
__device__ __forceinline__ float sqrt_rn_unscaled(float x) {
  const float s = __builtin_amdgcn_sqrtf(x);
  const float sdn = __int_as_float(__float_as_int(s) - 1);
  const float sup = __int_as_float(__float_as_int(s) + 1);
  float t = (__builtin_fmaf(-sdn, s, x) <= 0.0f) ? sdn : s;
  t = (__builtin_fmaf(-sup, s, x) > 0.0f) ? sup : t;
  return t;
}

// sqrtf's bits with the unscaled sequence unless a lane of the wave has 0 < x < 2^-96 (two
// particles closer than ~1e-14: only ever near the origin); call it where the whole wave (or
// the lanes a ballot should see) is active.
__device__ __forceinline__ float sqrt_rn_wave(float x) {
  const bool tiny = x > 0.0f && x < 0x1p-96f;
  return __builtin_amdgcn_ballot_w64(tiny) ? sqrtf(x) : sqrt_rn_unscaled(x);
}

// Particle-state layout in HBM.  STREAM mode keeps the state as *tiled SoA*
// (AoSoA): tiles of kTile particles, each tile holding four contiguous f32 segments
// [x | y | vx | vy] (128 KiB).  Lanes read 16 contiguous bytes of each field; a workgroup's
// streams fall in one tile instead of arrays gigabytes apart (tools/hbm_probe.hip: 6.35-6.6
// TB/s tiled vs 5.3 TB/s plain SoA on the in-place update).  The u16 lifetime expiries and
// the [next] index (one u16 per group of 64 particles: the group's earliest expiry, so a
// step reads the expiries only in the group-steps where one of them is due) are plain arrays
// of their own: inside the tiles they stretched the f32 tile stride from 128 to 148 KiB, and
// the C3 step ran 3.2 % slower (0.5112 -> 0.4949 ms, same box).  SPH and N-body keep plain SoA.
constexpr uint32_t kTileLog = 13;
constexpr uint64_t kTile = 1ull << kTileLog;
constexpr uint64_t kTileBytes = kTile * 16;  // 4 x f32 per particle (the u16 expiry and [next]
                                             // are arrays of their own)

// Element offset of particle i inside one field: (((i & ~mask) * mult) >> shift) + (i & mask).
// plain: mask = ~0 (offset i).  Tiled f32 fields: the tile stride is 4 * kTile floats
// (mult 32, shift 3).  The expiry and [next] arrays are plain.
struct Layout {
  uint64_t mask;
  uint64_t mult;
  uint32_t shift;
};
__host__ __device__ __forceinline__ uint64_t lidx(Layout L, uint64_t i) {
  return (((i & ~L.mask) * L.mult) >> L.shift) + (i & L.mask);
}
__host__ __device__ __forceinline__ Layout plain_layout() { return Layout{~0ull, 1, 0}; }
__host__ __device__ __forceinline__ Layout tiled_layout() { return Layout{kTile - 1, 32, 3}; }
__host__ __device__ __forceinline__ Layout tiled_exp_layout() { return plain_layout(); }
// Tiled offsets with compile-time constants (the stream kernel's address math).
__device__ __forceinline__ uint64_t tidx(uint64_t i) {
  return ((i & ~(kTile - 1)) << 2) + (i & (kTile - 1));
}
__device__ __forceinline__ uint64_t eidx(uint64_t i) { return i; }
// [next] holds one entry per group of kGroup particles (16 quads: the 16 lanes of a DPP row),
// so a step reads 2 B per 64 particles of it.  A group's expiries are 128 B, one cache line,
// and the lines of due groups are the ones that move either way: per-quad entries (0.5 B per
// particle) bought nothing over this but their own traffic.
constexpr uint32_t kGroupLog = 6;
constexpr uint64_t kGroup = 1ull << kGroupLog;
// [next] entry of the group holding particle i.
__host__ __device__ __forceinline__ uint64_t nidx(uint64_t i) { return i >> kGroupLog; }
// Earliest expiry of a quad as seen at lifetime clock c: the expiry e with the smallest
// (u16)(e - c), i.e. the next step in which one of the four respawns.
__host__ __device__ __forceinline__ uint16_t quad_next(uint16_t e0, uint16_t e1, uint16_t e2,
                                                       uint16_t e3, uint16_t c) {
  uint16_t best = e0;
  if ((uint16_t)(e1 - c) < (uint16_t)(best - c)) best = e1;
  if ((uint16_t)(e2 - c) < (uint16_t)(best - c)) best = e2;
  if ((uint16_t)(e3 - c) < (uint16_t)(best - c)) best = e3;
  return best;
}

// Base pointers of the fields; for the tiled layout f32 field f starts at tile-0 offset
// f * kTile floats; the expiry array is plain.
struct Fields {
  float* x;
  float* y;
  float* vx;
  float* vy;
  uint16_t* exp;  // lifetime expiry (STREAM only; may be null)
};

// Lifetime in whole steps: a lifetime of L seconds lasts
// clamp(ceil(L / dt), 1, 65535) active lifetime steps.  f32 division, correctly rounded on
// both sides (oracle: orc_life_steps).
__host__ __device__ __forceinline__ uint32_t life_steps(float life, float dt) {
  const float q = ceilf(life / dt);
  if (!(q >= 1.0f)) return 1u;
  if (q >= 65535.0f) return 65535u;
  return (uint32_t)q;
}

// Per-step uniforms of the streaming kernel.  Passed by value: the kernarg segment lands in
// SGPRs through s_load, so the 4-8 attractors cost no LDS and no VGPRs.
struct StreamArgs {
  float* __restrict__ x;
  float* __restrict__ y;
  float* __restrict__ vx;
  float* __restrict__ vy;
  uint16_t* __restrict__ exp;   // lifetime expiry, tiled u16 (eidx)
  uint16_t* __restrict__ next;  // per quad: its earliest expiry (nidx, quad_next)
  struct StatsPartial* partials;  // one per workgroup when stats are on
  uint64_t n;                     // particles in this shard
  uint64_t id_offset;             // global id of particle 0
  float dt, gx_dt, gy_dt, neg_g, half_dt, half_dt2, drag_f;
  uint32_t drag_on;
  uint32_t na;
  // Attractors of this step {x, y, strength, softening^2}.  Kernels read them through the
  // kernarg segment pointer with a uniform loop index (s_load_dwordx4 per attractor), so
  // they neither occupy ~32 SGPRs for the whole kernel nor get indexed through scratch.
  f4 att[kMaxAttractors];
  float x_min, x_max, y_min, y_max, damping;
  float emit_cx, emit_cy, emit_r, spd_min, spd_range, life_min, life_range;
  uint32_t key0, key1, step_lo, step_hi;
  uint32_t clock;      // lifetime clock of this step (low 16 bits compared with the expiry)
};

// Temporal fusion of up to kMaxFuse consecutive active steps in one launch: per-substep
// attractor positions (the only per-step uniforms besides the Philox step counter).
constexpr int kMaxFuse = 16;
struct FusedArgs {
  StreamArgs base;  // step_lo/step_hi = first substep's active-step index
  uint32_t nsub;
  f4 att[kMaxFuse][kMaxAttractors];  // per-substep attractors (base.att unused)
};

struct StatsPartial {  // 48 B, written once per workgroup, reduced in fixed order
  float bbox[4];
  double ke;
  unsigned long long count;
  unsigned long long respawned;
  unsigned long long _pad;
};

struct StatsResult {
  float bbox[4];
  double ke;
  unsigned long long count;
  unsigned long long respawned;
  unsigned long long step;
};

// A shard's stats in the form two in-place ncclAllReduce calls combine over the ranks
// (DESIGN.md §8): MAX over {-x_min, x_max, -y_min, y_max}, SUM over {KE, particles,
// respawns} (counts are exact in f64 below 2^53).
struct StatsGlobal {
  float neg_min_max[4];
  double sums[3];
};

// ---------------------------------------------------------------------------------------
// Random123 Philox4x32-10 (build-defined respawn stream, keyed by (seed, global id, step)).
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                              uint32_t k0, uint32_t k1, uint32_t out[4]) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r > 0) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    // One 32x32->64 product per word (v_mad_u64_u32: both halves from one quarter-rate op,
    // where mul_lo + mul_hi take two).
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
    const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
    const uint32_t n0 = hi1 ^ c1 ^ k0;
    const uint32_t n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
  }
  out[0] = c0;
  out[1] = c1;
  out[2] = c2;
  out[3] = c3;
}

__device__ __forceinline__ float u01(uint32_t w) {
  return (float)(w >> 8) * (1.0f / 16777216.0f);
}

// sin/cos(2*pi*u): quadrant split + fixed-order Taylor polynomials.
__device__ __forceinline__ void sincos_turns(float u, float& c_out, float& s_out) {
  const float u4 = u * 4.0f;
  const int q = (int)u4;
  const float f = u4 - (float)q;
  const float th = f * 1.57079632679489662f;
  const float t2 = th * th;
  float sp = -2.50521083854417188e-08f;
  sp = sp * t2 + 2.75573192239858907e-06f;
  sp = sp * t2 + -1.98412698412698413e-04f;
  sp = sp * t2 + 8.33333333333333333e-03f;
  sp = sp * t2 + -1.66666666666666667e-01f;
  const float s = th + (th * t2) * sp;
  float cp = 2.08767569878680990e-09f;
  cp = cp * t2 + -2.75573192239858907e-07f;
  cp = cp * t2 + 2.48015873015873016e-05f;
  cp = cp * t2 + -1.38888888888888889e-03f;
  cp = cp * t2 + 4.16666666666666667e-02f;
  cp = cp * t2 + -0.5f;
  const float c = 1.0f + t2 * cp;
  switch (q & 3) {
    case 0: c_out = c; s_out = s; break;
    case 1: c_out = -s; s_out = c; break;
    case 2: c_out = -c; s_out = -s; break;
    default: c_out = s; s_out = -c; break;
  }
}

// ln(u) for u in (0, 1] (normal): exponent split by bit operations, then the atanh series
// ln m = 2 s (1 + s^2/3 + ... + s^14/15), s = (m - 1)/(m + 1), m in [sqrt(1/2), sqrt(2)).
// Only exact bit operations and fixed-order correctly rounded +, *, / -- bit for bit the
// oracle's orc_log_unit; within 2 ulp of logf.
__device__ __forceinline__ float log_unit(float u) {
  const uint32_t b = __float_as_uint(u);
  int e = (int)((b >> 23) & 255u) - 127;
  float m = __uint_as_float((b & 0x007fffffu) | 0x3f800000u);
  if (m > 1.41421356f) {
    m = m * 0.5f;
    e = e + 1;
  }
  const float s = (m - 1.0f) / (m + 1.0f);
  const float s2 = s * s;
  float p = 6.66666666666666667e-02f;  // 1/15
  p = p * s2 + 7.69230769230769231e-02f;  // 1/13
  p = p * s2 + 9.09090909090909091e-02f;  // 1/11
  p = p * s2 + 1.11111111111111111e-01f;  // 1/9
  p = p * s2 + 1.42857142857142857e-01f;  // 1/7
  p = p * s2 + 2.00000000000000000e-01f;  // 1/5
  p = p * s2 + 3.33333333333333333e-01f;  // 1/3
  const float t = s + s;
  const float lnm = t + t * (s2 * p);
  const float ef = (float)e;
  return ef * 6.93145751953125e-01f + (ef * 1.42860682030941723e-06f + lnm);
}

// ---------------------------------------------------------------------------------------
// Reference helpers
// ---------------------------------------------------------------------------------------

// check_screen_bounds, compute_shader.wgsl:69-99.
__device__ __forceinline__ void wall(float x_min, float x_max, float y_min, float y_max,
                                     float damp, float& x, float& y, float& vx, float& vy) {
  if (x <= x_min) {
    x = x_min;
    vx = fabsf(vx) * damp;
  } else if (x >= x_max) {
    x = x_max;
    vx = -fabsf(vx) * damp;
  }
  if (y <= y_min) {
    y = y_min;
    vy = fabsf(vy) * damp;
  } else if (y >= y_max) {
    y = y_max;
    vy = -fabsf(vy) * damp;
  }
}

// set_color, compute_shader.wgsl:101-118.
__device__ __forceinline__ f4 set_color(float vx, float vy, float max_energy) {
  const float speed_sq = vx * vx + vy * vy;
  const float energy = 0.5f * speed_sq;
  float nrm = energy / max_energy;
  nrm = nrm < 0.0f ? 0.0f : nrm;
  nrm = nrm > 1.0f ? 1.0f : nrm;
  // rgb = mix(a, b, t) = a * (1 - t) + b * t per component, as WGSL defines it (no constant
  // folding: -fno-fast-math keeps 0 * t, so a NaN velocity colours NaN in every component, as
  // the shader does; for finite t the literal form has the bits of t / 1 - t / 0).
  const bool lo = nrm < 0.5f;
  const float t = lo ? nrm * 2.0f : (nrm - 0.5f) * 2.0f;
  const float a0 = 0.0f, a1 = lo ? 0.0f : 1.0f, a2 = lo ? 1.0f : 0.0f;  // blue -> green / green -> red
  const float b0 = lo ? 0.0f : 1.0f, b1 = lo ? 1.0f : 0.0f, b2 = 0.0f;
  const float u = 1.0f - t;
  return f4{a0 * u + b0 * t, a1 * u + b1 * t, a2 * u + b2 * t, 1.0f};
}

// hash_cell + get_key_from_hash, compute_shader.wgsl:132-142 (u32 wrap).
__device__ __forceinline__ uint32_t cell_key(int32_t cx, int32_t cy, uint32_t n) {
  const uint32_t a = (uint32_t)cx * 15823u;
  const uint32_t b = (uint32_t)cy * 9737333u;
  return (a + b) % n;
}

// WGSL i32(f32): truncate toward zero, saturate, NaN -> 0.
__device__ __forceinline__ int32_t f32_to_i32(float v) {
  if (v != v) return 0;
  if (v >= 2147483520.0f) return 2147483647;
  if (v <= -2147483648.0f) return (int32_t)0x80000000u;
  return (int32_t)v;
}

// 1/sqrt(r2) as specified in DESIGN.md §3.2: the bit-level initial guess 0x5f375a86 -
// (bits(r2) >> 1) and three Newton steps y = y * (1.5 - (h * y) * y), h = 0.5 * r2, every
// step a separately rounded IEEE f32 op (about 2 ulp from the true value).  Cheap on the
// VALU (v_pk_mul/add on particle pairs, no v_sqrt/v_div sequences) and exactly the same
// bits as the CPU oracle's orc_inv_sqrt.  Two particles at a time (f2 lanes).
typedef uint32_t u2 __attribute__((ext_vector_type(2)));
// Uniform attractor table in the kernarg (constant) address space: loads are s_load.
typedef __attribute__((address_space(4))) const f4* att_ptr;
__device__ __forceinline__ f2 inv_sqrt_nr(f2 r2) {
  const u2 b = __builtin_bit_cast(u2, r2);
  f2 y = __builtin_bit_cast(f2, u2{0x5f375a86u, 0x5f375a86u} - (b >> 1u));
  const f2 h = 0.5f * r2;
#pragma unroll
  for (int it = 0; it < 3; ++it) {
    f2 t = h * y;
    t = t * y;
    t = 1.5f - t;
    y = y * t;
  }
  return y;
}

// Sum of attractor accelerations at two particles (x, y), attractors in index order
// (DESIGN.md §3.2).  att: this step's {x, y, strength, softening^2} (uniform, kernarg).
// NP pairs at once: their serial Newton chains interleave, so dependent v_pk_* ops of one
// pair issue between those of the other instead of behind s_nop hazard padding.
template <int NP>
__device__ __forceinline__ void attract2(att_ptr att, uint32_t na, const f2 (&x)[NP],
                                         const f2 (&y)[NP], f2 (&ax)[NP], f2 (&ay)[NP]) {
  f2 sx[NP], sy[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) sx[p] = sy[p] = f2{0.0f, 0.0f};
  for (uint32_t k = 0; k < na; ++k) {
    const f4 A = att[k];
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const f2 dx = A[0] - x[p];
      const f2 dy = A[1] - y[p];
      const f2 r2 = (dx * dx + dy * dy) + A[3];
      const f2 inv = inv_sqrt_nr(r2);
      const f2 s = A[2] * ((inv * inv) * inv);
      sx[p] = sx[p] + dx * s;
      sy[p] = sy[p] + dy * s;
    }
  }
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    ax[p] = sx[p];
    ay[p] = sy[p];
  }
}

// Respawn at the emitter; returns the new lifetime in steps.
__device__ __forceinline__ uint32_t respawn(const StreamArgs& a, uint64_t step, uint64_t gid,
                                            float& x, float& y, float& vx, float& vy) {
  uint32_t w[4];
  philox4x32_10((uint32_t)gid, (uint32_t)(gid >> 32), (uint32_t)step, (uint32_t)(step >> 32), a.key0,
                a.key1, w);
  const float r = a.emit_r * sqrtf(u01(w[0]));
  float c, s;
  sincos_turns(u01(w[1]), c, s);
  x = a.emit_cx + r * c;
  y = a.emit_cy + r * s;
  const float spd = a.spd_min + u01(w[3]) * a.spd_range;
  vx = spd * c;
  vy = spd * s;
  return life_steps(a.life_min + u01(w[2]) * a.life_range, a.dt);
}

// Two particles, one active step (the kernels' unit: every op on the pair is one v_pk_*
// where the ISA has it), in two parts: step_pair_motion (forces, integration, walls) and
// step_pair_life (lifetime expiry and respawn, after the walls).  The kernels run the motion
// of all their pairs before the lifetime part, so a quad's expiries -- loaded only when one
// is due -- are needed last and their load overlaps the motion arithmetic.
template <bool VERLET, int NP>
__device__ __forceinline__ void step_pair_motion(const StreamArgs& a, att_ptr att, f2 (&x)[NP],
                                                 f2 (&y)[NP], f2 (&vx)[NP], f2 (&vy)[NP]) {
  const float dt = a.dt;
  if constexpr (!VERLET) {
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      vx[p] = vx[p] + a.gx_dt;  // apply_gravity, wgsl:397-400
      vy[p] = vy[p] + a.gy_dt;
    }
    if (a.na) {
      f2 ax[NP], ay[NP];
      attract2<NP>(att, a.na, x, y, ax, ay);
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        vx[p] = vx[p] + ax[p] * dt;
        vy[p] = vy[p] + ay[p] * dt;
      }
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      if (a.drag_on) {
        vx[p] = vx[p] * a.drag_f;
        vy[p] = vy[p] * a.drag_f;
      }
      x[p] = x[p] + vx[p] * dt;  // update_particle_positions, wgsl:392-395
      y[p] = y[p] + vy[p] * dt;
    }
  } else {
    f2 ax0[NP], ay0[NP], ax1[NP], ay1[NP], x1[NP], y1[NP];
    attract2<NP>(att, a.na, x, y, ax0, ay0);
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      ay0[p] = ay0[p] + a.neg_g;
      x1[p] = (x[p] + vx[p] * dt) + ax0[p] * a.half_dt2;
      y1[p] = (y[p] + vy[p] * dt) + ay0[p] * a.half_dt2;
    }
    attract2<NP>(att, a.na, x1, y1, ax1, ay1);
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      ay1[p] = ay1[p] + a.neg_g;
      vx[p] = vx[p] + (ax0[p] + ax1[p]) * a.half_dt;
      vy[p] = vy[p] + (ay0[p] + ay1[p]) * a.half_dt;
      if (a.drag_on) {
        vx[p] = vx[p] * a.drag_f;
        vy[p] = vy[p] * a.drag_f;
      }
      x[p] = x1[p];
      y[p] = y1[p];
    }
  }
#pragma unroll
  for (int p = 0; p < NP; ++p) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float px = x[p][i], py = y[p][i], qx = vx[p][i], qy = vy[p][i];
      wall(a.x_min, a.x_max, a.y_min, a.y_max, a.damping, px, py, qx, qy);
      x[p][i] = px;
      y[p][i] = py;
      vx[p][i] = qx;
      vy[p][i] = qy;
    }
  }
}

// The lifetime part of the step for two particles.  gid: global id of element 0 (element 1
// is gid + 1); step: the active-step index (Philox counter); clock: the step's lifetime-clock
// value; e[i]: expiries (the clock value of the step in which each particle respawns, mod
// 2^16).  Writes re[i] = element i respawned.  With `single`, element 1 duplicates element 0
// and only element 0's lifetime is advanced (n % 4 tails).
template <bool LIFETIME>
__device__ __forceinline__ void step_pair_life(const StreamArgs& a, uint64_t step, uint32_t clock,
                                               uint64_t gid, f2& x, f2& y, f2& vx, f2& vy,
                                               uint16_t e[2], bool re[2], bool single = false) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    re[i] = false;
    if constexpr (LIFETIME) {
      if ((i == 0 || !single) && e[i] == (uint16_t)clock) {
        float px, py, qx, qy;
        e[i] = (uint16_t)(clock + respawn(a, step, gid + i, px, py, qx, qy));
        x[i] = px;
        y[i] = py;
        vx[i] = qx;
        vy[i] = qy;
        re[i] = true;
      }
    }
  }
}

}  // namespace rps
