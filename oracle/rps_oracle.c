/*
 * rps_oracle.c — CPU restatement of assets/compute_shader.wgsl (+ build-defined extensions).
 *
 * TEST INFRASTRUCTURE ONLY (see rps_oracle.h).  PARITY UNPINNED at the WGSL-execution
 * boundary: no runnable reference and no reference golden vectors exist.
 *
 * Build: oracle/Makefile, always with -ffp-contract=off so every a*b+c below is two
 * roundings, exactly as the HIP kernels (also built with -ffp-contract=off) compute it.
 */
#include "rps_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ----------------------------------------------------------------------------------- */
/* RNG + deterministic trig (build-defined; no reference counterpart)                   */
/* ----------------------------------------------------------------------------------- */

/* Random123 Philox4x32-10 (Salmon et al., SC'11): 10 rounds, key bumped between rounds. */
void orc_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
  uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
  uint32_t k0 = key_in[0], k1 = key_in[1];
  for (int r = 0; r < 10; ++r) {
    if (r > 0) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0;
    uint32_t n2 = hi0 ^ c3 ^ k1;
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

static inline float u01(uint32_t w) { return (float)(w >> 8) * (1.0f / 16777216.0f); }

/* sin/cos of 2*pi*u by quadrant split + odd/even Taylor polynomials on [0, pi/2).  Only
 * exact scalings and fixed-order +,* — so the HIP kernel reproduces it bit for bit. */
void orc_sincos_turns(float u, float* c_out, float* s_out) {
  float u4 = u * 4.0f;
  int q = (int)u4;
  float f = u4 - (float)q;
  float th = f * 1.57079632679489662f;
  float t2 = th * th;
  float sp = -2.50521083854417188e-08f;            /* -1/11! */
  sp = sp * t2 + 2.75573192239858907e-06f;         /*  1/9!  */
  sp = sp * t2 + -1.98412698412698413e-04f;        /* -1/7!  */
  sp = sp * t2 + 8.33333333333333333e-03f;         /*  1/5!  */
  sp = sp * t2 + -1.66666666666666667e-01f;        /* -1/3!  */
  float s = th + (th * t2) * sp;
  float cp = 2.08767569878680990e-09f;             /*  1/12! */
  cp = cp * t2 + -2.75573192239858907e-07f;        /* -1/10! */
  cp = cp * t2 + 2.48015873015873016e-05f;         /*  1/8!  */
  cp = cp * t2 + -1.38888888888888889e-03f;        /* -1/6!  */
  cp = cp * t2 + 4.16666666666666667e-02f;         /*  1/4!  */
  cp = cp * t2 + -0.5f;                            /* -1/2!  */
  float c = 1.0f + t2 * cp;
  switch (q & 3) {
    case 0: *c_out = c; *s_out = s; break;
    case 1: *c_out = -s; *s_out = c; break;
    case 2: *c_out = -c; *s_out = -s; break;
    default: *c_out = s; *s_out = -c; break;
  }
}

/* ln(u) for normal u in (0, 1]: exponent split by bit operations, then the atanh series
 * ln m = 2s(1 + s^2/3 + ... + s^14/15), s = (m-1)/(m+1), m in [sqrt(1/2), sqrt(2)).  Exact
 * bit operations and fixed-order +, *, / only, so the HIP kernel (log_unit) reproduces it bit
 * for bit where glibc logf and the device logf differ in the last bit. */
float orc_log_unit(float u) {
  uint32_t b;
  memcpy(&b, &u, 4);
  int e = (int)((b >> 23) & 255u) - 127;
  uint32_t mb = (b & 0x007fffffu) | 0x3f800000u;
  float m;
  memcpy(&m, &mb, 4);
  if (m > 1.41421356f) {
    m = m * 0.5f;
    e = e + 1;
  }
  float s = (m - 1.0f) / (m + 1.0f);
  float s2 = s * s;
  float p = 6.66666666666666667e-02f;     /* 1/15 */
  p = p * s2 + 7.69230769230769231e-02f;  /* 1/13 */
  p = p * s2 + 9.09090909090909091e-02f;  /* 1/11 */
  p = p * s2 + 1.11111111111111111e-01f;  /* 1/9  */
  p = p * s2 + 1.42857142857142857e-01f;  /* 1/7  */
  p = p * s2 + 2.00000000000000000e-01f;  /* 1/5  */
  p = p * s2 + 3.33333333333333333e-01f;  /* 1/3  */
  float t = s + s;
  float lnm = t + t * (s2 * p);
  float ef = (float)e;
  return ef * 6.93145751953125e-01f + (ef * 1.42860682030941723e-06f + lnm);
}

void orc_attractor_pos(const rps_attractor* a, double t, float* px, float* py) {
  double ang = (double)a->angular_velocity * t + (double)a->phase;
  *px = (float)((double)a->center[0] + (double)a->orbit_radius * cos(ang));
  *py = (float)((double)a->center[1] + (double)a->orbit_radius * sin(ang));
}

/* ----------------------------------------------------------------------------------- */
/* Reference helpers                                                                     */
/* ----------------------------------------------------------------------------------- */

/* compute_shader.wgsl:101-118.  mix(e1,e2,t) with the constant blue/green/red endpoints
 * gives the same bits whether evaluated as e1*(1-t)+e2*t or e1+t*(e2-e1). */
void orc_set_color(float vx, float vy, float max_energy, float rgba[4]) {
  float speed_sq = vx * vx + vy * vy;
  float energy = 0.5f * speed_sq;
  float nrm = energy / max_energy;
  nrm = nrm < 0.0f ? 0.0f : nrm; /* clamp(x, 0, 1) = min(max(x, 0), 1) */
  nrm = nrm > 1.0f ? 1.0f : nrm;
  /* mix(a, b, t) = a * (1 - t) + b * t per component (WGSL's definition, computed: a NaN t
   * makes every component NaN, 0 * NaN included). */
  static const float A[2][3] = {{0.0f, 0.0f, 1.0f}, {0.0f, 1.0f, 0.0f}}; /* blue, green */
  static const float B[2][3] = {{0.0f, 1.0f, 0.0f}, {1.0f, 0.0f, 0.0f}}; /* green, red */
  const int hi = !(nrm < 0.5f);
  const float t = hi ? (nrm - 0.5f) * 2.0f : nrm * 2.0f;
  const float u = 1.0f - t;
  for (int c = 0; c < 3; ++c) rgba[c] = A[hi][c] * u + B[hi][c] * t;
  rgba[3] = 1.0f;
}

/* compute_shader.wgsl:132-137: u32(cell) * prime, wrapping. */
uint32_t orc_hash_cell(int32_t cx, int32_t cy) {
  uint32_t a = (uint32_t)cx * 15823u;
  uint32_t b = (uint32_t)cy * 9737333u;
  return a + b;
}

/* compute_shader.wgsl:139-142. */
uint32_t orc_cell_key(int32_t cx, int32_t cy, uint32_t n) { return orc_hash_cell(cx, cy) % n; }

int32_t orc_f32_to_i32(float v) {
  if (v != v) return 0;
  if (v >= 2147483520.0f) return 2147483647; /* largest f32 below 2^31 is 2^31-128 */
  if (v <= -2147483648.0f) return (int32_t)0x80000000u;
  return (int32_t)v; /* C cast truncates toward zero */
}

/* compute_shader.wgsl:69-99 check_screen_bounds. */
static inline void wall(const rps_config* c, float* x, float* y, float* vx, float* vy) {
  const float x_min = c->screen_bounds[0], x_max = c->screen_bounds[1];
  const float y_min = c->screen_bounds[2], y_max = c->screen_bounds[3];
  const float damp = c->damping_factor;
  if (*x <= x_min) {
    *x = x_min;
    *vx = fabsf(*vx) * damp;
  } else if (*x >= x_max) {
    *x = x_max;
    *vx = -fabsf(*vx) * damp;
  }
  if (*y <= y_min) {
    *y = y_min;
    *vy = fabsf(*vy) * damp;
  } else if (*y >= y_max) {
    *y = y_max;
    *vy = -fabsf(*vy) * damp;
  }
}

/* ----------------------------------------------------------------------------------- */
/* Stream step                                                                           */
/* ----------------------------------------------------------------------------------- */
typedef struct step_consts {
  float dt, gx_dt, gy_dt, neg_g, half_dt, half_dt2, drag_f;
  int drag_on, verlet, lifetime;
  uint32_t na;
  float ax[RPS_MAX_ATTRACTORS], ay[RPS_MAX_ATTRACTORS];
  float as[RPS_MAX_ATTRACTORS], ae2[RPS_MAX_ATTRACTORS];
  uint32_t key0, key1, step_lo, step_hi;
  uint32_t clock; /* lifetime clock of this step */
} step_consts;

static void make_consts(const rps_config* cfg, const rps_ext_config* ext, uint64_t active_step,
                        step_consts* k) {
  memset(k, 0, sizeof(*k));
  const float dt = cfg->fixed_delta_time;
  k->dt = dt;
  k->gx_dt = 0.0f * dt;           /* vec2(0.0, -gravity) * dt   (wgsl:399) */
  k->gy_dt = (-cfg->gravity) * dt;
  k->neg_g = -cfg->gravity;
  k->half_dt = 0.5f * dt;
  k->half_dt2 = (0.5f * dt) * dt;
  k->drag_on = ext->drag != 0.0f;
  k->drag_f = 1.0f - ext->drag * dt;
  k->verlet = ext->integrator == RPS_INTEGRATOR_VERLET;
  k->lifetime = (ext->flags & RPS_EXT_LIFETIME) != 0;
  k->na = ext->num_attractors > RPS_MAX_ATTRACTORS ? RPS_MAX_ATTRACTORS : ext->num_attractors;
  const double t = (double)active_step * (double)dt;
  for (uint32_t a = 0; a < k->na; ++a) {
    orc_attractor_pos(&ext->attractors[a], t, &k->ax[a], &k->ay[a]);
    k->as[a] = ext->attractors[a].strength;
    k->ae2[a] = ext->attractors[a].softening * ext->attractors[a].softening;
  }
  k->key0 = (uint32_t)ext->seed;
  k->key1 = (uint32_t)(ext->seed >> 32);
  k->step_lo = (uint32_t)active_step;
  k->step_hi = (uint32_t)(active_step >> 32);
}

/* 1/sqrt(r2) as specified: initial guess 0x5f375a86 - (bits(r2) >> 1), then
 * three Newton steps y = y * (1.5 - (h * y) * y) with h = 0.5 * r2, each op rounded to f32. */
static inline float inv_sqrt_f(float r2) {
  uint32_t b;
  memcpy(&b, &r2, 4);
  b = 0x5f375a86u - (b >> 1);
  float y;
  memcpy(&y, &b, 4);
  const float h = 0.5f * r2;
  for (int it = 0; it < 3; ++it) {
    float t = h * y;
    t = t * y;
    t = 1.5f - t;
    y = y * t;
  }
  return y;
}
float orc_inv_sqrt(float r2) { return inv_sqrt_f(r2); }

/* Sum of attractor accelerations at (x, y), attractors in index order. */
static inline void attract(const step_consts* k, float x, float y, float* ax, float* ay) {
  float sx = 0.0f, sy = 0.0f;
  for (uint32_t a = 0; a < k->na; ++a) {
    float dx = k->ax[a] - x;
    float dy = k->ay[a] - y;
    float r2 = (dx * dx + dy * dy) + k->ae2[a];
    float inv = inv_sqrt_f(r2);
    float s = k->as[a] * ((inv * inv) * inv);
    sx = sx + dx * s;
    sy = sy + dy * s;
  }
  *ax = sx;
  *ay = sy;
}

/* Lifetime in whole steps: clamp(ceil(L / dt), 1, 65535). */
uint32_t orc_life_steps(float life, float dt) {
  float q = ceilf(life / dt);
  if (!(q >= 1.0f)) return 1u;
  if (q >= 65535.0f) return 65535u;
  return (uint32_t)q;
}

/* life (seconds) <-> expiry at lifetime clock c: e = c + steps(L) - 1; L = ((u16)(e-c)+1)*dt. */
void orc_exp_from_life(const float* life, uint64_t n, uint32_t clock, float dt, uint16_t* exp) {
  for (uint64_t i = 0; i < n; ++i) exp[i] = (uint16_t)(clock + orc_life_steps(life[i], dt) - 1u);
}
void orc_life_from_exp(const uint16_t* exp, uint64_t n, uint32_t clock, float dt, float* life) {
  for (uint64_t i = 0; i < n; ++i)
    life[i] = (float)((uint32_t)(uint16_t)(exp[i] - (uint16_t)clock) + 1u) * dt;
}

/* Returns the new lifetime in steps. */
static inline uint32_t respawn(const rps_ext_config* ext, const step_consts* k, uint64_t gid,
                               float* x, float* y, float* vx, float* vy) {
  uint32_t ctr[4] = {(uint32_t)gid, (uint32_t)(gid >> 32), k->step_lo, k->step_hi};
  uint32_t key[2] = {k->key0, k->key1};
  uint32_t w[4];
  orc_philox4x32_10(ctr, key, w);
  float r = ext->emitter_radius * sqrtf(u01(w[0]));
  float c, s;
  orc_sincos_turns(u01(w[1]), &c, &s);
  *x = ext->emitter_center[0] + r * c;
  *y = ext->emitter_center[1] + r * s;
  float spd = ext->spawn_speed_min + u01(w[3]) * (ext->spawn_speed_max - ext->spawn_speed_min);
  *vx = spd * c;
  *vy = spd * s;
  return orc_life_steps(ext->life_min + u01(w[2]) * (ext->life_max - ext->life_min), k->dt);
}

/* Returns 1 if the particle respawned. */
/* pre_a: Euler only, the attractor acceleration at (x, y) already computed (NULL: compute). */
static inline int stream_one(const rps_config* cfg, const rps_ext_config* ext,
                             const step_consts* k, uint64_t gid, float* px, float* py,
                             float* pvx, float* pvy, uint16_t* pexp, const float* pre_a) {
  float x = *px, y = *py, vx = *pvx, vy = *pvy;
  const float dt = k->dt;
  if (!k->verlet) {
    /* apply_gravity (wgsl:397-400) */
    vx = vx + k->gx_dt;
    vy = vy + k->gy_dt;
    if (k->na) {
      float ax, ay;
      if (pre_a) {
        ax = pre_a[0];
        ay = pre_a[1];
      } else {
        attract(k, x, y, &ax, &ay);
      }
      vx = vx + ax * dt;
      vy = vy + ay * dt;
    }
    if (k->drag_on) {
      vx = vx * k->drag_f;
      vy = vy * k->drag_f;
    }
    /* update_particle_positions (wgsl:392-395) */
    x = x + vx * dt;
    y = y + vy * dt;
  } else {
    float ax0, ay0, ax1, ay1;
    attract(k, x, y, &ax0, &ay0);
    ay0 = ay0 + k->neg_g;
    float x1 = (x + vx * dt) + ax0 * k->half_dt2;
    float y1 = (y + vy * dt) + ay0 * k->half_dt2;
    attract(k, x1, y1, &ax1, &ay1);
    ay1 = ay1 + k->neg_g;
    vx = vx + (ax0 + ax1) * k->half_dt;
    vy = vy + (ay0 + ay1) * k->half_dt;
    if (k->drag_on) {
      vx = vx * k->drag_f;
      vy = vy * k->drag_f;
    }
    x = x1;
    y = y1;
  }
  /* check_screen_bounds (wgsl:69-99) */
  wall(cfg, &x, &y, &vx, &vy);
  int re = 0;
  if (k->lifetime && *pexp == (uint16_t)k->clock) { /* expiry reached: respawn */
    *pexp = (uint16_t)(k->clock + respawn(ext, k, gid, &x, &y, &vx, &vy));
    re = 1;
  }
  *px = x;
  *py = y;
  *pvx = vx;
  *pvy = vy;
  return re;
}

void orc_stream_step(const rps_config* cfg, const rps_ext_config* ext, uint64_t id_offset,
                     uint64_t active_step, uint32_t clock, float* x, float* y, float* vx,
                     float* vy, uint16_t* exp, uint64_t n, orc_stats* stats) {
  step_consts k;
  make_consts(cfg, ext, active_step, &k);
  k.clock = clock;
  if (!exp) k.lifetime = 0;
  float bx0 = INFINITY, bx1 = -INFINITY, by0 = INFINITY, by1 = -INFINITY;
  double ke = 0.0;
  uint64_t re = 0;
  for (uint64_t i = 0; i < n; ++i) {
    re += (uint64_t)stream_one(cfg, ext, &k, id_offset + i, &x[i], &y[i], &vx[i], &vy[i],
                               k.lifetime ? &exp[i] : NULL, NULL);
    if (stats) {
      bx0 = x[i] < bx0 ? x[i] : bx0;
      bx1 = x[i] > bx1 ? x[i] : bx1;
      by0 = y[i] < by0 ? y[i] : by0;
      by1 = y[i] > by1 ? y[i] : by1;
      ke += 0.5 * ((double)vx[i] * vx[i] + (double)vy[i] * vy[i]);
    }
  }
  if (stats) {
    stats->bbox[0] = bx0;
    stats->bbox[1] = bx1;
    stats->bbox[2] = by0;
    stats->bbox[3] = by1;
    stats->kinetic_energy = ke;
    stats->particles = n;
    stats->respawned = re;
  }
}

void orc_stream_step_omp(const rps_config* cfg, const rps_ext_config* ext, uint64_t id_offset,
                         uint64_t active_step, uint32_t clock, float* x, float* y, float* vx,
                         float* vy, uint16_t* exp, uint64_t n, int threads) {
  step_consts k;
  make_consts(cfg, ext, active_step, &k);
  k.clock = clock;
  if (!exp) k.lifetime = 0;
  /* Blocks of 64 particles: the Euler attractor sums first, attractor-major so the compiler
   * vectorises the branch-free inner loop over particles (AVX2), then the rest per particle.
   * Same f32 ops per particle in the same order as orc_stream_step: identical results. */
  enum { B = 64 };
  const int64_t nb = (int64_t)((n + B - 1) / B);
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(static)
#endif
  for (int64_t b = 0; b < nb; ++b) {
    const uint64_t i0 = (uint64_t)b * B;
    const int m = (int)((n - i0) < B ? (n - i0) : B);
    float acc[2 * B];
    const int pre = !k.verlet && k.na;
    if (pre) {
      float sx[B], sy[B];
      for (int j = 0; j < B; ++j) sx[j] = sy[j] = 0.0f;
      for (uint32_t a = 0; a < k.na; ++a) {
        const float pax = k.ax[a], pay = k.ay[a], e2 = k.ae2[a], st = k.as[a];
        for (int j = 0; j < m; ++j) {
          const float dx = pax - x[i0 + j];
          const float dy = pay - y[i0 + j];
          const float r2 = (dx * dx + dy * dy) + e2;
          const float inv = inv_sqrt_f(r2);
          const float sc = st * ((inv * inv) * inv);
          sx[j] = sx[j] + dx * sc;
          sy[j] = sy[j] + dy * sc;
        }
      }
      for (int j = 0; j < m; ++j) {
        acc[2 * j] = sx[j];
        acc[2 * j + 1] = sy[j];
      }
    }
    for (int j = 0; j < m; ++j) {
      const uint64_t i = i0 + (uint64_t)j;
      stream_one(cfg, ext, &k, id_offset + i, &x[i], &y[i], &vx[i], &vy[i],
                 k.lifetime ? &exp[i] : NULL, pre ? &acc[2 * j] : NULL);
    }
  }
  (void)threads;
}

/* Thread count of the OpenMP build's parallel loops (no-op in the serial checker). */
void orc_set_threads(int threads) {
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#else
  (void)threads;
#endif
}

/* Restatement of setup_particles_scatter (src/main.rs:182-216) with a seeded Philox stream
 * in place of the unseeded rand::rng() (src/main.rs:188). */
void orc_init_scatter(const rps_config* cfg, const rps_ext_config* ext, uint64_t seed,
                      uint64_t id_offset, uint64_t global_count, uint32_t clock, float* x,
                      float* y, float* vx, float* vy, uint16_t* exp, uint64_t n) {
  const float x_min = cfg->screen_bounds[0], x_max = cfg->screen_bounds[1];
  const float y_min = cfg->screen_bounds[2], y_max = cfg->screen_bounds[3];
  const float y_center = (y_min + y_max) / 2.0f;
  const float y_sd = (y_max - y_min) * 0.125f;
  const float inv_count = (float)global_count;
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  /* Particles are independent: the OpenMP build (orc_init_scatter through lib(omp=True), the
   * full-size GPU tests) returns the serial checker's bits. */
#pragma omp parallel for schedule(static)
  for (uint64_t i = 0; i < n; ++i) {
    uint64_t g = id_offset + i;
    float t = (float)g / inv_count;
    x[i] = x_min + t * (x_max - x_min);
    uint32_t ctr[4] = {(uint32_t)g, (uint32_t)(g >> 32), 0xFFFFFFFFu, 0xFFFFFFFFu};
    uint32_t w[4];
    orc_philox4x32_10(ctr, key, w);
    float u1 = (float)((w[0] >> 8) + 1u) * (1.0f / 16777216.0f); /* (0, 1] */
    float c, s;
    orc_sincos_turns(u01(w[1]), &c, &s);
    float z = sqrtf(-2.0f * orc_log_unit(u1)) * c;
    float yy = y_center + z * y_sd;
    yy = yy < y_min ? y_min : yy; /* y.clamp(y_min, y_max) (src/main.rs:205) */
    yy = yy > y_max ? y_max : yy;
    y[i] = yy;
    vx[i] = 0.0f;
    vy[i] = 0.0f;
    if (exp)
      exp[i] = (uint16_t)(clock +
                          orc_life_steps(ext->life_min + u01(w[2]) * (ext->life_max - ext->life_min),
                                         cfg->fixed_delta_time) -
                          1u);
  }
}

/* ----------------------------------------------------------------------------------- */
/* All-pairs N-body (build-defined)                                                      */
/* ----------------------------------------------------------------------------------- */
void orc_nbody_accel(const rps_ext_config* ext, const float* sx, const float* sy, uint64_t ns,
                     uint64_t t0, uint64_t nt, float* ax, float* ay) {
  const float eps2 = ext->nbody_softening * ext->nbody_softening;
  const float gm = ext->nbody_strength;
  for (uint64_t ii = 0; ii < nt; ++ii) {
    const float xi = sx[t0 + ii], yi = sy[t0 + ii];
    double accx = 0.0, accy = 0.0; /* double accumulation: the tolerance reference */
    for (uint64_t j = 0; j < ns; ++j) {
      double dx = (double)sx[j] - xi, dy = (double)sy[j] - yi;
      double r2 = dx * dx + dy * dy + (double)eps2;
      double inv = 1.0 / sqrt(r2);
      double s = inv * inv * inv;
      accx += dx * s;
      accy += dy * s;
    }
    ax[ii] = (float)(accx * gm);
    ay[ii] = (float)(accy * gm);
  }
}

/* The same f64 reference for targets [t0, t0 + nt) plus, per target, the scale of f32
 * summation error where the net force cancels: abs_sum[ii] = G * sum_j |f_ij| (f64).  Targets
 * are independent and each sums its sources in index order, so the OpenMP build (targets over
 * threads) returns the same bits as the serial one; used by the full-size N-body tests, whose
 * 2^27-source sums would take minutes on one core. */
void orc_nbody_accel_ref(const rps_ext_config* ext, const float* sx, const float* sy, uint64_t ns,
                         uint64_t t0, uint64_t nt, float* ax, float* ay, double* abs_sum) {
  const float eps2 = ext->nbody_softening * ext->nbody_softening;
  const float gm = ext->nbody_strength;
#pragma omp parallel for schedule(dynamic, 1)
  for (uint64_t ii = 0; ii < nt; ++ii) {
    const float xi = sx[t0 + ii], yi = sy[t0 + ii];
    double accx = 0.0, accy = 0.0, acca = 0.0;
    for (uint64_t j = 0; j < ns; ++j) {
      double dx = (double)sx[j] - xi, dy = (double)sy[j] - yi;
      double d2 = dx * dx + dy * dy;
      double r2 = d2 + (double)eps2;
      double inv = 1.0 / sqrt(r2);
      double s = inv * inv * inv;
      accx += dx * s;
      accy += dy * s;
      acca += sqrt(d2) * s;
    }
    ax[ii] = (float)(accx * gm);
    ay[ii] = (float)(accy * gm);
    abs_sum[ii] = acca * (double)gm;
  }
}

/* orc_nbody_accel_ref for an explicit list of target indices (the full-size GPU tests sample
 * thousands of targets spread over every target block of a launch).  Eight targets per
 * iteration, each with its own accumulators summing its sources in index order with the
 * scalar function's operations (no contraction: -ffp-contract=off), so the compiler's vector
 * lanes over the eight targets return the scalar function's bits target by target. */
void orc_nbody_accel_ref_idx(const rps_ext_config* ext, const float* sx, const float* sy,
                             uint64_t ns, const uint64_t* idx, uint64_t nt, float* ax, float* ay,
                             double* abs_sum) {
  enum { T = 8 };
  const double eps2 = (double)(ext->nbody_softening * ext->nbody_softening);
  const double gm = (double)ext->nbody_strength;
  const int64_t ng = (int64_t)((nt + T - 1) / T);
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t g = 0; g < ng; ++g) {
    double xi[T], yi[T], accx[T], accy[T], acca[T];
    for (int k = 0; k < T; ++k) {
      const uint64_t ii = (uint64_t)g * T + (uint64_t)k;
      const uint64_t t = idx[ii < nt ? ii : nt - 1];
      xi[k] = (double)sx[t];
      yi[k] = (double)sy[t];
      accx[k] = accy[k] = acca[k] = 0.0;
    }
    for (uint64_t j = 0; j < ns; ++j) {
      const double qx = (double)sx[j], qy = (double)sy[j];
#pragma omp simd
      for (int k = 0; k < T; ++k) {
        const double dx = qx - xi[k], dy = qy - yi[k];
        const double d2 = dx * dx + dy * dy;
        const double r2 = d2 + eps2;
        const double inv = 1.0 / sqrt(r2);
        const double s = inv * inv * inv;
        accx[k] += dx * s;
        accy[k] += dy * s;
        acca[k] += sqrt(d2) * s;
      }
    }
    for (int k = 0; k < T; ++k) {
      const uint64_t ii = (uint64_t)g * T + (uint64_t)k;
      if (ii >= nt) break;
      ax[ii] = (float)(accx[k] * gm);
      ay[ii] = (float)(accy[k] * gm);
      abs_sum[ii] = acca[k] * gm;
    }
  }
}

void orc_nbody_accel_f32_omp(const rps_ext_config* ext, const float* sx, const float* sy,
                             uint64_t ns, uint64_t t0, uint64_t nt, float* ax, float* ay,
                             int threads) {
  const float eps2 = ext->nbody_softening * ext->nbody_softening;
  const float gm = ext->nbody_strength;
  orc_set_threads(threads);
#pragma omp parallel for schedule(dynamic, 64)
  for (uint64_t ii = 0; ii < nt; ++ii) {
    const float xi = sx[t0 + ii], yi = sy[t0 + ii];
    float accx = 0.0f, accy = 0.0f;
#pragma omp simd reduction(+ : accx, accy)
    for (uint64_t j = 0; j < ns; ++j) {
      const float dx = sx[j] - xi, dy = sy[j] - yi;
      const float r2 = dx * dx + dy * dy + eps2;
      const float inv = 1.0f / sqrtf(r2);
      const float s = inv * inv * inv;
      accx += dx * s;
      accy += dy * s;
    }
    ax[ii] = accx * gm;
    ay[ii] = accy * gm;
  }
}

void orc_nbody_integrate(const rps_config* cfg, const rps_ext_config* ext, const float* ax,
                         const float* ay, float* x, float* y, float* vx, float* vy, uint64_t n) {
  step_consts k;
  make_consts(cfg, ext, 0, &k);
  const float dt = k.dt;
  for (uint64_t i = 0; i < n; ++i) {
    float px = x[i], py = y[i], qx = vx[i], qy = vy[i];
    qx = qx + k.gx_dt;
    qy = qy + k.gy_dt;
    qx = qx + ax[i] * dt;
    qy = qy + ay[i] * dt;
    if (k.drag_on) {
      qx = qx * k.drag_f;
      qy = qy * k.drag_f;
    }
    px = px + qx * dt;
    py = py + qy * dt;
    wall(cfg, &px, &py, &qx, &qy);
    x[i] = px;
    y[i] = py;
    vx[i] = qx;
    vy[i] = qy;
  }
}

/* ----------------------------------------------------------------------------------- */
/* SPH: the reference's five passes                                                      */
/* ----------------------------------------------------------------------------------- */

/* bin_particles_in_grid (wgsl:455-468) + particle_position_to_cell_coord (:121-130). */
void orc_sph_bin(const rps_config* cfg, const float* x, const float* y, uint32_t* lookup,
                 uint32_t* offsets, uint32_t n) {
  const float x_max = cfg->screen_bounds[1], y_max = cfg->screen_bounds[3];
  const float r = cfg->smoothing_radius;
#pragma omp parallel for schedule(static)
  for (uint32_t i = 0; i < n; ++i) {
    int32_t cx = orc_f32_to_i32((x[i] + x_max) / r);
    int32_t cy = orc_f32_to_i32((y[i] + y_max) / r);
    lookup[2 * i] = orc_cell_key(cx, cy, cfg->particle_count);
    lookup[2 * i + 1] = i;
    offsets[i] = 0xFFFFFFFFu;
  }
}

static uint32_t next_pow2(uint32_t n) {
  uint32_t p = 1;
  while (p < n) p <<= 1;
  return p;
}

/* sort_particles (wgsl:470-505) driven by the pass table of src/particle_buffers.rs:108-138
 * and the dispatch loop of src/particle_compute.rs:117-149.  Pairs within one pass are
 * disjoint, so serial execution equals the parallel dispatch. */
uint32_t orc_sph_sort(uint32_t* lookup, uint32_t n) {
  const uint32_t P = next_pow2(n);
  uint32_t stages = 0;
  while ((1u << stages) < P) ++stages;
  uint32_t passes = 0;
  for (uint32_t stage = 0; stage < stages; ++stage) {
    for (uint32_t step = 0; step <= stage; ++step) {
      const uint32_t gw = 1u << (stage - step);
      const uint32_t gh = 2u * gw - 1u;
#pragma omp parallel for schedule(static)
      for (uint32_t i = 0; i < P / 2u; ++i) {
        const uint32_t h = i & (gw - 1u);
        const uint32_t left = h + (gh + 1u) * (i / gw);
        const uint32_t rs = step == 0 ? gh - 2u * h : (gh + 1u) / 2u;
        const uint32_t right = left + rs;
        if (right >= P) continue;
        if (lookup[2 * left] > lookup[2 * right]) {
          uint32_t k = lookup[2 * left], v = lookup[2 * left + 1];
          lookup[2 * left] = lookup[2 * right];
          lookup[2 * left + 1] = lookup[2 * right + 1];
          lookup[2 * right] = k;
          lookup[2 * right + 1] = v;
        }
      }
      ++passes;
    }
  }
  return passes;
}

/* calculate_spatial_lookup_offsets (wgsl:507-525). */
void orc_sph_offsets(const uint32_t* lookup, uint32_t* offsets, uint32_t n) {
#pragma omp parallel for schedule(static) /* one writer per key: its run's first entry */
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t key = lookup[2 * i];
    uint32_t prev = i > 0 ? lookup[2 * (i - 1)] : 0xFFFFFFFFu;
    if (key != prev) offsets[key] = i;
  }
}

static const int32_t GRID_OFF[9][2] = {{-1, -1}, {-1, 0}, {-1, 1}, {0, -1}, {0, 0},
                                       {0, 1},   {1, -1}, {1, 0},  {1, 1}};

static inline int32_t wrap_add(int32_t a, int32_t b) {
  return (int32_t)((uint32_t)a + (uint32_t)b);
}

/* calculate_density (wgsl:207-254) of particle i at its predicted position pred[i], its
 * neighbours' predicted positions read from `nb` (pred itself: the snapshot semantics). */
static void density_one(const rps_config* cfg, const uint32_t* lookup, const uint32_t* offsets,
                        const float* pred, const float* nb, uint32_t i, float* d_out,
                        float* nd_out) {
  const float x_max = cfg->screen_bounds[1], y_max = cfg->screen_bounds[3];
  const float r = cfg->smoothing_radius, r2 = r * r;
  const uint32_t N = cfg->particle_count;
  const float px = pred[2 * i], py = pred[2 * i + 1];
  const int32_t cx = orc_f32_to_i32((px + x_max) / r);
  const int32_t cy = orc_f32_to_i32((py + y_max) / r);
  float d = 0.0f, nd = 0.0f;
  for (int o = 0; o < 9; ++o) {
    const uint32_t key = orc_cell_key(wrap_add(cx, GRID_OFF[o][0]), wrap_add(cy, GRID_OFF[o][1]), N);
    for (uint32_t j = offsets[key]; j < N; ++j) {
      if (lookup[2 * j] != key) break;
      const uint32_t oi = lookup[2 * j + 1];
      const float qx = oi == i ? px : nb[2 * oi], qy = oi == i ? py : nb[2 * oi + 1];
      const float dx = px - qx, dy = py - qy;
      const float sq = dx * dx + dy * dy;
      if (sq > r2) continue;
      const float dist = sqrtf(sq);
      float k1 = 0.0f, k2 = 0.0f;
      if (!(dist >= r)) {
        const float v = r - dist;
        k1 = (cfg->density_kernel_norm * v) * v;            /* :145-152 */
        k2 = ((cfg->near_density_kernel_norm * v) * v) * v; /* :163-170 */
      }
      d = d + k1;
      nd = nd + k2;
    }
  }
  *d_out = d;
  *nd_out = nd;
}

/* apply_gravity (wgsl:397-400) and update_predicted_positions (:402-405) of particle i. */
static inline void predict_one(const rps_config* cfg, float* vx, float* vy, const float* x,
                               const float* y, float* pred, uint32_t i) {
  const float dt = cfg->fixed_delta_time;
  vx[i] = vx[i] + 0.0f * dt;
  vy[i] = vy[i] + (-cfg->gravity) * dt;
  pred[2 * i] = x[i] + vx[i] * dt;
  pred[2 * i + 1] = y[i] + vy[i] * dt;
}

/* pre_simulation_step (wgsl:420-433): apply_gravity, update_predicted_positions for ALL
 * particles, then calculate_density (:207-254) against that snapshot. */
void orc_sph_pre(const rps_config* cfg, float* vx, float* vy, const float* x, const float* y,
                 const uint32_t* lookup, const uint32_t* offsets, float* dens, float* pred,
                 uint32_t n) {
#pragma omp parallel for schedule(static)
  for (uint32_t i = 0; i < n; ++i) predict_one(cfg, vx, vy, x, y, pred, i);
#pragma omp parallel for schedule(dynamic, 1024)
  for (uint32_t i = 0; i < n; ++i) density_one(cfg, lookup, offsets, pred, pred, i, &dens[2 * i], &dens[2 * i + 1]);
}

/* calculate_pressure_force (wgsl:256-334) of particle i. */
static void pressure_one(const rps_config* cfg, const uint32_t* lookup, const uint32_t* offsets,
                         const float* dens, const float* pred, uint32_t i, float* fx_out,
                         float* fy_out) {
  const float x_max = cfg->screen_bounds[1], y_max = cfg->screen_bounds[3];
  const float r = cfg->smoothing_radius, r2 = r * r;
  const uint32_t N = cfg->particle_count;
  const float td = cfg->target_density, pm = cfg->pressure_multiplier;
  const float nm = cfg->near_density_multiplier;
  const float dn = cfg->density_kernel_norm, ndn = cfg->near_density_kernel_norm;
  const float px = pred[2 * i], py = pred[2 * i + 1];
  const int32_t cx = orc_f32_to_i32((px + x_max) / r);
  const int32_t cy = orc_f32_to_i32((py + y_max) / r);
  const float rho = dens[2 * i], rhon = dens[2 * i + 1];
  const float P = (rho - td) * pm;
  const float Pn = rhon * nm;
  float fx = 0.0f, fy = 0.0f;
  for (int o = 0; o < 9; ++o) {
    const uint32_t key = orc_cell_key(wrap_add(cx, GRID_OFF[o][0]), wrap_add(cy, GRID_OFF[o][1]), N);
    for (uint32_t j = offsets[key]; j < N; ++j) {
      if (lookup[2 * j] != key) break;
      const uint32_t oi = lookup[2 * j + 1];
      if (oi == i) continue;
      const float dx = pred[2 * oi] - px, dy = pred[2 * oi + 1] - py;
      const float sq = dx * dx + dy * dy;
      if (sq > r2) continue;
      const float dist = sqrtf(sq);
      float dirx, diry;
      if (dist > 0.0001f) {
        dirx = dx / dist;
        diry = dy / dist;
      } else {
        dirx = 0.0f;
        diry = 1.0f;
      }
      const float rj = dens[2 * oi], rnj = dens[2 * oi + 1];
      const float Pj = (rj - td) * pm;
      const float Pnj = rnj * nm;
      const float pt = (P / (rho * rho)) + (Pj / (rj * rj));
      const float npt = (Pn / (rho * rho)) + (Pnj / (rj * rnj));
      float dk = 0.0f, ndk = 0.0f;
      if (!(dist >= r)) {
        const float v = r - dist;
        dk = (-2.0f * dn) * v;         /* :154-161 */
        ndk = ((-3.0f * ndn) * v) * v; /* :172-179 */
      }
      fx = fx + (dirx * pt) * dk;
      fy = fy + (diry * pt) * dk;
      fx = fx + (dirx * npt) * ndk;
      fy = fy + (diry * npt) * ndk;
    }
  }
  *fx_out = fx;
  *fy_out = fy;
}

/* calculate_viscocity (wgsl:336-384) of particle i, own velocity (qx, qy), the neighbours'
 * velocities read from (nvx, nvy). */
static void viscosity_one(const rps_config* cfg, const uint32_t* lookup, const uint32_t* offsets,
                          const float* pred, const float* nvx, const float* nvy, uint32_t i,
                          float qx, float qy, float* wx_out, float* wy_out) {
  const float x_max = cfg->screen_bounds[1], y_max = cfg->screen_bounds[3];
  const float r = cfg->smoothing_radius, r2 = r * r;
  const uint32_t N = cfg->particle_count;
  const float vn = cfg->viscocity_kernel_norm;
  const float px = pred[2 * i], py = pred[2 * i + 1];
  const int32_t cx = orc_f32_to_i32((px + x_max) / r);
  const int32_t cy = orc_f32_to_i32((py + y_max) / r);
  float wx = 0.0f, wy = 0.0f;
  for (int o = 0; o < 9; ++o) {
    const uint32_t key = orc_cell_key(wrap_add(cx, GRID_OFF[o][0]), wrap_add(cy, GRID_OFF[o][1]), N);
    for (uint32_t j = offsets[key]; j < N; ++j) {
      if (lookup[2 * j] != key) break;
      const uint32_t oi = lookup[2 * j + 1];
      if (oi == i) continue;
      const float dx = px - pred[2 * oi], dy = py - pred[2 * oi + 1];
      const float sq = dx * dx + dy * dy;
      if (sq > r2) continue;
      const float dist = sqrtf(sq);
      float k = 0.0f;
      if (!(dist >= r)) {
        const float v = r * r - dist * dist;
        k = ((vn * v) * v) * v; /* :181-188 */
      }
      wx = wx + (nvx[oi] - qx) * k;
      wy = wy + (nvy[oi] - qy) * k;
    }
  }
  *wx_out = wx;
  *wy_out = wy;
}

/* apply_viscocity_force (:413-417), update_particle_positions (:392-395), walls (:69-99). */
static inline void sim_finish(const rps_config* cfg, float* x, float* y, float* vx, float* vy,
                              uint32_t i, float qx, float qy, float wx, float wy) {
  const float dt = cfg->fixed_delta_time;
  qx = qx + (wx * cfg->viscocity_strength) * dt;
  qy = qy + (wy * cfg->viscocity_strength) * dt;
  float ox = x[i] + qx * dt;
  float oy = y[i] + qy * dt;
  wall(cfg, &ox, &oy, &qx, &qy);
  x[i] = ox;
  y[i] = oy;
  vx[i] = qx;
  vy[i] = qy;
}

/* simulation_step (wgsl:435-453): pressure (:256-334), viscosity (:336-384), Euler
 * (:392-395), walls (:69-99).  Neighbour velocities come from the start-of-pass snapshot;
 * the particle's own velocity is post-pressure (program order in one invocation). */
void orc_sph_sim(const rps_config* cfg, float* x, float* y, float* vx, float* vy,
                 const uint32_t* lookup, const uint32_t* offsets, const float* dens,
                 const float* pred, uint32_t n) {
  const float dt = cfg->fixed_delta_time;
  float* svx = (float*)malloc(sizeof(float) * n);
  float* svy = (float*)malloc(sizeof(float) * n);
  memcpy(svx, vx, sizeof(float) * n);
  memcpy(svy, vy, sizeof(float) * n);
  /* Iterations write only particle i and read neighbours from pred / dens / the velocity
   * snapshot, so the OpenMP build (bench cpu_baseline) equals the serial checker bit for bit. */
#pragma omp parallel for schedule(dynamic, 1024)
  for (uint32_t i = 0; i < n; ++i) {
    float fx, fy, wx, wy;
    pressure_one(cfg, lookup, offsets, dens, pred, i, &fx, &fy);
    const float qx = svx[i] + fx * dt; /* apply_pressure_force (:407-411) */
    const float qy = svy[i] + fy * dt;
    viscosity_one(cfg, lookup, offsets, pred, svx, svy, i, qx, qy, &wx, &wy);
    sim_finish(cfg, x, y, vx, vy, i, qx, qy, wx, wy);
  }
  free(svx);
  free(svy);
}

/* ----------------------------------------------------------------------------------- */
/* Other legal WGSL schedules of passes 4-5 (test infrastructure: the spread of outputs a   */
/* conforming WGSL implementation may produce; tools/wgsl_schedule_envelope.py).            */
/* ----------------------------------------------------------------------------------- */
/* The reference reads buffers that the same dispatch writes: calculate_density reads other
 * invocations' predicted_positions (wgsl:240) while they are written (:430), and
 * calculate_viscocity reads other particles' velocity (:371) while apply_pressure_force /
 * apply_viscocity_force / check_screen_bounds write it (:410, :416, :452).  WGSL orders none
 * of it.  These restatements execute invocation groups of `group` consecutive invocations one
 * group after another in the order `order[0 .. ceil(n / group))`, each group in lockstep (every
 * member finishes a statement before any member starts the next, as a wave does).  A group then
 * reads its own and the earlier groups' writes and the previous contents for later groups: the
 * previous frame's predicted positions, the start-of-pass velocities.  One group of all n
 * invocations gives orc_sph_pre's bits, and a sim whose neighbours' velocities are post-pressure
 * (the snapshot semantics of orc_sph_sim, start-of-pass velocities for every neighbour, is the
 * weak-memory execution in which no write is seen before the pass ends); groups of one in
 * index order are a serial CPU executor's schedule. */
void orc_sph_pre_sched(const rps_config* cfg, float* vx, float* vy, const float* x,
                       const float* y, const uint32_t* lookup, const uint32_t* offsets,
                       float* dens, float* pred, uint32_t n, const uint32_t* order,
                       uint32_t group) {
  const uint32_t ng = (n + group - 1u) / group;
  for (uint32_t k = 0; k < ng; ++k) {
    const uint32_t lo = order[k] * group, hi = lo + group < n ? lo + group : n;
    for (uint32_t i = lo; i < hi; ++i) predict_one(cfg, vx, vy, x, y, pred, i);
    for (uint32_t i = lo; i < hi; ++i) density_one(cfg, lookup, offsets, pred, pred, i, &dens[2 * i], &dens[2 * i + 1]);
  }
}

/* The weak-memory extreme of pass 4: no invocation sees another's new prediction (each
 * density reads the other particles' predicted positions of the previous frame, pred_prev; its
 * own is program-ordered, fresh).  Legal where the writes of other workgroups are not yet
 * visible (non-coherent caches). */
void orc_sph_pre_stale(const rps_config* cfg, float* vx, float* vy, const float* x, const float* y,
                       const uint32_t* lookup, const uint32_t* offsets, float* dens, float* pred,
                       const float* pred_prev, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i) predict_one(cfg, vx, vy, x, y, pred, i);
  for (uint32_t i = 0; i < n; ++i) density_one(cfg, lookup, offsets, pred, pred_prev, i, &dens[2 * i], &dens[2 * i + 1]);
}

void orc_sph_sim_sched(const rps_config* cfg, float* x, float* y, float* vx, float* vy,
                       const uint32_t* lookup, const uint32_t* offsets, const float* dens,
                       const float* pred, uint32_t n, const uint32_t* order, uint32_t group) {
  const float dt = cfg->fixed_delta_time;
  const uint32_t ng = (n + group - 1u) / group;
  float* w = (float*)malloc(sizeof(float) * 2u * (group < n ? group : n));
  for (uint32_t k = 0; k < ng; ++k) {
    const uint32_t lo = order[k] * group, hi = lo + group < n ? lo + group : n;
    for (uint32_t i = lo; i < hi; ++i) { /* apply_pressure_force: velocity written in place */
      float fx, fy;
      pressure_one(cfg, lookup, offsets, dens, pred, i, &fx, &fy);
      vx[i] = vx[i] + fx * dt;
      vy[i] = vy[i] + fy * dt;
    }
    for (uint32_t i = lo; i < hi; ++i) /* calculate_viscocity: every member reads before any writes */
      viscosity_one(cfg, lookup, offsets, pred, vx, vy, i, vx[i], vy[i], &w[2 * (i - lo)], &w[2 * (i - lo) + 1]);
    for (uint32_t i = lo; i < hi; ++i) sim_finish(cfg, x, y, vx, vy, i, vx[i], vy[i], w[2 * (i - lo)], w[2 * (i - lo) + 1]);
  }
  free(w);
}
