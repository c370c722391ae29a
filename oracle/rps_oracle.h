/*
 * rps_oracle.h — CPU restatement of the reference's per-particle step.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed CPU
 * baseline — never as the product path (librps.so has no dependency on it).
 *
 * PARITY UNPINNED at the WGSL-execution boundary: the reference (Rust + Bevy 0.16.1 +
 * wgpu 24.0.5, Cargo.lock:318/:4464) cannot be built or run in this pipeline and ships no
 * tests, fixtures or golden vectors.  This file restates
 * assets/compute_shader.wgsl operation by operation (each function cites the line it
 * follows) with IEEE binary32 arithmetic, no FMA contraction (-ffp-contract=off),
 * correctly-rounded division and sqrt, and snapshot semantics where the WGSL races
 * (DESIGN.md §3.3).  What *is* pinned: the known-answer values of tests/golden/ (kernel
 * norms, hash keys, bitonic pass counts, Random123 Philox KATs) computed independently.
 */
#ifndef RPS_ORACLE_H_
#define RPS_ORACLE_H_

#include <stdint.h>
#include "../include/rps.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_stats {
  float bbox[4];
  double kinetic_energy;
  uint64_t particles;
  uint64_t respawned;
} orc_stats;

/* Thread count of the OpenMP build (librps_oracle_omp.so); no-op in the serial checker. */
void orc_set_threads(int threads);
/* Random123 Philox4x32-10. */
void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
/* Deterministic polynomial sin/cos of 2*pi*u, u in [0,1). */
void orc_sincos_turns(float u, float* c, float* s);
/* Deterministic ln(u), u in (0, 1] normal (initial scatter's Box-Muller). */
float orc_log_unit(float u);
/* Attractor k position at time t (double precision, rounded to float). */
void orc_attractor_pos(const rps_attractor* a, double t, float* px, float* py);

/* compute_shader.wgsl:101-118 set_color. */
void orc_set_color(float vx, float vy, float max_energy, float rgba[4]);
/* compute_shader.wgsl:132-142 hash_cell + get_key_from_hash. */
uint32_t orc_hash_cell(int32_t cx, int32_t cy);
uint32_t orc_cell_key(int32_t cx, int32_t cy, uint32_t n);
/* WGSL i32(f32): truncate toward zero, saturate, NaN -> 0. */
int32_t orc_f32_to_i32(float v);

/* Lifetime (build-defined): a particle keeps a u16 expiry e = the lifetime-
 * clock value of the step in which it respawns; L seconds last clamp(ceil(L/dt), 1, 65535)
 * steps.  Conversions at lifetime clock c (the clock of the next step). */
uint32_t orc_life_steps(float life, float dt);
/* The attractor force's 1/sqrt (bit trick + 3 Newton steps). */
float orc_inv_sqrt(float r2);
void orc_exp_from_life(const float* life, uint64_t n, uint32_t clock, float dt, uint16_t* exp);
void orc_life_from_exp(const uint16_t* exp, uint64_t n, uint32_t clock, float dt, float* life);

/* One active stream step (mode STREAM) over n particles with global ids id_offset+i;
 * active_step keys the Philox respawn stream, clock is this step's lifetime clock.
 * exp may be NULL when RPS_EXT_LIFETIME is off.  stats may be NULL. */
void orc_stream_step(const rps_config* cfg, const rps_ext_config* ext, uint64_t id_offset,
                     uint64_t active_step, uint32_t clock, float* x, float* y, float* vx,
                     float* vy, uint16_t* exp, uint64_t n, orc_stats* stats);
/* Same, OpenMP-parallel over particles (bench cpu_baseline); identical results. */
void orc_stream_step_omp(const rps_config* cfg, const rps_ext_config* ext, uint64_t id_offset,
                         uint64_t active_step, uint32_t clock, float* x, float* y, float* vx,
                         float* vy, uint16_t* exp, uint64_t n, int threads);

/* Device-init restatement (rps_init_scatter) at lifetime clock `clock`. */
void orc_init_scatter(const rps_config* cfg, const rps_ext_config* ext, uint64_t seed,
                      uint64_t id_offset, uint64_t global_count, uint32_t clock, float* x,
                      float* y, float* vx, float* vy, uint16_t* exp, uint64_t n);

/* All-pairs softened gravity: acc of targets [t0, t0+nt) from all ns sources. */
void orc_nbody_accel(const rps_ext_config* ext, const float* sx, const float* sy, uint64_t ns,
                     uint64_t t0, uint64_t nt, float* ax, float* ay);
void orc_nbody_accel_ref(const rps_ext_config* ext, const float* sx, const float* sy, uint64_t ns,
                         uint64_t t0, uint64_t nt, float* ax, float* ay, double* abs_sum);
/* orc_nbody_accel_ref's bits for the targets idx[0 .. nt) (any order, any spread). */
void orc_nbody_accel_ref_idx(const rps_ext_config* ext, const float* sx, const float* sy,
                             uint64_t ns, const uint64_t* idx, uint64_t nt, float* ax, float* ay,
                             double* abs_sum);
/* The same force in f32 on every host core (bench.py's all-pairs cpu_baseline only, not a
 * checker): per target an f32 sum, vectorised by `omp simd` (its own summation order). */
void orc_nbody_accel_f32_omp(const rps_ext_config* ext, const float* sx, const float* sy,
                             uint64_t ns, uint64_t t0, uint64_t nt, float* ax, float* ay,
                             int threads);
/* Integrate given accelerations (mode NBODY second half). */
void orc_nbody_integrate(const rps_config* cfg, const rps_ext_config* ext, const float* ax,
                         const float* ay, float* x, float* y, float* vx, float* vy, uint64_t n);

/* SPH passes (compute_shader.wgsl:455-525, :420-453).  lookup has 2*P uint32 (P =
 * next_pow2(N)), offsets N, dens 2N, pred 2N. */
void orc_sph_bin(const rps_config* cfg, const float* x, const float* y, uint32_t* lookup,
                 uint32_t* offsets, uint32_t n);
uint32_t orc_sph_sort(uint32_t* lookup, uint32_t n); /* returns number of passes */
void orc_sph_offsets(const uint32_t* lookup, uint32_t* offsets, uint32_t n);
void orc_sph_pre(const rps_config* cfg, float* vx, float* vy, const float* x, const float* y,
                 const uint32_t* lookup, const uint32_t* offsets, float* dens, float* pred,
                 uint32_t n);
void orc_sph_sim(const rps_config* cfg, float* x, float* y, float* vx, float* vy,
                 const uint32_t* lookup, const uint32_t* offsets, const float* dens,
                 const float* pred, uint32_t n);
/* Passes 4-5 under another legal WGSL schedule: groups of `group` invocations in lockstep,
 * executed one after another in the order order[0 .. ceil(n / group)) (rps_oracle.c). */
void orc_sph_pre_sched(const rps_config* cfg, float* vx, float* vy, const float* x,
                       const float* y, const uint32_t* lookup, const uint32_t* offsets,
                       float* dens, float* pred, uint32_t n, const uint32_t* order,
                       uint32_t group);
void orc_sph_sim_sched(const rps_config* cfg, float* x, float* y, float* vx, float* vy,
                       const uint32_t* lookup, const uint32_t* offsets, const float* dens,
                       const float* pred, uint32_t n, const uint32_t* order, uint32_t group);
/* Pass 4 with every other particle's prediction of the previous frame (pred_prev). */
void orc_sph_pre_stale(const rps_config* cfg, float* vx, float* vy, const float* x, const float* y,
                       const uint32_t* lookup, const uint32_t* offsets, float* dens, float* pred,
                       const float* pred_prev, uint32_t n);

#ifdef __cplusplus
}
#endif

#endif
