/*
 * rps.h — C ABI of the MI355X-native particle integrator (librps.so).
 *
 * This is the drop-in boundary for the one hot path of mabrams4/Rust-Particle-System:
 * the per-particle step that the reference runs as
 *     ParticleComputeNode::run  (src/particle_compute.rs:91-195)
 *  -> five WGSL entry points     (assets/compute_shader.wgsl:420-525)
 * over buffers created by
 *     prepare_particle_buffers  (src/particle_buffers.rs:38-237).
 *
 * Every entry point below names the reference interface it replaces.  Plain C: no
 * exceptions or panics cross the boundary; every call returns an rps_status (0 = ok) and
 * the context keeps a human-readable message for rps_last_error().  Each context owns one
 * HIP stream on one device; calls are stream-ordered and only rps_sync(), the downloads and
 * rps_read_* block the host (the reference never synchronises on the hot path either:
 * src/particle_compute.rs:91-195 only records dispatches).
 *
 * Units, semantics and the build-defined extensions (attractors, drag, lifetime/respawn,
 * velocity-Verlet, all-pairs N-body, stats) are specified in DESIGN.md §3.
 */
#ifndef RPS_H_
#define RPS_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RPS_ABI_VERSION 2u  /* 2: lifetime kept as an expiry (RPS_FIELD_LIFE_STEPS, RPS_DEBUG_EXPIRY) */

/* ------------------------------------------------------------------------------------ */
/* Status codes                                                                          */
/* ------------------------------------------------------------------------------------ */
typedef enum rps_status {
  RPS_OK = 0,
  RPS_ERR_INVALID_ARGUMENT = 1, /* null pointer, size mismatch, bad enum, n > capacity  */
  RPS_ERR_DEVICE = 2,           /* a HIP runtime call failed (message has hipGetErrorString) */
  RPS_ERR_OUT_OF_MEMORY = 3,    /* hipMalloc / hipHostMalloc failed                     */
  RPS_ERR_UNSUPPORTED = 4,      /* mode/feature not available for this context          */
  RPS_ERR_COMM = 5,             /* RCCL call failed                                     */
  RPS_ERR_NO_DEVICE = 6         /* no HIP device visible                                */
} rps_status;

/* ------------------------------------------------------------------------------------ */
/* Data types that must stay byte-compatible with the reference                          */
/* ------------------------------------------------------------------------------------ */

/* == Particle, src/particle.rs:20-25 (encase std430 layout == compute_shader.wgsl:35-39):
 * 32 bytes, position @0, velocity @8, color @16. */
typedef struct rps_particle {
  float position[2];
  float velocity[2];
  float color[4];
} rps_particle;

/* == ParticleConfig, src/main.rs:43-69 (#[repr(C)], Pod) == WGSL Config,
 * compute_shader.wgsl:2-25.  144 bytes.  frame_count is advanced by rps_step() exactly as
 * prepare_particle_buffers does every frame (src/particle_buffers.rs:227). */
typedef struct rps_config {
  uint32_t particle_count;
  float particle_size;
  float smoothing_radius;
  float max_energy;

  float damping_factor;
  float fixed_delta_time;
  uint32_t frame_count;
  float gravity;

  float density_kernel_norm;
  float near_density_kernel_norm;
  float viscocity_kernel_norm;
  float _padding;

  float target_density;
  float pressure_multiplier;
  float viscocity_strength;
  float near_density_multiplier;

  float screen_bounds[4]; /* x_min, x_max, y_min, y_max */
  float view_proj[16];    /* column-major mat4; not read by the compute path */
} rps_config;

/* == SortingParams, src/particle_buffers.rs:28-35 (one bitonic compare-swap pass). */
typedef struct rps_sort_params {
  uint32_t n;
  uint32_t group_width;
  uint32_t group_height;
  uint32_t step_index;
} rps_sort_params;

/* ------------------------------------------------------------------------------------ */
/* Build-defined extensions (no reference counterpart)               */
/* ------------------------------------------------------------------------------------ */
#define RPS_MAX_ATTRACTORS 8

/* A point attractor moving on a circle: centre + orbit_radius*(cos, sin)(w*t + phase).
 * Acceleration on a particle at p: strength * d / (|d|^2 + softening^2)^(3/2), d = a - p. */
typedef struct rps_attractor {
  float center[2];
  float orbit_radius;
  float angular_velocity; /* rad/s */
  float phase;            /* rad   */
  float strength;
  float softening;
  float _pad;
} rps_attractor;

typedef enum rps_integrator {
  RPS_INTEGRATOR_EULER = 0,  /* reference order: v += a dt ; p += v dt (compute_shader.wgsl:392-400) */
  RPS_INTEGRATOR_VERLET = 1  /* velocity-Verlet, a(x) recomputed, no stored acceleration  */
} rps_integrator;

enum {
  RPS_EXT_LIFETIME = 1u << 0, /* lifetime in whole steps; respawn at the emitter on expiry (below) */
  RPS_EXT_STATS = 1u << 1,    /* fuse bbox / kinetic-energy / respawn-count reductions into the step */
  RPS_EXT_NBODY_EXTERNAL = 1u << 2 /* N-body shards: the caller exchanges the sources (rps_nbody_sources) */
};

typedef struct rps_ext_config {
  uint32_t integrator;     /* rps_integrator                                               */
  uint32_t num_attractors; /* 0..RPS_MAX_ATTRACTORS                                          */
  uint32_t flags;          /* RPS_EXT_*                                                      */
  uint32_t shader_delay;   /* steps gated off at start; reference SHADER_DELAY = 5 (wgsl:66) */
  float drag;              /* c in v *= (1 - c dt); 0 disables                                */
  float life_min;          /* respawn lifetime ~ U(life_min, life_max) seconds               */
  float life_max;
  float emitter_radius;    /* respawn position uniform in a disc                             */
  float emitter_center[2];
  float spawn_speed_min;   /* respawn velocity radial outward, speed ~ U(min, max)           */
  float spawn_speed_max;
  uint64_t seed;           /* Philox4x32-10 key                                              */
  float nbody_strength;    /* all-pairs: G*m per source particle                            */
  float nbody_softening;   /* all-pairs Plummer softening epsilon                          */
  uint32_t stats_interval; /* with RPS_EXT_STATS: reduce every k-th active step (>=1)       */
  uint32_t fuse_steps;     /* STREAM: advance up to this many steps per launch in registers
                              (state read/written once; bitwise == separate steps); 0/1 = off */
  rps_attractor attractors[RPS_MAX_ATTRACTORS];
} rps_ext_config;

/* ------------------------------------------------------------------------------------ */
/* Context                                                                               */
/* ------------------------------------------------------------------------------------ */
typedef enum rps_mode {
  RPS_MODE_STREAM = 0, /* gravity/attractors + integrate + wall + lifetime: one fused kernel per step */
  RPS_MODE_NBODY = 1,  /* all-pairs softened gravity (LDS position tiles) + integrate            */
  RPS_MODE_SPH = 2     /* the reference's five passes: bin, bitonic sort, offsets, pre-sim, sim  */
} rps_mode;

typedef struct rps_create_info {
  int32_t device;          /* HIP device ordinal                                            */
  uint32_t mode;           /* rps_mode                                                      */
  uint64_t particle_count; /* particles owned by this context (this rank's shard)          */
  uint64_t id_offset;      /* global id of local particle 0 (index-range sharding)         */
  uint64_t global_count;   /* particles in the whole system (>= id_offset + particle_count) */
} rps_create_info;

typedef struct rps_ctx rps_ctx;

/* Field selectors for SoA transfers and debug readback (mirrors src/debug.rs:121-265). */
typedef enum rps_field {
  RPS_FIELD_X = 0,
  RPS_FIELD_Y = 1,
  RPS_FIELD_VX = 2,
  RPS_FIELD_VY = 3,
  RPS_FIELD_LIFE = 4,        /* seconds = LIFE_STEPS * dt (STREAM)                  */
  RPS_FIELD_LIFE_STEPS = 5,  /* whole lifetime steps left, an exact f32 integer      */
  RPS_DEBUG_SPATIAL_LOOKUP = 16,  /* u32x2 (key, index) x next_pow2(N)   (wgsl:52)  */
  RPS_DEBUG_LOOKUP_OFFSETS = 17,  /* u32 x N                              (wgsl:55)  */
  RPS_DEBUG_DENSITIES = 18,       /* f32x2 (density, near) x N            (wgsl:58)  */
  RPS_DEBUG_PREDICTED = 19,       /* f32x2 x N                            (wgsl:61)  */
  RPS_DEBUG_ACCEL_X = 20,         /* f32 x N  N-body acceleration (build-defined)    */
  RPS_DEBUG_ACCEL_Y = 21,         /* f32 x N                                          */
  RPS_DEBUG_EXPIRY = 22           /* u16 x N  lifetime expiry (STREAM) */
} rps_field;

typedef struct rps_stats {
  float bbox[4];          /* x_min, x_max, y_min, y_max over live particles               */
  double kinetic_energy;  /* sum 0.5 |v|^2                                                */
  uint64_t particles;     /* particles reduced                                            */
  uint64_t respawned;     /* respawns in the reduced step                                 */
  uint64_t step;          /* active-step index the stats belong to                        */
} rps_stats;

/* Library / device introspection. */
uint32_t rps_abi_version(void);
/* Build provenance (no reference counterpart): the first 16 hex digits of the sha256 of the
 * sources the library was compiled from (rust-particle-system_amd/Makefile, BUILD_ID). */
const char* rps_build_id(void);
const char* rps_status_string(int status);
int rps_device_count(int* count);

/* Replaces prepare_particle_buffers' first-frame branch (src/particle_buffers.rs:50-216):
 * hipMalloc SoA state + aux buffers for `info->mode`; zero-initialised like wgpu buffers. */
int rps_create(const rps_create_info* info, rps_ctx** out);
/* Device buffers in the reference live for the app's lifetime; here they are freed. */
int rps_destroy(rps_ctx* ctx);
const char* rps_last_error(const rps_ctx* ctx);

/* == write_buffer(config, 144 B) (src/particle_buffers.rs:230-236): the config is written
 * into the device-resident copy by a kernel on the context stream (ordered before the next
 * rps_step; the caller's struct may be reused at once).  ext may be NULL (reference semantics:
 * Euler, no attractors, no drag, no lifetime, shader_delay 5). */
int rps_set_config(rps_ctx* ctx, const rps_config* cfg, const rps_ext_config* ext);
int rps_get_config(const rps_ctx* ctx, rps_config* cfg, rps_ext_config* ext);

/* == create_buffer_with_data(particles) (src/particle_buffers.rs:60-78): AoS upload,
 * transposed to SoA on the device.  Writes particles [offset, offset+n) of this context. */
int rps_upload_particles(rps_ctx* ctx, const rps_particle* aos, uint64_t offset, uint64_t n);
/* SoA -> AoS download; colour derived from velocity exactly as set_color (wgsl:101-118),
 * or the spawn colour (1,1,1,1) (src/main.rs:210) before the first active step. */
int rps_download_particles(rps_ctx* ctx, rps_particle* aos, uint64_t offset, uint64_t n);
/* Render interop: the reference's vertex shader reads the 32-B Particle storage buffer
 * (render_shader.wgsl:26-30, :44-45, :57).  Writes particles [offset, offset+n) in that AoS
 * layout (colour derived exactly as set_color, wgsl:101-118) into DEVICE memory `device_dst`
 * on the context's device, ordered on the context stream, with no host round trip. */
int rps_export_particles(rps_ctx* ctx, rps_particle* device_dst, uint64_t offset, uint64_t n);
/* Raw SoA field transfers (float32), for checkpoint/resume.  The lifetime (STREAM) is not
 * stored as seconds: each particle keeps a u16 expiry e, the lifetime-clock value c (= active
 * steps run with RPS_EXT_LIFETIME on) of the step in which it respawns, so it has
 * (u16)(e - c) + 1 steps left.  RPS_FIELD_LIFE_STEPS reads that count (exact; checkpoints) and
 * writes e = c + clamp(ceil(v), 1, 65535) - 1; RPS_FIELD_LIFE reads steps * dt seconds and
 * writes L seconds as clamp(ceil(L / dt), 1, 65535) steps. */
int rps_upload_field(rps_ctx* ctx, int field, const float* src, uint64_t offset, uint64_t n);
int rps_download_field(rps_ctx* ctx, int field, float* dst, uint64_t offset, uint64_t n);
/* Debug readback of SPH intermediates (src/debug.rs:121-265); bytes must equal the buffer. */
int rps_read_debug(rps_ctx* ctx, int which, void* dst, uint64_t bytes);

/* Device-side initial scatter, a seeded restatement of setup_particles_scatter
 * (src/main.rs:182-216): x linear in the global id, y ~ Normal(centre, 0.125 H) clamped,
 * v = 0, life ~ U(life_min, life_max) (kept as an expiry, see RPS_FIELD_LIFE).  Uses the
 * current config's screen_bounds. */
int rps_init_scatter(rps_ctx* ctx, uint64_t seed);

/* == ParticleComputeNode::run (src/particle_compute.rs:91-195), nsteps times.  Each step
 * first advances frame_count (src/particle_buffers.rs:227) and then records the mode's
 * kernels on the context stream; steps with frame_count < shader_delay only bin/sort in
 * SPH mode and do nothing in the other modes (wgsl:426, :442).  Asynchronous. */
int rps_step(rps_ctx* ctx, uint32_t nsteps);
/* == update (src/particle_compute.rs:197-199): no device work; kept for API parity. */
int rps_update(rps_ctx* ctx);
int rps_sync(rps_ctx* ctx);

/* Stats of the most recent reduced step (requires RPS_EXT_STATS); blocks.  With a
 * communicator (rps_comm_init, STREAM mode) they cover every rank's shard: each stats step
 * all-reduces bbox min/max and the KE / particle / respawn sums over the ranks (RCCL). */
int rps_get_stats(rps_ctx* ctx, rps_stats* out);
/* The same stats step over this rank's shard only (no reduction over the ranks), so a host
 * can check the library's RCCL all-reduce against its own transport (bench.py). */
int rps_get_shard_stats(rps_ctx* ctx, rps_stats* out);

/* Host-visible counters: frame_count of the device config and active steps executed. */
int rps_get_counters(const rps_ctx* ctx, uint32_t* frame_count, uint64_t* active_steps);

/* Per-launch kernel timing with HIP events on the context stream (for bench.py):
 * period 0 = off, k > 0 = bracket every k-th launch of the mode's dominant kernel (stream
 * step / N-body force / SPH simulation pass) with an event pair.  Stream steps that also
 * fuse the stats reduction are a different kernel variant and are not sampled. */
int rps_set_profiling(rps_ctx* ctx, int period);
/* Average duration (ms) and count of the bracketed dominant-kernel launches since profiling
 * was enabled; blocks until they completed. */
int rps_get_kernel_time(rps_ctx* ctx, double* avg_ms, uint64_t* launches);
/* The same launches one by one: the durations (ms, launch order) of up to `cap` of the
 * bracketed launches since profiling was enabled, and their total count; blocks until they
 * completed, and starts a new collection like rps_get_kernel_time. */
int rps_get_kernel_times(rps_ctx* ctx, double* ms, uint64_t cap, uint64_t* launches);
/* N-body: the shader clock the chip sustained during the most recent profiled force launch
 * (median over its workgroups of delta s_memtime / delta s_memrealtime x 100 MHz, stamped at
 * each workgroup's start and end), in MHz, and the number of workgroups it is the median of.
 * RPS_ERR_UNSUPPORTED before a profiled launch or outside N-body mode.  For reporting FP32
 * fractions against the clock actually held (MI355X peaks assume 2400 MHz). */
int rps_get_kernel_clock(rps_ctx* ctx, double* mhz, uint64_t* workgroups);
/* Time nsteps rps_step calls with a pair of HIP events on the context stream. */
int rps_time_steps(rps_ctx* ctx, uint32_t nsteps, double* total_ms);
/* The context's hipStream_t (as void*), for callers that interoperate on the same stream. */
void* rps_get_stream(rps_ctx* ctx);

/* Algorithmic HBM bytes (stream/SPH) or flops (N-body) one step moves for this context's
 * mode/config; `unit` receives 0 for bytes, 1 for flops.  SPH: the frame's
 * bytes of rps_sph_frame_cost, which launches a counting kernel on the context stream and
 * waits for it (so the context is not const; RPS_ERR_UNSUPPORTED unless the most recent
 * frame was active).  STREAM / N-body: host arithmetic only. */
int rps_step_cost(rps_ctx* ctx, double* amount, int* unit);

/* SPH frame cost, for rooflines: the algorithmic bytes of one active frame
 * of the current state.  E = neighbour entries the reference's scans visit (the nine runs of
 * every lookup slot's particle, wgsl:207-254 / :279-384), counted on the device; per kernel:
 *   sort     launches x P x 16 B (each launch reads and writes the 8-B lookup) + N x 8 B bin
 *   predict  P x 60 B (lookup, gathered state, slot records) + N x 8 B (offsets, ends)
 *   density  E x 8 B (neighbour predicted position) + P x 120 B (runs, own record, outputs)
 *   sim      E x 32 B (pressure {pos, P/rho^2, Pn/(rho rho_n)} + viscosity {pos, v} records)
 *            + P x 156 B (runs, masks, own records, state write)
 * The scans' neighbour records are re-read E/P times per frame and served by the caches, so
 * their roofline is the aggregate L2 bandwidth, not HBM.  Counts the most recent frame's
 * runs, which must have been active (RPS_ERR_UNSUPPORTED otherwise: a gated frame re-sorts
 * the lookup but keeps older predictions): launches a counting kernel on the context stream
 * into a buffer allocated at rps_create and waits for it (not for timed regions).  SPH only. */
typedef struct rps_sph_cost {
  uint64_t slots;            /* P = next_pow2(N) */
  uint64_t particles;        /* N */
  uint64_t scanned_entries;  /* E */
  uint64_t within_entries;   /* of E, within the smoothing radius (self included) */
  uint64_t sort_launches;
  double sort_bytes, predict_bytes, density_bytes, sim_bytes, frame_bytes;
} rps_sph_cost;
int rps_sph_frame_cost(rps_ctx* ctx, rps_sph_cost* out);

/* Multi-GPU: RCCL communicator over this rank's context.  N-body needs it (all-gather of
 * positions); STREAM uses it only for the all-rank stats (rps_get_stats).
 * unique_id is the 128-byte ncclUniqueId produced by rps_comm_unique_id on rank 0. */
int rps_comm_unique_id(void* out128);
/* N-body sources: the device array of float2 positions of ALL global particles (global_count
 * entries; this shard's at [id_offset, id_offset + n)).  pack != 0 first writes this shard's
 * current positions into it (and waits for that).  With RPS_EXT_NBODY_EXTERNAL set, rps_step
 * skips its own pack + ncclAllGather and uses the array as the caller left it, so a host can
 * exchange shards with any transport (peer copies, MPI, host staging). */
int rps_nbody_sources(rps_ctx* ctx, int pack, void** sources, uint64_t* count);
int rps_comm_init(rps_ctx* ctx, int rank, int nranks, const void* unique_id128);

#ifdef __cplusplus
}
#endif

#endif /* RPS_H_ */
