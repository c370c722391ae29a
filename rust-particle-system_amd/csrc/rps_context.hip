// rps_context.hip — implementation of the C ABI declared in include/rps.h.
//
// Replaces, for the hot path only:
//   prepare_particle_buffers   (src/particle_buffers.rs:38-237)  -> rps_create / rps_set_config
//   ParticleComputeNode::run    (src/particle_compute.rs:91-195)  -> rps_step
//   ParticleComputeNode::update (src/particle_compute.rs:197-199) -> rps_update
//   read_*_from_gpu             (src/debug.rs:121-265)           -> rps_read_debug
// Device state is SoA in one hipMalloc arena; every call is ordered on the
// context's own HIP stream.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "rps_internal.hpp"

using namespace rps;

struct rps_ctx {
  int device = 0;
  uint32_t mode = RPS_MODE_STREAM;
  uint64_t n = 0, id_offset = 0, global_count = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev_begin = nullptr, ev_end = nullptr;  // rps_time_steps (created with the stream)

  rps_config cfg{};
  rps_ext_config ext{};
  bool have_config = false;

  char* arena = nullptr;
  size_t arena_bytes = 0;
  Layout layout = plain_layout();  // tiled for STREAM (rps_device.hpp)
  Layout exp_layout = plain_layout();
  float* state = nullptr;          // STREAM: the tiled x|y|vx|vy|expiry block
  float *x = nullptr, *y = nullptr, *vx = nullptr, *vy = nullptr;
  uint16_t* exp = nullptr;         // STREAM: lifetime expiry (u16)
  uint16_t* next = nullptr;        // STREAM: per-quad earliest expiry (rps_device.hpp)
  // SPH: packed {x, y, vx, vy} state (x..vy point into st, layout sph_layout())
  f4* st = nullptr;
  SphSlots sl{};           // SPH slot records (rps_internal.hpp)
  uint32_t* ends = nullptr;
  uint2* lookup = nullptr;
  uint32_t* offsets = nullptr;
  f2* dens = nullptr;
  f2* pred = nullptr;
  uint32_t P = 0;
  uint32_t sort_passes = 0, sort_launches = 0;
  bool sort_fold = true;  // RPS_SPH_SORT_FOLD (rps_kernels.hip, launch_sph_sort)
  bool csort = true;      // RPS_SPH_CSORT: the compact sort at 2^11 <= P <= 2^16
  uint8_t csort_tlog = 0; // RPS_SPH_CSORT_TLOG (11..13; 0: by size)
  uint8_t csort_wide = 4; // RPS_SPH_CSORT_WIDE
  uint32_t pair_max_p = 0; // RPS_SPH_PAIRS: lane-pair scans up to this P
  bool sim_fuse = true;    // RPS_SPH_SIM_FUSE: the sim and its long scans in one launch
  uint8_t lane_group = 2;  // RPS_SPH_GROUP: lanes per slot of the small-P scans (2 or 4)
  uint8_t lane_group_s = 2;  // RPS_SPH_GROUP_S: the sim's (default: lane_group)
  uint8_t sph_batch_d = 0, sph_batch_s = 0;  // forced scan batches (0: by size)
  SphLayoutArgs lay{};     // spatial record layout (RPS_SPH_LAYOUT, P >= 2^20 by default): arrays
  uint32_t cell_cap = 0;   // their cell capacity (0: no layout)
  uint8_t* own_buf = nullptr;  // P != N with the layout: SphSlots::own_s of resident frames
  bool layout_last = false;  // the last active frame used the layout (slot records in storage order)
  bool last_frame_active = false;  // the most recent frame ran passes 4-5 (rps_sph_frame_cost)
  unsigned long long* d_count = nullptr;  // rps_sph_frame_cost's per-workgroup counts (SPH)
  // Slot-resident state (layout frames): after a layout frame st holds the
  // state in that frame's storage order, perm = sl.idx_s (slot -> particle), and bin_next the
  // next frame's bin entries.  Every API call that reads or writes particles in particle order
  // first puts the state back (sph_canonical).
  f4* st_alt = nullptr;         // particle-order target of sph_canonical (swapped with st)
  uint32_t* idx_alt = nullptr;  // the other slot -> particle buffer (alternates with sl.idx_s)
  uint2* bin_next = nullptr;
  bool resident = false;
  bool keys_valid = false;      // bin_next matches st and the current config
  bool pkeys_valid = false;     // bin_next = (key, i) of the particle-order state (no layout)
  const uint32_t* lookup_perm = nullptr;  // the lookup's payloads are slots of this perm
  // N-body
  f2* pos_all = nullptr;
  uint64_t ns_padded = 0;
  float *ax = nullptr, *ay = nullptr;
  f2* nb_part = nullptr;  // N-body source-split partials (nb_splits x n float2)
  uint32_t nb_splits = 0;  // source splits of the force launch (RPS_NBODY_SPLITS overrides)
  uint64_t* nb_stamps = nullptr;  // profiled force launches: per-workgroup clock stamps
  uint64_t nb_stamp_wgs = 0;      // workgroups of the last stamped launch (0: none yet)
  // device config (rps_set_config writes it on the stream: config_store_kernel)
  rps_config* d_cfg = nullptr;
  // stats
  StatsPartial* partials = nullptr;
  uint32_t partial_cap = 0;
  StatsResult* d_stats = nullptr;
  StatsGlobal* d_gstats = nullptr;  // all-rank stats (with a communicator)
  bool have_stats = false;
  // staging for AoS transfers
  rps_particle* d_staging = nullptr;
  uint64_t staging_cap = 0;
  // counters
  uint64_t active_steps = 0;
  uint64_t life_clock = 0;  // active steps run with RPS_EXT_LIFETIME on (the expiry clock)
  bool stepped = false;
  // profiling
  uint32_t profile_every = 0;  // 0: off; k: events around every k-th dominant launch
  uint64_t profile_seq = 0;
  bool profile_open = false;
  std::vector<hipEvent_t> ev_start, ev_stop;
  size_t ev_used = 0;
  int nontemporal = 3;  // stream cache policy (stream_nt_default)
  // comm
  ncclComm_t comm = nullptr;
  int rank = 0, nranks = 1;

  std::string err;
};

namespace {

thread_local std::string g_err;

int fail(rps_ctx* ctx, int code, const std::string& msg) {
  if (ctx)
    ctx->err = msg;
  else
    g_err = msg;
  return code;
}

#define RPS_HIP(ctx, call)                                                                   \
  do {                                                                                       \
    hipError_t e_ = (call);                                                                  \
    if (e_ != hipSuccess)                                                                    \
      return fail((ctx), e_ == hipErrorOutOfMemory ? RPS_ERR_OUT_OF_MEMORY : RPS_ERR_DEVICE, \
                  std::string(#call) + ": " + hipGetErrorString(e_));                        \
  } while (0)

size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

uint32_t next_pow2_u32(uint32_t n) {
  uint32_t p = 1;
  while (p < n) p <<= 1;
  return p;
}

rps_ext_config default_ext() {
  rps_ext_config e;
  std::memset(&e, 0, sizeof(e));
  e.integrator = RPS_INTEGRATOR_EULER;
  e.shader_delay = 5;  // SHADER_DELAY, compute_shader.wgsl:66
  e.stats_interval = 1;
  return e;
}

// Attractor position at time t; same formula as oracle/rps_oracle.c orc_attractor_pos.
void attractor_pos(const rps_attractor& a, double t, float& px, float& py) {
  const double ang = (double)a.angular_velocity * t + (double)a.phase;
  px = (float)((double)a.center[0] + (double)a.orbit_radius * std::cos(ang));
  py = (float)((double)a.center[1] + (double)a.orbit_radius * std::sin(ang));
}

int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return v && *v ? std::atoi(v) : dflt;
}

// Default cache policy of the stream step (bit 0 nontemporal loads, bit 1 nontemporal
// stores) from the 32 B/particle of state the step streams.  Nontemporal stores always;
// loads temporal while the state is within about twice the 256-MB Infinity Cache (MALL),
// which then still serves part of each step's reads.  Same box, C2 ext, us/step, both
// nontemporal vs temporal loads (round 2, tools/ab_stream.py with the since-removed NT knob):
//   2^20 (32 MiB) 6.00 / 6.44     2^21 11.25 / 9.48     2^22 22.37 / 21.29
//   2^23 42.89 / 39.38            2^24 (512 MiB) 82.48 / 75.03
//   20 Mi (640 MiB) 102.8 / 107.0 24 Mi 122.3 / 131.3   2^25 162.1 / 176.0   1e8 479 / 522
int stream_nt_default(uint64_t n) {
  const uint64_t bytes = n * 32;
  return (bytes > (48ull << 20) && bytes <= (576ull << 20)) ? 2 : 3;
}

int check_ctx(rps_ctx* ctx) {
  if (!ctx) return fail(nullptr, RPS_ERR_INVALID_ARGUMENT, "null context");
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return fail(ctx, RPS_ERR_DEVICE, std::string("hipSetDevice: ") + hipGetErrorString(e));
  return RPS_OK;
}

Fields fields(const rps_ctx* ctx) {
  return Fields{ctx->x, ctx->y, ctx->vx, ctx->vy, ctx->exp};
}

float* field_ptr(rps_ctx* ctx, int field) {
  switch (field) {
    case RPS_FIELD_X: return ctx->x;
    case RPS_FIELD_Y: return ctx->y;
    case RPS_FIELD_VX: return ctx->vx;
    case RPS_FIELD_VY: return ctx->vy;
    default: return nullptr;
  }
}

int ensure_staging(rps_ctx* ctx, uint64_t want) {
  if (ctx->staging_cap >= want) return RPS_OK;
  if (ctx->d_staging) RPS_HIP(ctx, hipFree(ctx->d_staging));
  ctx->d_staging = nullptr;
  ctx->staging_cap = 0;
  RPS_HIP(ctx, hipMalloc(&ctx->d_staging, want * sizeof(rps_particle)));
  ctx->staging_cap = want;
  return RPS_OK;
}

constexpr uint64_t kStagingChunk = 1ull << 21;  // 2 Mi particles = 64 MiB of AoS per chunk

StreamArgs make_stream_args(const rps_ctx* ctx, uint64_t k) {
  StreamArgs a;
  std::memset(&a, 0, sizeof(a));
  const rps_config& c = ctx->cfg;
  const rps_ext_config& e = ctx->ext;
  a.x = ctx->x;
  a.y = ctx->y;
  a.vx = ctx->vx;
  a.vy = ctx->vy;
  a.exp = ctx->exp;
  a.next = ctx->next;
  a.clock = (uint32_t)ctx->life_clock;
  a.partials = ctx->partials;
  a.n = ctx->n;
  a.id_offset = ctx->id_offset;
  const float dt = c.fixed_delta_time;
  a.dt = dt;
  a.gx_dt = 0.0f * dt;  // vec2(0.0, -gravity) * dt, compute_shader.wgsl:399
  a.gy_dt = (-c.gravity) * dt;
  a.neg_g = -c.gravity;
  a.half_dt = 0.5f * dt;
  a.half_dt2 = (0.5f * dt) * dt;
  a.drag_on = e.drag != 0.0f;
  a.drag_f = 1.0f - e.drag * dt;
  a.na = std::min<uint32_t>(e.num_attractors, RPS_MAX_ATTRACTORS);
  const double t = (double)k * (double)dt;
  for (uint32_t i = 0; i < a.na; ++i) {
    float px, py;
    attractor_pos(e.attractors[i], t, px, py);
    a.att[i] = f4{px, py, e.attractors[i].strength,
                  e.attractors[i].softening * e.attractors[i].softening};
  }
  a.x_min = c.screen_bounds[0];
  a.x_max = c.screen_bounds[1];
  a.y_min = c.screen_bounds[2];
  a.y_max = c.screen_bounds[3];
  a.damping = c.damping_factor;
  a.emit_cx = e.emitter_center[0];
  a.emit_cy = e.emitter_center[1];
  a.emit_r = e.emitter_radius;
  a.spd_min = e.spawn_speed_min;
  a.spd_range = e.spawn_speed_max - e.spawn_speed_min;
  a.life_min = e.life_min;
  a.life_range = e.life_max - e.life_min;
  a.key0 = (uint32_t)e.seed;
  a.key1 = (uint32_t)(e.seed >> 32);
  a.step_lo = (uint32_t)k;
  a.step_hi = (uint32_t)(k >> 32);
  return a;
}

// `sampled` = false for launches that are a different kernel variant than the dominant one
// (the stats-fused stream step every stats_interval steps), so the average matches the
// rocprofv3 per-kernel figure of the dominant kernel.
int prof_begin(rps_ctx* ctx, bool sampled = true) {
  ctx->profile_open = sampled && ctx->profile_every && (ctx->profile_seq++ % ctx->profile_every == 0);
  if (!ctx->profile_open) return RPS_OK;
  if (ctx->ev_used == ctx->ev_start.size()) {
    hipEvent_t a, b;
    RPS_HIP(ctx, hipEventCreate(&a));
    RPS_HIP(ctx, hipEventCreate(&b));
    ctx->ev_start.push_back(a);
    ctx->ev_stop.push_back(b);
  }
  RPS_HIP(ctx, hipEventRecord(ctx->ev_start[ctx->ev_used], ctx->stream));
  return RPS_OK;
}

int prof_end(rps_ctx* ctx) {
  if (!ctx->profile_open) return RPS_OK;
  ctx->profile_open = false;
  RPS_HIP(ctx, hipEventRecord(ctx->ev_stop[ctx->ev_used], ctx->stream));
  ++ctx->ev_used;
  return RPS_OK;
}

// SPH state: packed float4 per particle, so the field views are a layout (offset 4i).
Layout sph_layout() { return Layout{0, 4, 0}; }

void set_sph_fields(rps_ctx* ctx) {
  float* base = reinterpret_cast<float*>(ctx->st);
  ctx->x = base;
  ctx->y = base + 1;
  ctx->vx = base + 2;
  ctx->vy = base + 3;
}

SphBuffers sph_buffers(rps_ctx* ctx) {
  SphBuffers b;
  b.cfg = ctx->d_cfg;
  b.st = ctx->st;
  b.bin_next = ctx->bin_next;
  b.idx_prev = ctx->idx_alt;  // during a resident frame: the perm its sort payloads refer to
  b.resident = ctx->resident;
  b.pkeys = ctx->pkeys_valid;
  b.sl = ctx->sl;
  b.ends = ctx->ends;
  b.lookup = ctx->lookup;
  b.offsets = ctx->offsets;
  b.dens = ctx->dens;
  b.pred = ctx->pred;
  b.n = (uint32_t)ctx->n;
  b.p = ctx->P;
  b.batch_d = ctx->sph_batch_d;
  b.batch_s = ctx->sph_batch_s;
  b.lay = ctx->lay;
  b.cell_cap = ctx->cell_cap;
  b.layout = ctx->layout_last;
  b.sort_fold = ctx->sort_fold;
  b.csort = ctx->csort;
  b.csort_tlog = ctx->csort_tlog;
  b.csort_wide = ctx->csort_wide;
  b.pair_max_p = ctx->pair_max_p;
  b.sim_fuse = ctx->sim_fuse;
  b.lane_group = ctx->lane_group;
  b.lane_group_s = ctx->lane_group_s;
  return b;
}

// Sharded STREAM runs with a communicator: the stats of a stats step over all ranks, two
// in-place all-reduces of 16 + 24 bytes on the context stream (MAX of the bbox terms, SUM of
// KE and counts), amortised over stats_interval steps.
int allreduce_stats(rps_ctx* ctx) {
  if (!ctx->comm) return RPS_OK;
  ncclResult_t r = ncclAllReduce(ctx->d_gstats->neg_min_max, ctx->d_gstats->neg_min_max, 4, ncclFloat,
                                 ncclMax, ctx->comm, ctx->stream);
  if (r == ncclSuccess)
    r = ncclAllReduce(ctx->d_gstats->sums, ctx->d_gstats->sums, 3, ncclDouble, ncclSum, ctx->comm,
                      ctx->stream);
  if (r != ncclSuccess) return fail(ctx, RPS_ERR_COMM, std::string("ncclAllReduce(stats): ") + ncclGetErrorString(r));
  return RPS_OK;
}

int step_stream(rps_ctx* ctx) {
  const uint64_t k = ctx->active_steps;
  const rps_ext_config& e = ctx->ext;
  const bool stats = (e.flags & RPS_EXT_STATS) && (k % std::max<uint32_t>(e.stats_interval, 1u) == 0);
  StreamArgs a = make_stream_args(ctx, k);
  StreamLaunch l;
  l.verlet = e.integrator == RPS_INTEGRATOR_VERLET;
  l.lifetime = (e.flags & RPS_EXT_LIFETIME) != 0;
  l.stats = stats;
  l.nontemporal = ctx->nontemporal;
  l.grid = stream_blocks_for(ctx->n);
  if (stats && l.grid > ctx->partial_cap) {
    if (ctx->partials) RPS_HIP(ctx, hipFree(ctx->partials));
    ctx->partials = nullptr;
    RPS_HIP(ctx, hipMalloc(&ctx->partials, sizeof(StatsPartial) * (l.grid + kStatsFold)));
    ctx->partial_cap = l.grid;
    a.partials = ctx->partials;
  }
  int rc = prof_begin(ctx, !stats);
  if (rc) return rc;
  RPS_HIP(ctx, launch_stream_step(a, l, ctx->stream));
  rc = prof_end(ctx);
  if (rc) return rc;
  if (stats) {
    RPS_HIP(ctx, launch_stats_finalize(ctx->partials, l.grid, ctx->partials + ctx->partial_cap,
                                       ctx->d_stats, ctx->comm ? ctx->d_gstats : nullptr, k, ctx->stream));
    rc = allreduce_stats(ctx);
    if (rc) return rc;
    ctx->have_stats = true;
  }
  return RPS_OK;
}

// Temporal fusion (ext.fuse_steps > 1): `m` consecutive active steps starting at active-step
// index k0 in one launch; `stats` reduces the state after the last of them.
int step_stream_fused(rps_ctx* ctx, uint64_t k0, uint32_t m, bool stats, uint64_t clock0) {
  const rps_ext_config& e = ctx->ext;
  FusedArgs fa;
  std::memset(&fa, 0, sizeof(fa));
  fa.base = make_stream_args(ctx, k0);
  fa.base.clock = (uint32_t)clock0;
  fa.nsub = m;
  const double dt = (double)ctx->cfg.fixed_delta_time;
  for (uint32_t sub = 0; sub < m; ++sub)
    for (uint32_t i = 0; i < fa.base.na; ++i) {
      float px, py;
      attractor_pos(e.attractors[i], (double)(k0 + sub) * dt, px, py);
      fa.att[sub][i] = f4{px, py, fa.base.att[i][2], fa.base.att[i][3]};
    }
  StreamLaunch l;
  l.verlet = e.integrator == RPS_INTEGRATOR_VERLET;
  l.lifetime = (e.flags & RPS_EXT_LIFETIME) != 0;
  l.stats = stats;
  l.nontemporal = 3;
  l.grid = stream_blocks_for(ctx->n);
  if (stats && l.grid > ctx->partial_cap) {
    if (ctx->partials) RPS_HIP(ctx, hipFree(ctx->partials));
    ctx->partials = nullptr;
    RPS_HIP(ctx, hipMalloc(&ctx->partials, sizeof(StatsPartial) * (l.grid + kStatsFold)));
    ctx->partial_cap = l.grid;
  }
  fa.base.partials = ctx->partials;
  int rc = prof_begin(ctx, !stats);
  if (rc) return rc;
  RPS_HIP(ctx, launch_stream_fused(fa, l, ctx->stream));
  rc = prof_end(ctx);
  if (rc) return rc;
  if (stats) {
    RPS_HIP(ctx, launch_stats_finalize(ctx->partials, l.grid, ctx->partials + ctx->partial_cap,
                                       ctx->d_stats, ctx->comm ? ctx->d_gstats : nullptr, k0 + m - 1,
                                       ctx->stream));
    rc = allreduce_stats(ctx);
    if (rc) return rc;
    ctx->have_stats = true;
  }
  return RPS_OK;
}

int step_nbody(rps_ctx* ctx) {
  const rps_config& c = ctx->cfg;
  const rps_ext_config& e = ctx->ext;
  const bool external = (e.flags & RPS_EXT_NBODY_EXTERNAL) != 0;
  // External exchange: the caller packed (rps_nbody_pack) and filled the other shards.
  if (!external)
    RPS_HIP(ctx, launch_nbody_pack(ctx->x, ctx->y, ctx->pos_all + ctx->id_offset, ctx->n, ctx->stream));
  if (ctx->comm && !external) {
    // In-place all-gather of every rank's float2 positions over xGMI; with one
    // rank RCCL leaves the array as it is.
    ncclResult_t r = ncclAllGather(ctx->pos_all + ctx->id_offset, ctx->pos_all, ctx->n * 2,
                                   ncclFloat, ctx->comm, ctx->stream);
    if (r != ncclSuccess)
      return fail(ctx, RPS_ERR_COMM, std::string("ncclAllGather: ") + ncclGetErrorString(r));
  }
  const float eps2 = e.nbody_softening * e.nbody_softening;
  int rc = prof_begin(ctx);
  if (rc) return rc;
  uint64_t* stamps = ctx->profile_open ? ctx->nb_stamps : nullptr;
  RPS_HIP(ctx, launch_nbody_accel(ctx->pos_all, ctx->ns_padded, ctx->id_offset, ctx->n, eps2,
                                  e.nbody_strength, ctx->nb_part, ctx->nb_splits, ctx->ax, ctx->ay,
                                  stamps, ctx->stream));
  if (stamps) ctx->nb_stamp_wgs = nbody_workgroups(ctx->n, ctx->ns_padded, ctx->nb_splits);
  rc = prof_end(ctx);
  if (rc) return rc;
  NbodyIntegrateArgs ia;
  ia.x = ctx->x;
  ia.y = ctx->y;
  ia.vx = ctx->vx;
  ia.vy = ctx->vy;
  ia.ax = ctx->ax;
  ia.ay = ctx->ay;
  ia.n = ctx->n;
  ia.dt = c.fixed_delta_time;
  ia.gx_dt = 0.0f * c.fixed_delta_time;
  ia.gy_dt = (-c.gravity) * c.fixed_delta_time;
  ia.drag_on = e.drag != 0.0f;
  ia.drag_f = 1.0f - e.drag * c.fixed_delta_time;
  ia.x_min = c.screen_bounds[0];
  ia.x_max = c.screen_bounds[1];
  ia.y_min = c.screen_bounds[2];
  ia.y_max = c.screen_bounds[3];
  ia.damping = c.damping_factor;
  RPS_HIP(ctx, launch_nbody_integrate(ia, ctx->stream));
  return RPS_OK;
}

// Passes 1-3.  On an active frame the offsets pass (3) rides in pass 4's first kernel
// instead (the layout's runs kernel, or predict): nothing between them reads offsets/ends.
int step_sph_grid(rps_ctx* ctx, bool active) {
  SphBuffers b = sph_buffers(ctx);
  RPS_HIP(ctx, launch_sph_sort(b, ctx->stream, &ctx->sort_passes, &ctx->sort_launches));
  if (!active) RPS_HIP(ctx, launch_sph_offsets(b, ctx->stream));
  return RPS_OK;
}

// The state back in particle order (st_alt[perm[u]] = st[u], then the buffers swap).
int sph_canonical(rps_ctx* ctx) {
  if (!ctx->resident) return RPS_OK;
  const SphBuffers b = sph_buffers(ctx);
  RPS_HIP(ctx, launch_sph_materialize(b, ctx->st, ctx->sl.idx_s, ctx->st_alt, ctx->stream));
  // The lookup's payloads back to particle indices (slots of lookup_perm; P != N: flagged pads).
  RPS_HIP(ctx, launch_sph_lookup_canonical(b, ctx->lookup_perm, ctx->stream));
  ctx->lookup_perm = nullptr;
  std::swap(ctx->st, ctx->st_alt);
  set_sph_fields(ctx);
  ctx->resident = false;
  ctx->keys_valid = false;
  ctx->pkeys_valid = false;
  return RPS_OK;
}

// Before a frame's passes 1-3: a frame that does not use the layout needs particle order; a
// resident frame whose bin entries are stale (config changed) rebuilds them from the state;
// a resident frame writes its slot -> particle map to the other buffer (the sort payloads
// refer to the current one).
int sph_frame_begin(rps_ctx* ctx, bool layout) {
  // Every path out of the slot-resident state runs sph_canonical, which also turns the lookup's
  // payloads back into particle indices: the compact sort's 16-bit payloads (csort_ok) rely on
  // it for P != N, so a broken invariant fails here instead of sorting truncated payloads.
  if (!ctx->resident && ctx->lookup_perm)
    return fail(ctx, RPS_ERR_DEVICE, "internal: lookup payloads left slot-resident outside a resident frame");
  if (ctx->resident && !layout) {
    const int rc = sph_canonical(ctx);
    if (rc) return rc;
  }
  if (ctx->resident && !ctx->keys_valid) {
    RPS_HIP(ctx, launch_sph_rebin(sph_buffers(ctx), ctx->sl.idx_s, ctx->stream));
    ctx->keys_valid = true;
  }
  ctx->lookup_perm = ctx->resident ? ctx->sl.idx_s : nullptr;
  if (ctx->resident) std::swap(ctx->sl.idx_s, ctx->idx_alt);
  return RPS_OK;
}

int step_sph_sim(rps_ctx* ctx, bool layout, const SphGrid& g) {
  ctx->layout_last = layout;
  if (layout) {
    ctx->lay.g = g;
    // cell_info and key_cell records carry the build's epoch (the arena's zeros are epoch 0); at
    // the wrap the old records are cleared so none can match a reused epoch
    if (++ctx->lay.epoch >= (1u << 24)) {
      RPS_HIP(ctx, hipMemsetAsync(ctx->lay.cell_info, 0, (size_t)ctx->cell_cap * sizeof(uint4), ctx->stream));
      RPS_HIP(ctx, hipMemsetAsync(ctx->lay.key_cell, 0, (size_t)ctx->n * sizeof(uint2), ctx->stream));
      ctx->lay.epoch = 1;
    }
  }
  ++ctx->sl.owner_epoch;  // this active frame's owner claims (SphSlots::owner)
  // P != N: a slot-resident layout frame's owners are its unflagged entries (SphSlots::own_s)
  ctx->sl.own_s = ctx->own_buf && layout && ctx->resident ? ctx->own_buf : nullptr;
  SphBuffers b = sph_buffers(ctx);
  if (layout)
    RPS_HIP(ctx, launch_sph_layout_pre(b, ctx->stream));
  else
    RPS_HIP(ctx, launch_sph_pre(b, ctx->stream));
  int rc = prof_begin(ctx);
  if (rc) return rc;
  RPS_HIP(ctx, launch_sph_sim(b, ctx->stream));
  rc = prof_end(ctx);
  if (rc) return rc;
  if (layout) {  // the sim wrote st in this frame's slot order and the next bin entries
    ctx->resident = true;
    ctx->keys_valid = true;
  }
  ctx->pkeys_valid = !layout;  // else the sim wrote (key, i) for the next frame
  return RPS_OK;
}

}  // namespace

extern "C" {

uint32_t rps_abi_version(void) { return RPS_ABI_VERSION; }

#ifndef RPS_BUILD_ID
#define RPS_BUILD_ID "unknown"
#endif
const char* rps_build_id(void) { return RPS_BUILD_ID; }

const char* rps_status_string(int status) {
  switch (status) {
    case RPS_OK: return "ok";
    case RPS_ERR_INVALID_ARGUMENT: return "invalid argument";
    case RPS_ERR_DEVICE: return "device error";
    case RPS_ERR_OUT_OF_MEMORY: return "out of memory";
    case RPS_ERR_UNSUPPORTED: return "unsupported";
    case RPS_ERR_COMM: return "communication error";
    case RPS_ERR_NO_DEVICE: return "no device";
    default: return "unknown status";
  }
}

int rps_device_count(int* count) {
  if (!count) return fail(nullptr, RPS_ERR_INVALID_ARGUMENT, "null count");
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) {
    *count = 0;
    return fail(nullptr, RPS_ERR_NO_DEVICE, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
  }
  *count = c;
  return RPS_OK;
}

const char* rps_last_error(const rps_ctx* ctx) { return ctx ? ctx->err.c_str() : g_err.c_str(); }

int rps_create(const rps_create_info* info, rps_ctx** out) {
  if (!info || !out) return fail(nullptr, RPS_ERR_INVALID_ARGUMENT, "null argument");
  *out = nullptr;
  if (info->mode > RPS_MODE_SPH) return fail(nullptr, RPS_ERR_INVALID_ARGUMENT, "bad mode");
  // NonZeroU64::new(particle_buffer_size).unwrap() (src/particle_buffers.rs:73-74)
  if (info->particle_count == 0) return fail(nullptr, RPS_ERR_INVALID_ARGUMENT, "particle_count must be > 0");
  const uint64_t global = info->global_count ? info->global_count : info->id_offset + info->particle_count;
  if (info->id_offset + info->particle_count > global)
    return fail(nullptr, RPS_ERR_INVALID_ARGUMENT, "id_offset + particle_count > global_count");
  if (info->mode == RPS_MODE_SPH) {
    if (info->particle_count > 0x80000000ull || info->id_offset != 0 || global != info->particle_count)
      return fail(nullptr, RPS_ERR_INVALID_ARGUMENT,
                  "SPH mode: one unsharded system of at most 2^31 particles (u32 keys, wgsl:52)");
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return fail(nullptr, RPS_ERR_NO_DEVICE, "no HIP device visible");
  if (info->device < 0 || info->device >= ndev)
    return fail(nullptr, RPS_ERR_INVALID_ARGUMENT, "device ordinal out of range");

  rps_ctx* ctx = new (std::nothrow) rps_ctx();
  if (!ctx) return fail(nullptr, RPS_ERR_OUT_OF_MEMORY, "host allocation failed");
  ctx->device = info->device;
  ctx->mode = info->mode;
  ctx->n = info->particle_count;
  ctx->id_offset = info->id_offset;
  ctx->global_count = global;
  ctx->ext = default_ext();
  ctx->nontemporal = stream_nt_default(ctx->n);
  // Forced scan batches, read per context (tests force each variant at small N).
  {
    const int both = env_int("RPS_SPH_BATCH", 0);
    ctx->sph_batch_d = (uint8_t)std::max(0, std::min(255, env_int("RPS_SPH_BATCH_D", both)));
    ctx->sph_batch_s = (uint8_t)std::max(0, std::min(255, env_int("RPS_SPH_BATCH_S", both)));
  }

  auto bail = [&](int code) {
    std::string m = ctx->err;
    rps_destroy(ctx);
    g_err = m;
    return code;
  };
  if (hipSetDevice(ctx->device) != hipSuccess) {
    ctx->err = "hipSetDevice failed";
    return bail(RPS_ERR_DEVICE);
  }
  if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
    ctx->err = "hipStreamCreate failed";
    return bail(RPS_ERR_DEVICE);
  }
  if (hipEventCreate(&ctx->ev_begin) != hipSuccess || hipEventCreate(&ctx->ev_end) != hipSuccess) {
    ctx->err = "hipEventCreate failed";
    return bail(RPS_ERR_DEVICE);
  }

  // Carve the arena: every array 256-B aligned (16-B vector access + full cache lines).
  const size_t n = ctx->n;
  const size_t nf = align_up(n * sizeof(float), 256);
  size_t off = 0;
  struct Slot { void** p; size_t bytes; };
  std::vector<Slot> slots;
  if (ctx->mode == RPS_MODE_STREAM) {
    // Tiled SoA: ceil(n / kTile) tiles of 4 f32 + 2 u16 segments (rps_device.hpp).
    const size_t tiles = (n + kTile - 1) / kTile;
    slots.push_back({(void**)&ctx->state, tiles * kTileBytes});
    slots.push_back({(void**)&ctx->exp, align_up(tiles * kTile * sizeof(uint16_t), 256)});
    slots.push_back({(void**)&ctx->next, align_up((tiles * kTile >> kGroupLog) * sizeof(uint16_t), 256)});
  } else if (ctx->mode == RPS_MODE_NBODY) {
    slots.push_back({(void**)&ctx->x, nf});
    slots.push_back({(void**)&ctx->y, nf});
    slots.push_back({(void**)&ctx->vx, nf});
    slots.push_back({(void**)&ctx->vy, nf});
  }
  if (ctx->mode == RPS_MODE_SPH) {
    ctx->P = next_pow2_u32((uint32_t)n);  // spatial lookup sized next_pow2 (particle_buffers.rs:86)
    const size_t P = ctx->P;
    ctx->sort_fold = env_int("RPS_SPH_SORT_FOLD", 1) != 0;
    ctx->csort = env_int("RPS_SPH_CSORT", 1) != 0;
    ctx->csort_tlog = (uint8_t)std::max(0, std::min(13, env_int("RPS_SPH_CSORT_TLOG", 0)));
    ctx->csort_wide = (uint8_t)std::max(0, std::min(5, env_int("RPS_SPH_CSORT_WIDE", 4)));
    ctx->pair_max_p = (uint32_t)std::max(0, env_int("RPS_SPH_PAIRS", 1 << 17));
    ctx->sim_fuse = env_int("RPS_SPH_SIM_FUSE", 1) != 0;
    // Lanes per slot of the small-P scans: 4 below 65 536 particles (same box, ms/frame: 20 000
    // 0.0561 -> 0.0531, 50 000 0.0883 -> 0.0863), 2 from there (65 536 0.0761 / 0.0769 with 4,
    // 100 000 0.1215 / 0.1307); RPS_SPH_GROUP=2 or 4 forces one.
    {
      const int grp = env_int("RPS_SPH_GROUP", 0);
      ctx->lane_group = grp == 2 || grp == 4 ? (uint8_t)grp : (n < 65536 ? 4 : 2);
      const int gs = env_int("RPS_SPH_GROUP_S", 0);
      ctx->lane_group_s = gs == 2 || gs == 4 ? (uint8_t)gs : ctx->lane_group;
    }
    const int lay_mode = env_int("RPS_SPH_LAYOUT", 1);
    const bool lay_ok = lay_mode == 2 || (lay_mode == 1 && P >= (1u << 20));
    // With the layout the state is slot-resident (one entry per slot: P of them)
    const size_t st_n = lay_ok ? P : n;
    slots.push_back({(void**)&ctx->st, align_up(st_n * sizeof(f4), 256)});
    slots.push_back({(void**)&ctx->sl.pp_s, align_up(P * sizeof(f2), 256)});
    slots.push_back({(void**)&ctx->sl.rec_pv, align_up(P * sizeof(f4), 256)});
    slots.push_back({(void**)&ctx->sl.rec_pd, align_up(P * sizeof(f4), 256)});
    slots.push_back({(void**)&ctx->sl.dens_s, align_up(P * sizeof(f2), 256)});
    slots.push_back({(void**)&ctx->sl.idx_s, align_up(P * sizeof(uint32_t), 256)});
    slots.push_back({(void**)&ctx->sl.cur_s, align_up(P * sizeof(f2), 256)});
    slots.push_back({(void**)&ctx->ends, align_up(n * sizeof(uint32_t), 256)});
    slots.push_back({(void**)&ctx->sl.nbr_mask, align_up(2 * P * sizeof(uint64_t), 256)});
    if (P != n) slots.push_back({(void**)&ctx->sl.owner, align_up(n * sizeof(uint64_t), 256)});
    if (P != n && lay_ok) slots.push_back({(void**)&ctx->own_buf, align_up(P, 256)});
    // Long scans one per wave (rps_kernels.hip, kLongScan): P != N, where the reference's pad
    // hazard grows long duplicate runs.  RPS_SPH_LONGQ=0 keeps them in their lanes (A/B).
    if (P != n && env_int("RPS_SPH_LONGQ", 1) != 0) {
      slots.push_back({(void**)&ctx->sl.longq, align_up((P + 1) * sizeof(uint4), 256)});
      slots.push_back({(void**)&ctx->sl.longq_n, 256});
      slots.push_back({(void**)&ctx->sl.longtab, align_up((P + 1) * kLongTab * sizeof(uint2), 256)});
      // More than 64 entries up to P = 2^19 (same box, ms/frame: 50 000 0.1523 -> 0.1406,
      // 100 000 0.1797 -> 0.1665, 300 000 and 20 000 unchanged; 48 at 50 000: 0.2822), more than
      // 128 above (10^6: 0.4423 with 128, 0.4519 with 64).
      const int dflt = P <= (1u << 19) ? 64 : (int)kLongScan;
      ctx->sl.long_min = (uint32_t)std::min((int)kLongScan, std::max(8, env_int("RPS_SPH_LONG_MIN", dflt)));
    }
    slots.push_back({(void**)&ctx->lookup, align_up((size_t)ctx->P * sizeof(uint2), 256)});
    slots.push_back({(void**)&ctx->offsets, align_up(n * sizeof(uint32_t), 256)});
    slots.push_back({(void**)&ctx->dens, align_up(n * sizeof(f2), 256)});
    slots.push_back({(void**)&ctx->pred, align_up(n * sizeof(f2), 256)});
    slots.push_back({(void**)&ctx->d_count, align_up(2 * sph_count_blocks(ctx->P) * sizeof(unsigned long long), 256)});
    // Spatial record layout (rps_kernels.hip): RPS_SPH_LAYOUT=0 off, 1 (default) from P = 2^20
    // slots, where it is measured faster (with slot-resident state, same box: 2^20 frame
    // 0.3442 -> 0.3230 ms, 2^19 0.2274 -> 0.2269, 2^18 0.1429 -> 0.1458 slower),
    // 2 at any size.
    if (lay_ok) {
      // Up to 1 cell per particle (the bench's viewport, like the reference default, has
      // ~0.52), and at least the reference's default 1920 x 1080 viewport (~27 000 cells).
      ctx->cell_cap = (uint32_t)std::max<size_t>(n, 1u << 16);
      const size_t cap = ctx->cell_cap;
      slots.push_back({(void**)&ctx->lay.cell_info, align_up(cap * sizeof(uint4), 256)});
      slots.push_back({(void**)&ctx->lay.cellrun, align_up(cap * sizeof(uint2), 256)});
      slots.push_back({(void**)&ctx->lay.run2, align_up(n * sizeof(uint2), 256)});
      slots.push_back({(void**)&ctx->lay.part, align_up((cap / 256 + 2) * sizeof(uint32_t), 256)});
      slots.push_back({(void**)&ctx->lay.out_runs, align_up(n * sizeof(uint2), 256)});
      slots.push_back({(void**)&ctx->lay.key_cell, align_up(n * sizeof(uint2), 256)});
      slots.push_back({(void**)&ctx->lay.keybits, align_up((n / 32 + 1) * sizeof(uint32_t), 256)});
      slots.push_back({(void**)&ctx->lay.n_out, 256});
      // slot-resident state: the buffer st swaps with, the previous slot -> particle map, the
      // sim's bin entries
      slots.push_back({(void**)&ctx->st_alt, align_up(st_n * sizeof(f4), 256)});
      slots.push_back({(void**)&ctx->idx_alt, align_up(P * sizeof(uint32_t), 256)});
    }
    // the sim's bin entries for the next frame (slot-resident or particle order)
    slots.push_back({(void**)&ctx->bin_next, align_up(n * sizeof(uint2), 256)});
  }
  if (ctx->mode == RPS_MODE_NBODY) {
    ctx->ns_padded = (global + kNbodyTile - 1) / kNbodyTile * kNbodyTile;
    slots.push_back({(void**)&ctx->pos_all, align_up(ctx->ns_padded * sizeof(f2), 256)});
    slots.push_back({(void**)&ctx->ax, nf});
    slots.push_back({(void**)&ctx->ay, nf});
    const int forced = env_int("RPS_NBODY_SPLITS", 0);  // > 0: force the split count
    ctx->nb_splits = forced > 0 ? (uint32_t)std::min<uint64_t>((uint64_t)forced, ctx->ns_padded / kNbodyTile)
                                : nbody_splits_for(n, ctx->ns_padded);
    if (ctx->nb_splits > 1)
      slots.push_back({(void**)&ctx->nb_part, align_up((size_t)ctx->nb_splits * n * sizeof(f2), 256)});
  }
  slots.push_back({(void**)&ctx->d_cfg, align_up(sizeof(rps_config), 256)});
  slots.push_back({(void**)&ctx->d_stats, align_up(sizeof(StatsResult), 256)});
  slots.push_back({(void**)&ctx->d_gstats, align_up(sizeof(StatsGlobal), 256)});
  std::vector<size_t> offs;
  for (auto& s : slots) {
    offs.push_back(off);
    off += s.bytes;
  }
  ctx->arena_bytes = off;
  hipError_t e = hipMalloc(&ctx->arena, ctx->arena_bytes);
  if (e != hipSuccess) {
    ctx->err = std::string("hipMalloc(") + std::to_string(ctx->arena_bytes) + "): " + hipGetErrorString(e);
    return bail(e == hipErrorOutOfMemory ? RPS_ERR_OUT_OF_MEMORY : RPS_ERR_DEVICE);
  }
  for (size_t i = 0; i < slots.size(); ++i) *slots[i].p = ctx->arena + offs[i];
  if (ctx->mode == RPS_MODE_SPH) {
    ctx->layout = sph_layout();
    set_sph_fields(ctx);
    // A layout frame does not run pass 3, so its run ends go to the key-indexed ends array.
    if (ctx->cell_cap) ctx->lay.run_end = ctx->ends;
    // test hook: the epoch the layout builds count from (the wrap at 2^24, step_sph_sim)
    ctx->lay.epoch = (uint32_t)std::clamp(env_int("RPS_SPH_LAYOUT_EPOCH", 0), 0, (1 << 24) - 1);
  }
  if (ctx->mode == RPS_MODE_STREAM) {
    ctx->layout = tiled_layout();
    ctx->x = ctx->state;
    ctx->y = ctx->state + kTile;
    ctx->vx = ctx->state + 2 * kTile;
    ctx->vy = ctx->state + 3 * kTile;
    // exp / next: arrays of their own, zero-filled with the arena (expiries 0, clock 0, next 0)
    ctx->exp_layout = tiled_exp_layout();
  }
  // wgpu buffers are zero-initialised; the SPH lookup pad entries rely on it.
  if (hipMemsetAsync(ctx->arena, 0, ctx->arena_bytes, ctx->stream) != hipSuccess) {
    ctx->err = "hipMemsetAsync failed";
    return bail(RPS_ERR_DEVICE);
  }
  if (ctx->mode == RPS_MODE_NBODY &&
      launch_nbody_pad(ctx->pos_all, global, ctx->ns_padded, ctx->stream) != hipSuccess) {
    ctx->err = "nbody pad launch failed";
    return bail(RPS_ERR_DEVICE);
  }
  if (hipStreamSynchronize(ctx->stream) != hipSuccess) {
    ctx->err = "hipStreamSynchronize failed";
    return bail(RPS_ERR_DEVICE);
  }
  *out = ctx;
  return RPS_OK;
}

int rps_destroy(rps_ctx* ctx) {
  if (!ctx) return RPS_OK;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->comm) ncclCommDestroy(ctx->comm);
  for (auto ev : ctx->ev_start) (void)hipEventDestroy(ev);
  for (auto ev : ctx->ev_stop) (void)hipEventDestroy(ev);
  if (ctx->d_staging) (void)hipFree(ctx->d_staging);
  if (ctx->nb_stamps) (void)hipFree(ctx->nb_stamps);
  if (ctx->partials) (void)hipFree(ctx->partials);
  if (ctx->arena) (void)hipFree(ctx->arena);
  if (ctx->ev_begin) (void)hipEventDestroy(ctx->ev_begin);
  if (ctx->ev_end) (void)hipEventDestroy(ctx->ev_end);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  return RPS_OK;
}

int rps_set_config(rps_ctx* ctx, const rps_config* cfg, const rps_ext_config* ext) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (!cfg) return fail(ctx, RPS_ERR_INVALID_ARGUMENT, "null config");
  rps_ext_config e = ext ? *ext : default_ext();
  if (e.integrator > RPS_INTEGRATOR_VERLET) return fail(ctx, RPS_ERR_INVALID_ARGUMENT, "bad integrator");
  if (e.num_attractors > RPS_MAX_ATTRACTORS)
    return fail(ctx, RPS_ERR_INVALID_ARGUMENT, "num_attractors > RPS_MAX_ATTRACTORS");
  if ((e.flags & RPS_EXT_NBODY_EXTERNAL) && ctx->mode != RPS_MODE_NBODY)
    return fail(ctx, RPS_ERR_UNSUPPORTED, "RPS_EXT_NBODY_EXTERNAL is an N-body flag");
  if (ctx->mode != RPS_MODE_STREAM && (e.flags & (RPS_EXT_LIFETIME | RPS_EXT_STATS)))
    return fail(ctx, RPS_ERR_UNSUPPORTED, "lifetime/stats extensions exist in STREAM mode only");
  if (ctx->mode != RPS_MODE_STREAM && (e.integrator != RPS_INTEGRATOR_EULER || e.num_attractors))
    return fail(ctx, RPS_ERR_UNSUPPORTED, "attractors/Verlet exist in STREAM mode only");
  if (ctx->mode == RPS_MODE_NBODY && !(e.nbody_softening > 0.0f))
    return fail(ctx, RPS_ERR_INVALID_ARGUMENT, "nbody_softening must be > 0");
  if (ctx->mode == RPS_MODE_SPH && cfg->particle_count != (uint32_t)ctx->n)
    return fail(ctx, RPS_ERR_INVALID_ARGUMENT, "SPH mode: config.particle_count must equal the context's particles");
  if (!(cfg->fixed_delta_time == cfg->fixed_delta_time))
    return fail(ctx, RPS_ERR_INVALID_ARGUMENT, "fixed_delta_time is NaN");
  ctx->cfg = *cfg;
  ctx->ext = e;
  ctx->have_config = true;
  ctx->keys_valid = false;  // slot-resident bin entries were keyed with the old config
  ctx->pkeys_valid = false;
  // write_buffer(config) (src/particle_buffers.rs:230-236): the 144 B ride in a one-wave
  // kernel's arguments, ordered on the context stream before the next step's kernels.  A
  // pinned-staging hipMemcpyAsync cost 12-18 us a frame at 65 536 particles (STREAM) and
  // 35 us (SPH) against a kernel boundary (tools/config_upload_bench.py).
  RPS_HIP(ctx, launch_config_store(*cfg, ctx->d_cfg, ctx->stream));
  return RPS_OK;
}

int rps_get_config(const rps_ctx* ctx, rps_config* cfg, rps_ext_config* ext) {
  if (!ctx) return fail(nullptr, RPS_ERR_INVALID_ARGUMENT, "null context");
  if (cfg) *cfg = ctx->cfg;
  if (ext) *ext = ctx->ext;
  return RPS_OK;
}

int rps_upload_particles(rps_ctx* ctx, const rps_particle* aos, uint64_t offset, uint64_t n) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (!aos && n) return fail(ctx, RPS_ERR_INVALID_ARGUMENT, "null particles");
  if (offset + n > ctx->n) return fail(ctx, RPS_ERR_INVALID_ARGUMENT, "range exceeds particle_count");
  const uint64_t chunk = std::min<uint64_t>(n, kStagingChunk);
  if (n == 0) return RPS_OK;
  if ((rc = sph_canonical(ctx))) return rc;
  ctx->pkeys_valid = false;  // the state changes
  rc = ensure_staging(ctx, chunk);
  if (rc) return rc;
  for (uint64_t done = 0; done < n; done += chunk) {
    const uint64_t m = std::min(chunk, n - done);
    RPS_HIP(ctx, hipMemcpyAsync(ctx->d_staging, aos + done, m * sizeof(rps_particle),
                                hipMemcpyHostToDevice, ctx->stream));
    const uint64_t o = offset + done;
    RPS_HIP(ctx, launch_aos_to_soa(ctx->d_staging, fields(ctx), ctx->layout, o, m, ctx->stream));
    RPS_HIP(ctx, hipStreamSynchronize(ctx->stream));
  }
  return RPS_OK;
}

int rps_download_particles(rps_ctx* ctx, rps_particle* aos, uint64_t offset, uint64_t n) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (!aos && n) return fail(ctx, RPS_ERR_INVALID_ARGUMENT, "null particles");
  if (offset + n > ctx->n) return fail(ctx, RPS_ERR_INVALID_ARGUMENT, "range exceeds particle_count");
  if (n == 0) return RPS_OK;
  if ((rc = sph_canonical(ctx))) return rc;
  const uint64_t chunk = std::min<uint64_t>(n, kStagingChunk);
  rc = ensure_staging(ctx, chunk);
  if (rc) return rc;
  for (uint64_t done = 0; done < n; done += chunk) {
    const uint64_t m = std::min(chunk, n - done);
    const uint64_t o = offset + done;
    RPS_HIP(ctx, launch_soa_to_aos(fields(ctx), ctx->layout, o, ctx->d_staging, m,
                                   ctx->cfg.max_energy, ctx->stepped ? 0 : 1, ctx->stream));
    RPS_HIP(ctx, hipMemcpyAsync(aos + done, ctx->d_staging, m * sizeof(rps_particle),
                                hipMemcpyDeviceToHost, ctx->stream));
    RPS_HIP(ctx, hipStreamSynchronize(ctx->stream));
  }
  return RPS_OK;
}

int rps_export_particles(rps_ctx* ctx, rps_particle* device_dst, uint64_t offset, uint64_t n) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (!device_dst && n) return fail(ctx, RPS_ERR_INVALID_ARGUMENT, "null destination");
  if (offset + n > ctx->n) return fail(ctx, RPS_ERR_INVALID_ARGUMENT, "range exceeds particle_count");
  if (n) {
    hipPointerAttribute_t attr;
    const hipError_t pe = hipPointerGetAttributes(&attr, device_dst);
    if (pe != hipSuccess) (void)hipGetLastError();  // do not leave a sticky error for later launches
    if (pe != hipSuccess || attr.type != hipMemoryTypeDevice)
      return fail(ctx, RPS_ERR_INVALID_ARGUMENT, "device_dst is not device memory");
    if ((rc = sph_canonical(ctx))) return rc;
  }
  constexpr uint64_t kChunk = 1ull << 30;  // stays under the 2^31 work-item grid cap
  for (uint64_t done = 0; done < n; done += kChunk) {
    const uint64_t m = std::min(kChunk, n - done);
    RPS_HIP(ctx, launch_soa_to_aos(fields(ctx), ctx->layout, offset + done, device_dst + done, m,
                                   ctx->cfg.max_energy, ctx->stepped ? 0 : 1, ctx->stream));
  }
  return RPS_OK;
}

// RPS_FIELD_LIFE is not stored: it is derived from / converted to the u16 expiry at the
// current lifetime clock, through the staging buffer.
int rps_upload_field(rps_ctx* ctx, int field, const float* src, uint64_t offset, uint64_t n) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  const bool life = field == RPS_FIELD_LIFE || field == RPS_FIELD_LIFE_STEPS;
  float* p = life ? nullptr : field_ptr(ctx, field);
  if (life ? !ctx->exp : !p) return fail(ctx, RPS_ERR_INVALID_ARGUMENT, "field not present in this mode");
  if (!src && n) return fail(ctx, RPS_ERR_INVALID_ARGUMENT, "null source");
  if (offset + n > ctx->n) return fail(ctx, RPS_ERR_INVALID_ARGUMENT, "range exceeds particle_count");
  if (n == 0) return RPS_OK;
  if ((rc = sph_canonical(ctx))) return rc;
  ctx->pkeys_valid = false;  // the state changes
  if (!life) p = field_ptr(ctx, field);  // (sph_canonical may have swapped the state buffer)
  if (!life && ctx->layout.mask == plain_layout().mask) {
    RPS_HIP(ctx, hipMemcpyAsync(p + offset, src, n * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
    RPS_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return RPS_OK;
  }
  // Dense chunk -> staging -> scatter into the tiles (or convert into expiries).
  const uint64_t chunk = std::min<uint64_t>(n, kStagingChunk * (sizeof(rps_particle) / sizeof(float)));
  rc = ensure_staging(ctx, (chunk * sizeof(float) + sizeof(rps_particle) - 1) / sizeof(rps_particle));
  if (rc) return rc;
  float* stage = reinterpret_cast<float*>(ctx->d_staging);
  for (uint64_t done = 0; done < n; done += chunk) {
    const uint64_t m = std::min(chunk, n - done);
    RPS_HIP(ctx, hipMemcpyAsync(stage, src + done, m * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
    if (life)
    {
      RPS_HIP(ctx, launch_life_scatter(ctx->exp, ctx->exp_layout, offset + done, stage, m,
                                       (uint32_t)ctx->life_clock, ctx->cfg.fixed_delta_time,
                                       field == RPS_FIELD_LIFE ? 0 : 2, ctx->stream));
      RPS_HIP(ctx, launch_next_rebuild(ctx->exp, ctx->next, offset + done, m, ctx->n,
                                       (uint32_t)ctx->life_clock, ctx->stream));
    }
    else
      RPS_HIP(ctx, launch_field_scatter(p, ctx->layout, offset + done, stage, m, ctx->stream));
    RPS_HIP(ctx, hipStreamSynchronize(ctx->stream));
  }
  return RPS_OK;
}

int rps_download_field(rps_ctx* ctx, int field, float* dst, uint64_t offset, uint64_t n) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  const bool life = field == RPS_FIELD_LIFE || field == RPS_FIELD_LIFE_STEPS;
  float* p = life ? nullptr : field_ptr(ctx, field);
  if (life ? !ctx->exp : !p) return fail(ctx, RPS_ERR_INVALID_ARGUMENT, "field not present in this mode");
  if (!dst && n) return fail(ctx, RPS_ERR_INVALID_ARGUMENT, "null destination");
  if (offset + n > ctx->n) return fail(ctx, RPS_ERR_INVALID_ARGUMENT, "range exceeds particle_count");
  if (n == 0) return RPS_OK;
  if ((rc = sph_canonical(ctx))) return rc;
  if (!life) p = field_ptr(ctx, field);  // (sph_canonical may have swapped the state buffer)
  if (!life && ctx->layout.mask == plain_layout().mask) {
    RPS_HIP(ctx, hipMemcpyAsync(dst, p + offset, n * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
    RPS_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return RPS_OK;
  }
  const uint64_t chunk = std::min<uint64_t>(n, kStagingChunk * (sizeof(rps_particle) / sizeof(float)));
  rc = ensure_staging(ctx, (chunk * sizeof(float) + sizeof(rps_particle) - 1) / sizeof(rps_particle));
  if (rc) return rc;
  float* stage = reinterpret_cast<float*>(ctx->d_staging);
  for (uint64_t done = 0; done < n; done += chunk) {
    const uint64_t m = std::min(chunk, n - done);
    if (life)
      RPS_HIP(ctx, launch_life_gather(ctx->exp, ctx->exp_layout, offset + done, stage, m,
                                      (uint32_t)ctx->life_clock, ctx->cfg.fixed_delta_time,
                                      field == RPS_FIELD_LIFE ? 0 : 2, ctx->stream));
    else
      RPS_HIP(ctx, launch_field_gather(p, ctx->layout, offset + done, stage, m, ctx->stream));
    RPS_HIP(ctx, hipMemcpyAsync(dst + done, stage, m * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
    RPS_HIP(ctx, hipStreamSynchronize(ctx->stream));
  }
  return RPS_OK;
}

int rps_read_debug(rps_ctx* ctx, int which, void* dst, uint64_t bytes) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (!dst) return fail(ctx, RPS_ERR_INVALID_ARGUMENT, "null destination");
  const void* src = nullptr;
  uint64_t want = 0;
  switch (which) {
    case RPS_DEBUG_SPATIAL_LOOKUP: src = ctx->lookup; want = (uint64_t)ctx->P * 8; break;
    case RPS_DEBUG_LOOKUP_OFFSETS: src = ctx->offsets; want = ctx->n * 4; break;
    case RPS_DEBUG_DENSITIES: src = ctx->dens; want = ctx->n * 8; break;  // rebuilt below
    case RPS_DEBUG_PREDICTED: src = ctx->pred; want = ctx->n * 8; break;
    case RPS_DEBUG_ACCEL_X: src = ctx->ax; want = ctx->n * 4; break;
    case RPS_DEBUG_ACCEL_Y: src = ctx->ay; want = ctx->n * 4; break;
    case RPS_DEBUG_EXPIRY: src = ctx->exp; want = ctx->n * 2; break;
    default: return fail(ctx, RPS_ERR_INVALID_ARGUMENT, "unknown debug buffer");
  }
  if (!src) return fail(ctx, RPS_ERR_UNSUPPORTED, "debug buffer not present in this mode");
  if (bytes != want)
    return fail(ctx, RPS_ERR_INVALID_ARGUMENT, "bytes must equal the buffer size (" + std::to_string(want) + ")");
  if (which == RPS_DEBUG_EXPIRY) {  // tiled u16 -> dense, through the staging buffer
    const uint64_t chunk = kStagingChunk * (sizeof(rps_particle) / sizeof(uint16_t));
    rc = ensure_staging(ctx, kStagingChunk);
    if (rc) return rc;
    for (uint64_t done = 0; done < ctx->n; done += chunk) {
      const uint64_t m = std::min(chunk, ctx->n - done);
      RPS_HIP(ctx, launch_life_gather(ctx->exp, ctx->exp_layout, done,
                                      reinterpret_cast<float*>(ctx->d_staging), m, 0, 0.0f, 1,
                                      ctx->stream));
      RPS_HIP(ctx, hipMemcpyAsync(static_cast<uint16_t*>(dst) + done, ctx->d_staging,
                                  m * sizeof(uint16_t), hipMemcpyDeviceToHost, ctx->stream));
      RPS_HIP(ctx, hipStreamSynchronize(ctx->stream));
    }
    return RPS_OK;
  }
  if (which == RPS_DEBUG_DENSITIES || which == RPS_DEBUG_PREDICTED)
    RPS_HIP(ctx, launch_sph_debug_views(sph_buffers(ctx), ctx->stream));
  if (which == RPS_DEBUG_SPATIAL_LOOKUP && (ctx->lookup_perm || (ctx->resident && ctx->P != ctx->n))) {
    // Slot-resident frame: payloads are the previous frame's slots (and, with P != N, the pads'
    // flagged particle indices); the reference holds particle indices.  Translated into the
    // neighbour masks' buffer (2 x P x 8 B, dead between frames).
    uint2* scratch = reinterpret_cast<uint2*>(ctx->sl.nbr_mask);
    RPS_HIP(ctx, launch_sph_lookup_translate(ctx->lookup, ctx->lookup_perm, scratch, ctx->P, ctx->stream));
    src = scratch;
  }
  // A spatial-layout frame measures its runs without touching the reference's offsets:
  // bin_particles_in_grid's reset (wgsl:467) and pass 3 (wgsl:507-525) on the frame's sorted
  // lookup, on demand.
  if (which == RPS_DEBUG_LOOKUP_OFFSETS && ctx->layout_last) {
    RPS_HIP(ctx, hipMemsetAsync(ctx->offsets, 0xFF, ctx->n * sizeof(uint32_t), ctx->stream));
    RPS_HIP(ctx, launch_sph_offsets(sph_buffers(ctx), ctx->stream));
  }
  RPS_HIP(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
  RPS_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return RPS_OK;
}

int rps_init_scatter(rps_ctx* ctx, uint64_t seed) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (!ctx->have_config) return fail(ctx, RPS_ERR_INVALID_ARGUMENT, "rps_set_config first");
  // Leaving the slot-resident state like every other particle-order write: the lookup's payloads
  // back to particle indices (P != N: the pads unflagged) and lookup_perm cleared, so a later
  // DEBUG_SPATIAL_LOOKUP read and the compact sort's 16-bit payloads see particle indices.
  if ((rc = sph_canonical(ctx))) return rc;
  InitArgs a;
  a.f = fields(ctx);
  a.layout = ctx->layout;
  a.n = ctx->n;
  a.id_offset = ctx->id_offset;
  a.x_min = ctx->cfg.screen_bounds[0];
  a.x_max = ctx->cfg.screen_bounds[1];
  a.y_min = ctx->cfg.screen_bounds[2];
  a.y_max = ctx->cfg.screen_bounds[3];
  a.global_count_f = (float)ctx->global_count;
  a.life_min = ctx->ext.life_min;
  a.life_range = ctx->ext.life_max - ctx->ext.life_min;
  a.exp_layout = ctx->exp_layout;
  a.clock = (uint32_t)ctx->life_clock;
  a.dt = ctx->cfg.fixed_delta_time;
  a.key0 = (uint32_t)seed;
  a.key1 = (uint32_t)(seed >> 32);
  ctx->keys_valid = false;  // every particle rewritten in particle order
  ctx->pkeys_valid = false;
  RPS_HIP(ctx, launch_init_scatter(a, ctx->stream));
  if (ctx->next)
    RPS_HIP(ctx, launch_next_rebuild(ctx->exp, ctx->next, 0, ctx->n, ctx->n, (uint32_t)ctx->life_clock,
                                     ctx->stream));
  return RPS_OK;
}

int rps_step(rps_ctx* ctx, uint32_t nsteps) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (!ctx->have_config) return fail(ctx, RPS_ERR_INVALID_ARGUMENT, "rps_set_config first");
  const bool nb_external = (ctx->ext.flags & RPS_EXT_NBODY_EXTERNAL) != 0;
  if (ctx->mode == RPS_MODE_NBODY && ctx->nranks > 1 && !ctx->comm && !nb_external)
    return fail(ctx, RPS_ERR_COMM, "sharded N-body needs rps_comm_init");
  if (ctx->mode == RPS_MODE_NBODY && ctx->global_count != ctx->n && !ctx->comm && !nb_external)
    return fail(ctx, RPS_ERR_COMM, "sharded N-body needs rps_comm_init or RPS_EXT_NBODY_EXTERNAL");
  const uint32_t fuse = std::min<uint32_t>(ctx->ext.fuse_steps, kMaxFuse);
  const bool fused = ctx->mode == RPS_MODE_STREAM && fuse > 1;
  const uint32_t interval = std::max<uint32_t>(ctx->ext.stats_interval, 1u);
  uint32_t pending = 0;  // fused mode: active steps accumulated since the last launch
  uint64_t pending_k0 = 0, pending_clock0 = 0;
  const bool lifetime = (ctx->ext.flags & RPS_EXT_LIFETIME) != 0;
  for (uint32_t s = 0; s < nsteps; ++s) {
    ctx->cfg.frame_count += 1;  // src/particle_buffers.rs:227
    const bool active = ctx->cfg.frame_count >= ctx->ext.shader_delay;  // wgsl:426, :442
    SphGrid grid{};
    const bool layout = ctx->mode == RPS_MODE_SPH && active && sph_layout_grid(ctx->cfg, ctx->cell_cap, &grid);
    if (ctx->mode == RPS_MODE_SPH) {
      rc = sph_frame_begin(ctx, layout);
      if (rc) return rc;
      // passes 1-3 run every frame (particle_compute.rs:105-163); on an active frame the
      // offsets pass rides in the next kernel (the layout's runs kernel or predict)
      rc = step_sph_grid(ctx, active);
      if (rc) return rc;
    }
    if (ctx->mode == RPS_MODE_SPH) ctx->last_frame_active = active;
    if (!active) continue;
    if (fused) {
      const uint64_t k = ctx->active_steps;
      if (pending == 0) {
        pending_k0 = k;
        pending_clock0 = ctx->life_clock;
      }
      ++pending;
      ++ctx->active_steps;
      if (lifetime) ++ctx->life_clock;
      ctx->stepped = true;
      const bool stats = (ctx->ext.flags & RPS_EXT_STATS) && (k % interval == 0);
      if (pending == fuse || stats || s + 1 == nsteps) {
        rc = step_stream_fused(ctx, pending_k0, pending, stats, pending_clock0);
        if (rc) return rc;
        pending = 0;
      }
      continue;
    }
    switch (ctx->mode) {
      case RPS_MODE_STREAM: rc = step_stream(ctx); break;
      case RPS_MODE_NBODY: rc = step_nbody(ctx); break;
      default: rc = step_sph_sim(ctx, layout, grid); break;
    }
    if (rc) return rc;
    ++ctx->active_steps;
    if (lifetime && ctx->mode == RPS_MODE_STREAM) ++ctx->life_clock;
    ctx->stepped = true;
  }
  if (pending) return step_stream_fused(ctx, pending_k0, pending, false, pending_clock0);
  return RPS_OK;
}

int rps_update(rps_ctx* ctx) { return ctx ? RPS_OK : fail(nullptr, RPS_ERR_INVALID_ARGUMENT, "null context"); }

int rps_sync(rps_ctx* ctx) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  RPS_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return RPS_OK;
}

static int get_stats(rps_ctx* ctx, rps_stats* out, bool all_ranks) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (!out) return fail(ctx, RPS_ERR_INVALID_ARGUMENT, "null output");
  if (!ctx->have_stats) return fail(ctx, RPS_ERR_UNSUPPORTED, "no stats reduced yet (RPS_EXT_STATS)");
  StatsResult r;
  StatsGlobal g;
  const bool global = all_ranks && ctx->comm;
  RPS_HIP(ctx, hipMemcpyAsync(&r, ctx->d_stats, sizeof(r), hipMemcpyDeviceToHost, ctx->stream));
  if (global) RPS_HIP(ctx, hipMemcpyAsync(&g, ctx->d_gstats, sizeof(g), hipMemcpyDeviceToHost, ctx->stream));
  RPS_HIP(ctx, hipStreamSynchronize(ctx->stream));
  for (int k = 0; k < 4; ++k) out->bbox[k] = r.bbox[k];
  out->kinetic_energy = r.ke;
  out->particles = r.count;
  out->respawned = r.respawned;
  out->step = r.step;
  if (global) {  // every rank's shard (allreduce_stats)
    out->bbox[0] = -g.neg_min_max[0];
    out->bbox[1] = g.neg_min_max[1];
    out->bbox[2] = -g.neg_min_max[2];
    out->bbox[3] = g.neg_min_max[3];
    out->kinetic_energy = g.sums[0];
    out->particles = (uint64_t)g.sums[1];
    out->respawned = (uint64_t)g.sums[2];
  }
  return RPS_OK;
}

int rps_get_stats(rps_ctx* ctx, rps_stats* out) { return get_stats(ctx, out, true); }
int rps_get_shard_stats(rps_ctx* ctx, rps_stats* out) { return get_stats(ctx, out, false); }

int rps_get_counters(const rps_ctx* ctx, uint32_t* frame_count, uint64_t* active_steps) {
  if (!ctx) return fail(nullptr, RPS_ERR_INVALID_ARGUMENT, "null context");
  if (frame_count) *frame_count = ctx->cfg.frame_count;
  if (active_steps) *active_steps = ctx->active_steps;
  return RPS_OK;
}

int rps_set_profiling(rps_ctx* ctx, int enable) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (enable < 0) return fail(ctx, RPS_ERR_INVALID_ARGUMENT, "profiling period must be >= 0");
  ctx->profile_every = (uint32_t)enable;
  ctx->profile_seq = 0;
  ctx->ev_used = 0;
  if (enable && ctx->mode == RPS_MODE_NBODY && !ctx->nb_stamps)
    RPS_HIP(ctx, hipMalloc(&ctx->nb_stamps, 16 * nbody_workgroups(ctx->n, ctx->ns_padded, ctx->nb_splits)));
  return RPS_OK;
}

int rps_get_kernel_clock(rps_ctx* ctx, double* mhz, uint64_t* workgroups) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (ctx->mode != RPS_MODE_NBODY) return fail(ctx, RPS_ERR_UNSUPPORTED, "N-body mode only");
  if (!ctx->nb_stamp_wgs) return fail(ctx, RPS_ERR_UNSUPPORTED, "no profiled force launch yet (rps_set_profiling)");
  std::vector<uint64_t> h(2 * ctx->nb_stamp_wgs);
  RPS_HIP(ctx, hipMemcpyAsync(h.data(), ctx->nb_stamps, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost,
                              ctx->stream));
  RPS_HIP(ctx, hipStreamSynchronize(ctx->stream));
  std::vector<double> clk;
  clk.reserve(ctx->nb_stamp_wgs);
  for (uint64_t w = 0; w < ctx->nb_stamp_wgs; ++w)
    if (h[2 * w + 1] > 0) clk.push_back((double)h[2 * w] / (double)h[2 * w + 1] * 100.0);  // 100-MHz ticks
  if (clk.empty()) return fail(ctx, RPS_ERR_DEVICE, "no clock stamps recorded");
  std::nth_element(clk.begin(), clk.begin() + clk.size() / 2, clk.end());
  if (mhz) *mhz = clk[clk.size() / 2];
  if (workgroups) *workgroups = clk.size();
  return RPS_OK;
}

int rps_get_kernel_time(rps_ctx* ctx, double* avg_ms, uint64_t* launches) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  RPS_HIP(ctx, hipStreamSynchronize(ctx->stream));
  double total = 0.0;
  for (size_t i = 0; i < ctx->ev_used; ++i) {
    float ms = 0.0f;
    RPS_HIP(ctx, hipEventElapsedTime(&ms, ctx->ev_start[i], ctx->ev_stop[i]));
    total += ms;
  }
  if (avg_ms) *avg_ms = ctx->ev_used ? total / (double)ctx->ev_used : 0.0;
  if (launches) *launches = ctx->ev_used;
  ctx->ev_used = 0;
  return RPS_OK;
}

int rps_get_kernel_times(rps_ctx* ctx, double* ms, uint64_t cap, uint64_t* launches) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (!ms && cap) return fail(ctx, RPS_ERR_INVALID_ARGUMENT, "null output");
  RPS_HIP(ctx, hipStreamSynchronize(ctx->stream));
  for (size_t i = 0; i < ctx->ev_used && i < cap; ++i) {
    float t = 0.0f;
    RPS_HIP(ctx, hipEventElapsedTime(&t, ctx->ev_start[i], ctx->ev_stop[i]));
    ms[i] = t;
  }
  if (launches) *launches = ctx->ev_used;
  ctx->ev_used = 0;
  return RPS_OK;
}

int rps_time_steps(rps_ctx* ctx, uint32_t nsteps, double* total_ms) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  // The context's two events (created with its stream, so no allocation between the caller's
  // clock and the first launch).
  RPS_HIP(ctx, hipEventRecord(ctx->ev_begin, ctx->stream));
  rc = rps_step(ctx, nsteps);
  if (rc == RPS_OK) {
    RPS_HIP(ctx, hipEventRecord(ctx->ev_end, ctx->stream));
    RPS_HIP(ctx, hipEventSynchronize(ctx->ev_end));
    float ms = 0.0f;
    RPS_HIP(ctx, hipEventElapsedTime(&ms, ctx->ev_begin, ctx->ev_end));
    if (total_ms) *total_ms = ms;
  }
  return rc;
}

void* rps_get_stream(rps_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

static int sph_frame_cost(rps_ctx* ctx, rps_sph_cost* out) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (!out) return fail(ctx, RPS_ERR_INVALID_ARGUMENT, "null output");
  if (ctx->mode != RPS_MODE_SPH) return fail(ctx, RPS_ERR_UNSUPPORTED, "SPH mode only");
  if (!ctx->have_config) return fail(ctx, RPS_ERR_INVALID_ARGUMENT, "rps_set_config first");
  const SphBuffers b = sph_buffers(ctx);
  // The counts read the frame's sorted lookup, runs and predicted positions: they describe the
  // most recent frame only if that frame was active (a gated frame re-sorts the lookup and
  // resets the runs, but leaves the previous frame's predictions).
  if (!ctx->last_frame_active)
    return fail(ctx, RPS_ERR_UNSUPPORTED, "the most recent SPH frame was not active (run an active frame first)");
  const uint32_t nb = sph_count_blocks(ctx->P);
  std::vector<unsigned long long> h(2 * (size_t)nb);
  hipError_t e = launch_sph_count(b, ctx->d_count, ctx->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(h.data(), ctx->d_count, h.size() * sizeof(h[0]), hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) return fail(ctx, RPS_ERR_DEVICE, std::string("SPH cost count: ") + hipGetErrorString(e));
  uint64_t E = 0, W = 0;
  for (uint32_t i = 0; i < nb; ++i) {
    E += h[2 * (size_t)i];
    W += h[2 * (size_t)i + 1];
  }
  const double P = (double)ctx->P, N = (double)ctx->n;
  out->slots = ctx->P;
  out->particles = ctx->n;
  out->scanned_entries = E;
  out->within_entries = W;
  out->sort_launches = ctx->sort_launches;
  out->sort_bytes = (double)ctx->sort_launches * P * 16.0 + N * 8.0;
  out->predict_bytes = P * 60.0 + N * 8.0;
  out->density_bytes = (double)E * 8.0 + P * 120.0;
  out->sim_bytes = (double)E * 32.0 + P * 156.0;
  out->frame_bytes = out->sort_bytes + out->predict_bytes + out->density_bytes + out->sim_bytes;
  return RPS_OK;
}

int rps_sph_frame_cost(rps_ctx* ctx, rps_sph_cost* out) { return sph_frame_cost(ctx, out); }

int rps_step_cost(rps_ctx* ctx, double* amount, int* unit) {
  if (!ctx || !amount || !unit) return fail(nullptr, RPS_ERR_INVALID_ARGUMENT, "null argument");
  switch (ctx->mode) {
    case RPS_MODE_STREAM: {
      // r+w of x, y, vx, vy (+ the group's u16 [next] read, 2 B per 64 particles; the expiry
      // lines of the groups with one due are read, and written on respawn, on top): DESIGN.md §5.
      const double per = (ctx->ext.flags & RPS_EXT_LIFETIME) ? 32.0 + 2.0 / kGroup : 32.0;
      *amount = per * (double)ctx->n;
      *unit = 0;
      return RPS_OK;
    }
    case RPS_MODE_NBODY:
      *amount = 20.0 * (double)ctx->n * (double)ctx->global_count;  // GPU Gems 3 ch.31 convention
      *unit = 1;
      return RPS_OK;
    default: {
      rps_sph_cost c;
      const int rc = sph_frame_cost(ctx, &c);
      if (rc) return rc;
      *amount = c.frame_bytes;
      *unit = 0;
      return RPS_OK;
    }
  }
}

int rps_nbody_sources(rps_ctx* ctx, int pack, void** sources, uint64_t* count) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (ctx->mode != RPS_MODE_NBODY) return fail(ctx, RPS_ERR_UNSUPPORTED, "N-body mode only");
  if (pack) {
    RPS_HIP(ctx, launch_nbody_pack(ctx->x, ctx->y, ctx->pos_all + ctx->id_offset, ctx->n, ctx->stream));
    RPS_HIP(ctx, hipStreamSynchronize(ctx->stream));
  }
  if (sources) *sources = ctx->pos_all;
  if (count) *count = ctx->global_count;
  return RPS_OK;
}

int rps_comm_unique_id(void* out128) {
  if (!out128) return fail(nullptr, RPS_ERR_INVALID_ARGUMENT, "null output");
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId must be 128 bytes");
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return fail(nullptr, RPS_ERR_COMM, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
  std::memcpy(out128, &id, sizeof(id));
  return RPS_OK;
}

int rps_comm_init(rps_ctx* ctx, int rank, int nranks, const void* unique_id128) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (!unique_id128 || nranks < 1 || rank < 0 || rank >= nranks)
    return fail(ctx, RPS_ERR_INVALID_ARGUMENT, "bad rank/nranks/unique id");
  if (ctx->mode == RPS_MODE_NBODY &&
      (ctx->global_count != ctx->n * (uint64_t)nranks || ctx->id_offset != ctx->n * (uint64_t)rank))
    return fail(ctx, RPS_ERR_INVALID_ARGUMENT,
                "sharded N-body needs equal contiguous shards: global = nranks*n, id_offset = rank*n");
  ncclUniqueId id;
  std::memcpy(&id, unique_id128, sizeof(id));
  ncclResult_t r = ncclCommInitRank(&ctx->comm, nranks, id, rank);
  if (r != ncclSuccess) return fail(ctx, RPS_ERR_COMM, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  ctx->rank = rank;
  ctx->nranks = nranks;
  return RPS_OK;
}

}  // extern "C"
