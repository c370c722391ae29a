// rps_internal.hpp — launch interface between the C-ABI host code (rps_context.hip) and
// the gfx950 kernels (rps_kernels.hip).  Not installed; not part of the ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rps.h"
#include "rps_device.hpp"

namespace rps {

struct StreamLaunch {
  int verlet;
  int lifetime;
  int stats;
  int nontemporal;  // bit 0: nontemporal loads, bit 1: nontemporal stores
  uint32_t grid;  // workgroups (256 threads, 4 particles/thread/iteration)
};

// Workgroups a one-shot launch of the stream kernel needs for n particles.
uint32_t stream_blocks_for(uint64_t n);

hipError_t launch_stream_step(const StreamArgs& a, const StreamLaunch& l, hipStream_t s);
hipError_t launch_stream_fused(const FusedArgs& a, const StreamLaunch& l, hipStream_t s);
// Deterministic two-level reduction of per-workgroup partials (scratch: kStatsFold entries).
constexpr uint32_t kStatsFold = 256;
// `global` (nullable): also the shard's stats in the all-reduce form (StatsGlobal).
hipError_t launch_stats_finalize(const StatsPartial* partials, uint32_t count,
                                 StatsPartial* scratch, StatsResult* out, StatsGlobal* global,
                                 uint64_t step, hipStream_t s);

hipError_t launch_aos_to_soa(const rps_particle* aos, Fields f, Layout L, uint64_t offset,
                             uint64_t n, hipStream_t s);
hipError_t launch_config_store(const rps_config& cfg, rps_config* dst, hipStream_t s);
hipError_t launch_soa_to_aos(Fields f, Layout L, uint64_t offset, rps_particle* aos, uint64_t n,
                             float max_energy, int spawn_colour, hipStream_t s);
hipError_t launch_field_gather(const float* field, Layout L, uint64_t offset, float* out,
                               uint64_t n, hipStream_t s);
hipError_t launch_field_scatter(float* field, Layout L, uint64_t offset, const float* in,
                                uint64_t n, hipStream_t s);
// Lifetime expiry <-> its views at lifetime clock `clock`; mode 0 seconds, 1 raw u16
// (gather only), 2 steps left (kernels: life_gather/scatter_kernel).
hipError_t launch_life_gather(const uint16_t* exp, Layout L, uint64_t offset, float* out,
                              uint64_t n, uint32_t clock, float dt, int mode, hipStream_t s);
hipError_t launch_life_scatter(uint16_t* exp, Layout L, uint64_t offset, const float* in,
                               uint64_t n, uint32_t clock, float dt, int mode, hipStream_t s);

// Per-quad earliest expiries ([next], rps_device.hpp) of the full quads overlapping particles
// [first, first + n) of a shard of `total`, from the expiries at lifetime clock `clock`.
hipError_t launch_next_rebuild(const uint16_t* exp, uint16_t* next, uint64_t first, uint64_t n,
                               uint64_t total, uint32_t clock, hipStream_t s);

struct InitArgs {
  Fields f;  // exp may be null
  Layout layout, exp_layout;
  uint32_t clock;
  float dt;
  uint64_t n, id_offset;
  float x_min, x_max, y_min, y_max, global_count_f, life_min, life_range;
  uint32_t key0, key1;
};
hipError_t launch_init_scatter(const InitArgs& a, hipStream_t s);

// All-pairs N-body.
constexpr uint32_t kNbodyTile = 512;  // sources staged per LDS tile (float2: 4 KiB)
hipError_t launch_nbody_pack(const float* x, const float* y, f2* pos, uint64_t n, hipStream_t s);
hipError_t launch_nbody_pad(f2* pos, uint64_t from, uint64_t to, hipStream_t s);
// Source splits: at least kNbodyMinBlocks workgroups, so the last partial round of resident
// workgroups (768 at 3 per CU) is a small share of the launch: 2^21 particles 0.785 of FP32
// peak with 2 splits (2048 workgroups), 0.799 with 12, 0.801 with 24 and 48
// (tools/ab_nbody.py).  Each split adds nt float2 partials and a fixed-order reduce.
constexpr uint32_t kNbodyMinBlocks = 24576;
constexpr uint32_t kNbodyMaxSplits = 64;
uint32_t nbody_splits_for(uint64_t nt, uint64_t ns_padded);
// `splits` source splits (1: the kernel writes the accelerations directly; > 1: each split
// writes nt float2 partials into `part` and a fixed-order reduce follows).
// stamps (nullable): per workgroup {shader cycles, 100-MHz ticks} of its lifetime (16 B each,
// nbody_workgroups(nt, ns_padded, splits) of them), for the sustained-clock report of
// profiled launches.
hipError_t launch_nbody_accel(const f2* pos, uint64_t ns_padded, uint64_t t0, uint64_t nt,
                              float eps2, float gm, f2* part, uint32_t splits, float* ax,
                              float* ay, uint64_t* stamps, hipStream_t s);
uint64_t nbody_workgroups(uint64_t nt, uint64_t ns_padded, uint32_t splits);
struct NbodyIntegrateArgs {
  float* x;
  float* y;
  float* vx;
  float* vy;
  const float* ax;
  const float* ay;
  uint64_t n;
  float dt, gx_dt, gy_dt, drag_f;
  uint32_t drag_on;
  float x_min, x_max, y_min, y_max, damping;
};
hipError_t launch_nbody_integrate(const NbodyIntegrateArgs& a, hipStream_t s);

// SPH (the reference's five passes).
// Per-slot records in spatial-lookup order (slot t holds particle lookup[t].y's values), so
// a run's entries are contiguous.  Written by the predict pass except rec_pd (density pass).
// A sort payload with this bit set is a particle index, not a slot: the stale pad entries of a
// layout frame with P != N (rps_kernels.hip, resolve_payload).
constexpr uint32_t kPidFlag = 0x80000000u;
// Scans of more entries than this are "long" (rps_kernels.hip): the masks' capacity.
constexpr uint32_t kLongScan = 128u;
constexpr uint32_t kLongTab = 10u;  // uint2 per queued slot in SphSlots::longtab
struct SphSlots {
  f2* pp_s;      // P predicted positions                    (density scan: 8 B/entry)
  f4* rec_pv;    // P {predicted x, y, post-gravity vx, vy}  (viscosity scan)
  f4* rec_pd;    // P {predicted x, y, P/rho^2, Pn/(rho rho_n)} (pressure scan)
  f2* dens_s;    // P {density, near density}
  uint32_t* idx_s;  // P particle index (self-skip, wgsl:295 / :365)
  f2* cur_s;     // P current positions (Euler base)
  uint64_t* nbr_mask;  // 2 x P: bit f set <=> flat entry f of the nine runs is within the radius
  // P != N only (else nullptr): owner[i] = {owner_epoch, ~slot} of the lowest slot holding
  // particle i in the last active frame (claimed by atomicMax in its predict pass; an older
  // epoch loses, so no reset).  Pad slots repeat particles; a repeat computes
  // exactly its owner's values, so the sim runs on owner slots only, and slots >= N (never a
  // neighbour entry) skip the density too.
  uint64_t* owner;
  uint32_t owner_epoch;  // the last active frame's (1, 2, ...; the arena's zeros are epoch 0)
  // P != N, when the last active frame was a slot-resident layout frame (else nullptr): there
  // every stale pad entry is flagged (kPidFlag), so each particle has exactly one unflagged
  // entry, and its slot owns the particle: own_s[t] = 1 <=> slot t's entry is unflagged (written
  // in slot order by the write kernel; owner[] is then neither claimed nor read).
  uint8_t* own_s;
  // P != N only (else nullptr): the slots whose nine runs hold more than kLongScan entries,
  // appended by the density pass as {slot + 1, predicted x, y bits, 0} and computed one per
  // wave by the long-scan kernels (rps_kernels.hip).  P + 1 entries, {0, ...} past the last
  // one (the sim's long kernel clears what it read); longq_n is the append counter, which the
  // sim's long kernel zeroes for the next active frame.
  uint4* longq;
  uint32_t* longq_n;
  uint2* longtab;     // per queue entry: the slot's nine-run table (9 x {slot - f, f end}) + {runs, total}
  uint32_t long_min;  // a scan of more entries than this is long (kLongScan; RPS_SPH_LONG_MIN)
};
// Cell range of the spatial record layout (rps_kernels.hip): cells [cx_lo, cx_lo + w) x
// [cy_lo, cy_lo + h), enumerated in 8 x 8 tiles, tw tiles per row; cells = tiles x 64.
struct SphGrid {
  int32_t cx_lo, cy_lo;
  uint32_t w, h, tw, cells;
};
struct SphLayoutArgs {
  SphGrid g;
  uint4* cell_info;    // cells: {first slot, length | epoch << 8, 2 particle indices} of the run
                       //   a cell owns (another epoch: none; so it is never reset)
  uint32_t epoch;      // this layout build's (1 ... 2^24 - 1; cell_info, key_cell cleared at the wrap)
  uint2* cellrun;      // cells: storage {start, end} of the cell's key's run (start >= N: none)
  uint2* run2;         // N: storage {start, end} of the listed runs, by key (never reset)
  uint2* key_cell;     // N: {owner cell, or kCellOut for a listed run; epoch} of each key's run
                       //   (another epoch: the key has no run this build)
  uint32_t* part;      // cells / 256 + 2: 256-cell block sums -> bases; [blocks]: the grid's
                       //   total (the listed runs' storage starts there)
  uint2* out_runs;     // N: {first slot, storage base} of the runs placed after the grid's
  uint32_t* n_out;     // 1: their count (0 between frames)
  uint32_t* run_end;   // N: one past the last slot of each key's run (the runs kernel)
  uint32_t* keybits;   // N / 32: bit k set <=> key k has a run this frame (set by the runs
                       //   kernel, read by fixup, cleared by the density pass)
};
struct SphBuffers {
  const rps_config* cfg;  // device-resident ParticleConfig
  f4* st;            // N packed {x, y, vx, vy}: read by bin/predict, written in place by the sim
  uint2* lookup;     // P entries
  uint32_t* offsets; // N: first slot of each key's run (wgsl:55)
  uint32_t* ends;    // N: one past the last slot of each key's run in [0, N)
  f2* dens;          // N  debug views (wgsl:58, :61), rebuilt on readback
  f2* pred;          // N
  SphSlots sl;
  // Slot-resident state: after a layout frame `st` holds the state in that
  // frame's storage order (slot u: particle perm[u]) and bin_next the next frame's bin entries
  // (key, u) at position i.  With `resident`, this frame's sort payloads are those slots and
  // idx_prev (= perm) maps them to particle indices; the sim of a layout frame writes st[u]
  // and bin_next.
  uint2* bin_next;   // N
  const uint32_t* idx_prev;  // N (resident only)
  bool resident;
  // Without the layout, the last active frame's sim wrote bin_next[i] = (key, i) from the state
  // and config the next frame bins (rps_context.hip tracks their validity): its sort head reads them.
  bool pkeys;
  uint32_t n;        // N
  uint32_t p;        // next_pow2(N)
  uint8_t batch_d;   // scan entries in flight per lane, density / sim pass (4, 8, 16;
  uint8_t batch_s;   //   0: by size, sph_batch); per context, RPS_SPH_BATCH[_D|_S] at create
  bool layout;       // this frame uses the spatial record layout (lay.* valid)
  bool sort_fold;    // the first two later sort stages fold their global passes into the tails
  bool csort;        // 2^11 <= P <= 2^16: the compact (4-byte entry) sort, RPS_SPH_CSORT
  uint8_t csort_tlog;  // its tile (11..13; 0: by size), RPS_SPH_CSORT_TLOG
  uint8_t csort_wide;  // its stages of this many folded passes or more fold with twice the threads (0: none), RPS_SPH_CSORT_WIDE
  uint32_t pair_max_p;  // P <= this: density / sim scans by lane pairs (RPS_SPH_PAIRS)
  bool sim_fuse;        // P != N: the sim and its long scans in one launch (RPS_SPH_SIM_FUSE)
  uint8_t lane_group;   // lanes per slot of those scans: 2 or 4 (RPS_SPH_GROUP)
  uint8_t lane_group_s; // the same for the sim's scans (RPS_SPH_GROUP_S; default: lane_group)
  uint32_t cell_cap; // capacity of lay.cell_info / cellrun (0: layout never available)
  SphLayoutArgs lay;
};
// The layout's cell range for `c` if it fits `cell_cap` cells (false: frame without layout).
bool sph_layout_grid(const rps_config& c, uint32_t cell_cap, SphGrid* g);
// Active-frame passes 3-4 with the spatial layout: runs, count, scan, write + predict,
// fixup, density.
hipError_t launch_sph_layout_pre(const SphBuffers& b, hipStream_t s);
// Scan batch of the density (`density`) or sim pass at P entries; `forced` != 0 wins.
int sph_batch(bool density, uint32_t p, int forced, bool layout);
// Runs the whole bitonic network of src/particle_compute.rs:117-149; returns the number of
// reference passes covered (S(S+1)/2) in *passes.
hipError_t launch_sph_sort(const SphBuffers& b, hipStream_t s, uint32_t* passes,
                           uint32_t* launches);
hipError_t launch_sph_offsets(const SphBuffers& b, hipStream_t s);
// Active-frame passes 3-4 without the layout: the predict kernel also runs the offsets pass
// (it needs only the sorted lookup; one launch fewer: 65 536 0.1118 -> 0.1105 ms/frame), then
// density.
hipError_t launch_sph_pre(const SphBuffers& b, hipStream_t s);
hipError_t launch_sph_sim(const SphBuffers& b, hipStream_t s);
// Cost accounting (rps_sph_frame_cost): per workgroup of slots, the (scanned, within-radius)
// neighbour entries of the current frame, as u64 pairs in out[2 * sph_count_blocks(p)].
uint32_t sph_count_blocks(uint32_t p_slots);
hipError_t launch_sph_count(const SphBuffers& b, unsigned long long* out, hipStream_t s);
// Rebuild the per-particle predicted-position and density buffers from the slot records.
hipError_t launch_sph_debug_views(const SphBuffers& b, hipStream_t s);
// Slot-resident state: bin_next from the state (keys of the current config), the state back to
// particle order (dst[perm[u]] = st[u]), and the sorted lookup's payloads as particle indices.
hipError_t launch_sph_rebin(const SphBuffers& b, const uint32_t* perm, hipStream_t s);
hipError_t launch_sph_materialize(const SphBuffers& b, const f4* st, const uint32_t* perm, f4* dst, hipStream_t s);
// The lookup's payloads as particle indices in place (slots through perm, flagged pads unflagged).
hipError_t launch_sph_lookup_canonical(const SphBuffers& b, const uint32_t* perm, hipStream_t s);
hipError_t launch_sph_lookup_translate(const uint2* lookup, const uint32_t* perm, uint2* out, uint32_t p,
                                       hipStream_t s);

}  // namespace rps
