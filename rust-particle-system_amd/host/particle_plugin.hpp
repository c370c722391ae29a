// particle_plugin.hpp — C++ host mirror of the reference's particle-plugin surface, calling
// the gfx950 kernels through the C ABI (include/rps.h).  Header-only.
//
// Reference surface (mabrams4/Rust-Particle-System)            here
//   Particle                     src/particle.rs:20-25           rps_host::Particle
//   ParticleSystem               src/main.rs:37-41               rps_host::ParticleSystem
//   ParticleConfig + consts      src/main.rs:25-35, :43-108      rps_host::ParticleConfig, default_particle_config
//   get_screen_bounds            src/main.rs:136-153             rps_host::screen_bounds
//   setup_particles_scatter      src/main.rs:182-216             rps_host::setup_particles_scatter (seeded)
//   GUIConfig, apply_gui_updates src/parameter_gui.rs:6-22,78-102 rps_host::GUIConfig, apply_gui_updates
//   GPUPipelineBuffers           src/particle_buffers.rs:17-26   rps_host::GPUPipelineBuffers (owns an rps_ctx)
//   prepare_particle_buffers     src/particle_buffers.rs:38-237  rps_host::prepare_particle_buffers
//   ParticleComputeNode run/update src/particle_compute.rs:84-211 rps_host::ParticleComputeNode
//   read_*_from_gpu              src/debug.rs:121-265            GPUPipelineBuffers::read_debug
//
// Error behaviour follows the reference: setup failures that the reference `unwrap()`s
// (src/particle_buffers.rs:63-81) throw rps_host::Error; ParticleComputeNode::run skips
// entities whose buffers are not prepared yet (src/particle_compute.rs:102-103) and always
// "succeeds" for them, but a device error from a launched step is returned, not swallowed.
#pragma once

#include <cmath>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <memory>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/rps.h"

namespace rps_host {

struct Error : std::runtime_error {
  int status;
  Error(int s, const std::string& m) : std::runtime_error(m), status(s) {}
};

inline void check(int status, const rps_ctx* ctx, const char* what) {
  if (status != RPS_OK)
    throw Error(status, std::string(what) + ": " + rps_status_string(status) + ": " + rps_last_error(ctx));
}

// == Particle (src/particle.rs:20-25): 32 B, position @0, velocity @8, color @16.
struct Particle {
  float position[2];
  float velocity[2];
  float color[4];
};
static_assert(sizeof(Particle) == sizeof(rps_particle), "Particle must stay 32 bytes");
static_assert(offsetof(Particle, velocity) == 8 && offsetof(Particle, color) == 16, "Particle layout");

// == ParticleConfig (src/main.rs:43-69, #[repr(C)] Pod, 144 B).
using ParticleConfig = rps_config;
static_assert(sizeof(ParticleConfig) == 144, "ParticleConfig must stay 144 bytes");

// Constants, src/main.rs:25-35.
constexpr uint32_t PARTICLE_COUNT = 50000;
constexpr float PARTICLE_SIZE = 3.0f;
constexpr float SMOOTHING_RADIUS = PARTICLE_SIZE * PARTICLE_SIZE;
constexpr float GRAVITY = 0.0f;
constexpr float TARGET_DENSITY = 0.011f;
constexpr float PRESSURE_MULTIPLIER = 10000.0f;
constexpr float NEAR_DENSITY_MULTIPLIER = 1000.0f;
constexpr float VISCOCITY_STRENGTH = 5.0f;
constexpr float DAMPING_FACTOR = 0.1f;
constexpr float FIXED_DELTA_TIME = 1.0f / 100.0f;
constexpr float MAX_ENERGY = 2000.0f;
constexpr float PI_F32 = 3.14159265358979323846f;  // std::f32::consts::PI

// == ParticleSystem component (src/main.rs:37-41).
struct ParticleSystem {
  std::vector<Particle> particles;
};

// Kernel norms as in src/main.rs:96-98 / src/parameter_gui.rs:89-91 (f32 powf).
inline void kernel_norms(float r, float& density, float& near_density, float& viscosity) {
  density = 10.0f / (PI_F32 * std::pow(r, 5.0f));
  near_density = 15.0f / (PI_F32 * std::pow(r, 6.0f));
  viscosity = 4.0f / (PI_F32 * std::pow(r, 8.0f));
}

// get_screen_bounds (src/main.rs:136-153) for a camera at (cx, cy).
inline void screen_bounds(float width, float height, float cx, float cy, float out[4]) {
  out[0] = cx - width / 2.0f;
  out[1] = cx + width / 2.0f;
  out[2] = cy - height / 2.0f;
  out[3] = cy + height / 2.0f;
}

// The ParticleConfig resource main() inserts (src/main.rs:85-108).
inline ParticleConfig default_particle_config(uint32_t particle_count = PARTICLE_COUNT,
                                              float width = 1920.0f, float height = 1080.0f) {
  ParticleConfig c;
  std::memset(&c, 0, sizeof(c));
  c.particle_count = particle_count;
  c.particle_size = PARTICLE_SIZE;
  c.smoothing_radius = SMOOTHING_RADIUS;
  c.max_energy = MAX_ENERGY;
  c.damping_factor = DAMPING_FACTOR;
  c.fixed_delta_time = FIXED_DELTA_TIME;
  c.frame_count = 0;
  c.gravity = GRAVITY;
  kernel_norms(SMOOTHING_RADIUS, c.density_kernel_norm, c.near_density_kernel_norm, c.viscocity_kernel_norm);
  c.target_density = TARGET_DENSITY;
  c.pressure_multiplier = PRESSURE_MULTIPLIER;
  c.viscocity_strength = VISCOCITY_STRENGTH;
  c.near_density_multiplier = NEAR_DENSITY_MULTIPLIER;
  screen_bounds(width, height, 0.0f, 0.0f, c.screen_bounds);
  for (int k = 0; k < 16; ++k) c.view_proj[k] = (k % 5 == 0) ? 1.0f : 0.0f;  // Mat4::IDENTITY
  return c;
}

// setup_particles_scatter (src/main.rs:182-216) with a seeded generator in place of the
// unseeded rand::rng() (src/main.rs:188): x linear in i, y ~ Normal(centre, 0.125 H)
// clamped, v = 0, colour white.
inline ParticleSystem setup_particles_scatter(const ParticleConfig& cfg, uint64_t seed) {
  const float x_min = cfg.screen_bounds[0], x_max = cfg.screen_bounds[1];
  const float y_min = cfg.screen_bounds[2], y_max = cfg.screen_bounds[3];
  std::mt19937_64 rng(seed);
  std::normal_distribution<float> y_dist((y_min + y_max) / 2.0f, (y_max - y_min) * 0.125f);
  ParticleSystem sys;
  sys.particles.resize(cfg.particle_count);
  for (uint32_t i = 0; i < cfg.particle_count; ++i) {
    const float t = (float)i / (float)cfg.particle_count;
    float y = y_dist(rng);
    y = y < y_min ? y_min : (y > y_max ? y_max : y);
    sys.particles[i] = Particle{{x_min + t * (x_max - x_min), y}, {0.0f, 0.0f}, {1.0f, 1.0f, 1.0f, 1.0f}};
  }
  return sys;
}

// == GUIConfig (src/parameter_gui.rs:6-22).
struct GUIConfig {
  float fixed_delta_time = FIXED_DELTA_TIME;
  float gravity = GRAVITY;
  float damping_factor = DAMPING_FACTOR;
  float smoothing_radius = SMOOTHING_RADIUS;
  float max_energy = MAX_ENERGY;
  float target_density = TARGET_DENSITY;
  float pressure_multiplier = PRESSURE_MULTIPLIER;
  float viscocity_strength = VISCOCITY_STRENGTH;
  float near_density_multiplier = NEAR_DENSITY_MULTIPLIER;
  bool applied_changes = false;
};

// == apply_gui_updates (src/parameter_gui.rs:78-102).
inline void apply_gui_updates(ParticleConfig& sim, GUIConfig& gui) {
  if (!gui.applied_changes) return;
  sim.fixed_delta_time = gui.fixed_delta_time;
  sim.gravity = gui.gravity;
  sim.damping_factor = gui.damping_factor;
  kernel_norms(gui.smoothing_radius, sim.density_kernel_norm, sim.near_density_kernel_norm,
               sim.viscocity_kernel_norm);
  sim.smoothing_radius = gui.smoothing_radius;
  sim.max_energy = gui.max_energy;
  sim.target_density = gui.target_density;
  sim.pressure_multiplier = gui.pressure_multiplier;
  sim.viscocity_strength = gui.viscocity_strength;
  sim.near_density_multiplier = gui.near_density_multiplier;
  gui.applied_changes = false;
}

// == GPUPipelineBuffers (src/particle_buffers.rs:17-26): owns the device context (the
// hipMalloc'd tiled-SoA state, spatial lookup, offsets, densities, predicted positions and
// the device-resident config).  Move-only; freed on destruction.
class GPUPipelineBuffers {
 public:
  GPUPipelineBuffers(const rps_create_info& info) {
    rps_ctx* c = nullptr;
    check(rps_create(&info, &c), nullptr, "rps_create");
    ctx_.reset(c);
  }
  rps_ctx* ctx() const { return ctx_.get(); }
  uint64_t particle_count() const { return n_; }

  void set_config(const ParticleConfig& cfg, const rps_ext_config* ext) {
    check(rps_set_config(ctx(), &cfg, ext), ctx(), "rps_set_config");
  }
  void upload(const std::vector<Particle>& p) {
    n_ = p.size();
    check(rps_upload_particles(ctx(), reinterpret_cast<const rps_particle*>(p.data()), 0, p.size()),
          ctx(), "rps_upload_particles");
  }
  std::vector<Particle> download() const {
    std::vector<Particle> out(n_);
    check(rps_download_particles(ctx(), reinterpret_cast<rps_particle*>(out.data()), 0, n_), ctx(),
          "rps_download_particles");
    return out;
  }
  // src/debug.rs:121-265 readbacks (spatial lookup, offsets, densities, predicted).
  template <class T>
  std::vector<T> read_debug(int which, size_t count) const {
    std::vector<T> out(count);
    check(rps_read_debug(ctx(), which, out.data(), count * sizeof(T)), ctx(), "rps_read_debug");
    return out;
  }

 private:
  struct Deleter {
    void operator()(rps_ctx* c) const { rps_destroy(c); }
  };
  std::unique_ptr<rps_ctx, Deleter> ctx_;
  uint64_t n_ = 0;
};

// == prepare_particle_buffers (src/particle_buffers.rs:38-237).  First call: allocate and
// upload the particles once (:50-216).  Later calls model the render-world copy of the
// config: `config` is the main-world resource, whose frame_count is never incremented
// (only the render-world copy is, :227 — inside rps_step here).  Bevy re-extracts the
// resource only when the main-world value changed (ExtractResourcePlugin, src/particle.rs:35),
// and the extracted copy carries frame_count = 0: a GUI change therefore resets frame_count
// and re-arms the SHADER_DELAY gate.  Unchanged configs keep the device's
// running frame_count.
inline void prepare_particle_buffers(const ParticleSystem& system, ParticleConfig& config,
                                     std::unique_ptr<GPUPipelineBuffers>& buffers,
                                     uint32_t mode = RPS_MODE_SPH,
                                     const rps_ext_config* ext = nullptr, int device = 0) {
  if (!buffers) {
    rps_create_info info{device, mode, system.particles.size(), 0, system.particles.size()};
    buffers = std::make_unique<GPUPipelineBuffers>(info);
    buffers->set_config(config, ext);
    buffers->upload(system.particles);
    return;
  }
  rps_config cur;
  rps_ext_config cur_ext;
  check(rps_get_config(buffers->ctx(), &cur, &cur_ext), buffers->ctx(), "rps_get_config");
  rps_config probe = config;
  probe.frame_count = cur.frame_count;
  const bool changed = std::memcmp(&probe, &cur, sizeof(cur)) != 0 ||
                       (ext && std::memcmp(ext, &cur_ext, sizeof(cur_ext)) != 0);
  if (changed) buffers->set_config(config, ext);  // extract-on-change: frame_count <- main world's
}

// == ParticleComputeNode (src/particle_compute.rs:84-211).
class ParticleComputeNode {
 public:
  // update (:197-199): refresh the entity query; here the list of prepared buffers.
  void update(GPUPipelineBuffers* buffers) {
    if (buffers) {
      check(rps_update(buffers->ctx()), buffers->ctx(), "rps_update");
      entity_ = buffers;
    }
  }
  // run (:91-195): record bin -> sort -> offsets -> pre_sim -> sim (or the fused stream
  // step) on the context stream.  No-op while no buffers are prepared (:102-103).
  int run() {
    if (!entity_) return RPS_OK;
    return rps_step(entity_->ctx(), 1);
  }

 private:
  GPUPipelineBuffers* entity_ = nullptr;
};

}  // namespace rps_host
