// rps_demo.cpp — headless re-run of the reference app loop (src/main.rs:71-134) through the
// C++ host mirror: ParticleConfig defaults, seeded scatter, prepare_particle_buffers on the
// first frame, then per frame apply_gui_updates -> prepare (config upload) ->
// ParticleComputeNode::run.  Writes the initial and final AoS state so a test can replay
// the same frames on the CPU oracle.
//
//   rps_demo <mode:sph|stream> <particles> <frames> <out-prefix> [gui-change-frame]
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "particle_plugin.hpp"

using namespace rps_host;

static void dump(const std::string& path, const std::vector<Particle>& p) {
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) throw std::runtime_error("cannot write " + path);
  std::fwrite(p.data(), sizeof(Particle), p.size(), f);
  std::fclose(f);
}

int main(int argc, char** argv) {
  if (argc < 5) {
    std::fprintf(stderr, "usage: %s sph|stream <particles> <frames> <out-prefix> [gui-change-frame]\n", argv[0]);
    return 2;
  }
  try {
    const uint32_t mode = std::strcmp(argv[1], "stream") == 0 ? RPS_MODE_STREAM : RPS_MODE_SPH;
    const uint32_t n = (uint32_t)std::strtoul(argv[2], nullptr, 10);
    const int frames = std::atoi(argv[3]);
    const std::string out = argv[4];
    const int gui_frame = argc > 5 ? std::atoi(argv[5]) : -1;

    ParticleConfig config = default_particle_config(n);
    GUIConfig gui;
    ParticleSystem system = setup_particles_scatter(config, 0x5EED);
    dump(out + "_init.bin", system.particles);

    std::unique_ptr<GPUPipelineBuffers> buffers;
    ParticleComputeNode node;
    for (int frame = 0; frame < frames; ++frame) {
      if (frame == gui_frame) {  // a slider move (src/parameter_gui.rs:38-70)
        gui.gravity = 200.0f;
        gui.smoothing_radius = 12.0f;
        gui.applied_changes = true;
      }
      apply_gui_updates(config, gui);                          // PreUpdate
      prepare_particle_buffers(system, config, buffers, mode);  // RenderSet::Prepare
      node.update(buffers.get());
      int st = node.run();                                      // render graph
      if (st != RPS_OK) {
        std::fprintf(stderr, "run failed: %s\n", rps_last_error(buffers->ctx()));
        return 1;
      }
    }
    check(rps_sync(buffers->ctx()), buffers->ctx(), "rps_sync");
    uint32_t fc = 0;
    uint64_t active = 0;
    rps_get_counters(buffers->ctx(), &fc, &active);
    dump(out + "_final.bin", buffers->download());
    FILE* fc_out = std::fopen((out + "_config.bin").c_str(), "wb");  // main-world config at exit
    if (fc_out) {
      std::fwrite(&config, sizeof(config), 1, fc_out);
      std::fclose(fc_out);
    }
    std::printf("{\"frames\": %d, \"frame_count\": %u, \"active_steps\": %llu, \"particles\": %u}\n", frames, fc,
                (unsigned long long)active, n);
    return 0;
  } catch (const Error& e) {
    std::fprintf(stderr, "rps error %d: %s\n", e.status, e.what());
    return 1;
  }
}
