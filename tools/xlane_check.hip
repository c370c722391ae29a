// Checks rps_device.hpp's wave lane exchanges on the GPU: every lane_xor<D> / lane_mirror<M>
// returns lane (l ^ D)'s / (l ^ (M - 1))'s value.  Build: hipcc --offload-arch=gfx950 -O3
// -I include -o tools/xlane_check tools/xlane_check.hip; run: tools/xlane_check (exit 0 = pass).
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../rust-particle-system_amd/csrc/rps_device.hpp"

using namespace rps;

__global__ void probe(uint32_t* out) {
  const uint32_t l = threadIdx.x, x = 1000u + l;
  uint32_t* o = out + 64u * 0u;
  o[0 * 64 + l] = lane_xor<1>(x);
  o[1 * 64 + l] = lane_xor<2>(x);
  o[2 * 64 + l] = lane_xor<4>(x);
  o[3 * 64 + l] = lane_xor<8>(x);
  o[4 * 64 + l] = lane_xor<16>(x);
  o[5 * 64 + l] = lane_xor<32>(x);
  o[6 * 64 + l] = lane_mirror<2>(x);
  o[7 * 64 + l] = lane_mirror<4>(x);
  o[8 * 64 + l] = lane_mirror<8>(x);
  o[9 * 64 + l] = lane_mirror<16>(x);
  o[10 * 64 + l] = lane_mirror<32>(x);
  o[11 * 64 + l] = lane_mirror<64>(x);
}

int main() {
  uint32_t* d;
  if (hipMalloc(&d, 12 * 64 * 4) != hipSuccess) return 2;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  uint32_t h[12 * 64];
  if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 2;
  const char* names[12] = {"xor1", "xor2", "xor4", "xor8", "xor16", "xor32",
                           "mirror2", "mirror4", "mirror8", "mirror16", "mirror32", "mirror64"};
  const uint32_t mask[12] = {1, 2, 4, 8, 16, 32, 1, 3, 7, 15, 31, 63};
  int bad = 0;
  for (int k = 0; k < 12; ++k) {
    int fail = 0;
    for (uint32_t l = 0; l < 64; ++l)
      if (h[k * 64 + l] != 1000u + (l ^ mask[k])) {
        if (!fail) printf("%s: lane %u got lane %d\n", names[k], l, (int)h[k * 64 + l] - 1000);
        ++fail;
      }
    printf("%-9s %s\n", names[k], fail ? "FAIL" : "ok");
    bad += fail;
  }
  (void)hipFree(d);
  return bad ? 1 : 0;
}
