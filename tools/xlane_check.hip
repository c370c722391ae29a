// Wave lane exchanges of the round-5 cross-lane sort schedule (measured slower and not shipped,
// DESIGN.md Appendix A), checked on the GPU: every lane_xor<D> / lane_mirror<M> returns lane
// (l ^ D)'s / (l ^ (M - 1))'s value.  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o
// tools/xlane_check tools/xlane_check.hip; run: tools/xlane_check (exit 0 = pass).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

// Wave lane exchanges (VALU only, no LDS): lane_xor<D>(x) is lane (l ^ D)'s x, lane_mirror<M>(x)
// lane (l ^ (M - 1))'s (the mirror inside each group of M lanes).  DPP row moves for D <= 8 and
// M <= 16 (quad_perm, row_shl/shr:4 + a select, row_ror:8, row_[half_]mirror); gfx950's
// v_permlane16_swap / v_permlane32_swap for the 16- and 32-lane exchanges: with both operands x,
// the swap leaves the other half's x in the lanes of the first result's swapped half and of the
// second result's.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_mov(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
template <int D>
__device__ __forceinline__ uint32_t lane_xor(uint32_t x) {
  static_assert(D == 1 || D == 2 || D == 4 || D == 8 || D == 16 || D == 32, "lane_xor: D");
  if constexpr (D == 1) {
    return dpp_mov<0xB1>(x);  // quad_perm [1, 0, 3, 2]
  } else if constexpr (D == 2) {
    return dpp_mov<0x4E>(x);  // quad_perm [2, 3, 0, 1]
  } else if constexpr (D == 4) {
    const uint32_t up = dpp_mov<0x104>(x);  // row_shl:4: lane l + 4 (lanes with bit 2 clear)
    const uint32_t dn = dpp_mov<0x114>(x);  // row_shr:4: lane l - 4 (bit 2 set)
    return (lane_id() & 4u) ? dn : up;
  } else if constexpr (D == 8) {
    return dpp_mov<0x128>(x);  // row_ror:8 inside a 16-lane row: lane l ^ 8
  } else if constexpr (D == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    return (lane_id() & 16u) ? r[0] : r[1];
  } else {
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    return (lane_id() & 32u) ? r[0] : r[1];
  }
}
template <int M>
__device__ __forceinline__ uint32_t lane_mirror(uint32_t x) {
  static_assert(M == 2 || M == 4 || M == 8 || M == 16 || M == 32 || M == 64, "lane_mirror: M");
  if constexpr (M == 2) return dpp_mov<0xB1>(x);
  else if constexpr (M == 4) return dpp_mov<0x1B>(x);  // quad_perm [3, 2, 1, 0]
  else if constexpr (M == 8) return dpp_mov<0x141>(x);  // row_half_mirror
  else if constexpr (M == 16) return dpp_mov<0x140>(x);  // row_mirror
  else if constexpr (M == 32) return lane_xor<16>(dpp_mov<0x140>(x));
  else return lane_xor<32>(lane_xor<16>(dpp_mov<0x140>(x)));
}

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
