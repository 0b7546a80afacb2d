// xcd_map_probe.hip -- which XCD (and SE / CU) each workgroup of a launch
// runs on.  The row kernels' block orders assume round-robin dispatch,
// workgroup b on XCD b % 8 (spmv_device.cuh xcd_chunk_remap, the csort column
// parts); this records the mapping a box actually uses, next to host.txt,
// so a box whose dispatch differs can be told apart from a kernel change.
//
//   build:  make -C heterogeneous-spmv_amd build/xcd_map_probe
//   run:    build/xcd_map_probe [blocks] [threads]   -> one JSON line
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

// s_getreg_b32 hwreg(id, offset 0, size 32): XCC_ID = 20, HW_ID = 4 (gfx9)
#define HWREG32(id) ((31 << 11) | (id))

__global__ void probe(uint32_t *xcc, uint32_t *hwid) {
  if (threadIdx.x == 0) {
    xcc[blockIdx.x] = __builtin_amdgcn_s_getreg(HWREG32(20));
    hwid[blockIdx.x] = __builtin_amdgcn_s_getreg(HWREG32(4));
  }
}

int main(int argc, char **argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 2048;
  const int threads = argc > 2 ? atoi(argv[2]) : 256;
  uint32_t *dx = nullptr, *dh = nullptr;
  if (hipMalloc(&dx, 4 * blocks) != hipSuccess || hipMalloc(&dh, 4 * blocks) != hipSuccess) return 1;
  hipLaunchKernelGGL(probe, dim3(blocks), dim3(threads), 0, 0, dx, dh);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  std::vector<uint32_t> x(blocks), h(blocks);
  if (hipMemcpy(x.data(), dx, 4 * blocks, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(h.data(), dh, 4 * blocks, hipMemcpyDeviceToHost) != hipSuccess)
    return 1;
  int match = 0, nxcd = 0;
  std::vector<int> per(16, 0);
  for (int b = 0; b < blocks; ++b) {
    const int id = (int)(x[b] & 0xF);
    per[id]++;
    match += id == b % 8;
  }
  for (int v : per) nxcd += v > 0;
  printf("{\"blocks\":%d,\"threads\":%d,\"xcds_seen\":%d,\"round_robin_b_mod_8\":%.4f,\"first32_xcc\":[",
         blocks, threads, nxcd, (double)match / blocks);
  for (int b = 0; b < 32 && b < blocks; ++b) printf("%s%u", b ? "," : "", x[b] & 0xF);
  printf("],\"first8_hwid\":[");
  for (int b = 0; b < 8 && b < blocks; ++b) printf("%s\"0x%08x\"", b ? "," : "", h[b]);
  printf("],\"per_xcd\":[");
  for (int i = 0; i < 8; ++i) printf("%s%d", i ? "," : "", per[i]);
  printf("]}\n");
  return 0;
}
