// (diagnostics) HBM store rate by wave-instruction shape, on the split residual stream's tiles: 16-row tiles of 768-B
// rows (one [M][384] f16 tensor), one 12-wave workgroup per CU walking tiles, as mel_proj / res_proj store them.
//   shape 0: each wave stores one contiguous 1 KiB piece of the tile (16 B per lane)
//   shape 1: 16 rows x 32 B per instruction (8 B per lane: lane = 16 * (column quarter) + row), 2 per wave
//            (the swapped-MFMA accumulator's natural store: columns 64 w + 32 j .. + 32 of every row)
//   shape 2: 16 rows x 64 B per instruction (16 B per lane), 1 per wave
// Build: hipcc -O3 --offload-arch=gfx950 tools/store_bench.hip -o tools/store_bench ; run: tools/store_bench [rows]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int SHAPE>
__global__ __launch_bounds__(768, 1) void store_kernel(unsigned char* out, int tiles, int reps) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fk = lane >> 4;
  for (int r = 0; r < reps; ++r)
    for (int t = blockIdx.x; t < tiles; t += gridDim.x) {
      unsigned char* tile = out + (size_t)t * 16 * 768;
      if (SHAPE == 0) {
        *reinterpret_cast<uint4*>(tile + wave * 1024 + lane * 16) = make_uint4(t, r, lane, wave);
      } else if (SHAPE == 1) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
          *reinterpret_cast<uint2*>(tile + fr * 768 + 64 * wave + 32 * j + 8 * fk) = make_uint2(t, r + j);
      } else {
        *reinterpret_cast<uint4*>(tile + fr * 768 + 64 * wave + 16 * fk) = make_uint4(t, r, lane, wave);
      }
    }
}

int main(int argc, char** argv) {
  const int rows = argc > 1 ? atoi(argv[1]) : 29984;
  const int tiles = (rows + 15) / 16;
  unsigned char* out = nullptr;
  if (hipMalloc(&out, (size_t)tiles * 16 * 768) != hipSuccess) return 1;
  int ncu = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  void (*fns[3])(unsigned char*, int, int) = {store_kernel<0>, store_kernel<1>, store_kernel<2>};
  const char* names[3] = {"1 KiB contiguous / instr", "16 rows x 32 B / instr", "16 rows x 64 B / instr"};
  for (int rep = 0; rep < 2; ++rep)
    for (int s = 0; s < 3; ++s) {
      hipLaunchKernelGGL(fns[s], dim3(ncu), dim3(768), 0, 0, out, tiles, 1);
      (void)hipEventRecord(e0, 0);
      const int reps = 20;
      for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(fns[s], dim3(ncu), dim3(768), 0, 0, out, tiles, 1);
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      const double us = 1000.0 * ms / reps, bytes = (double)tiles * 16 * 768;
      printf("%-28s %8.2f us per launch  %6.2f TB/s  (%d rows, %.1f MB)\n", names[s], us, bytes / us * 1e-6, rows,
             bytes * 1e-6);
    }
  (void)hipFree(out);
  return 0;
}
