// Micro-benchmark (GPU): per-CU operand delivery rate from an L2-resident buffer, one 512-thread workgroup per CU,
// for the forms the GEMM kernels could use to fill LDS:
//   0  global_load_lds_dwordx4 (LDS-DMA), 16 rows x 64 B per wave-instruction   (diff_layer.hip's K-step images)
//   1  global_load_lds_dwordx4, 8 rows x 128 B per wave-instruction             (conv_gemm3 / conv_gemm4 images)
//   2  global_load_dwordx4 into VGPRs + ds_write_b128                           (register staging)
//   3  global_load_dwordx4 into VGPRs only (no LDS)
//   4  LDS-DMA, 64 B rows, 2 DMA-issuing waves of 8 (the others only wait at the barrier)
// Each iteration moves `kb` KiB per workgroup into a 4-slot ring (one barrier per iteration, vmcnt lookahead 2).
// Build: hipcc -O3 --offload-arch=gfx950 tools/dma_rate.hip -o tools/dma_rate ; run: tools/dma_rate
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

template <int N>
__device__ __forceinline__ void vmwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// per wave per iteration: NI wave-instructions of 1 KiB (NI = 3 -> 24 KiB per workgroup per iteration)
template <int MODE, int NI>
__global__ __launch_bounds__(512, 1) void rate_kernel(const unsigned char* src, size_t src_bytes, int iters,
                                                      float* sink) {
  extern __shared__ __align__(16) unsigned char sm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const size_t stride = 8 * NI * 1024;
  const size_t wrap = src_bytes - stride;
  float acc = 0.f;
  if constexpr (MODE <= 1 || MODE == 4) {
    for (int it = 0; it < iters; ++it) {
      unsigned char* dst = sm + (it & 3) * stride;
      const size_t base = ((size_t)it * stride) % wrap;
      if constexpr (MODE == 4) {
        if (wave < 2) {
#pragma unroll
          for (int v = 0; v < NI * 4; ++v) {
            const int piece = wave * NI * 4 + v;
            const size_t off = base + (size_t)piece * 1024 + (lane >> 2) * 64 + (lane & 3) * 16;
            __builtin_amdgcn_global_load_lds(src + off, (__attribute__((address_space(3))) void*)(dst + piece * 1024),
                                             16, 0, 0);
          }
          vmwait<24>();
        }
      } else {
#pragma unroll
        for (int v = 0; v < NI; ++v) {
          const int piece = wave * NI + v;
          size_t off;
          if constexpr (MODE == 0) off = base + (size_t)piece * 1024 + (lane >> 2) * 64 + (lane & 3) * 16;
          else off = base + (size_t)piece * 1024 + (lane >> 3) * 128 + (lane & 7) * 16;
          __builtin_amdgcn_global_load_lds(src + off, (__attribute__((address_space(3))) void*)(dst + piece * 1024),
                                           16, 0, 0);
        }
        vmwait<2 * NI>();  // two iterations in flight, as diff_layer's ring
      }
      bar();
    }
  } else {
    uint4 r0[NI], r1[NI], r2[NI];
    auto load = [&](uint4* r, int it) {
      const size_t base = ((size_t)it * stride) % wrap;
#pragma unroll
      for (int v = 0; v < NI; ++v)
        r[v] = *(reinterpret_cast<const uint4*>(src + base + (size_t)(wave * NI + v) * 1024 +
                                                                         lane * 16));
    };
    auto use = [&](uint4* r, int it) {
      if constexpr (MODE == 2) {
#pragma unroll
        for (int v = 0; v < NI; ++v)
          *reinterpret_cast<uint4*>(sm + (it & 3) * stride + (wave * NI + v) * 1024 + lane * 16) = r[v];
      } else {
#pragma unroll
        for (int v = 0; v < NI; ++v) acc += __uint_as_float(r[v].x ^ r[v].w);
      }
    };
    load(r0, 0);
    load(r1, 1);
    for (int it = 0; it < iters; it += 3) {
      load(r2, it + 2);
      use(r0, it);
      bar();
      load(r0, it + 3);
      use(r1, it + 1);
      bar();
      load(r1, it + 4);
      use(r2, it + 2);
      bar();
    }
  }
  vmwait<0>();
  acc += __uint_as_float(*reinterpret_cast<const unsigned*>(sm + tid * 4));
  if (acc == 1.2345f) sink[blockIdx.x] = acc;
}

template <int MODE, int NI>
void run(const unsigned char* src, size_t bytes, int ncu, float* sink, const char* name) {
  const int iters = 2001;
  const int lds = 4 * 8 * NI * 1024;
  CK(hipFuncSetAttribute((const void*)rate_kernel<MODE, NI>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL((rate_kernel<MODE, NI>), dim3(ncu), dim3(512), lds, 0, src, bytes, iters, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    const double per_cu = (double)iters * 8 * NI * 1024 / (ms * 1e-3) / 1e9;
    if (rep == 2) printf("%-46s %7.3f ms  %6.1f GB/s per CU  %6.2f TB/s chip\n", name, ms, per_cu, per_cu * ncu / 1e3);
  }
}

int main() {
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const size_t bytes = 2u << 20;  // 2 MiB: L2-resident on every XCD (the GEMM weight slabs are 0.3-1.8 MB)
  unsigned char* src;
  float* sink;
  CK(hipMalloc(&src, bytes));
  CK(hipMemset(src, 1, bytes));
  CK(hipMalloc(&sink, 4096 * 4));
  printf("CUs %d, source %zu KiB, one 512-thread workgroup per CU\n", ncu, bytes >> 10);
  run<0, 3>(src, bytes, ncu, sink, "LDS-DMA 64-B rows, 24 KiB/iter");
  run<1, 3>(src, bytes, ncu, sink, "LDS-DMA 128-B rows, 24 KiB/iter");
  run<0, 2>(src, bytes, ncu, sink, "LDS-DMA 64-B rows, 16 KiB/iter");
  run<2, 3>(src, bytes, ncu, sink, "VGPR load + ds_write_b128, 24 KiB/iter");
  run<3, 3>(src, bytes, ncu, sink, "VGPR load only, 24 KiB/iter");
  run<4, 3>(src, bytes, ncu, sink, "LDS-DMA 64-B rows, 2 issuing waves, 24 KiB");
  return 0;
}
