// Fused DiffSVC head for gfx950 (modules/diffsvc.py:311-321) after the skip sum, one launch per 128-row tile:
//   GEMM A  u = relu(s . W_sp + b_sp): s = the split-fp16 skip sum [hi | lo | hi] (K = 1152), N = 384, through a
//           4-slot ring of 32-deep K-steps (A 128 x 64 B + B 384 x 64 B = 32 KiB per slot, three steps ahead: one
//           tile per CU, so the step time is the DMA latency over the steps in flight); software-pipelined: a step's
//           MFMAs run on fragments read during the previous step, with the next step's reads and DMAs between them
//           (round 5: 58.5 -> 57.0 -> 56.2 us per full-batch launch, r05v / r05x);
//   GEMM B  eps = [u_hi | u_lo | u_hi] . W_out + b_out, N = 100 (packed rows to 128): u_hi as an f16 image in LDS
//           (over GEMM A's ring), u_lo packed in registers and written over the image for the last third, so the
//           138 MB split-fp16 intermediate of a full-batch call never reaches HBM; W_out K-steps through a 4-slot ring
//           whose first three steps load at kernel start.
//           K runs hi . W_hi, hi . W_lo, lo . W_hi (the unfused GEMM: hi, lo, hi), so the f32 sum differs from the
//           unfused path's in rounding order only (tests/test_gpu_stages.py::test_fused_head).
// Same epilogue expressions as conv_gemm3's LDS epilogue for these two calls (relu(acc + bias), hi = f16(v),
// lo = f16(v - hi); eps = acc + bias). Round 2 also built the following PLMS update and the next denoise's input
// projection into this epilogue, and a fused residual layer (gate GEMM + output projection in one launch); all three
// measured slower end to end and were removed in round 3. Round 6 built the PLMS update into this head's
// epilogue once more (its operands loaded at once, the stores undrained): bit-identical and 0.1 % slower end to end
// (2 x 101 fewer launches, but 8 waves per CU leave the epilogue's loads latency-bound), removed.
#include "common.h"

namespace svc {

constexpr int DL_BM = 128, DL_NT = 512, DL_C = 384;
constexpr int DL_KS2 = DL_C / 32;               // 12 K-steps per third of GEMM B
constexpr int DL_GCHUNK = DL_BM * 256;          // u image chunk: 128 rows x 128 channels f16
constexpr int DH_S1 = 3 * DL_C / 32;            // 36 K-steps of each GEMM
constexpr int DH_SLOT_A = 32 * 1024;            // GEMM A ring slot (4 slots)
constexpr int DH_IMG = 0;                       // u image [3 chunks][128 rows][256 B] = 96 KiB, over GEMM A's ring
constexpr int DH_RING_B = 128 * 1024;           // GEMM B ring: 4 x 8 KiB
constexpr int DH_LDS = DH_RING_B + 4 * 8192;    // 160 KiB

// 64-B image rows (one 32-deep K-step): a 16-B chunk q of row r sits at q ^ ((r >> 1) & 2); conflict-free for the
// ds_read_b128 lane groups of a 16-row MFMA fragment read (every 16 lanes of a group hit 16 distinct 16-B bank slots)
__device__ __forceinline__ int dl_sw64(int row, int q) { return q ^ ((row >> 1) & 2); }
// u image rows of 256 B (128 channels): chunk q at q ^ (row & 15), conflict-free for the GEMM B A fragments
__device__ __forceinline__ int dl_swg(int row, int q) { return q ^ (row & 15); }

__device__ __forceinline__ void dl_dma(const void* src, unsigned char* lds) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}
template <int N>
__device__ __forceinline__ void dl_vmwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void dl_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

union DlH4 {
  uint2 u;
  f16 h[4];
};

__device__ __forceinline__ int dl_xcd_remap() {  // consecutive tiles on one XCD
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
}

struct DiffHeadArgs {
  const f16* s16;    // [rows][1152] split-fp16 skip sum
  const f16* Wsp;    // skip_projection packed [>= 384][1152]
  const float* bsp;
  const f16* Wout;   // output_projection packed [>= 128][1152] (rows >= 100 zero)
  const float* bout;
  float* eps;        // [rows][ld_eps]
  int ld_eps, n_out, M;
};

template <bool BF>
__global__ __launch_bounds__(DL_NT, 1) void diff_head_kernel(DiffHeadArgs p, const f16* zpage) {
  using O = Op16<BF>;  // operand format (binary16 or bfloat16)
  extern __shared__ __align__(16) unsigned char sm[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int M = p.M;
  const int m0 = dl_xcd_remap() * DL_BM;
  const int fr = lane & 15, fk = lane >> 4;
  const f16* zsrc = zpage + lane * 8;
  constexpr int LDS_ = 3 * DL_C;  // 1152 halves per s16 row / packed weight row

  // GEMM A DMA slots: A row wave * 16 + (lane >> 2); B rows wave * 48 + v * 16 + (lane >> 2), v < 3
  const int ar = wave * 16 + (lane >> 2);
  const f16* a_p = (m0 + ar < M) ? p.s16 + (int64_t)(m0 + ar) * LDS_ + dl_sw64(ar, lane & 3) * 8 : nullptr;
  const f16* b_p[3];
#pragma unroll
  for (int v = 0; v < 3; ++v) {
    const int row = wave * 48 + v * 16 + (lane >> 2);
    b_p[v] = p.Wsp + (int64_t)row * LDS_ + dl_sw64(row, lane & 3) * 8;
  }
  const int orow = wave * 16 + (lane >> 2);  // GEMM B weight rows (128)
  const f16* o_p = p.Wout + (int64_t)orow * LDS_ + dl_sw64(orow, lane & 3) * 8;
  // A K-step's DMAs (GEMM A: 1 A piece + 3 B pieces per wave; GEMM B: 1 piece), issued between the step's MFMAs (below).
  // Steps past the end DMA the zero page into the free slot, so every step's vmcnt count is the same.
  auto dmaA = [&](int s, int v) __attribute__((always_inline)) {  // v = 0: A piece, 1..3: B pieces
    unsigned char* st = sm + (s & 3) * DH_SLOT_A;
    const bool live = s < DH_S1;
    if (v == 0)
      dl_dma(live && a_p ? (const void*)(a_p + s * 32) : (const void*)zsrc, st + wave * 1024);
    else
      dl_dma(live ? (const void*)(b_p[v - 1] + s * 32) : (const void*)zsrc, st + 8192 + (wave * 3 + v - 1) * 1024);
  };
  auto issueA = [&](int s_in) {
    int s;
    asm volatile("s_mov_b32 %0, %1" : "=s"(s) : "s"(s_in));
#pragma unroll
    for (int v = 0; v < 4; ++v) dmaA(s, v);
  };
  auto issueB = [&](int s_in) {  // GEMM B step s reads weight K-step 0-11, 24-35, 12-23 (see GEMM B)
    int s;
    asm volatile("s_mov_b32 %0, %1" : "=s"(s) : "s"(s_in));
    const int ws = s < DL_KS2 ? s : (s < 2 * DL_KS2 ? s + DL_KS2 : s - DL_KS2);
    dl_dma(s < DH_S1 ? (const void*)(o_p + ws * 32) : (const void*)zsrc, sm + DH_RING_B + (s & 3) * 8192 + wave * 1024);
  };

  // ---- GEMM A
  floatx4 acc[4][6];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  issueB(0);  // GEMM B's first weight steps: their own ring, older than every GEMM A DMA (in-order vmcnt)
  issueB(1);
  issueB(2);
  issueA(0);
  issueA(1);
  issueA(2);
  // Software-pipelined K-loop: step s's MFMAs run from fragments read during step s - 1, and between them go step
  // s + 1's fragment reads and step s + 3's four DMAs (one after every six MFMAs). Before, each step read its own
  // fragments after the barrier and waited on them, and both waves of a SIMD issued their DMAs in one burst (an
  // LDS-DMA costs its wave ~60 issue cycles among MFMAs but 100-185 in a burst, MI355X_MICROARCH.md): the matrix pipe
  // idled ~0.75 us per step (round 5). The wait before step s retires step s + 1 (one DMA step less in flight).
  half8 af[2][4], bf[2][6];
  auto readA = [&](int s, half8 (&a4)[4], half8 (&b6)[6], int part) __attribute__((always_inline)) {
    const unsigned char* A = sm + (s & 3) * DH_SLOT_A;
    const unsigned char* Bm = A + 8192;
    if (part == 0 || part < 0)
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int row = wn * 96 + j * 16 + fr;
        b6[j] = *reinterpret_cast<const half8*>(Bm + row * 64 + (dl_sw64(row, fk) << 4));
      }
    if (part == 1 || part < 0)
#pragma unroll
      for (int j = 3; j < 6; ++j) {
        const int row = wn * 96 + j * 16 + fr;
        b6[j] = *reinterpret_cast<const half8*>(Bm + row * 64 + (dl_sw64(row, fk) << 4));
      }
    if (part == 2 || part < 0)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = wm * 64 + i * 16 + fr;
        a4[i] = *reinterpret_cast<const half8*>(A + row * 64 + (dl_sw64(row, fk) << 4));
      }
    if (part == 3 || part < 0)
#pragma unroll
      for (int i = 2; i < 4; ++i) {
        const int row = wm * 64 + i * 16 + fr;
        a4[i] = *reinterpret_cast<const half8*>(A + row * 64 + (dl_sw64(row, fk) << 4));
      }
  };
  auto stepA = [&](int s, half8 (&ca)[4], half8 (&cb)[6], half8 (&na)[4], half8 (&nb6)[6])
                   __attribute__((always_inline)) {
    dl_vmwait<4>();  // step s + 1 landed (step s + 2 may be in flight)
    dl_barrier();    // ... for every wave; every wave finished reading step s - 1: its slot (s + 3) & 3 is free
    int sn;
    asm volatile("s_mov_b32 %0, %1" : "=s"(sn) : "s"(s + 3));
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int j = 0; j < 6; ++j) acc[i][j] = O::mfma(cb[j], ca[i], acc[i][j]);
      dmaA(sn, i);
      readA(s + 1, na, nb6, i);
    }
    __builtin_amdgcn_s_setprio(0);
    // per quarter: six MFMAs, one DMA, the next step's fragment reads (3, 3, 2, 2)
    __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
  };
  dl_vmwait<8>();  // step 0 landed
  dl_barrier();
  readA(0, af[0], bf[0], -1);
#pragma unroll 1
  for (int s = 0; s < DH_S1; s += 2) {
    stepA(s, af[0], bf[0], af[1], bf[1]);
    stepA(s + 1, af[1], bf[1], af[0], bf[0]);
  }
  dl_vmwait<0>();  // the dummy DMAs of the last steps land before the image overlays the ring
  // u = relu(acc + b_sp); hi = f16(u) goes to the LDS image, lo = f16(u - hi) stays in registers (packed, half the
  // registers of u), so GEMM A's f32 accumulators die here
  const int nb = wn * 96 + fk * 4;
  uint2 ulo[4][6];
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  dl_barrier();  // every wave finished GEMM A's last step: the ring under the image is free
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const int n = nb + j * 16;
    const float4 bi = *reinterpret_cast<const float4*>(p.bsp + n);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wm * 64 + i * 16 + fr;
      const float u[4] = {fmaxf(acc[i][j][0] + bi.x, 0.f), fmaxf(acc[i][j][1] + bi.y, 0.f),
                          fmaxf(acc[i][j][2] + bi.z, 0.f), fmaxf(acc[i][j][3] + bi.w, 0.f)};
      DlH4 hi, lo;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        hi.h[r] = O::enc(u[r]);
        lo.h[r] = O::enc_lo(u[r] - O::dec(hi.h[r]));
      }
      ulo[i][j] = lo.u;
      *reinterpret_cast<uint2*>(sm + DH_IMG + (n >> 7) * DL_GCHUNK + row * 256 + (dl_swg(row, (n & 127) >> 3) << 4) +
                                ((n >> 2) & 1) * 8) = hi.u;
    }
  }

  // ---- GEMM B: K steps in the order u_hi . W_hi (weight K-steps 0-11), u_hi . W_lo (24-35), u_lo . W_hi (12-23)
  floatx4 acc2[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc2[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int s = 0; s < DH_S1; ++s) {
    if (s == 2 * DL_KS2) {  // the lo image replaces the hi image once every wave has finished reading it
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      dl_barrier();
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        const int n = nb + j * 16;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = wm * 64 + i * 16 + fr;
          *reinterpret_cast<uint2*>(sm + DH_IMG + (n >> 7) * DL_GCHUNK + row * 256 +
                                    (dl_swg(row, (n & 127) >> 3) << 4) + ((n >> 2) & 1) * 8) = ulo[i][j];
        }
      }
    }
    dl_vmwait<2>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's image writes
    dl_barrier();
    int sn;
    asm volatile("s_mov_b32 %0, %1" : "=s"(sn) : "s"(s + 3));
    const int k2 = s % DL_KS2;  // K-step within the 384-channel image
    const unsigned char* Bm = sm + DH_RING_B + (s & 3) * 8192;
    half8 af[4], bf[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wm * 64 + i * 16 + fr;
      af[i] = *reinterpret_cast<const half8*>(sm + DH_IMG + (k2 >> 2) * DL_GCHUNK + row * 256 +
                                              (dl_swg(row, ((k2 & 3) << 2) + fk) << 4));
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = wn * 32 + j * 16 + fr;
      bf[j] = *reinterpret_cast<const half8*>(Bm + row * 64 + (dl_sw64(row, fk) << 4));
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc2[i][j] = O::mfma(bf[j], af[i], acc2[i][j]);
      if (i == 1) issueB(sn);
    }
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
  }
  dl_vmwait<0>();  // the dummy DMAs of the last steps land before the workgroup's LDS is released
  // ---- eps = acc + b_out, columns < n_out
  // both column groups' bias loaded and waited for once, before any store: waited for inside the per-row / per-column
  // branches, the compiler's wait insertion (conservative at their joins) put a vmcnt(0) before every store, each
  // draining the stores before it (assembly, r06)
  float4 bi[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = min(wn * 32 + j * 16 + fk * 4, p.n_out - 4);
    bi[j] = *reinterpret_cast<const float4*>(p.bout + n);
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) asm volatile("" : "+v"(bi[j].x), "+v"(bi[j].y), "+v"(bi[j].z), "+v"(bi[j].w));
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = wn * 32 + j * 16 + fk * 4;
    if (n >= p.n_out) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wm * 64 + i * 16 + fr;
      if (m >= M) continue;
      *reinterpret_cast<float4*>(p.eps + (int64_t)m * p.ld_eps + n) = make_float4(
          acc2[i][j][0] + bi[j].x, acc2[i][j][1] + bi[j].y, acc2[i][j][2] + bi[j].z, acc2[i][j][3] + bi[j].w);
    }
  }
}

int diff_head(const f16* s16, const f16* Wsp, const float* bsp, int Nsp, int Ksp, const f16* Wout, const float* bout,
              int Nout, int Kout, int Npad_out, float* eps, int ld_eps, int M, const f16* zpage, hipStream_t s,
              bool bf16) {
  SVC_REQUIRE(Nsp == DL_C && Ksp == 3 * DL_C && Kout == 3 * DL_C && Nout >= 1 && Nout <= 128 && Nout % 4 == 0 &&
                  Npad_out >= 128 && ld_eps % 4 == 0,
              "diff_head: shape (Nsp %d Ksp %d Nout %d Kout %d)", Nsp, Ksp, Nout, Kout);
  const void* ptrs[] = {s16, Wsp, bsp, Wout, bout, eps};
  for (const void* q : ptrs) SVC_REQUIRE(q && ((uintptr_t)q & 15) == 0, "diff_head: operand not 16-B aligned");
  const int64_t grid = cdiv64(M, DL_BM);
  SVC_REQUIRE(grid > 0 && grid < (1ll << 31), "diff_head: bad grid");
  DiffHeadArgs p{s16, Wsp, bsp, Wout, bout, eps, ld_eps, Nout, M};
  const void* fn = bf16 ? (const void*)diff_head_kernel<true> : (const void*)diff_head_kernel<false>;
  if (int st = ensure_dyn_lds(fn, DH_LDS)) return st;
  const double flops = 2.0 * M * (double)DL_C * 3 * DL_C + 2.0 * M * (double)Nout * 3 * DL_C;
  const int tok = prof_begin("diff_head<128>", flops, 0.0, s);
  void* args[] = {&p, const_cast<const f16**>(&zpage)};
  SVC_HIP_CHECK(hipLaunchKernel(fn, dim3((unsigned)grid), dim3(DL_NT), args, DH_LDS, s));
  prof_end(tok, s);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

}  // namespace svc
