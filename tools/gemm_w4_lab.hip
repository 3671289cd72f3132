// Four-wave GEMM lab (not shipped): 256x256x64 block tile on 4 waves (2 x 2), 128x128 outputs per
// wave, one wave per SIMD -- the shape hipBLASLt picks for bf16 8192^3 on gfx950
// (MT256x256x64_MI16x16x1, 256 threads, 130 KB LDS: profiles/gemm_torch_hipblaslt_kernels_mi355x.json).
//
// With one wave per SIMD nothing hides a stall but the wave's own instruction stream, so the loop is
// software-pipelined in registers: the fragments of the next K-step are read from LDS while the MFMAs
// of the current one run, and the LDS-DMA of the next K-tile is issued between the MFMAs of the first
// half.  One workgroup barrier per K-tile:
//
//   F0 = frags(tile t, k-step 0) already in registers
//   read F1 = frags(t, 1)            | 64 MFMA on F0, 16 LDS-DMA of tile t+1 -> other stage interleaved
//   vmcnt(0) + lgkmcnt(0), s_barrier: tile t+1 complete, every wave's reads of stage t retired
//   read F0 = frags(t+1, 0)          | 64 MFMA on F1
//
// Per K-tile and wave: 128 MFMA (2048 matrix-pipe cycles), 32 ds_read_b128 (32 KiB), 16 DMA
// (16 KiB): LDS reads are a quarter of the array's 256 B/clk and a third fewer per FLOP than the
// 8-wave 128x64 tile of gemm v3.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/gemm_w4_lab.hip -o tools/gemm_w4_lab.bin
#include <functional>

#include "../k8s_gpu_node_checker_amd/csrc/diag/diag.hip"

namespace {

constexpr int W4_THREADS = 256;

// LDS-DMA addressing, loop invariant: wave-instruction j in [0, 16) fills operand j >> 3, rows
// wid*64 + (j & 7)*8 + 0..7 (lane: row + (lane >> 3), physical chunk lane & 7).  The source chunk is
// XOR-swizzled by row; rows of one instruction share bit 3, so two lane offsets cover all j.
struct W4Dma {
  const __bf16* a;  // this lane's row of A at k = 0, chunk offset for even j folded in
  const __bf16* b;
  int odd_delta;    // extra elements for odd j (the swizzle of row bit 3)
  size_t row8;      // 8 rows of elements
};

__device__ __forceinline__ W4Dma w4_dma_setup(const __bf16* A, const __bf16* Bt, int K, int wid, int lane) {
  const int rsub = lane >> 3, phys = lane & 7;
  const int row = wid * 64 + rsub;  // j = 0; odd j add 8 rows (bit 3 set)
  const int c_even = phys ^ swz_row_xor(row, false), c_odd = phys ^ swz_row_xor(row + 8, false);
  W4Dma d;
  d.a = A + static_cast<size_t>(row) * K + c_even * 8;
  d.b = Bt + static_cast<size_t>(row) * K + c_even * 8;
  d.odd_delta = (c_odd - c_even) * 8;
  d.row8 = static_cast<size_t>(8) * K;
  return d;
}

__device__ __forceinline__ void w4_dma(const W4Dma& d, unsigned char* stage, int kt, int wid, int j) {
  const int op = j >> 3, r = j & 7;
  const __bf16* g = (op == 0 ? d.a : d.b) + r * d.row8 + (r & 1 ? d.odd_delta : 0) + kt * BK;
  unsigned char* l = stage + op * (V2_BM * BK * 2) + (wid * 64 + r * 8) * (BK * 2);
  __builtin_amdgcn_global_load_lds(g, (lds_void_t*)l, 16, 0, 0);
}

struct W4Frag {
  bf16x8 a[8], b[8];
};

__device__ __forceinline__ void w4_read(W4Frag& f, const unsigned char* stage, int wr, int wc, int frow, int fq,
                                        int ks) {
  const u32x4* a_img = reinterpret_cast<const u32x4*>(stage);
  const u32x4* b_img = reinterpret_cast<const u32x4*>(stage + V2_BM * BK * 2);
#pragma unroll
  for (int m = 0; m < 8; ++m) f.a[m] = __builtin_bit_cast(bf16x8, a_img[swz(wr * 128 + m * 16 + frow, fq + 4 * ks)]);
#pragma unroll
  for (int n = 0; n < 8; ++n) f.b[n] = __builtin_bit_cast(bf16x8, b_img[swz(wc * 128 + n * 16 + frow, fq + 4 * ks)]);
}

__device__ __forceinline__ void w4_mfma(floatx4 (&acc)[8][8], const W4Frag& f) {
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 8; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[m], f.b[n], acc[m][n], 0, 0, 0);
}

// Keep the MFMA block ahead of the s_waitcnt that follows it.  PIN 0: a scheduling fence only;
// PIN 1: plus an empty asm reading and writing every accumulator (AGPR), which no pass can reorder.
template <int PIN>
__device__ __forceinline__ void w4_pin(floatx4 (&acc)[8][8]) {
  if constexpr (PIN == 1) {
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int n = 0; n < 8; ++n) asm volatile("" : "+a"(acc[m][n]));
  }
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ void w4_read_one(W4Frag& f, const unsigned char* stage, int i, int wr, int wc, int frow,
                                            int fq, int ks) {
  const u32x4* img = reinterpret_cast<const u32x4*>(stage + (i < 8 ? 0 : V2_BM * BK * 2));
  const int row = (i < 8 ? wr : wc) * 128 + (i & 7) * 16 + frow;
  const bf16x8 v = __builtin_bit_cast(bf16x8, img[swz(row, fq + 4 * ks)]);
  if (i < 8) f.a[i] = v;
  else f.b[i - 8] = v;
}

// Four MFMA of one half (i in [0, 16)): rows block i >> 1, column blocks 4 (i & 1) .. +3.
__device__ __forceinline__ void w4_mfma4(floatx4 (&acc)[8][8], const W4Frag& f, int i) {
  const int m = i >> 1, n0 = (i & 1) * 4;
#pragma unroll
  for (int n = 0; n < 4; ++n)
    acc[m][n0 + n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[m], f.b[n0 + n], acc[m][n0 + n], 0, 0, 0);
}

// One K-tile: see the file comment.  SCHED 2 writes the interleave in program order
// (4 MFMA, then one LDS-DMA / fragment read); 0 and 1 leave it to the compiler (1: sched_group_barrier).
template <int SCHED, int PIN>
__device__ __forceinline__ void w4_step(floatx4 (&acc)[8][8], W4Frag& f0, W4Frag& f1, unsigned char* smem,
                                        const W4Dma& dma, int kt, int KT, int wid, int wr, int wc, int frow,
                                        int fq) {
  const unsigned char* cur = smem + (kt & 1) * V2_STAGE_BYTES;
  unsigned char* nxt = smem + ((kt + 1) & 1) * V2_STAGE_BYTES;
  // the last K-tile re-fetches itself into the idle stage: no branch in the step
  const int kn = kt + 1 < KT ? kt + 1 : kt;
  // F0 was read a whole MFMA block ago: waiting for it here is free, and it keeps the compiler's own
  // wait for F0 from also draining the F1 reads issued next
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
  w4_read(f1, cur, wr, wc, frow, fq, 1);
  if constexpr (SCHED == 3) {
    // the barrier moves to the end of the K-tile: DMA issued at its start has ~0.9 of the tile to
    // land; the last 16 MFMA (rows 6-7 of F1) run after the barrier and cover the F0 reads of t+1
#pragma unroll
    for (int j = 0; j < 16; ++j) w4_dma(dma, nxt, kn, wid, j);
    w4_mfma(acc, f0);
    w4_pin<PIN>(acc);
#pragma unroll
    for (int i = 0; i < 12; ++i) w4_mfma4(acc, f1, i);
    w4_pin<PIN>(acc);
    __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) + lgkmcnt(0)
    STG_BARRIER();
    w4_read(f0, nxt, wr, wc, frow, fq, 0);
#pragma unroll
    for (int i = 12; i < 16; ++i) w4_mfma4(acc, f1, i);
    w4_pin<PIN>(acc);
    return;
  }
  if constexpr (SCHED == 2) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      w4_mfma4(acc, f0, i);
      w4_dma(dma, nxt, kn, wid, i);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 16; ++j) w4_dma(dma, nxt, kn, wid, j);
    w4_mfma(acc, f0);
    if constexpr (SCHED == 1) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // MFMA
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM (LDS-DMA)
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // MFMA
      }
    }
  }
  w4_pin<PIN>(acc);  // the 64 MFMA stay ahead of the waits below
  // vmcnt(0) + lgkmcnt(0): this wave's part of tile t+1 landed and its F1 reads of stage t retired,
  // so after the barrier tile t+1 is complete and stage t is free for the DMA of tile t+2
  __builtin_amdgcn_s_waitcnt(0x0070);
  STG_BARRIER();
  if constexpr (SCHED == 2) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      w4_read_one(f0, nxt, i, wr, wc, frow, fq, 0);  // last K-tile: a harmless read of the re-fetch
      w4_mfma4(acc, f1, i);
    }
  } else {
    w4_read(f0, nxt, wr, wc, frow, fq, 0);
    w4_mfma(acc, f1);
    if constexpr (SCHED == 1) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 1);
      }
    }
  }
  w4_pin<PIN>(acc);
}

// SCHED: 0 = compiler's own order; 1 = sched_group_barrier interleave (MFMA / DS read / VMEM)
template <int SCHED, bool EPI_LDS, int PIN = 0>
__global__ void __launch_bounds__(W4_THREADS, 1)
gemm_w4_kernel(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt, float* __restrict__ C, int M, int N,
               int K) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];  // 2 stages x 64 KiB
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int tiles_m = M / V2_BM, tiles_n = N / V2_BN, nwg = tiles_m * tiles_n;
  int bid = blockIdx.x;
  {
    const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
  }
  constexpr int GROUP_M = 4;
  const int group = bid / (GROUP_M * tiles_n);
  const int first_m = group * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  const int tm = first_m + (bid % (GROUP_M * tiles_n)) % gsize;
  const int tn = (bid % (GROUP_M * tiles_n)) / gsize;
  const __bf16* Ab = A + static_cast<size_t>(tm) * V2_BM * K;
  const __bf16* Bb = Bt + static_cast<size_t>(tn) * V2_BN * K;

  floatx4 acc[8][8];
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 8; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int KT = K / BK;
  const int frow = lane & 15, fq = lane >> 4;

  const W4Dma dma = w4_dma_setup(Ab, Bb, K, wid, lane);
#pragma unroll
  for (int j = 0; j < 16; ++j) w4_dma(dma, smem, 0, wid, j);
  __builtin_amdgcn_s_waitcnt(0x3f70);  // vmcnt(0)
  STG_BARRIER();
  W4Frag f0, f1;
  w4_read(f0, smem, wr, wc, frow, fq, 0);
  for (int kt = 0; kt < KT; ++kt) w4_step<SCHED, PIN>(acc, f0, f1, smem, dma, kt, KT, wid, wr, wc, frow, fq);
  const int row0 = tm * V2_BM + wr * 128, col0 = tn * V2_BN + wc * 128;
  if constexpr (EPI_LDS) {
    constexpr int LD = 128 + 4;
    __syncthreads();
    float* patch = reinterpret_cast<float*>(smem) + wid * (16 * LD);
#pragma unroll
    for (int m = 0; m < 8; ++m) {
#pragma unroll
      for (int n = 0; n < 8; ++n)
#pragma unroll
        for (int j = 0; j < 4; ++j) patch[(fq * 4 + j) * LD + n * 16 + frow] = acc[m][n][j];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int r = q * 2 + (lane >> 5), c4 = (lane & 31) * 4;
        const floatx4 v = *reinterpret_cast<const floatx4*>(patch + r * LD + c4);
        *reinterpret_cast<floatx4*>(C + static_cast<size_t>(row0 + m * 16 + r) * N + col0 + c4) = v;
      }
    }
  } else {
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int n = 0; n < 8; ++n)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          C[static_cast<size_t>(row0 + m * 16 + fq * 4 + j) * N + col0 + n * 16 + frow] = acc[m][n][j];
  }
}

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      printf("%s: %s\n", #x, hipGetErrorString(e_));                           \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

template <class L>
double time_ms(L launch, int iters) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  launch();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < iters; ++i) launch();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / iters;
}

template <int SCHED, bool EPI, int PIN>
void prep() {
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_w4_kernel<SCHED, EPI, PIN>),
                         hipFuncAttributeMaxDynamicSharedMemorySize, 2 * V2_STAGE_BYTES));
}

template <int SCHED, bool EPI, int PIN>
void launch_w4(const __bf16* A, const __bf16* Bt, float* C, int M, int N, int K) {
  hipLaunchKernelGGL((gemm_w4_kernel<SCHED, EPI, PIN>), dim3((M / V2_BM) * (N / V2_BN)), dim3(W4_THREADS),
                     2 * V2_STAGE_BYTES, nullptr, A, Bt, C, M, N, K);
}

}  // namespace

int main(int argc, char** argv) {
  std::vector<int> sizes = {4096, 8192};
  if (argc > 1) sizes = {atoi(argv[1])};
  const int reps = argc > 2 ? atoi(argv[2]) : 3;  // timed rounds per kernel, interleaved (DVFS drift)
  prep<0, false, 0>();
  prep<1, false, 0>();
  prep<0, false, 1>();
  prep<1, false, 1>();
  prep<1, true, 0>();
  prep<2, false, 0>();
  prep<2, false, 1>();
  prep<2, true, 0>();
  prep<3, false, 1>();
  prep<3, true, 1>();
  for (int size : sizes) {
    const int M = size, N = size, K = size;
    __bf16 *A, *Bt;
    float *C0, *C1;
    CK(hipMalloc(&A, sizeof(__bf16) * M * K));
    CK(hipMalloc(&Bt, sizeof(__bf16) * N * K));
    CK(hipMalloc(&C0, sizeof(float) * M * N));
    CK(hipMalloc(&C1, sizeof(float) * M * N));
    hipLaunchKernelGGL(fill_bf16_kernel, dim3(2048), dim3(256), 0, nullptr, A, (size_t)M * K, 7ULL);
    hipLaunchKernelGGL(fill_bf16_kernel, dim3(2048), dim3(256), 0, nullptr, Bt, (size_t)N * K, 11ULL);
    const int nwg1 = (M / BM) * (N / BN), nwg2 = (M / V2_BM) * (N / V2_BN);
    hipLaunchKernelGGL(gemm_bf16_kernel, dim3(nwg1), dim3(THREADS), 0, nullptr, (const u32x4*)A, (const u32x4*)Bt, C0,
                       M, N, K);
    CK(hipDeviceSynchronize());
    std::vector<float> h0((size_t)M * N), h1((size_t)M * N);
    CK(hipMemcpy(h0.data(), C0, sizeof(float) * M * N, hipMemcpyDeviceToHost));
    const int it = size >= 8192 ? 20 : 50;
    struct Row {
      const char* name;
      std::function<void()> go;
      double best = 1e30, worst_diff = 0;
    };
    std::vector<Row> rows;
    rows.push_back({"v3(diag,lds-epi)", [&] { launch_v3<DT_BF16>(A, Bt, C1, M, N, K, nullptr); }});
    rows.push_back({"w4", [&] { launch_w4<0, false, 0>(A, Bt, C1, M, N, K); }});
    rows.push_back({"w4+sched", [&] { launch_w4<1, false, 0>(A, Bt, C1, M, N, K); }});
    rows.push_back({"w4+asmpin", [&] { launch_w4<0, false, 1>(A, Bt, C1, M, N, K); }});
    rows.push_back({"w4+sched+asmpin", [&] { launch_w4<1, false, 1>(A, Bt, C1, M, N, K); }});
    rows.push_back({"w4+sched+lds-epi", [&] { launch_w4<1, true, 0>(A, Bt, C1, M, N, K); }});
    rows.push_back({"w4+manual", [&] { launch_w4<2, false, 0>(A, Bt, C1, M, N, K); }});
    rows.push_back({"w4+manual+asmpin", [&] { launch_w4<2, false, 1>(A, Bt, C1, M, N, K); }});
    rows.push_back({"w4+manual+lds-epi", [&] { launch_w4<2, true, 0>(A, Bt, C1, M, N, K); }});
    rows.push_back({"w4+late-barrier+asmpin", [&] { launch_w4<3, false, 1>(A, Bt, C1, M, N, K); }});
    rows.push_back({"w4+late-barrier+asmpin+lds-epi", [&] { launch_w4<3, true, 1>(A, Bt, C1, M, N, K); }});
    for (int r = 0; r < reps; ++r) {
      for (Row& row : rows) {
        CK(hipMemset(C1, 0xff, sizeof(float) * M * N));
        const double ms = time_ms(row.go, it);
        row.best = std::min(row.best, ms);
        if (r == 0) {
          CK(hipMemcpy(h1.data(), C1, sizeof(float) * M * N, hipMemcpyDeviceToHost));
          for (size_t i = 0; i < h0.size(); ++i)
            row.worst_diff = std::max(row.worst_diff, (double)std::fabs(h0[i] - h1[i]) /
                                                          std::max(1.0, (double)std::fabs(h0[i])));
        }
      }
    }
    for (const Row& row : rows)
      printf("{\"kernel\": \"%s\", \"size\": %d, \"tflops\": %.1f, \"ms\": %.4f, \"max_rel_diff_vs_v1\": %.3g}\n", row.name,
             size, 2.0 * M * N * (double)K / (row.best * 1e-3) / 1e12, row.best, row.worst_diff);
    CK(hipFree(A));
    CK(hipFree(Bt));
    CK(hipFree(C0));
    CK(hipFree(C1));
  }
  return 0;
}
