// Four-wave GEMM lab, round 3 (not shipped): the round-2 w4 shape (256x256x64 block tile, 4 waves of
// 128x128, one wave per SIMD, 256 fp32 accumulators per lane pinned to AGPRs) with the staging fixed.
//
// Round 2's w4 (tools/gemm_w4_lab.hip) issued the LDS-DMA of tile t+1 at the start of tile t and waited
// for it half a K-tile later.  Here the DMA of tile t+2 goes into tile t's own stage as soon as every
// wave has read its last fragments of tile t (barrier X, mid-tile), and is waited for a whole K-tile
// later, just before tile t+2's first fragment reads:
//
//   F0 = frags(t, k-step 0) in registers
//   read F1 = frags(t, 1) from stage t&1          | 64 MFMA on F0
//   lgkmcnt(0), s_barrier X                        (stage t&1 read by everyone)
//   DMA tile t+2 -> stage t&1 (16 / wave)
//   vmcnt(16), s_barrier Y                         (tile t+1 landed: issued one K-tile ago)
//   read F0 = frags(t+1, 0) from stage (t+1)&1     | 64 MFMA on F1
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/gemm_w4b_lab.hip -o tools/gemm_w4b_lab.bin
#include <functional>

#include "../k8s_gpu_node_checker_amd/csrc/diag/diag.hip"

namespace {

constexpr int W4_THREADS = 256;

struct W4Dma {
  const __bf16* a;
  const __bf16* b;
  int odd_delta;
  size_t row8;
};

// wave-instruction j in [0, 16): operand j >> 3, rows wid*64 + (j & 7)*8 + 0..7 (lane: row + (lane >> 3),
// physical chunk lane & 7); the source chunk is XOR-swizzled by row (swz_row_xor), rows of one instruction
// share bit 3, so two lane offsets cover every j
__device__ __forceinline__ W4Dma dma_setup(const __bf16* A, const __bf16* Bt, int K, int wid, int lane) {
  const int rsub = lane >> 3, phys = lane & 7;
  const int row = wid * 64 + rsub;
  const int c_even = phys ^ swz_row_xor(row, false), c_odd = phys ^ swz_row_xor(row + 8, false);
  W4Dma d;
  d.a = A + static_cast<size_t>(row) * K + c_even * 8;
  d.b = Bt + static_cast<size_t>(row) * K + c_even * 8;
  d.odd_delta = (c_odd - c_even) * 8;
  d.row8 = static_cast<size_t>(8) * K;
  return d;
}

__device__ __forceinline__ void dma_tile(const W4Dma& d, unsigned char* stage, int kt, int wid) {
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int op = j >> 3, r = j & 7;
    const __bf16* g = (op == 0 ? d.a : d.b) + r * d.row8 + (r & 1 ? d.odd_delta : 0) + kt * BK;
    unsigned char* l = stage + op * (V2_BM * BK * 2) + (wid * 64 + r * 8) * (BK * 2);
    __builtin_amdgcn_global_load_lds(g, (lds_void_t*)l, 16, 0, 0);
  }
}

struct Frag {
  bf16x8 a[8], b[8];
};

__device__ __forceinline__ void read_frags(Frag& f, const unsigned char* stage, int wr, int wc, int frow, int fq,
                                           int ks) {
  const u32x4* a_img = reinterpret_cast<const u32x4*>(stage);
  const u32x4* b_img = reinterpret_cast<const u32x4*>(stage + V2_BM * BK * 2);
#pragma unroll
  for (int m = 0; m < 8; ++m) f.a[m] = __builtin_bit_cast(bf16x8, a_img[swz(wr * 128 + m * 16 + frow, fq + 4 * ks)]);
#pragma unroll
  for (int n = 0; n < 8; ++n) f.b[n] = __builtin_bit_cast(bf16x8, b_img[swz(wc * 128 + n * 16 + frow, fq + 4 * ks)]);
}

template <int PIN>
__device__ __forceinline__ void mfma_block(floatx4 (&acc)[8][8], const Frag& f) {
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 8; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[m], f.b[n], acc[m][n], 0, 0, 0);
  if constexpr (PIN == 1) {
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int n = 0; n < 8; ++n) asm volatile("" : "+a"(acc[m][n]));
  } else if constexpr (PIN == 2) {
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int n = 0; n < 8; ++n) asm volatile("" : "+v"(acc[m][n]));
  }
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ void dma_one(const W4Dma& d, unsigned char* stage, int kt, int wid, int j) {
  const int op = j >> 3, r = j & 7;
  const __bf16* g = (op == 0 ? d.a : d.b) + r * d.row8 + (r & 1 ? d.odd_delta : 0) + kt * BK;
  unsigned char* l = stage + op * (V2_BM * BK * 2) + (wid * 64 + r * 8) * (BK * 2);
  __builtin_amdgcn_global_load_lds(g, (lds_void_t*)l, 16, 0, 0);
}

__device__ __forceinline__ void read_one(Frag& f, const unsigned char* stage, int i, int wr, int wc, int frow, int fq,
                                         int ks) {
  const u32x4* img = reinterpret_cast<const u32x4*>(stage + (i < 8 ? 0 : V2_BM * BK * 2));
  const int row = (i < 8 ? wr : wc) * 128 + (i & 7) * 16 + frow;
  const bf16x8 v = __builtin_bit_cast(bf16x8, img[swz(row, fq + 4 * ks)]);
  if (i < 8) f.a[i] = v;
  else f.b[i - 8] = v;
}

__device__ __forceinline__ void mfma_one(floatx4 (&acc)[8][8], const Frag& f, int i) {
  acc[i >> 3][i & 7] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[i >> 3], f.b[i & 7], acc[i >> 3][i & 7], 0, 0, 0);
}

// Program-order interleave (each group fenced by sched_barrier):
//   block 1: 16 x {ds_read F1[i], FIRST/16 MFMA on F0}; lgkmcnt(0), barrier X;
//            16 x {LDS-DMA j of tile t+2, (64-FIRST)/16 MFMA on F0}; vmcnt, barrier Y
//   block 2: 16 x {ds_read F0(t+1)[i], 4 MFMA on F1}
template <int FIRST>
__global__ void __launch_bounds__(W4_THREADS, 1)
gemm_w4i_kernel(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt, float* __restrict__ C, int M, int N,
                int K) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
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
  const W4Dma dma = dma_setup(Ab, Bb, K, wid, lane);

  dma_tile(dma, smem, 0, wid);
  if (KT > 1) {
    dma_tile(dma, smem + V2_STAGE_BYTES, 1, wid);
    __builtin_amdgcn_s_waitcnt(0x7f70);
  } else {
    __builtin_amdgcn_s_waitcnt(0x3f70);
  }
  STG_BARRIER();
  Frag f0, f1;
  read_frags(f0, smem, wr, wc, frow, fq, 0);
  constexpr int PER1 = FIRST / 16, PER2 = (64 - FIRST) / 16;
  // branch-free body: near the end the DMA re-fetches tile KT-1 into the stage nobody reads any more, and
  // the last iteration's F0 reads load harmless stale fragments (drained before the epilogue)
  for (int kt = 0; kt < KT; ++kt) {
    unsigned char* cur = smem + (kt & 1) * V2_STAGE_BYTES;
    const unsigned char* nxt = smem + ((kt + 1) & 1) * V2_STAGE_BYTES;
    const int kd = min(kt + 2, KT - 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      read_one(f1, cur, i, wr, wc, frow, fq, 1);
#pragma unroll
      for (int u = 0; u < PER1; ++u) mfma_one(acc, f0, i * PER1 + u);
      __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    STG_BARRIER();                        // X
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      dma_one(dma, cur, kd, wid, j);
#pragma unroll
      for (int u = 0; u < PER2; ++u) mfma_one(acc, f0, FIRST + j * PER2 + u);
      __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_s_waitcnt(0x7f70);  // vmcnt(16): tile kt+1 landed
    STG_BARRIER();                        // Y
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      read_one(f0, nxt, i, wr, wc, frow, fq, 0);
#pragma unroll
      for (int u = 0; u < 4; ++u) mfma_one(acc, f1, i * 4 + u);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) lgkmcnt(0): the tail re-fetches landed before LDS is reused
  const int row0 = tm * V2_BM + wr * 128, col0 = tn * V2_BN + wc * 128;
  constexpr int LD = 128 + 4;
  __builtin_amdgcn_s_barrier();
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
}

// PIN: 0 = scheduling fence only, 1 = accumulators pinned to AGPRs, 2 = pinned to VGPRs (the compiler's own choice)
// PRIO: s_setprio(1) around the MFMA blocks
template <int PIN, bool PRIO>
__global__ void __launch_bounds__(W4_THREADS, 1)
gemm_w4b_kernel(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt, float* __restrict__ C, int M, int N,
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
  const W4Dma dma = dma_setup(Ab, Bb, K, wid, lane);

  dma_tile(dma, smem, 0, wid);
  if (KT > 1) {
    dma_tile(dma, smem + V2_STAGE_BYTES, 1, wid);
    __builtin_amdgcn_s_waitcnt(0x7f70);  // vmcnt(16): tile 0 landed, tile 1 may be in flight
  } else {
    __builtin_amdgcn_s_waitcnt(0x3f70);  // vmcnt(0)
  }
  STG_BARRIER();
  Frag f0, f1;
  read_frags(f0, smem, wr, wc, frow, fq, 0);
  for (int kt = 0; kt < KT; ++kt) {
    unsigned char* cur = smem + (kt & 1) * V2_STAGE_BYTES;
    const unsigned char* nxt = smem + ((kt + 1) & 1) * V2_STAGE_BYTES;
    read_frags(f1, cur, wr, wc, frow, fq, 1);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
    mfma_block<PIN>(acc, f0);
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): F1 in registers, this wave's reads of `cur` done
    STG_BARRIER();                        // X: every wave's reads of `cur` done
    const bool pre = kt + 2 < KT;
    if (pre) {
      dma_tile(dma, cur, kt + 2, wid);
      __builtin_amdgcn_s_waitcnt(0x7f70);  // vmcnt(16): tile kt+1 landed (this wave's part)
    } else {
      __builtin_amdgcn_s_waitcnt(0x3f70);  // vmcnt(0)
    }
    STG_BARRIER();  // Y: tile kt+1 landed (every wave's part)
    if (kt + 1 < KT) read_frags(f0, nxt, wr, wc, frow, fq, 0);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
    mfma_block<PIN>(acc, f1);
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
  }
  const int row0 = tm * V2_BM + wr * 128, col0 = tn * V2_BN + wc * 128;
  // LDS-staged epilogue: 16x128 fp32 slices as 16-byte row pieces (every DMA and read retired above)
  constexpr int LD = 128 + 4;
  __builtin_amdgcn_s_barrier();
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
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms / iters;
}

template <int PIN, bool PRIO>
void prep() {
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_w4b_kernel<PIN, PRIO>),
                         hipFuncAttributeMaxDynamicSharedMemorySize, 2 * V2_STAGE_BYTES));
}

template <int FIRST>
void prep_i() {
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_w4i_kernel<FIRST>),
                         hipFuncAttributeMaxDynamicSharedMemorySize, 2 * V2_STAGE_BYTES));
}

template <int FIRST>
void launch_w4i(const __bf16* A, const __bf16* Bt, float* C, int M, int N, int K) {
  hipLaunchKernelGGL((gemm_w4i_kernel<FIRST>), dim3((M / V2_BM) * (N / V2_BN)), dim3(W4_THREADS), 2 * V2_STAGE_BYTES,
                     nullptr, A, Bt, C, M, N, K);
}

template <int PIN, bool PRIO>
void launch_w4b(const __bf16* A, const __bf16* Bt, float* C, int M, int N, int K) {
  hipLaunchKernelGGL((gemm_w4b_kernel<PIN, PRIO>), dim3((M / V2_BM) * (N / V2_BN)), dim3(W4_THREADS),
                     2 * V2_STAGE_BYTES, nullptr, A, Bt, C, M, N, K);
}

}  // namespace

int main(int argc, char** argv) {
  std::vector<int> sizes = {4096, 8192};
  if (argc > 1) sizes = {atoi(argv[1])};
  const int reps = argc > 2 ? atoi(argv[2]) : 3;  // timed rounds per kernel, interleaved (DVFS drift)
  prep<0, false>();
  prep_i<16>();
  prep_i<32>();
  prep_i<48>();
  for (int size : sizes) {
    if (size % 256 || size < 512) {
      printf("size must be a multiple of 256, >= 512\n");
      return 1;
    }
    const int M = size, N = size, K = size;
    __bf16 *A, *Bt;
    float *C0, *C1;
    CK(hipMalloc(&A, sizeof(__bf16) * M * K));
    CK(hipMalloc(&Bt, sizeof(__bf16) * N * K));
    CK(hipMalloc(&C0, sizeof(float) * M * N));
    CK(hipMalloc(&C1, sizeof(float) * M * N));
    hipLaunchKernelGGL(fill_bf16_kernel, dim3(2048), dim3(256), 0, nullptr, A, (size_t)M * K, 7ULL);
    hipLaunchKernelGGL(fill_bf16_kernel, dim3(2048), dim3(256), 0, nullptr, Bt, (size_t)N * K, 11ULL);
    const int nwg1 = (M / BM) * (N / BN);
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
      std::vector<double> all;
    };
    std::vector<Row> rows;
    rows.push_back({"v3(diag,lds-epi)", [&] { launch_v3<DT_BF16>(A, Bt, C1, M, N, K, nullptr); }});
    rows.push_back({"w4b", [&] { launch_w4b<0, false>(A, Bt, C1, M, N, K); }});
    rows.push_back({"w4i16", [&] { launch_w4i<16>(A, Bt, C1, M, N, K); }});
    rows.push_back({"w4i32", [&] { launch_w4i<32>(A, Bt, C1, M, N, K); }});
    rows.push_back({"w4i48", [&] { launch_w4i<48>(A, Bt, C1, M, N, K); }});
    for (int r = 0; r < reps; ++r) {
      for (Row& row : rows) {
        CK(hipMemset(C1, 0xff, sizeof(float) * M * N));
        const double ms = time_ms(row.go, it);
        row.best = std::min(row.best, ms);
        row.all.push_back(ms);
        if (r == 0) {
          CK(hipMemcpy(h1.data(), C1, sizeof(float) * M * N, hipMemcpyDeviceToHost));
          for (size_t i = 0; i < h0.size(); ++i) {
            const double d = std::isnan(h1[i]) ? 1e30
                                               : (double)std::fabs(h0[i] - h1[i]) / std::max(1.0, (double)std::fabs(h0[i]));
            row.worst_diff = std::max(row.worst_diff, d);
          }
        }
      }
    }
    for (Row& row : rows) {
      std::sort(row.all.begin(), row.all.end());
      const double med = row.all[row.all.size() / 2];
      printf("{\"kernel\": \"%s\", \"size\": %d, \"tflops_best\": %.1f, \"tflops_median\": %.1f, \"ms\": %.4f, "
             "\"max_rel_diff_vs_v1\": %.3g}\n",
             row.name, size, 2.0 * M * N * (double)K / (row.best * 1e-3) / 1e12,
             2.0 * M * N * (double)K / (med * 1e-3) / 1e12, row.best, row.worst_diff);
    }
    CK(hipFree(A));
    CK(hipFree(Bt));
    CK(hipFree(C0));
    CK(hipFree(C1));
  }
  return 0;
}
