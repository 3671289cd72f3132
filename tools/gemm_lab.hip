// GEMM schedule lab (not shipped): variants of the diag MFMA GEMM, timed and checked against the
// v1 kernel on full outputs.  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/gemm_lab.hip
#include "../k8s_gpu_node_checker_amd/csrc/diag/diag.hip"

namespace {

// Ping-pong ("vP"): 8 waves in two groups of 4 (one wave of each group per SIMD); group 1 runs one
// barrier behind group 0, so on every SIMD one wave's MFMA segment overlaps the other's load segment.
// Per K-tile and wave:  L: read the B fragments -> s_barrier -> M: (group 0 only) issue the whole next
// tile by LDS-DMA, 64 MFMA with the A fragments read just ahead (2 per MFMA gap, ~free) -> s_barrier.
// Slots (interval between two workgroup barriers): group 0 does L_k in slot 2k and M_k in 2k+1, group 1
// L_k in 2k+1 and M_k in 2k+2.  Tile k+1 is issued at the start of slot 2k+1 into the buffer of tile k-1
// (last read by group 1 in M_{k-1}, slot 2k, lgkmcnt(0) before that slot's closing barrier) and retired
// (vmcnt(0)) by group 0 before the barrier closing slot 2k+1; its first reader is group 0's L_{k+1},
// slot 2k+2.  (Issuing it in L_k, slot 2k, races group 1's M_{k-1}; three stages do not fit in LDS.)
__device__ __forceinline__ void vp_fill(unsigned char* lds_stage, const __bf16* __restrict__ A,
                                        const __bf16* __restrict__ Bt, int K, int kt, int gw, int lane) {
  const int rsub = lane >> 3, phys = lane & 7;
#pragma unroll
  for (int op = 0; op < 2; ++op) {
    const __bf16* src = op == 0 ? A : Bt;
#pragma unroll
    for (int j = 0; j < 8; ++j) {  // 64 rows of each operand per group-0 wave
      const int row = gw * 64 + j * 8 + rsub;
      const int c = phys ^ ((row >> 1) & 7);
      const __bf16* g = src + static_cast<size_t>(row) * K + kt * BK + c * 8;
      unsigned char* l = lds_stage + op * (V2_BM * BK * 2) + (gw * 64 + j * 8) * (BK * 2);
      __builtin_amdgcn_global_load_lds(g, (lds_void_t*)l, 16, 0, 0);
    }
  }
}

template <bool PRIO>
__global__ void __launch_bounds__(V2_THREADS, 1)
gemm_vp_kernel(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt, float* __restrict__ C, int M, int N, int K) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int grp = wid >> 2, gw = wid & 3;
  const int wr = grp, wc = gw;  // output: rows wr*128..+128, cols wc*64..+64
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

  floatx4 acc[8][4];
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int KT = K / BK;
  const int frow = lane & 15, fq = lane >> 4;

  if (grp == 0) vp_fill(smem, Ab, Bb, K, 0, gw, lane);
  __builtin_amdgcn_s_waitcnt(0x3f70);  // vmcnt(0)
  __builtin_amdgcn_s_barrier();
  if (grp == 1) __builtin_amdgcn_s_barrier();  // the stagger
  for (int kt = 0; kt < KT; ++kt) {
    const unsigned char* cur = smem + (kt & 1) * V2_STAGE_BYTES;
    const u32x4* a_img = reinterpret_cast<const u32x4*>(cur);
    const u32x4* b_img = reinterpret_cast<const u32x4*>(cur + V2_BM * BK * 2);
    // ---- L segment
    bf16x8 bfr[2][4];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int n = 0; n < 4; ++n) bfr[s2][n] = __builtin_bit_cast(bf16x8, b_img[swz(wc * 64 + n * 16 + frow, fq + 4 * s2)]);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    // ---- M segment
    if (PRIO) __builtin_amdgcn_s_setprio(1);
    if (grp == 0 && kt + 1 < KT) vp_fill(smem + ((kt + 1) & 1) * V2_STAGE_BYTES, Ab, Bb, K, kt + 1, gw, lane);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const bf16x8 af = __builtin_bit_cast(bf16x8, a_img[swz(wr * 128 + m * 16 + frow, fq + 4 * s2)]);
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[s2][n], acc[m][n], 0, 0, 0);
      }
    if (PRIO) __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // A-fragment reads retired before the slot closes
    if (grp == 0) __builtin_amdgcn_s_waitcnt(0x3f70);  // tile k+1 landed before slot 2k+2
    __builtin_amdgcn_s_barrier();
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();  // balance the stagger
  const int row0 = tm * V2_BM + wr * 128, col0 = tn * V2_BN + wc * 64;
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        C[static_cast<size_t>(row0 + m * 16 + fq * 4 + j) * N + col0 + n * 16 + frow] = acc[m][n][j];
}

}  // namespace

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      printf("%s: %s\n", #x, hipGetErrorString(e_));                           \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

template <class L>
static double time_ms(L launch, int iters) {
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

int main(int argc, char** argv) {
  for (int size : {4096, 8192}) {
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
    hipLaunchKernelGGL(gemm_bf16_kernel, dim3(nwg1), dim3(THREADS), 0, nullptr, (const u32x4*)A, (const u32x4*)Bt, C0, M,
                       N, K);
    CK(hipDeviceSynchronize());
    std::vector<float> h0((size_t)M * N), h1((size_t)M * N);
    CK(hipMemcpy(h0.data(), C0, sizeof(float) * M * N, hipMemcpyDeviceToHost));
    CK(hipFuncSetAttribute((const void*)gemm_bf16_v2_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * V2_STAGE_BYTES));
    CK(hipFuncSetAttribute((const void*)gemm_vp_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * V2_STAGE_BYTES));
    CK(hipFuncSetAttribute((const void*)gemm_vp_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * V2_STAGE_BYTES));
    auto check = [&](const char* name, double ms) {
      CK(hipMemcpy(h1.data(), C1, sizeof(float) * M * N, hipMemcpyDeviceToHost));
      double worst = 0;
      for (size_t i = 0; i < h0.size(); ++i) worst = std::max(worst, (double)std::fabs(h0[i] - h1[i]) / std::max(1.0, (double)std::fabs(h0[i])));
      printf("{\"kernel\": \"%s\", \"size\": %d, \"tflops\": %.1f, \"ms\": %.4f, \"max_rel_diff_vs_v1\": %.3g}\n", name, size,
             2.0 * M * N * (double)K / (ms * 1e-3) / 1e12, ms, worst);
      CK(hipMemset(C1, 0xff, sizeof(float) * M * N));
    };
    const int it = size == 8192 ? 20 : 50;
    double ms;
    ms = time_ms([&] { hipLaunchKernelGGL(gemm_bf16_kernel, dim3(nwg1), dim3(THREADS), 0, nullptr, (const u32x4*)A, (const u32x4*)Bt, C1, M, N, K); }, it);
    check("v1", ms);
    ms = time_ms([&] { hipLaunchKernelGGL(gemm_bf16_v2_kernel, dim3(nwg2), dim3(V2_THREADS), 2 * V2_STAGE_BYTES, nullptr, A, Bt, C1, M, N, K); }, it);
    check("v2", ms);
    ms = time_ms([&] { hipLaunchKernelGGL(gemm_vp_kernel<false>, dim3(nwg2), dim3(V2_THREADS), 2 * V2_STAGE_BYTES, nullptr, A, Bt, C1, M, N, K); }, it);
    check("vP", ms);
    ms = time_ms([&] { hipLaunchKernelGGL(gemm_vp_kernel<true>, dim3(nwg2), dim3(V2_THREADS), 2 * V2_STAGE_BYTES, nullptr, A, Bt, C1, M, N, K); }, it);
    check("vP+prio", ms);
    hipFree(A);
    hipFree(Bt);
    hipFree(C0);
    hipFree(C1);
  }
  return 0;
}
