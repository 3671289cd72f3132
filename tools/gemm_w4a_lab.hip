// Four-wave bf16 GEMM lab: sweeps the schedule knobs of diag.hip's v4 kernel (gemm_v4_kernel: hipBLASLt's gfx950
// structure, 4 waves of 128x128 on a 256x256x64 tile, with the loop's MFMA / ds_read / LDS-DMA order written out
// in asm) against the 8-wave v3 kernel, in one process, interleaved rounds, every output compared with the v1
// kernel's.
//
// hipBLASLt's bf16 8192^3 kernel (Custom_Cijk_Alik_Bljk_BBS_BH_MT256x256x64_MI16x16x1, read with llvm-objdump
// from TensileLibrary_BB_BB_..._gfx950.co): 256 threads, a 256x256x64 tile, 2 LDS stages; one K-tile per loop
// iteration = 128 v_mfma_f32_16x16x32_bf16, 32 ds_read_b128 and 16 buffer_load_dwordx4 ... lds per wave,
// interleaved one instruction between MFMAs, 3 s_barriers.  Round 2/3's compiler-ordered four-wave kernels lost
// to v3 on AGPR<->VGPR shuffling; writing the loop as asm statements fixed that.  Knobs: see gemm_v4_kernel.
// The sweep that picked the shipped schedule (RS 1, X_AT 20, D1 8, Y_AT 8, GM 4):
// profiles/gemm_w4a_lab_mi355x.jsonl.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/gemm_w4a_lab.hip -o tools/gemm_w4a_lab.bin
#include <functional>

#include "../k8s_gpu_node_checker_amd/csrc/diag/diag.hip"

namespace {

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

template <class PLAN, int GM = 4, bool TR = false, bool M0G = false>
void launch_plan(const __bf16* A, const __bf16* Bt, float* C, int M, int N, int K) {
  static bool once = [] {
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_v4_kernel<OUT_F32, PLAN, GM, TR, DT_BF16, M0G>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, 2 * V2_STAGE_BYTES));
    return true;
  }();
  (void)once;
  hipLaunchKernelGGL((gemm_v4_kernel<OUT_F32, PLAN, GM, TR, DT_BF16, M0G>), dim3((M / V2_BM) * (N / V2_BN)),
                     dim3(V4_THREADS), 2 * V2_STAGE_BYTES, nullptr, A, Bt, C, nullptr, M, N, K);
}

// fp8 (K in bytes; the kernels take bf16 columns = bytes / 2)
template <class PLAN>
void launch_plan8(const void* A, const void* Bt, float* C, int M, int N, int K) {
  static bool once = [] {
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_v4_kernel<OUT_F32, PLAN, 4, false, DT_FP8U>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, 2 * V2_STAGE_BYTES));
    return true;
  }();
  (void)once;
  hipLaunchKernelGGL((gemm_v4_kernel<OUT_F32, PLAN, 4, false, DT_FP8U>), dim3((M / V2_BM) * (N / V2_BN)),
                     dim3(V4_THREADS), 2 * V2_STAGE_BYTES, nullptr, static_cast<const __bf16*>(A),
                     static_cast<const __bf16*>(Bt), C, nullptr, M, N, K / 2);
}

template <int RS, int X_AT, int D1, int Y_AT, int GM, int R2 = 2, bool TR = false>
void launch_w4a(const __bf16* A, const __bf16* Bt, float* C, int M, int N, int K) {
  launch_plan<V4PlanA<RS, X_AT, D1, Y_AT, R2>, GM, TR>(A, Bt, C, M, N, K);
}

}  // namespace

#ifdef DIAG_V4_STAMPS
// stamps mode (build with -DDIAG_V4_STAMPS -o tools/gemm_w4a_lab_stamps.bin): run the production v4 schedule at
// M = N = size, K = k a few times and print, per stamp, the median / p10 / p90 over all waves of the last launch
template <bool TR>
int run_stamps(int size, int K) {
  const int M = size, N = size;
  __bf16 *A, *Bt;
  float* C;
  CK(hipMalloc(&A, sizeof(__bf16) * M * K));
  CK(hipMalloc(&Bt, sizeof(__bf16) * N * K));
  CK(hipMalloc(&C, sizeof(float) * M * N));
  hipLaunchKernelGGL(fill_bf16_kernel, dim3(2048), dim3(256), 0, nullptr, A, (size_t)M * K, 7ULL);
  hipLaunchKernelGGL(fill_bf16_kernel, dim3(2048), dim3(256), 0, nullptr, Bt, (size_t)N * K, 11ULL);
  const double ms = time_ms([&] { launch_w4a<1, 20, 8, 8, 4, 2, TR>(A, Bt, C, M, N, K); }, 10);
  CK(hipDeviceSynchronize());
  const int nwg = (M / V2_BM) * (N / V2_BN);
  std::vector<unsigned long long> h(static_cast<size_t>(4096) * 4 * 8);
  CK(hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(g_v4_stamps), h.size() * sizeof(unsigned long long)));
  const char* names[7] = {"prologue", "k_loop", "epilogue", "mid_iter", "x_wait", "y_wait", "end_wait"};
  printf("{\"mode\": \"stamps\", \"tr\": %d, \"M\": %d, \"N\": %d, \"K\": %d, \"ms\": %.4f, \"tflops\": %.1f",
         TR ? 1 : 0, M, N, K, ms, 2.0 * M * N * (double)K / (ms * 1e-3) / 1e12);
  for (int q = 0; q < 7; ++q) {
    std::vector<double> v;
    for (int b = 0; b < std::min(nwg, 4096); ++b)
      for (int w = 0; w < 4; ++w) v.push_back(static_cast<double>(h[(static_cast<size_t>(b) * 4 + w) * 8 + q]));
    std::sort(v.begin(), v.end());
    printf(", \"%s\": [%.0f, %.0f, %.0f]", names[q], v[v.size() / 10], v[v.size() / 2], v[v.size() * 9 / 10]);
  }
  printf("}\n");
  fflush(stdout);
  CK(hipFree(A));
  CK(hipFree(Bt));
  CK(hipFree(C));
  return 0;
}
#endif

int main(int argc, char** argv) {
#ifdef DIAG_V4_STAMPS
  // stamps SIZE K: the production v4 schedule and its transposed-epilogue form
  const int ssize = argc > 1 ? atoi(argv[1]) : 8192, sk = argc > 2 ? atoi(argv[2]) : 8192;
  run_stamps<false>(ssize, sk);
  run_stamps<true>(ssize, sk);
  return 0;
#endif
  const bool fp8 = argc > 3 && strcmp(argv[3], "fp8") == 0;  // SIZES REPS fp8: the fp8 plan sweep against v3's fp8
  std::vector<int> sizes = {4096, 8192};
  if (argc > 1) {
    sizes.clear();
    for (char* p = strtok(argv[1], ","); p; p = strtok(nullptr, ",")) sizes.push_back(atoi(p));
  }
  const int reps = argc > 2 ? atoi(argv[2]) : 3;  // timed rounds per kernel, interleaved (DVFS drift)
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
    if (fp8) {
      hipLaunchKernelGGL(fill_fp8_kernel, dim3(2048), dim3(256), 0, nullptr, (uint8_t*)A, (size_t)M * K, 7ULL);
      hipLaunchKernelGGL(fill_fp8_kernel, dim3(2048), dim3(256), 0, nullptr, (uint8_t*)Bt, (size_t)N * K, 11ULL);
      CK(launch_v3<DT_FP8U>(A, Bt, C0, M, N, K / 2, nullptr) == 0 ? hipSuccess : hipErrorUnknown);
    } else {
      hipLaunchKernelGGL(fill_bf16_kernel, dim3(2048), dim3(256), 0, nullptr, A, (size_t)M * K, 7ULL);
      hipLaunchKernelGGL(fill_bf16_kernel, dim3(2048), dim3(256), 0, nullptr, Bt, (size_t)N * K, 11ULL);
      const int nwg1 = (M / BM) * (N / BN);
      hipLaunchKernelGGL(gemm_bf16_kernel, dim3(nwg1), dim3(THREADS), 0, nullptr, (const u32x4*)A, (const u32x4*)Bt,
                         C0, M, N, K);
    }
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
    if (fp8) {
      rows.push_back({"fp8 warmup (v3)", [&] { (void)launch_v3<DT_FP8U>(A, Bt, C1, M, N, K / 2, nullptr); }});
      rows.push_back({"fp8 v3", [&] { (void)launch_v3<DT_FP8U>(A, Bt, C1, M, N, K / 2, nullptr); }});
      rows.push_back({"fp8 x8 da12 x30 db31 y46", [&] { launch_plan8<V4PlanF8<8, 12, 30, 31, 46>>(A, Bt, C1, M, N, K); }});
      rows.push_back({"fp8 x8 da10 x26 db27 y42", [&] { launch_plan8<V4PlanF8<8, 10, 26, 27, 42>>(A, Bt, C1, M, N, K); }});
      rows.push_back({"fp8 x10 da12 x30 db31 y46", [&] { launch_plan8<V4PlanF8<10, 12, 30, 31, 46>>(A, Bt, C1, M, N, K); }});
      rows.push_back({"fp8 x10 da12 x28 db29 y44", [&] { launch_plan8<V4PlanF8<10, 12, 28, 29, 44>>(A, Bt, C1, M, N, K); }});
      rows.push_back({"fp8 x8 da12 x30 db31 y46 #2", [&] { launch_plan8<V4PlanF8<8, 12, 30, 31, 46>>(A, Bt, C1, M, N, K); }});
    } else {
    rows.push_back({"v3(diag,lds-epi)", [&] { launch_v3<DT_BF16>(A, Bt, C1, M, N, K, nullptr); }});
    rows.push_back({"w4a rs1 x20 d8 y8", [&] { launch_w4a<1, 20, 8, 8, 4>(A, Bt, C1, M, N, K); }});
    rows.push_back({"w4a rs1 x20 d8 y8 m0-grouped", [&] {
                      launch_plan<V4PlanA<1, 20, 8, 8, 2>, 4, false, true>(A, Bt, C1, M, N, K); }});
    rows.push_back({"w4a rs1 x20 d8 y8 #2", [&] { launch_w4a<1, 20, 8, 8, 4>(A, Bt, C1, M, N, K); }});
    rows.push_back({"w4a rs1 x20 d8 y8 m0-grouped #2", [&] {
                      launch_plan<V4PlanA<1, 20, 8, 8, 2>, 4, false, true>(A, Bt, C1, M, N, K); }});
    rows.push_back({"w4a rs1 x20 d8 y8 TR", [&] { launch_w4a<1, 20, 8, 8, 4, 2, true>(A, Bt, C1, M, N, K); }});
    rows.push_back({"w4a rs1 x24 d8 y8", [&] { launch_w4a<1, 24, 8, 8, 4>(A, Bt, C1, M, N, K); }});
    rows.push_back({"w4a rs1 x20 d8 y4", [&] { launch_w4a<1, 20, 8, 4, 4>(A, Bt, C1, M, N, K); }});
    rows.push_back({"A2 x20 d8 y8 h40", [&] { launch_plan<V4PlanA2<1, 20, 8, 8, 2, 40>>(A, Bt, C1, M, N, K); }});
    rows.push_back({"A2 x20 d8 y8 h33", [&] { launch_plan<V4PlanA2<1, 20, 8, 8, 2, 33>>(A, Bt, C1, M, N, K); }});
    rows.push_back({"A2 x20 d10 y8 h40", [&] { launch_plan<V4PlanA2<1, 20, 10, 8, 2, 40>>(A, Bt, C1, M, N, K); }});
    rows.push_back({"A2 x20 d12 y4 h38", [&] { launch_plan<V4PlanA2<1, 20, 12, 4, 2, 38>>(A, Bt, C1, M, N, K); }});
    rows.push_back({"A2 x20 d8 y4 r1 h24", [&] { launch_plan<V4PlanA2<1, 20, 8, 4, 1, 24>>(A, Bt, C1, M, N, K); }});
    rows.push_back({"S xa16 xb34 b3 y8", [&] { launch_plan<V4PlanS<16, 34, 3, 8>>(A, Bt, C1, M, N, K); }});
    rows.push_back({"S xa16 xb36 b5 y12", [&] { launch_plan<V4PlanS<16, 36, 5, 12>>(A, Bt, C1, M, N, K); }});
    }
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
      fflush(stdout);
    }
    CK(hipFree(A));
    CK(hipFree(Bt));
    CK(hipFree(C0));
    CK(hipFree(C1));
  }
  return 0;
}
