// MFMA datapath lab (not shipped): operand lane layouts and per-dtype peak rates on gfx950.
//
//   layout: one wave runs one MFMA on host-packed fragments of exact-valued logical A[16][K] and
//           B[K][16]; the result (C/D map col = lane&15, row = 4*(lane>>4) + r) is compared with the
//           host product for each candidate k-mapping, so the lane layout of every dtype is measured,
//           not assumed.
//   peak:   register-resident MFMA loops (4 independent accumulators per wave, 2 waves per SIMD,
//           every CU), TFLOP/s per dtype.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mfma_lab.hip -o tools/mfma_lab.bin
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                    \
  do {                                                           \
    hipError_t e_ = (x);                                         \
    if (e_ != hipSuccess) {                                      \
      printf("%s: %s\n", #x, hipGetErrorString(e_));             \
      exit(1);                                                   \
    }                                                            \
  } while (0)

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef int i32x8 __attribute__((ext_vector_type(8)));

enum Kind { BF16 = 0, FP8 = 1, MXFP8 = 2, MXFP4 = 3 };
static const char* kName[] = {"bf16_16x16x32", "fp8_16x16x32", "mxfp8_16x16x128", "mxfp4_16x16x128"};
static const int kK[] = {32, 32, 128, 128};

// ---------------------------------------------------------------- device --
template <int KIND>
__device__ __forceinline__ floatx4 mfma(const i32x8& a, const i32x8& b, floatx4 c) {
  if constexpr (KIND == BF16) {
    bf16x8 av, bv;
    memcpy(&av, &a, 16);
    memcpy(&bv, &b, 16);
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, c, 0, 0, 0);
  } else if constexpr (KIND == FP8) {
    long av, bv;
    memcpy(&av, &a, 8);
    memcpy(&bv, &b, 8);
    return __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(av, bv, c, 0, 0, 0);
  } else if constexpr (KIND == MXFP8) {
    return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);  // E4M3, scale 2^0
  } else {
    return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 4, 4, 0, 127, 0, 127);  // E2M1, scale 2^0
  }
}

// one wave: fragments in (32 bytes per lane each), C out (4 floats per lane)
template <int KIND>
__global__ void layout_kernel(const i32x8* fa, const i32x8* fb, floatx4* c) {
  const int l = threadIdx.x;
  c[l] = mfma<KIND>(fa[l], fb[l], floatx4{0.f, 0.f, 0.f, 0.f});
}

template <int KIND>
__global__ void __launch_bounds__(256) peak_kernel(const i32x8* seedf, float* out, int iters) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  i32x8 a = seedf[t & 1023], b = seedf[(t * 7 + 3) & 1023];
  floatx4 acc0 = {0, 0, 0, 0}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      acc0 = mfma<KIND>(a, b, acc0);
      acc1 = mfma<KIND>(b, a, acc1);
      acc2 = mfma<KIND>(a, a, acc2);
      acc3 = mfma<KIND>(b, b, acc3);
    }
  }
  const floatx4 s = acc0 + acc1 + acc2 + acc3;
  out[t] = s[0] + s[1] + s[2] + s[3];
}

// ------------------------------------------------------------------ host --
static uint32_t rng_state = 12345;
static uint32_t rnd() {
  rng_state ^= rng_state << 13;
  rng_state ^= rng_state >> 17;
  rng_state ^= rng_state << 5;
  return rng_state;
}

// exact small values per format and their encodings
static uint16_t bf16_bits(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return static_cast<uint16_t>(u >> 16);
}
static const float kFp8Vals[] = {0.f, 0.5f, 1.f, 1.5f, 2.f, 3.f, -1.f, -2.f};
static uint8_t fp8_e4m3(float f) {  // OCP E4M3 for the values above
  if (f == 0.f) return 0;
  uint8_t s = f < 0 ? 0x80 : 0;
  f = std::fabs(f);
  int e = static_cast<int>(std::floor(std::log2(f)));
  float m = f / std::ldexp(1.f, e) - 1.f;  // [0,1)
  return s | static_cast<uint8_t>(((e + 7) & 0xF) << 3) | static_cast<uint8_t>(std::lround(m * 8) & 7);
}
static const float kFp4Vals[] = {0.f, 0.5f, 1.f, 1.5f, 2.f, 3.f, 4.f, 6.f};
static uint8_t fp4_e2m1(float f) {
  for (int i = 0; i < 8; ++i)
    if (kFp4Vals[i] == std::fabs(f)) return static_cast<uint8_t>(i | (f < 0 ? 8 : 0));
  return 0;
}

// candidate k-mappings: lane l, element e -> k
static int kmap(int cand, int l, int e, int K) {
  const int per = K / 4;  // elements per lane
  switch (cand) {
    case 0: return per * (l >> 4) + e;                           // contiguous block per lane group
    case 1: return 4 * e + (l >> 4);                             // interleaved
    case 2: return (e / 8) * 32 + 8 * (l >> 4) + (e % 8);        // 8-element groups, lane-group inner
    case 3: return (e / 16) * 64 + 16 * (l >> 4) + (e % 16);     // 16-element groups
    default: return (e / 4) * 16 + 4 * (l >> 4) + (e % 4);      // 4-element groups
  }
}

template <int KIND>
static void layout_test() {
  const int K = kK[KIND], per = K / 4;
  std::vector<float> A(16 * K), B(K * 16);
  for (auto& v : A) v = (KIND == MXFP4) ? kFp4Vals[rnd() % 8] * ((rnd() & 1) ? 1.f : -1.f) : kFp8Vals[rnd() % 8];
  for (auto& v : B) v = (KIND == MXFP4) ? kFp4Vals[rnd() % 8] * ((rnd() & 1) ? 1.f : -1.f) : kFp8Vals[rnd() % 8];
  std::vector<float> ref(256, 0.f);
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j)
      for (int k = 0; k < K; ++k) ref[i * 16 + j] += A[i * K + k] * B[k * 16 + j];
  i32x8 *dA, *dB;
  floatx4* dC;
  CK(hipMalloc(&dA, 64 * sizeof(i32x8)));
  CK(hipMalloc(&dB, 64 * sizeof(i32x8)));
  CK(hipMalloc(&dC, 64 * sizeof(floatx4)));
  int found = -1;
  for (int cand = 0; cand < 5 && found < 0; ++cand) {
    for (int nib = 0; nib < (KIND == MXFP4 ? 2 : 1) && found < 0; ++nib) {
      std::vector<uint8_t> fa(64 * 32, 0), fb(64 * 32, 0);
      for (int l = 0; l < 64; ++l)
        for (int e = 0; e < per; ++e) {
          const int k = kmap(cand, l, e, K);
          const float av = A[(l & 15) * K + k], bv = B[k * 16 + (l & 15)];
          if (KIND == BF16) {
            uint16_t x = bf16_bits(av), y = bf16_bits(bv);
            memcpy(&fa[l * 32 + 2 * e], &x, 2);
            memcpy(&fb[l * 32 + 2 * e], &y, 2);
          } else if (KIND == MXFP4) {
            const int byte = e / 2, hi = (e & 1) ^ nib;
            fa[l * 32 + byte] |= static_cast<uint8_t>(fp4_e2m1(av) << (hi ? 4 : 0));
            fb[l * 32 + byte] |= static_cast<uint8_t>(fp4_e2m1(bv) << (hi ? 4 : 0));
          } else {
            fa[l * 32 + e] = fp8_e4m3(av);
            fb[l * 32 + e] = fp8_e4m3(bv);
          }
        }
      CK(hipMemcpy(dA, fa.data(), fa.size(), hipMemcpyHostToDevice));
      CK(hipMemcpy(dB, fb.data(), fb.size(), hipMemcpyHostToDevice));
      hipLaunchKernelGGL(layout_kernel<KIND>, dim3(1), dim3(64), 0, nullptr, dA, dB, dC);
      CK(hipDeviceSynchronize());
      std::vector<float> c(256);
      CK(hipMemcpy(c.data(), dC, 256 * sizeof(float), hipMemcpyDeviceToHost));
      double worst = 0;
      for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 4; ++r) {
          const int row = 4 * (l >> 4) + r, col = l & 15;
          worst = std::max(worst, static_cast<double>(std::fabs(c[l * 4 + r] - ref[row * 16 + col])));
        }
      if (worst == 0) found = cand * 2 + nib;
    }
  }
  printf("{\"layout\": \"%s\", \"k_mapping\": %d, \"fp4_high_nibble_first\": %d, \"exact\": %s}\n", kName[KIND],
         found < 0 ? -1 : found / 2, found < 0 ? -1 : found % 2, found >= 0 ? "true" : "false");
  CK(hipFree(dA));
  CK(hipFree(dB));
  CK(hipFree(dC));
}

template <int KIND>
static void peak_test(const i32x8* seed, float* out, int blocks) {
  const int iters = 2000;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL(peak_kernel<KIND>, dim3(blocks), dim3(256), 0, nullptr, seed, out, iters);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  const int reps = 5;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(peak_kernel<KIND>, dim3(blocks), dim3(256), 0, nullptr, seed, out, iters);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  const double waves = blocks * 4.0;
  const double flops = waves * iters * 16.0 * 2.0 * 16 * 16 * kK[KIND] * reps;
  printf("{\"peak\": \"%s\", \"tflops\": %.1f, \"ms\": %.3f}\n", kName[KIND], flops / (ms * 1e-3) / 1e12, ms / reps);
}

int main() {
  layout_test<BF16>();
  layout_test<FP8>();
  layout_test<MXFP8>();
  layout_test<MXFP4>();
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int blocks = cus * 2;  // 8 waves per CU = 2 per SIMD
  std::vector<uint8_t> host(1024 * 32);
  for (auto& v : host) v = static_cast<uint8_t>(rnd() & 0x3F);  // finite, modest values in every format
  i32x8* seed;
  float* out;
  CK(hipMalloc(&seed, host.size()));
  CK(hipMalloc(&out, blocks * 256 * sizeof(float)));
  CK(hipMemcpy(seed, host.data(), host.size(), hipMemcpyHostToDevice));
  peak_test<BF16>(seed, out, blocks);
  peak_test<FP8>(seed, out, blocks);
  peak_test<MXFP8>(seed, out, blocks);
  peak_test<MXFP4>(seed, out, blocks);
  CK(hipFree(seed));
  CK(hipFree(out));
  return 0;
}
