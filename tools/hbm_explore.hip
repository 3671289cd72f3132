// One-off HBM stream exploration on MI355X: which copy/read/write form is fastest.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef float f4v __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <int U, bool NT>
__global__ void __launch_bounds__(256) copy_k(const f4v* __restrict__ s, f4v* __restrict__ d, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    f4v v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(s + i + u * stride) : s[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT) __builtin_nontemporal_store(v[u], d + i + u * stride);
      else d[i + u * stride] = v[u];
    }
  }
  for (; i < n; i += stride) d[i] = s[i];
}

template <int U, bool NT>
__global__ void __launch_bounds__(256) read_k(const f4v* __restrict__ s, size_t n, float* sink) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  float acc = 0.f;
  for (; i + (U - 1) * stride < n; i += U * stride) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      f4v v = NT ? __builtin_nontemporal_load(s + i + u * stride) : s[i + u * stride];
      acc += v[0] + v[3];
    }
  }
  if (acc == 1234.5f) *sink = acc;
}

template <bool NT>
__global__ void __launch_bounds__(256) write_k(f4v* __restrict__ d, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const f4v x = f4v{1.f, 2.f, 3.f, 4.f};
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    if (NT) __builtin_nontemporal_store(x, d + i);
    else d[i] = x;
  }
}

// non-persistent forms: one block per 256*U contiguous float4 (the guide's 6.29 TB/s "float4 copy")
template <int U, bool NT>
__global__ void __launch_bounds__(256) copy_flat_k(const f4v* __restrict__ s, f4v* __restrict__ d, size_t n) {
  const size_t base = static_cast<size_t>(blockIdx.x) * 256 * U + threadIdx.x;
  f4v v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const size_t i = base + u * 256;
    if (i < n) v[u] = NT ? __builtin_nontemporal_load(s + i) : s[i];
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const size_t i = base + u * 256;
    if (i < n) {
      if (NT) __builtin_nontemporal_store(v[u], d + i);
      else d[i] = v[u];
    }
  }
}

template <int U, bool NT>
__global__ void __launch_bounds__(256) read_flat_k(const f4v* __restrict__ s, size_t n, float* sink) {
  const size_t base = static_cast<size_t>(blockIdx.x) * 256 * U + threadIdx.x;
  float acc = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const size_t i = base + u * 256;
    if (i < n) {
      f4v v = NT ? __builtin_nontemporal_load(s + i) : s[i];
      acc += v[0] + v[3];
    }
  }
  if (acc == 1234.5f) *sink = acc;
}

template <bool NT>
__global__ void __launch_bounds__(256) write_flat_k(f4v* __restrict__ d, size_t n) {
  const size_t i = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x;
  const f4v x = f4v{1.f, 2.f, 3.f, 4.f};
  if (i < n) {
    if (NT) __builtin_nontemporal_store(x, d + i);
    else d[i] = x;
  }
}

int main(int argc, char** argv) {
  size_t bytes = (argc > 1 ? atol(argv[1]) : 4096) << 20;
  size_t n = bytes / 16;
  f4v *a, *b;
  float* sink;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(a, 0, bytes));
  CK(hipMemset(b, 0, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto time = [&](const char* name, double moved, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    const int it = 20;
    for (int i = 0; i < it; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"kernel\": \"%s\", \"tbs\": %.3f}\n", name, moved * it / (ms * 1e-3) / 1e12);
  };
  {
    char nm[64];
    for (int u : {1, 4}) {
      const unsigned blocks = static_cast<unsigned>((n + 256 * u - 1) / (256 * u));
      snprintf(nm, sizeof nm, "copy_flat_u%d", u);
      if (u == 1) time(nm, 2.0 * bytes, [&] { hipLaunchKernelGGL((copy_flat_k<1, false>), blocks, 256, 0, 0, a, b, n); });
      else time(nm, 2.0 * bytes, [&] { hipLaunchKernelGGL((copy_flat_k<4, false>), blocks, 256, 0, 0, a, b, n); });
      snprintf(nm, sizeof nm, "copy_flat_nt_u%d", u);
      if (u == 1) time(nm, 2.0 * bytes, [&] { hipLaunchKernelGGL((copy_flat_k<1, true>), blocks, 256, 0, 0, a, b, n); });
      else time(nm, 2.0 * bytes, [&] { hipLaunchKernelGGL((copy_flat_k<4, true>), blocks, 256, 0, 0, a, b, n); });
      snprintf(nm, sizeof nm, "read_flat_nt_u%d", u);
      if (u == 1) time(nm, 1.0 * bytes, [&] { hipLaunchKernelGGL((read_flat_k<1, true>), blocks, 256, 0, 0, a, n, sink); });
      else time(nm, 1.0 * bytes, [&] { hipLaunchKernelGGL((read_flat_k<4, true>), blocks, 256, 0, 0, a, n, sink); });
    }
  }
  {
    const unsigned blocks = static_cast<unsigned>((n + 255) / 256);
    time("write_flat", 1.0 * bytes, [&] { hipLaunchKernelGGL((write_flat_k<false>), blocks, 256, 0, 0, b, n); });
    time("write_flat_nt", 1.0 * bytes, [&] { hipLaunchKernelGGL((write_flat_k<true>), blocks, 256, 0, 0, b, n); });
  }
  for (int bpc : {4, 8, 16, 32}) {
    int grid = 256 * bpc;
    char nm[64];
#define RUN(label, moved, ...) snprintf(nm, sizeof nm, "%s_b%d", label, bpc); time(nm, moved, [&] { __VA_ARGS__; });
    RUN("copy_u4", 2.0 * bytes, hipLaunchKernelGGL((copy_k<4, false>), grid, 256, 0, 0, a, b, n));
    RUN("copy_u8", 2.0 * bytes, hipLaunchKernelGGL((copy_k<8, false>), grid, 256, 0, 0, a, b, n));
    RUN("copy_u4_nt", 2.0 * bytes, hipLaunchKernelGGL((copy_k<4, true>), grid, 256, 0, 0, a, b, n));
    RUN("copy_u8_nt", 2.0 * bytes, hipLaunchKernelGGL((copy_k<8, true>), grid, 256, 0, 0, a, b, n));
    RUN("read_u4", 1.0 * bytes, hipLaunchKernelGGL((read_k<4, false>), grid, 256, 0, 0, a, n, sink));
    RUN("read_u8", 1.0 * bytes, hipLaunchKernelGGL((read_k<8, false>), grid, 256, 0, 0, a, n, sink));
    RUN("read_u8_nt", 1.0 * bytes, hipLaunchKernelGGL((read_k<8, true>), grid, 256, 0, 0, a, n, sink));
    RUN("write", 1.0 * bytes, hipLaunchKernelGGL((write_k<false>), grid, 256, 0, 0, b, n));
    RUN("write_nt", 1.0 * bytes, hipLaunchKernelGGL((write_k<true>), grid, 256, 0, 0, b, n));
  }
  return 0;
}
