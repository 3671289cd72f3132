// Host memory of a HIP process, step by step (VmRSS / RssAnon / RssFile from /proc/self/status after each):
// where the ~0.5 GiB a diagnostic child peaks at comes from -- the runtime's start, the first allocation, the first
// kernel launch (code object load), or the diagnostics library itself.  One JSON line per step.
//
//   hipcc --offload-arch=gfx950 -O2 tools/hip_rss_probe.hip -o tools/hip_rss_probe.bin -ldl
//   tools/hip_rss_probe.bin [path/to/libmi355x_diag.so]
#include <hip/hip_runtime.h>
#include <dlfcn.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

static void step(const char* name) {
  long rss = -1, anon = -1, file = -1, shmem = -1, hwm = -1;
  if (FILE* f = std::fopen("/proc/self/status", "r")) {
    char line[256];
    while (std::fgets(line, sizeof line, f)) {
      long v = 0;
      if (std::sscanf(line, "VmRSS: %ld", &v) == 1) rss = v;
      else if (std::sscanf(line, "VmHWM: %ld", &v) == 1) hwm = v;
      else if (std::sscanf(line, "RssAnon: %ld", &v) == 1) anon = v;
      else if (std::sscanf(line, "RssFile: %ld", &v) == 1) file = v;
      else if (std::sscanf(line, "RssShmem: %ld", &v) == 1) shmem = v;
    }
    std::fclose(f);
  }
  std::printf("{\"step\":\"%s\",\"rss_mib\":%ld,\"peak_mib\":%ld,\"anon_mib\":%ld,\"file_mib\":%ld,\"shmem_mib\":%ld}\n",
              name, rss / 1024, hwm / 1024, anon / 1024, file / 1024, shmem / 1024);
  std::fflush(stdout);
}

__global__ void fill(float* p, size_t n, float v) {
  size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x;
  if (i < n) p[i] = v;
}

__global__ void lds_user(float* p) {
  __shared__ float s[16384];  // 64 KiB
  s[threadIdx.x] = static_cast<float>(threadIdx.x);
  __syncthreads();
  p[blockIdx.x * blockDim.x + threadIdx.x] = s[(threadIdx.x * 7) & 255];
}

// a private array indexed at run time lives in scratch (private_segment_fixed_size > 0): the runtime sets up scratch
// for the queue at this kernel's first dispatch
__global__ void scratch_user(float* p, int k) {
  float a[256];
#pragma unroll 1
  for (int i = 0; i < 256; ++i) a[i] = p[(i * 7 + threadIdx.x) & 4095];
  p[blockIdx.x * blockDim.x + threadIdx.x] = a[(threadIdx.x * 13 + k) & 255];
}

#define CHECK(x)                                                             \
  do {                                                                       \
    hipError_t e_ = (x);                                                     \
    if (e_ != hipSuccess) {                                                  \
      std::printf("{\"error\":\"%s\",\"at\":\"%s\"}\n", hipGetErrorString(e_), #x); \
      return 1;                                                              \
    }                                                                        \
  } while (0)

int main(int argc, char** argv) {
  step("start");
  int n = 0;
  CHECK(hipGetDeviceCount(&n));
  step("hipGetDeviceCount");
  CHECK(hipSetDevice(0));
  CHECK(hipFree(nullptr));
  step("context");
  float* p = nullptr;
  const size_t elems = size_t(64) << 20;  // 256 MiB
  CHECK(hipMalloc(&p, elems * sizeof(float)));
  step("hipMalloc 256 MiB");
  CHECK(hipMemset(p, 0, elems * sizeof(float)));
  CHECK(hipDeviceSynchronize());
  step("hipMemset");
  hipLaunchKernelGGL(fill, dim3(static_cast<unsigned>(elems / 256)), dim3(256), 0, nullptr, p, elems, 1.0f);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  step("first kernel");
  hipLaunchKernelGGL(lds_user, dim3(1024), dim3(256), 0, nullptr, p);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  step("64 KiB LDS kernel");
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipLaunchKernelGGL(fill, dim3(static_cast<unsigned>(elems / 256)), dim3(256), 0, st, p, elems, 2.0f);
  CHECK(hipStreamSynchronize(st));
  step("second stream");
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  CHECK(hipEventRecord(a, st));
  CHECK(hipEventRecord(b, st));
  CHECK(hipEventSynchronize(b));
  step("events");
  hipLaunchKernelGGL(scratch_user, dim3(1024), dim3(256), 0, nullptr, p, 3);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  step("first kernel with scratch");
  // `probe LIB KIB [pinned]`: one device-to-host copy of KIB KiB (into pinned memory with "pinned") and nothing else
  if (argc > 2) {
    const size_t s = static_cast<size_t>(std::atol(argv[2])) << 10;
    const bool pinned = argc > 3 && std::strcmp(argv[3], "pinned") == 0;
    void* dst = nullptr;
    if (pinned) CHECK(hipHostMalloc(&dst, s, hipHostMallocDefault));
    else dst = std::malloc(s);
    step(pinned ? "hipHostMalloc" : "malloc");
    CHECK(hipMemcpy(dst, p, s, hipMemcpyDeviceToHost));
    char label[64];
    std::snprintf(label, sizeof label, "%s D2H %zu KiB", pinned ? "pinned" : "pageable", s >> 10);
    step(label);
    return 0;
  }
  // pageable (malloc'd) copies of growing size each way: does the runtime stage them through a buffer of its own?
  {
    static char host[64 << 20];
    const size_t sizes[] = {size_t(4) << 10, size_t(64) << 10, size_t(1) << 20, size_t(16) << 20, size_t(64) << 20};
    char label[64];
    for (size_t s : sizes) {
      CHECK(hipMemcpy(host, p, s, hipMemcpyDeviceToHost));
      std::snprintf(label, sizeof label, "pageable D2H %zu KiB", s >> 10);
      step(label);
    }
    for (size_t s : sizes) {
      CHECK(hipMemcpy(p, host, s, hipMemcpyHostToDevice));
      std::snprintf(label, sizeof label, "pageable H2D %zu KiB", s >> 10);
      step(label);
    }
  }
  if (argc > 1) {
    void* h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      std::printf("{\"error\":\"dlopen: %s\"}\n", dlerror());
      return 1;
    }
    step("dlopen diag library");
    using hbm_fn = int (*)(int, size_t, int, double*, double*, double*);
    auto hbm = reinterpret_cast<hbm_fn>(dlsym(h, "diag_hbm_bandwidth"));
    if (hbm) {
      double c = 0, r = 0, w = 0;
      int rc = hbm(0, size_t(256) << 20, 2, &c, &r, &w);
      std::printf("{\"diag_hbm_rc\":%d,\"read_tbs\":%.3f}\n", rc, r);
      step("diag_hbm 256 MiB (first launch from the library)");
    }
  }
  CHECK(hipFree(p));
  step("end");
  return 0;
}
