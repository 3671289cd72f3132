// Node-level xGMI fabric check with RCCL, in one process (no torchrun, no torch): the node agent's
// level-2 collective test.  ncclCommInitAll gives one communicator per local MI355X; every collective
// is issued for all GPUs inside one ncclGroupStart/End from this thread, the way a multi-GPU-per-process
// nccl-tests run drives them.  The four collectives cover RCCL's two algorithm families on the 7
// point-to-point xGMI links of each GPU: rings (all-reduce, reduce-scatter, all-gather) and direct peer
// exchanges (all-to-all).
//
// Every op runs on rank-coded fp32 data whose result is exact (sums of small integers), and every
// received element is compared on the GPU:
//   all_reduce      in_r = r+1                      -> out = n(n+1)/2
//   reduce_scatter  in_r chunk c = (r+1)(c+1)       -> out_r = (r+1) n(n+1)/2
//   all_gather      in_r = r+1                      -> out chunk c = c+1
//   all_to_all      in_r chunk c = r*n + c          -> out_r chunk c = c*n + r
// Bandwidth follows the nccl-tests convention: bytes = the larger of the per-rank input and output,
// algbw = bytes / t, busbw = algbw * 2(n-1)/n (all-reduce) or algbw * (n-1)/n (the others).
//
// Hangs are bounded: the communicators are non-blocking (ncclConfig_t.blocking = 0), every wait polls the
// streams and ncclCommGetAsyncError against a deadline instead of sitting in hipStreamSynchronize, and a
// deadline that passes aborts every communicator (ncclCommAbort), so a link that stopped passing traffic
// comes back as a failed, aborted collective instead of a thread stuck forever in the node agent.
//
// C ABI (ctypes, ops/fabric.py):  fabric_open -> fabric_run (any number) -> fabric_close.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <string>
#include <thread>
#include <vector>

#include <unistd.h>

namespace {

thread_local std::string g_err;

// RCCL prints its version banner on stdout during communicator init; callers (mi355x-diag, the
// fabric CLI) write JSON there, so the banner is sent to stderr instead while the scope lives.
struct StdoutToStderr {
  int saved = -1;
  StdoutToStderr() {
    fflush(stdout);
    saved = dup(STDOUT_FILENO);
    if (saved >= 0 && dup2(STDERR_FILENO, STDOUT_FILENO) < 0) {
      close(saved);
      saved = -1;
    }
  }
  ~StdoutToStderr() {
    fflush(stdout);
    if (saved >= 0) {
      dup2(saved, STDOUT_FILENO);
      close(saved);
    }
  }
};

#define HIP_OK(expr)                                                          \
  do {                                                                        \
    hipError_t e_ = (expr);                                                   \
    if (e_ != hipSuccess) {                                                   \
      (void)hipGetLastError(); /* not left for the next call's check */      \
      g_err = std::string(#expr) + ": " + hipGetErrorString(e_);              \
      return -1;                                                              \
    }                                                                         \
  } while (0)

#define NCCL_OK(expr)                                                         \
  do {                                                                        \
    ncclResult_t r_ = (expr);                                                 \
    if (r_ != ncclSuccess) {                                                  \
      g_err = std::string(#expr) + ": " + ncclGetErrorString(r_);             \
      return -2;                                                              \
    }                                                                         \
  } while (0)

enum Op { ALL_REDUCE = 0, REDUCE_SCATTER = 1, ALL_GATHER = 2, ALL_TO_ALL = 3 };

// value of element i of a buffer made of chunks of `chunk` elements: a * (i / chunk) + b
__global__ void __launch_bounds__(256) fill_kernel(float* p, size_t n, size_t chunk, float a, float b) {
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n; i += stride)
    p[i] = a * static_cast<float>(i / chunk) + b;
}

__global__ void __launch_bounds__(256) verify_kernel(const float* p, size_t n, size_t chunk, float a, float b,
                                                     unsigned long long* errors) {
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  unsigned long long bad = 0;
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n; i += stride)
    bad += p[i] != a * static_cast<float>(i / chunk) + b;
  if (bad) atomicAdd(errors, bad);
}

struct Dev {
  int device = -1;
  ncclComm_t comm = nullptr;
  hipStream_t stream = nullptr;
  float* in = nullptr;
  float* out = nullptr;
  unsigned long long* errors = nullptr;
  size_t cap = 0;  // bytes of `in` and of `out`
};

struct Ctx {
  std::vector<Dev> devs;
  bool aborted = false;  // ncclCommAbort ran: no further collectives, buffers left to the process's end
};

using Clock = std::chrono::steady_clock;

// a wait's deadline; ms <= 0 waits without one
struct Deadline {
  bool on = false;
  Clock::time_point at;
  double ms = 0.0;
  explicit Deadline(double limit_ms) : on(limit_ms > 0), ms(limit_ms) {
    if (on) at = Clock::now() + std::chrono::microseconds(static_cast<int64_t>(limit_ms * 1000.0));
  }
  bool passed() const { return on && Clock::now() >= at; }
};

// Abort every communicator: the collective kernels stop waiting for peers that never arrive and RCCL
// releases the communicators.  The device buffers are not freed (a hipFree would wait for the device) --
// an aborted fabric check leaves them to the process, which the agent's liveness probe replaces anyway.
int abort_all(Ctx& c, const std::string& what, const Deadline& dl) {
  for (Dev& d : c.devs) {
    if (d.comm) {
      (void)hipSetDevice(d.device);
      (void)ncclCommAbort(d.comm);
      d.comm = nullptr;
    }
  }
  c.aborted = true;
  char ms[32];
  snprintf(ms, sizeof(ms), "%.0f", dl.ms);
  g_err = what + ": not complete within " + ms + " ms: communicators aborted (ncclCommAbort)";
  return -4;
}

// Wait until no communicator is in ncclInProgress (non-blocking init and group launches); an async error
// or the deadline aborts them all.
int wait_comms(Ctx& c, const Deadline& dl, const char* what) {
  for (;;) {
    bool pending = false;
    for (Dev& d : c.devs) {
      if (!d.comm) continue;
      ncclResult_t st = ncclSuccess;
      ncclResult_t r = ncclCommGetAsyncError(d.comm, &st);
      if (r != ncclSuccess) st = r;
      if (st == ncclInProgress) {
        pending = true;
      } else if (st != ncclSuccess) {
        const std::string why = std::string(what) + ": " + ncclGetErrorString(st);
        abort_all(c, why, dl);
        g_err = why + " (communicators aborted)";
        return -4;  // aborted like a missed deadline: the caller stops re-running the suite in this process
      }
    }
    if (!pending) return 0;
    if (dl.passed()) return abort_all(c, what, dl);
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

unsigned grid_for(size_t n) { return static_cast<unsigned>(std::min<size_t>((n + 255) / 256, 4096)); }

int ensure_buffers(Dev& d, size_t bytes) {
  if (d.cap >= bytes) return 0;
  HIP_OK(hipSetDevice(d.device));
  if (d.in) HIP_OK(hipFree(d.in));
  if (d.out) HIP_OK(hipFree(d.out));
  d.in = d.out = nullptr;
  d.cap = 0;
  HIP_OK(hipMalloc(&d.in, bytes));
  HIP_OK(hipMalloc(&d.out, bytes));
  d.cap = bytes;
  return 0;
}

// in/out element counts per rank for op, given `count` = elements of the larger buffer
void shapes(int op, size_t count, int n, size_t* in_n, size_t* out_n, size_t* per_rank) {
  switch (op) {
    case REDUCE_SCATTER: *in_n = count; *out_n = count / n; *per_rank = count / n; break;
    case ALL_GATHER: *in_n = count / n; *out_n = count; *per_rank = count / n; break;
    case ALL_TO_ALL: *in_n = count; *out_n = count; *per_rank = count / n; break;
    default: *in_n = count; *out_n = count; *per_rank = count; break;
  }
}

// ncclSuccess, or ncclInProgress from a non-blocking communicator (completion is polled in wait_comms)
#define NCCL_NB(expr)                                                         \
  do {                                                                        \
    ncclResult_t r_ = (expr);                                                 \
    if (r_ != ncclSuccess && r_ != ncclInProgress) {                          \
      g_err = std::string(#expr) + ": " + ncclGetErrorString(r_);             \
      return -2;                                                              \
    }                                                                         \
  } while (0)

// One collective on every GPU in one group; returns once RCCL has enqueued it on every stream.
int issue(Ctx& c, int op, size_t count, const Deadline& dl) {
  const int n = static_cast<int>(c.devs.size());
  size_t in_n, out_n, per;
  shapes(op, count, n, &in_n, &out_n, &per);
  NCCL_NB(ncclGroupStart());
  for (Dev& d : c.devs) {
    switch (op) {
      case ALL_REDUCE: NCCL_NB(ncclAllReduce(d.in, d.out, per, ncclFloat32, ncclSum, d.comm, d.stream)); break;
      case REDUCE_SCATTER:
        NCCL_NB(ncclReduceScatter(d.in, d.out, per, ncclFloat32, ncclSum, d.comm, d.stream));
        break;
      case ALL_GATHER: NCCL_NB(ncclAllGather(d.in, d.out, per, ncclFloat32, d.comm, d.stream)); break;
      default: NCCL_NB(ncclAllToAll(d.in, d.out, per, ncclFloat32, d.comm, d.stream)); break;
    }
  }
  ncclResult_t r = ncclGroupEnd();
  if (r == ncclInProgress) return wait_comms(c, dl, "collective launch");
  if (r != ncclSuccess) {
    g_err = std::string("ncclGroupEnd: ") + ncclGetErrorString(r);
    return -2;
  }
  return 0;
}

// Every stream drained.  Polled (hipStreamQuery + the communicators' async errors) rather than blocking in
// hipStreamSynchronize, so a collective that never completes is aborted at the deadline.
int sync_all(Ctx& c, const Deadline& dl, const char* what) {
  for (;;) {
    bool busy = false;
    for (Dev& d : c.devs) {
      HIP_OK(hipSetDevice(d.device));
      hipError_t e = hipStreamQuery(d.stream);
      if (e == hipErrorNotReady) {
        (void)hipGetLastError();
        busy = true;
      } else if (e != hipSuccess) {
        (void)hipGetLastError();
        g_err = std::string(what) + ": " + hipGetErrorString(e);
        return -1;
      }
    }
    if (!busy) return 0;
    for (Dev& d : c.devs) {
      ncclResult_t st = ncclSuccess;
      if (d.comm && ncclCommGetAsyncError(d.comm, &st) == ncclSuccess && st != ncclSuccess && st != ncclInProgress) {
        const std::string why = std::string(what) + ": " + ncclGetErrorString(st);
        abort_all(c, why, dl);
        g_err = why + " (communicators aborted)";
        return -4;  // aborted like a missed deadline: the caller stops re-running the suite in this process
      }
    }
    if (dl.passed()) return abort_all(c, what, dl);
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

}  // namespace

extern "C" {

const char* fabric_last_error(void) { return g_err.c_str(); }

int fabric_rccl_version(void) {
  int v = 0;
  return ncclGetVersion(&v) == ncclSuccess ? v : -1;
}

// One non-blocking communicator, stream and error counter per device (devices = HIP ordinals, n >= 1);
// communicator setup not complete within timeout_ms (> 0) is aborted and fails the open.
void* fabric_open(const int* devices, int n, double timeout_ms) {
  if (n < 1 || n > 64) {
    g_err = "fabric_open: 1..64 devices";
    return nullptr;
  }
  Ctx* c = new Ctx();
  c->devs.resize(static_cast<size_t>(n));
  std::vector<ncclComm_t> comms(static_cast<size_t>(n));
  auto fail = [&]() -> void* {
    for (Dev& d : c->devs) {
      if (d.device < 0) continue;
      (void)hipSetDevice(d.device);
      if (d.stream) (void)hipStreamDestroy(d.stream);
      if (d.errors) (void)hipFree(d.errors);
    }
    delete c;
    return nullptr;
  };
  for (int i = 0; i < n; ++i) {
    Dev& d = c->devs[static_cast<size_t>(i)];
    d.device = devices[i];
    hipError_t e = hipSetDevice(d.device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&d.errors, sizeof(unsigned long long));
    if (e != hipSuccess) {
      g_err = std::string("device setup: ") + hipGetErrorString(e);
      return fail();
    }
  }
  const Deadline dl(timeout_ms);
  ncclResult_t r;
  {
    // what ncclCommInitAll does, with a non-blocking config: one unique id, every rank initialised from
    // this thread inside one group
    StdoutToStderr quiet;
    ncclUniqueId id;
    r = ncclGetUniqueId(&id);
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    if (r == ncclSuccess) r = ncclGroupStart();
    for (int i = 0; i < n && (r == ncclSuccess || r == ncclInProgress); ++i) {
      (void)hipSetDevice(devices[i]);
      r = ncclCommInitRankConfig(&comms[static_cast<size_t>(i)], n, id, i, &cfg);
    }
    ncclResult_t e = ncclGroupEnd();
    if (r == ncclSuccess || r == ncclInProgress) r = e;
  }
  if (r != ncclSuccess && r != ncclInProgress) {
    g_err = std::string("ncclCommInitRankConfig (non-blocking): ") + ncclGetErrorString(r);
    for (ncclComm_t cm : comms)
      if (cm) (void)ncclCommAbort(cm);
    return fail();
  }
  for (int i = 0; i < n; ++i) c->devs[static_cast<size_t>(i)].comm = comms[static_cast<size_t>(i)];
  if (wait_comms(*c, dl, "communicator init") != 0) {
    const std::string why = g_err;
    for (Dev& d : c->devs) d.comm = nullptr;  // aborted in wait_comms
    fail();
    g_err = why;
    return nullptr;
  }
  return c;
}

// Run `op` on `bytes` per rank (rounded down to a whole number of fp32 chunks): `warmup` untimed calls,
// `iters` timed calls (host wall clock from the first issue to the last stream's completion), then one
// verified call.  out[0] = ms per call, out[1] = algbw GB/s, out[2] = busbw GB/s, out[3] = bad elements
// summed over every GPU.  All of it within timeout_ms (> 0), else the communicators are aborted and the
// call returns -4 (the context then refuses further runs).
int fabric_run(void* ctx, int op, size_t bytes, int iters, int warmup, double* out, double timeout_ms) {
  if (!ctx || op < 0 || op > 3 || iters < 1 || warmup < 0) {
    g_err = "fabric_run: bad arguments";
    return -3;
  }
  Ctx& c = *static_cast<Ctx*>(ctx);
  if (c.aborted) {
    g_err = "fabric_run: communicators were aborted by an earlier timeout";
    return -4;
  }
  const Deadline dl(timeout_ms);
  const int n = static_cast<int>(c.devs.size());
  size_t count = bytes / sizeof(float);
  count -= count % static_cast<size_t>(n);
  if (count == 0) {
    g_err = "fabric_run: message smaller than one element per rank";
    return -3;
  }
  size_t in_n, out_n, per;
  shapes(op, count, n, &in_n, &out_n, &per);
  for (Dev& d : c.devs)
    if (ensure_buffers(d, count * sizeof(float)) != 0) return -1;

  for (int r = 0; r < n; ++r) {  // rank-coded inputs (see the header)
    Dev& d = c.devs[static_cast<size_t>(r)];
    HIP_OK(hipSetDevice(d.device));
    float a = 0.f, b = static_cast<float>(r + 1);
    size_t chunk = in_n;
    if (op == REDUCE_SCATTER) { a = static_cast<float>(r + 1); b = static_cast<float>(r + 1); chunk = per; }
    if (op == ALL_TO_ALL) { a = 1.f; b = static_cast<float>(r * n); chunk = per; }
    hipLaunchKernelGGL(fill_kernel, dim3(grid_for(in_n)), dim3(256), 0, d.stream, d.in, in_n, chunk, a, b);
    HIP_OK(hipGetLastError());
  }
  if (int rc = sync_all(c, dl, "input fill"); rc != 0) return rc;

  // the deadline is checked between launches too: a long run must not enqueue past it before any wait
  for (int i = 0; i < warmup; ++i) {
    if (dl.passed()) return abort_all(c, "warm-up collectives", dl);
    if (int rc = issue(c, op, count, dl); rc != 0) return rc;
  }
  if (int rc = sync_all(c, dl, "warm-up collectives"); rc != 0) return rc;
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < iters; ++i) {
    if (dl.passed()) return abort_all(c, "timed collectives", dl);
    if (int rc = issue(c, op, count, dl); rc != 0) return rc;
  }
  if (int rc = sync_all(c, dl, "timed collectives"); rc != 0) return rc;
  const double ms =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() / iters;

  // one more call on freshly zeroed outputs, then every element checked on its GPU
  for (Dev& d : c.devs) {
    HIP_OK(hipSetDevice(d.device));
    HIP_OK(hipMemsetAsync(d.out, 0, out_n * sizeof(float), d.stream));
    HIP_OK(hipMemsetAsync(d.errors, 0, sizeof(unsigned long long), d.stream));
  }
  if (int rc = issue(c, op, count, dl); rc != 0) return rc;
  const float tri = static_cast<float>(n) * static_cast<float>(n + 1) / 2.f;
  for (int r = 0; r < n; ++r) {
    Dev& d = c.devs[static_cast<size_t>(r)];
    HIP_OK(hipSetDevice(d.device));
    float a = 0.f, b = tri;
    size_t chunk = out_n;
    if (op == REDUCE_SCATTER) b = static_cast<float>(r + 1) * tri;
    if (op == ALL_GATHER) { a = 1.f; b = 1.f; chunk = per; }
    if (op == ALL_TO_ALL) { a = static_cast<float>(n); b = static_cast<float>(r); chunk = per; }
    hipLaunchKernelGGL(verify_kernel, dim3(grid_for(out_n)), dim3(256), 0, d.stream, d.out, out_n, chunk, a, b,
                       d.errors);
    HIP_OK(hipGetLastError());
  }
  if (int rc = sync_all(c, dl, "verified collective"); rc != 0) return rc;
  unsigned long long bad = 0;
  for (Dev& d : c.devs) {
    unsigned long long e = 0;
    HIP_OK(hipSetDevice(d.device));
    HIP_OK(hipMemcpy(&e, d.errors, sizeof(e), hipMemcpyDeviceToHost));
    bad += e;
  }
  const double moved = static_cast<double>(count * sizeof(float));  // the larger per-rank buffer
  const double algbw = moved / (ms * 1e-3) / 1e9;
  const double factor = op == ALL_REDUCE ? 2.0 * (n - 1) / n : static_cast<double>(n - 1) / n;
  out[0] = ms;
  out[1] = algbw;
  out[2] = algbw * factor;
  out[3] = static_cast<double>(bad);
  return 0;
}

int fabric_aborted(void* ctx) { return ctx && static_cast<Ctx*>(ctx)->aborted ? 1 : 0; }

void fabric_close(void* ctx) {
  if (!ctx) return;
  Ctx* c = static_cast<Ctx*>(ctx);
  if (c->aborted) {  // see abort_all: nothing that could wait on the device
    for (Dev& d : c->devs)
      if (d.device >= 0 && d.stream) {
        (void)hipSetDevice(d.device);
        (void)hipStreamDestroy(d.stream);
      }
    delete c;
    return;
  }
  for (Dev& d : c->devs) {
    if (d.device < 0) continue;
    (void)hipSetDevice(d.device);
    if (d.stream) (void)hipStreamSynchronize(d.stream);
    if (d.comm) (void)ncclCommDestroy(d.comm);
    if (d.stream) (void)hipStreamDestroy(d.stream);
    if (d.in) (void)hipFree(d.in);
    if (d.out) (void)hipFree(d.out);
    if (d.errors) (void)hipFree(d.errors);
  }
  delete c;
}

}  // extern "C"
