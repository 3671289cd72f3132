// Active MI355X diagnostics (gfx950 / CDNA4 only): the "deep" health checks the
// node agent can run besides the passive amd-smi probe.  A node can be
// Ready=True with clean ECC counters and still have a GPU that computes wrong
// results, runs at a fraction of its matrix rate (stuck clocks, throttling) or
// has a weak HBM stack; these kernels measure exactly that.
//
//   gemm_bf16   C[M,N] = A[M,K] . Bt[N,K]^T, bf16 in / fp32 out on MFMA
//               (v_mfma_f32_16x16x32_bf16), XOR-swizzled LDS (conflict-free
//               ds_read_b128 fragment loads), XCD-aware tile order.
//               v4: 256x256x64 tiles, 4 waves of 128x128 each, the loop's MFMA /
//                   ds_read / LDS-DMA interleave written out in asm on a checked
//                   plan (v4_plan.h); bf16 and fp8 (16x16x128, by quadrant), the
//                   default for large GEMMs;
//               v3: the same tile, 8 waves in two barrier-staggered groups, LDS-DMA
//                   restaged region by region (MX-fp4, the scaled MX-fp8 form, and
//                   bf16 / fp8 for A/B);
//               v2: the same tile, one barrier per K-tile (kept for A/B);
//               v1: 128x128x64 tiles, 4 waves, register-staged (small grids).
//               Verified against an fp32 reference kernel on sampled outputs.
//   hbm_copy / hbm_read / hbm_write
//               16-byte nontemporal streams, 8 loads in flight per thread,
//               32 blocks per CU; TB/s against the 8 TB/s HBM3E spec.
//   memtest     address-hash patterns written and verified (plus the
//               bit-inverted pass), mismatches counted with one atomic per
//               failing 16-byte word.
//   p2p_copy    xGMI pair check: peer copies between two GPUs of the node,
//               timed, and the received pattern verified on the destination.
//   host_link   pinned host <-> device copy bandwidth over the PCIe link.
//   mfma_burn   matrix-core datapath burn-in per precision (bf16, fp8, MX-fp8,
//               MX-fp4), register-resident, every lane's exact result checked.
//
// C ABI (ctypes, ops/diag.py).  Every HIP call is checked; on failure the
// function returns a negative code and diag_last_error() says what failed.
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

namespace {

thread_local std::string g_err;
// GEMM knobs are per calling thread: the node agent runs one diagnostic thread per GPU at once, and a
// test or tool that switches a variant must not change what another GPU's thread launches.
thread_local int g_gemm_variant = 0;
thread_local int g_gemm_schedule = 1;  // v3 restaging order (V3_PHASE): 1 = LDS-DMA pieces per phase 0/2/2/4, 0 = 2/0/4/2
thread_local int g_gemm_buffer_loads = 0;  // v3 operand staging: 0 = global_load_lds, 1 = buffer_load ... lds
// fp8 v3 MFMA: 1 = the unscaled v_mfma_f32_16x16x128_f8f6f4 (hipBLASLt's fp8 form, the default: +5.6 % over the
// scaled form at 4096^3 and 8192^3 with bit-identical C, profiles/gemm_fp8_mfma_ab_mi355x.jsonl), 0 = the
// v_mfma_scale_..._f8f6f4 MX path with unit E8M0 scales (kept for A/B)
thread_local int g_gemm_fp8_unscaled = 1;
// v4 bf16: a short last wave of 256^2 tiles runs as 128^2 quadrants (gemm_v4_tail_kernel; 0 = off, for A/B)
thread_local int g_gemm_tail = 1;
thread_local int g_gemm_epilogue = 1;  // 0 = direct 4-byte stores, 1 = LDS-staged 16-byte row pieces (v3
                                       // kernels; measured +2..12 %, profiles/gemm_fp8_mi355x.jsonl)

#define DIAG_CHECK(expr)                                                                  \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess) {                                                               \
      (void)hipGetLastError(); /* a failed allocation must not fail the next call's check */ \
      g_err = std::string(#expr) + ": " + hipGetErrorString(e_);                          \
      return -1;                                                                          \
    }                                                                                     \
  } while (0)

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));  // native 16-byte vector (SROA-friendly, unlike uint4)
typedef int i32x8 __attribute__((ext_vector_type(8)));            // 32 fp8 / 64 fp4 operand bytes

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int THREADS = 256;
constexpr int CHUNKS_PER_ROW = BK / 8;                 // 16-byte chunks per 64-wide bf16 row
constexpr int TILE_CHUNKS = BM * CHUNKS_PER_ROW;       // 1024 chunks per operand tile
constexpr int LOADS_PER_THREAD = TILE_CHUNKS / THREADS;  // 4

// LDS image: [row][8 chunks of 16 B], chunk c of row r stored at c ^ ((r >> 1) & 7).
// For the 16x16x32 fragment read (lane l: row l&15, chunk (l>>4)+4s) this puts
// every ds_read_b128 lane group on 16 distinct 16-byte slots (all 64 banks).
__device__ __forceinline__ int swz(int r, int c) { return r * CHUNKS_PER_ROW + (c ^ ((r >> 1) & 7)); }

// The fp8 16x16x128 fragment (lane l: row l&15, 32 bytes = chunks 2(l>>4), 2(l>>4)+1) needs another
// XOR: f8(r) = 3*r[3] ^ 4*r[1] puts each ds_read_b128 lane group of both chunk reads on 16 distinct
// 16-byte slots (searched exhaustively over GF(2)-linear swizzles; it is conflict-free for the bf16
// fragment pattern too).
__device__ __forceinline__ int swz_row_xor(int r, bool fp8) {
  return fp8 ? ((((r >> 3) & 1) * 3) ^ (((r >> 1) & 1) << 2)) : ((r >> 1) & 7);
}
__device__ __forceinline__ int swz8(int r, int c) { return r * CHUNKS_PER_ROW + (c ^ swz_row_xor(r, true)); }

__device__ __forceinline__ void gemm_gload(u32x4 (&ra)[LOADS_PER_THREAD], u32x4 (&rb)[LOADS_PER_THREAD],
                                           const u32x4* __restrict__ Ablk, const u32x4* __restrict__ Bblk,
                                           const int (&g_off)[LOADS_PER_THREAD], int kt) {
#pragma unroll
  for (int i = 0; i < LOADS_PER_THREAD; ++i) {
    ra[i] = Ablk[g_off[i] + kt * CHUNKS_PER_ROW];
    rb[i] = Bblk[g_off[i] + kt * CHUNKS_PER_ROW];
  }
}

__device__ __forceinline__ void gemm_lstore(u32x4 (&buf)[2][TILE_CHUNKS], const u32x4 (&ra)[LOADS_PER_THREAD],
                                            const u32x4 (&rb)[LOADS_PER_THREAD], const int (&l_off)[LOADS_PER_THREAD]) {
#pragma unroll
  for (int i = 0; i < LOADS_PER_THREAD; ++i) {
    buf[0][l_off[i]] = ra[i];
    buf[1][l_off[i]] = rb[i];
  }
}

// One BK=64 step: 2 x (4 A-fragments, 4 B-fragments, 16 MFMA 16x16x32).
__device__ __forceinline__ void gemm_compute(floatx4 (&acc)[4][4], const u32x4 (&buf)[2][TILE_CHUNKS], int wr, int wc,
                                             int frow, int fq) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    bf16x8 af[4], bfr[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) af[m] = __builtin_bit_cast(bf16x8, buf[0][swz(wr * 64 + m * 16 + frow, fq + 4 * s)]);
#pragma unroll
    for (int n = 0; n < 4; ++n) bfr[n] = __builtin_bit_cast(bf16x8, buf[1][swz(wc * 64 + n * 16 + frow, fq + 4 * s)]);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n)
        acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m], bfr[n], acc[m][n], 0, 0, 0);
  }
}

__global__ void __launch_bounds__(THREADS, 2)
gemm_bf16_kernel(const u32x4* __restrict__ A, const u32x4* __restrict__ Bt, float* __restrict__ C, int M, int N,
                 int K) {
  __shared__ u32x4 lds[2][2][TILE_CHUNKS];  // [buffer][A|B][chunk]  = 64 KiB
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;

  // XCD-aware, grouped tile order: consecutive blocks land on different XCDs
  // (round-robin dispatch), so regroup ids so one XCD walks a compact 2D patch.
  const int tiles_m = M / BM, tiles_n = N / BN;
  const int nwg = tiles_m * tiles_n;
  int bid = blockIdx.x;
  {
    const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
  }
  constexpr int GROUP_M = 8;
  const int group = bid / (GROUP_M * tiles_n);
  const int first_m = group * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  const int tm = first_m + (bid % (GROUP_M * tiles_n)) % gsize;
  const int tn = (bid % (GROUP_M * tiles_n)) / gsize;

  const int kchunks = K / 8;  // 16-byte chunks per row of A / Bt
  const u32x4* Ablk = A + static_cast<size_t>(tm) * BM * kchunks;
  const u32x4* Bblk = Bt + static_cast<size_t>(tn) * BN * kchunks;

  u32x4 ra[LOADS_PER_THREAD], rb[LOADS_PER_THREAD];
  // per-thread chunk coordinates are loop invariant
  int g_off[LOADS_PER_THREAD], l_off[LOADS_PER_THREAD];
#pragma unroll
  for (int i = 0; i < LOADS_PER_THREAD; ++i) {
    const int ch = tid + i * THREADS;
    const int r = ch / CHUNKS_PER_ROW, c = ch % CHUNKS_PER_ROW;
    g_off[i] = r * kchunks + c;
    l_off[i] = swz(r, c);
  }
  floatx4 acc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int KT = K / BK;
  const int frow = lane & 15, fq = lane >> 4;
  gemm_gload(ra, rb, Ablk, Bblk, g_off, 0);
  gemm_lstore(lds[0], ra, rb, l_off);
  __syncthreads();
  // two K-steps per trip so the LDS buffer index is a compile-time constant
  for (int kt = 0; kt < KT; kt += 2) {
    const bool more1 = kt + 1 < KT;
    if (more1) gemm_gload(ra, rb, Ablk, Bblk, g_off, kt + 1);
    gemm_compute(acc, lds[0], wr, wc, frow, fq);
    if (more1) gemm_lstore(lds[1], ra, rb, l_off);
    __syncthreads();
    if (!more1) break;
    const bool more2 = kt + 2 < KT;
    if (more2) gemm_gload(ra, rb, Ablk, Bblk, g_off, kt + 2);
    gemm_compute(acc, lds[1], wr, wc, frow, fq);
    if (more2) gemm_lstore(lds[0], ra, rb, l_off);
    __syncthreads();
  }
  // C/D layout of 16x16x32: col = lane & 15, row = (lane >> 4) * 4 + reg
  const int row0 = tm * BM + wr * 64, col0 = tn * BN + wc * 64;
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        C[static_cast<size_t>(row0 + m * 16 + fq * 4 + j) * N + col0 + n * 16 + frow] = acc[m][n][j];
}

// ---------------------------------------------------------------------------
// gemm v2: 256x256x64 block tile, 8 waves (2 M x 4 N, 128x64 each), operands
// streamed global -> LDS by LDS-DMA (global_load_lds_dwordx4: no VGPR staging,
// 8 per thread per stage), two LDS stages of 64 KiB (1 block per CU), the same
// XOR swizzle as v1 applied on the *global source* address because an LDS-DMA
// wave instruction writes 1 KiB lane-linearly (8 rows of 128 B).
constexpr int V2_BM = 256, V2_BN = 256, V2_THREADS = 512;
constexpr int V2_ROWS_PER_WAVE = 32;                   // rows of each operand one wave fills per stage
constexpr int V2_STAGE_BYTES = 2 * V2_BM * BK * 2;     // A + B, bf16 = 64 KiB

typedef __attribute__((address_space(3))) void lds_void_t;

template <bool FP8 = false>
__device__ __forceinline__ void v2_fill(unsigned char* lds_stage, const __bf16* __restrict__ A,
                                        const __bf16* __restrict__ Bt, int K, int kt, int wid, int lane) {
  // lane -> (row within an 8-row group, physical chunk); logical chunk = phys ^ swizzle(row)
  const int rsub = lane >> 3, phys = lane & 7;
#pragma unroll
  for (int op = 0; op < 2; ++op) {
    const __bf16* src = op == 0 ? A : Bt;
#pragma unroll
    for (int j = 0; j < V2_ROWS_PER_WAVE / 8; ++j) {
      const int row = wid * V2_ROWS_PER_WAVE + j * 8 + rsub;
      const int c = phys ^ swz_row_xor(row, FP8);
      const __bf16* g = src + static_cast<size_t>(row) * K + kt * BK + c * 8;
      unsigned char* l = lds_stage + op * (V2_BM * BK * 2) + (wid * V2_ROWS_PER_WAVE + j * 8) * (BK * 2);
      __builtin_amdgcn_global_load_lds(g, (lds_void_t*)l, 16, 0, 0);
    }
  }
}

__device__ __forceinline__ void v2_compute(floatx4 (&acc)[8][4], const u32x4* __restrict__ a_img,
                                           const u32x4* __restrict__ b_img, int wr, int wc, int frow, int fq) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    bf16x8 bfr[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) bfr[n] = __builtin_bit_cast(bf16x8, b_img[swz(wc * 64 + n * 16 + frow, fq + 4 * s)]);
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const bf16x8 af = __builtin_bit_cast(bf16x8, a_img[swz(wr * 128 + m * 16 + frow, fq + 4 * s)]);
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[n], acc[m][n], 0, 0, 0);
    }
  }
}

__global__ void __launch_bounds__(V2_THREADS, 1)
gemm_bf16_v2_kernel(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt, float* __restrict__ C, int M, int N,
                    int K) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];  // 2 stages x 64 KiB (dynamic)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
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
  v2_fill(smem, Ab, Bb, K, 0, wid, lane);
  __builtin_amdgcn_s_waitcnt(0x3f70);  // vmcnt(0) (gfx9 encoding: vmcnt[3:0]=0, vmcnt[15:14]=0)
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    unsigned char* cur = smem + (kt & 1) * V2_STAGE_BYTES;
    if (kt + 1 < KT) v2_fill(smem + ((kt + 1) & 1) * V2_STAGE_BYTES, Ab, Bb, K, kt + 1, wid, lane);
    v2_compute(acc, reinterpret_cast<const u32x4*>(cur), reinterpret_cast<const u32x4*>(cur + V2_BM * BK * 2), wr, wc,
               frow, fq);
    __builtin_amdgcn_s_waitcnt(0x3f70);  // this wave's LDS-DMA for stage kt+1 has landed
    __syncthreads();                     // ... and everyone's; stage kt is free for kt+2
  }
  const int row0 = tm * V2_BM + wr * 128, col0 = tn * V2_BN + wc * 64;
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        C[static_cast<size_t>(row0 + m * 16 + fq * 4 + j) * N + col0 + n * 16 + frow] = acc[m][n][j];
}

// ---------------------------------------------------------------------------
// gemm v3: the v2 tile and LDS image on a staggered 4-phase schedule (tools/gemm_lab.hip "v5";
// +5-7 % over v2 at 4096^3/8192^3 on MI355X, profiles/gemm_lab_*.jsonl).
// Waves 0-3 and 4-7 form two groups (one wave of each per SIMD); group 1 runs one s_barrier behind
// group 0, so on every SIMD one wave's MFMA slot covers the other's load slot and barrier wait.
// Each K-tile is 4 phases, one 64x32 quadrant of the wave's 128x64 output each (16 MFMA):
//   load slot: this quadrant's ds_reads (+ LDS-DMA restaging) -> s_barrier -> lgkmcnt(0) ->
//   MFMA slot -> s_barrier.
// Quadrant order (m0,n0) (m0,n1) (m1,n1) (m1,n0): phase 0 reads A(m0)+B(n0), phase 1 B(n1), phase 2
// A(m1), phase 3 reuses B(n0) from registers.  A stage is restaged region by region (16 KiB each):
// R0 = A rows of m0, R1 = B rows of n0, R2 = B rows of n1, R3 = A rows of m1.  Reads retire after
// the barrier that closes their load slot, so a region read in phase p is free two phases later:
// R0 of tile t+2 goes out in phase 2 of tile t, R1 and R2 in phase 3, and R3 of tile t+1 (other
// buffer, last read in phase 2 of tile t-1) in phase 1 (V3_PHASE: which phase carries which piece
// is worth 4-9 %).  Tile t+1 is retired at phase 3 of tile t with a counted vmcnt(6) (tile t+2's
// R0-R2 may stay in flight); raw s_barrier only -- __syncthreads() would drain the in-flight
// LDS-DMA with vmcnt(0).
#define STG_BARRIER()                  \
  do {                                 \
    __builtin_amdgcn_sched_barrier(0); \
    __builtin_amdgcn_s_barrier();      \
    __builtin_amdgcn_sched_barrier(0); \
  } while (0)

// One 16 KiB region of a stage: 16 LDS-DMA wave-instructions of 8 rows, 2 per wave.
template <bool FP8>
__device__ __forceinline__ void stg_region(unsigned char* lds_stage, const __bf16* __restrict__ A,
                                           const __bf16* __restrict__ Bt, int K, int kt, int region, int i, int wid,
                                           int lane) {
  const int rsub = lane >> 3, phys = lane & 7;
  const int g = wid * 2 + i;
  const bool is_a = region == 0 || region == 3;
  const int row0 = is_a ? (g >> 3) * 128 + (region == 0 ? 0 : 64) + (g & 7) * 8
                        : (g >> 2) * 64 + (region == 1 ? 0 : 32) + (g & 3) * 8;
  const int row = row0 + rsub;
  const int c = phys ^ swz_row_xor(row, FP8);
  const __bf16* gp = (is_a ? A : Bt) + static_cast<size_t>(row) * K + kt * BK + c * 8;
  unsigned char* l = lds_stage + (is_a ? 0 : V2_BM * BK * 2) + row0 * (BK * 2);
  __builtin_amdgcn_global_load_lds(gp, (lds_void_t*)l, 16, 0, 0);
}

// The same region through the buffer path (`buffer_load_dwordx4 ... lds`): the tile's A and B slabs
// are two scalar buffer resources, the per-lane byte offset is loop-invariant and the K-tile moves
// only the scalar soffset, so no 64-bit per-lane address math is redone per K-tile.
struct StgBuf {
  __amdgpu_buffer_rsrc_t a, b;
};

__device__ __forceinline__ StgBuf stg_buf(const __bf16* A, const __bf16* Bt, int K) {
  // CDNA raw-buffer dword3 (32-bit data format, no swizzle); num_records = one 256-row slab
  const int bytes = V2_BM * K * 2;
  return StgBuf{__builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(A), static_cast<short>(0), bytes, 0x00020000),
                __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(Bt), static_cast<short>(0), bytes, 0x00020000)};
}

template <bool FP8>
__device__ __forceinline__ void stg_region_buf(unsigned char* lds_stage, const StgBuf& rs, int K, int kt, int region,
                                               int i, int wid, int lane) {
  const int rsub = lane >> 3, phys = lane & 7;
  const int g = wid * 2 + i;
  const bool is_a = region == 0 || region == 3;
  const int row0 = is_a ? (g >> 3) * 128 + (region == 0 ? 0 : 64) + (g & 7) * 8
                        : (g >> 2) * 64 + (region == 1 ? 0 : 32) + (g & 3) * 8;
  const int row = row0 + rsub;
  const int c = phys ^ swz_row_xor(row, FP8);
  const int voff = (row * K + c * 8) * 2;
  unsigned char* l = lds_stage + (is_a ? 0 : V2_BM * BK * 2) + row0 * (BK * 2);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(is_a ? rs.a : rs.b, (lds_void_t*)l, 16, voff, kt * BK * 2, 0, 0);
}

template <bool FP8>
__device__ __forceinline__ void v2_fill_buf(unsigned char* lds_stage, const StgBuf& rs, int K, int kt, int wid,
                                            int lane) {
  const int rsub = lane >> 3, phys = lane & 7;
#pragma unroll
  for (int op = 0; op < 2; ++op) {
#pragma unroll
    for (int j = 0; j < V2_ROWS_PER_WAVE / 8; ++j) {
      const int row = wid * V2_ROWS_PER_WAVE + j * 8 + rsub;
      const int c = phys ^ swz_row_xor(row, FP8);
      unsigned char* l = lds_stage + op * (V2_BM * BK * 2) + (wid * V2_ROWS_PER_WAVE + j * 8) * (BK * 2);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(op == 0 ? rs.a : rs.b, (lds_void_t*)l, 16, (row * K + c * 8) * 2,
                                               kt * BK * 2, 0, 0);
    }
  }
}

__device__ __forceinline__ void stg_mfma(floatx4 (&acc)[8][4], const bf16x8 (&af)[4][2], const bf16x8 (&bf)[2][2],
                                         int m0, int n0) {
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n)
        acc[m0 + m][n0 + n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m][s], bf[n][s], acc[m0 + m][n0 + n], 0, 0, 0);
  // MFMAs are not memory operations, so IR passes may sink them past the next s_barrier into the
  // other group's slot; an empty volatile asm that reads and writes each result pins them here.
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n) asm volatile("" : "+v"(acc[m0 + m][n0 + n]));
}

// MX-fp8 (E4M3, unit E8M0 scales): one v_mfma_scale_f32_16x16x128_f8f6f4 covers the K-tile's 128 bytes.
__device__ __forceinline__ void stg_mfma(floatx4 (&acc)[8][4], const i32x8 (&af)[4], const i32x8 (&bf)[2], int m0,
                                         int n0) {
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
      acc[m0 + m][n0 + n] =
          __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[m], bf[n], acc[m0 + m][n0 + n], 0, 0, 0, 127, 0, 127);
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n) asm volatile("" : "+v"(acc[m0 + m][n0 + n]));
}

// The same K-tile on the unscaled instruction (zero scale operands select v_mfma_f32_16x16x128_f8f6f4): with unit
// scales the two compute the same products, so the knob only changes which matrix-core path runs.
__device__ __forceinline__ void stg_mfma_unscaled(floatx4 (&acc)[8][4], const i32x8 (&af)[4], const i32x8 (&bf)[2],
                                                  int m0, int n0) {
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
      acc[m0 + m][n0 + n] =
          __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[m], bf[n], acc[m0 + m][n0 + n], 0, 0, 0, 0, 0, 0);
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n) asm volatile("" : "+v"(acc[m0 + m][n0 + n]));
}

// Fragment of one 16-row block: bf16 = two K=32 steps (chunks fq, fq+4); fp8 = the lane's 32
// contiguous bytes of K (chunks 2fq, 2fq+1; lane layout measured by tools/mfma_lab.hip).
__device__ __forceinline__ void stg_load(bf16x8 (&f)[2], const u32x4* img, int row, int fq) {
  f[0] = __builtin_bit_cast(bf16x8, img[swz(row, fq)]);
  f[1] = __builtin_bit_cast(bf16x8, img[swz(row, fq + 4)]);
}
__device__ __forceinline__ void stg_load(i32x8& f, const u32x4* img, int row, int fq) {
  const u32x4 lo = img[swz8(row, 2 * fq)], hi = img[swz8(row, 2 * fq + 1)];
  f = i32x8{static_cast<int>(lo.x), static_cast<int>(lo.y), static_cast<int>(lo.z), static_cast<int>(lo.w),
            static_cast<int>(hi.x), static_cast<int>(hi.y), static_cast<int>(hi.z), static_cast<int>(hi.w)};
}

// MX-fp4 (E2M1): a 16-byte chunk is 32 values = one lane's share of a 16x16x128 MFMA, so the fp4
// fragments are read exactly like the bf16 ones (chunks fq, fq + 4) and feed two MFMAs per K-tile.
__device__ __forceinline__ void stg_load(u32x4 (&f)[2], const u32x4* img, int row, int fq) {
  f[0] = img[swz(row, fq)];
  f[1] = img[swz(row, fq + 4)];
}

__device__ __forceinline__ void stg_mfma(floatx4 (&acc)[8][4], const u32x4 (&af)[4][2], const u32x4 (&bf)[2][2],
                                         int m0, int n0) {
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const u32x4 a = af[m][s], b = bf[n][s];
        const i32x8 a8 = {static_cast<int>(a.x), static_cast<int>(a.y), static_cast<int>(a.z), static_cast<int>(a.w),
                          0, 0, 0, 0};
        const i32x8 b8 = {static_cast<int>(b.x), static_cast<int>(b.y), static_cast<int>(b.z), static_cast<int>(b.w),
                          0, 0, 0, 0};
        acc[m0 + m][n0 + n] =
            __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a8, b8, acc[m0 + m][n0 + n], 4, 4, 0, 127, 0, 127);
      }
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n) asm volatile("" : "+v"(acc[m0 + m][n0 + n]));
}

enum GemmDtype { DT_BF16 = 0, DT_FP8 = 1, DT_FP4 = 2, DT_FP8U = 3 /* fp8 operands, unscaled MFMA */ };

template <int DT>
struct StgFrags {
  bf16x8 a[4][2], b0[2][2], b1[2][2];
};
template <>
struct StgFrags<DT_FP8> {
  i32x8 a[4], b0[2], b1[2];
};
template <>
struct StgFrags<DT_FP8U> {
  i32x8 a[4], b0[2], b1[2];
};

// One phase's MFMAs for the kernel's data type.
template <int DT, typename FA, typename FB>
__device__ __forceinline__ void phase_mfma(floatx4 (&acc)[8][4], const FA& af, const FB& bf, int m0, int n0) {
  if constexpr (DT == DT_FP8U) stg_mfma_unscaled(acc, af, bf, m0, n0);
  else stg_mfma(acc, af, bf, m0, n0);
}
template <>
struct StgFrags<DT_FP4> {
  u32x4 a[4][2], b0[2][2], b1[2][2];
};

// v3 restaging orders (region r = 0: A rows of m0, 1: B rows of n0, 2: B rows of n1, 3: A rows of m1).
// V3_PHASE[s][r]: the phase of a K-tile whose load slot issues region r, for tile kt+2 into this buffer (R0/R1
// are free from phase 2 on, R2 from phase 3) or, R3, tile kt+1 into the other one (free since tile kt-1).
// Phase 3 retires tile kt+1 with vmcnt(6): tile kt+2's R0-R2 (2 pieces each) may stay in flight.
//   0: R3@0, R0 R1@2, R2@3 -> LDS-DMA pieces per phase 2/0/4/2 (round-2/3 kernel)
//   1: R3@1, R0@2, R1 R2@3 -> 0/2/2/4: no DMA issue beside phase 0's 12 fragment reads, 2 beside phase 2's 8
// An LDS-DMA piece costs 60-185 issue cycles depending on what else its slot does, and a load slot that outruns
// the other group's 256-cycle MFMA slot stalls both: schedule 1 is 4-9 % faster on MI355X (bf16 and MX-fp8,
// 4096^3 / 8192^3, tools/gemm_schedule_ab.py -> profiles/gemm_schedule_ab_mi355x.jsonl; orders 2/2/2/2,
// 0/4/2/2, 0/2/0/6 and DMA between the MFMAs of phase 3 measured in between or below it).
__device__ constexpr int V3_PHASE[2][4] = {{2, 2, 3, 0}, {2, 3, 3, 1}};

// In-kernel stamps of the v3 schedule (a diagnostic build only: -DDIAG_GEMM_STAMPS, tools/gemm_stamps.py).
// Lane 0 of wave 0 (group 0) and wave 4 (group 1) of the first 8 workgroups record s_memtime at four points
// of each phase of the middle K-tile -- load slot start, MFMA slot start, MFMA issue done, slot end -- into a
// buffer of their own that nothing else reads.  The production build compiles the macro to nothing.
#ifdef DIAG_GEMM_STAMPS
__device__ unsigned long long g_gemm_stamps[8][2][4][4];
#define V3_STAMP(p, q)                                                                                   \
  do {                                                                                                 \
    if (kt == KT / 2 && blockIdx.x < 8 && lane == 0 && (wid == 0 || wid == 4))                          \
      g_gemm_stamps[blockIdx.x][wid >> 2][p][q] = __builtin_amdgcn_s_memtime();                         \
  } while (0)
#else
#define V3_STAMP(p, q) \
  do {                 \
  } while (0)
#endif

// DT_BF16: bf16 A[M][K] . Bt[N][K]^T.  DT_FP8 / DT_FP4: MX operands (E4M3 bytes / packed E2M1 pairs,
// unit scales) passed as K = row bytes / 2 "bf16 columns", so the byte-identical LDS-DMA staging is
// shared (a 64-column bf16 K-tile is a 128-byte fp8 or fp4 K-tile); only the swizzle (fp8), the
// fragment reads and the MFMA differ.
// OUT_F32: C is fp32 [M][N].  OUT_BF16_CK (with EPI_LDS): C is bf16 [M][N] -- the output hipBLASLt writes, half
// the bytes -- and csum[M / 128][N] receives every column's sum over each wave row's 128 rows, formed in fp64
// from the fp32 accumulators before the rounding, so the whole-output check (gemm_checksum) needs no second
// pass over C and keeps the accumulators' precision.
enum GemmOut { OUT_F32 = 0, OUT_BF16_CK = 1 };
template <int DT, bool EPI_LDS = false, bool BUF = false, int SCHED = 1, int OUT = OUT_F32,
          bool PRIO_G1 = DT == DT_BF16 || DT == DT_FP8U>
__global__ void __launch_bounds__(V2_THREADS, 1)
gemm_v3_kernel(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt, void* __restrict__ Cv,
               double* __restrict__ csum, int M, int N, int K) {
  static_assert(OUT == OUT_F32 || EPI_LDS, "the bf16 output goes through the LDS-staged epilogue");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
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

  constexpr bool FP8 = DT == DT_FP8 || DT == DT_FP8U;
  const StgBuf rs = stg_buf(Ab, Bb, K);
  auto region = [&](unsigned char* stage, int kt_, int r, int i) {
    if constexpr (BUF) stg_region_buf<FP8>(stage, rs, K, kt_, r, i, wid, lane);
    else stg_region<FP8>(stage, Ab, Bb, K, kt_, r, i, wid, lane);
  };
  auto fill = [&](unsigned char* stage, int kt_) {
    if constexpr (BUF) v2_fill_buf<FP8>(stage, rs, K, kt_, wid, lane);
    else v2_fill<FP8>(stage, Ab, Bb, K, kt_, wid, lane);
  };
  fill(smem, 0);
  if (KT > 1) {
    fill(smem + V2_STAGE_BYTES, 1);
    __builtin_amdgcn_s_waitcnt(0x3f78);  // vmcnt(8): tile 0 landed, tile 1 may be in flight
  } else {
    __builtin_amdgcn_s_waitcnt(0x3f70);  // vmcnt(0)
  }
  STG_BARRIER();
  if (wr == 1) STG_BARRIER();  // the stagger
  // bf16 and fp8 (unscaled MFMA): the second wave group (waves 4-7, one barrier behind) issues at raised priority
  // for the whole loop, so on each SIMD its load slot is not starved behind the other group's MFMA stream (bf16
  // +2-3 % at 4096^3 and 8192^3, profiles/gemm_schedule_ab_mi355x.jsonl; fp8 unscaled +0.7-1.1 %,
  // profiles/gemm_fp8_prio_ab_mi355x.jsonl; neutral-to-negative for the scaled MX form); per-slot priority flips
  // measured below it
  if constexpr (PRIO_G1) {
    if (wr == 1) __builtin_amdgcn_s_setprio(1);
  }

  StgFrags<DT> f;
  for (int kt = 0; kt < KT; ++kt) {
    unsigned char* cur = smem + (kt & 1) * V2_STAGE_BYTES;
    unsigned char* nxt = smem + ((kt + 1) & 1) * V2_STAGE_BYTES;
    const u32x4* a_img = reinterpret_cast<const u32x4*>(cur);
    const u32x4* b_img = reinterpret_cast<const u32x4*>(cur + V2_BM * BK * 2);
    const bool pre = kt + 2 < KT;
    // the phase's restaging (V3_PHASE): R0-R2 of tile kt+2 into this buffer, R3 of tile kt+1 into the other
    // (tile 1 came whole with the prologue)
    auto restage = [&](int phase) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (V3_PHASE[SCHED][r] != phase) continue;
        if (r == 3 ? (kt >= 1 && kt + 1 < KT) : pre) {
          region(r == 3 ? nxt : cur, kt + (r == 3 ? 1 : 2), r, 0);
          region(r == 3 ? nxt : cur, kt + (r == 3 ? 1 : 2), r, 1);
        }
      }
    };
    // phase 0: A(m0), B(n0)
    V3_STAMP(0, 0);
    restage(0);
#pragma unroll
    for (int n = 0; n < 2; ++n) stg_load(f.b0[n], b_img, wc * 64 + n * 16 + frow, fq);
#pragma unroll
    for (int m = 0; m < 4; ++m) stg_load(f.a[m], a_img, wr * 128 + m * 16 + frow, fq);
    STG_BARRIER();
    V3_STAMP(0, 1);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    phase_mfma<DT>(acc, f.a, f.b0, 0, 0);
    V3_STAMP(0, 2);
    STG_BARRIER();
    V3_STAMP(0, 3);
    // phase 1: B(n1)
    V3_STAMP(1, 0);
    restage(1);
#pragma unroll
    for (int n = 0; n < 2; ++n) stg_load(f.b1[n], b_img, wc * 64 + (n + 2) * 16 + frow, fq);
    STG_BARRIER();
    V3_STAMP(1, 1);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    phase_mfma<DT>(acc, f.a, f.b1, 0, 2);
    V3_STAMP(1, 2);
    STG_BARRIER();
    V3_STAMP(1, 3);
    // phase 2: A(m1)
    V3_STAMP(2, 0);
    restage(2);
#pragma unroll
    for (int m = 0; m < 4; ++m) stg_load(f.a[m], a_img, wr * 128 + (m + 4) * 16 + frow, fq);
    STG_BARRIER();
    V3_STAMP(2, 1);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    phase_mfma<DT>(acc, f.a, f.b1, 4, 2);
    V3_STAMP(2, 2);
    STG_BARRIER();
    V3_STAMP(2, 3);
    // phase 3: no LDS reads; retire tile kt+1 (tile kt+2's pieces may stay in flight)
    V3_STAMP(3, 0);
    restage(3);
    if (pre) {
      __builtin_amdgcn_s_waitcnt(0x3f76);  // vmcnt(6)
    } else {
      __builtin_amdgcn_s_waitcnt(0x3f70);  // vmcnt(0)
    }
    STG_BARRIER();
    V3_STAMP(3, 1);
    phase_mfma<DT>(acc, f.a, f.b0, 4, 0);
    V3_STAMP(3, 2);
    STG_BARRIER();
    V3_STAMP(3, 3);
  }
  if (wr == 0) STG_BARRIER();  // balance the stagger
  const int row0 = tm * V2_BM + wr * 128, col0 = tn * V2_BN + wc * 64;
  float* __restrict__ C = static_cast<float*>(Cv);
  if constexpr (OUT == OUT_BF16_CK) {
    // column sums over this wave's 128 rows: 32 per lane (rows m * 16 + fq * 4 + j), then over the 4 lanes
    // (fq) that hold the same column
    double s[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      s[n] = 0.0;
#pragma unroll
      for (int m = 0; m < 8; ++m)
#pragma unroll
        for (int j = 0; j < 4; ++j) s[n] += static_cast<double>(acc[m][n][j]);
      s[n] += __shfl_xor(s[n], 16);
      s[n] += __shfl_xor(s[n], 32);
    }
    if (fq == 0) {
#pragma unroll
      for (int n = 0; n < 4; ++n) csum[static_cast<size_t>(row0 / 128) * N + col0 + n * 16 + frow] = s[n];
    }
    // C through the wave's LDS patch as in the fp32 epilogue, leaving as 8 bf16 (16 bytes) per lane: one
    // store instruction covers 8 rows x 128 contiguous bytes
    constexpr int LD = 64 + 4;
    __builtin_amdgcn_s_barrier();
    float* patch = reinterpret_cast<float*>(smem) + wid * (16 * LD);
    __bf16* __restrict__ Cb = static_cast<__bf16*>(Cv);
#pragma unroll
    for (int m = 0; m < 8; ++m) {
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int j = 0; j < 4; ++j) patch[(fq * 4 + j) * LD + n * 16 + frow] = acc[m][n][j];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int r = q * 8 + (lane >> 3), c8 = (lane & 7) * 8;
        const floatx4 lo = *reinterpret_cast<const floatx4*>(patch + r * LD + c8);
        const floatx4 hi = *reinterpret_cast<const floatx4*>(patch + r * LD + c8 + 4);
        const floatx8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        *reinterpret_cast<bf16x8*>(Cb + static_cast<size_t>(row0 + m * 16 + r) * N + col0 + c8) =
            __builtin_convertvector(v, bf16x8);
      }
    }
  } else if constexpr (EPI_LDS) {
    // Each 16x64 fp32 slice goes through the wave's own LDS patch (no DMA is in flight and every
    // fragment read retired before the last barrier), then leaves as 16-byte row pieces: one store
    // instruction covers 4 rows x 256 contiguous bytes instead of 4 rows x 64.
    constexpr int LD = 64 + 4;
    __builtin_amdgcn_s_barrier();
    float* patch = reinterpret_cast<float*>(smem) + wid * (16 * LD);
#pragma unroll
    for (int m = 0; m < 8; ++m) {
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int j = 0; j < 4; ++j) patch[(fq * 4 + j) * LD + n * 16 + frow] = acc[m][n][j];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = q * 4 + (lane >> 4), c4 = (lane & 15) * 4;
        const floatx4 v = *reinterpret_cast<const floatx4*>(patch + r * LD + c4);
#ifdef DIAG_GEMM_NO_STORE  // lab build (tools/gemm_stamps.py --no-store): everything but the C write itself
        if (N > (1 << 30))
#endif
        *reinterpret_cast<floatx4*>(C + static_cast<size_t>(row0 + m * 16 + r) * N + col0 + c4) = v;
      }
    }
  } else {
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          C[static_cast<size_t>(row0 + m * 16 + fq * 4 + j) * N + col0 + n * 16 + frow] = acc[m][n][j];
  }
}

// ---------------------------------------------------------------------------------------------------------------
// v4 (bf16): hipBLASLt's gfx950 structure -- 256 threads, a 256x256x64 tile, each wave 128x128 (256 accumulator
// AGPRs), 2 LDS stages -- with the loop's instruction order written out.  Every MFMA, fragment ds_read and LDS-DMA
// of the loop is an `asm volatile` statement, so hipcc keeps their interleave and allocates the accumulators to
// AGPRs ("+a") and the fragments to VGPRs once; the lgkmcnt / vmcnt waits are explicit.  Compiler-ordered
// four-wave versions (rounds 2-3) lost to v3 on accumulator shuffling between AGPRs and VGPRs; this one beats it
// (tools/gemm_w4a_lab.hip sweeps the schedule knobs, profiles/gemm_w4a_lab_mi355x.jsonl).
//
// Per K-tile kt (stage s = kt & 1; F0 = k-step 0 fragments of tile kt, already in registers):
//   half 1: 64 MFMA on F0; one ds_read of F1 (tile kt, k-step 1, stage s) after every RS-th of the first 16 * RS;
//           after MFMA X_AT lgkmcnt(0) + s_barrier X (every wave is done with stage s); D1 LDS-DMA pieces of tile
//           kt+2 into stage s spread over the rest
//   half 2: 64 MFMA on F1; after MFMA Y_AT vmcnt(D1) (tile kt+1, issued one K-tile ago, landed) + s_barrier Y;
//           ds_read F0' (tile kt+1, k-step 0, stage s^1) one per R2 MFMAs; the other 16 - D1 DMA pieces spread
//           over the rest; lgkmcnt(0) at the end
// Near the end the DMA re-fetches tile KT-1 into a stage nobody reads any more, and the last iteration's F0' reads
// load harmless stale fragments (branch-free loop); everything is drained before the epilogue.
// The wave's rows are m * 16 + fq * 4 + j (m = 0..7) and the K order is v3's, so C and the fused column sums are
// bit-identical to v3's.
constexpr int V4_THREADS = 256;
typedef int i32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void v4_mfma(floatx4& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
// the first MFMA into an accumulator: C = 0 as an inline constant, so the accumulators need no zeroing.  (Zeroing
// them in C++ let hipcc copy a zero AGPR into the others with v_accvgpr_mov right before the first asm MFMA, a
// sequence that left every accumulator wrong on the MI355X -- the K = 64 path, where no loop separated the two.)
__device__ __forceinline__ void v4_mfma_first(floatx4& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc) : "v"(a), "v"(b));
}

template <int OFF>
__device__ __forceinline__ void v4_read(bf16x8& f, uint32_t addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(f) : "v"(addr), "i"(OFF));
}

// one LDS-DMA wave instruction: 64 lanes x 16 B from rsrc + voff + soff into LDS at m0 + lane * 16, with
// m0 = base + IMM set in the same statement (nothing the compiler schedules in between can see or change it)
template <uint32_t IMM>
__device__ __forceinline__ void v4_dma_imm(uint32_t m0_base, uint32_t voff, const i32x4& rsrc, uint32_t soff) {
  asm volatile("s_add_u32 m0, %0, %1\n\tbuffer_load_dwordx4 %2, %3, %4 offen lds"
               :
               : "s"(m0_base), "i"(IMM), "v"(voff), "s"(rsrc), "s"(soff)
               : "memory");
}

// The grouped form (lab: gemm_v4_kernel<..., M0G = true>): the buffer instruction's immediate offset is added to
// the global address and to the LDS destination, so four DMAs 1 KiB apart in LDS share one m0 -- the group's first
// sets it (SET), the other three carry OFF = 1, 2, 3 KiB (the 12-bit field's reach) and per-row VGPR offsets
// reduced by OFF.  The later ones rely on m0 surviving the MFMA / ds_read statements in between.
template <uint32_t IMM, uint32_t OFF, bool SET>
__device__ __forceinline__ void v4_dma_grouped(uint32_t m0_base, uint32_t voff, const i32x4& rsrc, uint32_t soff) {
  if constexpr (SET) {
    asm volatile("s_add_u32 m0, %0, %1\n\tbuffer_load_dwordx4 %2, %3, %4 offen offset:%5 lds"
                 :
                 : "s"(m0_base), "i"(IMM), "v"(voff), "s"(rsrc), "s"(soff), "i"(OFF)
                 : "memory");
  } else {
    asm volatile("buffer_load_dwordx4 %0, %1, %2 offen offset:%3 lds"
                 :
                 : "v"(voff), "s"(rsrc), "s"(soff), "i"(OFF)
                 : "memory");
  }
}

__device__ __forceinline__ i32x4 v4_rsrc(const void* base, uint32_t bytes) {
  const uint64_t b = reinterpret_cast<uint64_t>(base);
  i32x4 r;
  r.x = static_cast<int>(b);
  r.y = static_cast<int>(b >> 32);
  r.z = static_cast<int>(bytes);
  r.w = 0x00020000;  // raw buffer, 32-bit data format
  return r;
}

struct V4Frags {
  bf16x8 a[8], b[8];
};

// piece p (0-7: A m-block p, 8-15: B n-block p-8) of a k-step's fragments; m-block offsets (2048 B) are immediates
template <int P>
__device__ __forceinline__ void v4_piece(V4Frags& f, uint32_t a_addr, uint32_t b_addr) {
  if constexpr (P < 8) v4_read<P * 2048>(f.a[P], a_addr);
  else v4_read<(P - 8) * 2048>(f.b[P - 8], b_addr);
}

template <int I, int N, typename F>
__device__ __forceinline__ void v4_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    v4_for<I + 1, N>(f);
  }
}

// In-kernel stamps of the v4 loop (a lab build only: -DDIAG_V4_STAMPS, tools/gemm_w4a_lab.hip --stamps).  Every
// wave records s_memtime deltas into a buffer nothing else reads: [0] prologue, [1] K loop, [2] epilogue up to its
// stores' completion, [3] the middle K-tile's iteration, and the time that iteration spent in [4] X (lgkmcnt +
// barrier), [5] Y (vmcnt + barrier), [6] the closing lgkmcnt.  Each stamp pair waits for its own s_memtime, so
// the stamped build runs a little slower than the production one, which compiles all of this out.
#ifdef DIAG_V4_STAMPS
constexpr bool kV4Stamps = true;
__device__ unsigned long long g_v4_stamps[4096][4][8];
#else
constexpr bool kV4Stamps = false;
#endif

// One recursive-halving step of a 16-lane sum: this lane keeps half `bit` of s[0, 2 * H) (the upper half when bit
// is 1) and adds the partner lane's copy of that half; the partner is the DPP permutation CTRL's image, a lane of
// the other `bit`.  Afterwards s[0, H) holds the kept half.
template <int H, int CTRL>
__device__ __forceinline__ void v4_halve(double (&s)[32], int bit) {
#pragma unroll
  for (int i = 0; i < H; ++i) {
    const double keep = bit ? s[i + H] : s[i];
    const double send = bit ? s[i] : s[i + H];
    const uint64_t u = __builtin_bit_cast(uint64_t, send);
    const int lo = __builtin_amdgcn_update_dpp(0, static_cast<int>(u), CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, static_cast<int>(u >> 32), CTRL, 0xf, 0xf, false);
    s[i] = keep + __builtin_bit_cast(double, (static_cast<uint64_t>(static_cast<uint32_t>(hi)) << 32) |
                                                 static_cast<uint32_t>(lo));
  }
}

#include "v4_plan.h"  // the K-loop plans and their compile-time checks (host-compilable, tests/test_gemm_plans.py)

// ---- fp8 (E4M3) form of the v4 kernel: the same tile, waves, staging (a K-tile is 128 bytes, the fp8 swizzle)
// and epilogue; one v_mfma_f32_16x16x128_f8f6f4 (hipBLASLt's fp8 instruction, unscaled) per output block and
// K-tile, so C is v3's fp8 C bit for bit.  A fragment is a lane's 32 contiguous bytes of a row (two 16-byte
// chunks, 8 VGPRs); the 16 fragments of a K-tile take 128 VGPRs, too many to double-buffer beside 256
// accumulators, so -- as hipBLASLt's MT256x256x128 fp8 kernel does -- the K-tile's 64 MFMAs run by quadrant
// (A0-3 x B0-3, A4-7 x B0-3, A0-3 x B4-7, A4-7 x B4-7) and each fragment is reloaded once its quadrants are done:
// this tile's A4-7 / B4-7 at the start of the K-tile, the next tile's B0-3 / A0-3 at its end.
struct V4F8Frags {
  u32x4 alo[8], ahi[8], blo[8], bhi[8];
};

__device__ __forceinline__ void v4_mfma8(floatx4& acc, const u32x4& alo, const u32x4& ahi, const u32x4& blo,
                                         const u32x4& bhi) {
  const i32x8 a = __builtin_bit_cast(i32x8, __builtin_shufflevector(alo, ahi, 0, 1, 2, 3, 4, 5, 6, 7));
  const i32x8 b = __builtin_bit_cast(i32x8, __builtin_shufflevector(blo, bhi, 0, 1, 2, 3, 4, 5, 6, 7));
  asm volatile("v_mfma_f32_16x16x128_f8f6f4 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void v4_mfma8_first(floatx4& acc, const u32x4& alo, const u32x4& ahi, const u32x4& blo,
                                               const u32x4& bhi) {
  const i32x8 a = __builtin_bit_cast(i32x8, __builtin_shufflevector(alo, ahi, 0, 1, 2, 3, 4, 5, 6, 7));
  const i32x8 b = __builtin_bit_cast(i32x8, __builtin_shufflevector(blo, bhi, 0, 1, 2, 3, 4, 5, 6, 7));
  asm volatile("v_mfma_f32_16x16x128_f8f6f4 %0, %1, %2, 0" : "=a"(acc) : "v"(a), "v"(b));
}
template <int OFF>
__device__ __forceinline__ void v4_read4(u32x4& f, uint32_t addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(f) : "v"(addr), "i"(OFF));
}
// fp8 read id r: 0-7 this tile's A blocks 4-7 (block 4 + r / 2, chunk half r % 2), 8-15 its B blocks 4-7, 16-23 the
// next tile's A blocks 0-3, 24-31 its B blocks 0-3.  ha / hb: the per-lane addresses of [half] in the stage read.
template <int R>
__device__ __forceinline__ void v4_piece8(V4F8Frags& g, const uint32_t (&ha)[2], const uint32_t (&hb)[2]) {
  constexpr int q = R & 15, blk = (R < 16 ? 4 : 0) + (q & 7) / 2, h = q & 1;
  constexpr bool is_b = q >= 8;
  if constexpr (!is_b) v4_read4<blk * 2048>(h ? g.ahi[blk] : g.alo[blk], ha[h]);
  else v4_read4<blk * 2048>(h ? g.bhi[blk] : g.blo[blk], hb[h]);
}
template <int OUT = OUT_F32, class PLAN = V4PlanA<1, 20, 8, 8, 2>, int GM = 4, bool TR = false, int DT = DT_BF16,
          bool M0G = false>
__global__ void __launch_bounds__(V4_THREADS, 1)
gemm_v4_kernel(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt, void* __restrict__ Cv,
               double* __restrict__ csum, int M, int N, int K) {
  constexpr bool FP8 = DT == DT_FP8U;
  static_assert(DT == DT_BF16 || DT == DT_FP8U, "v4: bf16 or fp8 (unscaled MFMA)");
  if constexpr (FP8) static_assert(v4f8_plan_ok<PLAN>(), "v4 fp8 plan breaks a read / DMA / barrier ordering rule");
  else static_assert(v4_plan_ok<PLAN>(), "v4 schedule plan breaks a read / DMA / barrier ordering rule");
  static_assert(!M0G || v4_m0_groups_ok<PLAN>(), "grouped m0: each group of 4 DMAs must be issued in order, back to back");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];  // 2 stages x 64 KiB
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: the DMA's m0 is an SGPR
  const int wr = wid >> 1, wc = wid & 1;
  const int tiles_m = M / V2_BM, tiles_n = N / V2_BN, nwg = tiles_m * tiles_n;
  int bid = blockIdx.x;
  {
    const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
  }
  const int group = bid / (GM * tiles_n);
  const int first_m = group * GM;
  const int gsize = min(tiles_m - first_m, GM);
  const int tm = first_m + (bid % (GM * tiles_n)) % gsize;
  const int tn = (bid % (GM * tiles_n)) / gsize;
  const __bf16* Ab = A + static_cast<size_t>(tm) * V2_BM * K;
  const __bf16* Bb = Bt + static_cast<size_t>(tn) * V2_BN * K;
  const int KT = K / BK;

  // LDS-DMA: wave instruction j (0-15) of a tile: operand j >> 3, rows wid * 64 + 8r + 0..7 with r = j & 7 (lane:
  // row + (lane >> 3), physical chunk lane & 7, source chunk XOR-swizzled by row: one VGPR offset per r), LDS
  // address m0 = the wave's base + an immediate per (stage, j), and the tile's column offset kt * 128 as soffset:
  // two instructions per DMA (s_add_u32 m0 + the load), as hipBLASLt issues them.  The K loop is unrolled by two so
  // the stage's addresses are immediates; that and the lean DMA issue were worth +2.5 % at 4096^3 and +4.7 % at
  // 8192^3 over a loop that selected them per K-tile (profiles/gemm_w4a_lab_mi355x.jsonl): with one wave per SIMD
  // every instruction between MFMAs costs issue cycles.
  const i32x4 rs_a = v4_rsrc(Ab, static_cast<uint32_t>(V2_BM) * K * 2);
  const i32x4 rs_b = v4_rsrc(Bb, static_cast<uint32_t>(V2_BN) * K * 2);
  const uint32_t lds0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_void_t*)smem));
  const uint32_t m0_wave = lds0 + wid * 64 * (BK * 2);
  uint32_t voff_r[8];
  {
    const int rsub = lane >> 3, phys = lane & 7;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int row = wid * 64 + 8 * r + rsub;
      voff_r[r] = static_cast<uint32_t>((row * K + (phys ^ swz_row_xor(row, FP8)) * 8) * 2) -
                  (M0G ? static_cast<uint32_t>((r & 3) * 8 * (BK * 2)) : 0u);
    }
  }
  auto dma = [&](auto S, auto J, uint32_t soff) {
    constexpr int s = decltype(S)::value, j = decltype(J)::value, op = j >> 3, r = j & 7;
    if constexpr (M0G)
      v4_dma_grouped<s * V2_STAGE_BYTES + op * (V2_BM * BK * 2) + (r >> 2) * 4 * 8 * (BK * 2), (r & 3) * 8 * (BK * 2),
                     (r & 3) == 0>(m0_wave, voff_r[r], op ? rs_b : rs_a, soff);
    else
      v4_dma_imm<s * V2_STAGE_BYTES + op * (V2_BM * BK * 2) + r * 8 * (BK * 2)>(m0_wave, voff_r[r],
                                                                                  op ? rs_b : rs_a, soff);
  };

  // fragment reads: lane (frow, fq); k-step 1 is chunk ^ 4
  const int frow = lane & 15, fq = lane >> 4, x = (frow >> 1) & 7;
  uint32_t ra[2][2], rb[2][2];  // [stage][k-step]
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const uint32_t c = static_cast<uint32_t>(((fq + 4 * ks) ^ x) * 16);
      ra[s][ks] = lds0 + s * V2_STAGE_BYTES + (wr * 128 + frow) * (BK * 2) + c;
      rb[s][ks] = lds0 + s * V2_STAGE_BYTES + V2_BM * BK * 2 + (wc * 128 + frow) * (BK * 2) + c;
    }

  // fp8: per-lane address of chunk half h (chunk 2 fq + h, swizzled by the row's bits 1 and 3) in each stage
  uint32_t ra8[2][2], rb8[2][2];
  if constexpr (FP8) {
    const int x8 = swz_row_xor(frow, true);
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t c = static_cast<uint32_t>(((2 * fq + h) ^ x8) * 16);
        ra8[st][h] = lds0 + st * V2_STAGE_BYTES + (wr * 128 + frow) * (BK * 2) + c;
        rb8[st][h] = lds0 + st * V2_STAGE_BYTES + V2_BM * BK * 2 + (wc * 128 + frow) * (BK * 2) + c;
      }
  }

  floatx4 acc[8][8];  // written first by the first K-tile's first MFMAs (v4_mfma_first / v4_mfma8_first)

  [[maybe_unused]] uint64_t st_k0 = 0, st_l0 = 0, st_l1 = 0, st_i0 = 0, st_i1 = 0, st_x = 0, st_y = 0, st_e = 0;
  if constexpr (kV4Stamps) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_k0)::"memory");
  // prologue: tiles 0 and 1 into stages 0 and 1, tile 0 waited for, F0 of tile 0 read
  v4_for<0, 16>([&](auto j) { dma(std::integral_constant<int, 0>{}, j, 0u); });
  v4_for<0, 16>([&](auto j) { dma(std::integral_constant<int, 1>{}, j, KT > 1 ? BK * 2u : 0u); });
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  STG_BARRIER();
  [[maybe_unused]] V4Frags f0, f1;
  [[maybe_unused]] V4F8Frags g;
  if constexpr (FP8) v4_for<16, 32>([&](auto r) { v4_piece8<r>(g, ra8[0], rb8[0]); });  // tile 0's A0-3, B0-3
  else v4_for<0, 16>([&](auto p) { v4_piece<p>(f0, ra[0][0], rb[0][0]); });
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if constexpr (kV4Stamps) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_l0)::"memory");

  // one K-tile kt in stage S (= kt & 1)
  auto iter = [&](auto S, auto FIRST, int kt) {
    constexpr int s = decltype(S)::value;
    constexpr bool first = decltype(FIRST)::value;  // K-tile 0: its k-step-0 MFMAs start the accumulators
    [[maybe_unused]] const uint32_t a1 = ra[s][1], b1 = rb[s][1], a0n = ra[s ^ 1][0], b0n = rb[s ^ 1][0];
    const uint32_t soff = static_cast<uint32_t>(min(kt + 2, KT - 1)) * (BK * 2);  // the tile the DMAs fetch
    [[maybe_unused]] const bool stamp = kV4Stamps && kt == KT / 2;
    if constexpr (kV4Stamps) {
      if (kt == KT / 2) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_i0)::"memory");
      if (kt == KT / 2 + 1) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_i1)::"memory");
    }
    v4_for<0, FP8 ? 64 : 128>([&](auto i) {
      constexpr V4Slot o = PLAN::at(i);
      if constexpr (FP8) {
        constexpr int m = v4f8_m(i), n = v4f8_n(i);
        floatx4& c = acc[m][n];
        if constexpr (first) {
          if constexpr (TR) v4_mfma8_first(c, g.blo[n], g.bhi[n], g.alo[m], g.ahi[m]);
          else v4_mfma8_first(c, g.alo[m], g.ahi[m], g.blo[n], g.bhi[n]);
        } else {
          if constexpr (TR) v4_mfma8(c, g.blo[n], g.bhi[n], g.alo[m], g.ahi[m]);
          else v4_mfma8(c, g.alo[m], g.ahi[m], g.blo[n], g.bhi[n]);
        }
        if constexpr (o.read >= 0 && o.read < 16) v4_piece8<o.read>(g, ra8[s], rb8[s]);
        if constexpr (o.read >= 16) v4_piece8<o.read>(g, ra8[s ^ 1], rb8[s ^ 1]);
      } else {
        const V4Frags& f = i < 64 ? f0 : f1;
        floatx4& c = acc[(i & 63) >> 3][i & 7];
        const bf16x8& fa = f.a[(i & 63) >> 3];
        const bf16x8& fb = f.b[i & 7];
        if constexpr (first && i < 64) {
          if constexpr (TR) v4_mfma_first(c, fb, fa);
          else v4_mfma_first(c, fa, fb);
        } else {
          if constexpr (TR) v4_mfma(c, fb, fa);
          else v4_mfma(c, fa, fb);
        }
        if constexpr (o.read >= 0 && o.read < 16) v4_piece<o.read>(f1, a1, b1);
        if constexpr (o.read >= 16) v4_piece<o.read - 16>(f0, a0n, b0n);
      }
      if constexpr (o.wait == 1) {
        if (stamp) {
          uint64_t t0, t1;
          asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier\n\ts_memtime %1\n\ts_waitcnt lgkmcnt(0)"
                       : "=s"(t0), "=s"(t1)::"memory");
          st_x += t1 - t0;
        } else {
          asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        }
      }
      if constexpr (o.wait == 2) {
        if (stamp) {
          uint64_t t0, t1;
          asm volatile("s_memtime %0\n\ts_waitcnt vmcnt(%2)\n\ts_barrier\n\ts_memtime %1\n\ts_waitcnt lgkmcnt(0)"
                       : "=s"(t0), "=s"(t1)
                       : "i"(o.vm)
                       : "memory");
          st_y = t1 - t0;
        } else {
          asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"i"(o.vm) : "memory");
        }
      }
      if constexpr (o.dma >= 0) dma(S, std::integral_constant<int, o.dma>{}, soff);
    });
    if (stamp) {
      uint64_t t0, t1;
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)\n\ts_memtime %1\n\ts_waitcnt lgkmcnt(0)"
                   : "=s"(t0), "=s"(t1)::"memory");
      st_e = t1 - t0;
    } else {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  iter(I0{}, std::true_type{}, 0);
  int kt = 1;
  for (; kt + 1 < KT; kt += 2) {
    iter(I1{}, std::false_type{}, kt);
    iter(I0{}, std::false_type{}, kt + 1);
  }
  if (kt < KT) iter(I1{}, std::false_type{}, kt);
  // drain; the s_nops are the wait states between the last MFMA's result and the epilogue's v_accvgpr_read, which
  // hipcc's hazard recognizer cannot insert for an MFMA written in asm
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if constexpr (kV4Stamps) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_l1)::"memory");
#ifdef DIAG_V4_STAMPS
  // after the epilogue's stores (below) the last stamp; written here by a lambda run at the end
  auto write_stamps = [&] {
    uint64_t t;
    asm volatile("s_waitcnt vmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    if (lane == 0 && blockIdx.x < 4096) {
      unsigned long long* o = g_v4_stamps[blockIdx.x][wid];
      o[0] = st_l0 - st_k0;
      o[1] = st_l1 - st_l0;
      o[2] = t - st_l1;
      o[3] = st_i1 - st_i0;
      o[4] = st_x;
      o[5] = st_y;
      o[6] = st_e;
      o[7] = KT;
    }
  };
#endif

  // The epilogue takes lane / frow / fq afresh from the lane id (v_mbcnt) instead of the values computed for the
  // prologue: those would be live across the K loop, where the 256 accumulators leave no VGPR for them, and the
  // bf16 + column-sum kernels spilled three (fp8: five) to scratch -- the kernel's only scratch use.
  {
  const int lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  const int frow = lane & 15, fq = lane >> 4;
  const int row0 = tm * V2_BM + wr * 128, col0 = tn * V2_BN + wc * 128;
  if constexpr (TR) {
    // Transposed blocks (the B fragment is the MFMA's first operand): lane (frow, fq) of block (m, n) holds row
    // m * 16 + frow, columns n * 16 + 4 * fq + 0..3 -- row pieces, stored straight from registers, no LDS.
    if constexpr (OUT == OUT_BF16_CK) {
      // column sums over the wave's 128 rows: 32 per lane (its 4 columns of 8 blocks) summed over m, then over
      // the 16 lanes holding the same columns by recursive halving (each step keeps half the columns and adds the
      // partner lane's half: 16 + 8 + 4 + 2 exchanged sums); lane frow ends with columns 2 * frow, 2 * frow + 1
      // of its 32 (index c = n * 4 + j)
      double s[32];
#pragma unroll
      for (int c = 0; c < 32; ++c) {
        s[c] = 0.0;
#pragma unroll
        for (int m = 0; m < 8; ++m) s[c] += static_cast<double>(acc[m][c >> 2][c & 3]);
      }
      v4_halve<16, 0x140>(s, (frow >> 3) & 1);  // row_mirror: lane i <-> 15 - i (differs in bit 3)
      v4_halve<8, 0x141>(s, (frow >> 2) & 1);   // row_half_mirror: i <-> 7 - i within 8 (bit 2)
      v4_halve<4, 0x4E>(s, (frow >> 1) & 1);    // quad_perm [2,3,0,1]: xor 2
      v4_halve<2, 0xB1>(s, frow & 1);           // quad_perm [1,0,3,2]: xor 1
      const int c0 = 2 * frow;  // columns n * 16 + 4 * fq + j for c = c0, c0 + 1: adjacent
      double2 v;
      v.x = s[0];
      v.y = s[1];
      *reinterpret_cast<double2*>(csum + static_cast<size_t>(row0 / 128) * N + col0 + (c0 >> 2) * 16 + 4 * fq +
                                  (c0 & 3)) = v;
      // bf16 C: block pair (2p, 2p+1) packed to 2 dwords each, then v_permlane16_swap between the 16-lane rows
      // fq even / odd: even rows end with columns 32p + 4fq + 0..7, odd rows with 32p + 16 + 4(fq - 1) + 0..7
      __bf16* __restrict__ Cb = static_cast<__bf16*>(Cv);
      const int cofs = (fq & 1) * 16 + (fq >> 1) * 8;
#pragma unroll
      for (int m = 0; m < 8; ++m) {
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
          typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
          u32x2 lo = __builtin_bit_cast(u32x2, __builtin_convertvector(acc[m][2 * p], bf16x4));
          u32x2 hi = __builtin_bit_cast(u32x2, __builtin_convertvector(acc[m][2 * p + 1], bf16x4));
          const auto x = __builtin_amdgcn_permlane16_swap(lo.x, hi.x, false, false);
          const auto y = __builtin_amdgcn_permlane16_swap(lo.y, hi.y, false, false);
          const u32x4 out = {x[0], y[0], x[1], y[1]};
          *reinterpret_cast<u32x4*>(Cb + static_cast<size_t>(row0 + m * 16 + frow) * N + col0 + p * 32 + cofs) = out;
        }
      }
    } else {
      float* __restrict__ C = static_cast<float*>(Cv);
#pragma unroll
      for (int m = 0; m < 8; ++m)
#pragma unroll
        for (int n = 0; n < 8; ++n)
          *reinterpret_cast<floatx4*>(C + static_cast<size_t>(row0 + m * 16 + frow) * N + col0 + n * 16 + 4 * fq) =
              acc[m][n];
    }
#ifdef DIAG_V4_STAMPS
    write_stamps();
#endif
    return;
  }
  // epilogue through each wave's own LDS patch (16 rows x 128 columns of fp32), as v3's
  constexpr int LD = 128 + 4;
  float* patch = reinterpret_cast<float*>(smem) + wid * (16 * LD);
  if constexpr (OUT == OUT_BF16_CK) {
    // column sums over the wave's 128 rows in v3's order (m, then j, then the 4 lanes fq holding the column)
    double cs[8];
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      cs[n] = 0.0;
#pragma unroll
      for (int m = 0; m < 8; ++m)
#pragma unroll
        for (int j = 0; j < 4; ++j) cs[n] += static_cast<double>(acc[m][n][j]);
      cs[n] += __shfl_xor(cs[n], 16);
      cs[n] += __shfl_xor(cs[n], 32);
    }
    if (fq == 0) {
#pragma unroll
      for (int n = 0; n < 8; ++n) csum[static_cast<size_t>(row0 / 128) * N + col0 + n * 16 + frow] = cs[n];
    }
    __bf16* __restrict__ Cb = static_cast<__bf16*>(Cv);
#pragma unroll
    for (int m = 0; m < 8; ++m) {
#pragma unroll
      for (int n = 0; n < 8; ++n)
#pragma unroll
        for (int j = 0; j < 4; ++j) patch[(fq * 4 + j) * LD + n * 16 + frow] = acc[m][n][j];
      // 8 bf16 (16 bytes) per lane: one store instruction covers 4 rows x 256 contiguous bytes
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = q * 4 + (lane >> 4), c8 = (lane & 15) * 8;
        const floatx4 lo = *reinterpret_cast<const floatx4*>(patch + r * LD + c8);
        const floatx4 hi = *reinterpret_cast<const floatx4*>(patch + r * LD + c8 + 4);
        const floatx8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        *reinterpret_cast<bf16x8*>(Cb + static_cast<size_t>(row0 + m * 16 + r) * N + col0 + c8) =
            __builtin_convertvector(v, bf16x8);
      }
    }
  } else {
    float* __restrict__ C = static_cast<float*>(Cv);
#pragma unroll
    for (int m = 0; m < 8; ++m) {
#pragma unroll
      for (int n = 0; n < 8; ++n)
#pragma unroll
        for (int j = 0; j < 4; ++j) patch[(fq * 4 + j) * LD + n * 16 + frow] = acc[m][n][j];
      // one store instruction covers 2 rows x 512 contiguous bytes
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int r = q * 2 + (lane >> 5), c4 = (lane & 31) * 4;
        const floatx4 v = *reinterpret_cast<const floatx4*>(patch + r * LD + c4);
        *reinterpret_cast<floatx4*>(C + static_cast<size_t>(row0 + m * 16 + r) * N + col0 + c4) = v;
      }
    }
  }
  }  // the epilogue's scope
#ifdef DIAG_V4_STAMPS
  write_stamps();
#endif
}

// ---------------------------------------------------------------------------
// v4's tail wave.  A grid of 256x256 tiles that is not a whole number of 256-CU waves leaves most of the chip idle in
// its last wave: 6144^3 is 576 tiles, 2.25 waves, so the third wave runs 64 tiles on 64 CUs while 192 wait (6144^3
// bf16 at 0.917 of hipBLASLt against 0.97 at 4096^3 and 8192^3, profiles/gemm_v4_sizes_ab_mi355x.jsonl).  The v4
// launch then covers only the whole waves -- V4_TAIL_MAIN(nwg) workgroups; v4's XCD remap leaves each XCD's last
// chunk of tile indices uncomputed -- and this kernel computes those tiles as four 128x128 quadrants each, 4x the
// workgroups for the same work, with v1's K loop (the same v_mfma_f32_16x16x32_bf16 per 32-wide K chunk, in the same
// order as v3 / v4: every C element and every fp64 column sum bit-identical to theirs).  Each 128x128 quadrant's
// column sums continue, in wave wr = 1, the partial sums wave wr = 0 left in LDS, so they follow v4's own order over
// the 128-row band (m, then j, then the xor-16 / xor-32 lane exchange).
__host__ __device__ constexpr int v4_tail_main(int nwg) { return nwg / 256 * 256; }
// only a short tail is worth it: a quarter wave of 256^2 tiles is one 2-per-CU wave of 128^2 quadrants
__host__ __device__ constexpr bool v4_tail_applies(int nwg) { return nwg > 256 && nwg % 256 != 0 && nwg % 256 <= 64; }

// fp8 (E4M3) form of v1's K-tile for the tail: a K-tile is 128 bytes, one v_mfma_f32_16x16x128_f8f6f4 per block on
// the lane's 32 contiguous bytes (chunks 2fq, 2fq + 1, the fp8 swizzle) -- v3 / v4's fp8 fragments and instruction
__device__ __forceinline__ void tail_compute_fp8(floatx4 (&acc)[4][4], const u32x4 (&buf)[2][TILE_CHUNKS], int wr,
                                                 int wc, int frow, int fq) {
  i32x8 af[4], bfr[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) stg_load(af[m], buf[0], wr * 64 + m * 16 + frow, fq);
#pragma unroll
  for (int n = 0; n < 4; ++n) stg_load(bfr[n], buf[1], wc * 64 + n * 16 + frow, fq);
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n)
      acc[m][n] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[m], bfr[n], acc[m][n], 0, 0, 0, 0, 0, 0);
}

template <int OUT, int GM = 4, int DT = DT_BF16>
__global__ void __launch_bounds__(THREADS, 2)
gemm_v4_tail_kernel(const u32x4* __restrict__ A, const u32x4* __restrict__ Bt, void* __restrict__ Cv,
                    double* __restrict__ csum, int M, int N, int K) {
  static_assert(DT == DT_BF16 || DT == DT_FP8U, "the tail runs v4's dtypes");
  constexpr bool FP8 = DT == DT_FP8U;
  __shared__ u32x4 lds[2][2][TILE_CHUNKS];  // [buffer][A|B][chunk] = 64 KiB
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  // which 256^2 tile (v4's numbering) and which quadrant of it
  const int tiles_m = M / V2_BM, tiles_n = N / V2_BN, nwg = tiles_m * tiles_n;
  const int q = nwg / 8, r = nwg % 8, qmain = v4_tail_main(nwg) / 8;
  int t = static_cast<int>(blockIdx.x) >> 2;
  int idx = -1;
  for (int x = 0; x < 8; ++x) {  // XCD x's tiles are [base, base + cnt); v4 computed the first qmain of them
    const int cnt = q + (x < r ? 1 : 0), base = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
    if (t < cnt - qmain) {
      idx = base + qmain + t;
      break;
    }
    t -= cnt - qmain;
  }
  if (idx < 0) return;  // the launch covers exactly the tail (host side); no workgroup reaches this
  const int group = idx / (GM * tiles_n), first_m = group * GM, gsize = min(tiles_m - first_m, GM);
  const int tm = first_m + (idx % (GM * tiles_n)) % gsize, tn = (idx % (GM * tiles_n)) / gsize;
  const int quad = static_cast<int>(blockIdx.x) & 3;
  const int rm = 2 * tm + (quad >> 1), rn = 2 * tn + (quad & 1);  // the 128x128 tile

  const int kchunks = K / 8;
  const u32x4* Ablk = A + static_cast<size_t>(rm) * BM * kchunks;
  const u32x4* Bblk = Bt + static_cast<size_t>(rn) * BN * kchunks;
  u32x4 ra[LOADS_PER_THREAD], rb[LOADS_PER_THREAD];
  int g_off[LOADS_PER_THREAD], l_off[LOADS_PER_THREAD];
#pragma unroll
  for (int i = 0; i < LOADS_PER_THREAD; ++i) {
    const int ch = tid + i * THREADS;
    const int rr = ch / CHUNKS_PER_ROW, c = ch % CHUNKS_PER_ROW;
    g_off[i] = rr * kchunks + c;
    l_off[i] = FP8 ? swz8(rr, c) : swz(rr, c);
  }
  floatx4 acc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int KT = K / BK;  // K-tiles of 64 bf16 columns = 128 fp8 bytes
  const int frow = lane & 15, fq = lane >> 4;
  auto compute = [&](const u32x4(&buf)[2][TILE_CHUNKS]) {
    if constexpr (FP8) tail_compute_fp8(acc, buf, wr, wc, frow, fq);
    else gemm_compute(acc, buf, wr, wc, frow, fq);
  };
  gemm_gload(ra, rb, Ablk, Bblk, g_off, 0);
  gemm_lstore(lds[0], ra, rb, l_off);
  __syncthreads();
  for (int kt = 0; kt < KT; kt += 2) {
    const bool more1 = kt + 1 < KT;
    if (more1) gemm_gload(ra, rb, Ablk, Bblk, g_off, kt + 1);
    compute(lds[0]);
    if (more1) gemm_lstore(lds[1], ra, rb, l_off);
    __syncthreads();
    if (!more1) break;
    const bool more2 = kt + 2 < KT;
    if (more2) gemm_gload(ra, rb, Ablk, Bblk, g_off, kt + 2);
    compute(lds[1]);
    if (more2) gemm_lstore(lds[0], ra, rb, l_off);
    __syncthreads();
  }
  // every wave is past its last LDS read (the loop ends on a barrier): the operand buffers are free for the epilogue
  const int row0 = rm * BM + wr * 64, col0 = rn * BN + wc * 64;
  unsigned char* scratch = reinterpret_cast<unsigned char*>(&lds[0][0][0]);
  if constexpr (OUT == OUT_BF16_CK) {
    // column sums of the 128-row band rm: wave wr = 0 sums its rows (m, then j) and hands the partials over, wave
    // wr = 1 continues them over its own rows -- v4's wave order over the band's 128 rows -- then the lane exchange
    double* part = reinterpret_cast<double*>(scratch) + wc * (4 * 64);  // [wc][n][lane]
    double cs[4] = {0.0, 0.0, 0.0, 0.0};
    if (wr == 0) {
#pragma unroll
      for (int n = 0; n < 4; ++n) {
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int j = 0; j < 4; ++j) cs[n] += static_cast<double>(acc[m][n][j]);
        part[n * 64 + lane] = cs[n];
      }
    }
    __syncthreads();
    if (wr == 1) {
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        cs[n] = part[n * 64 + lane];
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int j = 0; j < 4; ++j) cs[n] += static_cast<double>(acc[m][n][j]);
        cs[n] += __shfl_xor(cs[n], 16);
        cs[n] += __shfl_xor(cs[n], 32);
      }
      if (fq == 0) {
#pragma unroll
        for (int n = 0; n < 4; ++n) csum[static_cast<size_t>(rm) * N + rn * BN + wc * 64 + n * 16 + frow] = cs[n];
      }
    }
    __syncthreads();  // the partials are read: the scratch becomes the waves' store patches
    // bf16 C through each wave's own patch (16 rows x 64 fp32 columns): 16-byte row pieces per lane
    constexpr int LD = 64 + 4;
    float* patch = reinterpret_cast<float*>(scratch) + wid * (16 * LD);
    __bf16* __restrict__ Cb = static_cast<__bf16*>(Cv);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int j = 0; j < 4; ++j) patch[(fq * 4 + j) * LD + n * 16 + frow] = acc[m][n][j];
      // a wave's writes to its own patch are visible to its own later reads (one wave, in order: s_waitcnt)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int rr = h * 8 + (lane >> 3), c8 = (lane & 7) * 8;
        const floatx4 lo = *reinterpret_cast<const floatx4*>(patch + rr * LD + c8);
        const floatx4 hi = *reinterpret_cast<const floatx4*>(patch + rr * LD + c8 + 4);
        const floatx8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        *reinterpret_cast<bf16x8*>(Cb + static_cast<size_t>(row0 + m * 16 + rr) * N + col0 + c8) =
            __builtin_convertvector(v, bf16x8);
      }
    }
  } else {
    float* __restrict__ C = static_cast<float*>(Cv);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          C[static_cast<size_t>(row0 + m * 16 + fq * 4 + j) * N + col0 + n * 16 + frow] = acc[m][n][j];
  }
}

// fp32 reference for sampled outputs: one thread per (row, col) sample.
__global__ void gemm_ref_kernel(const __bf16* A, const __bf16* Bt, const int* rows, const int* cols, float* out,
                                int nsamp, int K) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nsamp) return;
  const __bf16* a = A + static_cast<size_t>(rows[i]) * K;
  const __bf16* b = Bt + static_cast<size_t>(cols[i]) * K;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += static_cast<float>(a[k]) * static_cast<float>(b[k]);
  out[i] = s;
}

template <typename T>
__global__ void gather_kernel(const T* C, const int* rows, const int* cols, float* out, int nsamp, int N) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nsamp) out[i] = static_cast<float>(C[static_cast<size_t>(rows[i]) * N + cols[i]]);
}

__device__ __forceinline__ uint32_t mix32(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return static_cast<uint32_t>(x);
}

// Deterministic pseudo-random bf16 in [-1, 1).
__global__ void fill_bf16_kernel(__bf16* p, size_t n, uint64_t seed) {
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<size_t>(gridDim.x) * blockDim.x) {
    const uint32_t h = mix32(i * 0x9E3779B97F4A7C15ULL + seed);
    p[i] = static_cast<__bf16>((h >> 8) * (2.0f / 16777216.0f) - 1.0f);
  }
}

// Finite OCP E4M3 bytes (exponent field <= 8, so |x| < 4 and no NaN encoding), hashed from the index.
__global__ void fill_fp8_kernel(uint8_t* p, size_t n, uint64_t seed) {
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n; i += stride) {
    uint64_t h = (i + 1) * 0x9E3779B97F4A7C15ULL ^ seed;
    h ^= h >> 31;
    h *= 0xBF58476D1CE4E5B9ULL;
    h ^= h >> 29;
    const uint32_t e = static_cast<uint32_t>(h % 9), m = static_cast<uint32_t>((h >> 8) & 7), s = (h >> 12) & 1;
    p[i] = static_cast<uint8_t>((s << 7) | (e << 3) | m);
  }
}

__device__ __forceinline__ double e4m3_value(uint8_t b) {
  const int e = (b >> 3) & 15, m = b & 7;
  const double v = e == 0 ? m / 8.0 * 0.015625 : (1.0 + m / 8.0) * ldexp(1.0, e - 7);
  return (b & 0x80) ? -v : v;
}

// fp64 reference of sampled fp8 outputs, plus sum |a*b| (the scale of the MX MFMA's accumulation error)
__global__ void gemm_ref_fp8_kernel(const uint8_t* A, const uint8_t* Bt, const int* rows, const int* cols,
                                    double* out, double* mag, int nsamp, int K) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nsamp) return;
  const uint8_t* a = A + static_cast<size_t>(rows[i]) * K;
  const uint8_t* b = Bt + static_cast<size_t>(cols[i]) * K;
  double acc = 0.0, m = 0.0;
  for (int k = 0; k < K; ++k) {
    const double p = e4m3_value(a[k]) * e4m3_value(b[k]);
    acc += p;
    m += fabs(p);
  }
  out[i] = acc;
  mag[i] = m;
}

// ---------------------------------------------------------------- whole-output GEMM check
// The sampled check above reads 4,096 of the 67 M outputs of an 8192^2 GEMM: a matrix core that corrupts the
// tiles of one workgroup slot is found only if a sample lands there.  Checksums cover every output at the cost
// of one pass over C (Huang & Abraham's algorithm-based fault tolerance): for each tile-high block of rows tb,
// sum_i C[i][j] (i in tb) must equal sum_k (sum_i A[i][k]) Bt[j][k].  Both sides are formed in fp64 from the
// exact operand values, so the only difference is the GEMM's own fp32 rounding, bounded by
// mag[tb][j] = sum_k (sum_i |A[i][k]|) |Bt[j][k]|; a column whose difference exceeds tol * mag marks the tile
// (tb, j / tile width) bad, and the launch's blockIdx -> tile order names the XCD that computed it.
template <int DT>
__device__ __forceinline__ double ck_value(const void* p, size_t i) {
  if constexpr (DT == DT_BF16) return static_cast<double>(static_cast<const __bf16*>(p)[i]);
  else return e4m3_value(static_cast<const uint8_t*>(p)[i]);
}

// asum[tb][k] = sum of the RB rows of block tb in column k, aabs the same over |A|; thread per column (coalesced)
template <int DT>
__global__ void __launch_bounds__(256) ck_asum_kernel(const void* A, double* asum, double* aabs, int K, int RB) {
  const int k = blockIdx.x * 256 + threadIdx.x, tb = blockIdx.y;
  if (k >= K) return;
  double s = 0.0, m = 0.0;
  for (int i = 0; i < RB; ++i) {
    const double v = ck_value<DT>(A, static_cast<size_t>(tb * RB + i) * K + k);
    s += v;
    m += fabs(v);
  }
  asum[static_cast<size_t>(tb) * K + k] = s;
  aabs[static_cast<size_t>(tb) * K + k] = m;
}

// ref[tb][j] = asum[tb] . Bt[j], mag[tb][j] = aabs[tb] . |Bt[j]|: thread per column j, CK_TB row blocks per
// workgroup, Bt staged through LDS 32 k at a time (coalesced along k; the +1 pad keeps the column reads apart)
constexpr int CK_TB = 8, CK_KC = 32;
template <int DT>
__global__ void __launch_bounds__(256) ck_ref_kernel(const void* Bt, const double* asum, const double* aabs,
                                                     double* ref, double* mag, int N, int K, int nblk) {
  __shared__ float bs[256][CK_KC + 1];
  __shared__ double as[CK_TB][CK_KC], am[CK_TB][CK_KC];
  const int tid = threadIdx.x, j0 = blockIdx.x * 256, tb0 = blockIdx.y * CK_TB;
  double r[CK_TB], g[CK_TB];
#pragma unroll
  for (int t = 0; t < CK_TB; ++t) r[t] = g[t] = 0.0;
  for (int k0 = 0; k0 < K; k0 += CK_KC) {
    for (int idx = tid; idx < 256 * CK_KC; idx += 256) {
      const int row = idx / CK_KC, kk = idx % CK_KC;
      bs[row][kk] = j0 + row < N ? static_cast<float>(ck_value<DT>(Bt, static_cast<size_t>(j0 + row) * K + k0 + kk))
                                 : 0.f;
    }
    for (int idx = tid; idx < CK_TB * CK_KC; idx += 256) {
      const int t = idx / CK_KC, kk = idx % CK_KC;
      const bool ok = tb0 + t < nblk;
      as[t][kk] = ok ? asum[static_cast<size_t>(tb0 + t) * K + k0 + kk] : 0.0;
      am[t][kk] = ok ? aabs[static_cast<size_t>(tb0 + t) * K + k0 + kk] : 0.0;
    }
    __syncthreads();
    for (int kk = 0; kk < CK_KC; ++kk) {
      const double b = bs[tid][kk], bb = fabs(b);
#pragma unroll
      for (int t = 0; t < CK_TB; ++t) {
        r[t] += as[t][kk] * b;
        g[t] += am[t][kk] * bb;
      }
    }
    __syncthreads();
  }
  if (j0 + tid >= N) return;
#pragma unroll
  for (int t = 0; t < CK_TB; ++t)
    if (tb0 + t < nblk) {
      ref[static_cast<size_t>(tb0 + t) * N + j0 + tid] = r[t];
      mag[static_cast<size_t>(tb0 + t) * N + j0 + tid] = g[t];
    }
}

// csum[tb][j] = sum of the RB rows of block tb of C in column j, in fp64; thread per column (coalesced)
__global__ void __launch_bounds__(256) ck_csum_kernel(const float* C, double* csum, int N, int RB) {
  const int j = blockIdx.x * 256 + threadIdx.x, tb = blockIdx.y;
  if (j >= N) return;
  double s = 0.0;
  for (int i = 0; i < RB; ++i) s += C[static_cast<size_t>(tb * RB + i) * N + j];
  csum[static_cast<size_t>(tb) * N + j] = s;
}

// ---------------------------------------------------------------- HBM streams
// Forms picked by the sweeps in tools/hbm_explore.hip on MI355X (profiles/hbm_explore_mi355x.json):
// one 16-byte element per thread and a grid over the whole buffer (no grid-stride loop), nontemporal
// loads/stores for copy and read, plain stores for write: copy 6.59, read 6.97, write 6.87 TB/s,
// vs 5.29 / 6.78 / 5.16 for the best persistent form (8-deep unrolled, 32 blocks of 256 per CU).
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) copy_kernel(const f32x4* __restrict__ src, f32x4* __restrict__ dst, size_t n) {
  const size_t i = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i < n) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

__global__ void __launch_bounds__(256) read_kernel(const f32x4* __restrict__ src, size_t n, float* sink) {
  const size_t i = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i < n) {
    const f32x4 v = __builtin_nontemporal_load(src + i);
    if (v[0] + v[3] == 1234.5678f) *sink = v[1];  // keeps the load alive, practically never stores
  }
}

__global__ void __launch_bounds__(256) write_kernel(f32x4* __restrict__ dst, size_t n, float v) {
  const size_t i = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i < n) dst[i] = f32x4{v, v, v, v};
}

// one thread per 16-byte element (grid-stride kernels launched with it run their loop once)
unsigned flat_grid(size_t n) { return static_cast<unsigned>(std::min<size_t>((n + 255) / 256, 0x7FFFFFFFu)); }

// ---------------------------------------------------------------- memtest
__device__ __forceinline__ uint4 pattern(size_t i, uint64_t seed, bool invert) {
  uint4 v;
  v.x = mix32(4 * i + seed);
  v.y = mix32(4 * i + 1 + seed);
  v.z = mix32(4 * i + 2 + seed);
  v.w = mix32(4 * i + 3 + seed);
  if (invert) {
    v.x = ~v.x;
    v.y = ~v.y;
    v.z = ~v.z;
    v.w = ~v.w;
  }
  return v;
}

__global__ void __launch_bounds__(256) mt_write_kernel(uint4* p, size_t n, uint64_t seed, int invert) {
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n; i += stride)
    p[i] = pattern(i, seed, invert != 0);
}

__global__ void __launch_bounds__(256) mt_verify_kernel(const uint4* p, size_t n, uint64_t seed, int invert,
                                                        unsigned long long* errors, unsigned long long* first_bad) {
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n; i += stride) {
    const uint4 v = p[i];
    const uint4 e = pattern(i, seed, invert != 0);
    if (v.x != e.x || v.y != e.y || v.z != e.z || v.w != e.w) {
      atomicAdd(errors, 1ULL);
      atomicMin(first_bad, static_cast<unsigned long long>(i));
    }
  }
}

int grid_for(int device, int blocks_per_cu) {
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) {
    (void)hipGetLastError();
    cus = 256;  // the MI355X's CU count (a grid size only: any value is correct, this one fills the chip)
  }
  return cus * blocks_per_cu;
}

float elapsed_ms(hipEvent_t a, hipEvent_t b) {
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, a, b) != hipSuccess) {
    (void)hipGetLastError();
    return -1.f;  // no time: a negative rate, which every rate check fails, rather than an infinite one
  }
  return ms;
}
// The time between two completed events, for DIAG_CHECK: a failure is reported as the error it is
hipError_t event_ms(hipEvent_t a, hipEvent_t b, float* ms) {
  *ms = 0.f;
  return hipEventElapsedTime(ms, a, b);
}

// ---------------------------------------------------------------------------
// Matrix-core datapath burn-in, one kernel per precision the MI355X computes in (operand lane layouts
// measured by tools/mfma_lab.hip: lane l holds A[l&15][k = (K/4)(l>>4) + e] and B[k][l&15] in element
// e, fp4 low nibble first):
//   0 bf16  v_mfma_f32_16x16x32_bf16          2 MX-fp8 (E4M3)  v_mfma_scale_f32_16x16x128_f8f6f4
//   1 fp8   v_mfma_f32_16x16x128_f8f6f4       3 MX-fp4 (E2M1)  v_mfma_scale_f32_16x16x128_f8f6f4
// Kind 1 is the unscaled f8f6f4 instruction (E4M3, no block scales): what hipBLASLt's fp8 GEMMs issue on gfx950
// (its TensileLibrary_F8F8_*_gfx950.co holds 13,773 of them and 12 of the gfx94x-era v_mfma_f32_16x16x32_fp8_fp8,
// which this kind used to burn; that older datapath ran at the bf16 rate and no production fp8 GEMM depends on
// it).  The builtin with zero scale operands is selected as the unscaled instruction (checked in the ISA).
// Register-resident (no memory traffic), 4 independent accumulators per wave, 2 waves per SIMD on every
// CU.  Operands are {-1, 0, +1}: every product and partial sum is an integer below 2^24, so the fp32
// result is exact and each lane's final sum must equal the host-computed value bit for bit -- a SIMD
// whose matrix core miscomputes is counted, not averaged away.
template <int KIND>
__device__ __forceinline__ floatx4 burn_mfma(const i32x8& a, const i32x8& b, floatx4 c) {
  if constexpr (KIND == 0) {
    bf16x8 av, bv;
    __builtin_memcpy(&av, &a, 16);
    __builtin_memcpy(&bv, &b, 16);
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, c, 0, 0, 0);
  } else if constexpr (KIND == 1) {
    return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 0, 0, 0);  // E4M3, unscaled form
  } else if constexpr (KIND == 2) {
    return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);  // E4M3, scales 2^0
  } else {
    return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 4, 4, 0, 127, 0, 127);  // E2M1, scales 2^0
  }
}

// Physical location of the calling wave: XCD (XCC_ID), shader engine, shader array and CU (HW_ID), packed
// as xcd<<7 | se<<5 | sh<<4 | cu -- one of BURN_SLOTS slots; the CUs of one MI355X occupy 256 of them.
constexpr int BURN_SLOTS = 1024;
__device__ __forceinline__ unsigned wave_slot() {
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);   // HW_ID, all 32 bits
  const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);  // XCC_ID[3:0]
  return ((xcc & 7u) << 7) | (((hw >> 13) & 3u) << 5) | (((hw >> 12) & 1u) << 4) | ((hw >> 8) & 15u);
}

template <int KIND>
__global__ void __launch_bounds__(256) mfma_burn_kernel(const i32x8* __restrict__ fa, const i32x8* __restrict__ fb,
                                                        const float* __restrict__ expect, int iters,
                                                        unsigned long long* errors, unsigned long long* cu_map) {
  const long long t0 = wall_clock64();  // constant-rate clock (hipDeviceAttributeWallClockRate)
  const int lane = threadIdx.x & 63;
  const i32x8 a = fa[lane], b = fb[lane];
  floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      acc0 = burn_mfma<KIND>(a, b, acc0);
      acc1 = burn_mfma<KIND>(b, a, acc1);
      acc2 = burn_mfma<KIND>(a, a, acc2);
      acc3 = burn_mfma<KIND>(b, b, acc3);
    }
  }
  const floatx4 s = acc0 + acc1 + acc2 + acc3;
  const bool bad = s[0] + s[1] + s[2] + s[3] != expect[lane];
  if (bad) atomicAdd(errors, 1ULL);
  if (cu_map != nullptr) {
    // per physical CU: waves run, wrong lanes, summed wave time -- a miscomputing CU is named, and an
    // XCD whose waves take longer than the others' (its own clock domain) stands out
    const unsigned long long nbad = __popcll(__ballot(bad));
    const unsigned long long dt = static_cast<unsigned long long>(wall_clock64() - t0);
    if (lane == 0) {
      unsigned long long* row = cu_map + 3 * wave_slot();
      atomicAdd(row, 1ULL);
      if (nbad) atomicAdd(row + 1, nbad);
      atomicAdd(row + 2, dt);
    }
  }
}

// ---------------------------------------------------------------------------
// LDS test: every workgroup takes the CU's whole LDS (160 KiB on gfx950), writes four patterns over it
// (address hash, its inverse, 0x55.., 0xAA..: every bit at 0 and at 1), and reads each back through a
// different thread than the one that wrote it (half-buffer rotation), so a stuck or coupled bit in any
// bank of any CU is counted -- the register-resident burn-in never touches LDS, and the GEMMs only
// sample their outputs.  Errors are attributed to the physical CU (wave_slot()); `inject_block` >= 0
// corrupts one word of that block's first pattern after the write (the test's own self-check).
__device__ __forceinline__ uint32_t lds_pattern(uint32_t i, uint32_t seed, int p) {
  switch (p & 3) {
    case 0: return mix32(static_cast<uint64_t>(i) * 0x9E3779B97F4A7C15ULL + seed);
    case 1: return ~mix32(static_cast<uint64_t>(i) * 0x9E3779B97F4A7C15ULL + seed);
    case 2: return 0x55555555u;
    default: return 0xAAAAAAAAu;
  }
}

__global__ void __launch_bounds__(1024) lds_test_kernel(uint32_t words, uint32_t seed, int inject_block,
                                                        unsigned long long* errors, unsigned long long* cu_map) {
  extern __shared__ uint32_t lds_words[];
  __shared__ unsigned int block_bad;
  if (threadIdx.x == 0) block_bad = 0;
  unsigned int bad = 0;
  for (int p = 0; p < 4; ++p) {
    for (uint32_t i = threadIdx.x; i < words; i += blockDim.x) lds_words[i] = lds_pattern(i, seed, p);
    __syncthreads();
    if (p == 0 && static_cast<int>(blockIdx.x) == inject_block && threadIdx.x == 0) lds_words[words / 3] ^= 0x10u;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < words; i += blockDim.x) {
      const uint32_t j = i + words / 2 < words ? i + words / 2 : i + words / 2 - words;
      bad += lds_words[j] != lds_pattern(j, seed, p);
    }
    __syncthreads();  // every read of pattern p done before pattern p+1 overwrites it
  }
  if (bad) atomicAdd(&block_bad, bad);
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long* row = cu_map + 2 * wave_slot();
    atomicAdd(row, 1ULL);
    if (block_bad) {
      atomicAdd(row + 1, static_cast<unsigned long long>(block_bad));
      atomicAdd(errors, static_cast<unsigned long long>(block_bad));
    }
  }
}

// ---------------------------------------------------------------------------
// L2 test: each XCD has its own 4 MiB L2.  Every workgroup finds its XCD (XCC_ID) and streams that XCD's
// private slice of the buffer (smaller than the L2) `passes` times, checking every word; after the
// untimed first launch the slice is L2-resident, so the timed launch measures each XCD's L2 read
// bandwidth.  Per-CU map as the burn-in's (waves, wrong words, wave time): an XCD whose L2 has lost
// ways or runs slow falls behind the others; a corrupting path is located to the CU that read it.
__global__ void __launch_bounds__(256) l2_read_kernel(const uint4* __restrict__ buf, uint32_t slice_vec, int passes,
                                                      uint32_t seed, unsigned long long* errors,
                                                      unsigned long long* cu_map) {
  const long long t0 = wall_clock64();
  const unsigned slot = wave_slot();
  const uint32_t base = (slot >> 7) * slice_vec;  // this XCD's slice
  unsigned int bad = 0;
  auto check = [&](const uint4& v, uint32_t i) {
    const uint32_t w = 4u * (base + i);
    return (v.x != (w ^ seed)) + (v.y != ((w + 1u) ^ seed)) + (v.z != ((w + 2u) ^ seed)) + (v.w != ((w + 3u) ^ seed));
  };
  // L2 hits still take hundreds of ns: 8 independent 16-byte loads per lane are issued before any is
  // consumed, so enough bytes are in flight per CU to reach the L2's bandwidth rather than its latency
  constexpr uint32_t U = 8;
  const uint32_t stride = blockDim.x, full = slice_vec - slice_vec % (U * stride);
  for (int p = 0; p < passes; ++p) {
    for (uint32_t i = threadIdx.x; i < full; i += U * stride) {
      uint4 v[U];
#pragma unroll
      for (uint32_t k = 0; k < U; ++k) v[k] = buf[base + i + k * stride];
#pragma unroll
      for (uint32_t k = 0; k < U; ++k) bad += check(v[k], i + k * stride);
    }
    for (uint32_t i = full + threadIdx.x; i < slice_vec; i += stride) bad += check(buf[base + i], i);
  }
  unsigned long long wave_bad = bad;
  for (int off = 32; off > 0; off >>= 1) wave_bad += __shfl_down(wave_bad, off, 64);
  const unsigned long long dt = static_cast<unsigned long long>(wall_clock64() - t0);
  if ((threadIdx.x & 63) == 0) {
    unsigned long long* row = cu_map + 3 * slot;
    atomicAdd(row, 1ULL);
    if (wave_bad) {
      atomicAdd(row + 1, wave_bad);
      atomicAdd(errors, wave_bad);
    }
    atomicAdd(row + 2, dt);
  }
}

// ---------------------------------------------------------------------------
// HBM per XCD: each XCD streams its own slice of a buffer far larger than the L2s and the 256 MiB MALL,
// so every byte comes from HBM through that XCD's path to memory.  The XCD's workgroups share its slice
// through a per-XCD chunk counter (found by XCC_ID, so the mapping of workgroups to XCDs does not matter);
// every word is checked.  All XCDs get the same bytes: on a healthy chip they finish together, and an XCD
// whose fabric path to the memory stacks runs slow falls behind the others (per-CU map as the burn-in's).
// Work queue exit: the counter only grows, so every workgroup leaves once it passes nchunks * passes.
constexpr uint32_t HBM_XCD_CHUNK_VEC = 8192;  // 128 KiB per grab
// only_xcd >= 0: the other XCDs' workgroups leave at once, so that XCD streams alone (its own path's rate,
// without the others contending for the memory stacks).
__global__ void __launch_bounds__(256) hbm_xcd_kernel(const uint4* __restrict__ buf, uint32_t slice_vec, int passes,
                                                      uint32_t seed, int only_xcd, unsigned int* next,
                                                      unsigned long long* errors, unsigned long long* cu_map) {
  __shared__ uint32_t s_chunk;
  const long long t0 = wall_clock64();
  const unsigned slot = wave_slot();
  const unsigned xcd = slot >> 7;
  if (only_xcd >= 0 && static_cast<int>(xcd) != only_xcd) return;
  const uint32_t nchunks = slice_vec / HBM_XCD_CHUNK_VEC;
  const uint32_t total = nchunks * static_cast<uint32_t>(passes);
  unsigned int bad = 0;
  constexpr uint32_t U = 8;
  constexpr uint32_t STEP = U * 256;
  static_assert(HBM_XCD_CHUNK_VEC % STEP == 0, "chunk is a whole number of 8-deep block steps");
  for (;;) {
    if (threadIdx.x == 0) s_chunk = atomicAdd(next + xcd, 1u);
    __syncthreads();
    const uint32_t c = s_chunk;
    __syncthreads();  // everyone has read it before thread 0 overwrites it
    if (c >= total) break;
    const uint32_t base = xcd * slice_vec + (c % nchunks) * HBM_XCD_CHUNK_VEC;
    for (uint32_t i = threadIdx.x; i < HBM_XCD_CHUNK_VEC; i += STEP) {
      u32x4 v[U];
      const u32x4* src = reinterpret_cast<const u32x4*>(buf) + base + i;
#pragma unroll
      for (uint32_t k = 0; k < U; ++k) v[k] = __builtin_nontemporal_load(src + k * 256);
#pragma unroll
      for (uint32_t k = 0; k < U; ++k) {
        const uint32_t w = 4u * (base + i + k * 256);
        bad += (v[k].x != (w ^ seed)) + (v[k].y != ((w + 1u) ^ seed)) + (v[k].z != ((w + 2u) ^ seed)) +
               (v[k].w != ((w + 3u) ^ seed));
      }
    }
  }
  unsigned long long wave_bad = bad;
  for (int off = 32; off > 0; off >>= 1) wave_bad += __shfl_down(wave_bad, off, 64);
  const unsigned long long dt = static_cast<unsigned long long>(wall_clock64() - t0);
  if ((threadIdx.x & 63) == 0) {
    unsigned long long* row = cu_map + 3 * slot;
    atomicAdd(row, 1ULL);
    if (wave_bad) {
      atomicAdd(row + 1, wave_bad);
      atomicAdd(errors, wave_bad);
    }
    atomicAdd(row + 2, dt);
  }
}

__global__ void __launch_bounds__(256) l2_fill_kernel(uint4* buf, uint32_t n_vec, uint32_t seed) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n_vec; i += gridDim.x * blockDim.x) {
    const uint32_t w = 4u * i;
    buf[i] = uint4{w ^ seed, (w + 1u) ^ seed, (w + 2u) ^ seed, (w + 3u) ^ seed};
  }
}

// Device allocation owned by its device (frees with that device current), for the multi-GPU test.
struct DevBuf {
  int device = -1;
  void* ptr = nullptr;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  hipError_t alloc(int dev, size_t bytes) {
    device = dev;
    hipError_t e = hipSetDevice(dev);
    return e != hipSuccess ? e : hipMalloc(&ptr, bytes);
  }
  ~DevBuf() {
    if (ptr) {
      int cur = 0;
      if (hipGetDevice(&cur) == hipSuccess && hipSetDevice(device) == hipSuccess) {
        (void)hipFree(ptr);
        (void)hipSetDevice(cur);
      }
    }
  }
};

// A pair of timing events and an optional stream, released on every return path: the agent calls the
// entry points below for the life of its pod, so an early DIAG_CHECK return must not leak them.
struct Timer {
  hipEvent_t e0 = nullptr, e1 = nullptr;
  hipStream_t stream = nullptr;
  Timer() = default;
  Timer(const Timer&) = delete;
  Timer& operator=(const Timer&) = delete;
  hipError_t create(bool own_stream = false) {
    hipError_t e = hipEventCreate(&e0);
    if (e == hipSuccess) e = hipEventCreate(&e1);
    if (e == hipSuccess && own_stream) e = hipStreamCreateWithFlags(&stream, hipStreamNonBlocking);
    return e;
  }
  ~Timer() {
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

// hipFuncAttributeMaxDynamicSharedMemorySize is a per-device property of a kernel: it is set once for
// every (kernel, device) pair, on the device current to the calling thread, before that pair's first
// launch.  Devices run concurrently (one agent thread per GPU, up to 64 in CPX), hence one once_flag per
// ordinal rather than one process-wide bool.
constexpr int kMaxDevices = 256;
struct LdsAttrOnce {
  std::once_flag once[kMaxDevices];
  hipError_t result[kMaxDevices] = {};
};

int ensure_dynamic_lds(LdsAttrOnce& slot, const void* kernel, int bytes, const char* what) {
  int dev = 0;
  DIAG_CHECK(hipGetDevice(&dev));
  if (dev < 0 || dev >= kMaxDevices) {
    DIAG_CHECK(hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
    return 0;
  }
  std::call_once(slot.once[dev], [&] {
    slot.result[dev] = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  });
  if (slot.result[dev] != hipSuccess) {
    g_err = std::string(what) + ": hipFuncSetAttribute(MaxDynamicSharedMemorySize) on device " +
            std::to_string(dev) + ": " + hipGetErrorString(slot.result[dev]);
    return -1;
  }
  return 0;
}

hipError_t enable_peer(int from, int to) {
  hipError_t e = hipSetDevice(from);
  if (e != hipSuccess) return e;
  e = hipDeviceEnablePeerAccess(to, 0);
  if (e == hipErrorPeerAccessAlreadyEnabled) {
    (void)hipGetLastError();  // sticky-free: clear it
    return hipSuccess;
  }
  return e;
}

template <int DT, bool EPI, bool BUF, int SCHED = 1, int OUT = OUT_F32, bool PRIO = DT == DT_BF16 || DT == DT_FP8U>
int launch_v3_inst(const void* A, const void* Bt, void* C, double* csum, int M, int N, int Kcols,
                   hipStream_t stream) {
  static LdsAttrOnce attr;
  if (ensure_dynamic_lds(attr, reinterpret_cast<const void*>(gemm_v3_kernel<DT, EPI, BUF, SCHED, OUT, PRIO>),
                         2 * V2_STAGE_BYTES, "gemm v3") != 0)
    return -1;
  const int nwg = (M / V2_BM) * (N / V2_BN);
  hipLaunchKernelGGL((gemm_v3_kernel<DT, EPI, BUF, SCHED, OUT, PRIO>), dim3(nwg), dim3(V2_THREADS),
                     2 * V2_STAGE_BYTES, stream, static_cast<const __bf16*>(A), static_cast<const __bf16*>(Bt), C,
                     csum, M, N, Kcols);
  return 0;
}
template <int DT, bool EPI, bool BUF, int SCHED = 1>
int launch_v3_inst(const void* A, const void* Bt, float* C, int M, int N, int Kcols, hipStream_t stream) {
  return launch_v3_inst<DT, EPI, BUF, SCHED, OUT_F32>(A, Bt, C, nullptr, M, N, Kcols, stream);
}

// bf16 C + fused 128-row column sums (OUT_BF16_CK), restaging order per g_gemm_schedule
template <int DT>
int launch_v3_ck(const void* A, const void* Bt, __bf16* C, double* csum, int M, int N, int Kcols,
                 hipStream_t stream) {
  return g_gemm_schedule == 0
             ? launch_v3_inst<DT, true, false, 0, OUT_BF16_CK>(A, Bt, C, csum, M, N, Kcols, stream)
             : launch_v3_inst<DT, true, false, 1, OUT_BF16_CK>(A, Bt, C, csum, M, N, Kcols, stream);
}

// fp8 operands on the MFMA form the thread's knob picks (g_gemm_fp8_unscaled); the unscaled form raises the second
// wave group's priority as the bf16 kernel does
int launch_v3_ck_fp8(const void* A, const void* Bt, __bf16* C, double* csum, int M, int N, int Kcols,
                     hipStream_t stream) {
  return g_gemm_fp8_unscaled ? launch_v3_ck<DT_FP8U>(A, Bt, C, csum, M, N, Kcols, stream)
                             : launch_v3_ck<DT_FP8>(A, Bt, C, csum, M, N, Kcols, stream);
}

// v4 launch (bf16; M, N multiples of 256, K of 64): fp32 C, or bf16 C + fused column sums (OUT_BF16_CK)
template <int OUT, bool TR, int DT>
int launch_v4_inst(const void* A, const void* Bt, void* C, double* csum, int M, int N, int K, hipStream_t stream) {
  using Plan = std::conditional_t<DT == DT_FP8U, V4PlanF8<8, 10, 26, 27, 42>, V4PlanA<1, 20, 8, 8, 2>>;
  constexpr auto kern = gemm_v4_kernel<OUT, Plan, 4, TR, DT>;
  if (static_cast<uint64_t>(V2_BM) * static_cast<uint64_t>(K) * 2 >= (1ull << 32)) {
    // the buffer resources cover a 256-row panel with 32-bit byte offsets
    g_err = "gemm v4: a 256-row operand panel must stay under 4 GiB (K < 8,388,608 bf16 columns)";
    return -2;
  }
  static LdsAttrOnce attr;
  if (ensure_dynamic_lds(attr, reinterpret_cast<const void*>(kern), 2 * V2_STAGE_BYTES, "gemm v4") != 0) return -1;
  const int nwg = (M / V2_BM) * (N / V2_BN);
  // a short last wave: v4 on the whole waves, the rest as 128^2 quadrants (gemm_v4_tail_kernel)
  const bool tail = g_gemm_tail && v4_tail_applies(nwg);
  const int main_wg = tail ? v4_tail_main(nwg) : nwg;
  hipLaunchKernelGGL(kern, dim3(main_wg), dim3(V4_THREADS), 2 * V2_STAGE_BYTES, stream, static_cast<const __bf16*>(A),
                     static_cast<const __bf16*>(Bt), C, csum, M, N, K);
  if (tail)
    hipLaunchKernelGGL((gemm_v4_tail_kernel<OUT, 4, DT>), dim3(4 * (nwg - main_wg)), dim3(THREADS), 0, stream,
                       static_cast<const u32x4*>(A), static_cast<const u32x4*>(Bt), C, csum, M, N, K);
  return 0;
}
// v4 with the LDS-patch epilogue (variant 4) or the transposed, register-direct one (variant 5); K in bf16 columns
// (fp8: row bytes / 2)
template <int OUT, int DT = DT_BF16>
int launch_v4(int variant, const void* A, const void* Bt, void* C, double* csum, int M, int N, int K,
              hipStream_t stream) {
  return variant == 5 ? launch_v4_inst<OUT, true, DT>(A, Bt, C, csum, M, N, K, stream)
                      : launch_v4_inst<OUT, false, DT>(A, Bt, C, csum, M, N, K, stream);
}

// The fp8 kernel the calling thread's knobs select: v4 (4 or 5) for auto / v4 / v4t with the unscaled MFMA, else v3
int fp8_variant() {
  const int v = g_gemm_variant == 0 ? 4 : g_gemm_variant;
  return v >= 4 && g_gemm_fp8_unscaled ? v : 3;
}

// fp8 bf16 C + fused column sums on the selected kernel (Kcols = row bytes / 2)
int launch_fp8_ck(const void* A, const void* Bt, __bf16* C, double* csum, int M, int N, int Kcols,
                  hipStream_t stream) {
  const int v = fp8_variant();
  return v >= 4 ? launch_v4<OUT_BF16_CK, DT_FP8U>(v, A, Bt, C, csum, M, N, Kcols, stream)
                : launch_v3_ck_fp8(A, Bt, C, csum, M, N, Kcols, stream);
}

// The diagnostic runs (diag_gemm_*_x) take the bf16-output kernel wherever the production v3 configuration
// would run (LDS-staged epilogue, global_load_lds staging); other knob settings keep fp32 C.  v4 has one
// configuration, always LDS-staged: it always has the bf16 output.
bool v3_ck_path() { return g_gemm_epilogue == 1 && !g_gemm_buffer_loads; }

// v3 launch (M, N multiples of 256; Kcols = bf16 columns, K8 / 2 for fp8), epilogue per g_gemm_epilogue,
// operand staging per g_gemm_buffer_loads, restaging order per g_gemm_schedule (the buffer path: order 1)
template <int DT>
int launch_v3(const void* A, const void* Bt, float* C, int M, int N, int Kcols, hipStream_t stream) {
  if (g_gemm_buffer_loads)
    return g_gemm_epilogue ? launch_v3_inst<DT, true, true>(A, Bt, C, M, N, Kcols, stream)
                           : launch_v3_inst<DT, false, true>(A, Bt, C, M, N, Kcols, stream);
  if (g_gemm_schedule == 0)
    return g_gemm_epilogue ? launch_v3_inst<DT, true, false, 0>(A, Bt, C, M, N, Kcols, stream)
                           : launch_v3_inst<DT, false, false, 0>(A, Bt, C, M, N, Kcols, stream);
  return g_gemm_epilogue ? launch_v3_inst<DT, true, false, 1>(A, Bt, C, M, N, Kcols, stream)
                         : launch_v3_inst<DT, false, false, 1>(A, Bt, C, M, N, Kcols, stream);
}

// The bf16 kernel diag_gemm_bf16_launch runs for M x N: 1 = v1 (128^2 tiles), 2 = v2, 3 = v3, 4 = v4 (256^2).
// v2-v4 need 256-multiples and enough 256^2 tiles to occupy the 256 CUs (one block per CU); below that the 128^2
// kernel's 4x larger grid wins (measured: 2048^3 v1 543 vs v2 321 TFLOP/s).
int bf16_variant(int M, int N) {
  const bool big_ok = M % V2_BM == 0 && N % V2_BN == 0 && (M / V2_BM) * (N / V2_BN) >= 256;
  return g_gemm_variant == 0 ? (big_ok ? 4 : 1) : g_gemm_variant;
}

// the bf16 launch with bf16 C + fused column sums: v4 when the thread's variant resolves to it, else v3
int launch_bf16_ck(const void* A, const void* Bt, __bf16* C, double* csum, int M, int N, int K, hipStream_t stream) {
  const int v = bf16_variant(M, N);
  return v >= 4 ? launch_v4<OUT_BF16_CK>(v, A, Bt, C, csum, M, N, K, stream)
                : launch_v3_ck<DT_BF16>(A, Bt, C, csum, M, N, K, stream);
}

// diag_gemm_bf16_x writes bf16 C with fused column sums (else fp32 C)
bool bf16_fused(int M, int N) {
  const int v = bf16_variant(M, N);
  return v >= 4 || (v == 3 && v3_ck_path());
}

// Output tiles of a launch and their blockIdx regrouping (the mapping at the top of every GEMM kernel).
struct TileGeom {
  int rows, cols, group_m;
};
constexpr TileGeom kGeomV1{BM, BN, 8}, kGeomV3{V2_BM, V2_BN, 4};

// The XCD that computed each tile: workgroup b is dispatched to XCD b % 8 and computes the tile the regrouping
// gives it.
std::vector<int> tile_xcds(int tiles_m, int tiles_n, int group_m) {
  const int nwg = tiles_m * tiles_n, q = nwg / 8, r = nwg % 8;
  std::vector<int> out(static_cast<size_t>(nwg), -1);
  for (int b = 0; b < nwg; ++b) {
    const int xcd = b % 8;
    const int bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
    const int first_m = bid / (group_m * tiles_n) * group_m;
    const int gsize = std::min(tiles_m - first_m, group_m);
    const int tm = first_m + (bid % (group_m * tiles_n)) % gsize, tn = (bid % (group_m * tiles_n)) / gsize;
    out[static_cast<size_t>(tm) * tiles_n + tn] = xcd;
  }
  return out;
}

// Whole-output check of C = A . Bt^T (the ck_* kernels).  ck_out[0] bad tiles, [1] bad columns, [2..9] bad tiles
// per XCD, [10] / [11] the first bad tile's (row, column) in tiles or -1; *max_err the worst |csum - ref| / mag.
// A NaN or infinite sum counts as bad.
constexpr int kCkOut = 12;
// With `fused` (the OUT_BF16_CK kernel's csum[M / 128][N], device memory) the column sums come from the
// kernel itself, its 128-row halves added per tile row in fp64, and C is not read.
template <int DT>
int gemm_checksum(int device, const void* A, const void* Bt, const float* C, int M, int N, int K, TileGeom g,
                  double tol, double* max_err, long long* ck_out, const double* fused = nullptr) {
  const int rb = g.rows;
  const int nblk = M / rb, tiles_n = N / g.cols;
  const size_t kb = sizeof(double) * static_cast<size_t>(nblk) * K, nb = sizeof(double) * static_cast<size_t>(nblk) * N;
  DevBuf asum, aabs, ref, mag, csum;
  DIAG_CHECK(asum.alloc(device, kb));
  DIAG_CHECK(aabs.alloc(device, kb));
  DIAG_CHECK(ref.alloc(device, nb));
  DIAG_CHECK(mag.alloc(device, nb));
  if (!fused) DIAG_CHECK(csum.alloc(device, nb));
  double* as = static_cast<double*>(asum.ptr);
  double* am = static_cast<double*>(aabs.ptr);
  hipLaunchKernelGGL(ck_asum_kernel<DT>, dim3((K + 255) / 256, nblk), dim3(256), 0, nullptr, A, as, am, K, rb);
  hipLaunchKernelGGL(ck_ref_kernel<DT>, dim3((N + 255) / 256, (nblk + CK_TB - 1) / CK_TB), dim3(256), 0, nullptr, Bt,
                     as, am, static_cast<double*>(ref.ptr), static_cast<double*>(mag.ptr), N, K, nblk);
  if (!fused)
    hipLaunchKernelGGL(ck_csum_kernel, dim3((N + 255) / 256, nblk), dim3(256), 0, nullptr, C,
                       static_cast<double*>(csum.ptr), N, rb);
  DIAG_CHECK(hipGetLastError());
  const size_t cnt = static_cast<size_t>(nblk) * N;
  std::vector<double> hr(cnt), hm(cnt), hc(cnt);
  DIAG_CHECK(hipMemcpy(hr.data(), ref.ptr, nb, hipMemcpyDeviceToHost));
  DIAG_CHECK(hipMemcpy(hm.data(), mag.ptr, nb, hipMemcpyDeviceToHost));
  if (fused) {
    const int halves = rb / 128;
    std::vector<double> h128(cnt * halves);
    DIAG_CHECK(hipMemcpy(h128.data(), fused, nb * halves, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < cnt; ++i) {
      const size_t tb = i / N, j = i % N;
      double v = 0.0;
      for (int h = 0; h < halves; ++h) v += h128[(tb * halves + h) * N + j];
      hc[i] = v;
    }
  } else {
    DIAG_CHECK(hipMemcpy(hc.data(), csum.ptr, nb, hipMemcpyDeviceToHost));
  }
  const std::vector<int> xcd = tile_xcds(nblk, tiles_n, g.group_m);
  std::vector<char> bad(static_cast<size_t>(nblk) * tiles_n, 0);
  double worst = 0.0;
  long long cols = 0;
  for (size_t i = 0; i < cnt; ++i) {
    const double e = std::fabs(hc[i] - hr[i]) / std::max(hm[i], 1e-30);
    if (!(e <= tol)) {  // also NaN
      ++cols;
      const size_t tb = i / N, j = i % N;
      bad[tb * tiles_n + j / g.cols] = 1;
    }
    worst = std::isfinite(e) ? std::max(worst, e) : HUGE_VAL;
  }
  for (int i = 0; i < kCkOut; ++i) ck_out[i] = 0;
  ck_out[1] = cols;
  ck_out[10] = ck_out[11] = -1;
  for (size_t t = 0; t < bad.size(); ++t) {
    if (!bad[t]) continue;
    ++ck_out[0];
    if (xcd[t] >= 0) ++ck_out[2 + xcd[t]];
    if (ck_out[10] < 0) {
      ck_out[10] = static_cast<long long>(t / tiles_n);
      ck_out[11] = static_cast<long long>(t % tiles_n);
    }
  }
  *max_err = worst;
  return 0;
}

// A test hook: overwrite output element `elem` of C with 1e6 (an error every check must see).
hipError_t inject_output(float* C, long long elem, long long count) {
  if (elem < 0 || elem >= count) return hipSuccess;
  const float v = 1e6f;
  return hipMemcpy(C + elem, &v, sizeof(v), hipMemcpyHostToDevice);
}

// The same for the bf16-output kernel: the element becomes 1e6 in C and in its 128-row block's fused column
// sum, as if the matrix core had produced that value.
hipError_t inject_output_ck(__bf16* C, double* csum, long long elem, int M, int N) {
  if (elem < 0 || elem >= static_cast<long long>(M) * N) return hipSuccess;
  __bf16 old;
  hipError_t e = hipMemcpy(&old, C + elem, sizeof(old), hipMemcpyDeviceToHost);
  if (e != hipSuccess) return e;
  const __bf16 v = static_cast<__bf16>(1e6f);
  if ((e = hipMemcpy(C + elem, &v, sizeof(v), hipMemcpyHostToDevice)) != hipSuccess) return e;
  double* cs = csum + (elem / N) / 128 * N + elem % N;
  double sum;
  if ((e = hipMemcpy(&sum, cs, sizeof(sum), hipMemcpyDeviceToHost)) != hipSuccess) return e;
  sum += static_cast<double>(static_cast<float>(v)) - static_cast<double>(static_cast<float>(old));
  return hipMemcpy(cs, &sum, sizeof(sum), hipMemcpyHostToDevice);
}

// |got - ref| beyond the rounding of a bf16 output (at most half an ulp: 2^-8 of |value|, with margin), so the
// sampled checks of the bf16-output kernel keep the tolerances of the fp32 one
// (a NaN stays NaN: std::max would turn it into 0)
inline double beyond_bf16_rounding(double got, double ref) {
  const double e = std::fabs(got - ref) - std::ldexp(std::max(std::fabs(got), std::fabs(ref)), -8) * 1.01;
  return e > 0.0 || std::isnan(e) ? e : 0.0;
}

}  // namespace

// Polled completion with a deadline (diag_p2p_copy_t): a hung copy engine or link must not block the caller.
namespace {
using SteadyClock = std::chrono::steady_clock;
struct PollDeadline {
  double limit_ms;
  SteadyClock::time_point t0 = SteadyClock::now();
  explicit PollDeadline(double ms) : limit_ms(ms) {}
  bool bounded() const { return limit_ms > 0.0; }
  bool passed() const {
    return bounded() && std::chrono::duration<double, std::milli>(SteadyClock::now() - t0).count() >= limit_ms;
  }
};
// hipSuccess once `ev` completed, hipErrorNotReady when the deadline passed first, else the query's error.
hipError_t wait_event_polled(hipEvent_t ev, const PollDeadline& dl) {
  if (!dl.bounded()) return hipEventSynchronize(ev);
  for (;;) {
    hipError_t q = hipEventQuery(ev);
    if (q != hipErrorNotReady) return q;
    if (dl.passed()) return hipErrorNotReady;
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
}
}  // namespace

extern "C" {

const char* diag_last_error(void) { return g_err.c_str(); }

// 0 = auto (bf16: v4 four-wave 256x256 tiles when M, N are multiples of 256 and the grid fills the chip, else
// v1), 1 = force v1 (128x128 register-staged), 2 = force v2, 3 = force v3 (8 waves, staggered), 4 = force v4,
// 5 = v4 with the transposed register-direct epilogue.  fp8: auto / 4 / 5 run v4 on the unscaled MFMA (the MX form,
// fp8_unscaled = 0, and 1-3 run v3); fp4 always runs v3.
void diag_set_gemm_variant(int v) { g_gemm_variant = v; }
void diag_set_gemm_epilogue(int e) { g_gemm_epilogue = e; }
void diag_set_gemm_tail(int t) { g_gemm_tail = t ? 1 : 0; }
int diag_get_gemm_tail(void) { return g_gemm_tail; }
void diag_set_gemm_buffer_loads(int b) { g_gemm_buffer_loads = b; }
void diag_set_gemm_schedule(int s) { g_gemm_schedule = s; }
int diag_get_gemm_schedule(void) { return g_gemm_schedule; }
void diag_set_gemm_fp8_unscaled(int u) { g_gemm_fp8_unscaled = u ? 1 : 0; }
int diag_get_gemm_fp8_unscaled(void) { return g_gemm_fp8_unscaled; }
int diag_get_gemm_variant(void) { return g_gemm_variant; }
int diag_get_gemm_epilogue(void) { return g_gemm_epilogue; }
int diag_get_gemm_buffer_loads(void) { return g_gemm_buffer_loads; }

#ifdef DIAG_GEMM_STAMPS
// the stamps of the last v3 launch (8 x 2 x 4 x 4 64-bit clock values, diagnostic build only)
int diag_gemm_stamps(unsigned long long* out) {
  DIAG_CHECK(hipDeviceSynchronize());
  DIAG_CHECK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_gemm_stamps), sizeof(g_gemm_stamps)));
  return 0;
}
#endif

int diag_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// "arch|name|CUs|bytes|PCI BDF" of a HIP device (arch e.g. "gfx950:sramecc+:xnack-").
int diag_device_arch(int device, char* buf, int len) {
  hipDeviceProp_t prop;
  DIAG_CHECK(hipGetDeviceProperties(&prop, device));
  snprintf(buf, static_cast<size_t>(len), "%s|%s|%d|%zu|%04x:%02x:%02x.0", prop.gcnArchName, prop.name,
           prop.multiProcessorCount, static_cast<size_t>(prop.totalGlobalMem), prop.pciDomainID, prop.pciBusID,
           prop.pciDeviceID);
  return 0;
}

// Raw kernel on caller-owned device pointers (used by the numerics tests with
// torch tensors).  M, N multiples of 128; K multiple of 64.
int diag_gemm_bf16_launch(const void* A, const void* Bt, float* C, int M, int N, int K, void* stream) {
  if (M % BM || N % BN || K % BK || M <= 0 || N <= 0 || K <= 0) {
    g_err = "gemm_bf16: M, N must be multiples of 128 and K a multiple of 64";
    return -2;
  }
  const int variant = bf16_variant(M, N);
  if (variant >= 2 && variant <= 5) {
    if (M % V2_BM || N % V2_BN) {
      g_err = "gemm_bf16 v2-v5: M, N must be multiples of 256";
      return -2;
    }
    if (variant >= 4) {
      const int rc = launch_v4<OUT_F32>(variant, A, Bt, C, nullptr, M, N, K, static_cast<hipStream_t>(stream));
      if (rc != 0) return rc;
    } else if (variant == 2) {
      static LdsAttrOnce attr;
      if (ensure_dynamic_lds(attr, reinterpret_cast<const void*>(gemm_bf16_v2_kernel), 2 * V2_STAGE_BYTES,
                             "gemm v2") != 0)
        return -1;
      const int nwg = (M / V2_BM) * (N / V2_BN);
      hipLaunchKernelGGL(gemm_bf16_v2_kernel, dim3(nwg), dim3(V2_THREADS), 2 * V2_STAGE_BYTES,
                         static_cast<hipStream_t>(stream), static_cast<const __bf16*>(A),
                         static_cast<const __bf16*>(Bt), C, M, N, K);
    } else if (launch_v3<DT_BF16>(A, Bt, C, M, N, K, static_cast<hipStream_t>(stream)) != 0) {
      return -1;
    }
  } else {
    const int nwg = (M / BM) * (N / BN);
    hipLaunchKernelGGL(gemm_bf16_kernel, dim3(nwg), dim3(THREADS), 0, static_cast<hipStream_t>(stream),
                       static_cast<const u32x4*>(A), static_cast<const u32x4*>(Bt), C, M, N, K);
  }
  DIAG_CHECK(hipGetLastError());
  return 0;
}

// MX-fp8 GEMM on caller-owned device pointers: C[M,N] (fp32) = A[M,K] . Bt[N,K]^T with OCP E4M3
// operands (one byte each) and unit block scales.  M, N multiples of 256; K a multiple of 128.
int diag_gemm_fp8_launch(const void* A, const void* Bt, float* C, int M, int N, int K, void* stream) {
  if (M % V2_BM || N % V2_BN || K % 128 || M <= 0 || N <= 0 || K <= 0) {
    g_err = "gemm_fp8: M, N must be multiples of 256 and K a multiple of 128";
    return -2;
  }
  const hipStream_t st = static_cast<hipStream_t>(stream);
  const int v = fp8_variant();
  const int rc = v >= 4 ? launch_v4<OUT_F32, DT_FP8U>(v, A, Bt, C, nullptr, M, N, K / 2, st)
                 : g_gemm_fp8_unscaled ? launch_v3<DT_FP8U>(A, Bt, C, M, N, K / 2, st)
                                       : launch_v3<DT_FP8>(A, Bt, C, M, N, K / 2, st);
  if (rc != 0) return rc;
  DIAG_CHECK(hipGetLastError());
  return 0;
}

// MX-fp4 GEMM: OCP E2M1 operands packed two per byte (element 2i in the low nibble), unit block
// scales, fp32 C.  M, N multiples of 256; K (elements) a multiple of 256.
int diag_gemm_fp4_launch(const void* A, const void* Bt, float* C, int M, int N, int K, void* stream) {
  if (M % V2_BM || N % V2_BN || K % 256 || M <= 0 || N <= 0 || K <= 0) {
    g_err = "gemm_fp4: M, N must be multiples of 256 and K a multiple of 256";
    return -2;
  }
  if (launch_v3<DT_FP4>(A, Bt, C, M, N, K / 4, static_cast<hipStream_t>(stream)) != 0) return -1;
  DIAG_CHECK(hipGetLastError());
  return 0;
}

// The v3 kernel with bf16 output and fused column sums (what the diagnostic runs time and check):
// C[M,N] (bf16) = A . Bt^T, csum[M / 128][N] (fp64) = each column's sum over every 128-row block, formed from
// the fp32 accumulators.  bf16 (dt 0) or MX-fp8 (dt 1) operands; M, N multiples of 256, K of 64 (bf16) or 128.
int diag_gemm_launch_ck(int dt, const void* A, const void* Bt, void* C, double* csum, int M, int N, int K,
                        void* stream) {
  if (M % V2_BM || N % V2_BN || K % (dt == DT_FP8 ? 128 : BK) || M <= 0 || N <= 0 || K <= 0 ||
      (dt != DT_BF16 && dt != DT_FP8)) {
    g_err = "gemm_ck: bf16 or fp8, M, N multiples of 256, K a multiple of 64 (bf16) or 128 (fp8)";
    return -2;
  }
  if (!A || !Bt || !C || !csum) {
    g_err = "gemm_ck: null operand, output or column-sum pointer";
    return -2;
  }
  const hipStream_t st = static_cast<hipStream_t>(stream);
  const int rc = dt == DT_FP8 ? launch_fp8_ck(A, Bt, static_cast<__bf16*>(C), csum, M, N, K / 2, st)
                              : launch_bf16_ck(A, Bt, static_cast<__bf16*>(C), csum, M, N, K, st);
  if (rc != 0) return rc;
  DIAG_CHECK(hipGetLastError());
  return 0;
}

// 1 when diag_gemm_bf16_x (dt 0) / diag_gemm_fp8_x (dt 1) at M x N would time the bf16-output kernel with fused
// column sums under the calling thread's knobs, 0 when it would write fp32 C
int diag_gemm_ck_path(int dt, int M, int N) {
  return (dt == DT_FP8 ? fp8_variant() >= 4 || v3_ck_path() : bf16_fused(M, N)) ? 1 : 0;
}

// Self-contained MFMA burn-in: allocate, fill, run `iters` GEMMs, time them, verify `nsamp` sampled outputs
// against the fp32 reference kernel and, with ck_tol >= 0, every output by tile checksums (gemm_checksum:
// *ck_err, ck_out[kCkOut]).  `inject_elem` >= 0 overwrites that output between the timing and the checks.
int diag_gemm_bf16_x(int device, int M, int N, int K, int warmup, int iters, int nsamp, long long inject_elem,
                     double ck_tol, double* tflops, double* max_rel_err, double* ms_per_iter, double* ck_err,
                     long long* ck_out) {
  if (inject_elem >= static_cast<long long>(M) * N) {
    g_err = "gemm: inject_elem outside the output";
    return -2;
  }
  if (M % BM || N % BN || K % BK) {
    g_err = "gemm_bf16: M, N must be multiples of 128 and K a multiple of 64";
    return -2;
  }
  DIAG_CHECK(hipSetDevice(device));
  // the v4 / v3 kernels write bf16 C and their own column sums (OUT_BF16_CK); the 128^2 v1 kernel fp32 C
  const bool fused = bf16_fused(M, N);
  DevBuf bA, bBt, bC, bref, brows, bcols, bgot, bcs;
  DIAG_CHECK(bA.alloc(device, sizeof(__bf16) * static_cast<size_t>(M) * K));
  DIAG_CHECK(bBt.alloc(device, sizeof(__bf16) * static_cast<size_t>(N) * K));
  DIAG_CHECK(bC.alloc(device, (fused ? sizeof(__bf16) : sizeof(float)) * static_cast<size_t>(M) * N));
  if (fused) DIAG_CHECK(bcs.alloc(device, sizeof(double) * static_cast<size_t>(M / 128) * N));
  double* cs = static_cast<double*>(bcs.ptr);
  auto run = [&]() -> int {
    return fused ? launch_bf16_ck(bA.ptr, bBt.ptr, static_cast<__bf16*>(bC.ptr), cs, M, N, K, nullptr)
                 : diag_gemm_bf16_launch(bA.ptr, bBt.ptr, static_cast<float*>(bC.ptr), M, N, K, nullptr);
  };
  DIAG_CHECK(bref.alloc(device, sizeof(float) * nsamp));
  DIAG_CHECK(brows.alloc(device, sizeof(int) * nsamp));
  DIAG_CHECK(bcols.alloc(device, sizeof(int) * nsamp));
  DIAG_CHECK(bgot.alloc(device, sizeof(float) * nsamp));
  __bf16* A = static_cast<__bf16*>(bA.ptr);
  __bf16* Bt = static_cast<__bf16*>(bBt.ptr);
  float* C = static_cast<float*>(bC.ptr);
  float* ref = static_cast<float*>(bref.ptr);
  int* rows = static_cast<int*>(brows.ptr);
  int* cols = static_cast<int*>(bcols.ptr);
  hipLaunchKernelGGL(fill_bf16_kernel, dim3(2048), dim3(256), 0, nullptr, A, static_cast<size_t>(M) * K, 0x1234ULL);
  hipLaunchKernelGGL(fill_bf16_kernel, dim3(2048), dim3(256), 0, nullptr, Bt, static_cast<size_t>(N) * K, 0xBEEFULL);
  DIAG_CHECK(hipGetLastError());
  std::vector<int> hr(nsamp), hc(nsamp);
  uint64_t x = 0x243F6A8885A308D3ULL;
  for (int i = 0; i < nsamp; ++i) {
    x = x * 6364136223846793005ULL + 1442695040888963407ULL;
    hr[i] = static_cast<int>((x >> 33) % static_cast<uint64_t>(M));
    x = x * 6364136223846793005ULL + 1442695040888963407ULL;
    hc[i] = static_cast<int>((x >> 33) % static_cast<uint64_t>(N));
  }
  DIAG_CHECK(hipMemcpy(rows, hr.data(), sizeof(int) * nsamp, hipMemcpyHostToDevice));
  DIAG_CHECK(hipMemcpy(cols, hc.data(), sizeof(int) * nsamp, hipMemcpyHostToDevice));
  Timer tm;
  DIAG_CHECK(tm.create());
  hipEvent_t e0 = tm.e0, e1 = tm.e1;
  for (int i = 0; i < warmup; ++i)
    if (run()) return -1;
  DIAG_CHECK(hipEventRecord(e0, nullptr));
  for (int i = 0; i < iters; ++i)
    if (run()) return -1;
  DIAG_CHECK(hipEventRecord(e1, nullptr));
  DIAG_CHECK(hipEventSynchronize(e1));
  DIAG_CHECK(hipGetLastError());
  float t_ms = 0.f;
  DIAG_CHECK(event_ms(e0, e1, &t_ms));
  const double ms = t_ms / std::max(iters, 1);
  if (fused) DIAG_CHECK(inject_output_ck(static_cast<__bf16*>(bC.ptr), cs, inject_elem, M, N));
  else DIAG_CHECK(inject_output(C, inject_elem, static_cast<long long>(M) * N));
  hipLaunchKernelGGL(gemm_ref_kernel, dim3((nsamp + 255) / 256), dim3(256), 0, nullptr, A, Bt, rows, cols, ref,
                     nsamp, K);
  DIAG_CHECK(hipGetLastError());
  // gather the sampled outputs on the device: one copy instead of nsamp tiny ones
  float* got = static_cast<float*>(bgot.ptr);
  if (fused)
    hipLaunchKernelGGL(gather_kernel<__bf16>, dim3((nsamp + 255) / 256), dim3(256), 0, nullptr,
                       static_cast<const __bf16*>(bC.ptr), rows, cols, got, nsamp, N);
  else
    hipLaunchKernelGGL(gather_kernel<float>, dim3((nsamp + 255) / 256), dim3(256), 0, nullptr, C, rows, cols, got,
                       nsamp, N);
  DIAG_CHECK(hipGetLastError());
  std::vector<float> href(nsamp), hC(nsamp);
  DIAG_CHECK(hipMemcpy(href.data(), ref, sizeof(float) * nsamp, hipMemcpyDeviceToHost));
  DIAG_CHECK(hipMemcpy(hC.data(), got, sizeof(float) * nsamp, hipMemcpyDeviceToHost));
  double worst = 0.0;
  for (int i = 0; i < nsamp; ++i) {
    const double denom = std::max(1.0, std::fabs(static_cast<double>(href[i])));
    const double d = fused ? beyond_bf16_rounding(hC[i], href[i]) : std::fabs(static_cast<double>(hC[i]) - href[i]);
    worst = std::max(worst, std::isnan(d) ? HUGE_VAL : d / denom);
  }
  *max_rel_err = worst;
  *ms_per_iter = ms;
  *tflops = 2.0 * M * N * static_cast<double>(K) / (ms * 1e-3) / 1e12;
  if (ck_tol >= 0.0) {
    const int v = bf16_variant(M, N);
    return gemm_checksum<DT_BF16>(device, A, Bt, C, M, N, K, v == 1 ? kGeomV1 : kGeomV3, ck_tol, ck_err, ck_out,
                                  fused ? cs : nullptr);
  }
  return 0;
}

int diag_gemm_bf16(int device, int M, int N, int K, int warmup, int iters, int nsamp, double* tflops,
                   double* max_rel_err, double* ms_per_iter) {
  return diag_gemm_bf16_x(device, M, N, K, warmup, iters, nsamp, -1, -1.0, tflops, max_rel_err, ms_per_iter,
                          nullptr, nullptr);
}

// MX-fp8 counterpart of diag_gemm_bf16_x: *max_err = max |C - ref| / sum|a*b| over the samples.
int diag_gemm_fp8_x(int device, int M, int N, int K, int warmup, int iters, int nsamp, long long inject_elem,
                    double ck_tol, double* tflops, double* max_err, double* ms_per_iter, double* ck_err,
                    long long* ck_out) {
  if (inject_elem >= static_cast<long long>(M) * N) {
    g_err = "gemm: inject_elem outside the output";
    return -2;
  }
  if (M % V2_BM || N % V2_BN || K % 128 || nsamp < 1) {
    g_err = "gemm_fp8: M, N must be multiples of 256, K a multiple of 128";
    return -2;
  }
  DIAG_CHECK(hipSetDevice(device));
  const bool fused = fp8_variant() >= 4 || v3_ck_path();  // bf16 C + the kernel's own column sums (OUT_BF16_CK)
  DevBuf A, Bt, C, ref, mag, rows, cols, got, bcs;
  DIAG_CHECK(A.alloc(device, static_cast<size_t>(M) * K));
  DIAG_CHECK(Bt.alloc(device, static_cast<size_t>(N) * K));
  DIAG_CHECK(C.alloc(device, (fused ? sizeof(__bf16) : sizeof(float)) * static_cast<size_t>(M) * N));
  if (fused) DIAG_CHECK(bcs.alloc(device, sizeof(double) * static_cast<size_t>(M / 128) * N));
  double* cs = static_cast<double*>(bcs.ptr);
  auto run = [&]() -> int {
    return fused ? launch_fp8_ck(A.ptr, Bt.ptr, static_cast<__bf16*>(C.ptr), cs, M, N, K / 2, nullptr)
                 : diag_gemm_fp8_launch(A.ptr, Bt.ptr, static_cast<float*>(C.ptr), M, N, K, nullptr);
  };
  DIAG_CHECK(ref.alloc(device, sizeof(double) * nsamp));
  DIAG_CHECK(mag.alloc(device, sizeof(double) * nsamp));
  DIAG_CHECK(rows.alloc(device, sizeof(int) * nsamp));
  DIAG_CHECK(cols.alloc(device, sizeof(int) * nsamp));
  DIAG_CHECK(got.alloc(device, sizeof(float) * nsamp));
  hipLaunchKernelGGL(fill_fp8_kernel, dim3(2048), dim3(256), 0, nullptr, static_cast<uint8_t*>(A.ptr),
                     static_cast<size_t>(M) * K, 0x5151ULL);
  hipLaunchKernelGGL(fill_fp8_kernel, dim3(2048), dim3(256), 0, nullptr, static_cast<uint8_t*>(Bt.ptr),
                     static_cast<size_t>(N) * K, 0xA7A7ULL);
  DIAG_CHECK(hipGetLastError());
  std::vector<int> hr(nsamp), hc(nsamp);
  uint64_t x = 0x13198A2E03707344ULL;
  for (int i = 0; i < nsamp; ++i) {
    x = x * 6364136223846793005ULL + 1442695040888963407ULL;
    hr[i] = static_cast<int>((x >> 33) % static_cast<uint64_t>(M));
    x = x * 6364136223846793005ULL + 1442695040888963407ULL;
    hc[i] = static_cast<int>((x >> 33) % static_cast<uint64_t>(N));
  }
  DIAG_CHECK(hipMemcpy(rows.ptr, hr.data(), sizeof(int) * nsamp, hipMemcpyHostToDevice));
  DIAG_CHECK(hipMemcpy(cols.ptr, hc.data(), sizeof(int) * nsamp, hipMemcpyHostToDevice));
  float* c = static_cast<float*>(C.ptr);
  for (int i = 0; i < warmup; ++i)
    if (run()) return -1;
  Timer tm;
  DIAG_CHECK(tm.create());
  hipEvent_t e0 = tm.e0, e1 = tm.e1;
  DIAG_CHECK(hipEventRecord(e0, nullptr));
  for (int i = 0; i < iters; ++i)
    if (run()) return -1;
  DIAG_CHECK(hipEventRecord(e1, nullptr));
  DIAG_CHECK(hipEventSynchronize(e1));
  DIAG_CHECK(hipGetLastError());
  float t_ms = 0.f;
  DIAG_CHECK(event_ms(e0, e1, &t_ms));
  const double ms = t_ms / std::max(iters, 1);
  if (fused) DIAG_CHECK(inject_output_ck(static_cast<__bf16*>(C.ptr), cs, inject_elem, M, N));
  else DIAG_CHECK(inject_output(c, inject_elem, static_cast<long long>(M) * N));
  const int* r = static_cast<const int*>(rows.ptr);
  const int* cl = static_cast<const int*>(cols.ptr);
  hipLaunchKernelGGL(gemm_ref_fp8_kernel, dim3((nsamp + 255) / 256), dim3(256), 0, nullptr,
                     static_cast<const uint8_t*>(A.ptr), static_cast<const uint8_t*>(Bt.ptr), r, cl,
                     static_cast<double*>(ref.ptr), static_cast<double*>(mag.ptr), nsamp, K);
  if (fused)
    hipLaunchKernelGGL(gather_kernel<__bf16>, dim3((nsamp + 255) / 256), dim3(256), 0, nullptr,
                       static_cast<const __bf16*>(C.ptr), r, cl, static_cast<float*>(got.ptr), nsamp, N);
  else
    hipLaunchKernelGGL(gather_kernel<float>, dim3((nsamp + 255) / 256), dim3(256), 0, nullptr, c, r, cl,
                       static_cast<float*>(got.ptr), nsamp, N);
  DIAG_CHECK(hipGetLastError());
  std::vector<double> href(nsamp), hmag(nsamp);
  std::vector<float> hC(nsamp);
  DIAG_CHECK(hipMemcpy(href.data(), ref.ptr, sizeof(double) * nsamp, hipMemcpyDeviceToHost));
  DIAG_CHECK(hipMemcpy(hmag.data(), mag.ptr, sizeof(double) * nsamp, hipMemcpyDeviceToHost));
  DIAG_CHECK(hipMemcpy(hC.data(), got.ptr, sizeof(float) * nsamp, hipMemcpyDeviceToHost));
  double worst = 0.0;
  for (int i = 0; i < nsamp; ++i) {
    const double d = fused ? beyond_bf16_rounding(hC[i], href[i]) : std::fabs(static_cast<double>(hC[i]) - href[i]);
    worst = std::max(worst, std::isnan(d) ? HUGE_VAL : d / std::max(hmag[i], 1e-30));
  }
  *max_err = worst;
  *ms_per_iter = ms;
  *tflops = 2.0 * M * N * static_cast<double>(K) / (ms * 1e-3) / 1e12;
  if (ck_tol >= 0.0)
    return gemm_checksum<DT_FP8>(device, A.ptr, Bt.ptr, c, M, N, K, kGeomV3, ck_tol, ck_err, ck_out,
                                 fused ? cs : nullptr);
  return 0;
}

int diag_gemm_fp8(int device, int M, int N, int K, int warmup, int iters, int nsamp, double* tflops,
                  double* max_err, double* ms_per_iter) {
  return diag_gemm_fp8_x(device, M, N, K, warmup, iters, nsamp, -1, -1.0, tflops, max_err, ms_per_iter, nullptr,
                         nullptr);
}

// HBM streams over `bytes` per buffer: copy (read+write), read-only, write-only, in TB/s.
int diag_hbm_bandwidth(int device, size_t bytes, int iters, double* copy_tbs, double* read_tbs, double* write_tbs) {
  DIAG_CHECK(hipSetDevice(device));
  const size_t n = bytes / sizeof(f32x4);
  DevBuf ba, bb, bsink;
  DIAG_CHECK(ba.alloc(device, n * sizeof(f32x4)));
  DIAG_CHECK(bb.alloc(device, n * sizeof(f32x4)));
  DIAG_CHECK(bsink.alloc(device, sizeof(float)));
  f32x4* a = static_cast<f32x4*>(ba.ptr);
  f32x4* b = static_cast<f32x4*>(bb.ptr);
  float* sink = static_cast<float*>(bsink.ptr);
  const unsigned grid = flat_grid(n);
  hipLaunchKernelGGL(write_kernel, dim3(grid), dim3(256), 0, nullptr, a, n, 1.0f);
  hipLaunchKernelGGL(write_kernel, dim3(grid), dim3(256), 0, nullptr, b, n, 2.0f);
  DIAG_CHECK(hipGetLastError());
  Timer tm;
  DIAG_CHECK(tm.create());
  hipEvent_t e0 = tm.e0, e1 = tm.e1;
  const size_t nb = n * sizeof(f32x4);
  float t_ms = 0.f;
  // copy
  hipLaunchKernelGGL(copy_kernel, dim3(grid), dim3(256), 0, nullptr, a, b, n);
  DIAG_CHECK(hipEventRecord(e0, nullptr));
  for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(copy_kernel, dim3(grid), dim3(256), 0, nullptr, a, b, n);
  DIAG_CHECK(hipEventRecord(e1, nullptr));
  DIAG_CHECK(hipEventSynchronize(e1));
  DIAG_CHECK(event_ms(e0, e1, &t_ms));
  *copy_tbs = 2.0 * nb * iters / (t_ms * 1e-3) / 1e12;
  // read
  hipLaunchKernelGGL(read_kernel, dim3(grid), dim3(256), 0, nullptr, a, n, sink);
  DIAG_CHECK(hipEventRecord(e0, nullptr));
  for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(read_kernel, dim3(grid), dim3(256), 0, nullptr, a, n, sink);
  DIAG_CHECK(hipEventRecord(e1, nullptr));
  DIAG_CHECK(hipEventSynchronize(e1));
  DIAG_CHECK(event_ms(e0, e1, &t_ms));
  *read_tbs = 1.0 * nb * iters / (t_ms * 1e-3) / 1e12;
  // write
  hipLaunchKernelGGL(write_kernel, dim3(grid), dim3(256), 0, nullptr, b, n, 3.0f);
  DIAG_CHECK(hipEventRecord(e0, nullptr));
  for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(write_kernel, dim3(grid), dim3(256), 0, nullptr, b, n, 3.0f);
  DIAG_CHECK(hipEventRecord(e1, nullptr));
  DIAG_CHECK(hipEventSynchronize(e1));
  DIAG_CHECK(event_ms(e0, e1, &t_ms));
  *write_tbs = 1.0 * nb * iters / (t_ms * 1e-3) / 1e12;
  DIAG_CHECK(hipGetLastError());
  return 0;
}

// Pattern test over `bytes` of HBM; `passes` x (pattern, inverted pattern).
// `inject_word` >= 0: that 16-byte word is overwritten (0xA5 bytes) between the first write and its verify --
// the fault-injection check that a corrupted word is counted and located (diag.memtest(inject_word=...))
int diag_memtest_x(int device, size_t bytes, uint64_t seed, int passes, long long inject_word,
                   unsigned long long* errors, unsigned long long* first_bad_byte, double* gbps) {
  DIAG_CHECK(hipSetDevice(device));
  if (inject_word >= 0 && static_cast<size_t>(inject_word) >= bytes / sizeof(uint4)) {
    g_err = "memtest: inject_word outside the buffer";
    return -2;
  }
  const size_t n = bytes / sizeof(uint4);
  DevBuf bp, bdev;
  DIAG_CHECK(bp.alloc(device, n * sizeof(uint4)));
  DIAG_CHECK(bdev.alloc(device, 2 * sizeof(unsigned long long)));
  uint4* p = static_cast<uint4*>(bp.ptr);
  unsigned long long* dev = static_cast<unsigned long long*>(bdev.ptr);
  const unsigned long long init[2] = {0ULL, ~0ULL};
  DIAG_CHECK(hipMemcpy(dev, init, sizeof init, hipMemcpyHostToDevice));
  const unsigned grid = flat_grid(n);
  Timer tm;
  DIAG_CHECK(tm.create());
  hipEvent_t e0 = tm.e0, e1 = tm.e1;
  DIAG_CHECK(hipEventRecord(e0, nullptr));
  for (int pass = 0; pass < passes; ++pass) {
    for (int inv = 0; inv < 2; ++inv) {
      const uint64_t s = seed + static_cast<uint64_t>(pass) * 0x9E3779B97F4A7C15ULL;
      hipLaunchKernelGGL(mt_write_kernel, dim3(grid), dim3(256), 0, nullptr, p, n, s, inv);
      if (inject_word >= 0 && pass == 0 && inv == 0)
        DIAG_CHECK(hipMemsetAsync(p + inject_word, 0xA5, sizeof(uint4), nullptr));
      hipLaunchKernelGGL(mt_verify_kernel, dim3(grid), dim3(256), 0, nullptr, p, n, s, inv, dev, dev + 1);
    }
  }
  DIAG_CHECK(hipEventRecord(e1, nullptr));
  DIAG_CHECK(hipEventSynchronize(e1));
  DIAG_CHECK(hipGetLastError());
  unsigned long long h[2];
  DIAG_CHECK(hipMemcpy(h, dev, sizeof h, hipMemcpyDeviceToHost));
  *errors = h[0];
  *first_bad_byte = h[0] ? h[1] * sizeof(uint4) : ~0ULL;
  float t_ms = 0.f;
  DIAG_CHECK(event_ms(e0, e1, &t_ms));
  *gbps = 4.0 * passes * static_cast<double>(n * sizeof(uint4)) / (t_ms * 1e-3) / 1e9;
  return 0;
}

int diag_memtest(int device, size_t bytes, uint64_t seed, int passes, unsigned long long* errors,
                 unsigned long long* first_bad_byte, double* gbps) {
  return diag_memtest_x(device, bytes, seed, passes, -1, errors, first_bad_byte, gbps);
}

// xGMI point-to-point check between two GPUs of the node: `iters` copies of `bytes` from `src` to
// `dst` (hipMemcpyPeerAsync on a src-device stream, peer access enabled both ways when the pair
// supports it -- on an MI355X hive every pair is one xGMI hop), timed with events; the received
// buffer is then verified against the address-hash pattern on `dst`.  *peer = 1 if direct peer
// access was available.  A slow pair (a link trained down or retrying) shows up as an outlier
// against the node's other pairs; a corrupting one as errors.
//
// `timeout_ms` > 0 bounds the copies and the verification: the completion events are polled rather than
// waited on, and a pair that has not finished by then returns -4 ("hung") instead of blocking the agent's
// node-level thread forever on a link that stopped making progress.  On that path the buffers, events and
// stream are deliberately leaked: freeing memory an in-flight copy still targets would block (hipFree
// synchronises the device) or let the engine write into a reused allocation.
int diag_p2p_copy_t(int src, int dst, size_t bytes, int iters, double timeout_ms, double* gbps,
                    unsigned long long* errors, int* peer) {
  int n = 0;
  DIAG_CHECK(hipGetDeviceCount(&n));
  if (src < 0 || dst < 0 || src >= n || dst >= n || src == dst || iters < 1 || bytes < 16) {
    g_err = "p2p: need two distinct devices, iters >= 1, bytes >= 16";
    return -2;
  }
  int cur = 0;
  DIAG_CHECK(hipGetDevice(&cur));
  int can_sd = 0, can_ds = 0;
  DIAG_CHECK(hipDeviceCanAccessPeer(&can_sd, src, dst));
  DIAG_CHECK(hipDeviceCanAccessPeer(&can_ds, dst, src));
  *peer = can_sd && can_ds;
  if (*peer) {
    DIAG_CHECK(enable_peer(src, dst));
    DIAG_CHECK(enable_peer(dst, src));
  }
  const size_t nvec = bytes / sizeof(uint4);
  const size_t nbytes = nvec * sizeof(uint4);
  DevBuf a, b, cnt;
  DIAG_CHECK(a.alloc(src, nbytes));
  DIAG_CHECK(b.alloc(dst, nbytes));
  DIAG_CHECK(cnt.alloc(dst, 2 * sizeof(unsigned long long)));
  const uint64_t seed = 0xC0FFEEULL + static_cast<uint64_t>(src) * 131 + static_cast<uint64_t>(dst);
  // pattern on src, junk on dst
  DIAG_CHECK(hipSetDevice(src));
  hipLaunchKernelGGL(mt_write_kernel, dim3(grid_for(src, 4)), dim3(256), 0, nullptr, static_cast<uint4*>(a.ptr), nvec,
                     seed, 0);
  DIAG_CHECK(hipGetLastError());
  DIAG_CHECK(hipDeviceSynchronize());
  DIAG_CHECK(hipSetDevice(dst));
  DIAG_CHECK(hipMemset(b.ptr, 0xA5, nbytes));
  const unsigned long long init[2] = {0ULL, ~0ULL};
  DIAG_CHECK(hipMemcpy(cnt.ptr, init, sizeof init, hipMemcpyHostToDevice));
  DIAG_CHECK(hipDeviceSynchronize());
  // timed copies on a stream of the source device
  DIAG_CHECK(hipSetDevice(src));
  Timer tm;
  DIAG_CHECK(tm.create(true));
  hipEvent_t e0 = tm.e0, e1 = tm.e1;
  hipStream_t st = tm.stream;
  DIAG_CHECK(hipMemcpyPeerAsync(b.ptr, dst, a.ptr, src, nbytes, st));  // warm-up (maps, engine)
  DIAG_CHECK(hipEventRecord(e0, st));
  for (int i = 0; i < iters; ++i) DIAG_CHECK(hipMemcpyPeerAsync(b.ptr, dst, a.ptr, src, nbytes, st));
  DIAG_CHECK(hipEventRecord(e1, st));
  const PollDeadline dl(timeout_ms);
  Timer tv;  // the verification's completion event lives on `dst`
  auto hung = [&](const char* stage) {
    a.ptr = b.ptr = cnt.ptr = nullptr;
    tm.e0 = tm.e1 = tv.e0 = tv.e1 = nullptr;
    tm.stream = nullptr;
    (void)hipSetDevice(cur);
    char msg[192];
    std::snprintf(msg, sizeof msg, "p2p %d->%d: %s did not complete within %.0f ms (xGMI link or engine hung)", src,
                  dst, stage, timeout_ms);
    g_err = msg;
    return -4;
  };
  hipError_t w = wait_event_polled(e1, dl);
  if (w == hipErrorNotReady) return hung("copies");
  DIAG_CHECK(w);
  float ms = 0.f;
  DIAG_CHECK(event_ms(e0, e1, &ms));
  *gbps = ms > 0.f ? static_cast<double>(iters) * static_cast<double>(nbytes) / (ms * 1e-3) / 1e9 : 0.0;
  // verify what arrived
  DIAG_CHECK(hipSetDevice(dst));
  DIAG_CHECK(tv.create(false));
  unsigned long long* c = static_cast<unsigned long long*>(cnt.ptr);
  hipLaunchKernelGGL(mt_verify_kernel, dim3(grid_for(dst, 4)), dim3(256), 0, nullptr,
                     static_cast<const uint4*>(b.ptr), nvec, seed, 0, c, c + 1);
  DIAG_CHECK(hipGetLastError());
  DIAG_CHECK(hipEventRecord(tv.e0, nullptr));
  w = wait_event_polled(tv.e0, dl);
  if (w == hipErrorNotReady) return hung("verification");
  DIAG_CHECK(w);
  unsigned long long h[2];
  DIAG_CHECK(hipMemcpy(h, cnt.ptr, sizeof h, hipMemcpyDeviceToHost));
  *errors = h[0];
  DIAG_CHECK(hipSetDevice(cur));
  return 0;
}

// Self-test of the polled deadline the pair copies wait with (wait_event_polled), on one GPU: queue `launches`
// full-buffer writes of 1 GiB (finite work, ~0.15 ms each on MI355X) on a stream of their own, wait for them
// with a `deadline_ms` deadline -- *timed_out = 1 when the deadline passed first, *waited_ms how long that
// took -- then drain the stream (*drained_ms) before freeing, so nothing is left running.  The hung-pair path
// of diag_p2p_copy_t cannot be provoked on a healthy node; this shows the same wait returning at its deadline.
int diag_poll_selftest(int device, int launches, double deadline_ms, int* timed_out, double* waited_ms,
                       double* drained_ms) {
  if (launches < 1 || launches > 100000 || deadline_ms <= 0.0) {
    g_err = "poll selftest: launches in [1, 100000] and a positive deadline";
    return -2;
  }
  int cur = 0;
  DIAG_CHECK(hipGetDevice(&cur));
  constexpr size_t bytes = size_t(1) << 30;
  DevBuf buf;
  DIAG_CHECK(buf.alloc(device, bytes));
  Timer tm;
  DIAG_CHECK(tm.create(true));
  const size_t n = bytes / sizeof(f32x4);
  for (int i = 0; i < launches; ++i)
    hipLaunchKernelGGL(write_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, tm.stream,
                       static_cast<f32x4*>(buf.ptr), n, 1.0f);
  DIAG_CHECK(hipGetLastError());
  DIAG_CHECK(hipEventRecord(tm.e1, tm.stream));
  const auto t0 = SteadyClock::now();
  const hipError_t w = wait_event_polled(tm.e1, PollDeadline(deadline_ms));
  const auto t1 = SteadyClock::now();
  *timed_out = w == hipErrorNotReady;
  *waited_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
  const hipError_t d = hipEventSynchronize(tm.e1);  // finite work: drain before the buffer is freed
  *drained_ms = std::chrono::duration<double, std::milli>(SteadyClock::now() - t1).count();
  if (w != hipSuccess && w != hipErrorNotReady) DIAG_CHECK(w);
  DIAG_CHECK(d);
  DIAG_CHECK(hipSetDevice(cur));
  return 0;
}

int diag_p2p_copy(int src, int dst, size_t bytes, int iters, double* gbps, unsigned long long* errors, int* peer) {
  return diag_p2p_copy_t(src, dst, bytes, iters, 0.0, gbps, errors, peer);
}

// The "fan" pass of the xGMI check: `src` copies to all `ndst` peers at once, so every one of its links carries
// traffic together (the pair pass loads one link at a time; a link that holds up alone but not under load -- a
// marginal lane retraining, an engine shared with another link -- only shows here).  One source buffer with the
// address-hash pattern, one destination buffer per peer, one non-blocking stream per peer on `src`; every stream
// waits on a common start event, runs `iters` hipMemcpyPeerAsync of `bytes` and records its own end, so
// gbps[i] = the rate peer i saw while all were running and *total_gbps = all bytes over the slowest stream's end.
// Each destination is then verified against the pattern (errors[i]); peer[i] = direct peer access both ways.
// `timeout_ms` > 0 bounds copies and verification as in diag_p2p_copy_t (-4 "hung", resources leaked on purpose).
int diag_p2p_fan_t(int src, const int* dsts, int ndst, size_t bytes, int iters, double timeout_ms, double* gbps,
                   unsigned long long* errors, int* peer, double* total_gbps) {
  constexpr int kMaxFan = 64;  // a CPX hive: 63 peers
  int n = 0;
  DIAG_CHECK(hipGetDeviceCount(&n));
  if (src < 0 || src >= n || ndst < 1 || ndst > kMaxFan || iters < 1 || bytes < 16) {
    g_err = "p2p fan: need a valid source, 1..64 peers, iters >= 1, bytes >= 16";
    return -2;
  }
  for (int i = 0; i < ndst; ++i) {
    if (dsts[i] < 0 || dsts[i] >= n || dsts[i] == src) {
      g_err = "p2p fan: every peer must be a device other than the source";
      return -2;
    }
    for (int j = 0; j < i; ++j)
      if (dsts[j] == dsts[i]) {
        g_err = "p2p fan: a peer is listed twice";
        return -2;
      }
  }
  int cur = 0;
  DIAG_CHECK(hipGetDevice(&cur));
  for (int i = 0; i < ndst; ++i) {
    int sd = 0, ds = 0;
    DIAG_CHECK(hipDeviceCanAccessPeer(&sd, src, dsts[i]));
    DIAG_CHECK(hipDeviceCanAccessPeer(&ds, dsts[i], src));
    peer[i] = sd && ds;
    if (peer[i]) {
      DIAG_CHECK(enable_peer(src, dsts[i]));
      DIAG_CHECK(enable_peer(dsts[i], src));
    }
    errors[i] = 0;
    gbps[i] = 0.0;
  }
  *total_gbps = 0.0;
  const size_t nvec = bytes / sizeof(uint4);
  const size_t nbytes = nvec * sizeof(uint4);
  const uint64_t seed = 0xFA17ULL + static_cast<uint64_t>(src) * 131;
  DevBuf a;
  DevBuf b[kMaxFan], cnt[kMaxFan];
  DIAG_CHECK(a.alloc(src, nbytes));
  DIAG_CHECK(hipSetDevice(src));
  hipLaunchKernelGGL(mt_write_kernel, dim3(grid_for(src, 4)), dim3(256), 0, nullptr, static_cast<uint4*>(a.ptr), nvec,
                     seed, 0);
  DIAG_CHECK(hipGetLastError());
  DIAG_CHECK(hipDeviceSynchronize());
  const unsigned long long init[2] = {0ULL, ~0ULL};
  for (int i = 0; i < ndst; ++i) {
    DIAG_CHECK(b[i].alloc(dsts[i], nbytes));
    DIAG_CHECK(cnt[i].alloc(dsts[i], sizeof init));
    DIAG_CHECK(hipMemset(b[i].ptr, 0xA5, nbytes));
    DIAG_CHECK(hipMemcpy(cnt[i].ptr, init, sizeof init, hipMemcpyHostToDevice));
    DIAG_CHECK(hipDeviceSynchronize());
  }
  // streams and events on the source device: a head stream records the common start, each peer's stream waits
  // on it, then copies (after one untimed warm-up copy per peer, mapping the pages and waking the engines)
  DIAG_CHECK(hipSetDevice(src));
  Timer head;
  DIAG_CHECK(head.create(true));
  Timer per[kMaxFan];
  for (int i = 0; i < ndst; ++i) {
    DIAG_CHECK(per[i].create(true));
    DIAG_CHECK(hipMemcpyPeerAsync(b[i].ptr, dsts[i], a.ptr, src, nbytes, per[i].stream));
    DIAG_CHECK(hipEventRecord(per[i].e0, per[i].stream));
  }
  for (int i = 0; i < ndst; ++i) DIAG_CHECK(hipStreamWaitEvent(head.stream, per[i].e0, 0));  // warm-ups done
  DIAG_CHECK(hipEventRecord(head.e0, head.stream));
  for (int i = 0; i < ndst; ++i) {
    DIAG_CHECK(hipStreamWaitEvent(per[i].stream, head.e0, 0));
    for (int it = 0; it < iters; ++it) DIAG_CHECK(hipMemcpyPeerAsync(b[i].ptr, dsts[i], a.ptr, src, nbytes, per[i].stream));
    DIAG_CHECK(hipEventRecord(per[i].e1, per[i].stream));
  }
  const PollDeadline dl(timeout_ms);
  Timer verify[kMaxFan];
  auto hung = [&](int i, const char* stage) {
    // in-flight copies may still target these buffers: leak everything rather than free under them
    a.ptr = nullptr;
    for (int j = 0; j < ndst; ++j) {
      b[j].ptr = cnt[j].ptr = nullptr;
      per[j].e0 = per[j].e1 = nullptr;
      per[j].stream = nullptr;
      verify[j].e0 = verify[j].e1 = nullptr;
    }
    head.e0 = head.e1 = nullptr;
    head.stream = nullptr;
    (void)hipSetDevice(cur);
    char msg[192];
    std::snprintf(msg, sizeof msg, "p2p fan %d->%d: %s did not complete within %.0f ms (xGMI link or engine hung)",
                  src, dsts[i], stage, timeout_ms);
    g_err = msg;
    return -4;
  };
  float slowest = 0.f;
  for (int i = 0; i < ndst; ++i) {
    hipError_t w = wait_event_polled(per[i].e1, dl);
    if (w == hipErrorNotReady) return hung(i, "copies");
    DIAG_CHECK(w);
    float ms = 0.f;
    DIAG_CHECK(event_ms(head.e0, per[i].e1, &ms));
    gbps[i] = ms > 0.f ? static_cast<double>(iters) * static_cast<double>(nbytes) / (ms * 1e-3) / 1e9 : 0.0;
    slowest = std::max(slowest, ms);
  }
  *total_gbps = slowest > 0.f
                    ? static_cast<double>(ndst) * iters * static_cast<double>(nbytes) / (slowest * 1e-3) / 1e9
                    : 0.0;
  for (int i = 0; i < ndst; ++i) {
    DIAG_CHECK(hipSetDevice(dsts[i]));
    DIAG_CHECK(verify[i].create(false));
    unsigned long long* c = static_cast<unsigned long long*>(cnt[i].ptr);
    hipLaunchKernelGGL(mt_verify_kernel, dim3(grid_for(dsts[i], 4)), dim3(256), 0, nullptr,
                       static_cast<const uint4*>(b[i].ptr), nvec, seed, 0, c, c + 1);
    DIAG_CHECK(hipGetLastError());
    DIAG_CHECK(hipEventRecord(verify[i].e0, nullptr));
  }
  for (int i = 0; i < ndst; ++i) {
    hipError_t w = wait_event_polled(verify[i].e0, dl);
    if (w == hipErrorNotReady) return hung(i, "verification");
    DIAG_CHECK(w);
    unsigned long long h[2];
    DIAG_CHECK(hipSetDevice(dsts[i]));
    DIAG_CHECK(hipMemcpy(h, cnt[i].ptr, sizeof h, hipMemcpyDeviceToHost));
    errors[i] = h[0];
  }
  DIAG_CHECK(hipSetDevice(cur));
  return 0;
}

// Matrix-core burn-in of one precision (`kind` as mfma_burn_kernel): `reps` launches of `iters`
// iterations on every CU; *tflops = dense rate, *errors = wave-lanes whose exact result differed.
int diag_mfma_burn_map(int device, int kind, int iters, int reps, double* tflops, unsigned long long* errors,
                       unsigned long long* cu_map);

int diag_mfma_burn(int device, int kind, int iters, int reps, double* tflops, unsigned long long* errors) {
  return diag_mfma_burn_map(device, kind, iters, reps, tflops, errors, nullptr);
}

int diag_mfma_burn_slots(void) { return BURN_SLOTS; }

// As diag_mfma_burn, plus (cu_map != NULL) a BURN_SLOTS x 3 table of (waves, wrong lanes, wave time in
// wall-clock ticks) per physical CU slot (wave_slot()), over every launch including the warm-up.
int diag_mfma_burn_map(int device, int kind, int iters, int reps, double* tflops, unsigned long long* errors,
                       unsigned long long* cu_map) {
  if (kind < 0 || kind > 3 || iters < 1 || iters > 65536 || reps < 1) {
    g_err = "mfma_burn: kind 0..3, 1 <= iters <= 65536, reps >= 1";
    return -2;
  }
  DIAG_CHECK(hipSetDevice(device));
  static const int kK[4] = {32, 128, 128, 128};
  const int K = kK[kind], per = K / 4;
  // a lane's final sum is bounded by 16 outputs * K * 4 MFMA per accumulator-iteration * iters
  if (16.0 * K * 4 * iters >= 16777216.0) {
    g_err = "mfma_burn: iters too large for an exact fp32 check (< 2048 at K=128, < 8192 at K=32)";
    return -2;
  }
  // operands in {-1, 0, +1}, per lane (the same in every wave, so every wave has the same answer)
  uint64_t st = 0x9E3779B97F4A7C15ULL ^ static_cast<uint64_t>(kind);
  auto rnd3 = [&st]() {
    st ^= st << 13;
    st ^= st >> 7;
    st ^= st << 17;
    return static_cast<int>(st % 3) - 1;
  };
  std::vector<int> va(64 * per), vb(64 * per);
  for (int& x : va) x = rnd3();
  for (int& x : vb) x = rnd3();
  std::vector<uint8_t> fa(64 * 32, 0), fb(64 * 32, 0);
  auto encode = [&](std::vector<uint8_t>& f, const std::vector<int>& v) {
    for (int l = 0; l < 64; ++l)
      for (int e = 0; e < per; ++e) {
        const int x = v[l * per + e];
        if (kind == 0) {
          const uint16_t bits = x == 0 ? 0 : (x > 0 ? 0x3F80 : 0xBF80);
          memcpy(&f[l * 32 + 2 * e], &bits, 2);
        } else if (kind == 3) {
          const uint8_t nib = x == 0 ? 0 : (x > 0 ? 0x2 : 0xA);
          f[l * 32 + e / 2] |= static_cast<uint8_t>(nib << ((e & 1) ? 4 : 0));
        } else {
          f[l * 32 + e] = x == 0 ? 0 : (x > 0 ? 0x38 : 0xB8);
        }
      }
  };
  encode(fa, va);
  encode(fb, vb);
  // host reference: C_xy[i][j] = sum_k x(lane i + 16(k/per), k%per) * y(lane j + 16(k/per), k%per)
  auto prod = [&](const std::vector<int>& x, const std::vector<int>& y, int i, int j) {
    long acc = 0;
    for (int k = 0; k < K; ++k) acc += static_cast<long>(x[(i + 16 * (k / per)) * per + k % per]) *
                                       y[(j + 16 * (k / per)) * per + k % per];
    return acc;
  };
  std::vector<float> expect(64);
  for (int l = 0; l < 64; ++l) {
    long tot = 0;
    for (int r = 0; r < 4; ++r) {
      const int row = 4 * (l >> 4) + r, col = l & 15;
      tot += prod(va, vb, row, col) + prod(vb, va, row, col) + prod(va, va, row, col) + prod(vb, vb, row, col);
    }
    expect[l] = static_cast<float>(tot * 4L * iters);  // exact: bounded below 2^24 by the check above
  }
  DevBuf dfa, dfb, dex, dcnt, dmap;
  const size_t map_bytes = static_cast<size_t>(BURN_SLOTS) * 3 * sizeof(unsigned long long);
  if (cu_map != nullptr) {
    DIAG_CHECK(dmap.alloc(device, map_bytes));
    DIAG_CHECK(hipMemset(dmap.ptr, 0, map_bytes));
  }
  DIAG_CHECK(dfa.alloc(device, fa.size()));
  DIAG_CHECK(dfb.alloc(device, fb.size()));
  DIAG_CHECK(dex.alloc(device, expect.size() * sizeof(float)));
  DIAG_CHECK(dcnt.alloc(device, sizeof(unsigned long long)));
  DIAG_CHECK(hipMemcpy(dfa.ptr, fa.data(), fa.size(), hipMemcpyHostToDevice));
  DIAG_CHECK(hipMemcpy(dfb.ptr, fb.data(), fb.size(), hipMemcpyHostToDevice));
  DIAG_CHECK(hipMemcpy(dex.ptr, expect.data(), expect.size() * sizeof(float), hipMemcpyHostToDevice));
  DIAG_CHECK(hipMemset(dcnt.ptr, 0, sizeof(unsigned long long)));
  const int blocks = grid_for(device, 2);  // 8 waves per CU = 2 per SIMD
  auto launch = [&]() {
    const i32x8* a = static_cast<const i32x8*>(dfa.ptr);
    const i32x8* b = static_cast<const i32x8*>(dfb.ptr);
    const float* ex = static_cast<const float*>(dex.ptr);
    unsigned long long* c = static_cast<unsigned long long*>(dcnt.ptr);
    unsigned long long* m = static_cast<unsigned long long*>(dmap.ptr);  // null without a map
    switch (kind) {
      case 0: hipLaunchKernelGGL(mfma_burn_kernel<0>, dim3(blocks), dim3(256), 0, nullptr, a, b, ex, iters, c, m); break;
      case 1: hipLaunchKernelGGL(mfma_burn_kernel<1>, dim3(blocks), dim3(256), 0, nullptr, a, b, ex, iters, c, m); break;
      case 2: hipLaunchKernelGGL(mfma_burn_kernel<2>, dim3(blocks), dim3(256), 0, nullptr, a, b, ex, iters, c, m); break;
      default: hipLaunchKernelGGL(mfma_burn_kernel<3>, dim3(blocks), dim3(256), 0, nullptr, a, b, ex, iters, c, m);
    }
  };
  launch();  // warm-up (also checked)
  DIAG_CHECK(hipGetLastError());
  DIAG_CHECK(hipDeviceSynchronize());
  Timer tm;
  DIAG_CHECK(tm.create());
  hipEvent_t e0 = tm.e0, e1 = tm.e1;
  DIAG_CHECK(hipEventRecord(e0, nullptr));
  for (int r = 0; r < reps; ++r) launch();
  DIAG_CHECK(hipEventRecord(e1, nullptr));
  DIAG_CHECK(hipEventSynchronize(e1));
  DIAG_CHECK(hipGetLastError());
  float ms = 0.f;
  DIAG_CHECK(event_ms(e0, e1, &ms));
  DIAG_CHECK(hipMemcpy(errors, dcnt.ptr, sizeof(unsigned long long), hipMemcpyDeviceToHost));
  if (cu_map != nullptr) DIAG_CHECK(hipMemcpy(cu_map, dmap.ptr, map_bytes, hipMemcpyDeviceToHost));
  const double flop = static_cast<double>(blocks) * 4 /*waves*/ * iters * 16 /*MFMA per iter*/ * 2.0 * 16 * 16 * K;
  *tflops = ms > 0.f ? flop * reps / (ms * 1e-3) / 1e12 : 0.0;
  return 0;
}

// LDS test over `rounds` x CUs workgroups of the largest LDS allocation a workgroup may take.
// cu_map: BURN_SLOTS x 2 (workgroups run, bad words) per physical CU slot; *lds_bytes = bytes per CU tested.
int diag_lds_test(int device, int rounds, uint32_t seed, int inject_block, unsigned long long* errors,
                  unsigned long long* cu_map, int* lds_bytes, double* ms) {
  if (rounds < 1 || rounds > 64) {
    g_err = "lds_test: 1 <= rounds <= 64";
    return -2;
  }
  DIAG_CHECK(hipSetDevice(device));
  int max_lds = 0;
  DIAG_CHECK(hipDeviceGetAttribute(&max_lds, hipDeviceAttributeMaxSharedMemoryPerBlock, device));
  if (max_lds < 65536 || max_lds > (1 << 20)) {
    g_err = "lds_test: unexpected LDS size " + std::to_string(max_lds);
    return -2;
  }
  // the kernel's own 4-byte counter shares the allocation
  const uint32_t dyn = static_cast<uint32_t>(max_lds) - 16u;
  DIAG_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(lds_test_kernel),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(dyn)));
  const size_t map_bytes = static_cast<size_t>(BURN_SLOTS) * 2 * sizeof(unsigned long long);
  DevBuf derr, dmap;
  DIAG_CHECK(derr.alloc(device, sizeof(unsigned long long)));
  DIAG_CHECK(dmap.alloc(device, map_bytes));
  DIAG_CHECK(hipMemset(derr.ptr, 0, sizeof(unsigned long long)));
  DIAG_CHECK(hipMemset(dmap.ptr, 0, map_bytes));
  const int blocks = grid_for(device, rounds);
  Timer tm;
  DIAG_CHECK(tm.create());
  hipEvent_t e0 = tm.e0, e1 = tm.e1;
  DIAG_CHECK(hipEventRecord(e0, nullptr));
  hipLaunchKernelGGL(lds_test_kernel, dim3(blocks), dim3(1024), dyn, nullptr, dyn / 4u, seed, inject_block,
                     static_cast<unsigned long long*>(derr.ptr), static_cast<unsigned long long*>(dmap.ptr));
  DIAG_CHECK(hipGetLastError());
  DIAG_CHECK(hipEventRecord(e1, nullptr));
  DIAG_CHECK(hipEventSynchronize(e1));
  float t_ms = 0.f;
  DIAG_CHECK(event_ms(e0, e1, &t_ms));
  *ms = t_ms;
  DIAG_CHECK(hipMemcpy(errors, derr.ptr, sizeof(unsigned long long), hipMemcpyDeviceToHost));
  DIAG_CHECK(hipMemcpy(cu_map, dmap.ptr, map_bytes, hipMemcpyDeviceToHost));
  *lds_bytes = static_cast<int>(dyn);
  return 0;
}

// L2 read bandwidth per XCD: 8 slices of `slice_bytes` (one per XCD id), `passes` reads of its slice by
// every workgroup, `blocks_per_cu` workgroups of 4 waves per CU.  *tbs = aggregate bytes read / timed launch; cu_map as
// diag_mfma_burn_map's (BURN_SLOTS x 3).
int diag_l2_bandwidth(int device, size_t slice_bytes, int passes, int blocks_per_cu, uint32_t seed, double* tbs,
                      unsigned long long* errors, unsigned long long* cu_map) {
  if (slice_bytes < 4096 || slice_bytes > (64u << 20) || slice_bytes % 16 || passes < 1 || passes > 1024 ||
      blocks_per_cu < 1 || blocks_per_cu > 8) {
    g_err = "l2_bandwidth: 4 KiB <= slice_bytes <= 64 MiB (multiple of 16), 1 <= passes <= 1024, 1..8 blocks/CU";
    return -2;
  }
  DIAG_CHECK(hipSetDevice(device));
  const uint32_t slice_vec = static_cast<uint32_t>(slice_bytes / 16);
  const uint32_t n_vec = 8u * slice_vec;  // XCC_ID is 0..7
  const size_t map_bytes = static_cast<size_t>(BURN_SLOTS) * 3 * sizeof(unsigned long long);
  DevBuf dbuf, derr, dmap;
  DIAG_CHECK(dbuf.alloc(device, static_cast<size_t>(n_vec) * 16));
  DIAG_CHECK(derr.alloc(device, sizeof(unsigned long long)));
  DIAG_CHECK(dmap.alloc(device, map_bytes));
  hipLaunchKernelGGL(l2_fill_kernel, dim3(1024), dim3(256), 0, nullptr, static_cast<uint4*>(dbuf.ptr), n_vec, seed);
  DIAG_CHECK(hipGetLastError());
  const int blocks = grid_for(device, blocks_per_cu);
  auto launch = [&]() {
    hipLaunchKernelGGL(l2_read_kernel, dim3(blocks), dim3(256), 0, nullptr, static_cast<const uint4*>(dbuf.ptr),
                       slice_vec, passes, seed, static_cast<unsigned long long*>(derr.ptr),
                       static_cast<unsigned long long*>(dmap.ptr));
  };
  launch();  // untimed: brings every slice into its XCD's L2
  DIAG_CHECK(hipGetLastError());
  DIAG_CHECK(hipDeviceSynchronize());
  DIAG_CHECK(hipMemset(derr.ptr, 0, sizeof(unsigned long long)));
  DIAG_CHECK(hipMemset(dmap.ptr, 0, map_bytes));
  Timer tm;
  DIAG_CHECK(tm.create());
  hipEvent_t e0 = tm.e0, e1 = tm.e1;
  DIAG_CHECK(hipEventRecord(e0, nullptr));
  launch();
  DIAG_CHECK(hipEventRecord(e1, nullptr));
  DIAG_CHECK(hipEventSynchronize(e1));
  DIAG_CHECK(hipGetLastError());
  float ms = 0.f;
  DIAG_CHECK(event_ms(e0, e1, &ms));
  DIAG_CHECK(hipMemcpy(errors, derr.ptr, sizeof(unsigned long long), hipMemcpyDeviceToHost));
  DIAG_CHECK(hipMemcpy(cu_map, dmap.ptr, map_bytes, hipMemcpyDeviceToHost));
  const double bytes = static_cast<double>(blocks) * passes * static_cast<double>(slice_bytes);
  *tbs = ms > 0.f ? bytes / (ms * 1e-3) / 1e12 : 0.0;
  return 0;
}

// HBM per XCD (hbm_xcd_kernel): `slice_bytes` per XCD (8 slices, a multiple of 128 KiB, at most 512 MiB),
// read `passes` times by the XCD's own workgroups, all XCDs at once: aggregate read TB/s, wrong words,
// per-CU map.  With `xcd_tbs` (8 doubles) each XCD then streams its slice alone: its own read TB/s (0 for an
// XCD without CUs on this device).
int diag_hbm_xcd(int device, size_t slice_bytes, int passes, int blocks_per_cu, uint32_t seed, double* tbs,
                 unsigned long long* errors, unsigned long long* cu_map, double* xcd_tbs) {
  const size_t chunk = static_cast<size_t>(HBM_XCD_CHUNK_VEC) * 16;
  if (slice_bytes < chunk || slice_bytes > (512u << 20) || slice_bytes % chunk || passes < 1 || passes > 64 ||
      blocks_per_cu < 1 || blocks_per_cu > 8) {
    g_err = "hbm_xcd: 128 KiB <= slice_bytes <= 512 MiB (multiple of 128 KiB), 1 <= passes <= 64, 1..8 blocks/CU";
    return -2;
  }
  DIAG_CHECK(hipSetDevice(device));
  const uint32_t slice_vec = static_cast<uint32_t>(slice_bytes / 16);
  const uint32_t n_vec = 8u * slice_vec;  // XCC_ID is 0..7; 8 x 512 MiB keeps word indices in 32 bits
  const size_t map_bytes = static_cast<size_t>(BURN_SLOTS) * 3 * sizeof(unsigned long long);
  DevBuf dbuf, dnext, derr, dmap;
  DIAG_CHECK(dbuf.alloc(device, static_cast<size_t>(n_vec) * 16));
  DIAG_CHECK(dnext.alloc(device, 8 * sizeof(unsigned int)));
  DIAG_CHECK(derr.alloc(device, sizeof(unsigned long long)));
  DIAG_CHECK(dmap.alloc(device, map_bytes));
  hipLaunchKernelGGL(l2_fill_kernel, dim3(4096), dim3(256), 0, nullptr, static_cast<uint4*>(dbuf.ptr), n_vec, seed);
  DIAG_CHECK(hipGetLastError());
  const int blocks = grid_for(device, blocks_per_cu);
  Timer tm;
  DIAG_CHECK(tm.create());
  // one timed run (the queue counters reset first); returns its milliseconds, < 0 on a HIP error
  auto timed = [&](int only_xcd) -> float {
    if (hipMemset(dnext.ptr, 0, 8 * sizeof(unsigned int)) != hipSuccess) return -1.f;
    if (hipEventRecord(tm.e0, nullptr) != hipSuccess) return -1.f;
    hipLaunchKernelGGL(hbm_xcd_kernel, dim3(blocks), dim3(256), 0, nullptr, static_cast<const uint4*>(dbuf.ptr),
                       slice_vec, passes, seed, only_xcd, static_cast<unsigned int*>(dnext.ptr),
                       static_cast<unsigned long long*>(derr.ptr), static_cast<unsigned long long*>(dmap.ptr));
    if (hipGetLastError() != hipSuccess || hipEventRecord(tm.e1, nullptr) != hipSuccess ||
        hipEventSynchronize(tm.e1) != hipSuccess)
      return -1.f;
    return elapsed_ms(tm.e0, tm.e1);
  };
  if (timed(-1) < 0.f) DIAG_CHECK(hipGetLastError());  // untimed warm-up: page tables, clocks up
  DIAG_CHECK(hipMemset(derr.ptr, 0, sizeof(unsigned long long)));
  DIAG_CHECK(hipMemset(dmap.ptr, 0, map_bytes));
  const float ms = timed(-1);
  if (ms < 0.f) {
    DIAG_CHECK(hipGetLastError());
    g_err = "hbm_xcd: timed run failed";
    return -1;
  }
  DIAG_CHECK(hipMemcpy(cu_map, dmap.ptr, map_bytes, hipMemcpyDeviceToHost));
  // bytes actually read: every XCD that has CUs reads its slice `passes` times
  bool present[8] = {false, false, false, false, false, false, false, false};
  int xcds_seen = 0;
  for (int x = 0; x < 8; ++x) {
    for (int sl = 0; sl < 128 && !present[x]; ++sl) present[x] = cu_map[3 * (x * 128 + sl)] != 0;
    xcds_seen += present[x];
  }
  const double bytes = static_cast<double>(xcds_seen) * passes * static_cast<double>(slice_bytes);
  *tbs = ms > 0.f ? bytes / (ms * 1e-3) / 1e12 : 0.0;
  if (xcd_tbs != nullptr) {
    // untimed: the first lone-XCD run of a process measured ~8 % low (one XCD's clocks and queues ramping
    // after the full-chip run), so the first present XCD streams once before the timed ones
    for (int x = 0; x < 8; ++x)
      if (present[x]) {
        if (timed(x) < 0.f) DIAG_CHECK(hipGetLastError());
        break;
      }
    for (int x = 0; x < 8; ++x) {
      xcd_tbs[x] = 0.0;
      if (!present[x]) continue;
      const float xms = timed(x);
      if (xms < 0.f) {
        DIAG_CHECK(hipGetLastError());
        g_err = "hbm_xcd: isolated run failed";
        return -1;
      }
      xcd_tbs[x] = xms > 0.f ? passes * static_cast<double>(slice_bytes) / (xms * 1e-3) / 1e12 : 0.0;
    }
  }
  DIAG_CHECK(hipMemcpy(errors, derr.ptr, sizeof(unsigned long long), hipMemcpyDeviceToHost));
  return 0;
}

// Host link check: pinned host <-> device copies of `bytes`, `iters` each way (SDMA over PCIe),
// timed with events.  A slot trained down to x8 / an older generation shows up here at half rate.
int diag_host_link(int device, size_t bytes, int iters, double* h2d_gbps, double* d2h_gbps) {
  if (bytes < 4096 || iters < 1) {
    g_err = "host_link: bytes >= 4096 and iters >= 1";
    return -2;
  }
  DIAG_CHECK(hipSetDevice(device));
  void* host = nullptr;
  DIAG_CHECK(hipHostMalloc(&host, bytes, hipHostMallocDefault));
  struct HostFree {
    void* p;
    ~HostFree() { (void)hipHostFree(p); }
  } hf{host};
  memset(host, 0x5A, bytes);
  DevBuf dev;
  DIAG_CHECK(dev.alloc(device, bytes));
  // on the null stream, as every single-device test: a stream of its own would be one more hardware queue, and each
  // queue the runtime creates holds ~170 MiB of host memory for the rest of the process (tools/hip_rss_probe.hip)
  Timer tm;
  DIAG_CHECK(tm.create());
  hipEvent_t e0 = tm.e0, e1 = tm.e1;
  hipStream_t st = nullptr;
  for (int dir = 0; dir < 2; ++dir) {
    auto copy = [&]() {
      return dir == 0 ? hipMemcpyAsync(dev.ptr, host, bytes, hipMemcpyHostToDevice, st)
                      : hipMemcpyAsync(host, dev.ptr, bytes, hipMemcpyDeviceToHost, st);
    };
    DIAG_CHECK(copy());  // warm-up
    DIAG_CHECK(hipEventRecord(e0, st));
    for (int i = 0; i < iters; ++i) DIAG_CHECK(copy());
    DIAG_CHECK(hipEventRecord(e1, st));
    DIAG_CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    DIAG_CHECK(event_ms(e0, e1, &ms));
    const double gbps = ms > 0.f ? static_cast<double>(iters) * static_cast<double>(bytes) / (ms * 1e-3) / 1e9 : 0.0;
    *(dir == 0 ? h2d_gbps : d2h_gbps) = gbps;
  }
  return 0;
}

}  // extern "C"
