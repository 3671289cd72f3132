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


// "v3": the v2 tile (256x256x64, 8 waves of 128x64, two 64 KiB LDS-DMA stages) on a staggered 4-phase
// schedule.  Each K-tile is 4 phases, one 64x32 quadrant of the wave's output each (16 MFMA); a phase is
// a load slot (this quadrant's ds_reads, retired with lgkmcnt(0) before the barrier) and an MFMA slot,
// separated by raw s_barriers.  Group 1 (waves 4-7) runs one barrier behind group 0, so on every SIMD
// one wave's MFMA slot covers the other's load slot and barrier wait.
// Quadrant order (m0,n0) (m0,n1) (m1,n1) (m1,n0): A(m0)+B(n0), B(n1), A(m1) are read in phases 0-2
// and phase 3 reuses B(n0) from registers, so the phase-3 load slot reads no LDS: there each wave
// issues its LDS-DMA share of tile t+2 into tile t's buffer (every read of tile t was retired before
// an earlier barrier) and then waits, counted vmcnt(8), for its share of tile t+1 issued one tile
// earlier; the barrier closing that slot precedes the first read of tile t+1 (next phase 0).
#define SLOT_BARRIER()                 \
  do {                                 \
    __builtin_amdgcn_sched_barrier(0); \
    __builtin_amdgcn_s_barrier();      \
    __builtin_amdgcn_sched_barrier(0); \
  } while (0)

template <bool PRIO>
__device__ __forceinline__ void v3_mfma(floatx4 (&acc)[8][4], const bf16x8 (&af)[4][2], const bf16x8 (&bf)[2][2],
                                        int m0, int n0) {
  if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n)
        acc[m0 + m][n0 + n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m][s], bf[n][s], acc[m0 + m][n0 + n], 0, 0, 0);
  // MFMAs are not memory operations: IR passes may sink them past the next s_barrier into the other
  // group's slot.  An empty volatile asm that "reads and writes" each result pins them to this slot.
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n) asm volatile("" : "+v"(acc[m0 + m][n0 + n]));
  if (PRIO) __builtin_amdgcn_s_setprio(0);
}

template <bool PRIO>
__global__ void __launch_bounds__(V2_THREADS, 1)
lab_v3_kernel(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt, float* __restrict__ C, int M, int N, int K) {
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

  v2_fill(smem, Ab, Bb, K, 0, wid, lane);
  if (KT > 1) {
    v2_fill(smem + V2_STAGE_BYTES, Ab, Bb, K, 1, wid, lane);
    __builtin_amdgcn_s_waitcnt(0x3f78);  // vmcnt(8): tile 0 landed, tile 1 may be in flight
  } else {
    __builtin_amdgcn_s_waitcnt(0x3f70);
  }
  SLOT_BARRIER();
  if (wr == 1) SLOT_BARRIER();  // the stagger

  bf16x8 af[4][2], b0[2][2], b1[2][2];
  for (int kt = 0; kt < KT; ++kt) {
    unsigned char* cur = smem + (kt & 1) * V2_STAGE_BYTES;
    const u32x4* a_img = reinterpret_cast<const u32x4*>(cur);
    const u32x4* b_img = reinterpret_cast<const u32x4*>(cur + V2_BM * BK * 2);
    // phase 0: A(m0), B(n0)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int s = 0; s < 2; ++s) b0[n][s] = __builtin_bit_cast(bf16x8, b_img[swz(wc * 64 + n * 16 + frow, fq + 4 * s)]);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int s = 0; s < 2; ++s) af[m][s] = __builtin_bit_cast(bf16x8, a_img[swz(wr * 128 + m * 16 + frow, fq + 4 * s)]);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    SLOT_BARRIER();
    v3_mfma<PRIO>(acc, af, b0, 0, 0);
    SLOT_BARRIER();
    // phase 1: B(n1)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        b1[n][s] = __builtin_bit_cast(bf16x8, b_img[swz(wc * 64 + (n + 2) * 16 + frow, fq + 4 * s)]);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    SLOT_BARRIER();
    v3_mfma<PRIO>(acc, af, b1, 0, 2);
    SLOT_BARRIER();
    // phase 2: A(m1)
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        af[m][s] = __builtin_bit_cast(bf16x8, a_img[swz(wr * 128 + (m + 4) * 16 + frow, fq + 4 * s)]);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    SLOT_BARRIER();
    v3_mfma<PRIO>(acc, af, b1, 4, 2);
    SLOT_BARRIER();
    // phase 3: no LDS reads; restage tile kt's buffer with tile kt+2, retire tile kt+1
    if (kt + 2 < KT) {
      v2_fill(cur, Ab, Bb, K, kt + 2, wid, lane);
      __builtin_amdgcn_s_waitcnt(0x3f78);  // vmcnt(8)
    } else {
      __builtin_amdgcn_s_waitcnt(0x3f70);  // vmcnt(0)
    }
    SLOT_BARRIER();
    v3_mfma<PRIO>(acc, af, b0, 4, 0);
    SLOT_BARRIER();
  }
  if (wr == 0) SLOT_BARRIER();  // balance the stagger
  const int row0 = tm * V2_BM + wr * 128, col0 = tn * V2_BN + wc * 64;
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        C[static_cast<size_t>(row0 + m * 16 + fq * 4 + j) * N + col0 + n * 16 + frow] = acc[m][n][j];
}


// "v4": v3 with the next-next tile's LDS-DMA spread over phases 1-3 as the regions of the current
// buffer free up.  Regions of a stage (16 KiB each, 16 DMA wave-instructions, 2 per wave):
//   0 = A rows read in phase 0 (m0 half of both wave rows), 1 = B rows of n0 (phase 0; phase 3 reuses
//   registers), 2 = B rows of n1 (phase 1), 3 = A rows of m1 (phase 2).
// A region read in phase p is restaged from phase p+1's load slot on: every wave retired its phase-p
// reads (lgkmcnt(0)) before the barrier that closed its load slot, and the other group's phase-p load
// slot closes before this group's phase p+1 load slot opens.  Issue: phase 1 R0 R0 R1, phase 2 R1 R2 R2,
// phase 3 R3 R3; retire tile t+1 at phase 3 of tile t with vmcnt(8) (tile t+2's 8 pieces may fly).
__device__ __forceinline__ void lab_piece(unsigned char* lds_stage, const __bf16* __restrict__ A,
                                         const __bf16* __restrict__ Bt, int K, int kt, int region, int i, int wid,
                                         int lane) {
  const int rsub = lane >> 3, phys = lane & 7;
  const int g = wid * 2 + i;  // 16 groups of 8 rows per region
  int row0;
  if (region == 0 || region == 3) {
    const int h = region == 0 ? 0 : 1;
    row0 = (g >> 3) * 128 + h * 64 + (g & 7) * 8;
  } else {
    const int h = region == 1 ? 0 : 1;
    row0 = (g >> 2) * 64 + h * 32 + (g & 3) * 8;
  }
  const int row = row0 + rsub;
  const int c = phys ^ ((row >> 1) & 7);
  const bool is_a = region == 0 || region == 3;
  const __bf16* gp = (is_a ? A : Bt) + static_cast<size_t>(row) * K + kt * BK + c * 8;
  unsigned char* l = lds_stage + (is_a ? 0 : V2_BM * BK * 2) + row0 * (BK * 2);
  __builtin_amdgcn_global_load_lds(gp, (lds_void_t*)l, 16, 0, 0);
}

template <bool PRIO>
__global__ void __launch_bounds__(V2_THREADS, 1)
gemm_lab_v4_kernel(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt, float* __restrict__ C, int M, int N, int K) {
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

  v2_fill(smem, Ab, Bb, K, 0, wid, lane);
  if (KT > 1) {
    v2_fill(smem + V2_STAGE_BYTES, Ab, Bb, K, 1, wid, lane);
    __builtin_amdgcn_s_waitcnt(0x3f78);  // vmcnt(8)
  } else {
    __builtin_amdgcn_s_waitcnt(0x3f70);
  }
  SLOT_BARRIER();
  if (wr == 1) SLOT_BARRIER();

  bf16x8 af[4][2], b0[2][2], b1[2][2];
  for (int kt = 0; kt < KT; ++kt) {
    unsigned char* cur = smem + (kt & 1) * V2_STAGE_BYTES;
    const u32x4* a_img = reinterpret_cast<const u32x4*>(cur);
    const u32x4* b_img = reinterpret_cast<const u32x4*>(cur + V2_BM * BK * 2);
    const bool pre = kt + 2 < KT;
    // phase 0
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int s = 0; s < 2; ++s) b0[n][s] = __builtin_bit_cast(bf16x8, b_img[swz(wc * 64 + n * 16 + frow, fq + 4 * s)]);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int s = 0; s < 2; ++s) af[m][s] = __builtin_bit_cast(bf16x8, a_img[swz(wr * 128 + m * 16 + frow, fq + 4 * s)]);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    SLOT_BARRIER();
    v3_mfma<PRIO>(acc, af, b0, 0, 0);
    SLOT_BARRIER();
    // phase 1
    if (pre) {
      lab_piece(cur, Ab, Bb, K, kt + 2, 0, 0, wid, lane);
      lab_piece(cur, Ab, Bb, K, kt + 2, 0, 1, wid, lane);
      lab_piece(cur, Ab, Bb, K, kt + 2, 1, 0, wid, lane);
    }
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        b1[n][s] = __builtin_bit_cast(bf16x8, b_img[swz(wc * 64 + (n + 2) * 16 + frow, fq + 4 * s)]);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    SLOT_BARRIER();
    v3_mfma<PRIO>(acc, af, b1, 0, 2);
    SLOT_BARRIER();
    // phase 2
    if (pre) {
      lab_piece(cur, Ab, Bb, K, kt + 2, 1, 1, wid, lane);
      lab_piece(cur, Ab, Bb, K, kt + 2, 2, 0, wid, lane);
      lab_piece(cur, Ab, Bb, K, kt + 2, 2, 1, wid, lane);
    }
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        af[m][s] = __builtin_bit_cast(bf16x8, a_img[swz(wr * 128 + (m + 4) * 16 + frow, fq + 4 * s)]);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    SLOT_BARRIER();
    v3_mfma<PRIO>(acc, af, b1, 4, 2);
    SLOT_BARRIER();
    // phase 3
    if (pre) {
      lab_piece(cur, Ab, Bb, K, kt + 2, 3, 0, wid, lane);
      lab_piece(cur, Ab, Bb, K, kt + 2, 3, 1, wid, lane);
      __builtin_amdgcn_s_waitcnt(0x3f78);  // vmcnt(8): tile kt+1 landed
    } else {
      __builtin_amdgcn_s_waitcnt(0x3f70);
    }
    SLOT_BARRIER();
    v3_mfma<PRIO>(acc, af, b0, 4, 0);
    SLOT_BARRIER();
  }
  if (wr == 0) SLOT_BARRIER();
  const int row0 = tm * V2_BM + wr * 128, col0 = tn * V2_BN + wc * 64;
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        C[static_cast<size_t>(row0 + m * 16 + fq * 4 + j) * N + col0 + n * 16 + frow] = acc[m][n][j];
}


// "v5": v4 with each phase's ds_reads retired AFTER the barrier that closes the load slot (at the top
// of the MFMA slot), so the read latency hides behind the barrier wait.  A region read in phase p is
// then only retired when the reading wave passes the barrier closing its MFMA slot, so it is restaged
// two phases later: R0/R1 (read phase 0) in phase 2, R2 (phase 1) in phase 3, R3 (phase 2) in phase 0
// of the next tile (into the other buffer, for tile t+1).  Retire tile t+1 at phase 3 of tile t:
// tile t+2's R0 R1 R2 pieces (6) were issued after tile t+1's last one -> vmcnt(6).
// ABL (timing ablations, wrong results): bit 0 = no LDS-DMA in the loop, bit 1 = no barriers in the loop,
// bit 2 = no vmcnt waits in the loop
template <bool PRIO, int ABL = 0, int GM = 4>
__global__ void __launch_bounds__(V2_THREADS, 1)
gemm_v5_kernel(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt, float* __restrict__ C, int M, int N, int K) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  const int tiles_m = M / V2_BM, tiles_n = N / V2_BN, nwg = tiles_m * tiles_n;
  int bid = blockIdx.x;
  {
    const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
  }
  constexpr int GROUP_M = GM;
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
  if (KT > 1) {
    v2_fill(smem + V2_STAGE_BYTES, Ab, Bb, K, 1, wid, lane);
    __builtin_amdgcn_s_waitcnt(0x3f78);  // vmcnt(8)
  } else {
    __builtin_amdgcn_s_waitcnt(0x3f70);
  }
  SLOT_BARRIER();
  if (wr == 1) SLOT_BARRIER();

  bf16x8 af[4][2], b0[2][2], b1[2][2];
  for (int kt = 0; kt < KT; ++kt) {
    unsigned char* cur = smem + (kt & 1) * V2_STAGE_BYTES;
    unsigned char* nxt = smem + ((kt + 1) & 1) * V2_STAGE_BYTES;
    const u32x4* a_img = reinterpret_cast<const u32x4*>(cur);
    const u32x4* b_img = reinterpret_cast<const u32x4*>(cur + V2_BM * BK * 2);
    const bool pre = kt + 2 < KT;
    // phase 0 (+ tile kt+1's R3 into the other buffer; tile 1 came whole with the prologue)
    if (!(ABL & 1) && kt >= 1 && kt + 1 < KT) {
      lab_piece(nxt, Ab, Bb, K, kt + 1, 3, 0, wid, lane);
      lab_piece(nxt, Ab, Bb, K, kt + 1, 3, 1, wid, lane);
    }
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int s = 0; s < 2; ++s) b0[n][s] = __builtin_bit_cast(bf16x8, b_img[swz(wc * 64 + n * 16 + frow, fq + 4 * s)]);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int s = 0; s < 2; ++s) af[m][s] = __builtin_bit_cast(bf16x8, a_img[swz(wr * 128 + m * 16 + frow, fq + 4 * s)]);
    if (!(ABL & 2)) SLOT_BARRIER();
    __builtin_amdgcn_s_waitcnt(0xc07f);
    v3_mfma<PRIO>(acc, af, b0, 0, 0);
    if (!(ABL & 2)) SLOT_BARRIER();
    // phase 1
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        b1[n][s] = __builtin_bit_cast(bf16x8, b_img[swz(wc * 64 + (n + 2) * 16 + frow, fq + 4 * s)]);
    if (!(ABL & 2)) SLOT_BARRIER();
    __builtin_amdgcn_s_waitcnt(0xc07f);
    v3_mfma<PRIO>(acc, af, b1, 0, 2);
    if (!(ABL & 2)) SLOT_BARRIER();
    // phase 2: restage R0, R1 of this buffer with tile kt+2
    if (!(ABL & 1) && pre) {
      lab_piece(cur, Ab, Bb, K, kt + 2, 0, 0, wid, lane);
      lab_piece(cur, Ab, Bb, K, kt + 2, 0, 1, wid, lane);
      lab_piece(cur, Ab, Bb, K, kt + 2, 1, 0, wid, lane);
      lab_piece(cur, Ab, Bb, K, kt + 2, 1, 1, wid, lane);
    }
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        af[m][s] = __builtin_bit_cast(bf16x8, a_img[swz(wr * 128 + (m + 4) * 16 + frow, fq + 4 * s)]);
    if (!(ABL & 2)) SLOT_BARRIER();
    __builtin_amdgcn_s_waitcnt(0xc07f);
    v3_mfma<PRIO>(acc, af, b1, 4, 2);
    if (!(ABL & 2)) SLOT_BARRIER();
    // phase 3: restage R2; retire tile kt+1
    if (!(ABL & 1) && pre) {
      lab_piece(cur, Ab, Bb, K, kt + 2, 2, 0, wid, lane);
      lab_piece(cur, Ab, Bb, K, kt + 2, 2, 1, wid, lane);
      if (!(ABL & 4)) __builtin_amdgcn_s_waitcnt(0x3f76);  // vmcnt(6)
    } else {
      if (!(ABL & 4)) __builtin_amdgcn_s_waitcnt(0x3f70);
    }
    if (!(ABL & 2)) SLOT_BARRIER();
    v3_mfma<PRIO>(acc, af, b0, 4, 0);
    if (!(ABL & 2)) SLOT_BARRIER();
  }
  if (wr == 0) SLOT_BARRIER();
  const int row0 = tm * V2_BM + wr * 128, col0 = tn * V2_BN + wc * 64;
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        C[static_cast<size_t>(row0 + m * 16 + fq * 4 + j) * N + col0 + n * 16 + frow] = acc[m][n][j];
}


// "v6": v5 with the LDS-DMA spread evenly, one region (2 DMA per wave) per phase, and a counted
// vmcnt(8) in every phase (4 regions = one tile in flight).  Phase p of tile t stages:
//   p=0: R2 of tile t+1 (other buffer; R2 there was last read at phase 1 of tile t-1)
//   p=1: R3 of tile t+1 (last read at phase 2 of tile t-1)
//   p=2: R0 of tile t+2 (this buffer; read at phase 0 of tile t)
//   p=3: R1 of tile t+2 (read at phase 0 of tile t)
// every restage is >= 2 phases after the region's last read (reads retire after the barrier, v5).
// The vmcnt(8) at phase q retires the region staged at phase q-4, which is first read at phase q+1
// or later.  Near the end (nothing left to stage) the wait falls back to vmcnt(0).
template <bool PRIO>
__global__ void __launch_bounds__(V2_THREADS, 1)
gemm_v6_kernel(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt, float* __restrict__ C, int M, int N, int K) {
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

  // prologue: tile 0 whole, tile 1's R0 R1 (its R2 R3 come with phases 0 and 1 of tile 0)
  v2_fill(smem, Ab, Bb, K, 0, wid, lane);
  if (KT > 1) {
    unsigned char* s1 = smem + V2_STAGE_BYTES;
    lab_piece(s1, Ab, Bb, K, 1, 0, 0, wid, lane);
    lab_piece(s1, Ab, Bb, K, 1, 0, 1, wid, lane);
    lab_piece(s1, Ab, Bb, K, 1, 1, 0, wid, lane);
    lab_piece(s1, Ab, Bb, K, 1, 1, 1, wid, lane);
    __builtin_amdgcn_s_waitcnt(0x3f74);  // vmcnt(4): tile 0 landed
  } else {
    __builtin_amdgcn_s_waitcnt(0x3f70);
  }
  SLOT_BARRIER();
  if (wr == 1) SLOT_BARRIER();

#define V6_STAGE(buf, tile, region)                                  \
  do {                                                               \
    if ((tile) < KT) {                                               \
      lab_piece((buf), Ab, Bb, K, (tile), (region), 0, wid, lane);    \
      lab_piece((buf), Ab, Bb, K, (tile), (region), 1, wid, lane);    \
      __builtin_amdgcn_s_waitcnt(0x3f78); /* vmcnt(8) */             \
    } else {                                                         \
      __builtin_amdgcn_s_waitcnt(0x3f70); /* vmcnt(0) */             \
    }                                                                \
  } while (0)

  bf16x8 af[4][2], b0[2][2], b1[2][2];
  for (int kt = 0; kt < KT; ++kt) {
    unsigned char* cur = smem + (kt & 1) * V2_STAGE_BYTES;
    unsigned char* nxt = smem + ((kt + 1) & 1) * V2_STAGE_BYTES;
    const u32x4* a_img = reinterpret_cast<const u32x4*>(cur);
    const u32x4* b_img = reinterpret_cast<const u32x4*>(cur + V2_BM * BK * 2);
    // phase 0
    V6_STAGE(nxt, kt + 1, 2);
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int s = 0; s < 2; ++s) b0[n][s] = __builtin_bit_cast(bf16x8, b_img[swz(wc * 64 + n * 16 + frow, fq + 4 * s)]);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int s = 0; s < 2; ++s) af[m][s] = __builtin_bit_cast(bf16x8, a_img[swz(wr * 128 + m * 16 + frow, fq + 4 * s)]);
    SLOT_BARRIER();
    __builtin_amdgcn_s_waitcnt(0xc07f);
    v3_mfma<PRIO>(acc, af, b0, 0, 0);
    SLOT_BARRIER();
    // phase 1
    V6_STAGE(nxt, kt + 1, 3);
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        b1[n][s] = __builtin_bit_cast(bf16x8, b_img[swz(wc * 64 + (n + 2) * 16 + frow, fq + 4 * s)]);
    SLOT_BARRIER();
    __builtin_amdgcn_s_waitcnt(0xc07f);
    v3_mfma<PRIO>(acc, af, b1, 0, 2);
    SLOT_BARRIER();
    // phase 2
    V6_STAGE(cur, kt + 2, 0);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        af[m][s] = __builtin_bit_cast(bf16x8, a_img[swz(wr * 128 + (m + 4) * 16 + frow, fq + 4 * s)]);
    SLOT_BARRIER();
    __builtin_amdgcn_s_waitcnt(0xc07f);
    v3_mfma<PRIO>(acc, af, b1, 4, 2);
    SLOT_BARRIER();
    // phase 3
    V6_STAGE(cur, kt + 2, 1);
    SLOT_BARRIER();
    v3_mfma<PRIO>(acc, af, b0, 4, 0);
    SLOT_BARRIER();
  }
#undef V6_STAGE
  if (wr == 0) SLOT_BARRIER();
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
  // gemm_lab.bin [size [iters]]: one size only (for rocprofv3 --pmc runs), default 4096 and 8192
  std::vector<int> sizes = {4096, 8192};
  if (argc > 1) sizes = {atoi(argv[1])};
  const int iters_arg = argc > 2 ? atoi(argv[2]) : 0;
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
    hipLaunchKernelGGL(gemm_bf16_kernel, dim3(nwg1), dim3(THREADS), 0, nullptr, (const u32x4*)A, (const u32x4*)Bt, C0, M,
                       N, K);
    CK(hipDeviceSynchronize());
    std::vector<float> h0((size_t)M * N), h1((size_t)M * N);
    CK(hipMemcpy(h0.data(), C0, sizeof(float) * M * N, hipMemcpyDeviceToHost));
    CK(hipFuncSetAttribute((const void*)gemm_bf16_v2_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * V2_STAGE_BYTES));
    CK(hipFuncSetAttribute((const void*)gemm_vp_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * V2_STAGE_BYTES));
    CK(hipFuncSetAttribute((const void*)gemm_vp_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * V2_STAGE_BYTES));
    CK(hipFuncSetAttribute((const void*)lab_v3_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * V2_STAGE_BYTES));
    CK(hipFuncSetAttribute((const void*)lab_v3_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * V2_STAGE_BYTES));
    CK(hipFuncSetAttribute((const void*)gemm_lab_v4_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * V2_STAGE_BYTES));
    CK(hipFuncSetAttribute((const void*)gemm_lab_v4_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * V2_STAGE_BYTES));
    CK(hipFuncSetAttribute((const void*)gemm_v5_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * V2_STAGE_BYTES));
    CK(hipFuncSetAttribute((const void*)gemm_v5_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * V2_STAGE_BYTES));
    auto check = [&](const char* name, double ms) {
      CK(hipMemcpy(h1.data(), C1, sizeof(float) * M * N, hipMemcpyDeviceToHost));
      double worst = 0;
      for (size_t i = 0; i < h0.size(); ++i) worst = std::max(worst, (double)std::fabs(h0[i] - h1[i]) / std::max(1.0, (double)std::fabs(h0[i])));
      printf("{\"kernel\": \"%s\", \"size\": %d, \"tflops\": %.1f, \"ms\": %.4f, \"max_rel_diff_vs_v1\": %.3g}\n", name, size,
             2.0 * M * N * (double)K / (ms * 1e-3) / 1e12, ms, worst);
      CK(hipMemset(C1, 0xff, sizeof(float) * M * N));
    };
    const int it = iters_arg > 0 ? iters_arg : (size == 8192 ? 20 : 50);
    double ms;
    ms = time_ms([&] { hipLaunchKernelGGL(gemm_bf16_kernel, dim3(nwg1), dim3(THREADS), 0, nullptr, (const u32x4*)A, (const u32x4*)Bt, C1, M, N, K); }, it);
    check("v1", ms);
    ms = time_ms([&] { hipLaunchKernelGGL(gemm_bf16_v2_kernel, dim3(nwg2), dim3(V2_THREADS), 2 * V2_STAGE_BYTES, nullptr, A, Bt, C1, M, N, K); }, it);
    check("v2", ms);
    ms = time_ms([&] { hipLaunchKernelGGL(gemm_vp_kernel<false>, dim3(nwg2), dim3(V2_THREADS), 2 * V2_STAGE_BYTES, nullptr, A, Bt, C1, M, N, K); }, it);
    check("vP", ms);
    ms = time_ms([&] { hipLaunchKernelGGL(gemm_vp_kernel<true>, dim3(nwg2), dim3(V2_THREADS), 2 * V2_STAGE_BYTES, nullptr, A, Bt, C1, M, N, K); }, it);
    check("vP+prio", ms);
    ms = time_ms([&] { hipLaunchKernelGGL(lab_v3_kernel<false>, dim3(nwg2), dim3(V2_THREADS), 2 * V2_STAGE_BYTES, nullptr, A, Bt, C1, M, N, K); }, it);
    check("v3", ms);
    ms = time_ms([&] { hipLaunchKernelGGL(lab_v3_kernel<true>, dim3(nwg2), dim3(V2_THREADS), 2 * V2_STAGE_BYTES, nullptr, A, Bt, C1, M, N, K); }, it);
    check("v3+prio", ms);
    ms = time_ms([&] { hipLaunchKernelGGL(gemm_lab_v4_kernel<false>, dim3(nwg2), dim3(V2_THREADS), 2 * V2_STAGE_BYTES, nullptr, A, Bt, C1, M, N, K); }, it);
    check("v4", ms);
    ms = time_ms([&] { hipLaunchKernelGGL(gemm_lab_v4_kernel<true>, dim3(nwg2), dim3(V2_THREADS), 2 * V2_STAGE_BYTES, nullptr, A, Bt, C1, M, N, K); }, it);
    check("v4+prio", ms);
    ms = time_ms([&] { hipLaunchKernelGGL(gemm_v5_kernel<false>, dim3(nwg2), dim3(V2_THREADS), 2 * V2_STAGE_BYTES, nullptr, A, Bt, C1, M, N, K); }, it);
    check("v5", ms);
    ms = time_ms([&] { hipLaunchKernelGGL(gemm_v5_kernel<true>, dim3(nwg2), dim3(V2_THREADS), 2 * V2_STAGE_BYTES, nullptr, A, Bt, C1, M, N, K); }, it);
    check("v5+prio", ms);
    CK(hipFuncSetAttribute((const void*)gemm_v6_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * V2_STAGE_BYTES));
    CK(hipFuncSetAttribute((const void*)gemm_v6_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * V2_STAGE_BYTES));
    ms = time_ms([&] { hipLaunchKernelGGL(gemm_v6_kernel<false>, dim3(nwg2), dim3(V2_THREADS), 2 * V2_STAGE_BYTES, nullptr, A, Bt, C1, M, N, K); }, it);
    check("v6", ms);
    ms = time_ms([&] { hipLaunchKernelGGL(gemm_v6_kernel<true>, dim3(nwg2), dim3(V2_THREADS), 2 * V2_STAGE_BYTES, nullptr, A, Bt, C1, M, N, K); }, it);
    check("v6+prio", ms);
    CK(hipFuncSetAttribute((const void*)gemm_v5_kernel<false, 0, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * V2_STAGE_BYTES));
    CK(hipFuncSetAttribute((const void*)gemm_v5_kernel<false, 0, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * V2_STAGE_BYTES));
    CK(hipFuncSetAttribute((const void*)gemm_v5_kernel<false, 0, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * V2_STAGE_BYTES));
    CK(hipFuncSetAttribute((const void*)gemm_v5_kernel<false, 0, 16>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * V2_STAGE_BYTES));
    ms = time_ms([&] { hipLaunchKernelGGL((gemm_v5_kernel<false, 0, 1>), dim3(nwg2), dim3(V2_THREADS), 2 * V2_STAGE_BYTES, nullptr, A, Bt, C1, M, N, K); }, it);
    check("v5-groupm1", ms);
    ms = time_ms([&] { hipLaunchKernelGGL((gemm_v5_kernel<false, 0, 2>), dim3(nwg2), dim3(V2_THREADS), 2 * V2_STAGE_BYTES, nullptr, A, Bt, C1, M, N, K); }, it);
    check("v5-groupm2", ms);
    ms = time_ms([&] { hipLaunchKernelGGL((gemm_v5_kernel<false, 0, 8>), dim3(nwg2), dim3(V2_THREADS), 2 * V2_STAGE_BYTES, nullptr, A, Bt, C1, M, N, K); }, it);
    check("v5-groupm8", ms);
    ms = time_ms([&] { hipLaunchKernelGGL((gemm_v5_kernel<false, 0, 16>), dim3(nwg2), dim3(V2_THREADS), 2 * V2_STAGE_BYTES, nullptr, A, Bt, C1, M, N, K); }, it);
    check("v5-groupm16", ms);
    CK(hipFuncSetAttribute((const void*)gemm_v5_kernel<false, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * V2_STAGE_BYTES));
    ms = time_ms([&] { hipLaunchKernelGGL((gemm_v5_kernel<false, 4>), dim3(nwg2), dim3(V2_THREADS), 2 * V2_STAGE_BYTES, nullptr, A, Bt, C1, M, N, K); }, it);
    check("v5-ablation-no-vmcnt", ms);
    CK(hipFuncSetAttribute((const void*)gemm_v5_kernel<false, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * V2_STAGE_BYTES));
    CK(hipFuncSetAttribute((const void*)gemm_v5_kernel<false, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * V2_STAGE_BYTES));
    CK(hipFuncSetAttribute((const void*)gemm_v5_kernel<false, 3>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * V2_STAGE_BYTES));
    ms = time_ms([&] { hipLaunchKernelGGL((gemm_v5_kernel<false, 1>), dim3(nwg2), dim3(V2_THREADS), 2 * V2_STAGE_BYTES, nullptr, A, Bt, C1, M, N, K); }, it);
    check("v5-ablation-no-glds", ms);
    ms = time_ms([&] { hipLaunchKernelGGL((gemm_v5_kernel<false, 2>), dim3(nwg2), dim3(V2_THREADS), 2 * V2_STAGE_BYTES, nullptr, A, Bt, C1, M, N, K); }, it);
    check("v5-ablation-no-barrier", ms);
    ms = time_ms([&] { hipLaunchKernelGGL((gemm_v5_kernel<false, 3>), dim3(nwg2), dim3(V2_THREADS), 2 * V2_STAGE_BYTES, nullptr, A, Bt, C1, M, N, K); }, it);
    check("v5-ablation-neither", ms);
    hipFree(A);
    hipFree(Bt);
    hipFree(C0);
    hipFree(C1);
  }
  return 0;
}
