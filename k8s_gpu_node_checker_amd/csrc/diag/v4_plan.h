// Schedules of the four-wave v4 GEMM K loop (diag.hip gemm_v4_kernel) as compile-time plans, and the checks
// every plan must pass.  Plain constexpr C++: diag.hip includes this inside its anonymous namespace, and
// tests/test_gemm_plans.py compiles it with the host compiler to show the checks reject broken plans.
#ifndef K8S_GPU_NODE_CHECKER_AMD_V4_PLAN_H_
#define K8S_GPU_NODE_CHECKER_AMD_V4_PLAN_H_

// The K-tile's schedule as a plan over its 128 MFMA slots (slot i < 64: MFMA i on F0, the rest on F1).  After
// slot i's MFMA come, in this order: fragment read read(i) (0-15: F1 piece, from this tile's stage; 16-31: F0'
// piece of tile kt+1, from the other stage), wait(i) (1: lgkmcnt(0) + s_barrier, 2: vmcnt(vm(i)) + s_barrier) and
// LDS-DMA dma(i) (piece j of tile kt+2 into this tile's stage).  v4_plan_ok checks a plan at compile time: every
// F1 read retired (lgkmcnt barrier) before slot 64 and before any DMA into its operand's region, every F0' read
// after the vmcnt barrier that retires the previous K-tile's DMAs, vm = the DMAs issued since, 16 DMAs in all.
struct V4Slot {
  int read = -1, wait = 0, vm = 0, dma = -1;
};

// Plan A (knobs; the shipped values won tools/gemm_w4a_lab.hip's sweeps at 4096^3 and 8192^3):
//   RS    half 1 issues one F1 read after every RS-th MFMA (16 reads: the A pieces, then the B pieces)
//   X_AT  the slot after which lgkmcnt(0) + barrier X are taken (>= 16 * RS - 1)
//   D1    DMA pieces issued in half 1 after X, evenly; the other 16 - D1 in half 2 after Y
//   Y_AT  the slot of half 2 after which vmcnt(D1) + barrier Y are taken; F0' reads follow, one per R2 MFMAs
template <int RS, int X_AT, int D1, int Y_AT, int R2>
struct V4PlanA {
  static constexpr V4Slot at(int i) {
    V4Slot o;
    constexpr int SP1 = D1 > 0 ? (63 - X_AT) / D1 : 1, D2 = 16 - D1, SP2 = D2 > 0 ? (63 - Y_AT) / D2 : 1;
    if (i < 64) {
      if (i % RS == RS - 1 && i / RS < 16) o.read = i / RS;
      if (i == X_AT) o.wait = 1;
      if (i > X_AT && (i - X_AT) % SP1 == 0 && (i - X_AT) / SP1 - 1 < D1) o.dma = (i - X_AT) / SP1 - 1;
    } else {
      const int h = i - 64;
      if (h == Y_AT) {
        o.wait = 2;
        o.vm = D1;
      }
      if (h > Y_AT && (h - Y_AT - 1) % R2 == 0 && (h - Y_AT - 1) / R2 < 16) o.read = 16 + (h - Y_AT - 1) / R2;
      if (D2 > 0 && h > Y_AT && (h - Y_AT) % SP2 == 0 && (h - Y_AT) / SP2 - 1 < D2) o.dma = D1 + (h - Y_AT) / SP2 - 1;
    }
    return o;
  }
};

// Plan A2: plan A with the half-2 DMA pieces issued from slot H2S of half 2 on (after the F0' reads, say), so an
// MFMA gap carries a read or a DMA, not both (an LDS-DMA's issue costs ~60-185 cycles depending on what else its
// gap issues: MI355X_MICROARCH.md)
template <int RS, int X_AT, int D1, int Y_AT, int R2, int H2S>
struct V4PlanA2 {
  static constexpr V4Slot at(int i) {
    V4Slot o = V4PlanA<RS, X_AT, D1, Y_AT, R2>::at(i);
    if (i >= 64) {
      const int h = i - 64;
      constexpr int D2 = 16 - D1, SP = D2 > 0 ? (63 - H2S) / D2 + ((63 - H2S) / D2 == 0) : 1;
      o.dma = -1;
      if (D2 > 0 && h >= H2S && (h - H2S) % SP == 0 && (h - H2S) / SP < D2) o.dma = D1 + (h - H2S) / SP;
    }
    return o;
  }
};

// Plan S (hipBLASLt's order, read from its gfx950 MT256x256x64 kernel): the A pieces of F1 one per 2 MFMAs, barrier
// X1 (XA), then the B pieces of F1 one per 2 MFMAs with the A-operand DMAs between them, barrier X2 (XB), the
// B-operand DMAs one per BSP MFMAs, barrier Y (slot 64 + Y_AT) retiring the previous K-tile, F0' one per 2 MFMAs.
template <int XA, int XB, int BSP, int Y_AT>
struct V4PlanS {
  static constexpr V4Slot at(int i) {
    V4Slot o;
    if (i < 16 && i % 2 == 0) o.read = i / 2;                                       // A pieces 0-7
    if (i == XA) o.wait = 1;                                                         // X1
    if (i > XA && i <= XA + 16 && (i - XA) % 2 == 1) o.read = 8 + (i - XA) / 2;     // B pieces 8-15
    if (i > XA && i <= XA + 16 && (i - XA) % 2 == 0) o.dma = (i - XA) / 2 - 1;       // A DMAs 0-7
    if (i == XB) o.wait = 1;                                                         // X2
    if (i > XB && (i - XB) % BSP == 0 && (i - XB) / BSP <= 8) o.dma = 7 + (i - XB) / BSP;  // B DMAs 8-15
    const int y = 64 + Y_AT;
    if (i == y) {
      o.wait = 2;
      int n = 0;
      for (int k = 0; k < y; ++k)
        if (at_dma(k) >= 0) ++n;
      o.vm = n;
    }
    if (i > y && (i - y - 1) % 2 == 0 && (i - y - 1) / 2 < 16) o.read = 16 + (i - y - 1) / 2;
    return o;
  }
  static constexpr int at_dma(int i) {
    if (i > XA && i <= XA + 16 && (i - XA) % 2 == 0) return (i - XA) / 2 - 1;
    if (i > XB && (i - XB) % BSP == 0 && (i - XB) / BSP <= 8) return 7 + (i - XB) / BSP;
    return -1;
  }
};

template <class P>
constexpr bool v4_plan_ok() {
  int read_at[32] = {}, dma_at[16] = {}, lgk_barriers[128] = {}, vm_at = -1, vm = -1, nb = 0;
  for (int k = 0; k < 32; ++k) read_at[k] = -1;
  for (int k = 0; k < 16; ++k) dma_at[k] = -1;
  for (int i = 0; i < 128; ++i) {
    const V4Slot o = P::at(i);
    if (o.read >= 0) {
      if (o.read > 31 || read_at[o.read] >= 0) return false;
      read_at[o.read] = i;
    }
    if (o.wait == 1) lgk_barriers[nb++] = i;
    if (o.wait == 2) {
      if (vm_at >= 0) return false;
      vm_at = i;
      vm = o.vm;
    }
    if (o.dma >= 0) {
      if (o.dma > 15 || dma_at[o.dma] >= 0) return false;
      dma_at[o.dma] = i;
    }
  }
  if (vm_at < 0) return false;
  int issued = 0;
  for (int k = 0; k < 16; ++k) {
    if (dma_at[k] < 0) return false;
    if (dma_at[k] < vm_at) ++issued;
  }
  if (issued != vm) return false;
  // the first lgkmcnt barrier after slot t (or -1)
  auto barrier_after = [&](int t) {
    for (int b = 0; b < nb; ++b)
      if (lgk_barriers[b] >= t) return lgk_barriers[b];
    return -1;
  };
  for (int k = 0; k < 16; ++k) {
    const int b = barrier_after(read_at[k]);  // F1 piece k retired here (same slot: read, then the wait)
    if (read_at[k] < 0 || b < 0 || b >= 64) return false;
    // DMAs into the piece's operand region (A: pieces / DMAs 0-7, B: 8-15) only after that barrier
    for (int j = (k < 8 ? 0 : 8); j < (k < 8 ? 8 : 16); ++j)
      if (dma_at[j] <= b) return false;
  }
  for (int k = 16; k < 32; ++k)
    if (read_at[k] <= vm_at) return false;
  return true;
}

// fp8 slot i (0-63) -> output block: quadrant q = i / 16 in the order (A0-3, B0-3), (A4-7, B0-3), (A0-3, B4-7),
// (A4-7, B4-7)
constexpr int v4f8_m(int i) { return ((i >> 4) & 1) * 4 + ((i & 15) >> 2); }
constexpr int v4f8_n(int i) { return ((i >> 4) >> 1) * 4 + (i & 3); }

// fp8 plan: this tile's A4-7 reads in slots 0-7, barrier X1 at X1, its B4-7 reads in X1+1 .. X1+8 with the A-operand
// DMAs every second slot from DA, barrier X2 at X2, the B-operand DMAs every second slot from DB, barrier Y at Y
// (vmcnt: the previous K-tile's DMAs), then the next tile's B0-3 and (from slot 48, after their last use) A0-3
template <int X1, int DA, int X2, int DB, int Y>
struct V4PlanF8 {
  static constexpr int at_dma(int i) {
    if (i >= DA && i < DA + 16 && (i - DA) % 2 == 0) return (i - DA) / 2;
    if (i >= DB && i < DB + 16 && (i - DB) % 2 == 0) return 8 + (i - DB) / 2;
    return -1;
  }
  static constexpr V4Slot at(int i) {
    V4Slot o;
    if (i < 8) o.read = i;                                 // this tile's A4-7
    if (i > X1 && i <= X1 + 8) o.read = 8 + (i - X1 - 1);  // this tile's B4-7
    if (i > Y && i <= Y + 8) o.read = 24 + (i - Y - 1);    // next tile's B0-3
    const int a0 = (Y + 9 > 48 ? Y + 9 : 48);
    if (i >= a0 && i < a0 + 8) o.read = 16 + (i - a0);     // next tile's A0-3
    if (i == X1 || i == X2) o.wait = 1;
    if (i == Y) {
      o.wait = 2;
      for (int k = 0; k < Y; ++k)
        if (at_dma(k) >= 0) ++o.vm;
    }
    o.dma = at_dma(i);
    return o;
  }
};

// the fp8 plan rules (slot i: MFMA, read, wait, DMA): this tile's A4-7 / B4-7 reads retired by an lgkmcnt barrier
// before their first MFMA (slot 16 / 32) and before any DMA into their operand's region; the next tile's reads
// after the vmcnt barrier and no earlier than the last MFMA of the fragment they replace (B0-3: 31, A0-3: 47)
template <class P>
constexpr bool v4f8_plan_ok() {
  int read_at[32] = {}, dma_at[16] = {}, lgk[64] = {}, nb = 0, vm_at = -1, vm = -1;
  for (int k = 0; k < 32; ++k) read_at[k] = -1;
  for (int k = 0; k < 16; ++k) dma_at[k] = -1;
  for (int i = 0; i < 64; ++i) {
    const V4Slot o = P::at(i);
    if (o.read >= 0) {
      if (o.read > 31 || read_at[o.read] >= 0) return false;
      read_at[o.read] = i;
    }
    if (o.wait == 1) lgk[nb++] = i;
    if (o.wait == 2) {
      if (vm_at >= 0) return false;
      vm_at = i;
      vm = o.vm;
    }
    if (o.dma >= 0) {
      if (o.dma > 15 || dma_at[o.dma] >= 0) return false;
      dma_at[o.dma] = i;
    }
  }
  if (vm_at < 0) return false;
  int issued = 0;
  for (int k = 0; k < 16; ++k) {
    if (dma_at[k] < 0) return false;
    issued += dma_at[k] < vm_at;
  }
  if (issued != vm) return false;
  for (int op = 0; op < 2; ++op) {
    int last = -1;
    for (int k = op * 8; k < op * 8 + 8; ++k) last = read_at[k] > last ? read_at[k] : last;
    int b = -1;
    for (int x = 0; x < nb && b < 0; ++x)
      if (lgk[x] >= last) b = lgk[x];
    if (last < 0 || b < 0 || b >= (op ? 32 : 16)) return false;
    for (int j = op * 8; j < op * 8 + 8; ++j)
      if (dma_at[j] <= b) return false;
  }
  for (int k = 16; k < 32; ++k)
    if (read_at[k] <= vm_at || read_at[k] < (k < 24 ? 47 : 31)) return false;
  return true;
}

// Grouped m0 (gemm_v4_kernel<..., M0G>): DMA pieces 4g .. 4g+3 share one m0, set by piece 4g, so within a
// K-tile every piece 4g+t (t > 0) must be the next DMA issued after piece 4g+t-1 (slot order, 128 slots).
template <class P>
constexpr bool v4_m0_groups_ok() {
  int prev = -1;
  for (int i = 0; i < 128; ++i) {
    const int d = P::at(i).dma;
    if (d < 0) continue;
    if ((d & 3) != 0 && prev != d - 1) return false;
    prev = d;
  }
  return true;
}

#endif  // K8S_GPU_NODE_CHECKER_AMD_V4_PLAN_H_
