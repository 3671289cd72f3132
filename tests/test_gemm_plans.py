"""The v4 GEMM's K-loop plans and their compile-time checks (``csrc/diag/v4_plan.h``), on the host compiler.

diag.hip instantiates ``gemm_v4_kernel`` only with plans that pass ``v4_plan_ok`` / ``v4f8_plan_ok`` (a
``static_assert``); a plan that breaks an ordering rule would otherwise be a data race between the LDS-DMA and the
fragment reads, or an MFMA on a fragment still in flight -- wrong numbers, not a crash.  Here the shipped plans are
accepted and plans broken in each way the checks cover are rejected.
"""
import json
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
HEADER = os.path.join(HERE, "..", "k8s_gpu_node_checker_amd", "csrc", "diag", "v4_plan.h")

DRIVER = r"""
#include <cstdio>
namespace {
#include "v4_plan.h"

using Good = V4PlanA<1, 20, 8, 8, 2>;

// plan A with one override applied to slot I
template <int I, int READ, int WAIT, int VM, int DMA, bool CLEAR_READ = false, bool CLEAR_DMA = false>
struct Edit {
  static constexpr V4Slot at(int i) {
    V4Slot o = Good::at(i);
    if (i == I) {
      if (READ >= 0) o.read = READ;
      if (CLEAR_READ) o.read = -1;
      if (WAIT >= 0) { o.wait = WAIT; o.vm = VM; }
      if (DMA >= 0) o.dma = DMA;
      if (CLEAR_DMA) o.dma = -1;
    }
    return o;
  }
};
// move slot FROM's DMA to slot TO
template <int FROM, int TO>
struct MoveDma {
  static constexpr V4Slot at(int i) {
    V4Slot o = Good::at(i);
    if (i == FROM) o.dma = -1;
    if (i == TO) o.dma = Good::at(FROM).dma;
    return o;
  }
};
// move slot FROM's read to slot TO
template <class P, int FROM, int TO>
struct MoveRead {
  static constexpr V4Slot at(int i) {
    V4Slot o = P::at(i);
    if (i == FROM) o.read = -1;
    if (i == TO) o.read = P::at(FROM).read;
    return o;
  }
};
template <class P, int FROM, int TO>
struct MoveDmaP {
  static constexpr V4Slot at(int i) {
    V4Slot o = P::at(i);
    if (i == FROM) o.dma = -1;
    if (i == TO) o.dma = P::at(FROM).dma;
    return o;
  }
};
// exchange the DMA pieces of slots A and B
template <class P, int A, int B>
struct SwapDma {
  static constexpr V4Slot at(int i) {
    V4Slot o = P::at(i);
    if (i == A) o.dma = P::at(B).dma;
    if (i == B) o.dma = P::at(A).dma;
    return o;
  }
};
using F8 = V4PlanF8<8, 10, 26, 27, 42>;
}  // namespace

int main() {
  std::printf("{");
  std::printf("\"shipped_bf16\": %d,", v4_plan_ok<Good>());
  std::printf("\"a2\": %d,", v4_plan_ok<V4PlanA2<1, 20, 8, 4, 1, 24>>());
  std::printf("\"hipblaslt_order\": %d,", v4_plan_ok<V4PlanS<16, 34, 3, 8>>());
  // the first DMA (slot 25, into the A region of this stage) moved before barrier X (slot 20)
  std::printf("\"dma_before_x\": %d,", v4_plan_ok<MoveDma<25, 10>>());
  // an F0' read (next tile, slot 73) moved before the vmcnt barrier Y (slot 72)
  std::printf("\"next_read_before_y\": %d,", v4_plan_ok<MoveRead<Good, 73, 70>>());
  // an F1 read (slot 15) moved after barrier X: its MFMAs (half 2) would read a fragment still in flight
  std::printf("\"f1_read_after_x\": %d,", v4_plan_ok<MoveRead<Good, 15, 40>>());
  // Y waiting for too few DMAs: vmcnt(9) when 8 of this K-tile's are younger
  std::printf("\"wrong_vmcnt\": %d,", v4_plan_ok<Edit<72, -1, 2, 9, -1>>());
  // a DMA dropped: the tile would be staged incompletely
  std::printf("\"missing_dma\": %d,", v4_plan_ok<Edit<25, -1, -1, 0, -1, false, true>>());
  // a read dropped
  std::printf("\"missing_read\": %d,", v4_plan_ok<Edit<3, -1, -1, 0, -1, true>>());
  std::printf("\"shipped_fp8\": %d,", v4f8_plan_ok<F8>());
  std::printf("\"fp8_late_y\": %d,", v4f8_plan_ok<V4PlanF8<8, 12, 30, 32, 48>>());
  // the next tile's A0-3 read moved to slot 45, before quadrant 2's last MFMA on A0-3 (slot 47)
  std::printf("\"fp8_next_a_early\": %d,", v4f8_plan_ok<MoveRead<F8, 51, 45>>());
  // a B DMA (slot 27) moved before barrier X2 (slot 26) retires this tile's B4-7 reads
  std::printf("\"fp8_b_dma_before_x2\": %d,", v4f8_plan_ok<MoveDmaP<F8, 27, 17>>());
  // grouped m0 (lab): plan A issues its DMA pieces in order; swapping two pieces of a group breaks it
  std::printf("\"m0_groups_shipped\": %d,", v4_m0_groups_ok<Good>());
  std::printf("\"m0_groups_swapped\": %d", v4_m0_groups_ok<SwapDma<Good, 25, 30>>());
  std::printf("}\n");
  return 0;
}
"""


@pytest.fixture(scope="module")
def verdicts(tmp_path_factory):
    cxx = shutil.which("g++") or shutil.which("c++")
    if not cxx:
        pytest.skip("no host C++ compiler")
    d = tmp_path_factory.mktemp("plans")
    src, exe = d / "plans.cpp", d / "plans"
    src.write_text(DRIVER)
    subprocess.run([cxx, "-std=c++17", "-O1", "-I", os.path.dirname(HEADER), str(src), "-o", str(exe)], check=True,
                   capture_output=True, text=True, timeout=120)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True, timeout=30).stdout
    return json.loads(out)


def test_shipped_plans_pass_their_checks(verdicts):
    assert verdicts["shipped_bf16"] == 1 and verdicts["shipped_fp8"] == 1
    assert verdicts["a2"] == 1 and verdicts["hipblaslt_order"] == 1
    assert verdicts["m0_groups_shipped"] == 1


@pytest.mark.parametrize("broken", ["dma_before_x", "next_read_before_y", "f1_read_after_x", "wrong_vmcnt",
                                    "missing_dma", "missing_read", "fp8_late_y", "fp8_next_a_early",
                                    "fp8_b_dma_before_x2", "m0_groups_swapped"])
def test_broken_plans_are_rejected(verdicts, broken):
    assert verdicts[broken] == 0, broken


@pytest.fixture
def diag_on_cpu():
    """The in-tree diag library, on a host without a GPU: only argument checks that return before any HIP call are
    exercised (on a GPU host these calls would launch, so the test is skipped there)."""
    torch = pytest.importorskip("torch")
    if torch.cuda.device_count() > 0:
        pytest.skip("GPU present: the guard is exercised by the GPU suite's shapes instead")
    from k8s_gpu_node_checker_amd.ops import diag
    try:
        diag.lib()
    except OSError as e:
        pytest.skip(f"diag library not loadable: {e}")
    return diag


@pytest.mark.parametrize("dtype,k", [("bf16", 1 << 23), ("fp8", 1 << 24)])
def test_v4_rejects_panels_past_32_bit_offsets(diag_on_cpu, dtype, k):
    """v4's buffer resources address a 256-row operand panel with 32-bit byte offsets: K >= 2^23 bf16 columns
    (2^24 fp8) is refused as an invalid argument (-2) before anything is launched."""
    diag = diag_on_cpu
    with diag.gemm_config(variant="v4"), pytest.raises(RuntimeError, match=r"\(-2\).*4 GiB"):
        if dtype == "bf16":
            diag.gemm_launch(1, 1, 1, 256, 256, k, 0)
        else:
            diag.gemm_fp8_launch(1, 1, 1, 256, 256, k, 0)
    with diag.gemm_config(variant="v4"), pytest.raises(RuntimeError, match=r"\(-2\).*4 GiB"):
        diag.gemm_launch_ck(dtype, 1, 1, 1, 1, 256, 256, k, 0)
