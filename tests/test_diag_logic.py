"""ops/diag.py verdict logic on CPU: a fake C ABI stands in for libmi355x_diag.so (the real kernels
run under tests/test_gpu.py on the MI355X)."""
import ctypes

import pytest

from k8s_gpu_node_checker_amd.ops import diag


class FakeLib:
    """Implements the C ABI calls with scripted results (out-params written through ctypes)."""

    def __init__(self, mfma=None, link=(56.8, 56.7), rc=0, err=b"boom"):
        self.mfma = mfma or {0: (1900.0, 0), 1: (1950.0, 0), 2: (4300.0, 0), 3: (7600.0, 0)}
        self.link = link
        self.rc = rc
        self.err = err

    def diag_last_error(self):
        return self.err

    def diag_mfma_burn(self, device, kind, iters, reps, tflops, errors):
        if self.rc:
            return self.rc
        tf, e = self.mfma[kind]
        ctypes.cast(tflops, ctypes.POINTER(ctypes.c_double))[0] = tf
        ctypes.cast(errors, ctypes.POINTER(ctypes.c_ulonglong))[0] = e
        return 0

    def diag_host_link(self, device, nbytes, iters, h2d, d2h):
        ctypes.cast(h2d, ctypes.POINTER(ctypes.c_double))[0] = self.link[0]
        ctypes.cast(d2h, ctypes.POINTER(ctypes.c_double))[0] = self.link[1]
        return self.rc


@pytest.fixture
def fake(monkeypatch):
    def install(**kw):
        lib = FakeLib(**kw)
        monkeypatch.setattr(diag, "lib", lambda: lib)
        return lib
    return install


def test_mfma_burn_pass_and_each_failure_mode(fake):
    fake()
    r = diag.mfma_burn(0)
    assert r["pass"] and set(r["kinds"]) == {"bf16", "fp8", "mxfp8", "mxfp4"} and r["detail"] == ""
    fake(mfma={0: (1900.0, 0), 1: (1950.0, 0), 2: (4300.0, 3), 3: (7600.0, 0)})
    r = diag.mfma_burn(0)
    assert not r["pass"] and r["detail"] == "mxfp8: 3 wrong results"
    fake(mfma={0: (400.0, 0), 1: (1950.0, 0), 2: (4300.0, 0), 3: (7600.0, 0)})
    assert diag.mfma_burn(0)["detail"] == "bf16: 400 TFLOP/s"


def test_host_link_threshold(fake):
    fake()
    assert diag.host_link(0)["pass"]
    fake(link=(24.0, 56.0))  # a Gen4 / x8 link: half rate one way
    r = diag.host_link(0)
    assert not r["pass"] and "h2d 24.0" in r["detail"]


def test_c_abi_failure_raises_with_library_message(fake):
    fake(rc=-1, err=b"hipMalloc: out of memory")
    with pytest.raises(RuntimeError, match="out of memory"):
        diag.mfma_burn(0, kinds=("bf16",))


def test_run_turns_a_failing_test_into_a_verdict(fake, monkeypatch):
    fake()

    def broken(*a, **k):
        raise RuntimeError("mi355x diag failed (-1): hipMemcpy: illegal address")
    monkeypatch.setattr(diag, "gemm", broken)
    monkeypatch.setattr(diag, "gemm_fp8", lambda *a, **k: {"pass": True})
    monkeypatch.setattr(diag, "hbm", lambda *a, **k: {"pass": True})
    out = diag.run(1, 0)
    assert out["gemm"]["pass"] is False and "illegal address" in out["gemm"]["detail"]
    assert out["mfma"]["pass"] and out["hbm"]["pass"]
