"""Host-side ASan/UBSan builds of the native CPU code (SURVEY §5 "Race detection / sanitizers").

The fast-path extension is rebuilt with ``-fsanitize=address,undefined`` into a
temp dir and the fuzzed native-vs-Python equivalence suite runs against it in
a child interpreter with the sanitizer runtimes preloaded.  (GPU sanitizers
are not available for the HIP library on this pool; see BENCH.md.)
"""
import os
import shutil
import subprocess
import sys
import sysconfig

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rt(name):
    p = subprocess.run(["g++", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


@pytest.mark.slow
def test_fastpath_under_asan_ubsan(tmp_path):
    if not shutil.which("g++"):
        pytest.skip("no g++")
    asan, ubsan = _rt("libasan.so"), _rt("libubsan.so")
    if not asan or not ubsan:
        pytest.skip("sanitizer runtimes not installed")
    out = tmp_path / ("_fastpath" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))
    src = os.path.join(REPO, "k8s_gpu_node_checker_amd", "csrc", "fastpath", "fastpath.cpp")
    r = subprocess.run(["g++", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
                        "-fno-sanitize-recover=undefined", "-std=c++17", "-shared", "-fPIC", "-I",
                        sysconfig.get_paths()["include"], src, "-o", str(out)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    # the sanitizer runtimes go first (ASan must be the first DSO); anything already preloaded stays
    preload = " ".join(x for x in (asan, ubsan, os.environ.get("LD_PRELOAD", "")) if x)
    env = dict(os.environ, K8SGPU_NATIVE_DIR=str(tmp_path), LD_PRELOAD=preload,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    which = subprocess.run([sys.executable, "-c", "from k8s_gpu_node_checker_amd.ops import fastpath; "
                            "print(fastpath.ext().__file__)"], capture_output=True, text=True, env=env, cwd=REPO)
    assert which.stdout.strip() == str(out), (which.stdout, which.stderr[-1000:])
    p = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        os.path.join(REPO, "tests", "test_fastpath.py")], capture_output=True, text=True, env=env,
                       cwd=REPO, timeout=600)
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-3000:])
    assert "passed" in p.stdout
