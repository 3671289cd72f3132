"""Host-side ASan/UBSan builds of the native CPU code (SURVEY §5 "Race detection / sanitizers").

The C++ amd-smi probe (csrc/probe) is built with ASan/UBSan and TSan against a replay stub of
libamd_smi (tests/amdsmi_stub) that serves a recorded MI355X probe and the DRIVER_NOT_LOADED / NO_PERM
error statuses.  The fast-path extension is rebuilt with ``-fsanitize=address,undefined`` into a
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
                        os.path.join(REPO, "tests", "test_fastpath.py"), os.path.join(REPO, "tests", "test_native_loads.py")],
                       capture_output=True, text=True, env=env,
                       cwd=REPO, timeout=600)
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-3000:])
    assert "passed" in p.stdout


# --- the C++ amd-smi probe (csrc/probe) under ASan/UBSan and TSan, against a replay stub of libamd_smi ---

STUB_DIR = os.path.join(REPO, "tests", "amdsmi_stub")
PROBE_DIR = os.path.join(REPO, "k8s_gpu_node_checker_amd", "csrc", "probe")
RECORDED = os.path.join(STUB_DIR, "mi355x_probe_recorded.json")  # mi355x-probe on an MI355X box (round 2)
SAN = ["-O1", "-g", "-fno-omit-frame-pointer", "-std=c++17", "-Wall", "-Wextra", "-I", "/opt/rocm/include"]
ASAN_ENV = {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1", "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"}


def _recorded_gpu():
    import json
    with open(RECORDED) as f:
        return json.load(f)["gpus"][0]


def scenario(path, gpus=8, init_status=0, per_gpu=None):
    """The stub's key=value scenario: the recorded MI355X replicated to ``gpus`` OAMs (distinct BDFs /
    UUIDs / KFD nodes), with ``per_gpu[i]`` overriding fields of GPU i."""
    import json
    with open(RECORDED) as f:
        rec = json.load(f)
    g0 = rec["gpus"][0]
    lines = [f"init_status={init_status}", f"gpus={gpus}"]
    if (rec.get("driver") or {}).get("version"):
        lines.append(f"driver_version={rec['driver']['version']}")

    def flat(prefix, v):  # nested objects (fw, ecc_blocks, throttle_acc) become dotted keys, lists commas
        if isinstance(v, dict):
            for a, b in v.items():
                flat(f"{prefix}.{a}", b)
        elif isinstance(v, list):
            lines.append(f"{prefix}={','.join(str(x) for x in v)}")
        else:
            lines.append(f"{prefix}={v}")
    bdfs = [f"0000:{0x05 + 0x10 * i:02x}:00.0" for i in range(gpus)]
    for i in range(gpus):
        g = dict(g0)
        g["bdf"] = bdfs[i]
        g["uuid"] = g0["uuid"][:-2] + f"{i:02x}"
        g["kfd_node"] = 2 + i
        g["xgmi_peers"] = [b for b in bdfs if b != bdfs[i]]  # one board: every link reaches another GPU of it
        g.update((per_gpu or {}).get(i, {}))
        g = {k: v for k, v in g.items() if v is not None}
        for k, v in g.items():
            if k in ("index", "probe_us", "processes", "kfd", "xgmi_kb"):
                continue
            if k == "procs":
                v = ",".join(f"{p['pid']}:{p['vram_mb']}" for p in v)
            flat(f"gpu.{i}.{k}", v)
    path.write_text("\n".join(lines) + "\n")
    return str(path)


def _need(*names):
    if not shutil.which("g++") or not os.path.exists("/opt/rocm/include/amd_smi/amdsmi.h"):
        pytest.skip("needs g++ and the amd-smi headers")
    rts = [_rt(n) for n in names]
    if not all(rts):
        pytest.skip("sanitizer runtimes not installed")
    return rts


def _gxx(args):
    r = subprocess.run(["g++"] + args, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]


@pytest.fixture(scope="module")
def asan_probe(tmp_path_factory):
    """libamd_smi.so (stub), libmi355x_probe.so and mi355x-probe, all built with -fsanitize=address,undefined."""
    asan, ubsan = _need("libasan.so", "libubsan.so")
    d = tmp_path_factory.mktemp("probe_asan")
    flags = SAN + ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"]
    _gxx(flags + ["-shared", "-fPIC", os.path.join(STUB_DIR, "amdsmi_stub.cpp"), "-o", str(d / "libamd_smi.so")])
    # DT_RPATH (not RUNPATH): found before LD_LIBRARY_PATH, which may name /opt/rocm/lib's real library
    link = ["-L", str(d), "-lamd_smi", f"-Wl,-rpath,{d}", "-Wl,--disable-new-dtags"]
    _gxx(flags + ["-shared", "-fPIC", os.path.join(PROBE_DIR, "probe.cpp"), "-o", str(d / "libmi355x_probe.so")] + link)
    _gxx(flags + [os.path.join(PROBE_DIR, "probe_main.cpp"), os.path.join(PROBE_DIR, "probe.cpp"),
                  "-o", str(d / "mi355x-probe")] + link)
    return d, asan, ubsan


def _run_cli(d, scen, *args):
    env = dict(os.environ, AMDSMI_STUB_SCENARIO=scen, **ASAN_ENV)
    env.pop("LD_PRELOAD", None)  # an executable linked with -fsanitize loads its runtime itself
    return subprocess.run([str(d / "mi355x-probe"), "--node", "n1"] + list(args), capture_output=True, text=True,
                          env=env, timeout=120)


@pytest.mark.slow
def test_probe_cli_under_asan_replays_recorded_mi355x(asan_probe, tmp_path):
    import json

    from k8s_gpu_node_checker_amd.models import health as H
    d, _, _ = asan_probe
    # GPU 3 holds 100 processes (past the probe's 64-entry buffer: the OUT_OF_RESOURCES branch)
    scen = scenario(tmp_path / "s.txt", per_gpu={3: {"nprocs": 100}})
    p = _run_cli(d, scen, "--repeat", "3")
    assert p.returncode == 0 and "ERROR: AddressSanitizer" not in p.stderr and "runtime error" not in p.stderr, \
        p.stderr[-3000:]
    docs = [json.loads(x) for x in p.stdout.splitlines()]
    assert len(docs) == 3
    rec = _recorded_gpu()
    rep = docs[-1]
    assert rep["schema"] == "mi355x-health/v1" and rep["node"] == "n1" and len(rep["gpus"]) == 8
    for i, g in enumerate(rep["gpus"]):
        assert g["index"] == i and g["bdf"] == f"0000:{0x05 + 0x10 * i:02x}:00.0" and g["kfd_node"] == 2 + i
        for k in ("gfx", "market_name", "product_name", "vbios_name", "device_id", "cus", "vram_type", "vram_mb",
                  "ecc_uncorrectable", "bad_pages", "xgmi", "compute_partition", "memory_partition", "pcie_width",
                  "pcie_max_speed_mts", "power_w", "power_cap_w", "power_cap_default_w", "vram_used_mb",
                  "gfx_activity", "hbm_temp_c", "gfxclk_mhz", "throttle_acc"):
            assert g[k] == rec[k], (i, k, g[k], rec[k])
    assert rep["gpus"][3]["processes"] == 100 and len(rep["gpus"][3]["procs"]) == 64
    assert rep["gpus"][0]["procs"] == rec["procs"]
    v = H.evaluate_report(rep, 8, H.HealthExpectations(xgmi_links=7), now=rep["ts"])
    assert v.state == H.HEALTHY and (v.gpus_ok, v.gpus_seen) == (8, 8), v.to_dict()


@pytest.mark.slow
@pytest.mark.parametrize("status,name", [(34, "AMDSMI_STATUS_DRIVER_NOT_LOADED"), (10, "AMDSMI_STATUS_NO_PERM")])
def test_probe_cli_under_asan_maps_init_errors_to_unknown(asan_probe, tmp_path, status, name):
    import json

    from k8s_gpu_node_checker_amd.models import health as H
    d, _, _ = asan_probe
    p = _run_cli(d, scenario(tmp_path / "s.txt", init_status=status))
    assert p.returncode == 1, (p.stdout, p.stderr[-2000:])  # the CLI's "amd-smi could not be initialised"
    assert "ERROR: AddressSanitizer" not in p.stderr and "runtime error" not in p.stderr
    rep = json.loads(p.stdout)
    assert rep["error"] == name and rep["gpus"] == []
    v = H.evaluate_report(rep, 8, now=rep["ts"])
    assert v.state == H.UNKNOWN and v.reasons == [f"probe failed: {name}"]


@pytest.mark.slow
def test_probe_c_abi_under_asan_from_python(asan_probe, tmp_path):
    """The ctypes path the agent uses (ops/amdsmi_probe.probe_native), sanitized library preloaded; one
    GPU whose asic query fails (NO_PERM) is reported per GPU, the others still probed."""
    d, asan, ubsan = asan_probe
    scen = scenario(tmp_path / "s.txt", gpus=4, per_gpu={2: {"asic_status": 10}, 1: {"xgmi": "XUUDUUUU"}})
    code = ("import json; from k8s_gpu_node_checker_amd.ops import amdsmi_probe as P; "
            "from k8s_gpu_node_checker_amd.models import health as H\n"
            "for _ in range(5): r = P.probe_native('n2')\n"
            "v = H.evaluate_report(r, 4, H.HealthExpectations(xgmi_links=7), now=r['ts'])\n"
            "print(json.dumps({'errors': [g.get('error') for g in r['gpus']], 'state': v.state, 'reasons': v.reasons,"
            " 'ok': v.gpus_ok, 'seen': v.gpus_seen}))")
    preload = " ".join(x for x in (asan, ubsan, os.environ.get("LD_PRELOAD", "")) if x)
    env = dict(os.environ, K8SGPU_NATIVE_DIR=str(d), AMDSMI_STUB_SCENARIO=scen, LD_PRELOAD=preload,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS=ASAN_ENV["UBSAN_OPTIONS"])
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, cwd=REPO, timeout=120)
    assert p.returncode == 0 and "runtime error" not in p.stderr, p.stderr[-3000:]
    import json
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["errors"] == [None, None, "AMDSMI_STATUS_NO_PERM", None]
    assert out["state"] == "unhealthy" and (out["ok"], out["seen"]) == (2, 4)
    assert "gpu2: probe error AMDSMI_STATUS_NO_PERM" in out["reasons"]
    assert any(r.startswith("gpu1: 1 xGMI link(s) down") for r in out["reasons"])


@pytest.mark.slow
def test_probe_concurrent_calls_under_tsan(tmp_path):
    """8 threads interleaving open / json / gpu_count / close (the agent's probe loop, its HTTP handlers
    and a shutdown) must be race-free: the probe's mutex covers every amd-smi call and handle."""
    _need("libtsan.so")
    flags = SAN + ["-fsanitize=thread", "-pthread"]
    _gxx(flags + ["-shared", "-fPIC", os.path.join(STUB_DIR, "amdsmi_stub.cpp"), "-o", str(tmp_path / "libamd_smi.so")])
    _gxx(flags + ["-I", PROBE_DIR, os.path.join(STUB_DIR, "probe_stress.cpp"), os.path.join(PROBE_DIR, "probe.cpp"),
                  "-o", str(tmp_path / "probe_stress"), "-L", str(tmp_path), "-lamd_smi", f"-Wl,-rpath,{tmp_path}",
                  "-Wl,--disable-new-dtags"])
    env = dict(os.environ, AMDSMI_STUB_SCENARIO=scenario(tmp_path / "s.txt"), TSAN_OPTIONS="halt_on_error=1")
    env.pop("LD_PRELOAD", None)
    p = subprocess.run([str(tmp_path / "probe_stress"), "8", "40"], capture_output=True, text=True, env=env,
                       timeout=300)
    assert p.returncode == 0 and "WARNING: ThreadSanitizer" not in p.stderr, p.stderr[-4000:]
    assert '"bad_documents":0' in p.stdout and '"threads":8' in p.stdout


@pytest.mark.slow
def test_probe_cli_under_asan_firmware_ras_blocks_xgmi_error(asan_probe, tmp_path):
    """The probe's per-block ECC read (only when the totals are non-zero), the firmware table (read once
    per open, reused across probes) and the xGMI error status, under ASan/UBSan; the verdict names the
    failing block and the half-updated GPU."""
    import json

    from k8s_gpu_node_checker_amd.models import health as H
    d, _, _ = asan_probe
    rec = _recorded_gpu()
    fw5 = dict(rec["fw"], psp_sos=rec["fw"]["psp_sos"] - 47)
    scen = scenario(tmp_path / "s.txt", per_gpu={5: {"ecc_uncorrectable": 3, "ecc_correctable": 2, "fw": fw5,
                                                     "ecc_blocks": {"umc": {"ce": 2, "ue": 3, "de": 0}},
                                                     "xgmi_error": 1}})
    p = _run_cli(d, scen, "--repeat", "2")
    assert p.returncode == 0 and "ERROR: AddressSanitizer" not in p.stderr and "runtime error" not in p.stderr, \
        p.stderr[-3000:]
    r = json.loads(p.stdout.splitlines()[-1])
    assert r["driver"]["name"] == "amdgpu" and r["driver"]["version"]
    g5, g0 = r["gpus"][5], r["gpus"][0]
    assert g5["ecc_blocks"] == {"umc": {"ce": 2, "ue": 3, "de": 0}} and "ecc_blocks" not in g0
    assert g5["xgmi_error"] == 1 and g5["fw"] == fw5 and g0["fw"] == rec["fw"]
    assert "xgmi_error" not in g0 or g0["xgmi_error"] == 0
    v = H.evaluate_report(r, 8, H.HealthExpectations(xgmi_links=7), now=r["ts"])
    assert v.state == H.UNHEALTHY and v.reasons == ["gpu5: 3 uncorrectable ECC errors (umc 3)"]
    assert "gpu5: xGMI error status errors" in v.warnings
    assert any(w.startswith("firmware differs across GPUs: psp_sos: gpu0-4,6,7") or
               w.startswith("firmware differs across GPUs: psp_sos: gpu0-4,6-7") for w in v.warnings), v.warnings


@pytest.mark.slow
def test_probe_cli_under_asan_pages_cper_records(asan_probe, tmp_path):
    """CPER records walked page by page (71 records > the probe's 64 header slots: MORE_DATA + cursor), every
    header pointer bounds-checked against the buffer, severities counted, newest timestamp kept; a
    NO_PERM GPU reports cper_error."""
    import json

    from k8s_gpu_node_checker_amd.models import health as H
    d, _, _ = asan_probe
    recs = ",".join([f"2@2610160900{i % 60:02d}" for i in range(70)] + ["1@20261016101500"])
    scen = scenario(tmp_path / "s.txt", gpus=2, per_gpu={0: {"cper_entries": recs, "cper_error": None},
                                                         1: {"cper_error": "AMDSMI_STATUS_NO_PERM"}})
    p = _run_cli(d, scen)
    assert p.returncode == 0 and "ERROR: AddressSanitizer" not in p.stderr and "runtime error" not in p.stderr, \
        p.stderr[-3000:]
    r = json.loads(p.stdout)
    assert r["gpus"][0]["cper"] == {"uncorrected": 0, "fatal": 1, "corrected": 70,
                                    "last_fatal": "2026-10-16T10:15:00Z", "last_corrected": "2026-10-16T09:00:59Z"}
    assert r["gpus"][1]["cper_error"] == "AMDSMI_STATUS_NO_PERM" and "cper" not in r["gpus"][1]
    r["ts"] = H.parse_k8s_time("2026-10-16T12:00:00Z")  # records are aged against the report's own time: pin it
    v = H.evaluate_report(r, 2, H.HealthExpectations(xgmi_links=0), now=H.parse_k8s_time("2026-10-16T12:00:00Z"))
    assert v.reasons == ["gpu0: fatal RAS error record (CPER) at 2026-10-16T10:15:00Z"], v.to_dict()


@pytest.mark.slow
def test_probe_cli_under_asan_retired_pages_threshold_eeprom(asan_probe, tmp_path):
    """Retired HBM pages by status, the driver's threshold and the RAS EEPROM checksum (root-only: NO_PERM
    leaves them out); the EEPROM is validated once per GPU while the page count stands still."""
    import json

    from k8s_gpu_node_checker_amd.models import health as H
    d, _, _ = asan_probe
    scen = scenario(tmp_path / "s.txt", gpus=3, per_gpu={
        0: {"bad_pages": 5, "bad_page_status": "rrppu", "bad_page_threshold": 10, "ras_eeprom": "ok"},
        1: {"bad_pages": 9, "bad_page_threshold": 10, "ras_eeprom": "corrupted"},
        2: {"bad_page_threshold": "noperm", "ras_eeprom": "noperm"}})
    log = tmp_path / "eeprom.log"
    env = dict(os.environ, AMDSMI_STUB_SCENARIO=scen, AMDSMI_STUB_EEPROM_LOG=str(log), **ASAN_ENV)
    env.pop("LD_PRELOAD", None)
    p = subprocess.run([str(d / "mi355x-probe"), "--node", "n1", "--repeat", "3"], capture_output=True, text=True,
                       env=env, timeout=120)
    assert p.returncode == 0 and "ERROR: AddressSanitizer" not in p.stderr and "runtime error" not in p.stderr, \
        p.stderr[-3000:]
    r = json.loads(p.stdout.splitlines()[-1])
    pick = ("bad_pages", "bad_pages_pending", "bad_pages_unreservable", "bad_page_threshold", "ras_eeprom")
    got = [{k: g[k] for k in pick if k in g} for g in r["gpus"]]
    assert got == [{"bad_pages": 5, "bad_pages_pending": 2, "bad_pages_unreservable": 1, "bad_page_threshold": 10,
                    "ras_eeprom": "ok"},
                   {"bad_pages": 9, "bad_pages_pending": 0, "bad_pages_unreservable": 0, "bad_page_threshold": 10,
                    "ras_eeprom": "corrupted"},
                   {"bad_pages": 0}]
    assert log.read_text().count("validate") == 3  # once per GPU over 3 probes: the count did not move
    v = H.evaluate_report(r, 3, H.HealthExpectations(xgmi_links=0), now=r["ts"])
    assert v.state == H.UNHEALTHY
    assert v.reasons == ["gpu0: 1 bad HBM page(s) could not be retired (still in use)",
                         "gpu1: RAS EEPROM checksum invalid (the retired-page list may not survive a reboot)"]
    assert "gpu0: 2 bad HBM page(s) pending retirement (retired at the next GPU reset)" in v.warnings
    assert "gpu1: 9 retired pages, 10 is the driver's threshold" in v.warnings


@pytest.mark.slow
def test_probe_reenumerates_after_a_repartition_or_a_lost_gpu(asan_probe, tmp_path):
    """The amd-smi session is re-opened when it is older than the re-open interval (a repartition turned
    2 GPUs into 3 processors here) and right after a probe in which a GPU stopped answering -- once: a GPU
    that still fails in the fresh session does not re-open it every probe."""
    d, asan, ubsan = asan_probe
    scen = tmp_path / "s.txt"
    scenario(scen, gpus=2)
    log = tmp_path / "init.log"
    code = f"""
import json, time, shutil
from k8s_gpu_node_checker_amd.ops import amdsmi_probe as P
L = P._native()
L.mi355x_probe_set_reopen_interval.argtypes = [__import__('ctypes').c_double]
out = []
L.mi355x_probe_set_reopen_interval(0.5)
out.append(len(P.probe_native('n')['gpus']))
shutil.copy({str(tmp_path / 's3.txt')!r}, {str(scen)!r})
out.append(len(P.probe_native('n')['gpus']))   # session younger than 0.5 s: still 2
time.sleep(0.6)
out.append(len(P.probe_native('n')['gpus']))   # re-opened: 3
shutil.copy({str(tmp_path / 'sbad.txt')!r}, {str(scen)!r})
time.sleep(0.6)
r = P.probe_native('n'); out.append([g.get('error') for g in r['gpus']])  # re-opened by age, GPU 1 fails
L.mi355x_probe_set_reopen_interval(0)
for _ in range(3):
    P.probe_native('n')
print(json.dumps(out))
"""
    scenario(tmp_path / "s3.txt", gpus=3)
    scenario(tmp_path / "sbad.txt", gpus=2, per_gpu={1: {"asic_status": 10}})
    preload = " ".join(x for x in (asan, ubsan, os.environ.get("LD_PRELOAD", "")) if x)
    env = dict(os.environ, K8SGPU_NATIVE_DIR=str(d), AMDSMI_STUB_SCENARIO=str(scen), AMDSMI_STUB_INIT_LOG=str(log),
               LD_PRELOAD=preload, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS=ASAN_ENV["UBSAN_OPTIONS"])
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, cwd=REPO, timeout=120)
    assert p.returncode == 0 and "runtime error" not in p.stderr, p.stderr[-3000:]
    import json
    assert json.loads(p.stdout.splitlines()[-1]) == [2, 2, 3, [None, "AMDSMI_STATUS_NO_PERM"]]
    # opens: first, age (3 GPUs), age (bad GPU), once more after the failing probe, then no more
    assert log.read_text().count("init") == 4
