"""The shipped artefact installs and starts (R18 packaging; reference: /root/reference/pyproject.toml:1-11,
/root/reference/README.md:13-33).

The tree is installed the way ``deploy/Dockerfile`` installs it -- into a venv, offline, with
``pip install --no-build-isolation`` on this image's setuptools (59.6, pre-PEP 621) -- and every console
script the manifests run is started with the source tree off ``sys.path``.
"""
import glob
import os
import re
import shutil
import subprocess
import sys

import pytest
import yaml

from test_cli_golden import HELP

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = "k8s_gpu_node_checker_amd"
REF = os.environ.get("K8SGPU_REFERENCE", "/root/reference/check-gpu-node.py")
STUBS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "refstub")
SCRIPTS = ("check-gpu-node", "kubectl-gpu_node_checker", "k8s-gpu-node-agent", "mi355x-diag", "mi355x-fabric")


def _clean_env(**extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("PYTHONPATH", "SLACK_WEBHOOK_URL", "KUBECONFIG", "K8SGPU_NATIVE_DIR", "VIRTUAL_ENV")}
    env["COLUMNS"] = "80"
    env.update(extra)
    return env


@pytest.fixture(scope="module")
def venv(tmp_path_factory):
    """A copy of the built tree installed into a fresh venv: returns (venv dir, scratch cwd)."""
    base = tmp_path_factory.mktemp("install")
    src = base / "src"
    src.mkdir()
    for f in ("setup.py", "pyproject.toml", "README.md"):
        shutil.copy2(os.path.join(REPO, f), src / f)
    shutil.copytree(os.path.join(REPO, PKG), src / PKG,
                    ignore=shutil.ignore_patterns("__pycache__", "*.pyc", "*.tmp"))
    env_dir = base / "venv"
    # the image's venv has its own pip; this container has no ensurepip, so the venv borrows the system pip
    # (--system-site-packages) -- the install scheme is the venv's either way, which is what matters here
    subprocess.run([sys.executable, "-m", "venv", "--without-pip", "--system-site-packages", str(env_dir)],
                   check=True)
    py = str(env_dir / "bin" / "python")
    p = subprocess.run([py, "-m", "pip", "install", "--no-deps", "--no-build-isolation", "--no-index", str(src)],
                       capture_output=True, text=True, cwd=str(base), timeout=300,
                       env=_clean_env(K8SGNC_NATIVE_PREBUILT="1", PIP_DISABLE_PIP_VERSION_CHECK="1"))
    assert p.returncode == 0, p.stdout + p.stderr
    assert "UNKNOWN" not in p.stdout, p.stdout
    cwd = base / "cwd"
    cwd.mkdir()
    return env_dir, cwd


def _run(venv, argv, **kw):
    env_dir, cwd = venv
    return subprocess.run(argv, capture_output=True, text=True, cwd=str(cwd), env=_clean_env(HOME=str(cwd)),
                          timeout=120, **kw)


def test_distribution_is_named_and_versioned(venv):
    env_dir, _ = venv
    from k8s_gpu_node_checker_amd import __version__
    dists = [os.path.basename(d) for d in glob.glob(str(env_dir / "lib" / "python3*" / "site-packages" / "*.dist-info"))]
    assert f"k8s_gpu_node_checker_amd-{__version__}.dist-info" in dists, dists


def test_package_imports_from_the_venv_not_the_tree(venv):
    env_dir, _ = venv
    p = _run(venv, [str(env_dir / "bin" / "python"), "-c",
                    "import sys, k8s_gpu_node_checker_amd as k; print(k.__file__); print(sys.path)"])
    assert p.returncode == 0, p.stderr
    path = p.stdout.splitlines()[0]
    assert path.startswith(str(env_dir)), path
    assert REPO not in p.stdout.splitlines()[1]


def test_every_console_script_resolves(venv):
    env_dir, _ = venv
    for s in SCRIPTS:
        exe = env_dir / "bin" / s
        assert exe.exists(), s
        p = _run(venv, [str(exe), "--help"])
        assert p.returncode == 0, (s, p.stderr)
        assert p.stdout.startswith(f"usage: {s} "), (s, p.stdout[:200])


def test_installed_help_is_byte_identical_to_the_reference(venv, tmp_path):
    """argparse names the program after argv[0]; started under the reference's file name the
    installed console script prints the golden help byte for byte."""
    env_dir, _ = venv
    link = tmp_path / "check-gpu-node.py"
    os.symlink(env_dir / "bin" / "check-gpu-node", link)
    p = _run(venv, [str(link), "--help"])
    assert p.returncode == 0, p.stderr
    assert p.stdout == HELP


@pytest.mark.reference
@pytest.mark.skipif(not os.path.exists(REF), reason="reference script not mounted")
def test_installed_help_matches_the_reference_under_the_console_script_name(venv, tmp_path):
    """The unmodified reference started as ``check-gpu-node`` (a symlink, so its argparse prog is the same)
    against the installed console script: identical ``--help`` and identical usage error + exit 2."""
    env_dir, _ = venv
    ref_dir = tmp_path / "ref"
    ref_dir.mkdir()
    os.symlink(REF, ref_dir / "check-gpu-node")
    for args in (["--help"], ["--bogus"]):
        env = _clean_env(HOME=str(tmp_path), PYTHONPATH=STUBS)
        a = subprocess.run([sys.executable, str(ref_dir / "check-gpu-node")] + args, capture_output=True,
                           text=True, env=env, cwd=str(tmp_path), timeout=60)
        b = _run(venv, [str(env_dir / "bin" / "check-gpu-node")] + args)
        assert (b.returncode, b.stdout, b.stderr) == (a.returncode, a.stdout, a.stderr), args


def test_native_libraries_load_from_the_installed_location(venv):
    env_dir, _ = venv
    built = sorted(f for f in os.listdir(os.path.join(REPO, PKG, "_native"))
                   if f.endswith(".so") or f == "mi355x-probe")
    assert any(f.startswith("_fastpath") for f in built), "conftest builds the fast path first"
    site = glob.glob(str(env_dir / "lib" / "python3*" / "site-packages" / PKG / "_native"))[0]
    assert sorted(f for f in os.listdir(site) if f in built) == built
    if "mi355x-probe" in built:
        assert os.access(os.path.join(site, "mi355x-probe"), os.X_OK), "the probe CLI lost its exec bit"
    code = (
        "from k8s_gpu_node_checker_amd.ops import native, fastpath\n"
        "print(native.NATIVE_DIR)\n"
        "assert fastpath.backend() == 'native', fastpath.backend()\n"
        "import sys\n"
        "print([m.__file__ for m in sys.modules.values() if getattr(m, '__file__', '') and '_fastpath' in m.__file__])\n"
    )
    if "libmi355x_probe.so" in built:
        code += "print(native.load_cdll('libmi355x_probe.so', required=True)._name)\n"
    p = _run(venv, [str(env_dir / "bin" / "python"), "-c", code])
    assert p.returncode == 0, p.stderr
    lines = p.stdout.splitlines()
    assert lines[0] == site
    assert lines[1].count(site) == 1, lines[1]
    if "libmi355x_probe.so" in built:
        assert lines[2].startswith(site), lines[2]


def test_installed_checker_runs_a_check(venv, mock_cluster, tmp_path):
    """The installed console script does a real check (BASELINE config #1) off-tree: JSON + exit 0."""
    from k8s_gpu_node_checker_amd.testing import fixtures
    from k8s_gpu_node_checker_amd.testing.mock_apiserver import write_kubeconfig
    env_dir, _ = venv
    srv = mock_cluster([fixtures.realistic_node("n0", "amd.com/gpu", 1)])
    kc = write_kubeconfig(str(tmp_path / "kubeconfig"), srv.url, None)
    p = _run(venv, [str(env_dir / "bin" / "check-gpu-node"), "--json", "--kubeconfig", kc])
    assert p.returncode == 0, p.stdout + p.stderr
    assert '"total_nodes": 1' in p.stdout and '"ready_nodes": 1' in p.stdout


def _manifest_commands():
    for path in glob.glob(os.path.join(REPO, "deploy", "**", "*.yaml"), recursive=True):
        with open(path, encoding="utf-8") as f:
            for doc in yaml.safe_load_all(f):
                if not isinstance(doc, dict):
                    continue
                spec = doc.get("spec", {}) or {}
                tpl = spec.get("jobTemplate", {}).get("spec", {}).get("template") or spec.get("template") or {}
                pod = tpl.get("spec", {}) if isinstance(tpl, dict) else {}
                for c in (pod.get("containers") or []) + (pod.get("initContainers") or []):
                    if c.get("command"):
                        yield os.path.relpath(path, REPO), c["command"][0]


def test_every_manifest_command_is_an_installed_console_script(venv):
    env_dir, _ = venv
    cmds = list(_manifest_commands())
    assert len(cmds) >= 4, cmds
    for path, cmd in cmds:
        assert (env_dir / "bin" / cmd).exists(), (path, cmd)


def test_dockerfile_installs_into_a_venv_on_path():
    """The image reproduces the layout the tests above install: one venv at the same path in both stages,
    on PATH, holding the console scripts; no ``--prefix`` tree copied onto /usr/local."""
    with open(os.path.join(REPO, "deploy", "Dockerfile"), encoding="utf-8") as f:
        text = "\n".join(ln for ln in f.read().splitlines() if not ln.lstrip().startswith("#"))
    build, runtime = ("\n" + text).split("\nFROM ", 2)[1:]
    m = re.search(r"python3 -m venv (\S+)", build)
    assert m, "build stage makes no venv"
    venv_dir = m.group(1)
    assert f"{venv_dir}/bin/pip install" in build and "--no-build-isolation ." in build
    assert "--prefix" not in text and "--root" not in text
    assert f"COPY --from=build {venv_dir} {venv_dir}" in runtime
    assert re.search(rf"ENV PATH={re.escape(venv_dir)}/bin:\$PATH", runtime)
    entry = re.search(r'ENTRYPOINT \["([^"]+)"', runtime).group(1)
    assert entry in SCRIPTS
    # the runtime stage's interpreter is the one the venv's bin/python links to
    assert "python3" in runtime.split("COPY")[0]
