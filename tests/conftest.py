"""Shared fixtures.  GPU tests are marked ``@pytest.mark.gpu`` (run on an MI355X via gpurun)."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

# Property tests (hypothesis): the same examples every run, so the suite's result is a function of the tree (the
# round driver and CI run it once); HYPOTHESIS_PROFILE=explore draws fresh examples to hunt for new failures.
try:
    from hypothesis import settings as _hsettings

    _hsettings.register_profile("ci", derandomize=True, print_blob=True)
    _hsettings.register_profile("explore", derandomize=False, print_blob=True)
    _hsettings.load_profile(os.environ.get("HYPOTHESIS_PROFILE", "ci"))
except ImportError:  # hypothesis is optional: its tests import it themselves
    pass


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: takes more than a few seconds")
    config.addinivalue_line("markers", "reference: runs the unmodified reference script (skipped if absent)")


def pytest_sessionstart(session):
    # The CPU fast path is part of the product: build it if the tree has no .so yet (g++ takes ~5 s).
    from k8s_gpu_node_checker_amd.ops import native
    have = os.path.isdir(native.NATIVE_DIR) and any(f.startswith("_fastpath") for f in os.listdir(native.NATIVE_DIR))
    if not have:
        subprocess.run([sys.executable, "-m", "k8s_gpu_node_checker_amd.build", "--only", "fastpath,probe"],
                       cwd=REPO, check=False)


@pytest.fixture
def repo():
    return REPO


@pytest.fixture
def mock_cluster():
    """Factory: ``mock_cluster(nodes, **MockConfig kwargs)`` -> started MockApiServer (stopped at teardown)."""
    from k8s_gpu_node_checker_amd.testing.mock_apiserver import MockApiServer, MockConfig
    servers = []

    def make(nodes, **cfg):
        srv = MockApiServer(nodes, cfg=MockConfig(**cfg)).start()
        servers.append(srv)
        return srv
    yield make
    for s in servers:
        s.stop()


@pytest.fixture
def sink():
    from k8s_gpu_node_checker_amd.testing.webhook_sink import WebhookSink
    s = WebhookSink(slow_s=2.5).start()
    yield s
    s.stop()


@pytest.fixture
def run_cli(tmp_path):
    """Run ``check-gpu-node.py`` in a subprocess: ``run_cli(args, env=None) -> CompletedProcess``."""
    def run(args, env=None, timeout=60):
        e = {k: v for k, v in os.environ.items() if k not in ("SLACK_WEBHOOK_URL", "KUBECONFIG")}
        e["HOME"] = str(tmp_path)
        if env:
            e.update(env)
        return subprocess.run([sys.executable, os.path.join(REPO, "check-gpu-node.py")] + list(args),
                              capture_output=True, text=True, env=e, timeout=timeout, cwd=str(tmp_path))
    return run


@pytest.fixture(scope="session")
def certs(tmp_path_factory):
    """A self-signed server certificate for 127.0.0.1 / localhost: (crt path, key path)."""
    d = tmp_path_factory.mktemp("pki")
    key, crt = d / "srv.key", d / "srv.crt"
    r = subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", str(key), "-out", str(crt),
                        "-days", "1", "-subj", "/CN=mock-apiserver", "-addext", "subjectAltName=IP:127.0.0.1,DNS:localhost"],
                       capture_output=True)
    if r.returncode != 0:
        pytest.skip("openssl unavailable")
    return str(crt), str(key)
