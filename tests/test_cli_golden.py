"""CLI end-to-end against the mock apiserver: output, streams and exit codes (R13-R17, Appendix A)."""
import json

import pytest

from k8s_gpu_node_checker_amd.testing import fixtures
from k8s_gpu_node_checker_amd.testing.mock_apiserver import write_kubeconfig

from test_report import A1, A3_NOGPU, A3_NOTREADY, A4

HELP = """usage: check-gpu-node.py [-h] [--kubeconfig KUBECONFIG] [--json]
                         [--slack-webhook SLACK_WEBHOOK]
                         [--slack-username SLACK_USERNAME]
                         [--slack-only-on-error]
                         [--slack-retry-count SLACK_RETRY_COUNT]
                         [--slack-retry-delay SLACK_RETRY_DELAY]

Kubernetes GPU 노드 점검 스크립트

options:
  -h, --help            show this help message and exit
  --kubeconfig KUBECONFIG
                        kubeconfig 경로 직접 지정
  --json                JSON 형태로만 출력(머신 판독용)

슬랙 알림:
  슬랙으로 메시지를 전송하는 옵션들

  --slack-webhook SLACK_WEBHOOK
                        슬랙 웹훅 URL (환경변수 SLACK_WEBHOOK_URL로도 설정 가능)
  --slack-username SLACK_USERNAME
                        슬랙 봇 사용자명 (기본: k8s-gpu-checker)
  --slack-only-on-error
                        GPU 노드가 없거나 Ready 상태가 아닐 때만 슬랙 메시지 전송
  --slack-retry-count SLACK_RETRY_COUNT
                        슬랙 메시지 전송 실패시 최대 재시도 횟수 (기본: 3)
  --slack-retry-delay SLACK_RETRY_DELAY
                        슬랙 메시지 재시도 간격(초) (기본: 30)
"""


@pytest.fixture
def kc(tmp_path, mock_cluster):
    def make(name_or_nodes, **cfg):
        nodes = fixtures.golden(name_or_nodes) if isinstance(name_or_nodes, str) else name_or_nodes
        srv = mock_cluster(nodes, **cfg)
        return write_kubeconfig(str(tmp_path / "kubeconfig"), srv.url, cfg.get("token")), srv
    return make


def test_help_is_byte_identical(run_cli):
    p = run_cli(["--help"], env={"COLUMNS": "80"})
    assert p.returncode == 0
    assert p.stdout == HELP


def test_help_all_lists_extensions(run_cli):
    p = run_cli(["--help-all"], env={"COLUMNS": "120"})
    assert p.returncode == 0
    for flag in ("--health-policy", "--mi355x", "--probe-endpoint", "--page-size", "--json-extended"):
        assert flag in p.stdout


def test_usage_error_exit_2(run_cli):
    p = run_cli(["--bogus"], env={"COLUMNS": "80"})
    assert p.returncode == 2
    assert p.stderr.endswith("check-gpu-node.py: error: unrecognized arguments: --bogus\n")
    assert p.stdout == ""


@pytest.mark.parametrize("name,text,code", [("readme", A1, 0), ("nogpu", A3_NOGPU, 2), ("notready", A3_NOTREADY, 3),
                                            ("edge", A4, 0), ("empty", A3_NOGPU, 2)])
def test_text_output_and_exit_code(run_cli, kc, name, text, code):
    path, _ = kc(name)
    p = run_cli(["--kubeconfig", path])
    assert p.returncode == code
    assert p.stdout == text
    assert p.stderr == ""


@pytest.mark.parametrize("name,code", [("readme", 0), ("nogpu", 2), ("notready", 3), ("edge", 0), ("nometa", 0)])
def test_json_output(run_cli, kc, name, code):
    path, _ = kc(name)
    p = run_cli(["--kubeconfig", path, "--json"])
    assert p.returncode == code
    doc = json.loads(p.stdout)
    assert p.stdout == json.dumps(doc, ensure_ascii=False, indent=2) + "\n"
    assert set(doc) == {"total_nodes", "ready_nodes", "nodes"}


def test_kubeconfig_env_var(run_cli, kc):
    path, _ = kc("readme")
    p = run_cli(["--json"], env={"KUBECONFIG": path})
    assert p.returncode == 0 and json.loads(p.stdout)["total_nodes"] == 2


def test_missing_kubeconfig_json_error(run_cli, tmp_path):
    p = run_cli(["--json", "--kubeconfig", str(tmp_path / "nope")])
    assert p.returncode == 1
    assert p.stdout == '{"error": "Invalid kube-config file. No configuration found."}\n'


def test_missing_kubeconfig_text_error(run_cli, tmp_path):
    p = run_cli(["--kubeconfig", str(tmp_path / "nope")])
    assert p.returncode == 1
    assert p.stdout == ""
    assert p.stderr.startswith("에러: Invalid kube-config file. No configuration found.\nTraceback (most recent call last):")


def test_forbidden_is_exit_1_with_api_exception_text(run_cli, kc):
    path, _ = kc("readme", status=403)
    p = run_cli(["--kubeconfig", path, "--json", "--kube-retries", "0"])
    assert p.returncode == 1
    err = json.loads(p.stdout)["error"]
    assert err.startswith("(403)\nReason: Forbidden\nHTTP response headers: HTTPHeaderDict({")
    assert "nodes is forbidden" in err


def test_bearer_token_is_sent(run_cli, kc):
    path, srv = kc("readme", token="s3cret")
    p = run_cli(["--kubeconfig", path, "--json"])
    assert p.returncode == 0
    assert srv.log[-1]["auth"] == "Bearer s3cret"


def test_dotenv_supplies_webhook(run_cli, kc, sink, tmp_path):
    path, _ = kc("readme")
    (tmp_path / ".env").write_text(f"SLACK_WEBHOOK_URL={sink.url('200')}\n")
    p = run_cli(["--kubeconfig", path])
    assert p.returncode == 0
    assert p.stdout.startswith("✅ 슬랙 메시지를 성공적으로 전송했습니다.\n✅ Ready 상태의 GPU 노드")
    assert len(sink.requests) == 1


def test_module_entry_point(kc, tmp_path, repo):
    import subprocess
    import sys
    path, _ = kc("readme")
    p = subprocess.run([sys.executable, "-m", "k8s_gpu_node_checker_amd", "--kubeconfig", path, "--json"],
                       capture_output=True, text=True, cwd=repo)
    assert p.returncode == 0 and json.loads(p.stdout)["ready_nodes"] == 2


def test_trace_and_extended(run_cli, kc):
    nodes = fixtures.cluster(3, "amd", with_health=True)
    path, _ = kc(nodes)
    p = run_cli(["--kubeconfig", path, "--json-extended", "--trace"])
    assert p.returncode == 0
    doc = json.loads(p.stdout)
    assert doc["mi355x"]["health_summary"]["healthy"] == 3
    assert "list" in doc["timings_ms"] and "total" in doc["timings_ms"]
    assert "[trace]" in p.stderr and "backend=" in p.stderr
