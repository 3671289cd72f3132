"""R8/R9/R11: Slack URL resolution, gating and the retry state machine (both policies)."""
import io
import json
import time


from k8s_gpu_node_checker_amd.notify import slack
from k8s_gpu_node_checker_amd.utils.backoff import Backoff, parse_retry_after


def send(url, policy="backoff", retries=3, delay=0, sleep=None):
    err = io.StringIO()
    slept = []
    ok = slack.send_slack_message(url, "hello ✅", "bot", retries, delay, policy=policy, err=err,
                                  sleep=sleep or slept.append, backoff=Backoff(base=1.0, cap=30, jitter=0))
    return ok, err.getvalue().splitlines(), slept


def test_url_resolution(monkeypatch):
    monkeypatch.setenv("SLACK_WEBHOOK_URL", "http://env")
    assert slack.get_slack_webhook_url("http://flag") == "http://flag"
    assert slack.get_slack_webhook_url("") == "http://env"  # `or` semantics
    monkeypatch.delenv("SLACK_WEBHOOK_URL")
    assert slack.get_slack_webhook_url(None) is None


def test_gating():
    assert not slack.should_send(None, False, 0)
    assert slack.should_send("u", False, 5)
    assert not slack.should_send("u", True, 1)
    assert slack.should_send("u", True, 0)


def test_success_first_attempt(sink):
    ok, lines, _ = send(sink.url("200"))
    assert ok and lines == []
    req = sink.requests[-1]
    assert req["headers"]["Content-Type"] == "application/json"
    assert json.loads(req["body"]) == {"text": "hello ✅", "username": "bot", "icon_emoji": ":robot_face:"}


def test_reference_policy_retries_5xx_immediately(sink):
    ok, lines, slept = send(sink.url("500"), policy="reference")
    assert not ok and slept == []
    assert lines == ["슬랙 메시지 전송 실패 (HTTP 500): server_error"] * 4


def test_backoff_policy_sleeps_between_5xx(sink):
    ok, lines, slept = send(sink.url("500"), policy="backoff", delay=30)
    assert not ok and len(lines) == 4
    assert slept == [1.0, 2.0, 4.0]  # exponential, capped by retry_delay; no sleep after the last attempt


def test_backoff_honours_retry_after_on_429(sink):
    ok, lines, slept = send(sink.url("429"), retries=1, delay=30)
    assert slept == [1.0] and len(lines) == 2


def test_backoff_stops_on_permanent_4xx(sink):
    ok, lines, slept = send(sink.url("404"))
    assert not ok and lines == ["슬랙 메시지 전송 실패 (HTTP 404): no_service"] and slept == []
    assert sink.counts["/404"] == 1


def test_reference_policy_retries_4xx(sink):
    ok, lines, _ = send(sink.url("404"), policy="reference")
    assert len(lines) == 4


def test_flaky_then_success_message(sink):
    ok, lines, _ = send(sink.url("flaky2"))
    assert ok
    assert lines[-1] == "✅ 슬랙 메시지를 3번째 시도에서 성공적으로 전송했습니다."


def test_204_is_failure(sink):
    ok, lines, _ = send(sink.url("204"), policy="reference")
    assert not ok and lines[0] == "슬랙 메시지 전송 실패 (HTTP 204): "


def test_reset_sleeps_retry_delay_then_final_failure(sink):
    ok, lines, slept = send(sink.url("reset"), delay=7)
    assert not ok and slept == [7, 7, 7]
    assert lines[0].startswith("슬랙 메시지 전송 실패 (1/4회 시도): ('Connection aborted.', ")
    assert lines[1] == "⏳ 7초 후 재시도합니다..."
    assert lines[-1].startswith("슬랙 메시지 전송 최종 실패: ('Connection aborted.'")


def test_close_without_response_counts_as_aborted(sink):
    ok, lines, slept = send(sink.url("close"), retries=1, delay=0)
    assert not ok and "RemoteDisconnected" in lines[0]


def test_reset_then_success(sink):
    ok, lines, slept = send(sink.url("resetflaky"), delay=1)
    assert ok and slept == [1]
    assert lines[-1] == "✅ 슬랙 메시지를 2번째 시도에서 성공적으로 전송했습니다."


def test_refused_gives_up_immediately():
    ok, lines, slept = send("http://127.0.0.1:9/x")
    assert not ok and len(lines) == 1 and slept == []
    assert lines[0].startswith("슬랙 메시지 전송 실패: HTTPConnectionPool(host='127.0.0.1', port=9): Max retries exceeded")
    assert "Connection refused" in lines[0]


def test_read_timeout_gives_up(sink):
    err = io.StringIO()
    t = time.time()
    ok = slack.send_slack_message(sink.url("slow"), "x", "bot", 3, 0, timeout=0.5, err=err)
    assert not ok and time.time() - t < 2.4
    assert "Read timed out. (read timeout=0.5)" in err.getvalue()


def test_invalid_url():
    ok, lines, _ = send("not-a-url")
    assert not ok and lines == ["슬랙 메시지 전송 실패: Invalid URL 'not-a-url': No scheme supplied. "
                                "Perhaps you meant https://not-a-url?"]


def test_no_url_returns_false():
    assert slack.send_slack_message("", "x") is False


def test_negative_retry_count_sends_nothing(sink):
    ok, lines, _ = send(sink.url("200"), retries=-1)
    assert not ok and lines == [] and "/200" not in sink.counts


def test_retry_after_parsing():
    assert parse_retry_after("3") == 3.0
    assert parse_retry_after(None) is None
    assert parse_retry_after("garbage") is None
    assert 0 <= parse_retry_after("Wed, 21 Oct 2015 07:28:00 GMT") == 0.0
    b = Backoff(base=0.5, cap=4, jitter=0)
    assert [b.delay(i) for i in range(5)] == [0.5, 1.0, 2.0, 4.0, 4.0]
    assert b.delay(0, "10") == 4  # Retry-After is capped too
    j = Backoff(base=1, cap=10, jitter=0.5)
    assert all(0.5 <= j.delay(0) <= 1.0 for _ in range(50))


def test_cli_negative_delay_is_clamped_not_a_crash(run_cli, mock_cluster, sink, tmp_path):
    from k8s_gpu_node_checker_amd.testing import fixtures
    from k8s_gpu_node_checker_amd.testing.mock_apiserver import write_kubeconfig
    srv = mock_cluster(fixtures.golden("readme"))
    kc = write_kubeconfig(str(tmp_path / "kc"), srv.url)
    p = run_cli(["--kubeconfig", kc, "--slack-webhook", sink.url("resetflaky"), "--slack-retry-delay", "-1"])
    assert p.returncode == 0  # the reference crashes with exit 1 here (PARITY.md)
    assert "✅ Ready 상태의 GPU 노드" in p.stdout


def test_cli_slack_failure_line_on_stderr(run_cli, mock_cluster, sink, tmp_path):
    from k8s_gpu_node_checker_amd.testing import fixtures
    from k8s_gpu_node_checker_amd.testing.mock_apiserver import write_kubeconfig
    srv = mock_cluster(fixtures.golden("notready"))
    kc = write_kubeconfig(str(tmp_path / "kc"), srv.url)
    p = run_cli(["--kubeconfig", kc, "--slack-webhook", sink.url("404"), "--slack-only-on-error"])
    assert p.returncode == 3
    assert p.stderr.splitlines() == ["슬랙 메시지 전송 실패 (HTTP 404): no_service", "❌ 슬랙 메시지 전송에 실패했습니다."]
    assert p.stdout.startswith("⚠️ GPU 노드는 2개 있으나")
