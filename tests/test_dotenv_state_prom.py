"""R7 .env loading, alert de-dup state file, Prometheus textfile output."""
import json
import os


from k8s_gpu_node_checker_amd.utils import dotenv, prom, statefile


def test_dotenv_parsing(tmp_path, monkeypatch):
    p = tmp_path / ".env"
    p.write_text("# comment\nSLACK_WEBHOOK_URL=https://hooks/x # trailing\nexport A='lit ${B}'\nB=\"two\\nlines\"\n"
                 "C=${B}-${MISSING:-dflt}\nNOVAL\nEXISTING=file\n")
    monkeypatch.setenv("EXISTING", "env")
    vals = dotenv.dotenv_values(str(p))
    assert vals["SLACK_WEBHOOK_URL"] == "https://hooks/x"
    assert vals["A"] == "lit ${B}"
    assert vals["B"] == "two\nlines"
    assert vals["C"] == "two\nlines-dflt"
    assert vals["NOVAL"] is None
    for k in ("SLACK_WEBHOOK_URL", "A", "B", "C"):
        monkeypatch.setenv(k, "")  # recorded, so what load_dotenv sets is undone after the test
        monkeypatch.delenv(k)
    assert dotenv.load_dotenv(str(p))
    assert os.environ["EXISTING"] == "env"  # real env wins (override=False)
    assert os.environ["SLACK_WEBHOOK_URL"] == "https://hooks/x"


def test_find_dotenv_walks_up(tmp_path):
    (tmp_path / ".env").write_text("X=1\n")
    deep = tmp_path / "a" / "b"
    deep.mkdir(parents=True)
    assert dotenv.find_dotenv(start=str(deep)) == str(tmp_path / ".env")


class R:
    def __init__(self, code, nodes, slack=None):
        self.exit_code = code
        self.gpu_nodes = nodes
        self.ready_gpu_nodes = [n for n in nodes if n["ready"]]
        self.slack_sent = slack
        self.verdicts = []
        self.tracer = None


def node(name, ready):
    return {"name": name, "ready": ready, "gpus": 8, "gpu_breakdown": {"amd.com/gpu": 8}}


def test_state_dedup_and_recovery(tmp_path):
    path = str(tmp_path / "state.json")
    bad = R(3, [node("a", False)])
    good = R(0, [node("a", True)])
    assert statefile.should_notify(None, bad, only_on_error=True)
    statefile.save(path, bad)
    prev = statefile.load(path)
    assert prev["exit_code"] == 3 and prev["not_ready"] == ["a"] and prev["runs"] == 1
    assert not statefile.should_notify(prev, bad, only_on_error=True)  # unchanged: no re-alert
    assert statefile.should_notify(prev, good, only_on_error=True)  # recovery
    statefile.save(path, good, prev)
    prev = statefile.load(path)
    assert not statefile.should_notify(prev, good, only_on_error=True)
    assert statefile.load(str(tmp_path / "missing")) is None


def test_cli_slack_on_change(run_cli, mock_cluster, sink, tmp_path):
    from k8s_gpu_node_checker_amd.testing import fixtures
    from k8s_gpu_node_checker_amd.testing.mock_apiserver import write_kubeconfig
    srv = mock_cluster(fixtures.golden("notready"))
    kc = write_kubeconfig(str(tmp_path / "kc"), srv.url)
    args = ["--kubeconfig", kc, "--slack-webhook", sink.url("200"), "--slack-only-on-error",
            "--state-file", str(tmp_path / "st.json"), "--slack-on-change"]
    for _ in range(3):
        assert run_cli(args).returncode == 3
    assert len(sink.requests) == 1  # first failure only
    srv.state.set_nodes(fixtures.golden("readme"))
    assert run_cli(args).returncode == 0
    assert len(sink.requests) == 2  # recovery announced
    assert run_cli(args).returncode == 0
    assert len(sink.requests) == 2


def test_prometheus_textfile(run_cli, mock_cluster, tmp_path):
    from k8s_gpu_node_checker_amd.testing import fixtures
    from k8s_gpu_node_checker_amd.testing.mock_apiserver import write_kubeconfig
    srv = mock_cluster(fixtures.cluster(2, "amd", not_ready=[1], with_health=True))
    kc = write_kubeconfig(str(tmp_path / "kc"), srv.url)
    out = tmp_path / "m" / "gpu.prom"
    p = run_cli(["--kubeconfig", kc, "--prometheus-textfile", str(out)])
    assert p.returncode == 0
    text = out.read_text()
    assert "k8s_gpu_checker_gpu_nodes 2" in text and "k8s_gpu_checker_ready_gpu_nodes 1" in text
    assert 'k8s_gpu_checker_node_ready{node="mi355x-node-0001"} 0' in text
    assert 'k8s_gpu_checker_mi355x_health{node="mi355x-node-0000",state="healthy"} 1' in text
    p = run_cli(["--kubeconfig", str(tmp_path / "missing"), "--prometheus-textfile", str(out)])
    assert p.returncode == 1 and "k8s_gpu_checker_exit_code 1" in out.read_text()


def test_prom_escaping():
    r = R(0, [node('we"ird\\name', True)])
    lines = prom.render(r)
    assert 'k8s_gpu_checker_node_ready{node="we\\"ird\\\\name"} 1' in lines


def test_cli_watch_bounded(run_cli, mock_cluster, sink, tmp_path):
    """``--watch P --watch-count N``: N checks on a fixed cadence, exit code of the last one; with
    ``--state-file --slack-on-change`` a long-running watcher alerts once per state change."""
    import json
    import time
    from k8s_gpu_node_checker_amd.testing import fixtures
    from k8s_gpu_node_checker_amd.testing.mock_apiserver import write_kubeconfig
    srv = mock_cluster(fixtures.golden("readme"))
    kc = write_kubeconfig(str(tmp_path / "kc"), srv.url)
    t = time.monotonic()
    p = run_cli(["--kubeconfig", kc, "--json", "--watch", "0.3", "--watch-count", "3"])
    elapsed = time.monotonic() - t
    assert p.returncode == 0, p.stderr
    docs = []
    dec = json.JSONDecoder()
    text = p.stdout.strip()
    while text:
        d, i = dec.raw_decode(text)
        docs.append(d)
        text = text[i:].strip()
    assert len(docs) == 3 and all(d["ready_nodes"] == 2 for d in docs)
    assert elapsed >= 0.6  # two full periods between three checks
    args = ["--kubeconfig", kc, "--slack-webhook", sink.url("200"), "--slack-only-on-error",
            "--state-file", str(tmp_path / "st.json"), "--slack-on-change", "--watch", "0.05", "--watch-count", "4"]
    srv.state.set_nodes(fixtures.golden("notready"))
    assert run_cli(args).returncode == 3
    assert len(sink.requests) == 1  # four failing checks, one alert


def test_cli_slack_on_change_keeps_an_undelivered_alert_due(run_cli, mock_cluster, sink, tmp_path):
    """A failing webhook does not consume the alert: the next run (same outcome) sends it, then it is
    de-duplicated as usual."""
    from k8s_gpu_node_checker_amd.testing import fixtures
    from k8s_gpu_node_checker_amd.testing.mock_apiserver import write_kubeconfig
    srv = mock_cluster(fixtures.golden("notready"))
    kc = write_kubeconfig(str(tmp_path / "kc"), srv.url)
    base = ["--kubeconfig", kc, "--slack-only-on-error", "--slack-retry-count", "0",
            "--state-file", str(tmp_path / "st.json"), "--slack-on-change"]
    assert run_cli(base + ["--slack-webhook", sink.url("500")]).returncode == 3
    assert statefile.load(str(tmp_path / "st.json"))["slack_pending"] is True
    assert len(sink.requests) == 1
    for _ in range(2):
        assert run_cli(base + ["--slack-webhook", sink.url("200")]).returncode == 3
    assert len(sink.requests) == 2  # delivered on the second run, not repeated on the third
    assert statefile.load(str(tmp_path / "st.json"))["slack_pending"] is False


def _cronjob_command():
    import os
    import yaml
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(repo, "deploy", "cronjob.yaml"), encoding="utf-8") as f:
        cj = yaml.safe_load(f)
    return cj["spec"]["jobTemplate"]["spec"]["template"]["spec"]["containers"][0]["command"]


def test_shipped_cronjob_alerts_once_per_single_node_failure_and_recovery(run_cli, mock_cluster, sink, tmp_path):
    """with the shipped CronJob's flags, 1 of 8 MI355X nodes turning unhealthy (exit code stays
    0: seven are Ready) is one Slack POST, and its recovery one more; unchanged runs send nothing."""
    from k8s_gpu_node_checker_amd.testing import fixtures
    from k8s_gpu_node_checker_amd.testing.mock_apiserver import write_kubeconfig
    cmd = _cronjob_command()
    assert cmd[0] == "check-gpu-node" and "--slack-on-node-change" in cmd and "--slack-only-on-error" in cmd
    healthy = fixtures.cluster(8, "amd", with_health=True)
    sick = fixtures.cluster(8, "amd", with_health=True)
    rep = fixtures.mi355x_probe_report(sick[3]["metadata"]["name"], 8, gpu2={"ecc_uncorrectable": 4})
    sick[3]["metadata"]["annotations"].update(fixtures.health_annotation(rep))
    sick[3]["status"]["conditions"] = [c for c in sick[3]["status"]["conditions"] if c["type"] != "AMDGPUHealthy"] + \
        [fixtures.health_condition(rep, 8)]
    srv = mock_cluster(healthy)
    kc = write_kubeconfig(str(tmp_path / "kc"), srv.url)
    args = [a for a in cmd[1:] if a != "--in-cluster"]
    args[args.index("/state/last.json")] = str(tmp_path / "last.json")
    args += ["--kubeconfig", kc]
    env = {"SLACK_WEBHOOK_URL": sink.url("200")}
    for _ in range(2):
        assert run_cli(args, env=env).returncode == 0
    assert len(sink.requests) == 0  # all healthy: nothing to say
    srv.state.set_nodes(sick)
    for _ in range(3):
        p = run_cli(args, env=env)
        assert p.returncode == 0, p.stderr  # 7 of 8 Ready
    assert len(sink.requests) == 1
    text = sink.payloads()[0]["text"]
    assert f"`{sick[3]['metadata']['name']}`: ❌ Not Ready" in text
    srv.state.set_nodes(healthy)
    for _ in range(2):
        assert run_cli(args, env=env).returncode == 0
    assert len(sink.requests) == 2  # the recovery, once
    # without --slack-on-node-change (the round-2 CronJob) the same failure never reaches Slack
    base = [a for a in args if a != "--slack-on-node-change"]
    base[base.index(str(tmp_path / "last.json"))] = str(tmp_path / "other.json")
    srv.state.set_nodes(sick)
    assert run_cli(base, env=env).returncode == 0
    assert len(sink.requests) == 2


def test_should_notify_on_node_change_rules():
    bad = R(0, [node("a", True), node("b", False)])
    good = R(0, [node("a", True), node("b", True)])
    assert statefile.should_notify(None, bad, True, on_node_change=True)
    assert not statefile.should_notify(None, good, True, on_node_change=True)
    assert not statefile.should_notify(None, bad, True)  # the reference rule: ready > 0 -> quiet
    prev = {"fingerprint": statefile.fingerprint(bad), "exit_code": 0, "not_ready": ["b"]}
    assert not statefile.should_notify(prev, bad, True, on_node_change=True)
    assert statefile.should_notify(prev, good, True, on_node_change=True)


def test_state_file_with_wrong_types_is_tolerated(tmp_path):
    """A hand-edited state file with fields of the wrong type does not fail the run: those fields are dropped
    (the gate then treats the run as it would a first one for them)."""
    import json as _json
    import types
    from k8s_gpu_node_checker_amd.utils import statefile
    p = tmp_path / "state.json"
    p.write_text(_json.dumps({"version": 1, "not_ready": 5, "exit_code": "x", "runs": True, "fingerprint": "f"}))
    doc = statefile.load(str(p))
    assert doc == {"version": 1, "fingerprint": "f"}
    res = types.SimpleNamespace(exit_code=0, gpu_nodes=[{"name": "a", "ready": False, "gpus": 8},
                                                         {"name": "b", "ready": True, "gpus": 8}])
    assert statefile.should_notify(doc, res, only_on_error=True, on_node_change=True) is True
    p.write_text("[" * 100000)
    assert statefile.load(str(p)) is None


def test_env_template_copied_as_is_changes_nothing(run_cli, mock_cluster, tmp_path):
    """The shipped .env-template, copied to .env unedited (the reference's setup step), leaves the webhook
    unset: the check runs, no Slack line is printed, the output is the plain report."""
    import shutil
    from k8s_gpu_node_checker_amd.testing import fixtures
    from k8s_gpu_node_checker_amd.testing.mock_apiserver import write_kubeconfig
    shutil.copy(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), ".env-template"),
                tmp_path / ".env")
    kc = write_kubeconfig(str(tmp_path / "kc"), mock_cluster(fixtures.golden("readme")).url)
    p = run_cli(["--kubeconfig", kc])
    assert p.returncode == 0 and "슬랙" not in p.stdout + p.stderr, p.stdout + p.stderr
