"""Command line: ``check-gpu-node``.

``--help`` is byte-identical to the reference: the
reference's seven flags, the same Korean help strings, the same ``슬랙 알림``
group.  The MI355X extensions are real flags but hidden from ``--help``;
``--help-all`` lists them.

Exit codes (reference ``:289-293``, ``:319-327``): 0 = at least one Ready GPU
node, 3 = GPU nodes but none Ready, 2 = no GPU nodes (and argparse usage
errors, as in the reference), 1 = any exception (kubeconfig, API, transport).
"""

from __future__ import annotations

import os
import sys
TYPE_CHECKING = False
if TYPE_CHECKING:  # annotations only (PEP 563): importing typing is ~10 ms of a cold start
    from typing import Any, Dict, List, Optional, Tuple

# Every flag once: (group, flag, options).  group "" = top level, "slack" = the reference's 슬랙 알림
# group, "x" = MI355X extensions (hidden unless --help-all).  build_parser() turns this table into the
# argparse parser (--help byte-identical to the reference); _fast_parse() reads the same table to skip
# the argparse import (+ gettext + locale, ~2.5 ms of a 1-node cold start) for a plain command line.
_FLAGS: Tuple[Tuple[str, str, Dict[str, Any]], ...] = (
    ("", "--kubeconfig", {"help": "kubeconfig 경로 직접 지정"}),
    ("", "--json", {"action": "store_true", "help": "JSON 형태로만 출력(머신 판독용)"}),
    ("slack", "--slack-webhook", {"help": "슬랙 웹훅 URL (환경변수 SLACK_WEBHOOK_URL로도 설정 가능)"}),
    ("slack", "--slack-username", {"default": "k8s-gpu-checker", "help": "슬랙 봇 사용자명 (기본: k8s-gpu-checker)"}),
    ("slack", "--slack-only-on-error", {"action": "store_true",
                                        "help": "GPU 노드가 없거나 Ready 상태가 아닐 때만 슬랙 메시지 전송"}),
    ("slack", "--slack-retry-count", {"type": int, "default": 3,
                                      "help": "슬랙 메시지 전송 실패시 최대 재시도 횟수 (기본: 3)"}),
    ("slack", "--slack-retry-delay", {"type": int, "default": 30, "help": "슬랙 메시지 재시도 간격(초) (기본: 30)"}),
    ("x", "--help-all", {"action": "store_true", "help": "모든 옵션(확장 포함) 도움말"}),
    ("slack*", "--slack-retry-policy", {"choices": ("backoff", "reference"), "default": "backoff",
                                        "help": "5xx/429 재시도 정책: backoff(지수 백오프, 기본) | reference(즉시 재시도)"}),
    ("slack*", "--slack-on-change", {"action": "store_true",
                                     "help": "--state-file 과 함께: 상태가 바뀌었을 때만 전송 (복구 알림 포함)"}),
    ("slack*", "--slack-on-node-change", {"action": "store_true",
                                          "help": "--slack-on-change 포함: --slack-only-on-error 여도 Ready 가 아닌 "
                                                  "GPU 노드 집합이 바뀌면 전송 (노드 하나의 장애/복구)"}),
    ("x", "--context", {"help": "kubeconfig context (기본: current-context)"}),
    ("x", "--in-cluster", {"action": "store_true", "help": "Pod ServiceAccount 로 접속"}),
    ("x", "--kube-timeout", {"type": float, "default": 30.0, "help": "kube-apiserver 요청 타임아웃(초) (기본: 30)"}),
    ("x", "--kube-env-proxy", {"action": "store_true",
                               "help": "kubeconfig 에 proxy-url 이 없으면 HTTPS_PROXY / NO_PROXY 환경변수로 apiserver 에 접속 "
                                       "(kubectl 과 같음; 기본: 환경변수 무시, PARITY.md #18)"}),
    ("x", "--kube-retries", {"type": int, "default": 2, "help": "LIST 재시도 횟수 (429/5xx/연결 오류, 기본: 2)"}),
    ("x", "--page-size", {"type": int, "default": 500, "help": "LIST 페이지 크기 (0 = 한 번에, 기본: 500)"}),
    ("x", "--label-selector", {"help": "노드 labelSelector"}),
    ("x", "--resource-version", {"help": "LIST resourceVersion (예: 0 = watch cache)"}),
    ("x", "--gpu-source", {"choices": ("capacity", "allocatable"), "default": "capacity",
                           "help": "GPU 수를 읽을 status 필드 (기본: capacity = reference)"}),
    ("x", "--health-policy", {"choices": ("off", "auto", "require"), "default": "auto",
                              "help": "MI355X 헬스 게이트: off | auto(리포트가 있으면 반영, 기본) | require"}),
    ("x", "--probe-max-age", {"type": float, "default": 900.0, "help": "프로브 리포트 최대 나이(초) (기본: 900)"}),
    ("x", "--probe-unknown", {"choices": ("allow", "deny"), "default": "allow",
                              "help": "프로브 상태 unknown(만료/실패) 노드 처리 (기본: allow)"}),
    ("x", "--xgmi-links", {"type": int, "default": 7, "help": "GPU 당 기대 xGMI 링크 수 (0 = 검사 안 함, 기본: 7)"}),
    ("x", "--health-reeval", {"action": "store_true",
                              "help": "AMDGPUHealthy 조건 대신 프로브 리포트(annotation)를 이 임계값으로 재평가"}),
    ("x", "--probe-endpoint", {"help": "노드별 프로브 URL 템플릿, 예: http://{pod_ip}:9464/probe "
                                       "({pod_ip}: --probe-service 의 EndpointSlice, {ip}: 노드 InternalIP, {name})"}),
    ("x", "--probe-service", {"default": "gpu-health/mi355x-node-agent", "metavar": "NS/NAME",
                              "help": "{pod_ip} 를 채울 에이전트 Service (기본: gpu-health/mi355x-node-agent)"}),
    ("x", "--probe-concurrency", {"type": int, "default": 64, "help": "프로브 fan-out 동시성 (기본: 64)"}),
    ("x", "--probe-timeout", {"type": float, "default": 2.0, "help": "노드별 프로브 타임아웃(초) (기본: 2)"}),
    ("x", "--probe-ca", {"help": "https 프로브 엔드포인트를 검증할 CA 파일 (기본: 시스템 CA)"}),
    ("x", "--probe-tls-server-name", {"metavar": "NAME",
                                      "help": "https 프로브의 서버 인증서를 URL 의 호스트 대신 이 이름으로 검증 "
                                              "({pod_ip} 처럼 인증서에 없는 주소로 접속할 때, 예: "
                                              "mi355x-node-agent.gpu-health.svc)"}),
    ("x", "--probe-cache-ttl", {"type": float, "default": 30.0, "metavar": "SEC",
                                "help": "--watch-events + --probe-endpoint: 노드별로 가져온 리포트를 이 시간(초) 동안 "
                                        "재사용 (에이전트는 1분마다 프로브; 기본: 30)"}),
    ("x", "--probe-client-cert", {"help": "에이전트가 클라이언트 인증서를 요구할 때 제시할 인증서 (PEM)"}),
    ("x", "--probe-client-key", {"help": "--probe-client-cert 의 개인 키 (PEM)"}),
    ("x", "--require-schedulable", {"action": "store_true",
                                    "help": "cordon(spec.unschedulable) 되었거나 amd.com/gpu-unhealthy taint 가 있는 "
                                            "GPU 노드는 Ready 로 세지 않음"}),
    ("x", "--mi355x", {"action": "store_true",
                       "help": "MI355X 프리셋: --gpu-source allocatable --health-policy require --require-schedulable"}),
    ("x", "--json-extended", {"action": "store_true", "help": "JSON 에 MI355X 헬스/타이밍 필드 추가"}),
    ("x", "--trace", {"action": "store_true", "help": "단계별 소요 시간을 stderr 로 출력"}),
    ("x", "--explain", {"metavar": "NODE", "help": "한 노드가 Ready 로 집계되는(또는 안 되는) 이유를 출력"}),
    ("x", "--fleet", {"action": "store_true", "help": "MI355X 플릿 요약 (판정별 노드 수, 문제 노드, 드라이버/펌웨어 버전)"}),
    ("x", "--prometheus-textfile", {"help": "node-exporter textfile 메트릭 경로"}),
    ("x", "--metrics-listen", {"metavar": "HOST:PORT",
                               "help": "--watch-events: Prometheus /metrics 를 이 주소에서 제공 (예: 0.0.0.0:9465)"}),
    ("x", "--state-file", {"help": "직전 결과 저장 파일 (알림 중복 제거)"}),
    ("x", "--watch", {"type": float, "default": 0.0, "help": "N초마다 반복 점검 (0 = 한 번, 기본)"}),
    ("x", "--watch-count", {"type": int, "default": 0,
                            "help": "--watch 반복 횟수 / --watch-events 보고 횟수 (0 = 무제한, 기본); 종료 코드는 "
                                    "마지막 점검의 것"}),
    ("x", "--watch-events", {"action": "store_true",
                             "help": "이벤트 기반 감시: LIST 한 번 후 watch 스트림을 따라가며 상태가 바뀔 때만 보고"}),
    ("x", "--watch-debounce", {"type": float, "default": 0.2,
                               "help": "--watch-events: 이 시간(초) 안에 도착한 이벤트를 한 번에 평가 (기본: 0.2)"}),
    ("x", "--watch-duration", {"type": float, "default": 0.0, "help": "--watch-events: N초 후 종료 (0 = 무제한, 기본)"}),
    ("x", "--leader-elect", {"action": "store_true",
                             "help": "--watch-events 를 여러 복제본으로: coordination.k8s.io Lease 를 가진 하나만 감시/보고"}),
    ("x", "--leader-elect-lease", {"help": "--leader-elect: Lease 네임스페이스/이름 (기본: <파드 네임스페이스>/gpu-node-watcher)"}),
    ("x", "--leader-elect-timing", {"default": "15,10,2",
                                    "help": "--leader-elect: lease 기간, 갱신 기한, 재시도 간격(초) (기본: 15,10,2)"}),
)


def build_parser(show_all: bool = False, prog: Optional[str] = None) -> "argparse.ArgumentParser":
    import argparse
    if prog is None:
        base = os.path.basename(sys.argv[0]) if sys.argv and sys.argv[0] else "check-gpu-node"
        prog = "check-gpu-node" if base in ("__main__.py", "-c", "") else base
    p = argparse.ArgumentParser(prog=prog, description="Kubernetes GPU 노드 점검 스크립트")
    g = x = None
    for group, flag, opts in _FLAGS:
        if group == "slack" and g is None:
            g = p.add_argument_group("슬랙 알림", "슬랙으로 메시지를 전송하는 옵션들")
        if group == "x" and x is None:
            x = p.add_argument_group("MI355X / 확장 옵션", "reference 에 없는 옵션들 (--help-all 에서만 표시)") \
                if show_all else p
        kw = dict(opts)
        if group in ("x", "slack*") and not show_all:
            kw["help"] = argparse.SUPPRESS
        {"": p, "slack": g, "slack*": g, "x": x}[group].add_argument(flag, **kw)
    return p


class _Args:
    """The parsed flags as attributes (what argparse's Namespace gives, without importing argparse)."""

    def __init__(self, values: Dict[str, Any]) -> None:
        self.__dict__.update(values)


def _fast_parse(argv: List[str]) -> Optional[Any]:
    """The parse argparse would produce, for command lines made only of exact long flags (``--flag``,
    ``--flag value``, ``--flag=value``) with valid values; ``None`` for anything else (help, errors,
    abbreviations, values that look like options), which then goes through argparse itself."""
    table = {flag: opts for _, flag, opts in _FLAGS}
    ns = {flag[2:].replace("-", "_"): opts.get("default", False if opts.get("action") == "store_true" else None)
          for flag, opts in table.items()}
    i = 0
    while i < len(argv):
        tok = argv[i]
        flag, eq, val = tok.partition("=")
        opts = table.get(flag)
        if opts is None or flag == "--help-all":
            return None
        dest = flag[2:].replace("-", "_")
        if opts.get("action") == "store_true":
            if eq:
                return None
            ns[dest] = True
            i += 1
            continue
        if not eq:
            if i + 1 >= len(argv):
                return None
            val = argv[i + 1]
            if val.startswith("-"):
                return None
            i += 2
        else:
            i += 1
        try:
            v = opts.get("type", str)(val)
        except ValueError:
            return None
        if "choices" in opts and v not in opts["choices"]:
            return None
        ns[dest] = v
    return _Args(ns)


#: the reference's long options in its parser's order (``check-gpu-node.py:298-311``)
_REF_FLAGS = ("--help", "--kubeconfig", "--json", "--slack-webhook", "--slack-username", "--slack-only-on-error",
              "--slack-retry-count", "--slack-retry-delay")


def _reference_abbrevs(argv: List[str]) -> List[str]:
    """argparse accepts any unique prefix of a long option (``--js``, ``--kube PATH``, ``--slack-o``, ``--he``).
    The hidden extension flags (``--json-extended``, ``--kube-timeout``, ``--slack-on-change``, ``--health-*``)
    would make such a prefix ambiguous here while it is unique in the reference: a prefix that names exactly
    one reference flag is spelled out, and one that names several reference flags gets the reference's own
    ``ambiguous option`` error (listing only its flags).  Anything else -- exact flags, prefixes of extension
    flags only, everything after ``--`` -- is left to argparse."""
    known = {flag for _, flag, _ in _FLAGS}
    known.update(("--help", "-h"))
    out: List[str] = []
    for i, tok in enumerate(argv):
        if tok == "--":
            out.extend(argv[i:])
            break
        if tok.startswith("--") and tok not in known:
            prefix, eq, rest = tok.partition("=")
            if prefix not in known:
                hits = [f for f in _REF_FLAGS if f.startswith(prefix)]
                if len(hits) == 1:
                    tok = hits[0] + eq + rest
                elif hits:
                    build_parser().error(f"ambiguous option: {tok} could match {', '.join(hits)}")
        out.append(tok)
    return out


def parse_args(argv: Optional[List[str]] = None) -> Any:
    argv = sys.argv[1:] if argv is None else argv
    if any(t.startswith("--") for t in argv):
        argv = _reference_abbrevs(argv)
    if "--help-all" in argv:
        build_parser(show_all=True).print_help()
        sys.exit(0)
    args = _fast_parse(argv)
    if args is None:
        args = build_parser().parse_args(argv)
    if args.mi355x:
        args.gpu_source = "allocatable"
        args.health_policy = "require"
        args.require_schedulable = True
    if args.json_extended:
        args.json = True
    if args.slack_on_node_change:
        args.slack_on_change = True
    return args


def _load_cluster(args: Any):
    from .kube.config import incluster_connection, load_kube_config
    from .kube.errors import ConfigException
    if args.in_cluster:
        conn = incluster_connection()
        if conn is None:
            raise ConfigException("Service host/port is not set.")
    else:
        conn = load_kube_config(args.kubeconfig, args.context)
    if getattr(args, "kube_env_proxy", False) and not conn.proxy_url:
        # opt-in (PARITY.md #18): the environment's proxy for the apiserver URL, NO_PROXY honoured, as client-go's
        # http.ProxyFromEnvironment does for kubectl; the kubeconfig's proxy-url, when set, wins
        from .utils.http import env_proxy
        conn.proxy_url = env_proxy(conn.server)
    return conn


def _run_once(args: Any) -> int:
    """Reference ``main`` body (``:316-327``) for one iteration."""
    try:
        from .checker import CheckOptions, check_and_report
        cluster = _load_cluster(args)
        opts = CheckOptions.from_args(args)
        prev = None
        if args.state_file:
            from .utils import statefile
            prev = statefile.load(args.state_file)
            if args.slack_on_change:
                opts.slack_webhook = statefile.gate_webhook(prev, opts, cluster, args.slack_on_node_change)
        result = check_and_report(cluster, opts)
        if args.state_file:
            statefile.save(args.state_file, result, prev)
        if args.prometheus_textfile:
            from .utils.prom import write_textfile
            write_textfile(args.prometheus_textfile, result)
        return result.exit_code
    except Exception as e:
        return _report_error(args, e)


def _report_error(args: Any, e: BaseException) -> int:
    """Reference error reporter (``:319-327``): JSON one-liner on stdout or message + traceback."""
    import json
    if getattr(args, "json", False):
        print(json.dumps({"error": str(e)}, ensure_ascii=False))
    else:
        import traceback
        print(f"에러: {e}", file=sys.stderr)
        traceback.print_exc()
    if args.prometheus_textfile:
        try:
            from .utils.prom import write_error_textfile
            write_error_textfile(args.prometheus_textfile, str(e))
        except Exception:
            pass
    return 1


def main(argv: Optional[List[str]] = None) -> int:
    args = parse_args(argv)
    if args.explain:
        try:
            from .checker import CheckOptions
            from .explain import explain
            return explain(_load_cluster(args), args.explain, CheckOptions.from_args(args), sys.stdout)
        except Exception as e:
            return _report_error(args, e)
    if args.fleet:
        try:
            from .checker import CheckOptions
            from .explain import fleet
            return fleet(_load_cluster(args), CheckOptions.from_args(args), sys.stdout)
        except Exception as e:
            return _report_error(args, e)
    if args.watch_events:
        return _watch_events(args)
    if args.watch and args.watch > 0:
        return _watch(args)
    return _run_once(args)


def _watch_events(args: Any) -> int:
    """``--watch-events``: LIST once, follow the watch stream, report each change of outcome.

    Every report is a complete one-shot report (same JSON/text, same exit-code rule); Slack goes
    through the ``--slack-on-change`` de-dup gate (first report, changes, one recovery notice under
    ``--slack-only-on-error``).  Ends after ``--watch-count`` reports, ``--watch-duration`` seconds
    or Ctrl-C, with the exit code of the last report.
    """
    last = {"code": 0}
    try:
        from .checker import CheckOptions, CheckResult, apply_health, apply_schedulability, emit_report
        from .kube.watch import NodeWatcher
        from .utils import statefile
        from .utils.timing import NullTracer, Tracer
        cluster = _load_cluster(args)
        opts = CheckOptions.from_args(args)
        prev = statefile.load(args.state_file) if args.state_file else None
        memo = {"prev": prev}
        only = opts.slack_only_on_error
        opts.slack_gate = lambda result: statefile.should_notify(memo["prev"], result, only,
                                                                 args.slack_on_node_change)
        opts.slack_only_on_error = False  # the gate decides (a recovery must be able to send)
        if opts.probe_endpoint:
            # every batch of events re-evaluates the fleet: reuse the agents' reports and EndpointSlices a while
            from .parallel.fanout import ProbeCache
            opts.probe_cache = ProbeCache(opts.probe_cache_ttl)
        metrics = None
        if args.metrics_listen:
            from .utils.prom import MetricsServer, parse_listen
            metrics = MetricsServer(*parse_listen(args.metrics_listen)).start()
            print(f"metrics: serving http://{args.metrics_listen.rpartition(':')[0] or '0.0.0.0'}:{metrics.port}"
                  "/metrics", file=sys.stderr, flush=True)
        elector = None

        def evaluate(scan):
            tr = Tracer() if (opts.trace or opts.json_extended) else NullTracer()
            warnings: list = []
            fleet: dict = {}
            result = CheckResult(scan, apply_health(scan, opts, tr, warnings, cluster, fleet), tr)
            result.warnings = warnings
            result.fleet_diag = fleet.get("summary")
            apply_schedulability(scan, opts)
            return result

        def report(result) -> None:
            emit_report(result, opts)
            memo["prev"] = statefile.outcome(result)
            if args.state_file:
                statefile.save(args.state_file, result, prev)
            if args.prometheus_textfile:
                from .utils.prom import write_textfile
                write_textfile(args.prometheus_textfile, result)
            if metrics is not None:
                metrics.update(result)
            if elector is not None:
                # the last-notified outcome rides on the Lease: a replica taking over starts from it (no repeated
                # alert, no lost recovery notice across a failover)
                if not elector.publish_state(statefile.compact(memo["prev"])):
                    print("leader state does not fit the Lease even compacted: a replica taking over starts "
                          "without it", file=sys.stderr, flush=True)
            last["code"] = result.exit_code

        if not args.leader_elect:
            try:
                NodeWatcher(cluster, opts, debounce=args.watch_debounce).run(
                    evaluate, report, max_reports=args.watch_count, duration=args.watch_duration)
            finally:
                if metrics is not None:
                    metrics.stop()
            return last["code"]
        elector = _start_elector(args, cluster)
        if metrics is not None:
            metrics.set_leader(False)
        try:
            while not elector.leading.wait(0.2):
                pass
            if elector.inherited_state:  # {}: the previous holder's state was too large to keep on the Lease
                memo["prev"] = elector.inherited_state
            if metrics is not None:
                metrics.set_leader(True)
            print(f"leader election: {elector.identity} leads {elector.namespace}/{elector.name}"
                  + (" (resuming the previous leader's notification state)" if elector.inherited_state else ""),
                  file=sys.stderr, flush=True)
            NodeWatcher(cluster, opts, debounce=args.watch_debounce).run(
                evaluate, report, max_reports=args.watch_count, duration=args.watch_duration,
                should_stop=lambda: not elector.is_leader())
            if elector.lost.is_set() or not elector.is_leader():
                # client-go's rule: a replica that could not renew in time stops acting and exits; the
                # Deployment restarts it as a candidate
                print(f"leader election: {elector.identity} lost {elector.namespace}/{elector.name} "
                      f"({elector.last_error or 'not renewed in time'}): stopping", file=sys.stderr, flush=True)
            return last["code"]
        finally:
            elector.stop()  # a holder releases the Lease: the next replica takes over without waiting it out
            if metrics is not None:
                metrics.stop()
    except KeyboardInterrupt:
        return last["code"]
    except Exception as e:
        return _report_error(args, e)


def _start_elector(args: Any, cluster: Any) -> Any:
    """``--leader-elect``: campaign for the Lease (kube/lease.py) from a thread; SIGTERM (pod deletion, rolling
    update) ends the watch like Ctrl-C, so the holder releases the Lease on its way out."""
    import signal
    import threading
    from .kube.client import KubeClient
    from .kube.lease import LeaderElector, default_identity, default_namespace
    spec = args.leader_elect_lease or f"{default_namespace()}/gpu-node-watcher"
    ns, _, name = spec.rpartition("/")
    try:
        duration, renew, retry = (float(x) for x in args.leader_elect_timing.split(","))
    except ValueError:
        raise ValueError(f"--leader-elect-timing: three numbers 'lease,renew,retry', not {args.leader_elect_timing!r}")
    if threading.current_thread() is threading.main_thread():
        def _term(*_: Any) -> None:
            raise KeyboardInterrupt
        signal.signal(signal.SIGTERM, _term)
    elector = LeaderElector(lambda: KubeClient(cluster, timeout=max(0.5, min(5.0, renew / 2)), retries=0),
                            ns or default_namespace(), name, default_identity(), duration, renew, retry)
    print(f"leader election: {elector.identity} campaigning for {elector.namespace}/{elector.name}", file=sys.stderr,
          flush=True)
    return elector.start()


def _watch(args: Any) -> int:
    """Repeat the check every ``--watch`` seconds (fixed cadence, not fixed sleep).

    Ends after ``--watch-count`` checks (0 = forever) or on Ctrl-C, with the
    exit code of the last completed check.  Combine with ``--state-file
    --slack-on-change`` for de-duplicated alerts from a long-running Pod.
    """
    import time
    code = 0
    n = 0
    next_at = time.monotonic()
    try:
        while True:
            code = _run_once(args)
            n += 1
            sys.stdout.flush()
            if args.watch_count > 0 and n >= args.watch_count:
                return code
            next_at += args.watch
            now = time.monotonic()
            if next_at < now:  # a check overran the period: skip the missed slots
                next_at = now
            time.sleep(next_at - now)
    except KeyboardInterrupt:
        return code


def entry() -> None:
    """Console-script entry: load ``.env`` (reference ``:331``) then exit with ``main()``."""
    from .utils.dotenv import load_dotenv
    load_dotenv()
    sys.exit(main())


if __name__ == "__main__":
    entry()
