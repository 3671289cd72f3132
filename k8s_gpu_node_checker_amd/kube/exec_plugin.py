"""kubeconfig ``exec`` credential plugins (``client.authentication.k8s.io``).

Runs the configured command (e.g. ``aws eks get-token``, ``gke-gcloud-auth-plugin``)
as a child process, passes ``KUBERNETES_EXEC_INFO`` and parses the
``ExecCredential`` it prints.  In the reference this happens inside
``kubernetes.config.load_kube_config`` (SURVEY §3.1 "exec credential plugins
spawn a subprocess here").
"""

from __future__ import annotations

import json
import os
import shutil
import subprocess
from datetime import datetime
from typing import Any, Dict, Optional, Tuple

from .errors import ConfigException


def _parse_ts(ts: Optional[str]) -> float:
    if not ts:
        return 0.0
    try:
        return datetime.fromisoformat(ts.replace("Z", "+00:00")).timestamp()
    except ValueError:
        return 0.0


def run_exec_plugin(spec: Dict[str, Any], base: Optional[str], conn: Any = None,
                    timeout: float = 60.0) -> Tuple[Dict[str, Any], float]:
    """Return ``(ExecCredential.status, expiry_epoch or 0)``."""
    command = spec.get("command")
    if not command:
        raise ConfigException("exec: missing command")
    api_version = spec.get("apiVersion") or "client.authentication.k8s.io/v1"
    if "/" in command and not os.path.isabs(command) and base:
        command = os.path.join(base, command)
    elif "/" not in command:
        command = shutil.which(command) or command
    env = dict(os.environ)
    for item in spec.get("env") or []:
        if isinstance(item, dict) and "name" in item:
            env[str(item["name"])] = str(item.get("value", ""))
    info: Dict[str, Any] = {"apiVersion": api_version, "kind": "ExecCredential",
                            "spec": {"interactive": False}}
    if spec.get("provideClusterInfo"):
        c = dict(spec.get("__cluster__") or {})
        cluster: Dict[str, Any] = {"server": c.get("server")}
        if c.get("certificate-authority-data"):
            cluster["certificate-authority-data"] = c["certificate-authority-data"]
        if c.get("insecure-skip-tls-verify"):
            cluster["insecure-skip-tls-verify"] = True
        if c.get("tls-server-name"):
            cluster["tls-server-name"] = c["tls-server-name"]
        if c.get("proxy-url"):
            cluster["proxy-url"] = c["proxy-url"]
        if c.get("config") is not None:
            cluster["config"] = c["config"]
        info["spec"]["cluster"] = cluster
    env["KUBERNETES_EXEC_INFO"] = json.dumps(info)
    args = [command] + [str(a) for a in (spec.get("args") or [])]
    try:
        proc = subprocess.run(args, env=env, stdin=subprocess.DEVNULL, stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, timeout=timeout, check=False)
    except (OSError, subprocess.TimeoutExpired) as e:
        hint = spec.get("installHint")
        raise ConfigException("exec: failed to run %s: %s%s" % (spec.get("command"), e,
                                                                 ("\n" + hint) if hint else ""))
    if proc.returncode != 0:
        raise ConfigException("exec: process returned %d. %s" % (proc.returncode,
                                                                 proc.stderr.decode(errors="replace").strip()))
    try:
        cred = json.loads(proc.stdout)
    except ValueError as e:
        raise ConfigException("exec: failed to decode process output: %s" % e)
    if not isinstance(cred, dict) or cred.get("kind") != "ExecCredential":
        raise ConfigException("exec: output is not an ExecCredential")
    if cred.get("apiVersion") and cred.get("apiVersion") != api_version:
        raise ConfigException("exec: plugin api version %s does not match %s" % (cred.get("apiVersion"), api_version))
    status = cred.get("status") or {}
    if not (status.get("token") or (status.get("clientCertificateData") and status.get("clientKeyData"))):
        raise ConfigException("exec: missing token or clientCertificateData field in plugin output")
    return status, _parse_ts(status.get("expirationTimestamp"))

