"""MI355X-native Kubernetes GPU-node checker.

Same CLI flags, JSON schema, exit codes and Slack behaviour as
ahaljh/k8s-gpu-node-checker (``check-gpu-node.py``), re-centred on
``amd.com/gpu`` and gated on an amd-smi health probe of every MI355X
(gfx950, 288 GB HBM3E, ECC, xGMI).  See ``SURVEY.md`` for the component map.

Layout::

    cli.py, checker.py, report.py   CLI / orchestration / presentation
    models/                         resource registry, node projection, MI355X health model
    kube/                           kubeconfig + auth, apiserver client
    notify/                         Slack webhook sender
    ops/                            native code: NodeList fast path, amd-smi probe, HIP diagnostics
    parallel/                       async per-node fan-out, RCCL/xGMI collective diagnostics
    agent/                          DaemonSet node agent (probe -> annotation / HTTP)
    testing/                        mock kube-apiserver, webhook sink, cluster fixtures
    utils/                          HTTP transport, backoff, dotenv, tracing, metrics, state
"""

__version__ = "0.1.0"

__all__ = ["__version__"]
