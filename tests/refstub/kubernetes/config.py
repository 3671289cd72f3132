"""Stand-in ``kubernetes.config``: resolves server + bearer token from a kubeconfig."""
import os

import yaml

_STATE = {"server": None, "token": None, "calls": []}


class ConfigException(Exception):
    pass


def load_kube_config(config_file=None, context=None, **kwargs):
    _STATE["calls"].append(config_file)
    if os.environ.get("REFSTUB_TRACE"):
        with open(os.environ["REFSTUB_TRACE"], "a") as f:
            f.write(repr(config_file) + "\n")
    paths = config_file if config_file is not None else os.environ.get("KUBECONFIG", os.path.expanduser("~/.kube/config"))
    cfg = None
    for p in str(paths).split(os.pathsep):
        if p and os.path.exists(p):
            with open(p) as f:
                cfg = yaml.safe_load(f)
            if cfg:
                break
    if not cfg:
        raise ConfigException("Invalid kube-config file. No configuration found.")
    ctx = next(c for c in cfg["contexts"] if c["name"] == cfg["current-context"])["context"]
    cluster = next(c for c in cfg["clusters"] if c["name"] == ctx["cluster"])["cluster"]
    user = next((u for u in cfg.get("users") or [] if u["name"] == ctx.get("user")), {}).get("user") or {}
    _STATE["server"] = cluster["server"]
    _STATE["token"] = user.get("token")
