"""Stand-in ``kubernetes.client``: ``CoreV1Api.list_node`` over ``requests``."""
import requests

from .config import _STATE


class _Model:
    def __init__(self, **kw):
        self.__dict__.update(kw)


class V1NodeCondition(_Model):
    pass


class V1Taint(_Model):
    pass


class V1Node(_Model):
    pass


class V1NodeList(_Model):
    pass


class ApiException(Exception):
    def __init__(self, status=None, reason=None, headers=None, body=None):
        self.status, self.reason, self.headers, self.body = status, reason, headers, body

    def __str__(self):
        msg = "({0})\nReason: {1}\n".format(self.status, self.reason)
        if self.headers:
            msg += "HTTP response headers: HTTPHeaderDict({0})\n".format(self.headers)
        if self.body:
            msg += "HTTP response body: {0}\n".format(self.body)
        return msg


def _strdict(d):
    if d is None:
        return None
    return {k: (None if v is None else str(v)) for k, v in d.items()}


def _node(raw):
    meta = raw.get("metadata")
    spec = raw.get("spec")
    status = raw.get("status")
    m = None if meta is None else _Model(name=meta.get("name"), labels=meta.get("labels"),
                                        annotations=meta.get("annotations"))
    s = None
    if spec is not None:
        taints = spec.get("taints")
        s = _Model(taints=None if taints is None else [V1Taint(key=t.get("key"), value=t.get("value"),
                                                                effect=t.get("effect")) for t in taints])
    st = None
    if status is not None:
        conds = status.get("conditions")
        st = _Model(capacity=_strdict(status.get("capacity")), allocatable=_strdict(status.get("allocatable")),
                    conditions=None if conds is None else [V1NodeCondition(type=c.get("type"), status=c.get("status"))
                                                           for c in conds])
    return V1Node(metadata=m, spec=s, status=st)


class CoreV1Api:
    def list_node(self, **kwargs):
        headers = {"Accept": "application/json"}
        if _STATE.get("token"):
            headers["Authorization"] = "Bearer " + _STATE["token"]
        r = requests.get(_STATE["server"] + "/api/v1/nodes", headers=headers)
        if not 200 <= r.status_code < 300:
            raise ApiException(r.status_code, r.reason, dict(r.headers), r.text)
        doc = r.json()
        return V1NodeList(items=[_node(i) for i in (doc.get("items") or [])])
