"""A small evaluator for the subset of CEL (Common Expression Language) that ``deploy/agent-policy.yaml`` uses.

Kubernetes evaluates ValidatingAdmissionPolicy expressions with cel-go; there is no CEL library in this
environment, so the tests evaluate the policy's own expressions with this one against admission requests
for allowed and refused writes.  Covered: literals (int, string, bool, null, lists, maps), field selection
and indexing on JSON-like values, ``has()``, ``size()``, ``in``, ``== != < <= > >=``, ``+ -``, ``! && ||``
(commutative with errors, as CEL's are), ``? :``, the ``all / exists / filter / map`` macros on lists and
maps (maps iterate their keys), and the string methods ``startsWith / endsWith / contains``.
Variables (``variables.<name>``) are evaluated lazily in the policy's order.
"""

from __future__ import annotations

from typing import Any, Callable, Dict, List, Optional, Tuple


class CelError(Exception):
    """An evaluation error (missing field, type mismatch): CEL's error value."""


_PUNCT = ("&&", "||", "==", "!=", "<=", ">=", "!", "<", ">", "?", ":", ".", ",", "(", ")", "[", "]", "{", "}",
          "+", "-")


def tokenize(src: str) -> List[Tuple[str, Any]]:
    out: List[Tuple[str, Any]] = []
    i, n = 0, len(src)
    while i < n:
        c = src[i]
        if c.isspace():
            i += 1
            continue
        if c in "'\"":
            j, buf = i + 1, []
            while j < n and src[j] != c:
                if src[j] == "\\" and j + 1 < n:
                    buf.append({"n": "\n", "t": "\t"}.get(src[j + 1], src[j + 1]))
                    j += 2
                    continue
                buf.append(src[j])
                j += 1
            if j >= n:
                raise SyntaxError("unterminated string")
            out.append(("str", "".join(buf)))
            i = j + 1
            continue
        if c.isdigit():
            j = i
            while j < n and src[j].isdigit():
                j += 1
            out.append(("int", int(src[i:j])))
            i = j
            continue
        if c.isalpha() or c == "_":
            j = i
            while j < n and (src[j].isalnum() or src[j] == "_"):
                j += 1
            word = src[i:j]
            out.append(("kw", word) if word in ("true", "false", "null", "in") else ("id", word))
            i = j
            continue
        for p in _PUNCT:
            if src.startswith(p, i):
                out.append(("op", p))
                i += len(p)
                break
        else:
            raise SyntaxError(f"unexpected {c!r} at {i}")
    out.append(("end", None))
    return out


class _Parser:
    def __init__(self, src: str):
        self.toks = tokenize(src)
        self.i = 0

    def peek(self, kind: str, val: Any = None) -> bool:
        k, v = self.toks[self.i]
        return k == kind and (val is None or v == val)

    def take(self, kind: str, val: Any = None) -> Any:
        if not self.peek(kind, val):
            raise SyntaxError(f"expected {val or kind}, got {self.toks[self.i]}")
        v = self.toks[self.i][1]
        self.i += 1
        return v

    def parse(self) -> tuple:
        e = self.expr()
        self.take("end")
        return e

    def expr(self) -> tuple:
        c = self.or_()
        if self.peek("op", "?"):
            self.take("op", "?")
            a = self.expr()
            self.take("op", ":")
            b = self.expr()
            return ("cond", c, a, b)
        return c

    def or_(self) -> tuple:
        e = self.and_()
        while self.peek("op", "||"):
            self.take("op")
            e = ("or", e, self.and_())
        return e

    def and_(self) -> tuple:
        e = self.rel()
        while self.peek("op", "&&"):
            self.take("op")
            e = ("and", e, self.rel())
        return e

    def rel(self) -> tuple:
        e = self.add()
        for op in ("==", "!=", "<=", ">=", "<", ">"):
            if self.peek("op", op):
                self.take("op")
                return ("bin", op, e, self.add())
        if self.peek("kw", "in"):
            self.take("kw")
            return ("in", e, self.add())
        return e

    def add(self) -> tuple:
        e = self.unary()
        while self.peek("op", "+") or self.peek("op", "-"):
            op = self.take("op")
            e = ("bin", op, e, self.unary())
        return e

    def unary(self) -> tuple:
        if self.peek("op", "!"):
            self.take("op")
            return ("not", self.unary())
        if self.peek("op", "-"):
            self.take("op")
            return ("neg", self.unary())
        return self.member()

    def args(self) -> List[tuple]:
        self.take("op", "(")
        out: List[tuple] = []
        while not self.peek("op", ")"):
            out.append(self.expr())
            if not self.peek("op", ")"):
                self.take("op", ",")
        self.take("op", ")")
        return out

    def member(self) -> tuple:
        e = self.primary()
        while True:
            if self.peek("op", "."):
                self.take("op")
                name = self.take("id")
                if self.peek("op", "("):
                    e = ("call", name, e, self.args())
                else:
                    e = ("sel", e, name)
            elif self.peek("op", "["):
                self.take("op")
                idx = self.expr()
                self.take("op", "]")
                e = ("index", e, idx)
            else:
                return e

    def primary(self) -> tuple:
        k, v = self.toks[self.i]
        if k in ("int", "str"):
            self.i += 1
            return ("lit", v)
        if k == "kw" and v in ("true", "false", "null"):
            self.i += 1
            return ("lit", {"true": True, "false": False, "null": None}[v])
        if k == "id":
            self.i += 1
            if self.peek("op", "("):
                return ("call", v, None, self.args())
            return ("ident", v)
        if self.peek("op", "("):
            self.take("op")
            e = self.expr()
            self.take("op", ")")
            return e
        if self.peek("op", "["):
            self.take("op")
            items: List[tuple] = []
            while not self.peek("op", "]"):
                items.append(self.expr())
                if not self.peek("op", "]"):
                    self.take("op", ",")
            self.take("op", "]")
            return ("list", items)
        if self.peek("op", "{"):
            self.take("op")
            pairs: List[Tuple[tuple, tuple]] = []
            while not self.peek("op", "}"):
                key = self.expr()
                self.take("op", ":")
                pairs.append((key, self.expr()))
                if not self.peek("op", "}"):
                    self.take("op", ",")
            self.take("op", "}")
            return ("map", pairs)
        raise SyntaxError(f"unexpected {self.toks[self.i]}")


def parse(src: str) -> tuple:
    return _Parser(src).parse()


class Env:
    """Top-level bindings plus lazily evaluated ``variables.<name>`` (a policy's ``spec.variables``)."""

    def __init__(self, bindings: Dict[str, Any], variables: Optional[List[Tuple[str, str]]] = None):
        self.bindings = dict(bindings)
        self.var_src = {name: parse(src) for name, src in (variables or [])}
        self.var_val: Dict[str, Any] = {}

    def variable(self, name: str) -> Any:
        if name not in self.var_val:
            if name not in self.var_src:
                raise CelError(f"no variable {name}")
            try:
                self.var_val[name] = ("ok", evaluate(self.var_src[name], self))
            except CelError as e:
                self.var_val[name] = ("err", e)
        kind, v = self.var_val[name]
        if kind == "err":
            raise v
        return v


class _Vars:
    def __init__(self, env: Env):
        self.env = env


def _select(obj: Any, name: str) -> Any:
    if isinstance(obj, _Vars):
        return obj.env.variable(name)
    if isinstance(obj, dict):
        if name not in obj:
            raise CelError(f"no such key: {name}")
        return obj[name]
    raise CelError(f"cannot select {name} from {type(obj).__name__}")


def _has(node: tuple, env: Env) -> bool:
    if node[0] != "sel":
        raise CelError("has() needs a field selection")
    obj = evaluate(node[1], env)
    if isinstance(obj, dict):
        return node[2] in obj and obj[node[2]] is not None
    raise CelError("has() on a non-map")


def _eq(a: Any, b: Any) -> bool:
    if isinstance(a, bool) != isinstance(b, bool):
        return False
    return a == b


def _truth(v: Any) -> bool:
    if not isinstance(v, bool):
        raise CelError(f"expected bool, got {type(v).__name__}")
    return v


def _macro(name: str, recv: Any, args: List[tuple], env: Env) -> Any:
    if len(args) != 2 or args[0][0] != "ident":
        raise CelError(f"{name}() needs (var, expr)")
    var = args[0][1]
    items = list(recv.keys()) if isinstance(recv, dict) else recv
    if not isinstance(items, list):
        raise CelError(f"{name}() on {type(recv).__name__}")

    def run(x: Any) -> Any:
        saved = env.bindings.get(var, _MISSING)
        env.bindings[var] = x
        try:
            return evaluate(args[1], env)
        finally:
            if saved is _MISSING:
                del env.bindings[var]
            else:
                env.bindings[var] = saved
    if name == "all":
        return all(_truth(run(x)) for x in items)
    if name == "exists":
        return any(_truth(run(x)) for x in items)
    if name == "filter":
        return [x for x in items if _truth(run(x))]
    return [run(x) for x in items]  # map


_MISSING = object()
_STR_METHODS: Dict[str, Callable[[str, str], bool]] = {
    "startsWith": str.startswith, "endsWith": str.endswith, "contains": lambda s, p: p in s}


def evaluate(node: tuple, env: Env) -> Any:
    kind = node[0]
    if kind == "lit":
        return node[1]
    if kind == "ident":
        name = node[1]
        if name == "variables":
            return _Vars(env)
        if name not in env.bindings:
            raise CelError(f"undeclared reference {name}")
        return env.bindings[name]
    if kind == "sel":
        return _select(evaluate(node[1], env), node[2])
    if kind == "index":
        obj, idx = evaluate(node[1], env), evaluate(node[2], env)
        if isinstance(obj, dict):
            if idx not in obj:
                raise CelError(f"no such key: {idx}")
            return obj[idx]
        if isinstance(obj, list) and isinstance(idx, int) and not isinstance(idx, bool):
            if not 0 <= idx < len(obj):
                raise CelError("index out of range")
            return obj[idx]
        raise CelError("bad index")
    if kind == "list":
        return [evaluate(x, env) for x in node[1]]
    if kind == "map":
        return {evaluate(k, env): evaluate(v, env) for k, v in node[1]}
    if kind == "not":
        return not _truth(evaluate(node[1], env))
    if kind == "neg":
        v = evaluate(node[1], env)
        if not isinstance(v, int) or isinstance(v, bool):
            raise CelError("negation of a non-int")
        return -v
    if kind in ("and", "or"):
        decisive = kind == "or"  # the value that settles the operator on its own
        err: Optional[CelError] = None
        for side in (node[1], node[2]):
            try:
                v = _truth(evaluate(side, env))
            except CelError as e:  # CEL's logical operators are commutative with errors
                err = err or e
                continue
            if v == decisive:
                return decisive
        if err is not None:
            raise err
        return not decisive
    if kind == "cond":
        return evaluate(node[2] if _truth(evaluate(node[1], env)) else node[3], env)
    if kind == "in":
        elem, coll = evaluate(node[1], env), evaluate(node[2], env)
        if isinstance(coll, dict):
            return elem in coll
        if isinstance(coll, list):
            return any(_eq(elem, x) for x in coll)
        raise CelError("'in' needs a list or map")
    if kind == "bin":
        op, a, b = node[1], evaluate(node[2], env), evaluate(node[3], env)
        if op == "==":
            return _eq(a, b)
        if op == "!=":
            return not _eq(a, b)
        if op == "+":
            if type(a) is not type(b) or not isinstance(a, (int, str, list)):
                raise CelError("bad operands for +")
            return a + b
        if op == "-":
            if not (isinstance(a, int) and isinstance(b, int)):
                raise CelError("bad operands for -")
            return a - b
        if type(a) is not type(b) or not isinstance(a, (int, str)):
            raise CelError(f"bad operands for {op}")
        return {"<": a < b, "<=": a <= b, ">": a > b, ">=": a >= b}[op]
    if kind == "call":
        name, recv_node, args = node[1], node[2], node[3]
        if recv_node is None:
            if name == "has":
                return _has(args[0], env)
            if name == "size":
                v = evaluate(args[0], env)
                if not isinstance(v, (str, list, dict)):
                    raise CelError("size() of a scalar")
                return len(v)
            raise CelError(f"unknown function {name}")
        recv = evaluate(recv_node, env)
        if name in ("all", "exists", "filter", "map"):
            return _macro(name, recv, args, env)
        if name in _STR_METHODS:
            arg = evaluate(args[0], env)
            if not isinstance(recv, str) or not isinstance(arg, str):
                raise CelError(f"{name}() on a non-string")
            return _STR_METHODS[name](recv, arg)
        raise CelError(f"unknown method {name}")
    raise CelError(f"bad node {kind}")


def eval_expr(src: str, bindings: Dict[str, Any], variables: Optional[List[Tuple[str, str]]] = None) -> Any:
    return evaluate(parse(src), Env(bindings, variables))


def admit(policy: Dict[str, Any], request: Dict[str, Any], obj: Any, old: Any) -> Tuple[Optional[bool], str]:
    """Apply a ValidatingAdmissionPolicy's spec to one request: (None, '') when its matchConditions do not
    select the request, (True, '') when every validation holds, else (False, the first failure's message).  An
    evaluation error counts as a failure (failurePolicy: Fail)."""
    spec = policy["spec"]
    rules = spec["matchConstraints"]["resourceRules"]
    res = request["resource"]["resource"] + ("/" + request["subResource"] if request.get("subResource") else "")
    if not any(res in r["resources"] and request["operation"] in r["operations"] for r in rules):
        return None, ""
    env = Env({"request": request, "object": obj, "oldObject": old},
              [(v["name"], v["expression"]) for v in spec.get("variables") or []])
    for mc in spec.get("matchConditions") or []:
        if not _truth(evaluate(parse(mc["expression"]), env)):
            return None, ""
    for v in spec["validations"]:
        try:
            ok = _truth(evaluate(parse(v["expression"]), env))
        except CelError as e:
            return False, f"{v.get('message', '')} (evaluation error: {e})"
        if not ok:
            msg = v.get("message", "")
            if v.get("messageExpression"):
                try:
                    msg = str(evaluate(parse(v["messageExpression"]), env))
                except CelError:
                    pass
            return False, msg
    return True, ""
