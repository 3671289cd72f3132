"""Minimal ``.env`` loader (replaces python-dotenv).

The reference calls ``load_dotenv()`` under ``__main__`` only
(``check-gpu-node.py:331``); python-dotenv then searches for ``.env`` from
the running script's directory up to ``/`` and never overrides variables that
are already set.  This module keeps those semantics (``override=False``) and
supports the syntax the ``.env-template`` needs and the common extras:

* ``KEY=value``, ``export KEY=value``, blank lines and ``# comments``
* single quotes (literal), double quotes (``\\n``, ``\\t``, ``\\"``, ``\\\\`` escapes)
* ``value # trailing comment`` for unquoted values
* ``${VAR}`` / ``${VAR:-default}`` expansion (existing environment first)
"""

from __future__ import annotations

import os
import sys
TYPE_CHECKING = False
if TYPE_CHECKING:  # annotations only (PEP 563): importing typing is ~10 ms of a cold start
    from typing import Callable, Dict, Iterator, Optional, Tuple

_KEY_CHARS = frozenset("ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789_.-")
_DQ_ESC = {"n": "\n", "t": "\t", "r": "\r", '"': '"', "\\": "\\", "'": "'", "$": "$"}


def _unquote(raw: str) -> Tuple[str, bool]:
    """Return (value, expand) for the right-hand side of an assignment."""
    raw = raw.strip()
    if raw[:1] == "'":
        end = raw.find("'", 1)
        return (raw[1:end] if end > 0 else raw[1:]), False
    if raw[:1] == '"':
        out = []
        i = 1
        while i < len(raw):
            c = raw[i]
            if c == "\\" and i + 1 < len(raw):
                out.append(_DQ_ESC.get(raw[i + 1], "\\" + raw[i + 1]))
                i += 2
                continue
            if c == '"':
                break
            out.append(c)
            i += 1
        return "".join(out), True
    for i in range(1, len(raw)):
        if raw[i] == "#" and raw[i - 1] in " \t":
            raw = raw[:i]
            break
    return raw.strip(), True


def _split_line(line: str) -> Optional[Tuple[str, Optional[str]]]:
    s = line.strip()
    if s.startswith("export ") or s.startswith("export\t"):
        s = s[7:].lstrip()
    eq = s.find("=")
    key = (s if eq < 0 else s[:eq]).rstrip()
    if not key or not (key[0].isalpha() or key[0] == "_") or not all(c in _KEY_CHARS for c in key):
        return None
    return key, (None if eq < 0 else s[eq + 1:].lstrip())


def _expand(val: str, lookup: Callable[[str], Optional[str]]) -> str:
    """``${VAR}`` / ``${VAR:-default}`` expansion."""
    out = []
    i = 0
    while i < len(val):
        j = val.find("${", i)
        k = val.find("}", j + 2) if j >= 0 else -1
        if j < 0 or k < 0:
            out.append(val[i:])
            break
        out.append(val[i:j])
        name, _, default = val[j + 2:k].partition(":-")
        if name and (name[0].isalpha() or name[0] == "_") and all(c.isalnum() or c == "_" for c in name):
            got = lookup(name)
            out.append(got if got else default)
        else:
            out.append(val[j:k + 1])
        i = k + 1
    return "".join(out)


def parse_dotenv(text: str) -> Iterator[Tuple[str, Optional[str], bool]]:
    for line in text.splitlines():
        s = line.strip()
        if not s or s.startswith("#"):
            continue
        kv = _split_line(line)
        if kv is None:
            continue
        key, rhs = kv
        if rhs is None:
            yield key, None, False
            continue
        val, expand = _unquote(rhs)
        yield key, val, expand


def dotenv_values(path: str, environ: Optional[Dict[str, str]] = None) -> Dict[str, Optional[str]]:
    env = os.environ if environ is None else environ
    try:
        with open(path, encoding="utf-8") as f:
            text = f.read()
    except OSError:
        return {}
    values: Dict[str, Optional[str]] = {}
    for key, val, expand in parse_dotenv(text):
        if val is not None and expand and "${" in val:
            val = _expand(val, lambda name: env.get(name) if env.get(name) is not None else values.get(name))
        values[key] = val
    return values


def find_dotenv(filename: str = ".env", start: Optional[str] = None) -> str:
    """Search ``filename`` from ``start`` (default: the script's directory, then cwd) up to ``/``."""
    starts = []
    if start:
        starts.append(start)
    else:
        script = sys.argv[0] if sys.argv and sys.argv[0] else ""
        if script and os.path.isfile(script):
            starts.append(os.path.dirname(os.path.abspath(script)))
        starts.append(os.getcwd())
    seen = set()
    for s in starts:
        d = os.path.abspath(s)
        while True:
            if d not in seen:
                seen.add(d)
                cand = os.path.join(d, filename)
                if os.path.isfile(cand):
                    return cand
            parent = os.path.dirname(d)
            if parent == d:
                break
            d = parent
    return ""


def load_dotenv(path: Optional[str] = None, override: bool = False) -> bool:
    """Load ``.env`` into ``os.environ``; existing variables win unless ``override``."""
    path = path or find_dotenv()
    if not path:
        return False
    vals = dotenv_values(path)
    for k, v in vals.items():
        if v is None:
            continue
        if override or k not in os.environ:
            os.environ[k] = v
    return bool(vals)
