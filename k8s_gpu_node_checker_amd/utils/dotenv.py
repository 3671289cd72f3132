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
import re
import sys
from typing import Dict, Iterator, Optional, Tuple

_LINE = re.compile(r"^\s*(?:export\s+)?([A-Za-z_][A-Za-z0-9_.\-]*)\s*(?:=\s*(.*))?$")
_EXPAND = re.compile(r"\$\{([A-Za-z_][A-Za-z0-9_]*)(?::-([^}]*))?\}")
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
    m = re.search(r"\s#", raw)
    if m:
        raw = raw[:m.start()]
    return raw.strip(), True


def parse_dotenv(text: str) -> Iterator[Tuple[str, Optional[str], bool]]:
    for line in text.splitlines():
        s = line.strip()
        if not s or s.startswith("#"):
            continue
        m = _LINE.match(line)
        if not m:
            continue
        key, rhs = m.group(1), m.group(2)
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
            def sub(m: "re.Match[str]") -> str:
                name = m.group(1)
                got = env.get(name)
                if got is None:
                    got = values.get(name)
                if got is None or got == "":
                    return m.group(2) or ""
                return got
            val = _EXPAND.sub(sub, val)
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
