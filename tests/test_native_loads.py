"""ops.fastpath.loads (native JSON parser of the health annotation) == json.loads, value for value and
type for type; every document it cannot prove identical goes to json.loads (same result / exception)."""
import json
import math

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from k8s_gpu_node_checker_amd.ops import fastpath
from k8s_gpu_node_checker_amd.testing import fixtures

pytestmark = pytest.mark.skipif(fastpath.ext() is None, reason="native extension not built")


def same(a, b):
    if isinstance(a, float) and isinstance(b, float) and math.isnan(a) and math.isnan(b):
        return True
    if type(a) is not type(b):
        return False
    if isinstance(a, dict):
        return list(a) == list(b) and all(same(a[k], b[k]) for k in a)
    if isinstance(a, list):
        return len(a) == len(b) and all(same(x, y) for x, y in zip(a, b))
    if isinstance(a, float):
        return a == b and math.copysign(1, a) == math.copysign(1, b)
    return a == b


def check(doc):
    try:
        ref = json.loads(doc)
    except Exception as e:
        with pytest.raises(type(e)):
            fastpath.loads(doc)
        return
    got = fastpath.loads(doc)
    assert same(got, ref), (doc, got, ref)


json_values = st.recursive(
    st.none() | st.booleans() | st.integers(min_value=-10**30, max_value=10**30) |
    st.floats(allow_nan=True, allow_infinity=True) | st.text(),
    lambda kids: st.lists(kids, max_size=4) | st.dictionaries(st.text(max_size=5), kids, max_size=4), max_leaves=20)


@settings(max_examples=600, deadline=None)
@given(json_values, st.booleans(), st.booleans())
def test_roundtrip_of_generated_documents(v, ascii_, as_bytes):
    doc = json.dumps(v, ensure_ascii=ascii_, indent=None if ascii_ else 1)
    check(doc.encode("utf-8", "surrogatepass") if as_bytes else doc)
    # the native parser really handled the representable ones (no silent fallback)
    if not as_bytes and not any(0xD800 <= ord(c) <= 0xDFFF for c in doc):
        assert same(fastpath.ext().loads(doc), json.loads(doc))


@settings(max_examples=800, deadline=None)
@given(st.text(alphabet='{}[]",:0123456789.eE+-tfnulrsaINy \t\n\\/u\x01é', max_size=24))
def test_arbitrary_text(doc):
    check(doc)


CASES = ['{"a": 1, "a": 2, "b": 3}', '[1, -0, -0.0, 1e400, -1e400, 1E-400, 0.5e+3]', "NaN", "-Infinity",
         "[Infinity, NaN]", "-NaN", '"\\ud83d\\ude00"', '"\\ud83d"', '"\\ude00x"', '"a\\u0000b"', '"tab\there"',
         '"\\x"', "01", "1.", ".5", "1e", "-", "[1,]", '{"a":1,}', "[] x", "﻿{}", "", "  ", "1" * 5000,
         '{"k": ' * 300 + "1" + "}" * 300, "[" * 100 + "]" * 100, '" "', "true", "nul", "[1 2]",
         '{"a" 1}', '{1: 2}', '"unterminated', "12345678901234567890123", "-12345678901234567890123.5"]


@pytest.mark.parametrize("doc", CASES)
def test_edge_cases(doc):
    check(doc)
    check(doc.encode("utf-8", "surrogatepass"))


@pytest.mark.parametrize("raw", [b"\xef\xbb\xbf{}", b'"\xff"', b'"\xed\xa0\x80"', b"{\x00}", bytearray(b"[1]"),
                                 memoryview(b'{"x": [true]}')])
def test_bytes_inputs(raw):
    check(raw)


def test_real_annotation_is_parsed_natively():
    rep = fixtures.mi355x_probe_report("n", gpus=8)
    raw = fixtures.health_annotation(rep)["amd.com/mi355x-health"]
    assert fastpath.ext().loads(raw) == json.loads(raw) == rep
