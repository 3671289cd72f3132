"""Native NodeList scanner / JSON emitter == the pure-Python reference semantics (byte for byte)."""
import json

import pytest
from hypothesis import HealthCheck, given, settings, strategies as st

from k8s_gpu_node_checker_amd.models.node import HEALTH_ANNOTATION, HEALTH_CONDITION, NodeExtras, ScanResult, scan_items
from k8s_gpu_node_checker_amd.models.resources import GPU_RESOURCE_KEYS
from k8s_gpu_node_checker_amd.ops import fastpath
from k8s_gpu_node_checker_amd.testing import fixtures

ext = fastpath.ext()
pytestmark = pytest.mark.skipif(ext is None, reason="native fast path not built")


def native_scan(body, src="capacity", extras=True, mode=2):
    r = ScanResult()
    tok = ext.scan_nodelist(body, r, GPU_RESOURCE_KEYS, src == "allocatable", extras, HEALTH_ANNOTATION, NodeExtras,
                            HEALTH_CONDITION, mode)
    return r, tok


def py_scan(body, src="capacity", extras=True, mode=2):
    doc = json.loads(body)
    r = scan_items(doc.get("items") or [], None, GPU_RESOURCE_KEYS, src, extras, mode)
    tok = (doc.get("metadata") or {}).get("continue") or None
    return r, (tok, r.items_seen)


def canon(r):
    ex = [dict(e.to_dict(), h=e.health_annotation) for e in r.extras]
    return json.dumps([r.gpu_nodes, r.ready_gpu_nodes, ex, r.items_seen], ensure_ascii=False)


def assert_same(body, src="capacity", mode=2):
    try:
        a, ta = native_scan(body, src, mode=mode)
    except ext.FallbackError:
        return "fallback"
    b, tb = py_scan(body, src, mode=mode)
    assert canon(a) == canon(b)
    assert ta == tb
    return "native"


@pytest.mark.parametrize("g", fixtures.GOLDEN)
@pytest.mark.parametrize("src", ["capacity", "allocatable"])
def test_golden(g, src):
    assert assert_same(json.dumps(fixtures.node_list(fixtures.golden(g), "tok")).encode(), src) == "native"


def test_realistic_cluster_with_health_and_addresses():
    body = json.dumps(fixtures.node_list(fixtures.cluster(50, "mixed", not_ready=[3], with_health=True))).encode()
    for mode in (0, 1, 2):
        assert assert_same(body, mode=mode) == "native"
    r1, _ = native_scan(body, mode=1)
    assert r1.extras[0].health_annotation is None and r1.extras[0].health_condition[0] == "True"
    r, _ = native_scan(body)
    assert r.extras[0].internal_ip == "10.0.0.0" and r.extras[0].health_annotation.startswith("{")


EDGE_BODIES = [
    b'{"items": [{"metadata": {"name": "e\\\\", "labels": {"a\\\\\\"b": "\\\\\\\\"}}, "status": {"capacity": {"amd.com/gpu": "1"}}}]}',
    b'{"items": [{"metadata": {"name": "long-' + b"x" * 70 + b'\\"q"}, "status": {"capacity": {"amd.com/gpu": "1"},'
    b' "images": [{"names": ["' + b"y" * 40 + b'\\\\", "z\\"{[]}"]}]}}]}',
    b'{"items": null}',
    b'{"items": []}',
    b'{"metadata": {"continue": ""}, "items": []}',
    b'{"items": [{"metadata": {"name": "a"}, "status": {"capacity": {"amd.com/gpu": 8},'
    b' "conditions": [{"type": "Ready", "status": "True"}]}}]}',
    b'{"items": [{"metadata": {"name": "a"}, "status": {"capacity": {"amd.com/gpu": "8", "amd.com/gpu": "2"}}}]}',
    b'{"items": [{"metadata": {"name": "a"}, "status": {"capacity": {"amd.com/gpu": " 8 "}}}]}',
    b'{"items": [{"metadata": {"name": "a"}, "status": {"capacity": {"amd.com/gpu": "1_0"}}}]}',
    b'{"items": [{"metadata": {"name": "a"}, "status": {"capacity": {"amd.com/gpu": 8.0, "nvidia.com/gpu": true}}}]}',
    b'{"items": [{"metadata": {"name": "a"}, "status": {"capacity": {"amd.com/gpu": null, "nvidia.com/gpu": "-1"}}}]}',
    b'{"items": [{"metadata": {"name": "a\\u00e9\\ud83d\\ude00", "labels": {"k\\"q": "v\\n"}},'
    b' "status": {"capacity": {"amd\\u002ecom/gpu": "3"}, "conditions": [{"type": "Re\\u0061dy", "status": "True"}]}}]}',
    b'{"items": [{"metadata": null, "spec": null, "status": {"capacity": {"amd.com/gpu": "1"}}}]}',
    b'{"items": [{"metadata": {}, "status": {"capacity": {"amd.com/gpu": "1"}}}]}',
    b'{"items": [{"metadata": {"name": "a"}, "spec": {"taints": [{"key": "k"}, 5, {"effect": "NoSchedule", "value": null}]},'
    b' "status": {"capacity": {"amd.com/gpu": "1"}}}]}',
    b'{"items": [{"metadata": {"name": "a"}, "status": {"capacity": {"amd.com/gpu": "1"},'
    b' "conditions": [{"type": "Ready", "status": "True", "status": "False"}]}}]}',
    b'{"items": [{"status": {"capacity": {"amd.com/gpu": "1"}}, "status": {"capacity": {"nvidia.com/gpu": "2"}}}]}',
    b'{"items": [5, "x", null, {"metadata": {"name": "b"}, "status": {"capacity": {"amd.com/gpu": "99999999999999999999"}}}]}',
    b'{"items": [{"metadata": {"name": "a", "labels": {}}, "status": {"capacity": {"amd.com/gpu": "1"},'
    b' "extra": [1, 2.5e3, -0.1, NaN, true, {"x": [[]]}]}}]}',
    b'  \n{"kind":"NodeList","items":[{"metadata":{"name":"w"},"status":{"capacity":{"amd.com/gpu":"4"}}}]}\n',
]


@pytest.mark.parametrize("body", EDGE_BODIES)
def test_edge_shapes(body):
    assert_same(body)


@pytest.mark.parametrize("body", [b"[]", b'{"items": {}}', b'{"items": [', b"", b'{"items": [{"metadata": {"name": 5}}]}',
                                  b'{"items": [{"metadata": {"labels": ["x"]}}]}', b'{"a": 1} x'])
def test_unmodelled_or_malformed_falls_back_without_side_effects(body):
    r = ScanResult()
    with pytest.raises(ext.FallbackError):
        ext.scan_nodelist(body, r, GPU_RESOURCE_KEYS, False, True, HEALTH_ANNOTATION, NodeExtras)
    assert r.gpu_nodes == [] and r.items_seen == 0


def test_scan_page_wrapper_falls_back_to_python():
    r = ScanResult()
    tok, n = fastpath.scan_page(b'{"items": [{"metadata": {"name": 5}, "status": {"capacity": {"amd.com/gpu": "1"}}}]}', r)
    assert n == 1 and r.gpu_nodes[0]["name"] == 5
    with pytest.raises(ValueError):
        fastpath.scan_page(b"[1]", ScanResult())


scalar = st.one_of(st.none(), st.booleans(), st.integers(-5, 10), st.text(max_size=6),
                   st.sampled_from(["0", "8", "1k", " 3", "+2", "", "Ready", "True", "False"]))
cap = st.dictionaries(st.sampled_from(list(GPU_RESOURCE_KEYS) + ["cpu"]), scalar, max_size=5)
cond = st.fixed_dictionaries({}, optional={"type": st.sampled_from(["Ready", "Other", 1, "AMDGPUHealthy"]),
                                           "status": st.sampled_from(["True", "False", "Unknown", None]),
                                           "reason": st.one_of(st.none(), st.sampled_from(["MI355XDegraded", "x"])),
                                           "message": st.text(max_size=5),
                                           "lastHeartbeatTime": st.sampled_from(["2025-10-10T00:00:00Z",
                                                                                 "2026-02-28T23:59:59Z", None])})
node = st.fixed_dictionaries({}, optional={
    "metadata": st.one_of(st.none(), st.fixed_dictionaries({}, optional={
        "name": st.one_of(st.none(), st.text(max_size=8)),
        "labels": st.one_of(st.none(), st.dictionaries(st.text(max_size=4), st.text(max_size=4), max_size=3)),
        "annotations": st.dictionaries(st.sampled_from([HEALTH_ANNOTATION, "x"]), st.text(max_size=5), max_size=2)})),
    "spec": st.one_of(st.none(), st.fixed_dictionaries({}, optional={
        "taints": st.lists(st.fixed_dictionaries({}, optional={"key": st.text(max_size=3),
                                                              "value": st.one_of(st.none(), st.text(max_size=3)),
                                                              "effect": st.text(max_size=3)}), max_size=2),
        "unschedulable": st.booleans()})),
    "status": st.fixed_dictionaries({}, optional={"capacity": cap, "allocatable": cap,
                                                  "conditions": st.lists(cond, max_size=3)}),
})


@settings(max_examples=300, suppress_health_check=[HealthCheck.too_slow])
@given(st.lists(node, max_size=6), st.sampled_from(["capacity", "allocatable"]), st.booleans(),
       st.sampled_from([0, 1, 2]))
def test_fuzz_equivalence(items, src, ascii_only, mode):
    body = json.dumps({"items": items}, ensure_ascii=ascii_only).encode()
    assert_same(body, src, mode)


json_tree = st.recursive(
    st.one_of(st.none(), st.booleans(), st.integers(), st.floats(allow_nan=True), st.text()),
    lambda ch: st.one_of(st.lists(ch, max_size=4), st.dictionaries(st.text(max_size=5), ch, max_size=4)),
    max_leaves=30)


@settings(max_examples=400)
@given(json_tree)
def test_dumps_indent2_byte_identical(tree):
    try:
        got = ext.dumps_indent2(tree)
    except ext.FallbackError:
        return
    assert got == json.dumps(tree, ensure_ascii=False, indent=2)


def test_dumps_control_chars_and_unicode():
    s = "".join(chr(i) for i in range(0, 0x30)) + " é😀\x7f\"\\"
    obj = {"k": [s, {"": None}, [], {}, 1.5, -0.0, 10 ** 30, True]}
    assert ext.dumps_indent2(obj) == json.dumps(obj, ensure_ascii=False, indent=2)
    assert fastpath.dumps_indent2({1: 2}) == json.dumps({1: 2}, ensure_ascii=False, indent=2)  # fallback path


@settings(max_examples=300, suppress_health_check=[HealthCheck.too_slow])
@given(st.text(alphabet=st.sampled_from('ab"\\\n\x01é😀\x7fz'), max_size=80), st.integers(0, 40))
def test_dumps_long_strings_escapes_at_every_offset(tail, pad):
    """The emitter copies 16 bytes at a time: escapes and non-ASCII bytes before, inside and after a 16-byte run."""
    obj = {"k" * pad: ["x" * pad + tail, tail + "y" * pad, -(2 ** 63), 2 ** 63 - 1, 2 ** 63, -7, 0]}
    assert ext.dumps_indent2(obj) == json.dumps(obj, ensure_ascii=False, indent=2)


def test_dumps_deep_indent_and_large_output():
    deep = []
    cur = deep
    for _ in range(120):  # beyond the preallocated indent run (64 levels)
        nxt = [1]
        cur.append(nxt)
        cur = nxt
    assert ext.dumps_indent2(deep) == json.dumps(deep, ensure_ascii=False, indent=2)
    big = {"nodes": [{"name": f"n{i}", "labels": {f"l{j}": "v" * 40 for j in range(20)}} for i in range(2000)]}
    assert ext.dumps_indent2(big) == json.dumps(big, ensure_ascii=False, indent=2)


@settings(max_examples=300, suppress_health_check=[HealthCheck.too_slow])
@given(json_tree, st.integers(0, 70), st.booleans())
def test_skipped_subtrees_with_escapes(junk, pad, ascii_only):
    """Arbitrary JSON (quotes, backslash runs, brackets inside strings) in skipped fields, at every
    alignment relative to the 64-byte SIMD blocks, must not change the scan."""
    node = {"metadata": {"name": "n" * pad, "annotations": {"x": json.dumps(junk)}},
            "spec": {"providerID": "\\\\\"[{" * (pad % 7)},
            "status": {"images": [junk, {"names": ["\\" * pad + '"]}']}],
                       "capacity": {"amd.com/gpu": "8"},
                       "nodeInfo": junk,
                       "conditions": [{"type": "Ready", "status": "True"}]}}
    body = json.dumps({"kind": "NodeList", "pad": "x" * pad, "items": [node, junk, node]}, ensure_ascii=ascii_only)
    if assert_same(body.encode()) == "native":
        r, _ = native_scan(body.encode())
        assert len(r.gpu_nodes) == 2


@settings(max_examples=300, suppress_health_check=[HealthCheck.too_slow])
@given(json_tree, st.integers(0, 130), st.integers(0, 9), st.booleans())
def test_escaped_modelled_strings_at_every_alignment(junk, pad, run, ascii_only):
    """Modelled strings with escapes (the health annotation is JSON stored in a string) are read
    64 bytes per step after their first backslash: backslash runs of every parity ending right
    before a quote, at every offset from the block edge, and a quote as the final byte, must all
    decode like json.loads."""
    tricky = "a" * pad + "\\" * run + '"' + "b" * (pad % 13) + "\\" * (run + 1) + '"'
    node = {"metadata": {"name": "n" + "\\" * run + '"' + "x" * pad,
                         "labels": {"k" * (pad % 5) + '"': tricky, "plain": "p" * pad},
                         "annotations": {HEALTH_ANNOTATION: json.dumps({"j": junk, "t": tricky})}},
            "spec": {"taints": [{"key": tricky, "value": "\\" * pad, "effect": '"' * run}]},
            "status": {"capacity": {"amd.com/gpu": "8"}, "conditions": [{"type": "Ready", "status": "True"}]}}
    body = json.dumps({"items": [node]}, ensure_ascii=ascii_only).encode()
    assert assert_same(body) == "native"
    # the same string ending exactly at the end of the buffer is unterminated, never read past
    with pytest.raises(ext.FallbackError):
        native_scan(b'{"items": [{"metadata": {"name": "' + b"a" * pad + b"\\\\" * run + b'\\"')


def test_string_cache_overflow_escapes_and_long_values():
    """Pass 2 shares repeated short label/taint strings through a per-page cache: a page with more
    distinct strings than the cache holds, escaped and long (uncached) strings, and repeats of each,
    must still equal the Python path."""
    items = []
    for i in range(700):
        labels = {f"k{i}": f"v{i}", "shared/key": "shared-value", "esc\\u00e9\"q": "a\\nb",
                  "long": "x" * (90 + i % 20), f"dup{i % 3}": "é" * (i % 4)}
        node = fixtures.realistic_node(f"n{i}", gpu_count=1 + i % 2, ready=i % 5 != 0)
        node["metadata"]["labels"] = labels
        node["spec"]["taints"] = [{"key": "amd.com/gpu", "value": None if i % 2 else f"t{i}", "effect": "NoSchedule"}]
        items.append(node)
    for ascii_only in (True, False):
        body = json.dumps({"kind": "NodeList", "metadata": {"continue": "tok"}, "items": items},
                          ensure_ascii=ascii_only).encode()
        assert assert_same(body) != "fallback"
    a, _ = native_scan(body)
    # shared strings really are shared objects, distinct ones stay distinct
    l0, l1 = a.gpu_nodes[1]["labels"], a.gpu_nodes[2]["labels"]
    k0 = [k for k in l0 if k == "shared/key"][0]
    k1 = [k for k in l1 if k == "shared/key"][0]
    assert k0 is k1 and l0["k1"] == "v1" and l1["k2"] == "v2"


def test_node_extras_built_without_init_has_every_slot():
    body = json.dumps({"items": [fixtures.realistic_node("a", gpu_count=2)]}).encode()
    a, _ = native_scan(body)
    ex = a.extras[0]
    assert type(ex) is NodeExtras
    for slot in NodeExtras.__slots__:
        if slot.startswith("_"):
            continue  # a lazily filled cache (NodeExtras.report), not data the scanner sets
        getattr(ex, slot)  # AttributeError if a slot was left unset
    assert ex.report() is None  # the cache fills on first use (this node carries no report)

    class Custom:  # not a __slots__ type with member descriptors: the constructor path is used
        def __init__(self, *args):
            self.args = args
    r = ScanResult()
    ext.scan_nodelist(body, r, GPU_RESOURCE_KEYS, False, True, HEALTH_ANNOTATION, Custom, HEALTH_CONDITION, 2)
    assert isinstance(r.extras[0], Custom) and len(r.extras[0].args) == 7


def test_prescan_then_finish_equals_one_shot_scan():
    """The page reader's pass 1 (prescan, any thread) + the main thread's pass 2 give exactly what one
    scan_nodelist call gives, for modelled pages, for pages that fall back, and with other keys."""
    body = json.dumps(fixtures.node_list(fixtures.cluster(40, "mixed", not_ready=[3], with_health=True), "tok")).encode()
    for mode in (0, 1, 2):
        a, ta = native_scan(body, mode=mode)
        b = ScanResult()
        tb = fastpath.scan_page(body, b, want_extras=True, annotation_mode=mode, pre=fastpath.prescan(body))
        assert canon(a) == canon(b) and ta == tb
    # a page pass 1 cannot model: the Python path answers, as for scan_nodelist
    odd = b'{"items": [{"metadata": {"name": 5}, "status": {"capacity": {"amd.com/gpu": "1"}}}]}'
    r = ScanResult()
    assert fastpath.scan_page(odd, r, pre=fastpath.prescan(odd)) == (None, 1) and r.gpu_nodes[0]["name"] == 5
    # a prescan made with other keys is ignored, not misapplied
    r2 = ScanResult()
    fastpath.scan_page(body, r2, keys=("amd.com/gpu",), pre=fastpath.prescan(body))
    assert all(set(n["gpu_breakdown"]) <= {"amd.com/gpu"} for n in r2.gpu_nodes)
    with pytest.raises(ValueError):
        ext.scan_prescanned(fastpath.prescan(body)[1], ScanResult(), ("x",), False, False, NodeExtras)
